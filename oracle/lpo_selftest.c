/*
 * lpo_selftest.c -- drives every entry point of the C oracle (lpo.c) on small
 * LPs so that the sanitizer build (make -C oracle sanitize: ASan + UBSan)
 * checks its memory accesses and arithmetic. Test infrastructure only
 * (tests/test_sanitizers.py); exits non-zero on a wrong status.
 */
#include <stdio.h>
#include <stdlib.h>

#include "lpo.h"

static int fails = 0;
#define EXPECT(c)                                                             \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "selftest: %s failed (line %d)\n", #c, __LINE__); \
            fails++;                                                          \
        }                                                                     \
    } while (0)

int main(void) {
    lpo_result r;
    /* dense, Dantzig and Bland, to optimality */
    for (int rule = 0; rule < 2; rule++) {
        const int64_t m = 37, n = 53;
        lpo_ctx *c = lpo_create(m, n + m + 1, 2);
        EXPECT(lpo_generate(c, n, 20220518, LPO_GEN_DENSE) == 0);
        EXPECT(lpo_solve(c, 100000, rule, 1, &r) == 0 && r.status == LPO_OPTIMAL);
        int64_t *basis = calloc((size_t) m, sizeof *basis), *k = calloc((size_t) r.pivots, sizeof *k),
                *rr = calloc((size_t) r.pivots, sizeof *rr);
        double *rows = calloc((size_t) ((m + 1) * (n + m + 1)), sizeof *rows);
        EXPECT(lpo_get_basis(c, basis) == 0);
        EXPECT(lpo_get_log(c, k, rr, r.pivots) == r.pivots);
        EXPECT(lpo_get_rows(c, 0, m + 1, rows, n + m + 1) == 0);
        /* reload the final tableau into a fresh context: already optimal */
        lpo_ctx *d = lpo_create(m, n + m + 1, 1);
        EXPECT(lpo_load_rows(d, 0, m + 1, rows, n + m + 1) == 0 && lpo_set_basis(d, basis) == 0);
        EXPECT(lpo_solve(d, 10, rule, 1, &r) == 0 && r.status == LPO_OPTIMAL && r.pivots == 0);
        lpo_destroy(d);
        free(basis), free(k), free(rr), free(rows);
        lpo_destroy(c);
    }
    /* degenerate (KM-style) under Bland, capped; the multi-part solve */
    {
        lpo_ctx *c = lpo_create(24, 49, 2);
        EXPECT(lpo_generate(c, 24, 14, LPO_GEN_DEGENERATE) == 0);
        EXPECT(lpo_solve(c, 500, LPO_RULE_BLAND, 3, &r) == 0);
        EXPECT(r.status == LPO_OPTIMAL || r.status == LPO_ITER_LIMIT);
        lpo_destroy(c);
    }
    /* two-phase and Big-M with artificials */
    for (int method = 0; method < 2; method++) {
        const int64_t m = 40, n = 40, art_first = 1 + n + (m + 1) / 2;
        lpo_ctx *c = lpo_create2(m, n + m + 1, 2, method ? 2 : 1);
        EXPECT(lpo_generate(c, n, 7, LPO_GEN_ARTIFICIAL) == 0);
        if (method)
            EXPECT(lpo_solve_big_m(c, art_first, NULL, 100000, LPO_RULE_BLAND, &r) == 0);
        else
            EXPECT(lpo_solve_two_phase(c, art_first, NULL, 100000, LPO_RULE_BLAND, &r) == 0);
        EXPECT(r.status == LPO_OPTIMAL || r.status == LPO_INFEASIBLE || r.status == LPO_UNBOUNDED);
        lpo_destroy(c);
    }
    /* dual simplex */
    {
        const int64_t m = 30, n = 45;
        lpo_ctx *c = lpo_create(m, n + m + 1, 2);
        EXPECT(lpo_generate(c, n, 3, LPO_GEN_DUAL) == 0);
        EXPECT(lpo_solve_dual(c, 100000, &r) == 0 && (r.status == LPO_OPTIMAL || r.status == LPO_INFEASIBLE));
        lpo_destroy(c);
    }
    /* row-block primitives of the multi-rank model */
    {
        const int64_t m = 16, n = 20, N1 = n + m + 1;
        lpo_ctx *c = lpo_create(m, N1, 1);
        double out[4], *P = calloc((size_t) N1, sizeof *P);
        EXPECT(lpo_generate(c, n, 5, LPO_GEN_DENSE) == 0);
        const int64_t k = lpo_price_col(c, LPO_RULE_DANTZIG);
        EXPECT(k >= 1);
        EXPECT(lpo_ratio(c, k, LPO_RULE_DANTZIG, 0, out) == 0 && out[3] >= 0);
        EXPECT(lpo_pivot_row(c, (int64_t) out[3], k, P) == 0 && lpo_apply(c, k, (int64_t) out[3], P) == 0);
        (void) lpo_pivot(c, k == 1 ? 2 : 1, 0);   /* forced pivot: any element, no status to check */
        free(P);
        lpo_destroy(c);
    }
    printf("lpo_selftest: %s\n", fails ? "FAILED" : "ok");
    return fails != 0;
}
