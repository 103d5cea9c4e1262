/*
 * lpo.h — CPU fp64 dense-tableau simplex ORACLE (test infrastructure only).
 *
 * This is NOT product code. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load or call it, and only as the checker /
 * CPU baseline. The product path (include/lpg.h -> liblpg.so, HIP on gfx950)
 * never links, loads or falls back to it.
 *
 * What it restates. The reference (SomeBottle/LinearProgramming) builds the
 * simplex tableau but has no pivot loop: newSimplex stops after CreateSMatrix
 * (Source/simplex.c:27-73; insertion point simplex.c:40 -> :65). The tableau
 * layout is the reference's SimplexMatrix (Source/matrix.h:13-21) flattened to
 * fp64: row i = [b_i | a_i1 .. a_iN] exactly as CreateSMatrix fills
 * cMatrix[i][0] = b (matrix.c:42-48) and cMatrix[i][j+1] = a_ij
 * (matrix.c:62-66); column order is the LPAlign/TermsSort order
 * (simplex.c:238-260, 288-325). The pivot rules (Dantzig / Bland pricing,
 * min-ratio test, Gauss-Jordan rank-1 update) are the ones SURVEY.md §8(a)
 * rows a10-a12 fix for the missing loop.
 *
 * Parity pinning. The pre-pivot pipeline is pinned by transcripts of the
 * reference binary built from /root/reference (oracle/Makefile target `ref` ->
 * oracle/_ref/lp, fixtures under tests/golden/). The pivot arithmetic has
 * no reference counterpart (the loop is absent upstream), so it is pinned by
 * (1) the hand-derived known answer for Source/testdata.txt with `max:`
 * (z* = 12, SURVEY.md Appendix A2, incl. the exact pivot sequence),
 * (2) the exact-rational restatement oracle/fraction_oracle.py, and
 * (3) scipy/HiGHS optima in the CPU test suite.
 *
 * Arithmetic contract shared with the device engine (bitwise):
 *   P[j]   = T[r][j] / T[r][k]                     (IEEE division)
 *   T[i][j]= fma(-C[i], P[j], T[i][j])  (i != r)   (C = old column k)
 *   T[r][j]= P[j]
 * Compile with -ffp-contract=off so no other expression is fused.
 */
#ifndef LPO_H
#define LPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { LPO_RUNNING = 0, LPO_OPTIMAL = 1, LPO_UNBOUNDED = 2, LPO_INFEASIBLE = 3,
       LPO_ITER_LIMIT = 4, LPO_NUMERIC = 5 };
enum { LPO_RULE_DANTZIG = 0, LPO_RULE_BLAND = 1 };
enum { LPO_GEN_DENSE = 0, LPO_GEN_DEGENERATE = 1, LPO_GEN_ARTIFICIAL = 2, LPO_GEN_DUAL = 3 };

typedef struct lpo_ctx lpo_ctx;

typedef struct {
    int32_t status;
    int32_t rule;
    int64_t pivots;       /* pivots applied by this ctx so far */
    double  objective;    /* T[m][0] (objective constant not included) */
    int64_t entering;     /* last pivot's column (1-based), -1 if none */
    int64_t leaving;      /* last pivot's row (0-based), -1 if none */
} lpo_result;

/* m constraint rows, ncols = N+1 columns (b + N variables). */
lpo_ctx *lpo_create(int64_t m, int64_t ncols, int nthreads);
/* nobj = 2: Big-M layout (row m = M part, row m+1 = real part). */
lpo_ctx *lpo_create2(int64_t m, int64_t ncols, int nthreads, int nobj);
void     lpo_destroy(lpo_ctx *ctx);
/* OpenMP threads of the row loops from now on (bench.py's 1-core CPU baseline). */
int      lpo_set_threads(lpo_ctx *ctx, int nthreads);
int      lpo_load_rows(lpo_ctx *ctx, int64_t row0, int64_t nrows, const double *rows, int64_t ld);
int      lpo_set_basis(lpo_ctx *ctx, const int64_t *basis);
/* Objective row from costs c[0..N-1] (max c.x) and the current basis:
 * d_j = sum_i c_B(i) T[i][j] - c_j, z = sum_i c_B(i) b_i (row order fixed). */
int      lpo_set_objective(lpo_ctx *ctx, const double *c);
int      lpo_set_objective_m(lpo_ctx *ctx, const double *c);
int      lpo_generate(lpo_ctx *ctx, int64_t n_struct, uint64_t seed, int kind);
int64_t  lpo_unit_column(int64_t m, int64_t n, int64_t i, int kind);
int      lpo_set_tolerances(lpo_ctx *ctx, double eps_piv, double eps_opt);
int      lpo_set_active_columns(lpo_ctx *ctx, int64_t nact);
/* Run up to max_pivots pivots. nparts > 1 emulates the row-block partition of
 * the multi-GPU engine: the ratio test is reduced per block, then across
 * blocks with the same lexicographic combine (loopback "allgather"). */
int      lpo_solve(lpo_ctx *ctx, int64_t max_pivots, int rule, int nparts, lpo_result *out);
int      lpo_get_rows(const lpo_ctx *ctx, int64_t row0, int64_t nrows, double *out, int64_t ld);
int      lpo_get_basis(const lpo_ctx *ctx, int64_t *basis);
/* Pivot log: k (1-based column) and r (0-based row) of every pivot applied. */
int64_t  lpo_get_log(const lpo_ctx *ctx, int64_t *k, int64_t *r, int64_t max);
int64_t  lpo_rows(const lpo_ctx *ctx);
int64_t  lpo_ld(const lpo_ctx *ctx);

/* Rank-1 update only (timing harness for the CPU baseline): applies pivot
 * (k, r) with the bitwise contract above, no pricing or ratio test. */
int      lpo_pivot(lpo_ctx *ctx, int64_t k, int64_t r);

/* Two-phase method, same algorithm as lpg_solve_two_phase (cost NULL: the
 * costs are -1 x the objective row as loaded, i.e. a slack-form -c row). */
int      lpo_solve_two_phase(lpo_ctx *ctx, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                             lpo_result *out);

/* Big-M method, same algorithm as lpg_solve_big_m (cost NULL: -1 x the
 * real objective row as loaded). */
int      lpo_solve_big_m(lpo_ctx *ctx, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                         lpo_result *out);

/* Dual simplex, same rules as lpg_solve_dual; -2 if the basis is not dual
 * feasible. */
int      lpo_solve_dual(lpo_ctx *ctx, int64_t max_pivots, lpo_result *out);

/* Row-block primitives for the multi-rank protocol model (tests only). */
int64_t  lpo_price_col(const lpo_ctx *ctx, int rule);
/* out = {theta, pivot element, key, global row (-1: no candidate)} */
int      lpo_ratio(const lpo_ctx *ctx, int64_t k, int rule, int64_t row_offset, double out[4]);
int      lpo_pivot_row(const lpo_ctx *ctx, int64_t rl, int64_t k, double *P);
int      lpo_apply(lpo_ctx *ctx, int64_t k, int64_t rl, const double *P);

/* splitmix64 uniform in [0,1): shared with the device generator. */
double   lpo_uniform(uint64_t key, uint64_t idx);
uint64_t lpo_subkey(uint64_t seed, uint64_t which);

#ifdef __cplusplus
}
#endif
#endif
