/*
 * lpo.c — CPU fp64 dense-tableau simplex ORACLE (test infrastructure only;
 * see lpo.h for what it restates, what pins it, and who may call it).
 *
 * Reference anchors (SomeBottle/LinearProgramming, /root/reference):
 *   tableau = SimplexMatrix flattened (Source/matrix.h:13-21,
 *             Source/matrix.c:42-66: column 0 = b, columns 1..N = a_ij);
 *   maximise form (Source/simplex.c:99-106): objective row holds
 *             d_j = z_j - c_j, optimal when every d_j >= -eps;
 *   pivot loop: absent upstream (Source/simplex.c:40 -> :65); rules per
 *             SURVEY.md §8(a) a10 (pricing), a11 (ratio), a12 (update).
 */
#include "lpo.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

struct lpo_ctx {
    int64_t m, ncols, ld, nobj, nact;
    double *T;          /* (m + nobj) x ld, row-major */
    double *P, *C;      /* pivot-row / pivot-column snapshots */
    int64_t *basis;     /* 1-based column of the basic variable of each row */
    int64_t *logk, *logr;
    int64_t logcap, pivots;
    double eps_piv, eps_opt;
    int status;
    int64_t last_k, last_r;
    int nthreads;
};

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t lpo_subkey(uint64_t seed, uint64_t which) { return splitmix64(seed ^ (which * 0xD1B54A32D192ED03ull)); }

double lpo_uniform(uint64_t key, uint64_t idx) {
    return (double)(splitmix64(key ^ (idx * 0x9E3779B97F4A7C15ull)) >> 11) * 0x1.0p-53;
}

int lpo_set_threads(lpo_ctx *c, int nthreads) {
    if (!c || nthreads < 1) return -1;
    c->nthreads = nthreads;
    return 0;
}

lpo_ctx *lpo_create(int64_t m, int64_t ncols, int nthreads) { return lpo_create2(m, ncols, nthreads, 1); }

lpo_ctx *lpo_create2(int64_t m, int64_t ncols, int nthreads, int nobj) {
    if (m <= 0 || ncols < 2 || nobj < 1 || nobj > 2) return NULL;
    lpo_ctx *c = (lpo_ctx *)calloc(1, sizeof(lpo_ctx));
    if (!c) return NULL;
    c->m = m; c->ncols = ncols; c->nobj = nobj; c->nact = ncols - 1;
    c->ld = (ncols + 7) & ~(int64_t)7;
    c->T = (double *)calloc((size_t)((m + c->nobj) * c->ld), sizeof(double));
    c->P = (double *)calloc((size_t)c->ld, sizeof(double));
    c->C = (double *)calloc((size_t)(m + c->nobj), sizeof(double));
    c->basis = (int64_t *)calloc((size_t)m, sizeof(int64_t));
    c->logcap = 1024;
    c->logk = (int64_t *)malloc((size_t)c->logcap * sizeof(int64_t));
    c->logr = (int64_t *)malloc((size_t)c->logcap * sizeof(int64_t));
    c->eps_piv = 1e-9; c->eps_opt = 1e-9;
    c->last_k = c->last_r = -1;
    c->nthreads = nthreads > 0 ? nthreads : 1;
    if (!c->T || !c->P || !c->C || !c->basis || !c->logk || !c->logr) { lpo_destroy(c); return NULL; }
    return c;
}

void lpo_destroy(lpo_ctx *c) {
    if (!c) return;
    free(c->T); free(c->P); free(c->C); free(c->basis); free(c->logk); free(c->logr);
    free(c);
}

int64_t lpo_rows(const lpo_ctx *c) { return c->m + c->nobj; }
int64_t lpo_ld(const lpo_ctx *c) { return c->ld; }

int lpo_load_rows(lpo_ctx *c, int64_t row0, int64_t nrows, const double *rows, int64_t ld) {
    if (!c || row0 < 0 || nrows < 0 || row0 + nrows > c->m + c->nobj || ld < c->ncols) return -1;
    for (int64_t i = 0; i < nrows; i++)
        memcpy(c->T + (row0 + i) * c->ld, rows + i * ld, (size_t)c->ncols * sizeof(double));
    c->status = LPO_RUNNING;
    return 0;
}

int lpo_set_basis(lpo_ctx *c, const int64_t *basis) {
    if (!c || !basis) return -1;
    for (int64_t i = 0; i < c->m; i++) {
        if (basis[i] < 1 || basis[i] >= c->ncols) return -1;
        c->basis[i] = basis[i];
    }
    return 0;
}

static int set_objective_row(lpo_ctx *c, const double *cost, int64_t orow);

/* (real) objective row m + nobj - 1 */
int lpo_set_objective(lpo_ctx *c, const double *cost) {
    if (!c || !cost) return -1;
    return set_objective_row(c, cost, c->m + c->nobj - 1);
}

/* Big-M: the M-part row m */
int lpo_set_objective_m(lpo_ctx *c, const double *cost) {
    if (!c || !cost || c->nobj != 2) return -1;
    return set_objective_row(c, cost, c->m);
}

static int set_objective_row(lpo_ctx *c, const double *cost, int64_t orow) {
    double *obj = c->T + orow * c->ld;
    /* d_j = sum_i cB_i * T[i][j] - c_j ; sum in row order with fma. */
    for (int64_t j = 0; j < c->ncols; j++) {
        double acc = 0.0;
        for (int64_t i = 0; i < c->m; i++)
            acc = fma(cost[c->basis[i] - 1], c->T[i * c->ld + j], acc);
        obj[j] = j == 0 ? acc : acc - cost[j - 1];
    }
    c->status = LPO_RUNNING;
    return 0;
}

int lpo_set_tolerances(lpo_ctx *c, double eps_piv, double eps_opt) {
    if (!c || !(eps_piv >= 0) || !(eps_opt >= 0)) return -1;
    c->eps_piv = eps_piv; c->eps_opt = eps_opt;
    return 0;
}

int lpo_set_active_columns(lpo_ctx *c, int64_t nact) {
    if (!c || nact < 1 || nact > c->ncols - 1) return -1;
    c->nact = nact;
    return 0;
}

/* Column of row i's initial unit (basic) column. Kinds 0/1: slack 1+n+i.
 * Kind 2: even rows (<= 0, degenerate) get slacks 1+n+i/2, odd rows
 * (equalities) get artificials from art_first = 1+n+ceil(m/2) on. */
int64_t lpo_unit_column(int64_t m, int64_t n, int64_t i, int kind) {
    if (kind != LPO_GEN_ARTIFICIAL) return 1 + n + i;
    return (i & 1) ? 1 + n + (m + 1) / 2 + i / 2 : 1 + n + i / 2;
}

/* Synthetic LPs. Dense: A_ij = u in [0,1), b_i = n/8 (1+u),
 * c_j = 1+u, all rows <= with a slack basis. Degenerate: lower-triangular
 * KM-style rows (a_ii = 1, a_ij = u/(i+1) for j < i, so the strictly-lower
 * part has infinity-norm < 1 and every basis inverse stays bounded; the 2u of
 * SURVEY.md's sketch grows like 3^i and makes fp64 Bland cycle by m = 256),
 * b_i = 0 on even rows (primal degenerate). Artificial (config 5): as
 * degenerate, but even rows have negative off-diagonals (a feasible
 * `<= 0` row) and odd rows are equalities whose unit columns are artificial
 * (columns art_first..N); the objective row still holds -c. */
int lpo_generate(lpo_ctx *c, int64_t n, uint64_t seed, int kind) {
    if (!c || n < 1 || c->ncols != n + c->m + 1 || kind < 0 || kind > LPO_GEN_DUAL) return -1;
    const int64_t m = c->m, ld = c->ld;
    const uint64_t kA = lpo_subkey(seed, 1), kB = lpo_subkey(seed, 2), kC = lpo_subkey(seed, 3);
    const double bscale = (double)n / 8.0;
#pragma omp parallel for schedule(static) num_threads(c->nthreads)
    for (int64_t i = 0; i < m; i++) {
        double *row = c->T + i * ld;
        memset(row, 0, (size_t)ld * sizeof(double));
        if (kind == LPO_GEN_DENSE || kind == LPO_GEN_DUAL) {
            const double sg = kind == LPO_GEN_DUAL ? -1.0 : 1.0;   /* dual: rows [-b | -A | I] */
            row[0] = sg * (bscale * (1.0 + lpo_uniform(kB, (uint64_t)i)));
            for (int64_t j = 0; j < n; j++) row[1 + j] = sg * lpo_uniform(kA, (uint64_t)(i * n + j));
        } else {
            row[0] = (i & 1) ? bscale * (1.0 + lpo_uniform(kB, (uint64_t)i)) : 0.0;
            const double sgn = (kind == LPO_GEN_ARTIFICIAL && !(i & 1)) ? -1.0 : 1.0;
            for (int64_t j = 0; j < n; j++) {
                double a = 0.0;
                if (j < i) a = sgn * (lpo_uniform(kA, (uint64_t)(i * n + j)) / (double)(i + 1));
                else if (j == i) a = 1.0;
                row[1 + j] = a;
            }
        }
        const int64_t u = lpo_unit_column(m, n, i, kind);
        row[u] = 1.0;
        c->basis[i] = u;
    }
    for (int64_t q = 0; q < c->nobj; q++) memset(c->T + (m + q) * ld, 0, (size_t)ld * sizeof(double));
    double *obj = c->T + (m + c->nobj - 1) * ld;   /* (real) objective row; a Big-M M row stays zero */
    for (int64_t j = 0; j < n; j++) {
        const double cj = 1.0 + lpo_uniform(kC, (uint64_t)j);
        obj[1 + j] = kind == LPO_GEN_DUAL ? cj : -cj;   /* dual: max -c.x, d_j = +c_j */
    }
    c->status = LPO_RUNNING;
    c->pivots = 0; c->last_k = c->last_r = -1;
    return 0;
}

/* ---- pivot rules ---- */

/* Eligibility class of column j: -1 not eligible; one objective row: 0 if
 * d_j < -eps (value d_j); Big-M: 0 if dM_j < -eps (value dM_j), 1 if
 * |dM_j| <= eps and dR_j < -eps (value dR_j). NaN is never eligible. */
static int price_class(const lpo_ctx *c, int64_t j, double *v) {
    const double dR = c->T[(c->m + c->nobj - 1) * c->ld + j];
    if (c->nobj == 1) {
        if (!(dR < -c->eps_opt)) return -1;
        *v = dR;
        return 0;
    }
    const double dM = c->T[c->m * c->ld + j];
    if (dM < -c->eps_opt) { *v = dM; return 0; }
    if (dM <= c->eps_opt && dR < -c->eps_opt) { *v = dR; return 1; }
    return -1;
}

static int64_t price(const lpo_ctx *c, int rule) {
    int64_t best = -1; int bc = 0; double bv = 0.0;
    for (int64_t j = 1; j <= c->nact; j++) {
        double v;
        const int cls = price_class(c, j, &v);
        if (cls < 0) continue;
        if (rule == LPO_RULE_BLAND) return j;
        if (best < 0 || cls < bc || (cls == bc && v < bv)) { best = j; bc = cls; bv = v; }
    }
    return best;
}

typedef struct { double theta; int64_t key; int64_t row; } cand_t;

static int cand_less(const cand_t *a, const cand_t *b) {
    if (a->row < 0) return 0;
    if (b->row < 0) return 1;
    if (a->theta != b->theta) return a->theta < b->theta;
    return a->key < b->key;
}

static cand_t ratio_block(const lpo_ctx *c, int64_t k, int rule, int64_t i0, int64_t i1) {
    cand_t best = {0.0, 0, -1};
    for (int64_t i = i0; i < i1; i++) {
        const double a = c->T[i * c->ld + k];
        if (!(a > c->eps_piv)) continue;
        const double b = c->T[i * c->ld];
        cand_t cd = {b > 0.0 ? b / a : 0.0, rule == LPO_RULE_BLAND ? c->basis[i] : i, i};
        if (cand_less(&cd, &best)) best = cd;
    }
    return best;
}

/* Gauss-Jordan rank-1 update (a12) with the bitwise contract of lpo.h. */
int lpo_pivot(lpo_ctx *c, int64_t k, int64_t r) {
    if (!c || k < 1 || k >= c->ncols || r < 0 || r >= c->m) return -1;
    const int64_t ld = c->ld, rows = c->m + c->nobj, nc = c->ncols;
    double *T = c->T;
    const double piv = T[r * ld + k];
    for (int64_t j = 0; j < nc; j++) c->P[j] = T[r * ld + j] / piv;
    for (int64_t i = 0; i < rows; i++) c->C[i] = T[i * ld + k];
    const double *P = c->P, *C = c->C;
#pragma omp parallel for schedule(static) num_threads(c->nthreads)
    for (int64_t i = 0; i < rows; i++) {
        double *row = T + i * ld;
        if (i == r) {
            memcpy(row, P, (size_t)nc * sizeof(double));
        } else {
            const double ci = -C[i];
            for (int64_t j = 0; j < nc; j++) row[j] = fma(ci, P[j], row[j]);
        }
    }
    c->basis[r] = k;
    if (c->pivots >= c->logcap) {
        int64_t cap = c->logcap * 2;
        int64_t *nk = (int64_t *)realloc(c->logk, (size_t)cap * sizeof(int64_t));
        if (nk) c->logk = nk;
        int64_t *nr = (int64_t *)realloc(c->logr, (size_t)cap * sizeof(int64_t));
        if (nr) c->logr = nr;
        if (!nk || !nr) return -1;
        c->logcap = cap;
    }
    c->logk[c->pivots] = k; c->logr[c->pivots] = r;
    c->pivots++;
    c->last_k = k; c->last_r = r;
    return 0;
}

int lpo_solve(lpo_ctx *c, int64_t max_pivots, int rule, int nparts, lpo_result *out) {
    if (!c || max_pivots < 0) return -1;
    if (nparts < 1) nparts = 1;
    int64_t done = 0;
    while (c->status == LPO_RUNNING && done < max_pivots) {
        const int64_t k = price(c, rule);
        if (k < 0) { c->status = LPO_OPTIMAL; break; }
        cand_t best = {0.0, 0, -1};
        for (int p = 0; p < nparts; p++) {          /* loopback "allgather" */
            const int64_t i0 = c->m * p / nparts, i1 = c->m * (p + 1) / nparts;
            cand_t cp = ratio_block(c, k, rule, i0, i1);
            if (cand_less(&cp, &best)) best = cp;
        }
        if (best.row < 0) { c->status = LPO_UNBOUNDED; break; }
        const double piv = c->T[best.row * c->ld + k];
        if (!isfinite(piv) || !isfinite(c->T[best.row * c->ld])) { c->status = LPO_NUMERIC; break; }
        if (lpo_pivot(c, k, best.row) != 0) return -1;
        done++;
    }
    if (c->status == LPO_RUNNING && done >= max_pivots) {
        /* peek: a finished LP reports OPTIMAL even when the budget ran out on its last pivot */
        if (price(c, rule) < 0) c->status = LPO_OPTIMAL;
    }
    if (out) {
        out->status = c->status == LPO_RUNNING ? LPO_ITER_LIMIT : c->status;
        out->rule = rule;
        out->pivots = c->pivots;
        out->objective = c->T[(c->m + c->nobj - 1) * c->ld];
        out->entering = c->last_k;
        out->leaving = c->last_r;
    }
    return 0;
}

int lpo_get_rows(const lpo_ctx *c, int64_t row0, int64_t nrows, double *out, int64_t ld) {
    if (!c || row0 < 0 || nrows < 0 || row0 + nrows > c->m + c->nobj || ld < c->ncols) return -1;
    for (int64_t i = 0; i < nrows; i++)
        memcpy(out + i * ld, c->T + (row0 + i) * c->ld, (size_t)c->ncols * sizeof(double));
    return 0;
}

int lpo_get_basis(const lpo_ctx *c, int64_t *basis) {
    if (!c || !basis) return -1;
    memcpy(basis, c->basis, (size_t)c->m * sizeof(int64_t));
    return 0;
}

int64_t lpo_get_log(const lpo_ctx *c, int64_t *k, int64_t *r, int64_t max) {
    if (!c) return -1;
    int64_t n = c->pivots < max ? c->pivots : max;
    if (k) memcpy(k, c->logk, (size_t)n * sizeof(int64_t));
    if (r) memcpy(r, c->logr, (size_t)n * sizeof(int64_t));
    return c->pivots;
}

/* ---- row-block primitives (multi-rank protocol model, tests only) ----
 * A ctx created with m = this rank's row count holds one row block plus the
 * replicated objective row. The gloo test drives the exchange itself:
 * lpo_price (replicated) -> lpo_ratio (local candidate) -> allgather ->
 * owner lpo_pivot_row, others zeros -> allreduce(sum) -> lpo_apply. */

int64_t lpo_price_col(const lpo_ctx *c, int rule) { return price(c, rule); }

int lpo_ratio(const lpo_ctx *c, int64_t k, int rule, int64_t row_offset, double out[4]) {
    if (!c || k < 1 || k >= c->ncols) return -1;
    cand_t b = ratio_block(c, k, rule, 0, c->m);
    out[0] = b.theta;
    out[1] = b.row >= 0 ? c->T[b.row * c->ld + k] : 0.0;
    out[2] = (double)(rule == LPO_RULE_BLAND ? b.key : (b.row >= 0 ? b.row + row_offset : 0));
    out[3] = (double)(b.row >= 0 ? b.row + row_offset : -1);
    return 0;
}

int lpo_pivot_row(const lpo_ctx *c, int64_t rl, int64_t k, double *P) {
    if (!c || rl < 0 || rl >= c->m || k < 1 || k >= c->ncols) return -1;
    const double piv = c->T[rl * c->ld + k];
    for (int64_t j = 0; j < c->ncols; j++) P[j] = c->T[rl * c->ld + j] / piv;
    return 0;
}

int lpo_apply(lpo_ctx *c, int64_t k, int64_t rl, const double *P) {
    if (!c || k < 1 || k >= c->ncols || rl >= c->m) return -1;
    const int64_t ld = c->ld, rows = c->m + c->nobj, nc = c->ncols;
    for (int64_t i = 0; i < rows; i++) c->C[i] = c->T[i * ld + k];
    for (int64_t i = 0; i < rows; i++) {
        double *row = c->T + i * ld;
        if (i == rl) {
            memcpy(row, P, (size_t)nc * sizeof(double));
        } else {
            const double ci = -c->C[i];
            for (int64_t j = 0; j < nc; j++) row[j] = fma(ci, P[j], row[j]);
        }
    }
    if (rl >= 0) c->basis[rl] = k;
    c->pivots++;
    return 0;
}

/* Two-phase restatement (same algorithm as lpg_solve_two_phase). */
int lpo_solve_two_phase(lpo_ctx *c, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                        lpo_result *out) {
    if (!c || art_first < 2 || art_first >= c->ncols) return -1;
    const int64_t N = c->ncols - 1;
    double *own = NULL;
    if (!cost) {
        own = (double *)malloc((size_t)N * sizeof(double));
        if (!own) return -1;
        for (int64_t j = 1; j <= N; j++) own[j - 1] = -c->T[c->m * c->ld + j];
        cost = own;
    }
    double *c1 = (double *)calloc((size_t)N, sizeof(double));
    if (!c1) return -1;
    for (int64_t j = art_first; j <= N; j++) c1[j - 1] = -1.0;
    c->nact = N;
    lpo_set_objective(c, c1);
    free(c1);
    lpo_result r1;
    lpo_solve(c, max_pivots, rule, 1, &r1);
    if (r1.status == LPO_ITER_LIMIT || r1.status == LPO_NUMERIC || r1.status == LPO_UNBOUNDED) {
        if (out) { *out = r1; if (r1.status == LPO_UNBOUNDED) out->status = LPO_NUMERIC; }
        free(own);
        return 0;
    }
    double bsum = 0;
    for (int64_t i = 0; i < c->m; i++) bsum += fabs(c->T[i * c->ld]);
    if (r1.objective < -1e-9 * (bsum > 1.0 ? bsum : 1.0)) {
        if (out) { *out = r1; out->status = LPO_INFEASIBLE; }
        free(own);
        return 0;
    }
    for (int64_t i = 0; i < c->m; i++) {
        if (c->basis[i] < art_first) continue;
        for (int64_t j = 1; j < art_first; j++)
            if (fabs(c->T[i * c->ld + j]) > c->eps_piv) { lpo_pivot(c, j, i); break; }
    }
    c->nact = art_first - 1;
    lpo_set_objective(c, cost);
    int64_t left = max_pivots - c->pivots;
    lpo_solve(c, left > 0 ? left : 0, rule, 1, out);
    free(own);
    return 0;
}

/* Big-M restatement (same algorithm as lpg_solve_big_m): artificial columns
 * art_first..N cost -M, kept as the M-part objective row. */
int lpo_solve_big_m(lpo_ctx *c, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                    lpo_result *out) {
    if (!c || c->nobj != 2 || art_first < 2 || art_first >= c->ncols) return -1;
    const int64_t N = c->ncols - 1;
    double *cr = (double *)malloc((size_t)N * sizeof(double));
    double *cm = (double *)calloc((size_t)N, sizeof(double));
    if (!cr || !cm) { free(cr); free(cm); return -1; }
    for (int64_t j = 1; j <= N; j++) cr[j - 1] = cost ? cost[j - 1] : -c->T[(c->m + 1) * c->ld + j];
    for (int64_t j = art_first; j <= N; j++) { cr[j - 1] = 0.0; cm[j - 1] = -1.0; }
    c->nact = N;
    lpo_set_objective_m(c, cm);
    lpo_set_objective(c, cr);
    free(cr); free(cm);
    lpo_result r;
    lpo_solve(c, max_pivots, rule, 1, &r);
    /* artificials still positive -> infeasible; also at UNBOUNDED: the pricing
     * takes a negative M part first, and such a column is never a ray (every
     * basic artificial would grow along it), so a ray found while the M
     * objective is still negative leaves the artificials positive for good */
    if (r.status == LPO_OPTIMAL || r.status == LPO_UNBOUNDED) {
        double bsum = 0;
        for (int64_t i = 0; i < c->m; i++) bsum += fabs(c->T[i * c->ld]);
        if (c->T[c->m * c->ld] < -1e-9 * (bsum > 1.0 ? bsum : 1.0)) r.status = LPO_INFEASIBLE;
    }
    if (out) *out = r;
    return 0;
}

/* Dual simplex restatement (same rules as lpg_solve_dual): leaving row =
 * most negative b_i < -eps_opt (ties: smallest row); entering column =
 * min d_j / (-a_rj) over a_rj < -eps_piv (ties: smallest j). */
int lpo_solve_dual(lpo_ctx *c, int64_t max_pivots, lpo_result *out) {
    if (!c || max_pivots < 0) return -1;
    const double *d = c->T + (c->m + c->nobj - 1) * c->ld;
    for (int64_t j = 1; j <= c->nact; j++)
        if (d[j] < -c->eps_opt) return -2;            /* not dual feasible */
    int status = LPO_RUNNING;
    int64_t done = 0;
    while (done < max_pivots) {
        int64_t r = -1; double br = 0.0;
        for (int64_t i = 0; i < c->m; i++) {
            const double b = c->T[i * c->ld];
            if (b < -c->eps_opt && (r < 0 || b < br)) { r = i; br = b; }
        }
        if (r < 0) { status = LPO_OPTIMAL; break; }
        int64_t k = -1; double best = 0.0;
        const double *row = c->T + r * c->ld;
        d = c->T + (c->m + c->nobj - 1) * c->ld;
        for (int64_t j = 1; j <= c->nact; j++) {
            const double a = row[j];
            if (!(a < -c->eps_piv)) continue;
            const double v = d[j] > 0.0 ? d[j] / -a : 0.0;
            if (k < 0 || v < best) { k = j; best = v; }
        }
        if (k < 0) { status = LPO_INFEASIBLE; break; }
        if (lpo_pivot(c, k, r) != 0) return -1;
        done++;
    }
    if (status == LPO_RUNNING) {                        /* peek, like the device's last step */
        int any = 0;
        for (int64_t i = 0; i < c->m; i++) any |= c->T[i * c->ld] < -c->eps_opt;
        status = any ? LPO_ITER_LIMIT : LPO_OPTIMAL;
    }
    if (out) {
        out->status = status;
        out->rule = LPO_RULE_DANTZIG;
        out->pivots = c->pivots;
        out->objective = c->T[(c->m + c->nobj - 1) * c->ld];
        out->entering = c->last_k;
        out->leaving = c->last_r;
    }
    return 0;
}
