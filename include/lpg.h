/*
 * lpg.h — C-ABI of the MI355X (gfx950) dense-tableau simplex pivot engine.
 *
 * This is the drop-in boundary for the pivot loop that the reference
 * (SomeBottle/LinearProgramming) is missing. The reference's solver driver
 * `void newSimplex(LPModel *model)` (Source/simplex.h:13, Source/simplex.c:27-73)
 * builds the tableau with
 *   `SimplexMatrix CreateSMatrix(LPModel *model, size_t **lack, short int *valid)`
 *   (Source/matrix.h:23, Source/matrix.c:19-91)
 * and frees it with `void RevokeSMatrix(SimplexMatrix *)` (matrix.h:25,
 * matrix.c:97-123) without ever pivoting (the loop belongs between
 * simplex.c:40 and simplex.c:65). Every entry point below replaces a piece of
 * that missing loop, or of the SimplexMatrix (matrix.h:13-21) storage it would
 * have run on; the binding a maintainer adds to simplex.c is in INTEGRATION.md.
 *
 * Tableau layout (row-major fp64, same as SimplexMatrix.cMatrix flattened):
 *   rows 0..m-1  constraint rows  [b_i | a_i1 .. a_iN]   (matrix.c:42-48, 62-66)
 *   row  m       objective row    [z   | d_1  .. d_N ]   d_j = z_j - c_j
 *   (LPG_FLAG_BIG_M: row m = M part, row m+1 = real part; d_j = dM_j M + dR_j)
 *   columns      0 = b, 1..N = variables in LPAlign order (simplex.c:238-260)
 * The reference maximises (LPStandardize turns min into max, simplex.c:99-106),
 * so the engine maximises; the optimum is reached when every d_j >= -eps_opt.
 *
 * Conventions follow the reference's C style: plain pointers and sizes, caller
 * owns host buffers (they are copied), the context owns device memory. Return
 * codes: 0 = success, < 0 = error (lpg_last_error has the text); a host
 * wrapper maps this onto the reference's `short int valid` (valid = rc == 0).
 * One context per host thread; not reentrant.
 *
 * Multi-GPU: one process per GPU. Each rank creates its context with
 * lpg_create_dist() and owns the row block [row0, row0 + nrows) of the m
 * constraint rows (row0 = floor(m*rank/world)); the objective row and the
 * basis are replicated. Per pivot the ranks exchange the ratio-test
 * candidates and the normalised pivot row. Default for world > 1 (round 3):
 * the owner push (lpg_comm_init_push*: the owner stores the row straight into
 * every rank's IPC-mapped buffer over xGMI, flag per chunk). With a
 * communicator only (or env LPG_EXCHANGE=rccl): RCCL collectives, an
 * allgather of the candidates and an allreduce of the owner's row and zeros
 * (= a broadcast from a device-resident root).
 */
#ifndef LPG_H
#define LPG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---- */
#define LPG_OK           0
#define LPG_ERR_ARG     -1
#define LPG_ERR_DEVICE  -2
#define LPG_ERR_OOM     -3
#define LPG_ERR_STATE   -4
#define LPG_ERR_COMM    -5

/* ---- solve status (SURVEY.md §5 failure detection) ---- */
#define LPG_RUNNING      0
#define LPG_OPTIMAL      1
#define LPG_UNBOUNDED    2
#define LPG_INFEASIBLE   3
#define LPG_ITER_LIMIT   4
#define LPG_NUMERIC      5

/* ---- pricing rules ---- */
#define LPG_RULE_DANTZIG 0   /* k = argmin d_j, ties -> smallest j; ratio ties -> smallest row */
#define LPG_RULE_BLAND   1   /* k = min{j : d_j < -eps}; ratio ties -> smallest basic column */

/* ---- synthetic generators (device-side) ---- */
#define LPG_GEN_DENSE      0  /* A_ij = u, b_i = n/8 (1+u), c_j = 1+u, <= rows, slack basis */
#define LPG_GEN_DEGENERATE 1  /* lower-triangular KM-style rows (a_ii = 1, a_ij = u/(i+1)), b_i = 0 on even rows */
#define LPG_GEN_DUAL       3  /* dual-simplex LP: min c.x, A x >= b (A = u, b = n/8 (1+u), c = 1+u) as
                                 rows [-b | -A | I], objective row [0 | c | 0] */
#define LPG_GEN_ARTIFICIAL 2  /* config 5: KM-style; even rows `<= 0` (a_ij = -u/(i+1)), odd rows equalities whose
                                 unit columns are artificials at columns 1+n+ceil(m/2) .. N */

/* ---- lpg_create flags ---- */
#define LPG_FLAG_NO_LOG  0x1u  /* do not record the (entering, leaving) pivot log */
#define LPG_FLAG_NO_SKIP 0x2u  /* update every column (no skipping of P[j] == 0 slices) */
#define LPG_FLAG_BIG_M   0x4u  /* two objective rows: row m = M part, row m+1 = real part (Big-M) */
#define LPG_FLAG_EAGER   0x8u  /* one rank-1 update pass per pivot instead of deferred (blocked) updates */

/* Deferred updates (default): the constraint rows are brought up to date in
 * one HBM pass per block of up to LPG_DEFER_MAX pivots. Default K (decided
 * from the largest rank's tableau bytes): 96 in region mode (lpg_info.region)
 * from 2 GB on one rank and from 1 GB on the ranks of a row partition, where
 * the region-mode slices hold 96 slots (config 3); 96 from 16 GB (the
 * two-kernel pair, config 4); 64 from 200 MB; 32 below. Env LPG_DEFER=K picks
 * K, K in 1 .. 128; 0 = eager. The persistent pivot kernel takes blocks of up
 * to 96 slots where its slices fit (lpg_info.pivot_wg > 0), else the pair
 * runs the pivots. Values,
 * pivot sequence and log are bitwise those of eager updates; every call that
 * reads or replaces the tableau (lpg_get_rows, lpg_get_column0, lpg_load_rows,
 * lpg_set_basis, lpg_set_objective*, lpg_sync, lpg_device_sync, the end of
 * lpg_solve) applies the pending block first. Single-rank contexts may keep the
 * columns in a different physical order between such calls (nonbasic columns
 * contiguous); every call that exposes or takes columns sees caller order. */
#define LPG_DEFER_MAX    128

typedef struct lpg_ctx lpg_ctx;

/* Same field layout as oracle/lpo.h's lpo_result. */
typedef struct {
    int32_t status;       /* LPG_* status */
    int32_t rule;         /* rule of the last solve */
    int64_t pivots;       /* pivots applied so far */
    double  objective;    /* T[m][0]: z without the objective constant (matrix.c:23-28) */
    int64_t entering;     /* last pivot's column (1-based, like cMatrix columns), -1 if none */
    int64_t leaving;      /* last pivot's row (0-based), -1 if none */
} lpg_result;

typedef struct {
    int64_t m, ncols, ld;       /* constraint rows, N+1 columns, row pitch (doubles) */
    int64_t row0, nrows;        /* this rank's constraint-row block */
    int32_t world, rank, device;
    int32_t nobj;               /* objective rows (1) */
    int32_t defer_k;            /* pivots per deferred block (0: eager updates) */
    int32_t pivot_wg;           /* workgroups of the persistent pivot kernel (one launch per run of
                                   pivots, lpg_block.hip); 0: two kernels per pivot */
    double  bytes_per_pivot;    /* algorithmic HBM bytes of one rank-1 update on this rank:
                                   16 * (nrows + nobj) * ncols (one read + one write) */
    int32_t exchange;           /* per-pivot exchange of a multi-rank context: 0 collectives (or none),
                                   1 owner push, 2 owner push into uncached exchange buffers */
    int32_t column_trade;       /* 1: the deferred path keeps the nonbasic columns contiguous (a column
                                   trade at every block's end; default from 2 GB per single rank, env
                                   LPG_NO_REORDER=0/1) */
    int32_t residency_fallbacks;  /* persistent pivot launches that found their grid (every rank's) not resident
                                     at once -- another kernel or process held CUs -- and handed the loop to the
                                     two-kernel pair (pivot_wg is 0 from then on) */
    int32_t region;             /* 1: the persistent pivot kernel runs in region mode -- its slices hold only the
                                   block start's nonbasic columns plus a spare slot per pending pivot for the
                                   column leaving the basis then (one rank, one objective row, column trade on;
                                   the default where it fits, env LPG_REGION=0 turns it off) */
    int32_t region_recoveries;  /* region-mode launches that found a block's column trade incomplete
                                   (DevState::rbad), ran no pivot and were re-run after a region rebuild */
} lpg_info_t;

typedef struct {
    double  update_ms;          /* summed device time of the update kernel (eager: rank-1 update per
                                   pivot; deferred: the block flush) */
    double  select_ms;          /* summed device time of pricing + ratio-test kernels (eager mode;
                                   deferred mode times the flushes only and reports 0) */
    double  comm_ms;            /* summed device time of the collectives */
    int64_t update_count;       /* update / flush launches timed */
    double  update_bytes;       /* bytes the update / flush kernels read + wrote (8 B x 2 per tableau
                                   entry in a column not skipped); eager: equals update_count *
                                   bytes_per_pivot when nothing is skipped */
} lpg_timing;

/* Host-staged collectives supplied by the caller (tests, non-RCCL transports).
 * Buffers are HOST memory; calls block until complete. */
typedef struct {
    void *user;
    int (*allgather)(void *user, const void *send, void *recv, size_t bytes_per_rank);
    int (*allreduce_sum_f64)(void *user, double *buf, size_t count);
} lpg_host_comm_ops;

/* ---- lifecycle ---- */
int  lpg_device_count(int *count);
/* Single-GPU engine for an m x ncols tableau (ncols = N+1).
 * Replaces the SimplexMatrix allocation of CreateSMatrix (matrix.c:33-48). */
int  lpg_create(lpg_ctx **out, int device, int64_t m, int64_t ncols, uint32_t flags);
/* One rank of a row-block partitioned engine; attach a communicator next. */
int  lpg_create_dist(lpg_ctx **out, int device, int world, int rank,
                     int64_t m, int64_t ncols, uint32_t flags);
int  lpg_comm_unique_id(void *uid, size_t len);              /* RCCL id, len >= 128 */
/* Attach an RCCL communicator (all ranks call it together). A world-1
 * context may attach one too: the per-pivot collectives then run for real on
 * a 1-rank communicator (used to test and time the exchange on one GPU). */
int  lpg_comm_init_rccl(lpg_ctx *ctx, const void *uid, size_t len);
int  lpg_comm_init_host(lpg_ctx *ctx, const lpg_host_comm_ops *ops);
/* Owner-push exchange for the deferred multi-rank loop (the north star's
 * pivot-row broadcast and candidate all-reduce, SURVEY.md §8(e), without a
 * collective per pivot): the owner of the pivot row stores it straight into
 * every rank's exchange buffer and raises per-chunk flags, every rank stores
 * its ratio candidates into every rank's buffer as self-validating tagged
 * words. Attach a communicator first (setup and bootstrap still use it),
 * then give every rank all ranks' buffers: IPC handles between processes
 * (lpg_comm_push_handle -> exchange -> lpg_comm_init_push), device pointers
 * between ranks of one process (lpg_comm_push_base -> lpg_comm_init_push_local).
 * Waits are bounded (2 s): a rank that waits longer ends the solve with
 * LPG_NUMERIC and lpg_last_error names the exchange. With the push attached,
 * each block (<= 96 pivots; region mode with K = 96 from 1 GB per rank, see
 * above) runs as one persistent launch per block on every
 * rank (lpg_info.pivot_wg > 0; each rank needs its own GPU, or launches
 * small enough to be resident together; env LPG_PERSIST_MR=0: two kernels
 * per pivot). The exchange's kernels spin-wait on their peers, so attaching
 * is refused (LPG_ERR_STATE, lpg_last_error names the reason) when ranks
 * would depend on each other for hardware queues or CUs: ranks that are
 * threads of one process (lpg_comm_init_push_local, world > 1), or ranks of
 * several processes on one GPU (same PCI bus id). Nothing has pivoted then:
 * the caller keeps the collectives. Env LPG_PUSH_SHARED_QUEUES=1 /
 * LPG_PUSH_SHARED_DEVICE=1 acknowledge the sharing (tests on one GPU). */
#define LPG_PUSH_HANDLE_BYTES 64
int  lpg_comm_push_handle(lpg_ctx *ctx, void *handle, size_t len);
int  lpg_comm_push_base(lpg_ctx *ctx, void **base);
int  lpg_comm_init_push(lpg_ctx *ctx, const void *handles, size_t len);
int  lpg_comm_init_push_local(lpg_ctx *ctx, void *const *bases, int world);
/* Replaces RevokeSMatrix (matrix.c:97-123). NULL is a no-op. */
void lpg_destroy(lpg_ctx *ctx);
int  lpg_info(const lpg_ctx *ctx, lpg_info_t *out);
const char *lpg_last_error(const lpg_ctx *ctx);
/* The source stamp this library was built from (16 hex digits: sha256 over
 * the engine's csrc/ files and this header, linearprogramming_amd/_stamp.py).
 * No reference counterpart: a loader compares it with the sources beside the
 * library and refuses a stale binary. */
const char *lpg_build_stamp(void);

/* ---- loading (host buffers are copied) ---- */
/* Rows [row0, row0+nrows) in GLOBAL numbering, each [b | a_1..a_N] with pitch
 * ld >= ncols. Row index m is the objective row. Rows outside this rank's
 * block are skipped. Replaces CreateSMatrix's cell fill (matrix.c:42-66). */
int  lpg_load_rows(lpg_ctx *ctx, int64_t row0, int64_t nrows, const double *rows, int64_t ld);
/* basis[i] = 1-based column of row i's basic variable (all m rows, every
 * rank). Replaces SimplexMatrix.basicVars (matrix.c:67-78). */
int  lpg_set_basis(lpg_ctx *ctx, const int64_t *basis);
/* Objective row from costs c[0..N-1] of `max c.x` and the current basis:
 * d_j = sum_i c_B(i) T[i][j] - c_j, z = sum_i c_B(i) b_i, summed in global
 * row order with fma (bitwise independent of the partition). Replaces
 * SimplexMatrix.ofCosts / basicCosts (matrix.c:55-57, 76-77). The pivot
 * count and log are kept (phase I -> phase II). */
int  lpg_set_objective(lpg_ctx *ctx, const double *c);
/* Big-M contexts: the M-part objective row from M-part costs (the real row
 * comes from lpg_set_objective). */
int  lpg_set_objective_m(lpg_ctx *ctx, const double *costM);
int  lpg_set_tolerances(lpg_ctx *ctx, double eps_piv, double eps_opt);
/* Price only columns 1..nact (e.g. to exclude artificials). */
int  lpg_set_active_columns(lpg_ctx *ctx, int64_t nact);
/* Device-side synthetic LP with n structural columns (ncols == n + m + 1). */
int  lpg_generate(lpg_ctx *ctx, int64_t n, uint64_t seed, int kind);

/* ---- the pivot loop (the part simplex.c:40-65 lacks) ---- */
/* Pivot until optimal / unbounded / numeric trouble or max_pivots more
 * pivots; blocks; fills *out. A status of LPG_ITER_LIMIT means the budget
 * ran out first. */
int  lpg_solve(lpg_ctx *ctx, int64_t max_pivots, int rule, lpg_result *out);
/* Asynchronous form for benchmarking: enqueue exactly npivots pivots on the
 * context's stream without any host synchronisation (pivots after the LP
 * finishes are no-ops on the device); lpg_sync waits and reports. */
int  lpg_enqueue(lpg_ctx *ctx, int64_t npivots, int rule);
/* Waits for everything enqueued, applies any pending deferred block (so the
 * tableau is current) and reports. */
int  lpg_sync(lpg_ctx *ctx, lpg_result *out);
/* Pre-size the device pivot log for npivots more pivots so that no
 * reallocation (and host synchronisation) happens inside a timed region. */
int  lpg_reserve_log(lpg_ctx *ctx, int64_t npivots);
/* Build, ahead of the pivot loop, the replayed HIP graph that lpg_enqueue /
 * lpg_solve use for runs of at least two blocks under this rule (capture +
 * instantiate, ~0.5 ms of host time), so that it does not land inside a timed
 * region. No pivot runs; a pending deferred block is applied first. A no-op
 * where the loop does not replay graphs (graphs disabled, eager timing, a
 * host communicator). */
int  lpg_prepare(lpg_ctx *ctx, int rule);

/* Apply one caller-chosen pivot (entering column k, 1-based; leaving row r,
 * 0-based) with the same arithmetic as the loop; |T[r][k]| must exceed
 * eps_piv (either sign). Counts as a pivot and is logged. On a row partition
 * every rank calls it with the same (k, r). */
int  lpg_pivot(lpg_ctx *ctx, int64_t k, int64_t r);
/* Two-phase method for a tableau whose columns art_first..N are artificial
 * unit columns basic in the rows that lacked an identity column
 * (reference: the empty `case 2:` of simplex.c:61-62, lack list from
 * matrix.c:80-89). Phase I maximises -sum(artificials); a negative optimum
 * means LPG_INFEASIBLE. Artificials left basic at zero are pivoted out on the
 * first usable original column of their row. Phase II prices columns
 * 1..art_first-1 only, with the objective row recomputed from cost[0..N-1]
 * (cost NULL: -1 x the objective row as loaded, i.e. a slack-form -c row).
 * On a row partition every rank calls it with the same arguments (it is
 * collective): the |b| sum of the feasibility test runs over the ranks in
 * global row order, and each artificial row's owner finds its column and
 * shares it through the communicator before every rank pivots (round 3). */
int  lpg_solve_two_phase(lpg_ctx *ctx, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                         lpg_result *out);

/* Big-M method (reference: the empty `case 1:` of simplex.c:58-60, constant
 * M of dataReader.c:165-173) on a LPG_FLAG_BIG_M context: artificial columns
 * art_first..N cost -M, kept symbolic as a second objective row, so pricing
 * is lexicographic (M part first) exactly like the reference's Number with a
 * constant (numOprts.h:15-37); no numeric M is ever formed. An optimum with a
 * negative M part means LPG_INFEASIBLE. cost NULL: -1 x the real objective
 * row as loaded. */
int  lpg_solve_big_m(lpg_ctx *ctx, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                     lpg_result *out);

/* Dual simplex (reference: router option 2, router.c:32-34, a no-op; the
 * tableau LPStandardize(model, 1) builds by flipping >= rows, simplex.c:178-179).
 * Needs a dual-feasible basis (every d_j >= -eps_opt, else LPG_ERR_STATE).
 * Leaving row: most negative b_i < -eps_opt (ties: smallest row); entering
 * column: min d_j / (-a_rj) over a_rj < -eps_piv (ties: smallest j); none ->
 * LPG_INFEASIBLE; no negative b -> LPG_OPTIMAL. Same update kernel and
 * arithmetic as the primal loop. On a row partition (round 3) every rank
 * calls it (collective) and the deferred form runs: the row candidates are
 * allgathered and the leaving row is summed from its owner; LPG_FLAG_EAGER
 * is single rank. */
int  lpg_solve_dual(lpg_ctx *ctx, int64_t max_pivots, lpg_result *out);

/* ---- readout ---- */
int  lpg_get_rows(lpg_ctx *ctx, int64_t row0, int64_t nrows, double *out, int64_t ld);
int  lpg_get_basis(lpg_ctx *ctx, int64_t *basis);            /* m entries */
int  lpg_get_column0(lpg_ctx *ctx, double *xB);               /* local rows' b (x_B) */
int64_t lpg_get_log(lpg_ctx *ctx, int64_t *k, int64_t *r, int64_t max);

/* ---- measurement ---- */
int  lpg_set_timing(lpg_ctx *ctx, int enable);
int  lpg_get_timing(lpg_ctx *ctx, lpg_timing *out);          /* syncs; resets the sums */
int  lpg_device_sync(lpg_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
