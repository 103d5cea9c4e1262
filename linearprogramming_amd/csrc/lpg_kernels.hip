// lpg_kernels.hip — gfx950 kernels of the dense-tableau simplex pivot engine.
//
// One pivot t = prep_t -> select_t -> update_t on one stream (plus, with
// world > 1, an allreduce of P after prep and an allgather of the ratio
// candidates after select). The arithmetic is the bitwise contract of
// oracle/lpo.h (built with -ffp-contract=off; every fused multiply-add below
// is an explicit fma):
//   P[j]    = T[r][j] / T[r][k]
//   T[i][j] = fma(-C[i], P[j], T[i][j])   for i != r,   T[r][j] = P[j]
// Reference anchors: the loop these kernels implement is absent upstream
// (Source/simplex.c:40 -> :65); the tableau they run on is SimplexMatrix
// (Source/matrix.h:13-21) with column 0 = b (Source/matrix.c:42-48).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stddef.h>
#include <stdlib.h>

#include <algorithm>

#include "lpg_internal.h"
#include "lpg_device.h"

namespace lpg {

// ------------------------------------------------------------------------
// synthetic generator (bitwise identical to oracle lpo_generate)
// ------------------------------------------------------------------------

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double uniform01(uint64_t key, uint64_t idx) {
    return (double)(splitmix64(key ^ (idx * 0x9E3779B97F4A7C15ull)) >> 11) * 0x1.0p-53;
}

static inline uint64_t splitmix64_host(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t subkey(uint64_t seed, uint64_t which) {
    return splitmix64_host(seed ^ (which * 0xD1B54A32D192ED03ull));
}

// Column of row i's initial unit column (oracle lpo_unit_column): kinds 0/1
// slack 1+n+i; kind 2 slacks of even rows first, then the artificials of the
// odd (equality) rows from art_first = 1+n+ceil(m/2).
__host__ __device__ __forceinline__ int64_t unit_column(int64_t m, int64_t n, int64_t i, int kind) {
    if (kind != 2) return 1 + n + i;
    return (i & 1) ? 1 + n + (m + 1) / 2 + i / 2 : 1 + n + i / 2;
}

// grid: x = local row, y = chunk of 512 columns (256 lanes x 2). Every rank
// fills all m basis entries (slack basis) through k_basis_slack.
__global__ __launch_bounds__(kBlock) void k_generate(double *__restrict__ T, Geo g, int64_t n, uint64_t kA,
                                                     uint64_t kB, uint64_t kC, int kind) {
    const int64_t i = blockIdx.x;
    const int64_t j0 = ((int64_t)blockIdx.y * kBlock + threadIdx.x) * 2;
    if (j0 >= g.ld) return;
    double *row = T + i * g.ld;
    const double bscale = (double)n / 8.0;
    double v[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int64_t j = j0 + e;
        double x = 0.0;
        if (i < g.nloc) {
            const int64_t gi = g.row0 + i;
            if (j == 0) {
                if (kind == 0 || kind == 3 || (gi & 1))
                    x = bscale * (1.0 + uniform01(kB, (uint64_t)gi));
                if (kind == 3) x = -x;
            } else if (j <= n) {
                const int64_t jj = j - 1;
                if (kind == 0 || kind == 3) {
                    x = uniform01(kA, (uint64_t)(gi * n + jj));
                    if (kind == 3) x = -x;
                } else {
                    const double sgn = (kind == 2 && !(gi & 1)) ? -1.0 : 1.0;
                    if (jj < gi) x = sgn * (uniform01(kA, (uint64_t)(gi * n + jj)) / (double)(gi + 1));
                    else if (jj == gi) x = 1.0;
                }
            } else if (j == unit_column(g.m, n, gi, kind)) {
                x = 1.0;
            }
        } else if (i == g.nloc + g.nobj - 1) {   // (real) objective row; a Big-M M row stays zero
            if (j >= 1 && j <= n) {
                x = 1.0 + uniform01(kC, (uint64_t)(j - 1));
                if (kind != 3) x = -x;            // kind 3: max -c.x, d_j = +c_j (dual feasible)
            }
        }
        v[e] = x;
    }
    *(d2 *)(row + j0) = d2{v[0], v[1]};
}

__global__ void k_basis_slack(int64_t *__restrict__ basis, int64_t m, int64_t n, int kind) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < m) basis[i] = unit_column(m, n, i, kind);
}

int launch_generate(const Launch &L, const Geo &g, int64_t n, uint64_t seed, int kind, int64_t *basis_dev) {
    hipStream_t st = (hipStream_t)L.stream;
    const int64_t rows = g.nloc + g.nobj;
    const int64_t chunks = (g.ld / 2 + kBlock - 1) / kBlock;
    if (rows > 0x7fffffff || chunks > 65535) return -1;
    dim3 grid((unsigned)rows, (unsigned)chunks);
    hipLaunchKernelGGL(k_generate, grid, dim3(kBlock), 0, st, g.T, g, n, subkey(seed, 1), subkey(seed, 2),
                       subkey(seed, 3), kind);
    hipLaunchKernelGGL(k_basis_slack, dim3((unsigned)((g.m + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       basis_dev, g.m, n, kind);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// objective row from costs: d_j = sum_i cB_i T[i][j] - c_j, chained across
// ranks in global row order (acc_in = previous rank's partial chain)
// ------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void k_objective_chain(const double *__restrict__ T, Geo g,
                                                            const double *__restrict__ cb,
                                                            const double *__restrict__ acc_in,
                                                            double *__restrict__ acc_out) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= g.ncols) return;
    double acc = acc_in ? acc_in[j] : 0.0;
    for (int64_t i = 0; i < g.nloc; i++) acc = fma(cb[i], T[i * g.ld + j], acc);
    acc_out[j] = acc;
}

__global__ __launch_bounds__(kBlock) void k_objective_finish(double *__restrict__ T, Geo g,
                                                             const double *__restrict__ acc,
                                                             const double *__restrict__ cost, int64_t orow) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= g.ld) return;
    double *obj = T + orow * g.ld;
    obj[j] = j == 0 ? acc[0] : (j < g.ncols ? acc[j] - cost[j - 1] : 0.0);
}

int launch_objective_chain(const Launch &L, const Geo &g, const double *cb, const double *acc_in,
                           double *acc_out) {
    hipLaunchKernelGGL(k_objective_chain, dim3((unsigned)((g.ncols + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)L.stream, g.T, g, cb, acc_in, acc_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_objective_finish(const Launch &L, const Geo &g, const double *acc, const double *cost, int64_t orow) {
    hipLaunchKernelGGL(k_objective_finish, dim3((unsigned)((g.ld + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)L.stream, g.T, g, acc, cost, orow);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// pricing (a10). mode 0: price the objective row as stored (bootstrap);
// mode 1: price d_{t+1} = fma(-C_t[obj], P_t[j], d_t[j]) before the update
// writes it (multi-GPU path, after the allreduce of P).
// ------------------------------------------------------------------------

int price_blocks(const Geo &g) {
    const int64_t nvec = (g.ncols + 1) / 2;
    return (int)((nvec + kBlock - 1) / kBlock);
}

// Number of 16-byte slices of P that are not all zero (the slices k_update
// will read and write): per-block counts, summed once per pivot by k_select.
__device__ __forceinline__ void count_live(int *__restrict__ pc, bool live) {
    const int n = __syncthreads_count(live);
    if (threadIdx.x == 0) pc[blockIdx.x] = n;
}

// colmap / inv (deferred multi-rank path with reordered columns, lpg_internal.h):
// the pricing keys are logical (colmap of the physical column), as in
// k_prep_d; the block winner's physical column comes back through inv.
template <int RULE, int MODE>
__global__ __launch_bounds__(kBlock) void k_price(double *__restrict__ T, Geo g,
                                                  const DevState *__restrict__ st, int s,
                                                  const double *__restrict__ P, const double *__restrict__ Cs,
                                                  PricePart *__restrict__ pp, int *__restrict__ pc, int defer,
                                                  const int32_t *__restrict__ colmap, const int32_t *__restrict__ inv) {
    if (MODE == 1 && st->slot[s].status != RUNNING) return;
    const int64_t j2 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t nvec = (g.ncols + 1) / 2;
    PricePart best{0.0, -1, 0, 0};
    bool live = false;
    if (j2 < nvec) {
        const int64_t rM = g.nloc, rR = g.nloc + g.nobj - 1;   // M-part row (Big-M) and real row
        d2 dM = *(const d2 *)(T + rM * g.ld + 2 * j2);
        d2 dR = *(const d2 *)(T + rR * g.ld + 2 * j2);
        if (MODE == 1) {
            const d2 p = *(const d2 *)(P + 2 * j2);
            const double cM = -Cs[rM], cR = -Cs[rR];
            dM.x = fma(cM, p.x, dM.x);
            dM.y = fma(cM, p.y, dM.y);
            dR.x = fma(cR, p.x, dR.x);
            dR.y = fma(cR, p.y, dR.y);
            live = p.x != 0.0 || p.y != 0.0;
            if (defer) {   // deferred mode keeps the objective row(s) current
                *(d2 *)(T + rR * g.ld + 2 * j2) = dR;
                if (g.nobj == 2) *(d2 *)(T + rM * g.ld + 2 * j2) = dM;
            }
        }
        const int2 lj = colmap ? ((const int2 *)colmap)[j2] : int2{(int)(2 * j2), (int)(2 * j2 + 1)};
        price_one<RULE>(best, dM.x, dR.x, lj.x, g);
        price_one<RULE>(best, dM.y, dR.y, lj.y, g);
    }
    if (MODE == 1) count_live(pc, live);
    best = block_argmin_pp<RULE>(best);   // unique keys: no struct selects (see below)
    // pad (the physical column) == j in caller order. Set it here: hipcc
    // (ROCm 7.2) miscompiled the pad field of the inlined price_one's
    // "if (better) best = c" in this kernel (pad kept the previous best's
    // value while v, j, cls took the new one), which sent k_select_d to the
    // neighbouring column under a communicator.
    if (threadIdx.x == 0) {
        best.pad = (int32_t)(best.j >= 0 && inv ? inv[best.j] : best.j);
        pp[blockIdx.x] = best;
    }
}

int launch_price(const Launch &L, const Geo &g, int rule, int mode, const DevState *st, int s,
                 const double *P, const double *Cs, PricePart *pp, int *pc, int npp, bool defer,
                 const int32_t *colmap, const int32_t *inv) {
    hipStream_t stream = (hipStream_t)L.stream;
    dim3 grid(npp), blk(kBlock);
    const int d = defer ? 1 : 0;
    if (rule == RULE_BLAND) {
        if (mode == 0) hipLaunchKernelGGL((k_price<RULE_BLAND, 0>), grid, blk, 0, stream, g.T, g, st, s, P, Cs, pp, pc, d, colmap, inv);
        else hipLaunchKernelGGL((k_price<RULE_BLAND, 1>), grid, blk, 0, stream, g.T, g, st, s, P, Cs, pp, pc, d, colmap, inv);
    } else {
        if (mode == 0) hipLaunchKernelGGL((k_price<RULE_DANTZIG, 0>), grid, blk, 0, stream, g.T, g, st, s, P, Cs, pp, pc, d, colmap, inv);
        else hipLaunchKernelGGL((k_price<RULE_DANTZIG, 1>), grid, blk, 0, stream, g.T, g, st, s, P, Cs, pp, pc, d, colmap, inv);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// prep_t: leaving row from the gathered ratio candidates, normalised pivot
// row P (owner rank; zeros elsewhere), and — single rank — the pricing of
// d_{t+1} fused in (it only needs P and the objective row).
// ------------------------------------------------------------------------

template <int RULE, bool FUSE, bool DEFER>
__global__ __launch_bounds__(kBlock) void k_prep(double *__restrict__ T, Geo g, DevState *st, int s,
                                                 const Cand *__restrict__ cand, int ncand,
                                                 double *__restrict__ P, const double *__restrict__ Cs,
                                                 PricePart *__restrict__ pp, int *__restrict__ pc, Defer D) {
    const int64_t j2 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t nvec = (g.ncols + 1) / 2;
    // with a communicator (!FUSE) an allreduce of P follows even when no pivot
    // runs (the loop ended): send its identity, not the previous pivot's row
    auto no_pivot = [&]() {
        if (!FUSE && j2 < nvec) *(d2 *)(P + 2 * j2) = d2{-0.0, -0.0};
    };
    if (st->slot[s].status != RUNNING) {
        no_pivot();
        return;
    }
    Cand best{0.0, 0.0, 0, -1};
    for (int q = threadIdx.x; q < ncand; q += kBlock) {
        const Cand c = cand[q];
        cand_take(best, c, cand_better(c, best));
    }
    best = block_reduce_cand(best);
    // the oracle's rule (oracle/lpo.c lpo_solve): NUMERIC iff the pivot element or
    // the row's b is not finite (a non-finite b arrives as piv = NaN); an
    // overflowing ratio b / a is an ordinary (largest) candidate
    if (best.row < 0 || !isfinite(best.piv)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = best.row < 0 ? UNBOUNDED : NUMERIC;
            st->slot[s].r = -1;
        }
        no_pivot();
        return;
    }
    const int64_t rl = best.row - g.row0;
    const bool own = rl >= 0 && rl < g.nloc;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->slot[s].r = best.row;
        st->work[s] = 0;   // k_update's dequeue head for this pivot (runs after this kernel)
        if (DEFER) {       // no per-pivot update kernel: the pivot is booked here
            const int64_t k = st->slot[s].k;
            D.rq[D.q] = own ? rl : -1;
            st->npend = D.q + 1;
            D.basis[best.row] = k;
            const int64_t n = st->pivots;
            if (D.logk && n < st->logcap) {
                D.logk[n] = k;
                D.logr[n] = best.row;
            }
            st->pivots = n + 1;
            st->last_k = k;
            st->last_r = best.row;
        }
    }
    const double piv = best.piv;   // == T_t[r][k_t] (select_{t-1} computed and stored it)
    d2 t = d2{0.0, 0.0};           // the pivot row as stored (issued before the staging barrier)
    if (own && j2 < nvec) t = *(const d2 *)(T + rl * g.ld + 2 * j2);
    __shared__ double s_c[LPG_DEFER_MAX];
    __shared__ int64_t s_rq[LPG_DEFER_MAX];
    if (DEFER && own) {            // the chain's per-pivot scalars, staged once per block
        for (int q = threadIdx.x; q < D.q; q += kBlock) {
            s_rq[q] = D.rq[q];
            s_c[q] = -D.Cbuf[(int64_t)q * D.cs + rl];
        }
        __syncthreads();
    }

    PricePart pbest{0.0, -1, 0, 0};
    bool live = false;
    if (j2 < nvec) {
        // a rank that does not hold row r contributes -0, the identity of the
        // allreduce that follows (+0 would turn an owner's -0 into +0)
        d2 p = (FUSE || own) ? d2{0.0, 0.0} : d2{-0.0, -0.0};
        if (own) {
            if (DEFER) {   // row r of the current tableau: the pending chain
                // chunks of 16 pending rows: all loads of a chunk in flight at once
                for (int q0 = 0; q0 < D.q; q0 += 16) {
                    d2 pq[16];
#pragma unroll
                    for (int u = 0; u < 16; u++)
                        if (q0 + u < D.q) pq[u] = *(const d2 *)(D.Pbuf + (int64_t)(q0 + u) * g.ld + 2 * j2);
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        const int q = q0 + u;
                        if (q < D.q) {
                            if (s_rq[q] == rl) {
                                t = pq[u];
                            } else {
                                const double c = s_c[q];
                                t.x = fma(c, pq[u].x, t.x);
                                t.y = fma(c, pq[u].y, t.y);
                            }
                        }
                    }
                }
            }
            p.x = t.x / piv;
            p.y = t.y / piv;
        }
        *(d2 *)(P + 2 * j2) = p;
        if (FUSE) {
            const int64_t rM = g.nloc, rR = g.nloc + g.nobj - 1;
            d2 dM = *(const d2 *)(T + rM * g.ld + 2 * j2);
            d2 dR = *(const d2 *)(T + rR * g.ld + 2 * j2);
            const double cM = -Cs[rM], cR = -Cs[rR];
            dM.x = fma(cM, p.x, dM.x);
            dM.y = fma(cM, p.y, dM.y);
            dR.x = fma(cR, p.x, dR.x);
            dR.y = fma(cR, p.y, dR.y);
            if (DEFER) {   // the objective row(s) stay current
                *(d2 *)(T + rR * g.ld + 2 * j2) = dR;
                if (g.nobj == 2) *(d2 *)(T + rM * g.ld + 2 * j2) = dM;
            }
            price_one<RULE>(pbest, dM.x, dR.x, 2 * j2, g);
            price_one<RULE>(pbest, dM.y, dR.y, 2 * j2 + 1, g);
            live = p.x != 0.0 || p.y != 0.0;
        }
    }
    if (FUSE) {
        count_live(pc, live);
        pbest = block_reduce_pp<RULE>(pbest);
        pbest.pad = (int32_t)pbest.j;    // caller order (see k_price)
        if (threadIdx.x == 0) pp[blockIdx.x] = pbest;
    }
}

int launch_prep(const Launch &L, const Geo &g, int rule, bool fuse, DevState *st, int s, const Cand *cand,
                int ncand, double *P, const double *Cs, PricePart *pp, int *pc, int npp, const Defer &D) {
    hipStream_t stream = (hipStream_t)L.stream;
    dim3 grid(npp), blk(kBlock);
#define LPG_PREP(R, F, DF) \
    hipLaunchKernelGGL((k_prep<R, F, DF>), grid, blk, 0, stream, g.T, g, st, s, cand, ncand, P, Cs, pp, pc, D)
    if (rule == RULE_BLAND) {
        if (D.on) { if (fuse) LPG_PREP(RULE_BLAND, true, true); else LPG_PREP(RULE_BLAND, false, true); }
        else { if (fuse) LPG_PREP(RULE_BLAND, true, false); else LPG_PREP(RULE_BLAND, false, false); }
    } else {
        if (D.on) { if (fuse) LPG_PREP(RULE_DANTZIG, true, true); else LPG_PREP(RULE_DANTZIG, false, true); }
        else { if (fuse) LPG_PREP(RULE_DANTZIG, true, false); else LPG_PREP(RULE_DANTZIG, false, false); }
    }
#undef LPG_PREP
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// select_t (a10 finish + a11): entering column k_{t+1} from the pricing
// partials, then the ratio test on T_{t+1}'s columns 0 and k_{t+1}, computed
// from T_t with the same fma the update will apply (the update runs after
// this kernel, so T still holds T_t). Also stores C_{t+1} = T_{t+1}[:, k].
// FIRST: bootstrap on the tableau as loaded (no pending pivot).
// ------------------------------------------------------------------------

template <int RULE, bool FIRST, bool DEFER>
__global__ __launch_bounds__(kBlock) void k_select(const double *__restrict__ T, Geo g, DevState *st, int s,
                                                   int s1, const double *__restrict__ P,
                                                   const double *__restrict__ Cs, double *__restrict__ Cs1,
                                                   const PricePart *__restrict__ pp, int npp,
                                                   const int64_t *__restrict__ basis, Cand *__restrict__ part,
                                                   int64_t force_k, int64_t force_r,
                                                   const int *__restrict__ pc, int skip, Defer D) {
    Slot *dst = &st->slot[s1];
    if (!FIRST) {
        const int32_t stt = st->slot[s].status;
        if (stt != RUNNING) {
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                dst->status = stt;
                dst->k = -1;
                dst->r = -1;
            }
            return;
        }
    }
    if (DEFER && !FIRST) {
        // pivot t is pending: keep its column C_t for the chain and the flush
        for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < g.nloc; i += (int64_t)gridDim.x * kBlock)
            D.Cbuf[(int64_t)D.q * D.cs + i] = Cs[i];
    }
    if (!FIRST && !DEFER && blockIdx.x == 0) {
        // the update of this pivot (next on the stream) touches the live
        // slices of P (all slices without column skipping) in every row
        const int64_t nvec = (g.ncols + 1) / 2;
        int64_t live = 0;
        if (skip)
            for (int q = threadIdx.x; q < npp; q += kBlock) live += pc[q];
        else if (threadIdx.x == 0)
            live = nvec;
#pragma unroll
        for (int mask = 32; mask > 0; mask >>= 1) live += __shfl_xor((long long)live, mask, 64);
        __shared__ int64_t wsum[kBlock / 64];
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = live;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tot = 0;
            for (int w = 0; w < kBlock / 64; w++) tot += wsum[w];
            st->touched += 2ull * (unsigned long long)tot * (unsigned long long)(g.nloc + g.nobj);
        }
    }
    PricePart pb{0.0, -1, 0, 0};
    if (force_k > 0) {              // forced pivot (lpg_pivot): no pricing
        pb.j = force_k;
        pb.v = -1.0;
    } else {
        for (int q = threadIdx.x; q < npp; q += kBlock) {
            const PricePart c = pp[q];
            pp_take(pb, c, pp_better<RULE>(c, pb));
        }
        pb = block_reduce_pp<RULE>(pb);
    }
    const bool optimal = pb.j < 0;   // only eligible columns (d_j < 0, lexicographically) are candidates
    if (optimal) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            dst->status = OPTIMAL;
            dst->k = -1;
            dst->r = -1;
        }
        return;
    }
    const int64_t kn = pb.j;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dst->status = RUNNING;
        dst->k = kn;
    }
    int64_t rl = -1, kc = 0, r = -1;
    double p0 = 0.0, pk = 0.0;
    if (!FIRST) {
        r = st->slot[s].r;
        kc = st->slot[s].k;
        rl = (r >= g.row0 && r < g.row0 + g.nloc) ? r - g.row0 : -1;
        p0 = P[0];
        pk = P[kn];
    }
    // this thread's first row: its two tableau loads go out before the staging barrier
    const int64_t ifirst = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t nrows = g.nloc + g.nobj;
    double ob0 = 0.0, oa0 = 0.0;
    if (ifirst < nrows) {
        ob0 = T[ifirst * g.ld];
        oa0 = T[ifirst * g.ld + kn];
    }
    __shared__ double s_p0[LPG_DEFER_MAX + 1], s_pk[LPG_DEFER_MAX + 1];
    __shared__ int64_t s_rq[LPG_DEFER_MAX + 1];
    if (DEFER && !FIRST) {          // the chain's per-pivot scalars, staged once per block
        for (int q = threadIdx.x; q <= D.q; q += kBlock) {
            const double *Pq = D.Pbuf + (int64_t)q * g.ld;
            s_p0[q] = Pq[0];
            s_pk[q] = Pq[kn];
            s_rq[q] = D.rq[q];
        }
        __syncthreads();
    }
    Cand best{0.0, 0.0, 0, -1};
    for (int64_t i = ifirst; i < nrows; i += (int64_t)gridDim.x * kBlock) {
        const double ob = i == ifirst ? ob0 : T[i * g.ld];
        const double oa = i == ifirst ? oa0 : T[i * g.ld + kn];
        double b, a;
        if (FIRST) {
            b = ob;
            a = oa;
        } else if (DEFER) {
            if (i >= g.nloc) {          // objective rows are current (prep / price wrote d_{t+1})
                b = ob;
                a = oa;
            } else {                    // columns 0 and k_{t+1}: chain over pivots 0..q
                b = ob;
                a = oa;
                // chunks of 32 pending pivots: all multiplier loads of a chunk in flight at once
                for (int q0 = 0; q0 < D.q; q0 += 32) {
                    double cv[32];
#pragma unroll
                    for (int u = 0; u < 32; u++)
                        if (q0 + u < D.q) cv[u] = D.Cbuf[(int64_t)(q0 + u) * D.cs + i];
#pragma unroll
                    for (int u = 0; u < 32; u++) {
                        const int q = q0 + u;
                        if (q < D.q) {
                            if (i == s_rq[q]) {
                                b = s_p0[q];
                                a = s_pk[q];
                            } else {
                                b = fma(-cv[u], s_p0[q], b);
                                a = fma(-cv[u], s_pk[q], a);
                            }
                        }
                    }
                }
                if (i == s_rq[D.q]) {       // pivot t itself: C_t is Cs
                    b = s_p0[D.q];
                    a = s_pk[D.q];
                } else {
                    const double c = -Cs[i];
                    b = fma(c, s_p0[D.q], b);
                    a = fma(c, s_pk[D.q], a);
                }
            }
        } else if (i == rl) {
            b = p0;
            a = pk;
        } else {
            const double c = -Cs[i];
            b = fma(c, p0, ob);
            a = fma(c, pk, oa);
        }
        Cs1[i] = a;
        const bool eligible = force_r >= 0 ? (g.row0 + i == force_r && fabs(a) > g.eps_piv) : a > g.eps_piv;
        if (i < g.nloc && eligible) {
            const int64_t grow = g.row0 + i;
            Cand c;
            c.theta = b > 0.0 ? b / a : 0.0;
            c.piv = isfinite(b) ? a : __longlong_as_double(0x7ff8000000000000ll);   // b_r not finite: NUMERIC at prep
            c.row = grow;
            c.key = RULE == RULE_BLAND ? (grow == r ? kc : basis[grow]) : grow;
            cand_take(best, c, cand_better(c, best));
        }
    }
    best = block_reduce_cand(best);
    if (threadIdx.x == 0) part[blockIdx.x] = best;
}

int launch_select(const Launch &L, const Geo &g, int rule, bool first, DevState *st, int s, int s1, const double *P,
                  const double *Cs, double *Cs1, const PricePart *pp, int npp, const int64_t *basis, Cand *part,
                  int nsel, int64_t force_k, int64_t force_r, const int *pc, int skip, const Defer &D) {
    hipStream_t stream = (hipStream_t)L.stream;
    dim3 grid(nsel), blk(kBlock);
#define LPG_SEL(R, F, DF)                                                                                     \
    hipLaunchKernelGGL((k_select<R, F, DF>), grid, blk, 0, stream, g.T, g, st, s, s1, P, Cs, Cs1, pp, npp, basis, \
                       part, force_k, force_r, pc, skip, D)
    if (rule == RULE_BLAND) {
        if (first) LPG_SEL(RULE_BLAND, true, false);
        else if (D.on) LPG_SEL(RULE_BLAND, false, true);
        else LPG_SEL(RULE_BLAND, false, false);
    } else {
        if (first) LPG_SEL(RULE_DANTZIG, true, false);
        else if (D.on) LPG_SEL(RULE_DANTZIG, false, true);
        else LPG_SEL(RULE_DANTZIG, false, false);
    }
#undef LPG_SEL
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// Deferred-mode pivot kernels without a communicator (the default path):
// the same arithmetic as k_prep<FUSE, DEFER> / k_select<DEFER>, with every
// load that does not depend on this pivot's choices issued at kernel start,
// so that each kernel has two dependent memory round trips instead of five
// (prep: [status, candidates, pending P rows, objective rows] -> [pivot row,
// its multipliers]; select: [status, pricing partials, pending multipliers,
// column 0] -> [column k, P_q[k]]). At most kPF pending pivots are
// prefetched (kPF = the chain length rounded up to 16, at most 64; one block
// per CU at most, so the registers are there); longer chains would load the
// rest in the chain.
// ------------------------------------------------------------------------

#ifdef LPG_PHASES
// Phase probe (tools/phase_probe.py, built into tools/liblpg_phases.so only):
// s_memrealtime (100 MHz) stamps of block 0's thread 0 at phase boundaries,
// plus the earliest start and latest end over all blocks.
__device__ unsigned long long g_ph[2][16];
#define LPG_PH(kern, k)                                                                  \
    do {                                                                                 \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                      \
        if (threadIdx.x == 0) {                                                          \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();              \
            if (blockIdx.x == 0) g_ph[kern][k] = t_;                                     \
            if ((k) == 0) atomicMin(&g_ph[kern][14], t_);                                \
            if ((k) == 5) atomicMax(&g_ph[kern][15], t_);                                \
        }                                                                                \
    } while (0)
#else
#define LPG_PH(kern, k) do { } while (0)
#endif

constexpr long long kXSpinTicks = 200000000ll;     // s_memrealtime (100 MHz): 2 s, then NUMERIC + stall

// The candidates of every rank for this pivot (tag X.tag), polled by the
// whole block until every word carries the tag; false on timeout.
template <int NT>
__device__ bool xch_gather(const Xch &X, Cand &best) {
    const int par = X.tag & 1, n = X.world * X.nx;
    const long long t0 = (long long)wall_clock64();
    for (;;) {
        bool ok = true;
        Cand b{0.0, 0.0, 0, -1};
        for (int e = threadIdx.x; e < n; e += NT) {
            const uint64_t *w = xch_cand(X, X.rank, par, e / X.nx, e % X.nx);
            uint64_t v[6];
#pragma unroll
            for (int k = 0; k < 6; k++) v[k] = ld_sys64(w + k);
#pragma unroll
            for (int k = 0; k < 6; k++) ok = ok && (uint32_t)(v[k] >> 32) == X.tag;
            Cand c;
            c.theta = __longlong_as_double((long long)(((v[1] & 0xffffffffull) << 32) | (v[0] & 0xffffffffull)));
            c.piv = __longlong_as_double((long long)(((v[3] & 0xffffffffull) << 32) | (v[2] & 0xffffffffull)));
            c.key = (int64_t)(int32_t)(uint32_t)v[4];
            c.row = (int64_t)(int32_t)(uint32_t)v[5];
            cand_take(b, c, cand_better(c, b));
        }
        if (__syncthreads_and(ok)) {
            best = b;
            return true;
        }
        if ((long long)wall_clock64() - t0 > kXSpinTicks) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// MODE 0 (one rank): pricing fused. MODE 1 (multi-rank, allreduce): the
// pivot row lives on one rank; the owner computes P, every other rank writes
// -0 (the identity of the allreduce that follows, so the sum is the owner's
// row bit for bit, signed zeros included), and the pricing runs after the
// exchange (k_price), not here. MODE 2 (multi-rank, owner push): the
// candidates come from every rank's push, the owner stores its P chunk into
// every other rank's xP and raises that chunk's flag, every other rank's
// block waits for its chunk's flag and reads it; then every rank prices
// (k_price's work, fused as in MODE 0).
template <int RULE, int kPF, int NT, int MODE>
__global__ __launch_bounds__(NT, kPF == 96 ? 2 : 1) void k_prep_d(double *__restrict__ T, Geo g, DevState *st, int s,
                                                   const Cand *__restrict__ cand, int ncand, double *__restrict__ P,
                                                   const double *__restrict__ Cs, PricePart *__restrict__ pp, Defer D,
                                                   Xch X) {
    constexpr bool MR = MODE != 0;
    const int64_t j2 = (int64_t)blockIdx.x * NT + threadIdx.x;
    const int64_t nvec = (g.ncols + 1) / 2;
    const bool col = j2 < nvec;
    const int64_t rM = g.nloc, rR = g.nloc + g.nobj - 1;
    const int lane = threadIdx.x & 63;
    LPG_PH(0, 0);
    // ---- round 1: nothing here depends on the leaving row
    const int32_t status = st->slot[s].status;
    Cand best{0.0, 0.0, 0, -1};
    if (MODE != 2 || X.from_cand) {
        for (int q = threadIdx.x; q < ncand; q += NT) {
            const Cand c = cand[q];
            cand_take(best, c, cand_better(c, best));
        }
    }
    d2 dM = d2{0.0, 0.0}, dR = d2{0.0, 0.0};
    if (col) {
        dM = *(const d2 *)(T + rM * g.ld + 2 * j2);
        dR = *(const d2 *)(T + rR * g.ld + 2 * j2);
    }
    const double cM = -Cs[rM], cR = -Cs[rR];
    // kPF = 96 / 128: two banks of B0 = 48 / 64 slots (blocks of up to 96 /
    // 128 pivots); bank 1 holds slots B0 .. kPF - 1 in lanes 0 .. B1 - 1 and
    // its P rows are loaded after bank 0's chain (the registers of a whole
    // prefetch are not there: one more memory round trip, ~1 us). kPF = 96
    // exists for the grid: 48-slot banks keep the kernel at 2 waves per SIMD,
    // so config 4's 385 blocks run in one round on 256 CUs where kPF = 64's
    // one wave per SIMD needed two (~8-10 us per pivot, profiles/r04_phase_probe_c4.log)
    constexpr int B0 = kPF < 64 ? kPF : (kPF == 96 ? 48 : 64);
    constexpr int B1 = kPF > 64 ? kPF - B0 : 0;
    constexpr bool TWO = B1 > 0;
    static_assert(kPF <= 64 || kPF == 96 || kPF == 128, "prefetch slots");
    static_assert(B1 <= B0 && B1 <= 64, "bank 1 reuses bank 0's registers, one slot per lane");
    const int npf = D.q < B0 ? D.q : B0;
    // slots past the block are (+0, +0) and their multiplier is -0: the chain
    // step fma(-0, +0, x) == x for every x, so the loop below needs no bound
    // (slots past the block load from an all-zero row: no branch and no
    // select per load, either of which makes the 64 loads wait in turn)
    d2 pq[B0];
    const int64_t jc = col ? 2 * j2 : 0;
#pragma unroll
    for (int u = 0; u < B0; u++)
        pq[u] = *(const d2 *)((u < npf ? D.Pbuf + (int64_t)u * g.ld : D.zrow) + jc);
    const int64_t rqv = lane < B0 && lane < D.q ? D.rq[lane] : -1;   // lane q of every wave holds r_q
    const int64_t rqv1 = TWO && lane < B1 && B0 + lane < D.q ? D.rq[B0 + lane] : -1;   // bank 1: r_{B0 + lane}
    const int2 lj = col ? ((const int2 *)D.colmap)[j2] : int2{0, 0};   // logical indices of the two columns
    // MODE 1: the allreduce of P runs whether or not a pivot does (the loop
    // may have ended): then every rank sends the identity, -0
    if (status != RUNNING) {
        if (MODE == 1 && col) *(d2 *)(P + 2 * j2) = d2{-0.0, -0.0};
        return;
    }
    if (MODE == 2 && !X.from_cand && !xch_gather<NT>(X, best)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = NUMERIC;
            st->stall = 2;
        }
        return;
    }
    LPG_PH(0, 1);
    best = block_argmin_cand<NT / 64>(best);
    LPG_PH(0, 2);
    // the oracle's rule (oracle/lpo.c lpo_solve): NUMERIC iff the pivot element or
    // the row's b is not finite (a non-finite b arrives as piv = NaN); an
    // overflowing ratio b / a is an ordinary (largest) candidate
    if (best.row < 0 || !isfinite(best.piv)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = best.row < 0 ? UNBOUNDED : NUMERIC;
            st->slot[s].r = -1;
        }
        if (MODE == 1 && col) *(d2 *)(P + 2 * j2) = d2{-0.0, -0.0};
        return;
    }
    const bool own = !MR || (best.row >= g.row0 && best.row < g.row0 + g.nloc);   // uniform
    const int64_t rl = own ? best.row - g.row0 : -1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t k = st->slot[s].k;
        st->slot[s].r = best.row;
        D.rq[D.q] = rl;
        st->npend = D.q + 1;
        D.kq[D.q] = k;                       // entering and leaving variables of the block (k_swap_plan)
        D.lv[D.q] = D.basis[best.row];
        D.pv[D.q] = best.piv;                // pivot element, known to every rank (k_swap_plan)
        D.basis[best.row] = k;
        const int64_t n = st->pivots;
        if (D.logk && n < st->logcap) {
            D.logk[n] = k;
            D.logr[n] = best.row;
        }
        st->pivots = n + 1;
        st->last_k = k;
        st->last_r = best.row;
    }
    // ---- round 2: the pivot row as stored and its pending multipliers
    // (lane q: -C_q[r]); the chain restarts at the last pending pivot qs on
    // this row (x = P_qs), found by a ballot, so each step is one fma with
    // the multiplier read back from lane q (v_readlane: no LDS, no barrier)
    d2 t = d2{0.0, 0.0};
    if (col && own) t = *(const d2 *)(T + rl * g.ld + 2 * j2);
    const double cl = (own && lane < B0 && lane < D.q) ? -D.Cbuf[(int64_t)lane * D.cs + rl] : -0.0;
    const double cl1 = (TWO && own && lane < B1 && B0 + lane < D.q) ? -D.Cbuf[(int64_t)(B0 + lane) * D.cs + rl] : -0.0;
    const unsigned long long hit = __ballot(own && lane < B0 && lane < D.q && rqv == rl);
    const unsigned long long hit1 = TWO ? __ballot(own && lane < B1 && B0 + lane < D.q && rqv1 == rl) : 0ull;
    const int qs = hit1 ? B0 + 63 - __clzll((long long)hit1) : hit ? 63 - __clzll((long long)hit) : -1;
    LPG_PH(0, 3);
    PricePart pbest{0.0, -1, 0, 0};
    const uint64_t clb = (uint64_t)__double_as_longlong(cl);
    const uint64_t clb1 = (uint64_t)__double_as_longlong(cl1);
    const int npf1 = TWO && D.q > B0 ? D.q - B0 : 0;
    // The chain runs in every lane (EXEC full, uniform branches only): a
    // readlane returns the source lane's register whether or not that lane
    // was active when the register was written, so the multipliers must never
    // sit behind a per-lane condition. Straight-line steps: a uniform branch
    // per step cost ~100 cycles on a lone wave; the common case has no
    // restart on this row.
    if (qs < 0) {
#pragma unroll
        for (int u = 0; u < B0; u++) {
            const double c = __longlong_as_double((long long)rdl64(clb, u));
            t.x = fma(c, pq[u].x, t.x);
            t.y = fma(c, pq[u].y, t.y);
        }
    } else {
#pragma unroll
        for (int u = 0; u < B0; u++) {
            const double c = __longlong_as_double((long long)rdl64(clb, u));
            const double fx = fma(c, pq[u].x, t.x), fy = fma(c, pq[u].y, t.y);
            t.x = u == qs ? pq[u].x : (u > qs ? fx : t.x);
            t.y = u == qs ? pq[u].y : (u > qs ? fy : t.y);
        }
    }
    if (TWO && D.q > B0) {                  // bank 1: slots B0 .. D.q - 1 (uniform)
        asm volatile("" ::: "memory");      // its loads stay behind bank 0's chain
#pragma unroll
        for (int u = 0; u < B1; u++)
            pq[u] = *(const d2 *)((u < npf1 ? D.Pbuf + (int64_t)(B0 + u) * g.ld : D.zrow) + jc);
        const int qs1 = qs - B0;
        if (qs1 < 0) {
#pragma unroll
            for (int u = 0; u < B1; u++) {
                const double c = __longlong_as_double((long long)rdl64(clb1, u));
                t.x = fma(c, pq[u].x, t.x);
                t.y = fma(c, pq[u].y, t.y);
            }
        } else {
#pragma unroll
            for (int u = 0; u < B1; u++) {
                const double c = __longlong_as_double((long long)rdl64(clb1, u));
                const double fx = fma(c, pq[u].x, t.x), fy = fma(c, pq[u].y, t.y);
                t.x = u == qs1 ? pq[u].x : (u > qs1 ? fx : t.x);
                t.y = u == qs1 ? pq[u].y : (u > qs1 ? fy : t.y);
            }
        }
    }
    if (MODE == 1) {
        if (col) *(d2 *)(P + 2 * j2) = own ? d2{t.x / best.piv, t.y / best.piv} : d2{-0.0, -0.0};
        return;
    }
    d2 p = d2{0.0, 0.0};
    if (col && own) {
        p.x = t.x / best.piv;
        p.y = t.y / best.piv;
    }
    if (MODE == 2) {
        const int par = X.tag & 1;
        if (own) {                 // push this block's chunk to every other rank, then its flag
            if (col)
                for (int rk = 0; rk < X.world; rk++) {
                    if (rk == X.rank) continue;
                    double *xp = xch_row(X, rk, par, 0, g.ld) + 2 * j2;
                    st_sys64(xp, (uint64_t)__double_as_longlong(p.x));
                    st_sys64(xp + 1, (uint64_t)__double_as_longlong(p.y));
                }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                release_system();
                for (int rk = 0; rk < X.world; rk++)
                    if (rk != X.rank)
                        __hip_atomic_store(xch_flag(X, rk, par, blockIdx.x), X.tag, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {                   // wait for this block's chunk from the owner
            __shared__ int xok;
            if (threadIdx.x == 0) {
                const long long t0 = (long long)wall_clock64();
                int ok = 1;
                while (__hip_atomic_load(xch_flag(X, X.rank, par, blockIdx.x), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) != X.tag) {
                    if ((long long)wall_clock64() - t0 > kXSpinTicks) {
                        ok = 0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                xok = ok;                  // the chunk is read with system-scope loads: no acquire
            }
            __syncthreads();
            if (!xok) {
                if (threadIdx.x == 0) {
                    st->slot[s].status = NUMERIC;
                    st->stall = 3;
                }
                return;
            }
            if (col) {
                const double *xp = xch_row(X, X.rank, par, 0, g.ld) + 2 * j2;
                p.x = __longlong_as_double((long long)ld_sys64(xp));
                p.y = __longlong_as_double((long long)ld_sys64(xp + 1));
            }
        }
    }
    if (col) {
        *(d2 *)(P + 2 * j2) = p;
        dM.x = fma(cM, p.x, dM.x);
        dM.y = fma(cM, p.y, dM.y);
        dR.x = fma(cR, p.x, dR.x);
        dR.y = fma(cR, p.y, dR.y);
        *(d2 *)(T + rR * g.ld + 2 * j2) = dR;
        if (g.nobj == 2) *(d2 *)(T + rM * g.ld + 2 * j2) = dM;
        price_one<RULE>(pbest, dM.x, dR.x, lj.x, g, 2 * j2);
        price_one<RULE>(pbest, dM.y, dR.y, lj.y, g, 2 * j2 + 1);
        // the physical column of this thread's winner, from its logical index
        // (not through the struct select, see k_price)
        pbest.pad = (int32_t)(pbest.j == lj.y ? 2 * j2 + 1 : 2 * j2);
    }
    LPG_PH(0, 4);
    pbest = block_argmin_pp<RULE, NT / 64>(pbest);
    if (threadIdx.x == 0) pp[blockIdx.x] = pbest;
    LPG_PH(0, 5);
}

// PUSH (owner-push exchange, Xch): each block also stores its candidate into
// every rank's xC as 6 self-validating {payload, tag + 1} words.
template <int RULE, int kPF, int NT, bool PUSH>
__global__ __launch_bounds__(NT) void k_select_d(const double *__restrict__ T, Geo g, DevState *st, int s,
                                                     int s1, const double *__restrict__ Cs, double *__restrict__ Cs1,
                                                     const PricePart *__restrict__ pp, int npp,
                                                     const int64_t *__restrict__ basis, Cand *__restrict__ part,
                                                     Defer D, Xch X) {
    const int64_t nrows = g.nloc + g.nobj;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;   // one row per thread (launcher checks)
    const bool row = i < nrows;
    const bool crow = i < g.nloc;
    const int lane = threadIdx.x & 63;
    LPG_PH(1, 0);
    // ---- round 1: nothing here depends on the entering column
    const int32_t stt = st->slot[s].status;
    const int64_t r = st->slot[s].r, kc = st->slot[s].k;
    PricePart pb{0.0, -1, 0, 0};
    for (int q = threadIdx.x; q < npp; q += NT) {
        const PricePart c = pp[q];
        pp_take(pb, c, pp_better<RULE>(c, pb));
    }
    double ob = 0.0, csi = 0.0;
    if (row) {
        ob = T[i * g.ld];
        csi = Cs[i];
    }
    // kPF = 96 / 128: two banks of B0 = 48 / 64 slots (blocks of up to 96 /
    // 128 pivots; k_prep_d): 96 chain steps instead of 128 from 64 to 95
    // pending pivots
    constexpr int B0 = kPF < 64 ? kPF : (kPF == 96 ? 48 : 64);
    constexpr int B1 = kPF > 64 ? kPF - B0 : 0;
    constexpr bool TWO = B1 > 0;
    static_assert(kPF <= 64 || kPF == 96 || kPF == 128, "prefetch slots");
    const int npf = D.q < B0 ? D.q : B0;
    // slots past the pending block: +0 (with P entries +0 below: no-op steps).
    // The loads are unconditional (a clamped address, then a select): a load
    // behind a per-slot condition became a branch, and the compiler then
    // waited for each load before issuing the next (64 round trips)
    double cv[B0];
    const int64_t ic = crow ? i : 0;
#pragma unroll
    for (int u = 0; u < B0; u++) {
        const double v = D.Cbuf[(int64_t)(u < npf ? u : 0) * D.cs + ic];
        cv[u] = (u < npf && crow) ? v : 0.0;
    }
    double cv1[TWO ? B1 : 1];        // bank 1: slots B0 .. D.q - 1 (pivot t's own C_t is added below)
    const int npf1 = TWO && D.q > B0 ? D.q - B0 : 0;
#pragma unroll
    for (int u = 0; u < (TWO ? B1 : 1); u++) {
        cv1[u] = 0.0;
        if (TWO) {
            const double v = D.Cbuf[(int64_t)(u < npf1 ? B0 + u : 0) * D.cs + ic];
            cv1[u] = (u < npf1 && crow) ? v : 0.0;
        }
    }
    // lane q of every wave holds P_q[0], r_q (q <= D.q: pivot t included);
    // bank 1 slot B0 + q in lane q
    const bool lq = lane <= D.q;
    const double p0l = lq ? D.Pbuf[(int64_t)lane * g.ld] : 0.0;
    const int32_t rql = lq ? (int32_t)D.rq[lane] : -1;
    const bool lq1 = TWO && lane < B1 && B0 + lane <= D.q;
    const double p0l1 = lq1 ? D.Pbuf[(int64_t)(B0 + lane) * g.ld] : 0.0;
    const int32_t rql1 = lq1 ? (int32_t)D.rq[B0 + lane] : -1;
    const int64_t bkey = (RULE == RULE_BLAND && crow) ? basis[g.row0 + i] : 0;
    Slot *dst = &st->slot[s1];
    if (stt != RUNNING) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            dst->status = stt;
            dst->k = -1;
            dst->r = -1;
        }
        return;
    }
    if (crow) D.Cbuf[(int64_t)D.q * D.cs + i] = csi;   // pivot t is pending: its column C_t
    LPG_PH(1, 1);
    pb = block_argmin_pp<RULE, NT / 64>(pb);
    LPG_PH(1, 2);
    if (pb.j < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            dst->status = OPTIMAL;
            dst->k = -1;
            dst->r = -1;
        }
        return;
    }
    // logical (log, basis, slot) and physical (loads) column; with more partials
    // than threads the round-1 loop selects structs again, and the physical
    // column is then read through inv rather than trusted to that select (k_price)
    const int64_t kn = pb.j, kp = npp > NT ? (int64_t)D.inv[kn] : (int64_t)pb.pad;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dst->status = RUNNING;
        dst->k = kn;
    }
    // ---- round 2: column k_{t+1} as stored and P_q[k_{t+1}] (lane q)
    double oa = 0.0;
    if (row) oa = T[i * g.ld + kp];
    const double pkl = lq ? D.Pbuf[(int64_t)lane * g.ld + kp] : 0.0;
    const double pkl1 = lq1 ? D.Pbuf[(int64_t)(B0 + lane) * g.ld + kp] : 0.0;
    LPG_PH(1, 3);
    const uint64_t p0b = (uint64_t)__double_as_longlong(p0l), pkb = (uint64_t)__double_as_longlong(pkl);
    Cand best{0.0, 0.0, 0, -1};
    // columns 0 and k_{t+1}: the chain over pivots 0..q, in EVERY lane (rows
    // past the tableau and objective rows compute junk that is dropped below):
    // a readlane returns the source lane's register whether or not that lane
    // was active when it was written, so no chain input may be computed behind
    // a per-lane condition
    double b = ob, a = oa;
    const int32_t ii = (int32_t)i;
    if (D.q <= B0) {
        // straight line over B0 slots: lanes >= D.q read as (P = +0, r = -1)
        // and cv = +0 there, so those steps are fma(-0, +0, x) == x
        const bool lp = lane < D.q;
        const uint64_t p0m = lp ? p0b : 0ull, pkm = lp ? pkb : 0ull;
        const uint32_t rqm = lp ? (uint32_t)rql : 0xffffffffu;
#pragma unroll
        for (int u = 0; u < B0; u++) {
            const double q0 = __longlong_as_double((long long)rdl64(p0m, u));
            const double qk = __longlong_as_double((long long)rdl64(pkm, u));
            const bool hit = ii == (int32_t)rdl32(rqm, u);
            const double fb = fma(-cv[u], q0, b), fa = fma(-cv[u], qk, a);
            b = hit ? q0 : fb;
            a = hit ? qk : fa;
        }
    } else {
#pragma unroll
        for (int u = 0; u < B0; u++) {
            const double q0 = __longlong_as_double((long long)rdl64(p0b, u));
            const double qk = __longlong_as_double((long long)rdl64(pkb, u));
            const bool hit = ii == (int32_t)rdl32((uint32_t)rql, u);
            const double fb = fma(-cv[u], q0, b), fa = fma(-cv[u], qk, a);
            b = hit ? q0 : fb;
            a = hit ? qk : fa;
        }
    }
    if (TWO && D.q >= B0) {
        // bank 1, pivot t included (slot D.q, multiplier -Cs): lanes past
        // D.q - B0 read as (P = +0, r = -1) with multiplier +0
        const uint64_t p0b1 = (uint64_t)__double_as_longlong(p0l1), pkb1 = (uint64_t)__double_as_longlong(pkl1);
        const int qt = D.q - B0;
#pragma unroll
        for (int u = 0; u < B1; u++) {
            const double q0 = __longlong_as_double((long long)rdl64(p0b1, u));
            const double qk = __longlong_as_double((long long)rdl64(pkb1, u));
            const bool hit = ii == (int32_t)rdl32((uint32_t)rql1, u);
            const double c = u == qt ? csi : cv1[u];
            const double fb = fma(-c, q0, b), fa = fma(-c, qk, a);
            b = hit ? q0 : fb;
            a = hit ? qk : fa;
        }
    }
    if (D.q < B0) {           // pivot t itself: C_t is Cs
        const int q = D.q;
        const double q0 = __longlong_as_double((long long)rdl64(p0b, q));
        const double qk = __longlong_as_double((long long)rdl64(pkb, q));
        const bool hit = ii == (int32_t)rdl32((uint32_t)rql, q);
        const double fb = fma(-csi, q0, b), fa = fma(-csi, qk, a);
        b = hit ? q0 : fb;
        a = hit ? qk : fa;
    }
    if (!crow) {              // objective rows are current (prep wrote d_{t+1})
        b = ob;
        a = oa;
    }
    // objective rows past the grid: the single-rank launch covers only the
    // constraint rows (pivot_d_blocks(g, 2, nt): config 4's 65536 rows take
    // 256 blocks, one per CU, where 257 left one block for a second round at
    // one wave per SIMD); block 0 then writes their C_{t+1} entries, which
    // are column k as stored (the objective rows are current), and the
    // candidates of the blocks the grid left out, none (the consumers read
    // pivot_d_blocks(g, 1, nt) of them). Loaded after the chain (no
    // registers held across it), stored after the block argmin.
    const int64_t iob = g.nloc + threadIdx.x;
    const bool fold = blockIdx.x == 0 && threadIdx.x < g.nobj && iob >= (int64_t)gridDim.x * NT;
    const double foa = fold ? T[iob * g.ld + kp] : 0.0;
    if (row) {
        Cs1[i] = a;
        if (crow && a > g.eps_piv) {
            const int64_t grow = g.row0 + i;
            Cand c;
            c.theta = b > 0.0 ? b / a : 0.0;
            c.piv = isfinite(b) ? a : __longlong_as_double(0x7ff8000000000000ll);   // b_r not finite: NUMERIC at prep
            c.row = grow;
            c.key = RULE == RULE_BLAND ? (grow == r ? kc : bkey) : grow;
            cand_take(best, c, cand_better(c, best));
        }
    }
    LPG_PH(1, 4);
    best = block_argmin_cand<NT / 64>(best);
    if (threadIdx.x == 0) part[blockIdx.x] = best;
    if (blockIdx.x == 0) {
        if (fold) Cs1[iob] = foa;
        const int64_t bn = (int64_t)gridDim.x + threadIdx.x;   // the grid leaves out at most NT blocks
        if (bn * NT < nrows) {                                 // {0, 0, 0, row -1}: none
            double2 *w = (double2 *)(part + bn);
            w[0] = double2{0.0, 0.0};
            w[1] = double2{0.0, __longlong_as_double(-1ll)};
        }
    }
    if (PUSH && threadIdx.x == 0) {
        const uint32_t tg = X.tag + 1;
        const uint64_t th = (uint64_t)__double_as_longlong(best.theta), pv = (uint64_t)__double_as_longlong(best.piv);
        const uint32_t w[6] = {(uint32_t)th, (uint32_t)(th >> 32), (uint32_t)pv, (uint32_t)(pv >> 32),
                               (uint32_t)best.key, (uint32_t)best.row};
        for (int rk = 0; rk < X.world; rk++) {
            uint64_t *d = xch_cand(X, rk, tg & 1, X.rank, blockIdx.x);
#pragma unroll
            for (int k = 0; k < 6; k++) st_sys64(d + k, ((uint64_t)tg << 32) | w[k]);
        }
    }
    LPG_PH(1, 5);
}

#ifdef LPG_PHASES
int debug_phases(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ph), sizeof g_ph) != hipSuccess) return -1;
    if (reset) {
        unsigned long long init[2][16];
        for (int k = 0; k < 2; k++)
            for (int j = 0; j < 16; j++) init[k][j] = j == 14 ? ~0ull : 0ull;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ph), init, sizeof init) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// prefetch slots of k_prep_d / k_select_d: the pending chain rounded up to
// 16 (padding slots cost a load and two fmas each, ~1.4 us per kernel for 32
// of them), two banks of 64 past 64 pending pivots; k_prep_d takes two banks
// of 48 from 48 to 95 pending pivots (2 waves per SIMD, see kPF = 96)
static int pivot_pf(int q) { return q < 16 ? 16 : q < 32 ? 32 : q < 48 ? 48 : q < 64 ? 64 : 128; }
static int prep_pf(int q) { return q < 48 ? pivot_pf(q) : q < 96 ? 96 : 128; }
static int select_pf(int q) { return q < 64 ? pivot_pf(q) : q < 96 ? 96 : 128; }

// which 0: k_prep_d's column blocks; 1: k_select_d's row blocks covering the
// objective rows (its candidate count, every form); 2: the single-rank pair's
// select grid, the constraint rows only (k_select_d folds the objective rows
// and the missing blocks' candidates into block 0)
int pivot_d_blocks(const Geo &g, int which, int nt) {
    if (which == 0) return (int)(((g.ncols + 1) / 2 + nt - 1) / nt);
    if (which == 2) return (int)std::max<int64_t>(1, (g.nloc + nt - 1) / nt);
    return (int)((g.nloc + g.nobj + nt - 1) / nt);
}

int launch_pivot_d(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, Cand *part, int nsel,
                   double *P, const double *Cs, double *Cs1, PricePart *pp, int npp, const int64_t *basis,
                   const Defer &D, int nt) {
    // 256-thread blocks only: 64- and 128-thread forms were no faster at
    // config 3 (17.8k / 18.9k vs 19.4k pivots/s) and diverged from the
    // oracle at m = 16384 (first pivots identical, later ones not), so they
    // are not offered.
    if (nt != 256 || npp != pivot_d_blocks(g, 0, nt) || nsel != pivot_d_blocks(g, 1, nt)) return -1;
    const int nselg = pivot_d_blocks(g, 2, nt);   // the grid: constraint rows only (k_select_d folds the rest)
    hipStream_t stream = (hipStream_t)L.stream;
    const Xch X0{};
#define LPG_PD(R, PFP, PFS)                                                                                            \
    do {                                                                                                               \
        hipLaunchKernelGGL((k_prep_d<R, PFP, 256, 0>), dim3(npp), dim3(256), 0, stream, g.T, g, st, s, part, nsel, P,   \
                           Cs, pp, D, X0);                                                                             \
        hipLaunchKernelGGL((k_select_d<R, PFS, 256, false>), dim3(nselg), dim3(256), 0, stream, g.T, g, st, s, s1, Cs,  \
                           Cs1, pp, npp, basis, part, D, X0);                                                          \
    } while (0)
#define LPG_PD_R(R)                                          \
    do {                                                     \
        const int pf = select_pf(D.q);                       \
        if (pf == 16) LPG_PD(R, 16, 16);                     \
        else if (pf == 32) LPG_PD(R, 32, 32);                \
        else if (pf == 48) LPG_PD(R, 48, 48);                \
        else if (pf == 64) LPG_PD(R, 96, 64);                \
        else if (pf == 96) LPG_PD(R, 96, 96);                \
        else LPG_PD(R, 128, 128);                            \
    } while (0)
    if (rule == RULE_BLAND) LPG_PD_R(RULE_BLAND);
    else LPG_PD_R(RULE_DANTZIG);
#undef LPG_PD_R
#undef LPG_PD
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Multi-rank deferred pivot, first half: k_prep_d<MR> over npp_d column
// blocks reading ncand gathered candidates (P: owner's row, -0 elsewhere).
int launch_prep_dm(const Launch &L, const Geo &g, int rule, DevState *st, int s, const Cand *cand, int ncand,
                   double *P, const double *Cs, int npp_d, const Defer &D) {
    if (npp_d != pivot_d_blocks(g, 0, 256)) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
    const Xch X0{};
#define LPG_PM(R, PF)                                                                                                 \
    hipLaunchKernelGGL((k_prep_d<R, PF, 256, 1>), dim3(npp_d), dim3(256), 0, stream, g.T, g, st, s, cand, ncand, P,    \
                       Cs, nullptr, D, X0)
    const int pf = prep_pf(D.q);   // as launch_pivot_d
    if (rule == RULE_BLAND) {
        if (pf == 16) LPG_PM(RULE_BLAND, 16);
        else if (pf == 32) LPG_PM(RULE_BLAND, 32);
        else if (pf == 48) LPG_PM(RULE_BLAND, 48);
        else if (pf == 96) LPG_PM(RULE_BLAND, 96);
        else LPG_PM(RULE_BLAND, 128);
    } else {
        if (pf == 16) LPG_PM(RULE_DANTZIG, 16);
        else if (pf == 32) LPG_PM(RULE_DANTZIG, 32);
        else if (pf == 48) LPG_PM(RULE_DANTZIG, 48);
        else if (pf == 96) LPG_PM(RULE_DANTZIG, 96);
        else LPG_PM(RULE_DANTZIG, 128);
    }
#undef LPG_PM
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ... second half, after the pivot-row exchange and k_price: k_select_d over
// nsel blocks (>= the local rows + objective rows), npp pricing partials.
int launch_select_dm(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, const double *Cs,
                     double *Cs1, const PricePart *pp, int npp, const int64_t *basis, Cand *part, int nsel,
                     const Defer &D) {
    if ((int64_t)nsel * 256 < g.nloc + g.nobj) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
    const Xch X0{};
#define LPG_SM(R, PF)                                                                                               \
    hipLaunchKernelGGL((k_select_d<R, PF, 256, false>), dim3(nsel), dim3(256), 0, stream, g.T, g, st, s, s1, Cs, Cs1, \
                       pp, npp, basis, part, D, X0)
    const int pf = select_pf(D.q);   // as launch_pivot_d
    if (rule == RULE_BLAND) {
        if (pf == 16) LPG_SM(RULE_BLAND, 16);
        else if (pf == 32) LPG_SM(RULE_BLAND, 32);
        else if (pf == 48) LPG_SM(RULE_BLAND, 48);
        else if (pf == 64) LPG_SM(RULE_BLAND, 64);
        else if (pf == 96) LPG_SM(RULE_BLAND, 96);
        else LPG_SM(RULE_BLAND, 128);
    } else {
        if (pf == 16) LPG_SM(RULE_DANTZIG, 16);
        else if (pf == 32) LPG_SM(RULE_DANTZIG, 32);
        else if (pf == 48) LPG_SM(RULE_DANTZIG, 48);
        else if (pf == 64) LPG_SM(RULE_DANTZIG, 64);
        else if (pf == 96) LPG_SM(RULE_DANTZIG, 96);
        else LPG_SM(RULE_DANTZIG, 128);
    }
#undef LPG_SM
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Owner-push exchange: the buffer's size and the offsets of its parts (256-byte aligned).
int64_t xch_bytes(int64_t ld, int world, int nblk, int nx, int64_t *offF, int64_t *offC, int64_t *offG) {
    const int64_t f = (2 * (int64_t)world * ld * (int64_t)sizeof(double) + 255) & ~(int64_t)255;   // xP[2][world][ld]
    const int64_t c = (f + 2 * (int64_t)world * nblk * 4 + 255) & ~(int64_t)255;                  // xF[2][world][nblk]
    const int64_t gg = (c + 2 * (int64_t)world * nx * 6 * 8 + 255) & ~(int64_t)255;               // xC[2][world][nx][6]
    if (offF) *offF = f;
    if (offC) *offC = c;
    if (offG) *offG = gg;
    return gg + 256;                                                                               // {gcnt, gdec}
}

int launch_prep_x(const Launch &L, const Geo &g, int rule, DevState *st, int s, const Cand *cand, int ncand,
                  double *P, const double *Cs, PricePart *pp, int npp_d, const Defer &D, const Xch &X) {
    if (npp_d != pivot_d_blocks(g, 0, 256) || X.nblk < npp_d) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
#define LPG_PX(R, PF)                                                                                                 \
    hipLaunchKernelGGL((k_prep_d<R, PF, 256, 2>), dim3(npp_d), dim3(256), 0, stream, g.T, g, st, s, cand, ncand, P,    \
                       Cs, pp, D, X)
    const int pf = prep_pf(D.q);   // as launch_pivot_d
    if (rule == RULE_BLAND) {
        if (pf == 16) LPG_PX(RULE_BLAND, 16);
        else if (pf == 32) LPG_PX(RULE_BLAND, 32);
        else if (pf == 48) LPG_PX(RULE_BLAND, 48);
        else if (pf == 96) LPG_PX(RULE_BLAND, 96);
        else LPG_PX(RULE_BLAND, 128);
    } else {
        if (pf == 16) LPG_PX(RULE_DANTZIG, 16);
        else if (pf == 32) LPG_PX(RULE_DANTZIG, 32);
        else if (pf == 48) LPG_PX(RULE_DANTZIG, 48);
        else if (pf == 96) LPG_PX(RULE_DANTZIG, 96);
        else LPG_PX(RULE_DANTZIG, 128);
    }
#undef LPG_PX
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_select_x(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, const double *Cs,
                    double *Cs1, const PricePart *pp, int npp, const int64_t *basis, Cand *part, int nsel,
                    const Defer &D, const Xch &X) {
    if ((int64_t)nsel * 256 < g.nloc + g.nobj || nsel != X.nx) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
#define LPG_SX(R, PF)                                                                                              \
    hipLaunchKernelGGL((k_select_d<R, PF, 256, true>), dim3(nsel), dim3(256), 0, stream, g.T, g, st, s, s1, Cs, Cs1, \
                       pp, npp, basis, part, D, X)
    const int pf = select_pf(D.q);   // as launch_pivot_d
    if (rule == RULE_BLAND) {
        if (pf == 16) LPG_SX(RULE_BLAND, 16);
        else if (pf == 32) LPG_SX(RULE_BLAND, 32);
        else if (pf == 48) LPG_SX(RULE_BLAND, 48);
        else if (pf == 64) LPG_SX(RULE_BLAND, 64);
        else if (pf == 96) LPG_SX(RULE_BLAND, 96);
        else LPG_SX(RULE_BLAND, 128);
    } else {
        if (pf == 16) LPG_SX(RULE_DANTZIG, 16);
        else if (pf == 32) LPG_SX(RULE_DANTZIG, 32);
        else if (pf == 48) LPG_SX(RULE_DANTZIG, 48);
        else if (pf == 64) LPG_SX(RULE_DANTZIG, 64);
        else if (pf == 96) LPG_SX(RULE_DANTZIG, 96);
        else LPG_SX(RULE_DANTZIG, 128);
    }
#undef LPG_SX
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// Dual simplex (reference: router option 2, router.c:32-34, a no-op; the
// tableau LPStandardize(model, 1) builds, simplex.c:178-179). Same update
// kernel; the pricing roles swap. Pivot t:
//   k_dual_price : leaving row r_t = argmin b_i over b_i < -eps (ties: smallest
//                  row) from the row candidates of the previous step; ratio
//                  test over row r_t: argmin d_j / (-a_rj) over a_rj < -eps_piv
//                  (ties: smallest j) -> per-block partials; live-slice counts
//   k_dual_prep  : entering column k_t; P = T[r]/T[r][k]; C = column k; the
//                  next step's row candidates from b' = fma(-C, P[0], b)
//   k_update     : as in the primal
// Single rank.
// ------------------------------------------------------------------------

// Row candidate: (theta = b_i, key = row) through the Cand min-reduction.
__device__ __forceinline__ void dual_row_cand(Cand &best, double b, int64_t grow, const Geo &g) {
    if (!(b < -g.eps_opt)) return;
    Cand c;
    c.theta = b;
    c.piv = 0.0;
    c.key = grow;
    c.row = grow;
    cand_take(best, c, cand_better(c, best));
}

__global__ __launch_bounds__(kBlock) void k_dual_rows(const double *__restrict__ T, Geo g, Cand *__restrict__ part) {
    Cand best{0.0, 0.0, 0, -1};
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < g.nloc; i += (int64_t)gridDim.x * kBlock)
        dual_row_cand(best, T[i * g.ld], g.row0 + i, g);
    best = block_reduce_cand(best);
    if (threadIdx.x == 0) part[blockIdx.x] = best;
}

__global__ __launch_bounds__(kBlock) void k_dual_price(const double *__restrict__ T, Geo g, DevState *st, int s,
                                                       const Cand *__restrict__ part, int npart,
                                                       PricePart *__restrict__ pp, int *__restrict__ pc) {
    if (st->slot[s].status != RUNNING) return;
    Cand best{0.0, 0.0, 0, -1};
    for (int q = threadIdx.x; q < npart; q += kBlock) {
        const Cand c = part[q];
        cand_take(best, c, cand_better(c, best));
    }
    best = block_reduce_cand(best);
    if (best.row < 0) {                      // primal feasible: optimal
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = OPTIMAL;
            st->slot[s].r = -1;
        }
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->slot[s].r = best.row;
        st->work[s] = 0;
    }
    const int64_t rl = best.row - g.row0;
    const int64_t j2 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t nvec = (g.ncols + 1) / 2;
    PricePart pb{0.0, -1, 0, 0};
    bool live = false;
    if (j2 < nvec) {
        const d2 a = *(const d2 *)(T + rl * g.ld + 2 * j2);
        const d2 d = *(const d2 *)(T + (g.nloc + g.nobj - 1) * g.ld + 2 * j2);
        live = a.x != 0.0 || a.y != 0.0;     // P = row / pivot is non-zero exactly here
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const int64_t j = 2 * j2 + e;
            const double aj = e ? a.y : a.x, dj = e ? d.y : d.x;
            if (j < 1 || j > g.nact || !(aj < -g.eps_piv)) continue;
            PricePart c;
            c.v = dj > 0.0 ? dj / -aj : 0.0;
            c.j = j;
            c.cls = 0;
            c.pad = 0;
            pp_take(pb, c, pp_better<RULE_DANTZIG>(c, pb));
        }
    }
    count_live(pc, live);
    pb = block_reduce_pp<RULE_DANTZIG>(pb);
    if (threadIdx.x == 0) pp[blockIdx.x] = pb;
}

// Blocks [0, npp): P; blocks [npp, npp + nsel): column snapshot C and the next
// step's row candidates.
__global__ __launch_bounds__(kBlock) void k_dual_prep(const double *__restrict__ T, Geo g, DevState *st, int s,
                                                      int s1, const PricePart *__restrict__ pp, int npp,
                                                      const int *__restrict__ pc, int skip, double *__restrict__ P,
                                                      double *__restrict__ Cs, Cand *__restrict__ part) {
    const int32_t stt = st->slot[s].status;
    if (stt != RUNNING) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s1].status = stt;
            st->slot[s1].k = -1;
            st->slot[s1].r = -1;
        }
        return;
    }
    PricePart pb{0.0, -1, 0, 0};
    for (int q = threadIdx.x; q < npp; q += kBlock) {
        const PricePart c = pp[q];
        pp_take(pb, c, pp_better<RULE_DANTZIG>(c, pb));
    }
    pb = block_reduce_pp<RULE_DANTZIG>(pb);
    if (pb.j < 0) {                          // no a_rj < 0: the LP is primal infeasible
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = INFEASIBLE;
            st->slot[s1].status = INFEASIBLE;
            st->slot[s1].k = -1;
            st->slot[s1].r = -1;
        }
        return;
    }
    const int64_t k = pb.j;
    const int64_t r = st->slot[s].r;
    const int64_t rl = r - g.row0;
    const double piv = T[rl * g.ld + k];
    const double p0 = T[rl * g.ld] / piv;     // == P[0]
    if (blockIdx.x == 0) {
        int64_t live = 0;
        const int64_t nvec = (g.ncols + 1) / 2;
        if (skip)
            for (int q = threadIdx.x; q < npp; q += kBlock) live += pc[q];
        else if (threadIdx.x == 0)
            live = nvec;
#pragma unroll
        for (int mask = 32; mask > 0; mask >>= 1) live += __shfl_xor((long long)live, mask, 64);
        __shared__ int64_t wsum[kBlock / 64];
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = live;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tot = 0;
            for (int w = 0; w < kBlock / 64; w++) tot += wsum[w];
            st->touched += 2ull * (unsigned long long)tot * (unsigned long long)(g.nloc + g.nobj);
            st->slot[s].k = k;
            st->slot[s1].status = RUNNING;
            st->slot[s1].k = -1;
        }
    }
    if ((int)blockIdx.x < npp) {
        const int64_t j2 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
        if (j2 < (g.ncols + 1) / 2) {
            const d2 t = *(const d2 *)(T + rl * g.ld + 2 * j2);
            d2 p;
            p.x = t.x / piv;
            p.y = t.y / piv;
            *(d2 *)(P + 2 * j2) = p;
        }
        return;
    }
    const int64_t nrows = g.nloc + g.nobj;
    const int64_t nb = (int64_t)gridDim.x - npp;
    Cand best{0.0, 0.0, 0, -1};
    for (int64_t i = ((int64_t)blockIdx.x - npp) * kBlock + threadIdx.x; i < nrows; i += nb * kBlock) {
        const double c = T[i * g.ld + k];
        Cs[i] = c;
        if (i < g.nloc) {
            const double b = i == rl ? p0 : fma(-c, p0, T[i * g.ld]);
            dual_row_cand(best, b, g.row0 + i, g);
        }
    }
    best = block_reduce_cand(best);
    if (threadIdx.x == 0) part[blockIdx.x - npp] = best;
}

int launch_dual_rows(const Launch &L, const Geo &g, Cand *part, int nsel) {
    hipLaunchKernelGGL(k_dual_rows, dim3(nsel), dim3(kBlock), 0, (hipStream_t)L.stream, g.T, g, part);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dual_pivot(const Launch &L, const Geo &g, DevState *st, int s, Cand *part, int nsel, PricePart *pp,
                      int *pc, int npp, int skip, double *P, double *Cs, bool price_only) {
    hipStream_t stream = (hipStream_t)L.stream;
    hipLaunchKernelGGL(k_dual_price, dim3(npp), dim3(kBlock), 0, stream, g.T, g, st, s, part, nsel, pp, pc);
    if (!price_only) hipLaunchKernelGGL(k_dual_prep, dim3(npp + nsel), dim3(kBlock), 0, stream, g.T, g, st, s, s ^ 1, pp, npp, pc,
                       skip, P, Cs, part);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// update_t (a12): Gauss-Jordan rank-1 elimination, the HBM-bound hot loop.
//
// Work item = (column tile, row strip). A tile is 256 lanes x VPT 16-byte
// column slices (4*VPT KB of a row); a strip is SR rows. Each lane keeps its
// slice of the normalised pivot row P in VGPRs for the whole strip (the
// register form of staging the pivot row on chip: no lane ever needs another
// lane's P, so LDS would only add a round trip). The per-row multiplier C[i]
// is wave-uniform and comes through the scalar cache. RU rows are loaded
// before any is stored (RU*VPT 16-byte loads in flight per lane); with PIPE
// the next RU rows are loaded before the current ones are stored, so the
// stream never drains between batches. With a persistent grid (PERSIST)
// a fixed number of blocks per CU walks the items with a grid stride, which
// removes the partial last wave of a one-block-per-item launch.
// ------------------------------------------------------------------------

template <int VPT, int RU, bool NT>
__device__ __forceinline__ void upd_load(d2 (&t)[RU][VPT], const d2 *__restrict__ Tv, int64_t i, int64_t ld2,
                                         int64_t cb, const bool (&ok)[VPT]) {
#pragma unroll
    for (int u = 0; u < RU; u++)
#pragma unroll
        for (int v = 0; v < VPT; v++)
            if (ok[v]) {
                const d2 *a = Tv + (i + u) * ld2 + cb + v * kBlock;
                t[u][v] = NT ? __builtin_nontemporal_load(a) : *a;
            }
}

template <int VPT, int RU, bool NT>
__device__ __forceinline__ void upd_compute_store(d2 (&t)[RU][VPT], d2 *__restrict__ Tv, int64_t i, int64_t ld2,
                                                  int64_t cb, const bool (&ok)[VPT], const d2 (&p)[VPT],
                                                  const double *__restrict__ Cs, int64_t rl) {
#pragma unroll
    for (int u = 0; u < RU; u++) {
        const double c = -Cs[i + u];
        const bool isr = (i + u) == rl;
#pragma unroll
        for (int v = 0; v < VPT; v++) {
            d2 x;
            x.x = fma(c, p[v].x, t[u][v].x);
            x.y = fma(c, p[v].y, t[u][v].y);
            t[u][v] = isr ? p[v] : x;
        }
    }
#pragma unroll
    for (int u = 0; u < RU; u++)
#pragma unroll
        for (int v = 0; v < VPT; v++)
            if (ok[v]) {
                d2 *a = Tv + (i + u) * ld2 + cb + v * kBlock;
                if (NT) __builtin_nontemporal_store(t[u][v], a);
                else *a = t[u][v];
            }
}

template <int VPT, int RU, bool NT, bool PIPE, bool DYN>
__global__ __launch_bounds__(kBlock) void k_update(double *__restrict__ T, Geo g, DevState *__restrict__ st, int s,
                                                   const double *__restrict__ P, const double *__restrict__ Cs,
                                                   int64_t ntiles, int64_t strip_rows, int64_t nitems,
                                                   int64_t *__restrict__ basis, int64_t *__restrict__ logk,
                                                   int64_t *__restrict__ logr, int skip) {
    const int32_t status = st->slot[s].status;
    if (status != RUNNING) return;
    const int64_t rglob = st->slot[s].r;
    // local index of the pivot row, -1 on a non-owner rank (never alias the
    // objective row at local index nloc)
    const int64_t rl = (rglob >= g.row0 && rglob < g.row0 + g.nloc) ? rglob - g.row0 : -1;
    const int64_t nrows = g.nloc + g.nobj;
    const int64_t nvec = (g.ncols + 1) / 2;
    const int64_t ld2 = g.ld / 2;
    d2 *__restrict__ Tv = (d2 *)T;
    const d2 *__restrict__ Pv = (const d2 *)P;

    __shared__ int64_t next_item;
    for (int64_t item = DYN ? -1 : blockIdx.x;; item += DYN ? 0 : gridDim.x) {
        if (DYN) {
            // dynamic balance: one device-scope dequeue per 4*VPT KB x SR-row item
            __syncthreads();
            if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->work[s], 1ull);
            __syncthreads();
            item = next_item;
        }
        if (item >= nitems) break;
        const int64_t tile = item % ntiles;
        const int64_t strip = item / ntiles;
        const int64_t i0 = strip * strip_rows;
        const int64_t i1 = i0 + strip_rows < nrows ? i0 + strip_rows : nrows;
        const int64_t cb = tile * (kBlock * VPT) + threadIdx.x;
        d2 p[VPT];
        bool ok[VPT];
        int live = 0;   // slices this lane still updates
#pragma unroll
        for (int v = 0; v < VPT; v++) {
            ok[v] = cb + v * kBlock < nvec;
            p[v] = ok[v] ? Pv[cb + v * kBlock] : d2{0.0, 0.0};
            // Column skipping: where both P
            // entries are zero the update leaves the slice's values unchanged
            // (fma(-c, 0, t) == t; only the sign of a zero could differ), so
            // the slice is neither read nor written. Basic columns other than
            // the leaving one always have P == 0.
            if (skip && p[v].x == 0.0 && p[v].y == 0.0) ok[v] = false;
            live += ok[v] ? 1 : 0;
        }
        // a tile whose pivot-row slice is all zero is skipped as a whole
        if (skip && !__syncthreads_or(live)) continue;
        int64_t i = i0;
        if (PIPE) {
            if (i + RU <= i1) {
                d2 t[RU][VPT];
                upd_load<VPT, RU, NT>(t, Tv, i, ld2, cb, ok);
                for (;;) {
                    const bool more = i + 2 * RU <= i1;
                    d2 nx[RU][VPT];
                    if (more) upd_load<VPT, RU, NT>(nx, Tv, i + RU, ld2, cb, ok);
                    upd_compute_store<VPT, RU, NT>(t, Tv, i, ld2, cb, ok, p, Cs, rl);
                    i += RU;
                    if (!more) break;
#pragma unroll
                    for (int u = 0; u < RU; u++)
#pragma unroll
                        for (int v = 0; v < VPT; v++) t[u][v] = nx[u][v];
                }
            }
        } else {
            for (; i + RU <= i1; i += RU) {
                d2 t[RU][VPT];
                upd_load<VPT, RU, NT>(t, Tv, i, ld2, cb, ok);
                upd_compute_store<VPT, RU, NT>(t, Tv, i, ld2, cb, ok, p, Cs, rl);
            }
        }
        for (; i < i1; i++) {
            d2 t[1][VPT];
            upd_load<VPT, 1, NT>(t, Tv, i, ld2, cb, ok);
            upd_compute_store<VPT, 1, NT>(t, Tv, i, ld2, cb, ok, p, Cs, rl);
        }
    }

    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t k = st->slot[s].k;
        basis[rglob] = k;
        const int64_t n = st->pivots;
        if (logk && n < st->logcap) {
            logk[n] = k;
            logr[n] = rglob;
        }
        st->pivots = n + 1;
        st->last_k = k;
        st->last_r = rglob;
    }
}

struct UpdateCfg {
    int vpt, ru;
    bool nt, pipe;
    int strip;
    int persist;      // blocks per CU of a persistent grid; 0 = one block per item
};

// Two forms (LPG_UPDATE_VARIANT), bit-identical: 0 = one block per
// (256-lane column tile x 64-row strip) item, 8 rows of loads in flight;
// 1 = persistent grid (8 blocks per CU) with a dynamic dequeue, non-temporal
// streaming and pipelined rows. (Round 1 swept 25 forms; these two were the
// defaults.)
static const UpdateCfg kUpdateCfgs[] = {
    {1, 8, false, false, 64, 0},    // 0
    {1, 8, true, true, 64, 8},      // 1
};
constexpr int kNumUpdateCfgs = sizeof(kUpdateCfgs) / sizeof(kUpdateCfgs[0]);

int update_variants() { return kNumUpdateCfgs; }

// Default (variant < 0): large tableaus use the persistent grid (variant 1:
// steady at the read-modify-write ceiling when skipped columns make the work
// per tile uneven; measured best from 2048 to 16385 rows); small ones (fewer
// than 2048 work items, e.g. config 2, MALL-resident) use one block per item
// (variant 0), where the dequeue atomics would cost more than they balance.
int update_auto_variant(const Geo &g) {
    const int64_t nvec = (g.ncols + 1) / 2;
    const int64_t items = ((nvec + kBlock - 1) / kBlock) * ((g.nloc + g.nobj + 63) / 64);
    return items >= 2048 ? 1 : 0;
}

int launch_update(const Launch &L, const Geo &g, DevState *st, int s, const double *P, const double *Cs,
                  int64_t *basis, int64_t *logk, int64_t *logr, int variant, int skip) {
    if (variant < 0 || variant >= kNumUpdateCfgs) variant = update_auto_variant(g);
    const UpdateCfg cfg = kUpdateCfgs[variant];
    const int64_t nvec = (g.ncols + 1) / 2;
    const int64_t ntiles = (nvec + kBlock * cfg.vpt - 1) / (kBlock * cfg.vpt);
    const int64_t nrows = g.nloc + g.nobj;
    // Small tableaus: shrink the strip (down to RU rows) until there are at
    // least ~4 work items per CU, so a config-2-sized update fills 256 CUs.
    int64_t strip = cfg.strip;
    while (strip > cfg.ru && strip > 8 && ntiles * ((nrows + strip - 1) / strip) < 1024) strip /= 2;
    const int64_t nstrips = (nrows + strip - 1) / strip;
    const int64_t nitems = ntiles * nstrips;
    int64_t nblocks = nitems;
    if (cfg.persist > 0) nblocks = std::min<int64_t>(nitems, (int64_t)256 * cfg.persist);
    if (nblocks > 0x7fffffff) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
    dim3 grid((unsigned)nblocks), blk(kBlock);
#define LPG_UPD_(V, R, N, PI, D)                                                                              \
    hipLaunchKernelGGL((k_update<V, R, N, PI, D>), grid, blk, 0, stream, g.T, g, st, s, P, Cs, ntiles, strip, \
                       nitems, basis, logk, logr, skip)
#define LPG_UPD(V, R, N, PI) LPG_UPD_(V, R, N, PI, false)
    if (variant == 1)
        LPG_UPD_(1, 8, true, true, true);
    else
        LPG_UPD(1, 8, false, false);
#undef LPG_UPD
#undef LPG_UPD_
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------------
// flush (deferred mode, a12 blocked): apply the np pending pivots to the
// constraint rows 0..nloc-1 in ONE read-modify-write pass over HBM instead
// of np passes. Per element the np fma run in pending order -- bit for bit
// what np eager updates compute; the (at most np) pivot rows, whose chain
// restarts at x = P_q[j], are rewritten by k_flush_pivot_rows right after.
// Columns whose pending P entries are all zero are skipped (as in k_update).
// Two kernels, both on the matrix cores: k_flushm (blocks of <= 32 pivots)
// and k_flushw (64-pivot blocks). (Round 1 also carried VALU-fma and
// one-column-per-lane MFMA forms, bitwise identical and slower; removed.)
// ------------------------------------------------------------------------

// ------------------------------------------------------------------------
// k_flushm: the flush on the matrix cores. A block of np pending pivots is
// the rank-np update T -= C (rows x np) * P (np x cols) evaluated in pending
// order per element, and v_mfma_f64_16x16x4_f64 computes
//   D[i][j] = fma(A[i][3], B[3][j], fma(A[i][2], B[2][j], fma(A[i][1], B[1][j],
//             fma(A[i][0], B[0][j], C[i][j]))))
// bit for bit (tools/mfma_f64_probe.hip, profiles/r01_mfma_f64_probe.log:
// random, subnormal, signed-zero and inf/nan operands), i.e. four steps of
// the eager chain with A = -C_q[i], B = P_q[j]. K/4 chained MFMAs per 16x16
// tile therefore reproduce K eager updates exactly, with no LDS broadcast of
// C and no per-element VALU work. Slots q >= np use A = -0, B = +0
// (x + -0 == x).
//
// Wave tile: 16 rows x 32*NPAIR columns. Lane l owns column pair
// 2*(l & 15) (+32 pp) and rows (l >> 4) + 4r, r = 0..3: one 16-byte load per
// (pair, r), whose .x / .y halves are the accumulators of the even-column and
// odd-column MFMA tiles (D layout: col = l & 15, row = (l >> 4) + 4r). The
// B fragments (P_q[j], q = 4g + (l >> 4)) stay in VGPRs for the whole strip;
// the A fragments (-C_q[i + (l & 15)]) are loaded per 16-row step. The next
// step's tableau loads are issued before the current step's MFMAs.
// ------------------------------------------------------------------------

typedef double d4 __attribute__((ext_vector_type(4)));

template <int KMAX, int NPAIR, bool NT, int SR, int LB>
__global__ __launch_bounds__(kBlock, LB > 0 ? LB : 1) void k_flushm(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                   const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                   int64_t cs, int64_t ntiles, int64_t nitems, int skip) {
    constexpr int G = KMAX / 4;             // MFMA k-steps
    constexpr int WC = 32 * NPAIR;          // columns per wave
    constexpr int64_t strip_rows = SR;
    __shared__ __attribute__((aligned(16))) double sC[KMAX * SR];   // the strip's C, [slot][row]
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    __shared__ int64_t next_item;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * strip_rows;
        const int64_t i1 = i0 + strip_rows < g.nloc ? i0 + strip_rows : g.nloc;
        const int64_t c0 = tile * (4 * WC) + wave * WC;
        // B fragments and column liveness
        double b[NPAIR][2][G];
        bool ok[NPAIR];
        int nlive = 0;
#pragma unroll
        for (int pp = 0; pp < NPAIR; pp++) {
            const int64_t col = c0 + 32 * pp + 2 * lc;
            const bool in = col < g.ncols;     // col even, ld even: col + 1 < ld
            bool live = false;
#pragma unroll
            for (int gq = 0; gq < G; gq++) {
                const int q = 4 * gq + lk;
                d2 v = d2{0.0, 0.0};
                if (in && q < np) v = *(const d2 *)(Pbuf + (int64_t)q * ld + col);
                b[pp][0][gq] = v.x;
                b[pp][1][gq] = v.y;
                live = live || v.x != 0.0 || v.y != 0.0;
            }
            // a column pair is live if any of its P entries over all slots is
            // non-zero: OR over the 4 lanes holding its k-slices
            live = __shfl_xor((int)live, 16, 64) | (int)live;
            live = __shfl_xor((int)live, 32, 64) | (int)live;
            ok[pp] = in && (!skip || live);
            nlive += ok[pp] ? (col + 1 < g.ncols ? 2 : 1) : 0;
        }
        const int cnt = __syncthreads_count(nlive > 0);
        if (cnt == 0) continue;
        {   // touched doubles: each pair counted once (by its lk == 0 lane)
            int mine = lk == 0 ? nlive : 0;
            for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
            __shared__ int wsum[kBlock / 64];
            if (lane == 0) wsum[wave] = mine;
            __syncthreads();
            if (threadIdx.x == 0)
                touched += (unsigned long long)(wsum[0] + wsum[1] + wsum[2] + wsum[3]) * (unsigned long long)(i1 - i0);
        }
        // stage C_q[i0 .. i0 + SR) for every slot (zeros past np and past i1: A = -0 there)
        for (int e = threadIdx.x; e < KMAX * SR / 2; e += kBlock) {
            const int q = e / (SR / 2), rr = 2 * (e % (SR / 2));
            d2 v = d2{0.0, 0.0};
            if (q < np && i0 + rr < i1) v = *(const d2 *)(Cbuf + (int64_t)q * cs + i0 + rr);   // i0 + rr + 1 < cs
            *(d2 *)(sC + q * SR + rr) = v;
        }
        __syncthreads();
        d2 t[NPAIR][4];
        auto load = [&](d2 (&x)[NPAIR][4], int64_t i) {
#pragma unroll
            for (int pp = 0; pp < NPAIR; pp++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i + lk + 4 * r;
                    const d2 *a = (const d2 *)(T + row * ld + c0 + 32 * pp + 2 * lc);
                    x[pp][r] = (ok[pp] && row < i1) ? (NT ? __builtin_nontemporal_load(a) : *a) : d2{0.0, 0.0};
                }
        };
        int64_t i = i0;
        load(t, i);
        for (;;) {
            const bool more = i + 16 < i1;
            d2 tn[NPAIR][4];
            if (more) load(tn, i + 16);
            const int lr = (int)(i - i0) + lc;
#pragma unroll
            for (int pp = 0; pp < NPAIR; pp++) {
                d4 ae = d4{t[pp][0].x, t[pp][1].x, t[pp][2].x, t[pp][3].x};
                d4 ao = d4{t[pp][0].y, t[pp][1].y, t[pp][2].y, t[pp][3].y};
                // A fragments from LDS in groups of 4 k-steps (a compiler fence between
                // groups keeps at most 8 of them live: fewer VGPRs, more waves per SIMD)
#pragma unroll
                for (int g0 = 0; g0 < G; g0 += 4) {
                    double a[4];
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (g0 + u < G) a[u] = -sC[(4 * (g0 + u) + lk) * SR + lr];
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        if (g0 + u < G) {
                            ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[pp][0][g0 + u], ae, 0, 0, 0);
                            ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[pp][1][g0 + u], ao, 0, 0, 0);
                        }
                    }
                    if (LB > 0) asm volatile("" ::: "memory");
                }
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i + lk + 4 * r;
                    if (ok[pp] && row < i1) {
                        d2 *dst = (d2 *)(T + row * ld + c0 + 32 * pp + 2 * lc);
                        const d2 v = d2{ae[r], ao[r]};
                        if (NT) __builtin_nontemporal_store(v, dst);
                        else *dst = v;
                    }
                }
            }
            if (!more) break;
            i += 16;
#pragma unroll
            for (int pp = 0; pp < NPAIR; pp++)
#pragma unroll
                for (int r = 0; r < 4; r++) t[pp][r] = tn[pp][r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

// k_flushw: k_flushm's wave tile (16 rows x 32 columns, 16-byte accesses,
// even/odd-column MFMA chains, B fragments in VGPRs) on TALL items, which is
// what keeps 64-pivot blocks memory-bound. A block's 4 waves sweep `rows`
// rows (runtime, multiple of 16) of a 128-column tile in 16-row bands, in
// step: the multipliers of band s (-C_q[i] in A-fragment order [q][row],
// 8 KB at KMAX = 64) sit in an NB-deep LDS ring, loaded into registers one
// band ahead and written one barrier later, and tableau band s+1 is loaded
// while band s is on the matrix cores. k_flushm instead stages the C of a
// whole 64-128-row strip per item (the LDS tile caps the strip at 64 rows
// for 64 slots) and restarts its pipeline per item: 2.36 ms vs 1.64 ms for
// this kernel at config 3, K = 64 (tools/flush_lab.hip,
// profiles/r01_flush_lab_k64.log). Same chain, same MFMA, bitwise identical.
// WPB waves per block: a tile is 32 * WPB columns wide, and every column
// tile reads all of C once (WPB = 8 halves that on-chip traffic: C is
// 8.4 MB at config 3, read by every tile from the Infinity Cache).
template <int KMAX, int NB, int LB, int WPB = 4>
__global__ __launch_bounds__(64 * WPB, LB) void k_flushw(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                         const double *__restrict__ Pbuf,
                                                         const double *__restrict__ Cbuf, int64_t cs, int64_t ntiles,
                                                         int64_t nitems, int64_t rows, int skip, FlushX X,
                                                         const int32_t *__restrict__ tlive,
                                                         const int64_t *__restrict__ lv,
                                                         const int32_t *__restrict__ inv) {
    constexpr int NTH = 64 * WPB;
    constexpr int G = KMAX / 4;
    constexpr int BAND = KMAX * 16;                 // doubles per band
    constexpr int NPC = BAND / 2;                   // 16-byte multiplier pieces per band
    constexpr int PER = (NPC + NTH - 1) / NTH;      // ... per thread (the last round partial when NTH does not divide)
    static_assert(PER >= 1, "band staging");
    __shared__ __attribute__((aligned(16))) double sC[NB][BAND];
    __shared__ int64_t next_item;
    __shared__ int next_grp;
    __shared__ int wsum[WPB];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    const int g0 = (int)(blockIdx.x & 7);   // blocks with the same b % 8 share an XCD
    int gd = 0;                             // X.on: queue g0 + gd (mod 8) is being drained
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if (X.on) {
                int64_t it = -1;
                int grp = 0;
                for (; gd < 8; gd++) {
                    grp = (g0 + gd) & 7;
                    const int64_t cnt = flushx_group(X, grp).count;
                    if (cnt == 0) continue;
                    it = (int64_t)atomicAdd(&st->gwork[grp], 1ull);
                    if (it < cnt) break;
                    it = -1;
                }
                next_item = it;
                next_grp = grp;
            } else {
                next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
            }
        }
        __syncthreads();
        const int64_t item = next_item;
        int64_t tile, i0, i1;
        if (X.on) {
            if (item < 0) break;
            const int grp = next_grp;
            flushx_item(X, flushx_group(X, grp), grp, item, tile, i0, i1);
        } else {
            if (item >= nitems) break;
            flush_item(item, ntiles, rows, g.nloc, tile, i0, i1);
        }
        // region mode (launch_flush_main): a tile without block-start nonbasic
        // columns holds live entries only in a leaving column of the block, if
        // any (one whose trade did not move it); otherwise it is skipped
        // without reading its pending P entries
        if (tlive) {
            constexpr int NCH = 32 * WPB / 64;
            const int64_t ch = tile * NCH + threadIdx.x;
            const bool maybe = threadIdx.x < NCH && ch < ld / 64 && tlive[ch] != 0;
            if (!__syncthreads_or(maybe)) {
                bool hit = false;
                if ((int)threadIdx.x < np) {
                    const int64_t L = lv[threadIdx.x];
                    if (L > 0) {
                        const int64_t p = inv[L];
                        hit = p >= tile * (32 * WPB) && p < (tile + 1) * (32 * WPB);
                    }
                }
                if (!__syncthreads_or(hit)) continue;
            }
        }
        const int64_t cl = tile * (32 * WPB) + wave * 32 + 2 * lc;   // this lane's column pair
        const bool in = cl < g.ncols;                                // cl even, ld even: cl + 1 < ld
        double be[G], bo[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            d2 v = d2{0.0, 0.0};
            if (in && q < np) v = *(const d2 *)(Pbuf + (int64_t)q * ld + cl);
            be[gq] = v.x;
            bo[gq] = v.y;
            live = live || v.x != 0.0 || v.y != 0.0;
        }
        // a column pair is live if any of its P entries over all slots is
        // non-zero: OR over the 4 lanes holding its k-slices
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? (cl + 1 < g.ncols ? 2 : 1) : 0;   // live doubles per row, pairs counted once
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        const bool wlive = mine > 0;                                   // wave-uniform
        if (lane == 0) wsum[wave] = mine;
        if (__syncthreads_count(wlive && lane == 0) == 0) continue;    // the whole tile is skipped
        if (threadIdx.x == 0) {
            int sum = 0;
#pragma unroll
            for (int w = 0; w < WPB; w++) sum += wsum[w];
            touched += (unsigned long long)sum * (unsigned long long)(i1 - i0);
        }
        const int nb = (int)((i1 - i0 + 15) / 16);
        // multiplier piece e of band s: slot q = e / 8, band rows 2 (e % 8) .. +1
        // (zeros past np and past i1: A = -0 there, x + -0 == x)
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                const int q = e >> 3, rr = 2 * (e & 7);
                const int64_t row = i0 + 16 * s + rr;
                d2 v = d2{0.0, 0.0};
                if (s < nb && q < np && row < i1 && (NPC % NTH == 0 || e < NPC))
                    v = *(const d2 *)(Cbuf + (int64_t)q * cs + row);   // row + 1 < cs
                cr[u] = -v;
            }
        };
        auto cstore = [&](const d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++)
                if (NPC % NTH == 0 || threadIdx.x + u * NTH < NPC) *(d2 *)(&sC[s % NB][2 * (threadIdx.x + u * NTH)]) = cr[u];
        };
        for (int s = 0; s < NB - 1; s++) {   // prologue: bands 0 .. NB-2 into the ring
            d2 cr[PER];
            cload(cr, s);
            cstore(cr, s);
        }
        d2 cn[PER];
        cload(cn, NB - 1);
        auto tload = [&](d2 (&x)[4], int s) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                x[r] = (ok && row < i1) ? __builtin_nontemporal_load((const d2 *)(T + row * ld + cl)) : d2{0.0, 0.0};
            }
        };
        d2 t[4];
        tload(t, 0);
        for (int s = 0; s < nb; s++) {
            d2 tn[4];                         // one band ahead (two ahead measured no faster)
            if (s + 1 < nb) tload(tn, s + 1);
            __syncthreads();                  // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
            if (wlive) {
                d4 ae = d4{t[0].x, t[1].x, t[2].x, t[3].x};
                d4 ao = d4{t[0].y, t[1].y, t[2].y, t[3].y};
                const double *sa = &sC[s % NB][lk * 16 + lc];
                // the next pair of A operands is read while this pair's four
                // MFMAs run: left to the scheduler, every ds_read sat behind
                // the MFMAs of the pair before and the chain waited an LDS
                // round trip per four MFMAs (config 3, K = 96: 29.7-29.8k vs
                // 28.6-28.8k pivots/s, profiles/r05_ab_flushw_aprefetch.log)
                double a0 = sa[0], a1 = sa[64];
#pragma unroll
                for (int gq = 0; gq < G; gq += 2) {
                    double n0 = 0.0, n1 = 0.0;
                    if (gq + 2 < G) {
                        n0 = sa[(gq + 2) * 64];
                        n1 = sa[(gq + 3) * 64];
                    }
                    __builtin_amdgcn_sched_barrier(0);   // the reads stay in front of the MFMAs
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, be[gq], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bo[gq], ao, 0, 0, 0);
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, be[gq + 1], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bo[gq + 1], ao, 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                    a0 = n0;
                    a1 = n1;
                }
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * s + lk + 4 * r;
                    if (ok && row < i1) __builtin_nontemporal_store(d2{ae[r], ao[r]}, (d2 *)(T + row * ld + cl));
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

// The pivot rows of the block, after the block pass: row r_q (q its last
// pivot in the block) = P_q continued by the chain of the later pivots,
// x = fma(mul[u][q], P_u[j], x) for u = q+1 .. np-1 (mul[u][q] = -C_u[r_q],
// built by k_swap_plan). These values do not depend on T_base, so the rows
// the pass wrote without the replacement are simply overwritten. A block
// takes 64 columns and every pivot row: the block's P entries and the
// multipliers are staged in LDS once, so each P entry leaves HBM once (the
// per-row form re-read P_u for every earlier pivot row: 98 us at config 3).
// Each wave runs groups of 4 consecutive rows, so one LDS read of P_u[j]
// feeds 4 chains (groups {w, 7-w, 8+w, 15-w, ...}: equal work per wave); the
// first steps of a group, where only some of its rows have started, are
// peeled so that every row sees exactly its own steps. K = 64: the
// multipliers are staged in LDS too; K = 96 / 128 (72 / 128 KB of them) read them as
// wave-uniform loads, and r_q of slots 64 .. 127 sits in a second register.
template <int K>
__global__ __launch_bounds__(kBlock) void k_flush_pivot_rows(double *__restrict__ T, Geo g,
                                                             const DevState *__restrict__ st,
                                                             const double *__restrict__ Pbuf,
                                                             const double *__restrict__ mul,
                                                             const int64_t *__restrict__ rq) {
    static_assert((K == 64 || K == 96 || K == 128) && K <= LPG_DEFER_MAX && kBlock == 256,
                  "4 waves x K/16 groups of 4 rows");   // (96: measured, not launched)
    constexpr bool LM = K == 64;                        // multipliers in LDS
    constexpr int PW = K / (kBlock / 64);               // P rows staged per wave
    constexpr int MT = LM ? K * K / kBlock : 1;         // multipliers staged per thread
    __shared__ double sP[K][64];
    __shared__ __attribute__((aligned(32))) double sM[LM ? K * K : 4];   // [u][q]
    // K = 128: each wave stages its group's multipliers mul[u][q0 .. q0 + 3]
    // (4 KB) in its own LDS rows, all loads in flight at once (a uniform load
    // per chain step would wait for each in turn)
    __shared__ __attribute__((aligned(32))) double sMg[LM ? 1 : kBlock / 64][LM ? 1 : K][4];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * 64 + c;
    const bool ok = j < g.ncols;
    {
        double v[PW], m[MT];
#pragma unroll
        for (int k = 0; k < PW; k++) {
            const int u = w + 4 * k;
            v[k] = (ok && u < np) ? Pbuf[(int64_t)u * g.ld + j] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < MT; k++) {
            const int e = threadIdx.x + kBlock * k;   // [u][q] in rows of K
            m[k] = (LM && e / K < np) ? mul[(e / K) * LPG_DEFER_MAX + e % K] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < PW; k++) sP[w + 4 * k][c] = v[k];
        if (LM) {
#pragma unroll
            for (int k = 0; k < MT; k++) sM[threadIdx.x + kBlock * k] = m[k];
        }
    }
    const int64_t ru = c < np ? rq[c] : -1;             // lane u: r_u
    const int64_t ru1 = K > 64 && 64 + c < np ? rq[64 + c] : -1;   // lane u: r_{64 + u}
    __syncthreads();
#pragma unroll 1
    for (int k = 0; k < K / 16; k++) {
        const int grp = (k & 1) ? 8 * (k >> 1) + 7 - w : 8 * (k >> 1) + w;
        const int q0 = 4 * grp;
        if (q0 >= np) continue;                         // uniform
        double x0 = sP[q0][c], x1 = sP[q0 + 1][c], x2 = sP[q0 + 2][c], x3 = sP[q0 + 3][c];
        if (!LM) {                                      // this wave's rows only: no barrier
#pragma unroll
            for (int k = 0; k < (LM ? 1 : (K + 63) / 64); k++) {
                const int u = c + 64 * k;
                if (u < K) {
                    const d4 m = *(const d4 *)(mul + (u < np ? u : 0) * LPG_DEFER_MAX + q0);
                    *(d4 *)&sMg[LM ? 0 : w][LM ? 0 : u][0] = u < np ? m : d4{0.0, 0.0, 0.0, 0.0};
                }
            }
        }
        auto m4 = [&](int u) {                          // mul[u][q0 .. q0 + 3]
            return LM ? *(const d4 *)(sM + u * K + q0) : *(const d4 *)&sMg[LM ? 0 : w][LM ? 0 : u][0];
        };
        if (q0 + 1 < np) {
            const double p = sP[q0 + 1][c];
            const d4 m = m4(q0 + 1);
            x0 = fma(m[0], p, x0);
        }
        if (q0 + 2 < np) {
            const double p = sP[q0 + 2][c];
            const d4 m = m4(q0 + 2);
            x0 = fma(m[0], p, x0);
            x1 = fma(m[1], p, x1);
        }
        if (q0 + 3 < np) {
            const double p = sP[q0 + 3][c];
            const d4 m = m4(q0 + 3);
            x0 = fma(m[0], p, x0);
            x1 = fma(m[1], p, x1);
            x2 = fma(m[2], p, x2);
        }
#pragma unroll 2
        for (int u = q0 + 4; u < np; u++) {
            const double p = sP[u][c];
            const d4 m = m4(u);
            x0 = fma(m[0], p, x0);
            x1 = fma(m[1], p, x1);
            x2 = fma(m[2], p, x2);
            x3 = fma(m[3], p, x3);
        }
        const double xs[4] = {x0, x1, x2, x3};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int q = q0 + i;
            if (q >= np) break;                         // uniform
            const int64_t r = q < 64 ? (int64_t)rdl64((uint64_t)ru, q) : (int64_t)rdl64((uint64_t)ru1, q - 64);
            if (r < 0) continue;                        // pivot row on another rank
            if (__ballot(c > q && ru == r)) continue;   // a later pivot replaces this row again
            if (K > 64 && __ballot(64 + c > q && ru1 == r)) continue;
            if (ok) T[r * g.ld + j] = xs[i];
        }
    }
}

// ------------------------------------------------------------------------
// Basis-partitioned column order (lpg_internal.h). Events of the block: pivot
// q enters kq[q] and lets lv[q] leave. A column whose first and last events
// are both "enter" went nonbasic -> basic (set E), both "leave": basic ->
// nonbasic (set L); |E| == |L|. The i-th of E (in event order) trades
// physical positions with the i-th of L. One wave; pairs[0] = count, then
// triples (a, b, r): a = E's physical column, b = L's, r = the row E entered
// on (its last event).
//
// The trade happens around the block pass, not after it, so the pass never
// meets L's columns scattered over the basic region:
//   k_move_cols (before): constraint rows take L's base column at a, the
//     pending P rows take L's entries at a and +0 at b (b is then skipped by
//     the pass); the objective rows, which are current, swap a and b.
//   k_fill_cols (after the pass and the pivot-row rewrite): column b = E's
//     final column, the unit vector e_r. Exactly: when E enters at pivot q,
//     P_q[E] = piv / piv = 1 and every other row becomes fma(-x, 1, x) = +0;
//     a later pivot u has P_u[E] = +0 / piv_u = +0 when piv_u > 0, so every
//     row stays +0 (+0 + +-0 == +0) and row r stays 1. The plan therefore
//     pairs nothing in a block holding a pivot element that is not positive
//     (the forced pivots of lpg_pivot may be negative).
// ------------------------------------------------------------------------

// grid: 1 + kMulBlocks blocks of one wave. Block 0: the column plan (when
// plan != 0). Blocks 1..: the multipliers of k_flush_pivot_rows,
// mul[u][q] = -C_u[r_q] for u > q (+0 elsewhere), rows of LPG_DEFER_MAX.
constexpr int kMulBlocks = 8;
constexpr int kPlanNT = LPG_DEFER_MAX;                     // one thread per event / slot
//
// Every block first checks the pending block it is about to index with: npend
// within [0, kmax], and for each pending pivot q: rq[q] a local row in
// [-1, nloc) and, with a plan, kq[q] and lv[q] logical columns in [1, ncols). A block stopped
// mid-way (a stall, a give-up of the owner push) can leave npend ahead of the
// slots it filled. On a violation no block writes anything it indexes with
// those values; block 0 empties the pending block (npend = 0, pairs[0] = 0:
// every flush kernel after this one is a no-op), stops a RUNNING loop with
// NUMERIC and records kStallPending (lpg_last_error names it). Blocks that
// read npend after block 0 cleared it see an empty block: the same outcome.
__global__ __launch_bounds__(kPlanNT) void k_swap_plan(DevState *__restrict__ st, const int64_t *__restrict__ kq,
                                                  const int64_t *__restrict__ lv, const int64_t *__restrict__ rq,
                                                  const double *__restrict__ Cbuf, int64_t cs,
                                                  int32_t *__restrict__ colmap, int32_t *__restrict__ inv,
                                                  int32_t *__restrict__ pairs, double *__restrict__ mul, int plan,
                                                  const double *__restrict__ pv, int64_t nloc, int64_t ncols, int kmax) {
    const int64_t np64 = st->npend;
    const bool npbad = np64 < 0 || np64 > kmax;
    const int np = npbad ? 0 : (int)np64;
    {
        const int q = threadIdx.x;
        int what = npbad ? 1 : 0;
        int64_t val = np64;
        if (!npbad && q < np) {
            // kq / lv only feed the column plan (the generic deferred k_prep
            // records neither, and runs without one)
            const int64_t x = plan ? kq[q] : 1, y = plan ? lv[q] : 1, r = rq[q];
            if (x < 1 || x >= ncols) what = 2, val = x;
            else if (y < 1 || y >= ncols) what = 3, val = y;
            else if (r < -1 || r >= nloc) what = 4, val = r;
        }
        __shared__ int first;
        if (q == 0) first = kPlanNT;
        __syncthreads();
        if (what) atomicMin(&first, q);
        if (__syncthreads_or(what != 0)) {
            if (blockIdx.x == 0 && q == first) {
                if (st->stall == 0) {       // a stall already recorded (the cause, e.g. an exchange give-up) is kept
                    st->stall_info[0] = what;   // 1 npend, 2 kq, 3 lv, 4 rq
                    st->stall_info[1] = q;
                    st->stall_info[2] = val;
                    st->stall_info[3] = np64;
                    st->stall = kStallPending;
                }
                st->npend = 0;
                if (pairs) pairs[0] = 0;
                for (int u = 0; u < 2; u++)
                    if (st->slot[u].status == RUNNING) st->slot[u].status = NUMERIC;
            }
            return;
        }
    }
    if (blockIdx.x > 0) {                                   // mul[u][q], lane q
        constexpr int UB = LPG_DEFER_MAX / kMulBlocks;       // pivots u per block
        const int q = threadIdx.x;
        const int u0 = (blockIdx.x - 1) * UB;
        const int64_t r = q < np ? rq[q] : -1;
        double v[UB];
#pragma unroll
        for (int k = 0; k < UB; k++) {   // unconditional loads (clamped address, then a select): all in flight
            const int u = u0 + k;
            const bool on = u > q && u < np && r >= 0;
            const double c = Cbuf[(int64_t)(on ? u : 0) * cs + (on ? r : 0)];
            v[k] = on ? -c : 0.0;
        }
#pragma unroll
        for (int k = 0; k < UB; k++)
            if (u0 + k < np) mul[(u0 + k) * LPG_DEFER_MAX + q] = v[k];
        return;
    }
    if (!plan) return;
    const int q = threadIdx.x;
    const int64_t x = q < np ? kq[q] : -1, y = q < np ? lv[q] : -1, rx = q < np ? rq[q] : -1;
    // pivot element of pivot q (C_q[r_q], recorded by k_prep_d on every rank, so that every rank of a
    // row partition -- most of which do not hold row r_q -- makes the same plan)
    const bool pos = q >= np || pv[q] > 0.0;
    __shared__ int64_t sx[kPlanNT], sy[kPlanNT];          // the events, read back as broadcasts
    sx[q] = x;
    sy[q] = y;
    // x (entering at q) is in E iff no later event touches x and its first event is an entry
    bool inE = q < np, inL = q < np;
    int fx = q, fy = q;           // first event index of x / y, and its kind
    bool fxe = true, fye = false;
    const bool allpos = __syncthreads_count(!pos) == 0;   // also publishes sx / sy
    // an incomplete trade moves the nonbasic columns: region mode must rebuild (DevState::rbad)
    if (q == 0 && np > 0 && !allpos) st->rbad = 1;
#pragma unroll 8
    for (int u = 0; u < np; u++) {
        const int64_t a = sx[u], b = sy[u];
        if (u > q) {
            if (a == x || b == x) inE = false;
            if (a == y || b == y) inL = false;
        } else if (u < q) {
            if (a == x && u < fx) { fx = u; fxe = true; }
            if (b == x && u < fx) { fx = u; fxe = false; }
            if (a == y && u < fy) { fy = u; fye = true; }
            if (b == y && u < fy) { fy = u; fye = false; }
        }
    }
    inE = inE && fxe && allpos;
    inL = inL && !fye && allpos;
    // ranks in event order: within the wave by ballot, across waves by the counts of the waves before
    constexpr int NW = kPlanNT / 64;
    const int lane = q & 63, wv = q >> 6;
    const unsigned long long me = __ballot(inE), ml = __ballot(inL);
    __shared__ int cE[NW], cL[NW];
    if (lane == 0) {
        cE[wv] = __popcll(me);
        cL[wv] = __popcll(ml);
    }
    __syncthreads();
    int oE = 0, oL = 0, n = 0;   // n: |E| == |L|
#pragma unroll
    for (int w = 0; w < NW; w++) {
        oE += w < wv ? cE[w] : 0;
        oL += w < wv ? cL[w] : 0;
        n += cE[w];
    }
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int ie = oE + __popcll(me & below), il = oL + __popcll(ml & below);
    __shared__ int64_t eE[kPlanNT], eL[kPlanNT], eR[kPlanNT], eRL[kPlanNT];
    if (inE) {
        eE[ie] = x;
        eR[ie] = rx;
    }
    if (inL) {
        eL[il] = y;
        eRL[il] = rx;      // y was basic in row r_q from the block start until it left at q
    }
    __syncthreads();
    if (q < n) {
        const int64_t ce = eE[q], cl = eL[q];
        const int32_t a = inv[ce], b = inv[cl];
        pairs[1 + kPairW * q] = a;
        pairs[2 + kPairW * q] = b;
        pairs[3 + kPairW * q] = (int32_t)eR[q];
        pairs[4 + kPairW * q] = (int32_t)eRL[q];
        colmap[a] = (int32_t)cl;
        colmap[b] = (int32_t)ce;
        inv[cl] = a;
        inv[ce] = b;
    }
    if (q == 0) pairs[0] = n;
}

// grid: (row blocks + npb, 4). One thread per row (constraint and objective
// rows) and group of 16 pairs (blockIdx.y); the last npb x-blocks move the
// pending P entries, one (pending pivot, pair) per thread (a 96-pivot block
// trades up to 96 pairs: 9,216 moves, which one block's loop of dependent
// loads took ~40 us to make).
__global__ __launch_bounds__(kBlock) void k_move_cols(double *__restrict__ T, Geo g, const DevState *__restrict__ st,
                                                      double *__restrict__ Pbuf, const int32_t *__restrict__ pairs,
                                                      int npb, int unit) {
    const int n = pairs[0];
    if (n == 0) return;
    const int nrb = (int)gridDim.x - npb;
    if ((int)blockIdx.x >= nrb) {
        const int np = (int)st->npend;
        const int nt = npb * (int)gridDim.y * kBlock;
        for (int e = (((int)blockIdx.x - nrb) * (int)gridDim.y + (int)blockIdx.y) * kBlock + threadIdx.x; e < np * n;
             e += nt) {
            const int q = e / n, p = e - q * n;
            double *Pq = Pbuf + (int64_t)q * g.ld;
            const int32_t a = pairs[1 + kPairW * p], b = pairs[2 + kPairW * p];
            Pq[a] = Pq[b];
            Pq[b] = 0.0;
        }
        return;
    }
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= g.nloc + g.nobj) return;
    const bool obj = i >= g.nloc;
    double *row = T + i * g.ld;
    for (int p0 = 16 * blockIdx.y; p0 < n; p0 += 16 * gridDim.y) {      // 16 pairs' loads in flight at once
        double va[16], vb[16];
        int ia[16], ib[16], rl[16];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            ia[u] = p0 + u < n ? pairs[1 + kPairW * (p0 + u)] : 0;
            ib[u] = p0 + u < n ? pairs[2 + kPairW * (p0 + u)] : 0;
            rl[u] = p0 + u < n ? pairs[4 + kPairW * (p0 + u)] : -1;
        }
        // unit: L's base column is the unit vector of its row (-1: another
        // rank's), so a constraint row writes it without reading it
#pragma unroll
        for (int u = 0; u < 16; u++) {
            vb[u] = (unit && !obj) ? ((int64_t)rl[u] == i ? 1.0 : 0.0) : row[ib[u]];
            va[u] = obj ? row[ia[u]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (p0 + u < n) {
                row[ia[u]] = vb[u];
                if (obj) row[ib[u]] = va[u];
            }
    }
}

// grid: (row blocks, 4): constraint row i, pairs p = blockIdx.y (mod 4).
// st: the pending block is applied, clear it and the dequeue head (no kernel
// of this launch reads them)
// End of a block, after every consumer of its slots (the plan, the pass, the
// pivot-row rewrite): the slots return to the "never filled" sentinels, so a
// later block whose npend runs ahead of the slots it filled (a block stopped
// mid-way) meets a slot k_swap_plan refuses instead of the previous block's
// in-range values: rq = kNoSlot (< -1), kq = lv = 0 (no column).
// Region mode (spare_zero, lpg_block.hip REG): a column that left the basis
// during the block is held by a spare slot, which wrote its Pbuf entries; a
// column that left and entered again stays basic and is held by nobody in the
// next block, so its entries are zeroed here (every leaving column's, at its
// position after the trade -- a live column's are rewritten by the next block
// before they are read), keeping the next block's pass from applying them.
__device__ __forceinline__ void end_block(DevState *st, const Defer &D, int kmax, bool spare_zero = false,
                                          int64_t ld = 0) {
    const int q = threadIdx.x;
    if (spare_zero) {              // one leaving column per thread: its kmax entries, no dependent load inside
        const int64_t L = q < kmax ? D.lv[q] : 0;
        if (L > 0) {
            double *col = D.Pbuf + D.inv[L];
            for (int u = 0; u < kmax; u++) col[(int64_t)u * ld] = 0.0;
        }
        __syncthreads();
    }
    if (q == 0) {
        st->npend = 0;
        st->fwork = 0;
    }
    if (q < 8) st->gwork[q] = 0;
    for (int u = q; u < kmax; u += blockDim.x) {
        D.rq[u] = kNoSlot;
        if (D.kq) D.kq[u] = 0;
        if (D.lv) D.lv[u] = 0;
    }
}

__global__ __launch_bounds__(kBlock) void k_end_block(DevState *__restrict__ st, Defer D, int kmax) {
    end_block(st, D, kmax);
}

// bcol0 (region mode): every row's basic column for the next block, {logical, physical}
// (all m rows of the LP: on a rank of a row partition the spare of a pivot on
// another rank's row reads it too)
__global__ __launch_bounds__(kBlock) void k_fill_cols(double *__restrict__ T, Geo g, const int32_t *__restrict__ pairs,
                                                      DevState *__restrict__ st, Defer D, int kmax,
                                                      int64_t *__restrict__ bcol0) {
    if (st && blockIdx.x == 0 && blockIdx.y == 0) end_block(st, D, kmax, bcol0 != nullptr, g.ld);
    if (bcol0 && blockIdx.y == 0) {
        for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < g.m; r += (int64_t)gridDim.x * kBlock) {
            const int64_t v = D.basis[r];
            bcol0[r] = (v << 32) | (int64_t)(uint32_t)D.inv[v];
        }
    }
    const int n = pairs[0];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= g.nloc || n == 0) return;
    double *row = T + i * g.ld;
    for (int p = blockIdx.y; p < n; p += gridDim.y)
        row[pairs[2 + kPairW * p]] = (i == (int64_t)pairs[3 + kPairW * p]) ? 1.0 : 0.0;
}

int launch_swap_plan(const Launch &L, const Geo &g, DevState *st, const Defer &D, int32_t *colmap, int32_t *inv,
                     int32_t *pairs, int plan, int kmax) {
    kmax = flush_kmax_supported(kmax);
    if (!kmax || (plan && !pairs)) return -1;
    hipLaunchKernelGGL(k_swap_plan, dim3(1 + kMulBlocks), dim3(kPlanNT), 0, (hipStream_t)L.stream, st, D.kq, D.lv, D.rq,
                       D.Cbuf, D.cs, colmap, inv, pairs, D.mul, plan, D.pv, g.nloc, g.ncols, kmax);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_move_cols(const Launch &L, const Geo &g, const DevState *st, const Defer &D, const int32_t *pairs,
                     int unit) {
    const int64_t rows = g.nloc + g.nobj;
    const int npb = (LPG_DEFER_MAX * LPG_DEFER_MAX + 4 * kBlock - 1) / (4 * kBlock);   // one move per thread at the most
    hipLaunchKernelGGL(k_move_cols, dim3((unsigned)((rows + kBlock - 1) / kBlock + npb), 4), dim3(kBlock), 0,
                       (hipStream_t)L.stream, g.T, g, st, D.Pbuf, pairs, npb, unit);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_fill_cols(const Launch &L, const Geo &g, const int32_t *pairs, DevState *st, const Defer *D, int kmax,
                     int64_t *bcol0) {
    if (st && (!D || !D->rq || kmax < 1 || kmax > LPG_DEFER_MAX)) return -1;
    if (bcol0 && (!st || !D->basis || !D->inv || !D->lv || !D->Pbuf)) return -1;
    hipLaunchKernelGGL(k_fill_cols, dim3((unsigned)std::max<int64_t>((g.nloc + kBlock - 1) / kBlock, 1), 4), dim3(kBlock),
                       0, (hipStream_t)L.stream, g.T, g, pairs, st, D ? *D : Defer{}, kmax, bcol0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// tmp[r][j] = T[i0 + r][inv[j]], j < ncols (column 0 and the padding map to themselves)
__global__ __launch_bounds__(kBlock) void k_gather_rows(const double *__restrict__ T, Geo g,
                                                        const int32_t *__restrict__ inv, double *__restrict__ tmp,
                                                        int64_t i0, int64_t nr) {
    const int64_t r = blockIdx.y;
    if (r >= nr) return;
    const double *src = T + (i0 + r) * g.ld;
    double *dst = tmp + r * g.ld;
    for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < g.ncols; j += (int64_t)gridDim.x * kBlock)
        dst[j] = src[inv[j]];
}

int launch_gather_rows(const Launch &L, const Geo &g, const int32_t *inv, double *tmp, int64_t i0, int64_t nr) {
    const int64_t tiles = std::min<int64_t>((g.ncols + kBlock - 1) / kBlock, 64);
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)tiles, (unsigned)nr), dim3(kBlock), 0, (hipStream_t)L.stream,
                       g.T, g, inv, tmp, i0, nr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void k_iota(int32_t *a, int64_t n) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        a[j] = (int32_t)j;
}

int launch_iota(const Launch &L, int32_t *a, int64_t n) {
    hipLaunchKernelGGL(k_iota, dim3(256), dim3(kBlock), 0, (hipStream_t)L.stream, a, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int flush_kmax_supported(int k) {
    if (k <= 8) return 8;
    if (k <= 16) return 16;
    if (k <= 32) return 32;
    if (k <= 64) return 64;
    if (k <= 96) return 96;
    if (k <= 128 && k <= LPG_DEFER_MAX) return 128;
    return 0;
}

static_assert(offsetof(DevState, fwork) == offsetof(DevState, npend) + sizeof(int64_t),
              "launch_flush clears npend and fwork with one memset");

int launch_flush_tail(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, bool reset) {
    kmax = flush_kmax_supported(kmax);
    if (!kmax) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
    const int64_t ntiles_p = (g.ncols + 63) / 64;   // k_flush_pivot_rows column tiles
    // (96-slot blocks take the 128-slot form: a 96-slot instance, two blocks
    // per CU, measured 0.2% slower at config 4, profiles/r04_ab_pivrows96.log)
#ifdef LPG_PIVROWS96
    if (kmax == 96)
        hipLaunchKernelGGL(k_flush_pivot_rows<96>, dim3((unsigned)ntiles_p), dim3(kBlock), 0, stream, g.T, g, st,
                           D.Pbuf, D.mul, D.rq);
    else
#endif
    if (kmax > 64)
        hipLaunchKernelGGL(k_flush_pivot_rows<128>, dim3((unsigned)ntiles_p), dim3(kBlock), 0, stream, g.T, g, st,
                           D.Pbuf, D.mul, D.rq);
    else
        hipLaunchKernelGGL(k_flush_pivot_rows<64>, dim3((unsigned)ntiles_p), dim3(kBlock), 0, stream, g.T, g, st,
                           D.Pbuf, D.mul, D.rq);
    if (hipGetLastError() != hipSuccess) return -1;
    if (!reset) return 0;
    // the pending block is applied: clear it, the dequeue head and the slots
    hipLaunchKernelGGL(k_end_block, dim3(1), dim3(kBlock), 0, stream, st, D, kmax);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_flush(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, int skip, int variant) {
    int rc = launch_swap_plan(L, g, st, D, nullptr, nullptr, nullptr, 0, kmax);   // the multipliers only
    if (!rc) rc = launch_flush_main(L, g, st, D, kmax, skip, variant);
    return rc ? rc : launch_flush_tail(L, g, st, D, kmax);
}

// the short tail items of the banded passes (flush_item); LPG_FLUSH_TAIL=0 turns them off
static bool flush_tail_on() {
    static const int on = [] {
        const char *v = getenv("LPG_FLUSH_TAIL");
        return v ? atoi(v) != 0 : 1;
    }();
    return on != 0;
}

// item height of the banded pass (LPG_FLUSH_ROWS overrides the default, a
// multiple of 64 from 64 to 8192; A/B runs)
static int64_t flush_rows_env(int64_t def) {
    static const int64_t v = [] {
        const char *e = getenv("LPG_FLUSH_ROWS");
        const long r = e ? atol(e) : 0;
        return (int64_t)((r >= 64 && r <= 8192 && r % 64 == 0) ? r : 0);
    }();
    return v ? v : def;
}

// the fill rule's item count (LPG_FLUSH_MINITEMS overrides, 256 .. 65536; A/B runs)
static int64_t flush_minitems_env(int64_t def) {
    static const int64_t v = [] {
        const char *e = getenv("LPG_FLUSH_MINITEMS");
        const long r = e ? atol(e) : 0;
        return (int64_t)((r >= 256 && r <= 65536) ? r : 0);
    }();
    return v ? v : def;
}

static int64_t env_range(const char *name, int64_t lo, int64_t hi) {   // 0 when unset or out of range
    const char *e = getenv(name);
    const long long v = e ? atoll(e) : 0;
    return (v >= lo && v <= hi) ? (int64_t)v : 0;
}

// FlushX (lpg_internal.h) for k_flushw. The band's multipliers, rs x kmax
// doubles, are kept within a budget of that XCD's 4 MB L2 (LPG_FLUSH_CB, KB,
// default 2048): the most column classes H whose bands fit, so P is re-read
// by 8 / H bands (one P tile read per band: the tile's pieces run back to
// back); bands that do not fit at H = 1 are swept in sub-bands that do. The
// tail: two rounds of short items per group's blocks (LPG_FLUSH_XTAIL tiles,
// LPG_FLUSH_XPIECES row pieces each).
// xcd: -1 auto (tableaus of >= 1024 rows and >= 64 tiles), 0 off (the global
// queue, flush_item), 1 on at any size, 10 + H on with H column classes (tests).
static FlushX flushx_plan(int64_t ntiles, int64_t nloc, int kmax, int64_t nblocks, int xcd) {
    FlushX X{};
    if (xcd == 0 || nloc < 1 || ntiles < 1 || (xcd < 0 && (nloc < 1024 || ntiles < 64))) return X;
    static const int64_t cb = env_range("LPG_FLUSH_CB", 256, 65536) * 1024;
    static const int64_t ttf = env_range("LPG_FLUSH_XTAIL", 1, 1 << 20);
    static const int64_t tqf = env_range("LPG_FLUSH_XPIECES", 1, 64);
    const int64_t budget = cb ? cb : (int64_t)2048 * 1024;
    auto band = [&](int H) { return ((nloc + 8 / H - 1) / (8 / H) + 15) / 16 * 16; };
    int H = 1;
    if (xcd == 11 || xcd == 12 || xcd == 14 || xcd == 18)
        H = xcd - 10;
    else
        for (int h : {8, 4, 2})
            if (band(h) * kmax * 8 <= budget) {
                H = h;
                break;
            }
    X.ntiles = ntiles;
    X.nloc = nloc;
    X.H = H;
    const int64_t rb = band(H);
    const int64_t nsb = std::max<int64_t>(1, (rb * kmax * 8 + budget - 1) / budget);
    X.rb = (int32_t)rb;
    X.rs = (int32_t)std::min<int64_t>(rb, ((rb + nsb - 1) / nsb + 15) / 16 * 16);
    X.tt = (int32_t)(ttf ? ttf : std::max<int64_t>(1, nblocks / 8 / 2));
    // eighth-height pieces: config 3 pass 2.130 -> 2.100 ms, config 5 0.192 -> 0.170 ms,
    // config 4 flat (16 / 32 pieces lose at config 5; fewer tail tiles cost config 5,
    // whose live columns sit in a few low tiles, a third; profiles/r06_ab_flush_pieces.log)
    X.tq = (int32_t)(tqf ? tqf : 8);
    X.on = 1;
    return X;
}

// which: -1 = default (k_flushw), 0 = k_flushm (blocks of <= 32 pivots),
// 1 = k_flushw (LPG_FLUSH_KERNEL=m|w, tests). Both bitwise.
int launch_flush_main(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, int skip, int which,
                      int xcd, const int32_t *tlive) {
    kmax = flush_kmax_supported(kmax);
    if (!kmax) return -1;
    // k_flushw by default at every block size: at 32 slots too it beats
    // k_flushm by 3-4% (m = 1024 .. 4096, profiles/r02_k32_flush.log)
    if (which < 0) which = 1;
    hipStream_t stream = (hipStream_t)L.stream;
    if (kmax >= 64) which = 1;                              // k_flushm's C tile caps it at 32 slots
    if (which == 1) {
        // k_flushw: 4-wave blocks, 128-column x 2048-row items swept in 16-row
        // bands with a 2-deep LDS ring of multipliers; small tableaus shrink
        // the items until they fill the chip
        // 64 slots: 8-wave blocks over 256-column tiles (one B fragment load
        // per 8 waves instead of 4; config 3: 25.25k vs 25.04k pivots/s,
        // interleaved A/B, profiles/r03_ab_flushw_wpb8.log)
        constexpr int kW64 = 8;
        // 96 slots: 8-wave blocks too (2 KB per tableau row per block instead of
        // 1 KB, one multiplier band staged for 8 waves): pass 2.177 -> 2.144 ms at
        // config 3, 35.23 -> 34.73 ms at config 4, three interleaved pairs
        // (profiles/r05_ab_flushw_w8.log); LPG_FLUSH_W96=4 restores 4-wave blocks
        static const int w96 = env_range("LPG_FLUSH_W96", 4, 4) == 4 ? 4 : 8;
        const bool wide = kmax == 64 || (kmax == 96 && w96 == 8);
        const int tw = wide ? 32 * kW64 : 128;   // tile width: 32 columns per wave
        const int64_t ntiles = (g.ncols + tw - 1) / tw;
        // Items of up to 2048 rows (round 4, with the short tail items): config 4
        // pass 34.5 -> 33.5 ms per 96-pivot block at 2048 vs 512 rows, 4096 /
        // 8192 within 0.6% of 2048; config 3 (halved to 1024 by the fill rule
        // below) 1.69 -> 1.64 ms (profiles/r04_c4_rows*.log, r04_c3_rows*.log).
        // Round 3, before the tail items: 1024 / 2048 within 1% of 512, 128
        // rows 13% slower.
        int64_t rows = flush_rows_env(2048);
        const int64_t minitems = flush_minitems_env(2048);
        while (rows > 64 && ntiles * ((g.nloc + rows - 1) / rows) < minitems) rows /= 2;
        if (!flush_tail_on()) rows = -rows;
        const int64_t nitems = flush_nitems(ntiles, rows, g.nloc);
        const int lb = kmax == 128 ? 1 : kmax == 96 ? 2 : kmax == 64 ? 2 : 3;   // VGPRs: 184 at 64 slots, <= 128 below
        const int bmul = wide ? 2 : 1;                                            // 8-wave blocks at 64 slots
        const FlushX X = flushx_plan(ntiles, g.nloc, kmax, (int64_t)256 * lb / bmul, xcd);
        int64_t nblocks = std::min<int64_t>(nitems, (int64_t)256 * lb);
        if (X.on) nblocks = (int64_t)256 * lb;
        if (nblocks < 1) return 0;
        const unsigned grid = (unsigned)((nblocks + bmul - 1) / bmul);
        const int32_t *TL = (tlive && D.lv && D.inv && g.ld % 64 == 0) ? tlive : nullptr;
        if (kmax == 128)
            hipLaunchKernelGGL((k_flushw<128, 2, 1, 4>), dim3(grid), dim3(256), 0, stream, g.T, g, st, D.Pbuf, D.Cbuf,
                               D.cs, ntiles, nitems, rows, skip, X, TL, D.lv, D.inv);
        else if (kmax == 96 && wide)
            hipLaunchKernelGGL((k_flushw<96, 2, 1, 8>), dim3(grid), dim3(512), 0, stream, g.T, g, st, D.Pbuf, D.Cbuf,
                               D.cs, ntiles, nitems, rows, skip, X, TL, D.lv, D.inv);
        else if (kmax == 96)
            hipLaunchKernelGGL((k_flushw<96, 2, 2, 4>), dim3(grid), dim3(256), 0, stream, g.T, g, st, D.Pbuf, D.Cbuf,
                               D.cs, ntiles, nitems, rows, skip, X, TL, D.lv, D.inv);
        else if (kmax == 64)
            hipLaunchKernelGGL((k_flushw<64, 2, 2, kW64>), dim3(grid), dim3(64 * kW64), 0, stream, g.T, g, st, D.Pbuf,
                               D.Cbuf, D.cs, ntiles, nitems, rows, skip, X, TL, D.lv, D.inv);
        else
            hipLaunchKernelGGL((k_flushw<32, 2, 3, 4>), dim3(grid), dim3(256), 0, stream, g.T, g, st, D.Pbuf, D.Cbuf,
                               D.cs, ntiles, nitems, rows, skip, X, TL, D.lv, D.inv);
    } else {
        // k_flushm: 32-column wave tiles, 128-row strips (C tile <= 32 KB of LDS),
        // shorter strips for small tableaus; 4 blocks per CU
        const int64_t ntiles = (g.ncols + 127) / 128;
        int strip = 128;
        while (strip > 32 && ntiles * ((g.nloc + strip - 1) / strip) < 4096) strip /= 2;
        while (strip > 32 && kmax * strip * 8 > 32768) strip /= 2;
        const int64_t nitems = ntiles * ((g.nloc + strip - 1) / strip);
        const int64_t nblocks = std::min<int64_t>(nitems, (int64_t)256 * 4);
        if (nblocks < 1) return 0;
#define LPG_FM(K, S)                                                                                                 \
    hipLaunchKernelGGL((k_flushm<K, 1, true, S, 0>), dim3((unsigned)nblocks), dim3(kBlock), 0, stream, g.T, g, st,    \
                       D.Pbuf, D.Cbuf, D.cs, ntiles, nitems, skip)
#define LPG_FM_S(K)                                                              \
    switch (strip) {                                                             \
        case 32: LPG_FM(K, 32); break;                                           \
        case 64: LPG_FM(K, (K * 64 * 8 <= 32768 ? 64 : 32)); break;              \
        default: LPG_FM(K, (K * 128 * 8 <= 32768 ? 128 : 64)); break;            \
    }
        switch (kmax) {
            case 8: LPG_FM_S(8); break;
            case 16: LPG_FM_S(16); break;
            default: LPG_FM_S(32); break;
        }
#undef LPG_FM_S
#undef LPG_FM
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpg
