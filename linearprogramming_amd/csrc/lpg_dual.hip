// lpg_dual.hip — the dual simplex on the deferred (blocked) tableau.
//
// Reference: the router's option 2 (Source/router.c:32-34) prints a label and
// does nothing; LPStandardize(model, 1) (Source/simplex.c:178-179) builds the
// dual-feasible tableau it would start from. The rules are the eager dual's
// (lpg_kernels.hip k_dual_price / k_dual_prep, oracle/lpo.c lpo_solve_dual):
// leaving row r_t = argmin b_i over b_i < -eps_opt (ties: smallest row),
// entering column k_t = argmin d_j / (-a_rj) over a_rj < -eps_piv, d_j <= 0
// counted as 0 (ties: smallest j).
//
// The constraint rows lag behind by the pending pivots exactly as in the
// primal's deferred mode (lpg_internal.h): P_q, C_q, r_q fill the same Pbuf /
// Cbuf / rq slots, so k_swap_plan (no column trade) + k_flushw +
// k_flush_pivot_rows apply a block unchanged. The roles of the two pivot
// kernels swap with the pricing:
//
//   k_dual_row_d  (column blocks, 2 columns per thread)
//       the objective row's update of the previous pivot (deferred by one
//       kernel: d_k is only known once every block has chosen k, so the block
//       that owns column k could not update it in the same launch), then
//       r_t from the previous step's row candidates, row r_t of the current
//       tableau through the pending chain (-> R), and the ratio-test partials
//       over R and d.
//   k_dual_col_d  (column blocks + row blocks)
//       k_t from the partials; P_t = R / R[k_t] into Pbuf[q]; column k_t and
//       column 0 of the current tableau through the chain (one row per
//       thread); C_t into Cbuf[q] and Cs; b_{t+1} = fma(-C_t, P_t[0], b_t),
//       P_t[0] on row r_t, -> the next step's row candidates. Bookkeeping
//       (basis, log, pending slot) by one thread.
//
// Every value is the eager pivot's, operation for operation: the chain is
// what q eager updates compute (lpg_internal.h), and the objective update is
// the eager update's fma(-C_t[obj], P_t[j], d_j), one kernel later. The slot's
// `dpend` word carries "an objective update is owed" from col_d to the next
// row_d (or to the host's final row_d, which also peeks at optimality).
//
// Row partition (MR, round 3): the row candidates row_d reduces are every
// rank's (allgathered by the host); the owner of r_t writes row r_t into R and
// every other rank -0, the host sums R over the ranks (the owner's row bit
// for bit), and the ratio partials come from R and the replicated objective
// row in k_dual_ratio, the same on every rank; col_d then runs on each rank's
// rows with r_t's local index (-1 off the owner). P_t, the objective row, the
// basis and the log are replicated; C_t and the flush are per rank.
#include <hip/hip_runtime.h>

#include "lpg_device.h"
#include "lpg_internal.h"

namespace lpg {

// The eager dual's row candidate (k_dual_rows): theta = b, key = row.
__device__ __forceinline__ void dual_cand(Cand &best, double b, int64_t grow, double eps) {
    Cand c;
    c.theta = b;
    c.piv = 0.0;
    c.key = grow;
    c.row = (b < -eps) ? grow : -1;
    cand_take(best, c, cand_better(c, best));
}

// The ratio-test candidate of column j: theta = d_j / -a_rj (0 where d_j <= 0),
// key = j, row = j (>= 0: eligible).
__device__ __forceinline__ void ratio_cand(Cand &best, double a, double d, int64_t j, const Geo &g) {
    Cand c;
    c.theta = d > 0.0 ? d / -a : 0.0;
    c.piv = a;
    c.key = j;
    c.row = (j >= 1 && j <= g.nact && a < -g.eps_piv) ? j : -1;
    cand_take(best, c, cand_better(c, best));
}

template <int kPF, bool MR>
__global__ __launch_bounds__(256) void k_dual_row_d(double *__restrict__ T, Geo g, DevState *st, int s,
                                                    const Cand *__restrict__ rc, int nrc,
                                                    const double *__restrict__ Pprev, const double *__restrict__ Cprev,
                                                    double *__restrict__ R, Cand *__restrict__ cp, Defer D) {
    constexpr int NT = 256;
    const int64_t j2 = (int64_t)blockIdx.x * NT + threadIdx.x;
    const int64_t nvec = (g.ncols + 1) / 2;
    const bool col = j2 < nvec;
    const int64_t rR = g.nloc + g.nobj - 1;
    const int lane = threadIdx.x & 63;
    // ---- round 1: nothing here depends on the leaving row
    const int32_t status = st->slot[s].status;
    const bool dp = st->slot[s].dpend != 0;
    Cand best{0.0, 0.0, 0, -1};
    for (int q = threadIdx.x; q < nrc; q += NT) {
        const Cand c = rc[q];
        cand_take(best, c, cand_better(c, best));
    }
    const int64_t jc = col ? 2 * j2 : 0;
    d2 d = *(const d2 *)(T + rR * g.ld + jc);
    const d2 pp = *(const d2 *)(Pprev + jc);
    const double cprev = -Cprev[rR];
    constexpr int B0 = kPF < 64 ? kPF : 64;
    constexpr bool TWO = kPF > 64;
    static_assert(kPF <= 64 || kPF == 128, "prefetch slots");
    const int npf = D.q < B0 ? D.q : B0;
    d2 pq[B0];    // slots past the block: the all-zero row (see k_prep_d)
#pragma unroll
    for (int u = 0; u < B0; u++) pq[u] = *(const d2 *)((u < npf ? D.Pbuf + (int64_t)u * g.ld : D.zrow) + jc);
    const int64_t rqv = lane < D.q ? D.rq[lane] : -1;
    const int64_t rqv1 = TWO && 64 + lane < D.q ? D.rq[64 + lane] : -1;
    // MR: every exit that computes no row sends the identity of the sum, -0
    auto r_identity = [&]() {
        if (MR && col) *(d2 *)(R + 2 * j2) = d2{-0.0, -0.0};
    };
    if (status != RUNNING) {
        r_identity();
        return;
    }
    if (dp) {   // pivot t-1's objective update, as k_update applies it
        d.x = fma(cprev, pp.x, d.x);
        d.y = fma(cprev, pp.y, d.y);
        if (col) *(d2 *)(T + rR * g.ld + 2 * j2) = d;
    }
    best = block_reduce_cand(best);
    // Primal feasible: optimal. Only r = -1 is published here, never the
    // status: every block of this launch reads slot[s].status on entry, and a
    // block scheduled after block 0 had written OPTIMAL there would return
    // without the owed update above (the round-3 stale objective column).
    // k_dual_col_d (or the host, after the final row-only launch) turns
    // RUNNING with r < 0 into OPTIMAL.
    if (best.row < 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) st->slot[s].r = -1;
        r_identity();
        return;
    }
    const bool own = !MR || (best.row >= g.row0 && best.row < g.row0 + g.nloc);   // uniform
    const int64_t rl = own ? best.row - g.row0 : -1;
    if (blockIdx.x == 0 && threadIdx.x == 0) st->slot[s].r = best.row;
    if (!own) {                              // another rank's row: its owner sends it
        r_identity();
        return;
    }
    // ---- round 2: row r as stored and its pending multipliers; the chain as
    // in k_prep_d (restart at the last pending pivot on this row, every lane)
    d2 t = col ? *(const d2 *)(T + rl * g.ld + 2 * j2) : d2{0.0, 0.0};
    const double cl = lane < D.q ? -D.Cbuf[(int64_t)lane * D.cs + rl] : -0.0;
    const double cl1 = (TWO && 64 + lane < D.q) ? -D.Cbuf[(int64_t)(64 + lane) * D.cs + rl] : -0.0;
    const unsigned long long hit = __ballot(lane < D.q && rqv == rl);
    const unsigned long long hit1 = TWO ? __ballot(64 + lane < D.q && rqv1 == rl) : 0ull;
    const int qs = hit1 ? 127 - __clzll((long long)hit1) : hit ? 63 - __clzll((long long)hit) : -1;
    const uint64_t clb = (uint64_t)__double_as_longlong(cl);
    const uint64_t clb1 = (uint64_t)__double_as_longlong(cl1);
    const int npf1 = TWO && D.q > 64 ? D.q - 64 : 0;
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
    if (TWO && D.q > 64) {                  // bank 1: slots 64 .. D.q - 1 (uniform)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < 64; u++)
            pq[u] = *(const d2 *)((u < npf1 ? D.Pbuf + (int64_t)(64 + u) * g.ld : D.zrow) + jc);
        const int qs1 = qs - 64;
        if (qs1 < 0) {
#pragma unroll
            for (int u = 0; u < 64; u++) {
                const double c = __longlong_as_double((long long)rdl64(clb1, u));
                t.x = fma(c, pq[u].x, t.x);
                t.y = fma(c, pq[u].y, t.y);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 64; u++) {
                const double c = __longlong_as_double((long long)rdl64(clb1, u));
                const double fx = fma(c, pq[u].x, t.x), fy = fma(c, pq[u].y, t.y);
                t.x = u == qs1 ? pq[u].x : (u > qs1 ? fx : t.x);
                t.y = u == qs1 ? pq[u].y : (u > qs1 ? fy : t.y);
            }
        }
    }
    Cand cb{0.0, 0.0, 0, -1};
    if (col) {
        *(d2 *)(R + 2 * j2) = t;
        ratio_cand(cb, t.x, d.x, 2 * j2, g);
        ratio_cand(cb, t.y, d.y, 2 * j2 + 1, g);
    }
    if (MR) return;                          // the partials follow the exchange of R (k_dual_ratio)
    cb = block_reduce_cand(cb);
    if (threadIdx.x == 0) cp[blockIdx.x] = cb;
}

// MR: the ratio-test partials over the exchanged row R and the objective row
// (row_d has applied the owed update), exactly row_d's single-rank tail.
__global__ __launch_bounds__(256) void k_dual_ratio(const double *__restrict__ T, Geo g, const DevState *st, int s,
                                                    const double *__restrict__ R, Cand *__restrict__ cp) {
    constexpr int NT = 256;
    const int64_t j2 = (int64_t)blockIdx.x * NT + threadIdx.x;
    const bool col = j2 < (g.ncols + 1) / 2;
    if (st->slot[s].status != RUNNING || st->slot[s].r < 0) return;   // col_d stops too
    const int64_t rR = g.nloc + g.nobj - 1;
    Cand cb{0.0, 0.0, 0, -1};
    if (col) {
        const d2 d = *(const d2 *)(T + rR * g.ld + 2 * j2);
        const d2 t = *(const d2 *)(R + 2 * j2);
        ratio_cand(cb, t.x, d.x, 2 * j2, g);
        ratio_cand(cb, t.y, d.y, 2 * j2 + 1, g);
    }
    cb = block_reduce_cand(cb);
    if (threadIdx.x == 0) cp[blockIdx.x] = cb;
}

// Blocks [0, npp): P_t. Blocks [npp, npp + nsel): one row per thread.
template <int kPF>
__global__ __launch_bounds__(256) void k_dual_col_d(const double *__restrict__ T, Geo g, DevState *st, int s, int s1,
                                                    const Cand *__restrict__ cp, int ncp, const double *__restrict__ R,
                                                    double *__restrict__ Cs, Cand *__restrict__ rc, int npp, Defer D) {
    constexpr int NT = 256;
    const int64_t nrows = g.nloc + g.nobj;
    const bool sel = (int)blockIdx.x >= npp;
    const int64_t i = sel ? ((int64_t)blockIdx.x - npp) * NT + threadIdx.x : 0;
    const bool row = sel && i < nrows;
    const bool crow = sel && i < g.nloc;
    const int lane = threadIdx.x & 63;
    // ---- round 1: nothing here depends on the entering column
    const int32_t stt = st->slot[s].status;
    const int64_t r = st->slot[s].r;
    Cand pb{0.0, 0.0, 0, -1};
    for (int q = threadIdx.x; q < ncp; q += NT) {
        const Cand c = cp[q];
        cand_take(pb, c, cand_better(c, pb));
    }
    const double ob = row ? T[i * g.ld] : 0.0;
    constexpr int B0 = kPF < 64 ? kPF : 64;
    constexpr bool TWO = kPF > 64;
    const int npf = D.q < B0 ? D.q : B0;
    const int64_t ic = crow ? i : 0;
    double cv[B0];
#pragma unroll
    for (int u = 0; u < B0; u++) {
        const double v = D.Cbuf[(int64_t)(u < npf ? u : 0) * D.cs + ic];
        cv[u] = (u < npf && crow) ? v : 0.0;
    }
    double cv1[TWO ? 64 : 1];
    const int npf1 = TWO && D.q > 64 ? D.q - 64 : 0;
#pragma unroll
    for (int u = 0; u < (TWO ? 64 : 1); u++) {
        cv1[u] = 0.0;
        if (TWO) {
            const double v = D.Cbuf[(int64_t)(u < npf1 ? 64 + u : 0) * D.cs + ic];
            cv1[u] = (u < npf1 && crow) ? v : 0.0;
        }
    }
    // lane q holds P_q[0] and r_q for the pending pivots q < D.q
    const bool lq = lane < D.q;
    const double p0l = lq ? D.Pbuf[(int64_t)lane * g.ld] : 0.0;
    const uint32_t rql = lq ? (uint32_t)D.rq[lane] : 0xffffffffu;
    const bool lq1 = TWO && 64 + lane < D.q;
    const double p0l1 = lq1 ? D.Pbuf[(int64_t)(64 + lane) * g.ld] : 0.0;
    const uint32_t rql1 = lq1 ? (uint32_t)D.rq[64 + lane] : 0xffffffffu;
    Slot *dst = &st->slot[s1];
    if (stt != RUNNING || r < 0) {           // r < 0 while RUNNING: row_d found the basis optimal
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const int32_t sv = stt != RUNNING ? stt : OPTIMAL;
            st->slot[s].status = sv;         // every block of this launch returns here, whichever it reads
            dst->status = sv;
            dst->k = -1;
            dst->r = -1;
            dst->dpend = 0;
        }
        return;
    }
    pb = block_reduce_cand(pb);
    if (pb.row < 0) {                        // no a_rj < 0: the LP is primal infeasible
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->slot[s].status = INFEASIBLE;
            dst->status = INFEASIBLE;
            dst->k = -1;
            dst->r = -1;
            dst->dpend = 0;
        }
        return;
    }
    const int64_t k = pb.key;
    const int64_t rl = (r >= g.row0 && r < g.row0 + g.nloc) ? r - g.row0 : -1;   // -1: another rank's row
    const double piv = R[k];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->slot[s].k = k;
        dst->status = RUNNING;
        dst->k = -1;
        dst->r = -1;
        dst->dpend = 1;                      // the objective row owes this pivot's update
        D.rq[D.q] = rl;
        st->npend = D.q + 1;
        D.kq[D.q] = k;
        D.lv[D.q] = D.basis[r];
        D.pv[D.q] = piv;
        D.basis[r] = k;
        const int64_t n = st->pivots;
        if (D.logk && n < st->logcap) {
            D.logk[n] = k;
            D.logr[n] = r;
        }
        st->pivots = n + 1;
        st->last_k = k;
        st->last_r = r;
    }
    if (!sel) {                              // P_t = R / piv into the pending slot
        const int64_t j2 = (int64_t)blockIdx.x * NT + threadIdx.x;
        if (j2 < (g.ncols + 1) / 2) {
            const d2 t = *(const d2 *)(R + 2 * j2);
            *(d2 *)(D.Pbuf + (int64_t)D.q * g.ld + 2 * j2) = d2{t.x / piv, t.y / piv};
        }
        return;
    }
    // ---- round 2: column k as stored and P_q[k] (lane q)
    const double oa = row ? T[i * g.ld + k] : 0.0;
    const double pkl = lq ? D.Pbuf[(int64_t)lane * g.ld + k] : 0.0;
    const double pkl1 = lq1 ? D.Pbuf[(int64_t)(64 + lane) * g.ld + k] : 0.0;
    const double p0 = R[0] / piv;            // == P_t[0]
    // columns 0 and k over the pending pivots 0 .. q-1, in every lane (lanes
    // past D.q read as P = +0, r = -1, C = +0: no-op steps)
    const uint64_t p0b = (uint64_t)__double_as_longlong(p0l), pkb = (uint64_t)__double_as_longlong(pkl);
    double b = ob, a = oa;
    const uint32_t ii = (uint32_t)i;
#pragma unroll
    for (int u = 0; u < B0; u++) {
        const double q0 = __longlong_as_double((long long)rdl64(p0b, u));
        const double qk = __longlong_as_double((long long)rdl64(pkb, u));
        const bool hit = ii == rdl32(rql, u);
        const double fb = fma(-cv[u], q0, b), fa = fma(-cv[u], qk, a);
        b = hit ? q0 : fb;
        a = hit ? qk : fa;
    }
    if (TWO && D.q > 64) {
        const uint64_t p0b1 = (uint64_t)__double_as_longlong(p0l1), pkb1 = (uint64_t)__double_as_longlong(pkl1);
#pragma unroll
        for (int u = 0; u < 64; u++) {
            const double q0 = __longlong_as_double((long long)rdl64(p0b1, u));
            const double qk = __longlong_as_double((long long)rdl64(pkb1, u));
            const bool hit = ii == rdl32(rql1, u);
            const double fb = fma(-cv1[u], q0, b), fa = fma(-cv1[u], qk, a);
            b = hit ? q0 : fb;
            a = hit ? qk : fa;
        }
    }
    if (!crow) {              // the objective row is current (row_d applied pivot t-1)
        b = ob;
        a = oa;
    }
    Cand best{0.0, 0.0, 0, -1};
    if (row) {
        Cs[i] = a;
        if (crow) {
            D.Cbuf[(int64_t)D.q * D.cs + i] = a;   // pivot t is pending: its column C_t
            dual_cand(best, i == rl ? p0 : fma(-a, p0, b), g.row0 + i, g.eps_opt);
        }
    }
    best = block_reduce_cand(best);
    if (threadIdx.x == 0) rc[blockIdx.x - npp] = best;
}

static int dual_pf(int q) { return q < 16 ? 16 : q < 32 ? 32 : q < 48 ? 48 : q < 64 ? 64 : 128; }

int launch_dual_row_d(const Launch &L, const Geo &g, DevState *st, int s, const Cand *rc, int nrc, Cand *cp,
                      double *R, const double *Pprev, const double *Cprev, const Defer &D, bool mr) {
    if (g.nobj != 1) return -1;
    const int npp = pivot_d_blocks(g, 0, 256);
    hipStream_t stream = (hipStream_t)L.stream;
#define LPG_DR(PF)                                                                                                   \
    do {                                                                                                             \
        if (mr)                                                                                                      \
            hipLaunchKernelGGL((k_dual_row_d<PF, true>), dim3(npp), dim3(256), 0, stream, g.T, g, st, s, rc, nrc,    \
                               Pprev, Cprev, R, cp, D);                                                              \
        else                                                                                                         \
            hipLaunchKernelGGL((k_dual_row_d<PF, false>), dim3(npp), dim3(256), 0, stream, g.T, g, st, s, rc, nrc,   \
                               Pprev, Cprev, R, cp, D);                                                              \
    } while (0)
    switch (dual_pf(D.q)) {
        case 16: LPG_DR(16); break;
        case 32: LPG_DR(32); break;
        case 48: LPG_DR(48); break;
        case 64: LPG_DR(64); break;
        default: LPG_DR(128); break;
    }
#undef LPG_DR
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dual_ratio(const Launch &L, const Geo &g, const DevState *st, int s, const double *R, Cand *cp) {
    hipLaunchKernelGGL(k_dual_ratio, dim3(pivot_d_blocks(g, 0, 256)), dim3(256), 0, (hipStream_t)L.stream, g.T, g, st,
                       s, R, cp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// nrc_out row blocks (>= the rows + objective rows of this rank; the same on
// every rank of a partition, whose candidates are allgathered)
int launch_dual_col_d(const Launch &L, const Geo &g, DevState *st, int s, const Cand *cp, const double *R, double *Cs,
                      Cand *rc, int nrc_out, const Defer &D) {
    const int npp = pivot_d_blocks(g, 0, 256);
    if (g.nobj != 1 || nrc_out < pivot_d_blocks(g, 1, 256)) return -1;
    hipStream_t stream = (hipStream_t)L.stream;
#define LPG_DC(PF)                                                                                                   \
    hipLaunchKernelGGL((k_dual_col_d<PF>), dim3(npp + nrc_out), dim3(256), 0, stream, g.T, g, st, s, s ^ 1, cp, npp, \
                       R, Cs, rc, npp, D)
    switch (dual_pf(D.q)) {
        case 16: LPG_DC(16); break;
        case 32: LPG_DC(32); break;
        case 48: LPG_DC(48); break;
        case 64: LPG_DC(64); break;
        default: LPG_DC(128); break;
    }
#undef LPG_DC
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpg
