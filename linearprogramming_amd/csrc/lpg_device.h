// lpg_device.h — device helpers shared by the pivot kernels (lpg_kernels.hip)
// and the persistent block kernel (lpg_block.hip): the argmin reductions over
// ratio candidates and pricing partials, and the pricing rule of one column.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lpg_internal.h"

namespace lpg {

typedef double d2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------
// reductions: 64-lane wave shuffles, then the 4 waves through LDS
// ------------------------------------------------------------------------

// Keeping the better of several structs ("if (better(c, best)) best = c")
// is MISCOMPILED by hipcc (ROCm 7.2, gfx950) when `better` is written with
// early returns: the structurizer turns the nested conditions into exec-mask
// regions, and in the path "best valid -> compare" it parks best's old field
// in the very register that holds the new candidate's field, so a candidate
// that wins keeps some of best's old fields. Seen twice: the pad field of
// k_price's partials (round 1), and k_prep_d's gathered ratio candidates at
// config 4 over 2 ranks (2 x 129 candidates, 2 per thread): row 65436 of one
// candidate paired with the pivot element of another, so P was divided by
// the wrong number (tools/diag_mr4.py; the ISA showed `v_mov_b64 v[4:5],
// v[68:69]` overwriting the loaded piv before the conditional copy). So the
// comparisons below are branch-free (bitwise & |, selects) and every "take"
// is a per-field select on ONE predicate (cand_take / pp_take).
__device__ __forceinline__ bool cand_better(const Cand &a, const Cand &b) {
    const bool ord = (a.theta != b.theta) ? (a.theta < b.theta) : (a.key < b.key);
    return (a.row >= 0) & ((b.row < 0) | ord);
}

template <int RULE>
__device__ __forceinline__ bool pp_better(const PricePart &a, const PricePart &b) {
    bool ord;
    if (RULE == RULE_BLAND) ord = a.j < b.j;
    else ord = (a.cls != b.cls) ? (a.cls < b.cls) : ((a.v != b.v) ? (a.v < b.v) : (a.j < b.j));
    return (a.j >= 0) & ((b.j < 0) | ord);
}

__device__ __forceinline__ void cand_take(Cand &best, const Cand &c, bool t) {
    best.theta = t ? c.theta : best.theta;
    best.piv = t ? c.piv : best.piv;
    best.key = t ? c.key : best.key;
    best.row = t ? c.row : best.row;
}

__device__ __forceinline__ void pp_take(PricePart &best, const PricePart &c, bool t) {
    best.v = t ? c.v : best.v;
    best.j = t ? c.j : best.j;
    best.cls = t ? c.cls : best.cls;
    best.pad = t ? c.pad : best.pad;
}

__device__ __forceinline__ Cand shfl_xor_cand(const Cand &c, int mask) {
    Cand o;
    o.theta = __shfl_xor(c.theta, mask, 64);
    o.piv = __shfl_xor(c.piv, mask, 64);
    o.key = __shfl_xor((long long)c.key, mask, 64);
    o.row = __shfl_xor((long long)c.row, mask, 64);
    return o;
}

__device__ __forceinline__ PricePart shfl_xor_pp(const PricePart &p, int mask) {
    PricePart o;
    o.v = __shfl_xor(p.v, mask, 64);
    o.j = __shfl_xor((long long)p.j, mask, 64);
    o.cls = __shfl_xor(p.cls, mask, 64);
    o.pad = __shfl_xor(p.pad, mask, 64);
    return o;
}

// Block-wide min of a Cand; result valid in every thread.
inline __device__ Cand block_reduce_cand(Cand c) {
    __shared__ Cand sh[kBlock / 64];
#pragma unroll
    for (int mask = 32; mask > 0; mask >>= 1) {
        Cand o = shfl_xor_cand(c, mask);
        cand_take(c, o, cand_better(o, c));
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = c;
    __syncthreads();
    Cand b = sh[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; i++)
        cand_take(b, sh[i], cand_better(sh[i], b));
    return b;
}

template <int RULE>
__device__ PricePart block_reduce_pp(PricePart p) {
    __shared__ PricePart sh[kBlock / 64];
#pragma unroll
    for (int mask = 32; mask > 0; mask >>= 1) {
        PricePart o = shfl_xor_pp(p, mask);
        pp_take(p, o, pp_better<RULE>(o, p));
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = p;
    __syncthreads();
    PricePart b = sh[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; i++)
        pp_take(b, sh[i], pp_better<RULE>(sh[i], b));
    return b;
}

// ---- fast block argmins for the deferred pivot kernels -------------------
// Candidates are ordered by a unique lexicographic key (hi: u64, lo: u32);
// an invalid candidate is (~0, ~0). Ratio candidates: hi = the bits of
// theta >= 0 (non-negative doubles order like their bit patterns), lo = the
// tie key (row or basic column). Pricing partials: hi = cls << 63 | ~bits(v)
// (v < 0, so ~bits orders most-negative first), lo = j; Bland: hi = 0,
// lo = j. The minimum key is the same candidate block_reduce_cand /
// block_reduce_pp pick (a total order, so the reduction tree cannot change
// the winner). Within a wave: the minimum hi by six DPP steps (xor 1, xor 2,
// half-mirror, mirror within each 16-lane row, then row_bcast:15 and
// row_bcast:31 across rows; lane 63 ends with it), lo only where several
// lanes share that hi; the winning lane is found by ballot and its payload
// read with readlane; the four waves meet in LDS through their keys (one
// barrier, plus a leading one for callers that need it). Round 1's form
// (16-lane rows by DPP on the full 96-bit key, then the rows by readlane)
// took 1.16 / 0.90 us per pricing / ratio argmin in k_pivot_block
// (profiles/r02_block_probe_fine*_before.log).

__device__ __forceinline__ bool key_less(uint64_t ah, uint32_t al, uint64_t bh, uint32_t bl) {
    return ah < bh || (ah == bh && al < bl);
}

__device__ __forceinline__ uint32_t rdl32(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int lane) {
    return ((uint64_t)rdl32((uint32_t)(v >> 32), lane) << 32) | rdl32((uint32_t)v, lane);
}

// 64-bit DPP move: lanes outside ROWMASK's rows keep their own value
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v, CTRL, ROWMASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32), (int)(uint32_t)(v >> 32), CTRL,
                                                               ROWMASK, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t min64(uint64_t a, uint64_t b) { return b < a ? b : a; }

// the same move where every lane of every row takes a source lane (quad_perm,
// mirrors): no old value to keep, so no copy in front of the DPP move.
// PRECONDITION (every wave_min_* / wave_min_key below): the whole wave is
// active (EXEC = all 64 lanes). With bound_ctrl and no old value, a lane
// reading a disabled source lane gets 0, and 0 would become the "minimum";
// call these only from wave-uniform control flow (every caller in
// lpg_block.hip / lpg_kernels.hip / lpg_dual.hip does: out-of-range lanes
// take the neutral key ~0 instead of leaving the branch). ADVICE r5.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64f(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
    return ((uint64_t)hi << 32) | lo;
}

// minimum over the wave, in lane 63: four steps within each 16-lane row,
// then row_bcast:15 (rows 1, 3 take lane 15 of the row below) and
// row_bcast:31 (rows 2, 3 take lane 31)
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t m) {
    m = min64(m, dpp64f<0xB1>(m));         // quad_perm [1,0,3,2]: lane ^ 1
    m = min64(m, dpp64f<0x4E>(m));         // quad_perm [2,3,0,1]: lane ^ 2
    m = min64(m, dpp64f<0x141>(m));        // row_half_mirror
    m = min64(m, dpp64f<0x140>(m));        // row_mirror
    m = min64(m, dpp64<0x142, 0xA>(m));    // row_bcast:15
    m = min64(m, dpp64<0x143, 0xC>(m));    // row_bcast:31
    return rdl64(m, 63);
}

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ uint32_t dpp32m(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32f(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t m) {
    m = min(m, dpp32f<0xB1>(m));
    m = min(m, dpp32f<0x4E>(m));
    m = min(m, dpp32f<0x141>(m));
    m = min(m, dpp32f<0x140>(m));
    m = min(m, dpp32m<0x142, 0xA>(m));
    m = min(m, dpp32m<0x143, 0xC>(m));
    return rdl32(m, 63);
}

// minimum key (h, l) of the wave, uniform in every lane: the minimum h, then
// the minimum l among the lanes holding it. Branch-free: a uniform branch
// here made the compiler wait for the loads the callers keep in flight
// across it (k_select_d's 64 multiplier loads: 10 -> 20 us per launch).
__device__ __forceinline__ void wave_min_key(uint64_t &h, uint32_t &l) {
    const uint64_t hm = wave_min_u64(h);
    const uint32_t lm = wave_min_u32(h == hm ? l : ~0u);
    h = hm;
    l = lm;
}

__device__ __forceinline__ int winner_lane(bool mine) {
    const unsigned long long m = __ballot(mine);
    return m ? __ffsll((long long)m) - 1 : -1;
}

// == block_reduce_cand for candidates with theta >= 0 and unique keys
// (NW waves per block; NW == 1: no LDS, no barrier). LEAD: a barrier first,
// for callers that may still be reading the previous call's exchange.
template <int NW = kBlock / 64, bool LEAD = true>
__device__ Cand block_argmin_cand(const Cand &c) {
    const bool valid = c.row >= 0;
    uint64_t h = valid ? (uint64_t)__double_as_longlong(c.theta) : ~0ull;
    uint32_t l = valid ? (uint32_t)c.key : ~0u;
    const uint64_t mh = h;
    const uint32_t ml = l;
    wave_min_key(h, l);
    const int src = winner_lane(valid && mh == h && ml == l);
    Cand o{0.0, 0.0, 0, -1};
    if (src >= 0) {      // wave-uniform
        o.theta = __longlong_as_double((long long)h);
        o.key = (int64_t)l;
        o.piv = __longlong_as_double((long long)rdl64((uint64_t)__double_as_longlong(c.piv), src));
        o.row = (int64_t)rdl64((uint64_t)c.row, src);
    }
    if (NW == 1) return o;
    __shared__ Cand sw[NW];
    __shared__ uint64_t sh[NW];
    __shared__ uint32_t sl[NW];
    const int w = threadIdx.x >> 6;
    if (LEAD) __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        sw[w] = o;
        sh[w] = h;
        sl[w] = l;
    }
    __syncthreads();
    int bi = 0;
    uint64_t bh = sh[0];
    uint32_t bl = sl[0];
#pragma unroll
    for (int i = 1; i < NW; i++)
        if (key_less(sh[i], sl[i], bh, bl)) {
            bh = sh[i];
            bl = sl[i];
            bi = i;
        }
    return sw[bi];
}

// == block_reduce_pp<RULE> for eligible partials (v < 0, unique j)
template <int RULE, int NW = kBlock / 64, bool LEAD = true>
__device__ PricePart block_argmin_pp(const PricePart &p) {
    const bool valid = p.j >= 0;
    uint64_t h = ~0ull;
    if (valid)
        h = RULE == RULE_BLAND ? 0ull
                               : (((uint64_t)(uint32_t)p.cls << 63) |
                                  (~(uint64_t)__double_as_longlong(p.v) & 0x7fffffffffffffffull));
    uint32_t l = valid ? (uint32_t)p.j : ~0u;
    const uint64_t mh = h;
    const uint32_t ml = l;
    wave_min_key(h, l);
    const int src = winner_lane(valid && mh == h && ml == l);
    PricePart o{0.0, -1, 0, 0};
    if (src >= 0) {      // wave-uniform
        o.j = (int64_t)l;
        o.v = __longlong_as_double((long long)rdl64((uint64_t)__double_as_longlong(p.v), src));
        o.cls = (int32_t)rdl32((uint32_t)p.cls, src);
        o.pad = (int32_t)rdl32((uint32_t)p.pad, src);
    }
    if (NW == 1) return o;
    __shared__ PricePart sw[NW];
    __shared__ uint64_t sh[NW];
    __shared__ uint32_t sl[NW];
    const int w = threadIdx.x >> 6;
    if (LEAD) __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        sw[w] = o;
        sh[w] = h;
        sl[w] = l;
    }
    __syncthreads();
    int bi = 0;
    uint64_t bh = sh[0];
    uint32_t bl = sl[0];
#pragma unroll
    for (int i = 1; i < NW; i++)
        if (key_less(sh[i], sl[i], bh, bl)) {
            bh = sh[i];
            bl = sl[i];
            bi = i;
        }
    return sw[bi];
}

// Pricing candidate of column j: dR is the (real)
// objective row entry; with Big-M (g.nobj == 2) dM is the M-part entry and the
// comparison is lexicographic (M part first). NaN entries are never eligible.
// j is the column's logical index (the tie-break key and what the log and
// basis record), p its physical column in T (== j unless the single-rank
// deferred path has reordered columns, see k_swap_plan).
template <int RULE>
__device__ __forceinline__ void price_one(PricePart &best, double dM, double dR, int64_t j, const Geo &g,
                                          int64_t p = -1) {
    if (j < 1 || j > g.nact) return;
    PricePart c;
    c.j = j;
    c.pad = (int32_t)(p < 0 ? j : p);
    if (g.nobj == 1) {
        if (!(dR < -g.eps_opt)) return;
        c.cls = 0;
        c.v = dR;
    } else if (dM < -g.eps_opt) {
        c.cls = 0;
        c.v = dM;
    } else if (dM <= g.eps_opt && dR < -g.eps_opt) {
        c.cls = 1;
        c.v = dR;
    } else {
        return;
    }
    pp_take(best, c, pp_better<RULE>(c, best));
}

// ---- owner-push exchange (Xch, lpg_internal.h) ----
__device__ __forceinline__ void st_sys64(void *p, uint64_t v) {
    __hip_atomic_store((unsigned long long *)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const void *p) {
    return (uint64_t)__hip_atomic_load((unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// xP[par][src][ld]: the pivot row as stored by rank src (the pair uses src 0);
// xF[par][src][nblk]: its chunk flags
__device__ __forceinline__ double *xch_row(const Xch &X, int rank, int par, int src, int64_t ld) {
    return (double *)X.base[rank] + ((int64_t)par * X.world + src) * ld;
}
__device__ __forceinline__ uint32_t *xch_flag(const Xch &X, int rank, int par, int b, int src = 0) {
    return (uint32_t *)(X.base[rank] + X.offF) + ((int64_t)par * X.world + src) * X.nblk + b;
}
__device__ __forceinline__ uint64_t *xch_cand(const Xch &X, int rank, int par, int from, int e) {
    return (uint64_t *)(X.base[rank] + X.offC) + (((int64_t)par * X.world + from) * X.nx + e) * 6;
}

// Producer side of a cross-rank hand-off: the payload went out as
// system-scope (sc0 sc1) stores and every storing wave waited for them
// (s_waitcnt vmcnt(0), then a workgroup barrier); a system-scope RELEASE
// (buffer_wbl2 sc0 sc1, ~1.7 us) then the flag. The wait after the fence is
// inline asm so that the compiler cannot drop it (MI355X_MICROARCH.md,
// "Compiler hazard"). The consumer needs no acquire: it polls the flag and
// reads the payload with system-scope loads only, from uncached memory (the
// guide's "sc1 loads replace the acquire" form); __threadfence_system() is
// acq_rel (write-back AND invalidate, ~3.5 us) and was paid on both sides.
__device__ __forceinline__ void release_system() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace lpg
