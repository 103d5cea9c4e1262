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

__device__ __forceinline__ bool cand_better(const Cand &a, const Cand &b) {
    if (a.row < 0) return false;
    if (b.row < 0) return true;
    if (a.theta != b.theta) return a.theta < b.theta;
    return a.key < b.key;
}

template <int RULE>
__device__ __forceinline__ bool pp_better(const PricePart &a, const PricePart &b) {
    if (a.j < 0) return false;
    if (b.j < 0) return true;
    if (RULE == RULE_BLAND) return a.j < b.j;
    if (a.cls != b.cls) return a.cls < b.cls;
    if (a.v != b.v) return a.v < b.v;
    return a.j < b.j;
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
        if (cand_better(o, c)) c = o;
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = c;
    __syncthreads();
    Cand b = sh[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; i++)
        if (cand_better(sh[i], b)) b = sh[i];
    return b;
}

template <int RULE>
__device__ PricePart block_reduce_pp(PricePart p) {
    __shared__ PricePart sh[kBlock / 64];
#pragma unroll
    for (int mask = 32; mask > 0; mask >>= 1) {
        PricePart o = shfl_xor_pp(p, mask);
        if (pp_better<RULE>(o, p)) p = o;
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = p;
    __syncthreads();
    PricePart b = sh[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; i++)
        if (pp_better<RULE>(sh[i], b)) b = sh[i];
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
// the winner). Within a wave: four DPP steps (xor 1, xor 2, half-mirror,
// mirror) leave each 16-lane row's minimum in every lane of the row, then
// the four rows through readlane; the winning lane is found by ballot and
// its payload read with readlane; the four waves meet in LDS (one barrier
// pair instead of log2(64) LDS permutes per field).

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ bool key_less(uint64_t ah, uint32_t al, uint64_t bh, uint32_t bl) {
    return ah < bh || (ah == bh && al < bl);
}

template <int CTRL>
__device__ __forceinline__ void key_step(uint64_t &h, uint32_t &l) {
    const uint32_t h0 = dpp32<CTRL>((uint32_t)h), h1 = dpp32<CTRL>((uint32_t)(h >> 32)), l1 = dpp32<CTRL>(l);
    const uint64_t oh = ((uint64_t)h1 << 32) | h0;
    if (key_less(oh, l1, h, l)) {
        h = oh;
        l = l1;
    }
}

__device__ __forceinline__ uint32_t rdl32(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, int lane) {
    return ((uint64_t)rdl32((uint32_t)(v >> 32), lane) << 32) | rdl32((uint32_t)v, lane);
}

// minimum key of the wave, uniform in every lane
__device__ __forceinline__ void wave_min_key(uint64_t &h, uint32_t &l) {
    key_step<0xB1>(h, l);    // quad_perm [1,0,3,2]: lane ^ 1
    key_step<0x4E>(h, l);    // quad_perm [2,3,0,1]: lane ^ 2
    key_step<0x141>(h, l);   // row_half_mirror: i <-> 7 - i
    key_step<0x140>(h, l);   // row_mirror: i <-> 15 - i
    uint64_t bh = rdl64(h, 0);
    uint32_t bl = rdl32(l, 0);
#pragma unroll
    for (int r = 1; r < 4; r++) {
        const uint64_t rh = rdl64(h, 16 * r);
        const uint32_t rl = rdl32(l, 16 * r);
        if (key_less(rh, rl, bh, bl)) {
            bh = rh;
            bl = rl;
        }
    }
    h = bh;
    l = bl;
}

__device__ __forceinline__ int winner_lane(bool mine) {
    const unsigned long long m = __ballot(mine);
    return m ? __ffsll((long long)m) - 1 : -1;
}

// == block_reduce_cand for candidates with theta >= 0 and unique keys
// (NW waves per block; NW == 1: no LDS, no barrier)
template <int NW = kBlock / 64>
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
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sw[w] = o;
    __syncthreads();
    Cand b = sw[0];
#pragma unroll
    for (int i = 1; i < NW; i++)
        if (cand_better(sw[i], b)) b = sw[i];
    return b;
}

// == block_reduce_pp<RULE> for eligible partials (v < 0, unique j)
template <int RULE, int NW = kBlock / 64>
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
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sw[w] = o;
    __syncthreads();
    PricePart b = sw[0];
#pragma unroll
    for (int i = 1; i < NW; i++)
        if (pp_better<RULE>(sw[i], b)) b = sw[i];
    return b;
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
    if (pp_better<RULE>(c, best)) best = c;
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
