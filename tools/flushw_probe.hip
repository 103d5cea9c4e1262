// flushw_probe.hip — the block pass k_flushw<96,2,1,8> (the product's form at
// config 3) and two timing probes of the SAME code (round 6; lab only, the
// product never links this file; VERDICT r5 next #2: attribute the pass):
//   MODE 0  the product body (checked bitwise against lpg::k_flushw first)
//   MODE 1  no MFMA: the memory path alone (loads, ring, barrier, stores; the
//           A operands still read from LDS)
//   MODE 2  no tableau traffic: the matrix path alone (multiplier ring, LDS,
//           barrier, MFMAs; stores only under a never-true condition)
//   MODE 3  MODE 0 with buffer loads / stores predicated by their bounds (no
//           VMEM op behind an exec branch; checked bitwise too)
// over config 3's shape (16384 rows, 49153 columns, pitch 49216, the 32769
// first columns live, P zero beyond), random data, 96 pending slots, the
// product's XCD item map (flushx_plan). Run the probes under rocprofv3 --pmc
// too (LAB_MODE=m selects one).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/flushw_probe tools/flushw_probe.hip
//   tools/flushw_probe [reps]        (LAB_TS=1: per-item timestamps of MODE 0 / 2 as well)
#include "../linearprogramming_amd/csrc/lpg_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace lpg {

// LAB_TS=1: per-item timestamps of k_flushw_probe (s_memrealtime, 100 MHz):
// block b's record r = {start, end, tile, rows}; record kTsMax = {kernel entry,
// exit, items, 0}
constexpr int kTsMax = 96;
__device__ unsigned long long *g_ts = nullptr;

template <int KMAX, int NB, int LB, int WPB, int MODE>
__global__ __launch_bounds__(64 * WPB, LB) void k_flushw_probe(double *__restrict__ T, Geo g, DevState *__restrict__ st,
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
    unsigned long long *ts = g_ts ? g_ts + (size_t)blockIdx.x * (kTsMax + 1) * 4 : nullptr;
    int nrec = 0;
    if (ts && threadIdx.x == 0) ts[kTsMax * 4] = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __syncthreads();
        if (ts && threadIdx.x == 0 && nrec > 0 && nrec <= kTsMax) ts[(nrec - 1) * 4 + 1] = __builtin_amdgcn_s_memrealtime();
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
        if (ts && threadIdx.x == 0 && nrec < kTsMax) {
            ts[nrec * 4] = __builtin_amdgcn_s_memrealtime();
            ts[nrec * 4 + 2] = (unsigned long long)tile;
            ts[nrec * 4 + 3] = (unsigned long long)(i1 - i0);
        }
        nrec++;
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
        // MODE 3: the tableau and multiplier traffic as buffer loads / stores
        // whose bounds do the predication (rows past i1 and dead lanes out of
        // range: loads return 0, stores are dropped), so no VMEM op sits behind
        // an exec branch and the compiler can count vmcnt exactly (with the
        // branches every band ended on vmcnt(0): the band's stores and the
        // next band's loads drained before the next barrier)
        const int64_t i0u = ((int64_t)__builtin_amdgcn_readfirstlane((int)(i0 >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)i0);
        const int64_t i1u = ((int64_t)__builtin_amdgcn_readfirstlane((int)(i1 >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)i1);
        int voff[4];
#pragma unroll
        for (int r = 0; r < 4; r++) voff[r] = ok ? (int)(((int64_t)(lk + 4 * r) * ld + cl) * 8) : (int)0x80000000u;
        auto trs = [&](int s) {
            const int64_t row0 = i0u + 16 * s;
            int64_t nr = i1u - row0;
            nr = nr < 0 ? 0 : nr > 16 ? 16 : nr;
            return __builtin_amdgcn_make_buffer_rsrc((void *)(T + row0 * ld), 0, (int)(nr * ld * 8), 0x00020000);
        };
        const __amdgpu_buffer_rsrc_t crs =
            __builtin_amdgcn_make_buffer_rsrc((void *)Cbuf, 0, (int)((int64_t)np * cs * 8), 0x00020000);
        // multiplier piece e of band s: slot q = e / 8, band rows 2 (e % 8) .. +1
        // (zeros past np and past i1: A = -0 there, x + -0 == x)
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                const int q = e >> 3, rr = 2 * (e & 7);
                const int64_t row = i0 + 16 * s + rr;
                d2 v = d2{0.0, 0.0};
                if (MODE == 3)   // q >= np out of range (0); rows past i1 feed only rows that are not stored
                    v = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(crs, (int)(((int64_t)q * cs + row) * 8), 0, 0));
                else if (s < nb && q < np && row < i1 && (NPC % NTH == 0 || e < NPC))
                    v = *(const d2 *)(Cbuf + (int64_t)q * cs + row);   // row + 1 < cs
                cr[u] = MODE == 3 ? v : -v;   // MODE 3 negates at the LDS store (a wait there anyway)
            }
        };
        auto cstore = [&](const d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++)
                if (NPC % NTH == 0 || threadIdx.x + u * NTH < NPC)
                    *(d2 *)(&sC[s % NB][2 * (threadIdx.x + u * NTH)]) = MODE == 3 ? -cr[u] : cr[u];
        };
        for (int s = 0; s < NB - 1; s++) {   // prologue: bands 0 .. NB-2 into the ring
            d2 cr[PER];
            cload(cr, s);
            cstore(cr, s);
        }
        d2 cn[PER];
        cload(cn, NB - 1);
        auto tload = [&](d2 (&x)[4], int s) {
            if (MODE == 3) {
                const __amdgpu_buffer_rsrc_t rs = trs(s);
#pragma unroll
                for (int r = 0; r < 4; r++) x[r] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[r], 0, 2));
                return;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                x[r] = (MODE != 2 && ok && row < i1) ? __builtin_nontemporal_load((const d2 *)(T + row * ld + cl))
                                                     : d2{0.0, 0.0};
            }
        };
        d2 t[4];
        tload(t, 0);
        for (int s = 0; s < nb; s++) {
            d2 tn[4];                         // one band ahead (two ahead measured no faster)
            if (MODE == 3 || s + 1 < nb) tload(tn, s + 1);
            __syncthreads();                  // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
            d2 tout[4] = {t[0], t[1], t[2], t[3]};
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
                    if (MODE != 1) {
                        ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, be[gq], ae, 0, 0, 0);
                        ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bo[gq], ao, 0, 0, 0);
                        ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, be[gq + 1], ae, 0, 0, 0);
                        ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bo[gq + 1], ao, 0, 0, 0);
                    } else {
                        ae[0] += a0 * 0.0;               // keep the A reads (and their LDS traffic) live
                        ao[0] += a1 * 0.0;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    a0 = n0;
                    a1 = n1;
                }
                if (MODE != 3) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = i0 + 16 * s + lk + 4 * r;
                        if (ok && row < i1 && (MODE != 2 || ae[r] == 12345.0))
                            __builtin_nontemporal_store(d2{ae[r], ao[r]}, (d2 *)(T + row * ld + cl));
                    }
                } else {
                    tout[0] = d2{ae[0], ao[0]};
                    tout[1] = d2{ae[1], ao[1]};
                    tout[2] = d2{ae[2], ao[2]};
                    tout[3] = d2{ae[3], ao[3]};
                }
            }
            if (MODE == 3) {   // unconditional: a dead wave's lanes are all out of range
                const __amdgpu_buffer_rsrc_t rs = trs(s);
#pragma unroll
                for (int r = 0; r < 4; r++)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, tout[r]), rs, voff[r], 0, 2);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
    if (ts && threadIdx.x == 0) {
        if (nrec > 0 && nrec <= kTsMax) ts[(nrec - 1) * 4 + 1] = __builtin_amdgcn_s_memrealtime();
        ts[kTsMax * 4 + 1] = __builtin_amdgcn_s_memrealtime();
        ts[kTsMax * 4 + 2] = (unsigned long long)nrec;
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}


template <int KMAX, int NB, int LB, int WPB, int MODE, int SB>
__global__ __launch_bounds__(64 * WPB, LB) void k_flushw2_probe(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                         const double *__restrict__ Pbuf,
                                                         const double *__restrict__ Cbuf, int64_t cs, int64_t ntiles,
                                                         int64_t nitems, int64_t rows, int skip, FlushX X,
                                                         const int32_t *__restrict__ tlive,
                                                         const int64_t *__restrict__ lv,
                                                         const int32_t *__restrict__ inv) {
    constexpr int NTH = 64 * WPB;
    constexpr int G = KMAX / 4;
    constexpr int BAND = KMAX * 16 * SB;            // doubles per band (SB 16-row sub-bands)
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
        const int nb = (int)((i1 - i0 + 15) / 16);   // 16-row sub-bands
        const int nbb = (nb + SB - 1) / SB;           // bands of SB sub-bands, one barrier each
        // multiplier piece e of band s: slot q = e / 8, band rows 2 (e % 8) .. +1
        // (zeros past np and past i1: A = -0 there, x + -0 == x)
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                const int q = e / (8 * SB), rr = 2 * (e % (8 * SB));
                const int64_t row = i0 + 16 * SB * s + rr;
                d2 v = d2{0.0, 0.0};
                if (s < nbb && q < np && row < i1 && (NPC % NTH == 0 || e < NPC))
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
                x[r] = (MODE != 2 && ok && row < i1) ? __builtin_nontemporal_load((const d2 *)(T + row * ld + cl))
                                                     : d2{0.0, 0.0};
            }
        };
        d2 t[4];
        tload(t, 0);
        for (int s = 0; s < nbb; s++) {
            const int s0 = SB * s;
            d2 tn[4];                         // one sub-band ahead
            if (s0 + 1 < nb) tload(tn, s0 + 1);
            __syncthreads();                  // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
#pragma unroll
            for (int h = 0; h < SB; h++) {
                const int sub = s0 + h;
                if (sub >= nb) break;         // uniform
                if (h > 0) {
#pragma unroll
                    for (int r = 0; r < 4; r++) t[r] = tn[r];
                    if (sub + 1 < nb) tload(tn, sub + 1);
                }
                if (wlive) {
                    d4 ae = d4{t[0].x, t[1].x, t[2].x, t[3].x};
                    d4 ao = d4{t[0].y, t[1].y, t[2].y, t[3].y};
                    const double *sa = &sC[s % NB][lk * 16 * SB + 16 * h + lc];
                    double a0 = sa[0], a1 = sa[64 * SB];
#pragma unroll
                    for (int gq = 0; gq < G; gq += 2) {
                        double n0 = 0.0, n1 = 0.0;
                        if (gq + 2 < G) {
                            n0 = sa[(gq + 2) * 64 * SB];
                            n1 = sa[(gq + 3) * 64 * SB];
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        if (MODE != 1) {
                            ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, be[gq], ae, 0, 0, 0);
                            ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bo[gq], ao, 0, 0, 0);
                            ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, be[gq + 1], ae, 0, 0, 0);
                            ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bo[gq + 1], ao, 0, 0, 0);
                        } else {
                            ae[0] += a0 * 0.0;
                            ao[0] += a1 * 0.0;
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        a0 = n0;
                        a1 = n1;
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = i0 + 16 * sub + lk + 4 * r;
                        if (ok && row < i1 && (MODE != 2 || ae[r] == 12345.0))
                            __builtin_nontemporal_store(d2{ae[r], ao[r]}, (d2 *)(T + row * ld + cl));
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}



__global__ void k_fillr(double *p, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (seed + (uint64_t)i) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
}
__global__ void k_zero_cols_from(double *P, int64_t ld, int64_t c0, int K) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)K * ld; i += (int64_t)gridDim.x * blockDim.x)
        if (i % ld >= c0) P[i] = 0.0;
}
__global__ void k_diff(const double *a, const double *b, int64_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += __double_as_longlong(a[i]) != __double_as_longlong(b[i]);
    if (c) atomicAdd(bad, c);
}

}  // namespace lpg

using namespace lpg;

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int64_t m = 16384, nstruct = 32768, ncols = nstruct + m + 1, ld = (ncols + 63) / 64 * 64, cs = m;
    const int K = 96;
    const int64_t n = m * ld;
    double *T, *T0, *Tr, *Pbuf, *Cbuf;
    DevState *st;
    unsigned long long *bad;
    CHK(hipMalloc(&T, n * 8));
    CHK(hipMalloc(&T0, n * 8));
    CHK(hipMalloc(&Tr, n * 8));
    CHK(hipMalloc(&Pbuf, (size_t)K * ld * 8));
    CHK(hipMalloc(&Cbuf, (size_t)K * cs * 8));
    CHK(hipMalloc(&st, sizeof(DevState)));
    CHK(hipMalloc(&bad, 8));
    hipLaunchKernelGGL(k_fillr, dim3(8192), dim3(256), 0, 0, T0, n, 1ull);
    hipLaunchKernelGGL(k_fillr, dim3(1024), dim3(256), 0, 0, Pbuf, (int64_t)K * ld, 2ull);
    hipLaunchKernelGGL(k_fillr, dim3(1024), dim3(256), 0, 0, Cbuf, (int64_t)K * cs, 3ull);
    hipLaunchKernelGGL(k_zero_cols_from, dim3(1024), dim3(256), 0, 0, Pbuf, ld, nstruct + 1, K);
    CHK(hipDeviceSynchronize());
    Geo g{};
    g.T = T;
    g.ld = ld;
    g.nloc = m;
    g.nobj = 1;
    g.ncols = ncols;
    g.nact = ncols - 1;
    g.m = m;
    const int64_t ntiles = (ncols + 255) / 256;
    const int64_t rows = 2048, nitems = flush_nitems(ntiles, rows, m);
    const FlushX X = flushx_plan(ntiles, m, K, 256, -1);
    const unsigned grid = 256;
    auto reset = [&]() {
        DevState h{};
        h.npend = K;
        CHK(hipMemcpy(st, &h, sizeof h, hipMemcpyHostToDevice));
    };
    auto launch = [&](int which) {
        reset();
        if (which == 0)
            hipLaunchKernelGGL((k_flushw<96, 2, 1, 8>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, cs, ntiles,
                               nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        else if (which == 1)
            hipLaunchKernelGGL((k_flushw_probe<96, 2, 1, 8, 0>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, cs,
                               ntiles, nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        else if (which == 2)
            hipLaunchKernelGGL((k_flushw_probe<96, 2, 1, 8, 1>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, cs,
                               ntiles, nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        else if (which == 3)
            hipLaunchKernelGGL((k_flushw_probe<96, 2, 1, 8, 2>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, cs,
                               ntiles, nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
#define LPG_FW2(W, M, S)                                                                                              \
        else if (which == W)                                                                                          \
            hipLaunchKernelGGL((k_flushw2_probe<96, 2, 1, 8, M, S>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, \
                               cs, ntiles, nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,    \
                               (const int32_t *)nullptr);
        else if (which == 9)
            hipLaunchKernelGGL((k_flushw_probe<96, 2, 1, 8, 3>), dim3(grid), dim3(512), 0, 0, T, g, st, Pbuf, Cbuf, cs,
                               ntiles, nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        LPG_FW2(4, 0, 2)
        LPG_FW2(5, 1, 2)
        LPG_FW2(6, 2, 2)
        LPG_FW2(7, 0, 4)
        LPG_FW2(8, 2, 4)
    };
    // bitwise: the probe's MODE 0 against the product kernel
    CHK(hipMemcpy(T, T0, n * 8, hipMemcpyDeviceToDevice));
    launch(0);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(Tr, T, n * 8, hipMemcpyDeviceToDevice));
    CHK(hipMemcpy(T, T0, n * 8, hipMemcpyDeviceToDevice));
    launch(1);
    CHK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, T, Tr, n, bad);
    unsigned long long hb = 0;
    CHK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    const double bytes = 16.0 * m * (nstruct + 2), flops = bytes / 16.0 * 2.0 * K;
    printf("# flushw probe: %lld x %lld (ld %lld), K = %d, live columns 0..%lld, XCD map H = %d rb %d rs %d; "
           "probe MODE 0 vs lpg::k_flushw: %llu doubles differ\n", (long long)m, (long long)ncols, (long long)ld, K,
           (long long)nstruct, X.H, X.rb, X.rs, hb);
    if (hb) return 1;
    for (int w : {4, 7, 9}) {
        CHK(hipMemcpy(T, T0, n * 8, hipMemcpyDeviceToDevice));
        launch(w);
        CHK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, T, Tr, n, bad);
        CHK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        if (w == 9) printf("# MODE 3 (buffer ops) vs lpg::k_flushw: %llu doubles differ\n", hb);
        else printf("# %d-row bands vs lpg::k_flushw: %llu doubles differ\n", w == 4 ? 32 : 64, hb);
        if (hb) return 1;
    }
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const char *names[] = {"lpg::k_flushw<96,2,1,8> (product)", "probe MODE 0 (same body)",
                           "probe MODE 1 (no MFMA: memory path)", "probe MODE 2 (no T traffic: matrix path)",
                           "32-row bands MODE 0", "32-row bands MODE 1 (memory path)",
                           "32-row bands MODE 2 (matrix path)", "64-row bands MODE 0", "64-row bands MODE 2 (matrix path)",
                           "probe MODE 3 (buffer ops, no VMEM branches)"};
    const int only = getenv("LAB_MODE") ? atoi(getenv("LAB_MODE")) : -1;
    for (int round = 0; round < 2; round++)
        for (int w = 0; w < 10; w++) {
            if (only >= 0 && w != only) continue;
            if (only == -2 && w != 0 && w != 1 && w != 9) continue;
            std::vector<float> t;
            for (int r = 0; r <= reps; r++) {
                CHK(hipMemcpy(T, T0, n * 8, hipMemcpyDeviceToDevice));
                CHK(hipEventRecord(e0));
                launch(w);
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (r) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            printf("%-42s best %.3f ms  median %.3f ms  %6.0f GB/s  %5.1f TFLOP/s\n", names[w], t[0], t[t.size() / 2],
                   bytes / (t[0] * 1e-3) / 1e9, flops / (t[0] * 1e-3) / 1e12);
            fflush(stdout);
        }
    if (getenv("LAB_TS")) {
        // per-item timestamps of probe MODE 0 and MODE 2 (the last item's end
        // includes its final barrier; the dequeue of a queue past its end is
        // the "item" with rows = 0 that ends the block)
        unsigned long long *dts;
        const size_t nts = (size_t)grid * (kTsMax + 1) * 4;
        CHK(hipMalloc(&dts, nts * 8));
        CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_ts), &dts, sizeof dts));
        std::vector<unsigned long long> h(nts);
        for (int w : {1, 3, 9}) {
            for (int rep = 0; rep < 3; rep++) {
                CHK(hipMemset(dts, 0, nts * 8));
                CHK(hipMemcpy(T, T0, n * 8, hipMemcpyDeviceToDevice));
                launch(w);
                CHK(hipDeviceSynchronize());
                CHK(hipMemcpy(h.data(), dts, nts * 8, hipMemcpyDeviceToHost));
                unsigned long long k0 = ~0ull, k1 = 0;
                for (unsigned b = 0; b < grid; b++) {
                    const unsigned long long *r = &h[(size_t)b * (kTsMax + 1) * 4];
                    k0 = std::min(k0, r[kTsMax * 4]);
                    k1 = std::max(k1, r[kTsMax * 4 + 1]);
                }
                const double span = (k1 - k0) * 0.01;   // us
                double live = 0, dead = 0, head = 0, tail = 0, gaps = 0;
                std::vector<double> exits;
                int nlive = 0, ndead = 0, nshort = 0;
                double tshort = 0;
                for (unsigned b = 0; b < grid; b++) {
                    const unsigned long long *r = &h[(size_t)b * (kTsMax + 1) * 4];
                    const int nr = (int)std::min<unsigned long long>(r[kTsMax * 4 + 2], kTsMax);
                    head += (r[0] - r[kTsMax * 4]) * 0.01;
                    exits.push_back((k1 - r[kTsMax * 4 + 1]) * 0.01);
                    for (int i = 0; i < nr; i++) {
                        const double d = (r[i * 4 + 1] - r[i * 4]) * 0.01;
                        if (i > 0) gaps += (r[i * 4] - r[(i - 1) * 4 + 1]) * 0.01;
                        const bool isdead = r[i * 4 + 2] > (unsigned long long)(nstruct / 256);
                        if (r[i * 4 + 3] == 0) continue;
                        if (isdead) { dead += d; ndead++; }
                        else { live += d; nlive++; if (r[i * 4 + 3] < 2048) { nshort++; tshort += d; } }
                    }
                    tail += (k1 - r[kTsMax * 4 + 1]) * 0.01;
                }
                std::sort(exits.begin(), exits.end());
                const double tot = span * grid;
                printf("# ts %-40s span %.1f us: live items %d (%.1f%% of block-time, %d short ones %.1f us avg), "
                       "dead tiles %d (%.2f%%), head %.2f%%, gaps %.2f%%, idle after exit %.2f%% "
                       "(exit-to-end: min %.1f median %.1f max %.1f us)\n",
                       names[w], span, nlive, 100 * live / tot, nshort, nshort ? tshort / nshort : 0.0, ndead,
                       100 * dead / tot, 100 * head / tot, 100 * gaps / tot, 100 * tail / tot, exits[0],
                       exits[exits.size() / 2], exits.back());
                fflush(stdout);
            }
        }
    }
    return 0;
}
