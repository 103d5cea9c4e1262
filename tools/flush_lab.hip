// flush_lab.hip — standalone bench of deferred-flush kernel designs at the
// config-3 shape (16384 constraint rows x 49153 columns, ld 49216, fp64), on
// random T / Pbuf / Cbuf with the slack block's P entries zero (skipped, as in
// the first blocks of a solve). Blocks of 128 pending pivots: the reference is
// the engine's k_flushw<64> run twice (slots 0-63, then 64-127), which is the
// same per-element fma chain; every design is checked bitwise against it
// before it is timed. Tools only: the product never links this file.
//
// Round-2 result (profiles/r02_flush_lab_k128.log): no 128-slot design beats
// two 64-slot passes by enough to pay for 128-slot pivot chains. 2 x
// k_flushw<64> 3.31-3.36 ms; k_flushw<128> (1 wave/SIMD, 256 VGPR + AGPRs)
// 3.00 ms; k_flushx (A through LDS-DMA, 4 chains) 3.54 ms; k_flushy (roles
// swapped, P tile in LDS, no block barrier) 3.39 ms. k_flushy's parts: memory
// alone (no MFMA) 1.83 ms = 4.7 TB/s, matrix cores alone (no tableau traffic)
// 2.93 ms = 47 TFLOP/s of the 75 the f64 MFMA pipe reaches: at 128 slots the
// operands no longer fit beside a prefetch set, the compiler serialises each
// LDS read of B behind the MFMAs that consume the previous one, and 1 wave
// per SIMD cannot hide it. Two 16-row bands per step in k_flushw<128> (4
// independent MFMA chains per wave instead of 2) is no faster either: 3.07 ms
// (profiles/r02_flush_lab_k128_sb2.log), so the 1-wave issue stream, not the
// chain latency, is the limit. Reading the band's A operands 4-32 MFMA groups
// ahead: 3.00-3.02 ms; 3- or 4-deep multiplier rings: 3.02-3.08 ms
// (profiles/r02_flush_lab_k128_apre.log, _ring.log): the loop sits at ~46
// TFLOP/s whatever feeds it.
//
// Round 3 (profiles/r03_flush_lab_k128_v.log, _s.log, r03_mfma_rate2.log):
// an MFMA chain with A from LDS and B from a register array reaches 67-74
// TFLOP/s at 1-4 waves per SIMD, and 69 TFLOP/s while other waves of the same
// CUs stream 3.5 TB/s of HBM read-modify-write -- the pipe and the memory
// system do overlap. The passes still sit at 46-47: k_flushv (16-column wave
// tiles, one chain per wave, 8 or 16 waves per block, 2 or 4 per SIMD)
// 2.92-2.98 ms; k_flushs (loader waves moving tableau bands and multipliers
// into a 4-deep LDS ring by LDS-DMA, matrix waves only computing, one bare
// barrier per band) 3.25-3.79 ms, its data path alone 2.04 ms and its matrix
// path alone 2.69 ms (51 TFLOP/s: the per-band barrier of 12 waves). At
// config 4 on one GPU k_flushv<128,2,16> loses to k_flushw<128> (48.6 vs
// 47.5 ms per 128-pivot pass, profiles/r03_bench_config4_flushw_vs_flushv.log),
// so neither is in the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/flush_lab tools/flush_lab.hip
//   tools/flush_lab [rows]            (LAB_ONLY=substring picks designs)
#include "../linearprogramming_amd/csrc/lpg_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace lpg {

// k_flushv: k_flushw with 16-column wave tiles, ONE MFMA chain per wave and B
// (32 doubles per lane at 128 slots) in VGPRs, so that a wave needs about
// half the registers and WPB = 16 waves per block put 4 waves on each SIMD:
// at 128 slots k_flushw runs 1 wave per SIMD (256 VGPRs + AGPRs), and that
// single issue stream, not the operands, held its matrix cores at ~46 of the
// ~75 TFLOP/s the f64 MFMA pipe reaches (tools/flush_lab.hip). Lane (lk, lc)
// holds column lc of its wave's 16 and rows lk + 4r of the band; the chain,
// the multiplier ring and the dynamic item queue are k_flushw's, so the
// results are the same per-element fma chain (the skipping is per column
// here, per column pair there: they differ at most in the sign of a zero).
template <int KMAX, int NB, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_flushv(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                     const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                     int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows,
                                                     int skip) {
    constexpr int NTH = 64 * WPB;
    constexpr int G = KMAX / 4;
    constexpr int BAND = KMAX * 16;                 // doubles per band
    constexpr int NPC = BAND / 2;                   // 16-byte multiplier pieces per band
    constexpr int PER = (NPC + NTH - 1) / NTH;      // ... per thread
    __shared__ __attribute__((aligned(16))) double sC[NB][BAND];
    __shared__ int64_t next_item;
    __shared__ int wsum[WPB];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t cl = tile * (16 * WPB) + wave * 16 + lc;      // this lane's column
        const bool in = cl < g.ncols;
        double b[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            const double v = (in && q < np) ? Pbuf[(int64_t)q * ld + cl] : 0.0;
            b[gq] = v;
            live = live || v != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;     // OR over the 4 lanes of the column
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? 1 : 0;
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
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                const int q = e >> 3, rr = 2 * (e & 7);
                const int64_t row = i0 + 16 * s + rr;
                d2 v = d2{0.0, 0.0};
                if (e < NPC && s < nb && q < np && row < i1) v = *(const d2 *)(Cbuf + (int64_t)q * cs + row);
                cr[u] = -v;
            }
        };
        auto cstore = [&](const d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                if (e < NPC) *(d2 *)(&sC[s % NB][2 * e]) = cr[u];
            }
        };
        for (int s = 0; s < NB - 1; s++) {
            d2 cr[PER];
            cload(cr, s);
            cstore(cr, s);
        }
        d2 cn[PER];
        cload(cn, NB - 1);
        auto tload = [&](double (&x)[4], int s) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                x[r] = (ok && row < i1) ? __builtin_nontemporal_load(T + row * ld + cl) : 0.0;
            }
        };
        double t[4];
        tload(t, 0);
        for (int s = 0; s < nb; s++) {
            double tn[4];
            if (s + 1 < nb) tload(tn, s + 1);
            __syncthreads();                  // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
            if (wlive) {
                d4 acc = d4{t[0], t[1], t[2], t[3]};
                const double *sa = &sC[s % NB][lk * 16 + lc];
#pragma unroll
                for (int gq = 0; gq < G; gq++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], b[gq], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * s + lk + 4 * r;
                    if (ok && row < i1) __builtin_nontemporal_store(acc[r], T + row * ld + cl);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}


// k_flushs: the block pass with specialised waves. At 128 slots the pass is
// balanced (16 flop per tableau byte against the box's ~14.5 = 74 TFLOP/s /
// 5.1 TB/s), and k_flushw / k_flushv, whose waves each load, compute and
// store in turn, overlap the two streams badly (46-47 TFLOP/s, 2.9-3.0 ms at
// the config-3 shape, while an MFMA loop reaches ~69 TFLOP/s with an HBM
// stream of 3.5 TB/s running beside it on the same CUs: tools/mfma_rate2.hip).
// Here LW loader waves only move data: tableau bands (16 rows x 16*MW
// columns) and the band's multipliers go from HBM / the Infinity Cache into
// an LDS ring by LDS-DMA (global_load_lds, 16 B per lane, no registers), DT
// bands ahead; MW matrix waves only compute: each takes 16 columns (k_flushv's
// lane map), its accumulators from the ring, the chain on the matrix cores
// with B = -P in VGPRs, and stores the results. One barrier per band hands
// the ring on. Multipliers are raw C with B negated: fma(c, -p, x) ==
// fma(-c, p, x) bit for bit, and padding slots are A = +0 (the zero row) with
// B = -0, x + (+0)(-0) == x for every x: the same chain as every other pass.
template <int KMAX, int MW, int LW, int DT>
__global__ __launch_bounds__(64 * (MW + LW)) void k_flushs(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                           const double *__restrict__ Pbuf,
                                                           const double *__restrict__ Cbuf, int64_t cs, int64_t ntiles,
                                                           int64_t nitems, int64_t rows, int skip,
                                                           const double *__restrict__ zrow) {
    constexpr int G = KMAX / 4;
    constexpr int TW = 16 * MW;                     // tile width (columns)
    constexpr int RING = DT + 1;
    constexpr int TB = 16 * TW;                     // doubles of tableau per band
    constexpr int CB = 16 * KMAX;                   // doubles of multipliers per band
    constexpr int SLOT = TB + CB;
    constexpr int NT_DMA = TB / 128;                // 1 KB DMA instructions per band: tableau ...
    constexpr int NC_DMA = CB / 128;                // ... and multipliers
    static_assert(TW == 128 && NT_DMA % LW == 0 && NC_DMA % LW == 0, "one 1 KB row per tableau DMA");
    constexpr int TPW = NT_DMA / LW, CPW = NC_DMA / LW;   // per loader wave
    extern __shared__ __attribute__((aligned(16))) double ring[];
    __shared__ int64_t next_item;
    __shared__ int wsum[MW];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool mw = wave < MW;                      // matrix wave (else loader wave wave - MW)
    const int lw = wave - MW;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t c0 = tile * TW;
        const int64_t cl = c0 + (mw ? wave * 16 : 0) + lc;          // a matrix lane's column
        const bool in = mw && cl < g.ncols;
        double b[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            const double v = (in && q < np) ? Pbuf[(int64_t)q * ld + cl] : 0.0;
            b[gq] = -v;
            live = live || v != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? 1 : 0;
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        const bool wlive = mine > 0;                                   // wave-uniform
        if (mw && lane == 0) wsum[wave] = mine;
        if (__syncthreads_count(wlive && lane == 0) == 0) continue;    // the whole tile is skipped
        if (threadIdx.x == 0) {
            int sum = 0;
#pragma unroll
            for (int w = 0; w < MW; w++) sum += wsum[w];
            touched += (unsigned long long)sum * (unsigned long long)(i1 - i0);
        }
        const int nb = (int)((i1 - i0 + 15) / 16);
        // loader wave: band s into ring slot s % RING (rows past i1 and slots
        // past np read the zero row; the tableau's last tile reads into the
        // next row's padding, which the stores never write back)
        auto issue = [&](int s) {
            double *slot = ring + (size_t)(s % RING) * SLOT;
#pragma unroll
            for (int u = 0; u < TPW; u++) {
                const int rr = lw * TPW + u;
                const int64_t row = i0 + 16 * s + rr;
                const double *src = row < i1 ? T + row * ld + c0 + 2 * lane : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(slot + rr * TW), 16, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < CPW; u++) {
                const int e = lw * CPW + u;                 // 8 slots x 16 rows per instruction
                const int q = 8 * e + (lane >> 3);
                const int64_t row = i0 + 16 * s + 2 * (lane & 7);
                const double *src = (q < np && row < i1) ? Cbuf + (int64_t)q * cs + row : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(slot + TB + e * 128), 16, 0, 0);
            }
        };
        if (!mw)
            for (int s = 0; s < DT && s < nb; s++) issue(s);
        for (int s = 0; s < nb; s++) {
            if (!mw) {   // band s has landed (bands s+1 .. s+DT-1 may still be in flight)
                if (s + DT - 1 < nb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DT - 1) * (TPW + CPW)) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // band s is in the ring; slot (s - 1) % RING is free. A bare
            // s_barrier: __syncthreads() would also wait for every wave's
            // outstanding memory operations (vmcnt(0)), i.e. drain the DMA
            // ring and the matrix waves' stores each band
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (!mw) {
                if (s + DT < nb) issue(s + DT);
            } else if (wlive) {
                const double *slot = ring + (size_t)(s % RING) * SLOT;
                d4 acc;
#pragma unroll
                for (int r = 0; r < 4; r++) acc[r] = slot[(lk + 4 * r) * TW + wave * 16 + lc];
                const double *sa = slot + TB + lk * 16 + lc;
#pragma unroll
                for (int gq = 0; gq < G; gq++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], b[gq], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * s + lk + 4 * r;
                    if (ok && row < i1) __builtin_nontemporal_store(acc[r], T + row * ld + cl);
                }
            }
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

template <int KMAX>
constexpr size_t flushs_lds() { return (size_t)4 * (16 * 128 + 16 * KMAX) * sizeof(double); }   // DT = 3


// k_flushx: 128-slot blocks. Wave tile 32 columns (16-byte accesses, even /
// odd-column MFMA chains as k_flushw) x SB bands of 16 rows per step, so a
// wave runs 2*SB independent MFMA chains; B = -P in VGPRs for the item; the
// multipliers (raw C, A fragments) come into a 2-deep LDS ring straight from
// global memory (global_load_lds, 16 B per lane, lane-linear [band][q][16
// rows] image), slots past np read from a zero row. fma(c, -p, x) ==
// fma(-c, p, x) bit for bit, and for q >= np A = +0, B = -0: x + (+0)(-0) ==
// x for every x, signed zeros included.
template <int KMAX, int SB, int LB>
__global__ __launch_bounds__(256, LB) void k_flushx(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                    const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                    int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows, int skip,
                                                    const double *__restrict__ zbuf) {
    constexpr int G = KMAX / 4;
    constexpr int STEP = 16 * SB;                 // rows per step
    constexpr int SD = KMAX * STEP;               // doubles of A per step
    constexpr int GL = SD / 2 / 256;              // 16-byte LDS-DMA pieces per thread per step
    static_assert(GL >= 1 && (SD / 2) % 256 == 0, "staging");
    __shared__ __attribute__((aligned(16))) double sA[2][SD];
    __shared__ int64_t next_item;
    __shared__ int wsum[4];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t cl = tile * 128 + wave * 32 + 2 * lc;
        const bool in = cl < g.ncols;
        double be[G], bo[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            d2 v = d2{0.0, 0.0};
            if (in && q < np) v = *(const d2 *)(Pbuf + (int64_t)q * ld + cl);
            live = live || v.x != 0.0 || v.y != 0.0;
            be[gq] = -v.x;
            bo[gq] = -v.y;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? (cl + 1 < g.ncols ? 2 : 1) : 0;
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        const bool wlive = mine > 0;
        if (lane == 0) wsum[wave] = mine;
        if (__syncthreads_count(wlive && lane == 0) == 0) continue;
        if (threadIdx.x == 0) touched += (unsigned long long)(wsum[0] + wsum[1] + wsum[2] + wsum[3]) * (i1 - i0);
        const int nst = (int)((i1 - i0 + STEP - 1) / STEP);
        // A image of step s: element e (16 B) = doubles 2e, 2e+1 of [b][q][16]
        auto aload = [&](int s, int slot) {
#pragma unroll
            for (int u = 0; u < GL; u++) {
                const int e = u * 256 + threadIdx.x;
                const int d = 2 * e;
                const int b = d / (KMAX * 16), q = (d / 16) % KMAX, rr = d % 16;
                const int64_t row = i0 + (int64_t)s * STEP + 16 * b + rr;
                const double *src = (q < np && s < nst) ? Cbuf + (int64_t)q * cs + row : zbuf;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)&sA[slot][2 * (u * 256 + wave * 64)], 16, 0, 0);
            }
        };
        auto tload = [&](d2 (&x)[SB][4], int s) {
#pragma unroll
            for (int b = 0; b < SB; b++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + (int64_t)s * STEP + 16 * b + lk + 4 * r;
                    x[b][r] = (ok && row < i1) ? __builtin_nontemporal_load((const d2 *)(T + row * ld + cl))
                                               : d2{0.0, 0.0};
                }
        };
        d2 t[SB][4];
        aload(0, 0);
        tload(t, 0);
        for (int s = 0; s < nst; s++) {
            // A of step s (and the tableau of step s) have landed; the stores of step s - 1 may be in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * SB) : "memory");
            __builtin_amdgcn_s_barrier();
            d2 tn[SB][4];
            if (s + 1 < nst) {
                aload(s + 1, (s + 1) & 1);
                tload(tn, s + 1);
            }
            if (wlive) {
                d4 ae[SB], ao[SB];
#pragma unroll
                for (int b = 0; b < SB; b++) {
                    ae[b] = d4{t[b][0].x, t[b][1].x, t[b][2].x, t[b][3].x};
                    ao[b] = d4{t[b][0].y, t[b][1].y, t[b][2].y, t[b][3].y};
                }
                const double *sa = &sA[s & 1][lk * 16 + lc];
#pragma unroll
                for (int gq = 0; gq < G; gq++) {
#pragma unroll
                    for (int b = 0; b < SB; b++) {
                        const double a = sa[b * KMAX * 16 + gq * 64];
                        ae[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, be[gq], ae[b], 0, 0, 0);
                        ao[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bo[gq], ao[b], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int b = 0; b < SB; b++)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = i0 + (int64_t)s * STEP + 16 * b + lk + 4 * r;
                        if (ok && row < i1)
                            __builtin_nontemporal_store(d2{ae[b][r], ao[b][r]}, (d2 *)(T + row * ld + cl));
                    }
            }
#pragma unroll
            for (int b = 0; b < SB; b++)
#pragma unroll
                for (int r = 0; r < 4; r++) t[b][r] = tn[b][r];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}


// k_flushy: roles swapped against k_flushw. A block stages the negated P of
// a 64-column tile (all KMAX slots, padded rows) in LDS once per item; each
// wave then sweeps its own 16-row bands (wave w: bands w, w+4, ...) with no
// block barrier: A fragments (raw C of the band's 16 rows, 32 doubles per
// lane at KMAX = 128) in VGPRs, B from LDS (one ds_read_b128 feeds the even-
// and odd-column tiles), four independent MFMA chains per wave (two 32-column
// halves x even/odd), the next band's A and tableau loads issued before the
// current band's MFMAs (PF = 1).
template <int KMAX, int LB, int PF, int MODE = 0>
__global__ __launch_bounds__(256, LB) void k_flushy(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                    const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                    int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows, int skip) {
    constexpr int G = KMAX / 4;
    constexpr int PS = 68;                        // padded LDS row (doubles): rows lk = 0..3 start on different banks
    constexpr int SU = KMAX * 32 / 256;           // 16-byte P pieces staged per thread
    __shared__ __attribute__((aligned(16))) double sP[KMAX * PS];
    __shared__ int64_t next_item;
    __shared__ unsigned lmask;
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
            lmask = 0;
        }
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t c0 = tile * 64;
        {   // stage -P: piece e = (q, pair cp), cp = e % 32 is the same for all of this thread's pieces
            const int cp = threadIdx.x & 31;
            const int64_t cj = c0 + 2 * cp;
            bool lv = false;
#pragma unroll
            for (int u = 0; u < SU; u++) {
                const int q = (u * 256 + threadIdx.x) >> 5;
                d2 v = d2{0.0, 0.0};
                if (q < np && cj < g.ncols) v = *(const d2 *)(Pbuf + (int64_t)q * ld + cj);
                lv = lv || v.x != 0.0 || v.y != 0.0;
                *(d2 *)&sP[q * PS + 2 * cp] = -v;
            }
            if (lv) atomicOr(&lmask, 1u << cp);
        }
        __syncthreads();
        const unsigned lm = lmask;
        if (lm == 0 && skip) continue;                            // the whole tile is skipped
        const unsigned live = skip ? lm : 0xffffffffu;
        bool okh[2];
#pragma unroll
        for (int h = 0; h < 2; h++) okh[h] = ((live >> (16 * h + lc)) & 1u) && c0 + 32 * h + 2 * lc < g.ncols;
        if (threadIdx.x == 0) {
            unsigned long long cols = 0;
            for (int cp = 0; cp < 32; cp++)
                if (((live >> cp) & 1u) && c0 + 2 * cp < g.ncols) cols += (c0 + 2 * cp + 1 < g.ncols) ? 2 : 1;
            touched += cols * (unsigned long long)(i1 - i0);
        }
        const int nb = (int)((i1 - i0 + 15) / 16);
        auto aload = [&](double (&a)[G], int b) {
            const int64_t row = i0 + 16 * (int64_t)b + lc;
#pragma unroll
            for (int gq = 0; gq < G; gq++) {
                const int q = 4 * gq + lk;
                a[gq] = q < np ? Cbuf[(int64_t)q * cs + row] : 0.0;
            }
        };
        auto tload = [&](d2 (&x)[2][4], int b) {
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * (int64_t)b + lk + 4 * r;
                    x[h][r] = (MODE != 2 && okh[h] && row < i1)
                                  ? __builtin_nontemporal_load((const d2 *)(T + row * ld + c0 + 32 * h + 2 * lc))
                                  : d2{0.0, 0.0};
                }
        };
        int b = wave;
        if (b >= nb) continue;
        double a[G];
        d2 t[2][4];
        aload(a, b);
        tload(t, b);
        for (; b < nb; b += 4) {
            double an[G];
            d2 tn[2][4];
            const bool more = PF && b + 4 < nb;
            if (more) {
                aload(an, b + 4);
                tload(tn, b + 4);
            }
            d4 acc[4];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                acc[2 * h] = d4{t[h][0].x, t[h][1].x, t[h][2].x, t[h][3].x};
                acc[2 * h + 1] = d4{t[h][0].y, t[h][1].y, t[h][2].y, t[h][3].y};
            }
            const double *sp = &sP[lk * PS + 2 * lc];
            // B of step gq + 1 is read from LDS before the MFMAs of step gq (two register sets), so
            // the LDS latency hides behind four MFMAs instead of stalling every step
            d2 b0c = *(const d2 *)sp, b1c = *(const d2 *)(sp + 32);
#pragma unroll
            for (int gq = 0; gq < (MODE == 1 ? 0 : G); gq++) {
                d2 b0n = b0c, b1n = b1c;
                if (gq + 1 < G) {
                    b0n = *(const d2 *)(sp + 4 * (gq + 1) * PS);
                    b1n = *(const d2 *)(sp + 4 * (gq + 1) * PS + 32);
                }
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], b0c.x, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], b0c.y, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], b1c.x, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], b1c.y, acc[3], 0, 0, 0);
                b0c = b0n;
                b1c = b1n;
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // the 2 LDS reads of step gq + 1 ...
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // ... ahead of the 4 MFMAs of step gq
            }
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * (int64_t)b + lk + 4 * r;
                    if ((MODE != 2 || acc[2 * h][r] == 12345.0) && okh[h] && row < i1)
                        __builtin_nontemporal_store(d2{acc[2 * h][r], acc[2 * h + 1][r]},
                                                    (d2 *)(T + row * ld + c0 + 32 * h + 2 * lc));
                }
            if (!PF && b + 4 < nb) {
                aload(an, b + 4);
                tload(tn, b + 4);
            }
#pragma unroll
            for (int gq = 0; gq < G; gq++) a[gq] = an[gq];
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int r = 0; r < 4; r++) t[h][r] = tn[h][r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

// probe modes: 1 = no multiplier staging (ring left as is), 2 = no tableau loads / stores,
// 3 = no block barrier per band (timing only)
template <int KMAX, int NB, int WPB, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_flushv_probe(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                     const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                     int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows,
                                                     int skip) {
    constexpr int NTH = 64 * WPB;
    constexpr int G = KMAX / 4;
    constexpr int BAND = KMAX * 16;                 // doubles per band
    constexpr int NPC = BAND / 2;                   // 16-byte multiplier pieces per band
    constexpr int PER = (NPC + NTH - 1) / NTH;      // ... per thread
    __shared__ __attribute__((aligned(16))) double sC[NB][BAND];
    __shared__ int64_t next_item;
    __shared__ int wsum[WPB];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t cl = tile * (16 * WPB) + wave * 16 + lc;      // this lane's column
        const bool in = cl < g.ncols;
        double b[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            const double v = (in && q < np) ? Pbuf[(int64_t)q * ld + cl] : 0.0;
            b[gq] = v;
            live = live || v != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;     // OR over the 4 lanes of the column
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? 1 : 0;
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
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                const int q = e >> 3, rr = 2 * (e & 7);
                const int64_t row = i0 + 16 * s + rr;
                d2 v = d2{0.0, 0.0};
                if (MODE != 1 && e < NPC && s < nb && q < np && row < i1) v = *(const d2 *)(Cbuf + (int64_t)q * cs + row);
                cr[u] = -v;
            }
        };
        auto cstore = [&](const d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * NTH;
                if (MODE != 1 && e < NPC) *(d2 *)(&sC[s % NB][2 * e]) = cr[u];
            }
        };
        for (int s = 0; s < NB - 1; s++) {
            d2 cr[PER];
            cload(cr, s);
            cstore(cr, s);
        }
        d2 cn[PER];
        cload(cn, NB - 1);
        auto tload = [&](double (&x)[4], int s) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                x[r] = (MODE != 2 && ok && row < i1) ? __builtin_nontemporal_load(T + row * ld + cl) : 0.0;
            }
        };
        double t[4];
        tload(t, 0);
        for (int s = 0; s < nb; s++) {
            double tn[4];
            if (s + 1 < nb) tload(tn, s + 1);
            if (MODE != 3) __syncthreads();     // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
            if (wlive) {
                d4 acc = d4{t[0], t[1], t[2], t[3]};
                const double *sa = &sC[s % NB][lk * 16 + lc];
#pragma unroll
                for (int gq = 0; gq < G; gq++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], b[gq], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * s + lk + 4 * r;
                    if (MODE != 2 && ok && row < i1) __builtin_nontemporal_store(acc[r], T + row * ld + cl);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}


// probe modes (timing only): 1 = no MFMA (the data path alone), 2 = no DMA (the matrix path alone)
template <int KMAX, int MW, int LW, int DT, int MODE>
__global__ __launch_bounds__(64 * (MW + LW)) void k_flushs_probe(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                           const double *__restrict__ Pbuf,
                                                           const double *__restrict__ Cbuf, int64_t cs, int64_t ntiles,
                                                           int64_t nitems, int64_t rows, int skip,
                                                           const double *__restrict__ zrow) {
    constexpr int G = KMAX / 4;
    constexpr int TW = 16 * MW;                     // tile width (columns)
    constexpr int RING = DT + 1;
    constexpr int TB = 16 * TW;                     // doubles of tableau per band
    constexpr int CB = 16 * KMAX;                   // doubles of multipliers per band
    constexpr int SLOT = TB + CB;
    constexpr int NT_DMA = TB / 128;                // 1 KB DMA instructions per band: tableau ...
    constexpr int NC_DMA = CB / 128;                // ... and multipliers
    static_assert(TW == 128 && NT_DMA % LW == 0 && NC_DMA % LW == 0, "one 1 KB row per tableau DMA");
    constexpr int TPW = NT_DMA / LW, CPW = NC_DMA / LW;   // per loader wave
    extern __shared__ __attribute__((aligned(16))) double ring[];
    __shared__ int64_t next_item;
    __shared__ int wsum[MW];
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool mw = wave < MW;                      // matrix wave (else loader wave wave - MW)
    const int lw = wave - MW;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) next_item = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = next_item;
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t c0 = tile * TW;
        const int64_t cl = c0 + (mw ? wave * 16 : 0) + lc;          // a matrix lane's column
        const bool in = mw && cl < g.ncols;
        double b[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            const double v = (in && q < np) ? Pbuf[(int64_t)q * ld + cl] : 0.0;
            b[gq] = -v;
            live = live || v != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? 1 : 0;
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        const bool wlive = mine > 0;                                   // wave-uniform
        if (mw && lane == 0) wsum[wave] = mine;
        if (__syncthreads_count(wlive && lane == 0) == 0) continue;    // the whole tile is skipped
        if (threadIdx.x == 0) {
            int sum = 0;
#pragma unroll
            for (int w = 0; w < MW; w++) sum += wsum[w];
            touched += (unsigned long long)sum * (unsigned long long)(i1 - i0);
        }
        const int nb = (int)((i1 - i0 + 15) / 16);
        // loader wave: band s into ring slot s % RING (rows past i1 and slots
        // past np read the zero row; the tableau's last tile reads into the
        // next row's padding, which the stores never write back)
        auto issue = [&](int s) {
            double *slot = ring + (size_t)(s % RING) * SLOT;
#pragma unroll
            for (int u = 0; u < TPW; u++) {
                const int rr = lw * TPW + u;
                const int64_t row = i0 + 16 * s + rr;
                const double *src = row < i1 ? T + row * ld + c0 + 2 * lane : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(slot + rr * TW), 16, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < CPW; u++) {
                const int e = lw * CPW + u;                 // 8 slots x 16 rows per instruction
                const int q = 8 * e + (lane >> 3);
                const int64_t row = i0 + 16 * s + 2 * (lane & 7);
                const double *src = (q < np && row < i1) ? Cbuf + (int64_t)q * cs + row : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(slot + TB + e * 128), 16, 0, 0);
            }
        };
        if (!mw && MODE != 2)
            for (int s = 0; s < DT && s < nb; s++) issue(s);
        for (int s = 0; s < nb; s++) {
            if (!mw) {   // band s has landed (bands s+1 .. s+DT-1 may still be in flight)
                if (s + DT - 1 < nb) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DT - 1) * (TPW + CPW)) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            // band s is in the ring; slot (s - 1) % RING is free. A bare
            // s_barrier: __syncthreads() would also wait for every wave's
            // outstanding memory operations (vmcnt(0)), i.e. drain the DMA
            // ring and the matrix waves' stores each band
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (!mw) {
                if (MODE != 2 && s + DT < nb) issue(s + DT);
            } else if (wlive) {
                const double *slot = ring + (size_t)(s % RING) * SLOT;
                d4 acc;
#pragma unroll
                for (int r = 0; r < 4; r++) acc[r] = slot[(lk + 4 * r) * TW + wave * 16 + lc];
                const double *sa = slot + TB + lk * 16 + lc;
#pragma unroll
                for (int gq = 0; gq < G; gq++) if (MODE != 1) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], b[gq], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i0 + 16 * s + lk + 4 * r;
                    if (ok && row < i1) __builtin_nontemporal_store(acc[r], T + row * ld + cl);
                }
            }
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}


// k_flushg (round 3): no LDS and no barrier. Each WAVE takes its own items
// (32-column tile x `rows` rows) from the queue; B = P in VGPRs for the item,
// A = -C straight from the Infinity Cache / L2 by buffer loads (one VGPR
// offset, the slot stride in an SGPR), A of band s+1 loaded into the register
// its band-s MFMA just read, tableau bands DEP ahead. Same chain as k_flushw
// (slots in ascending order, A = -C, B = P; past np A = -0, B = +0), so the
// results are bitwise. Every 16-byte store is followed by s_nop 1: hipcc
// emits none after raw buffer stores, and a VALU write of the store's data
// registers right behind it corrupts the stored value when other waves share
// the SIMD (tools/overlap_lab.hip, tools/store_hazard_scan.py).
template <int KMAX, int DEP, int LB>
__global__ __launch_bounds__(256, LB) void k_flushg(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                    const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                    int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows,
                                                    int skip) {
    constexpr int G = KMAX / 4;
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    const __amdgpu_buffer_rsrc_t rc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Cbuf), (short)0, (int)(KMAX * cs * 8), 0x00020000);
    for (;;) {
        int64_t item = 0;
        if (lane == 0) item = (int64_t)atomicAdd(&st->fwork, 1ull);
        item = (int64_t)__builtin_amdgcn_readfirstlane((int)item);
        if (item >= nitems) break;
        const int64_t tile = item % ntiles, strip = item / ntiles;
        const int64_t i0 = strip * rows;
        const int64_t i1 = i0 + rows < g.nloc ? i0 + rows : g.nloc;
        const int64_t cl = tile * 32 + 2 * lc;
        const bool in = cl < g.ncols;
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
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? (cl + 1 < g.ncols ? 2 : 1) : 0;
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        if (mine == 0) continue;                        // wave-uniform: the whole tile is skipped
        if (lane == 0) touched += (unsigned long long)mine * (unsigned long long)(i1 - i0);
        const int nb = (int)((i1 - i0 + 15) / 16);
        const int voffT = (int)(((int64_t)lk * ld + cl) * 8);
        const int voffA = (int)(((int64_t)lk * cs + i0 + lc) * 8);
        auto band_rsrc = [&](int s) {
            return __builtin_amdgcn_make_buffer_rsrc(T + (i0 + (int64_t)16 * s) * ld, (short)0, (int)(16 * ld * 8),
                                                     0x00020000);
        };
        auto tload = [&](d2 (&x)[4], int s) {
            const __amdgpu_buffer_rsrc_t rt = band_rsrc(s);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool v = ok && i0 + 16 * s + lk + 4 * r < i1;
                const u4v w = __builtin_amdgcn_raw_buffer_load_b128(rt, voffT, (int)(r * 4 * ld * 8), 2);
                x[r] = v ? __builtin_bit_cast(d2, w) : d2{0.0, 0.0};
            }
        };
        auto aload1 = [&](int s, int gq) -> double {
            const bool v = s < nb && 4 * gq + lk < np && i0 + 16 * s + lc < i1;
            const auto w = __builtin_amdgcn_raw_buffer_load_b64(rc, voffA + s * 16 * 8, (int)(gq * 4 * cs * 8), 0);
            return v ? -__builtin_bit_cast(double, w) : -0.0;
        };
        double a[G];
#pragma unroll
        for (int gq = 0; gq < G; gq++) a[gq] = aload1(0, gq);
        d2 tb[DEP][4];
#pragma unroll
        for (int d = 0; d < DEP; d++) tload(tb[d], d);
        for (int s0 = 0; s0 < nb; s0 += DEP) {
#pragma unroll
            for (int d = 0; d < DEP; d++) {
                const int s = s0 + d;
                if (s < nb) {
                    d4 ae = d4{tb[d][0].x, tb[d][1].x, tb[d][2].x, tb[d][3].x};
                    d4 ao = d4{tb[d][0].y, tb[d][1].y, tb[d][2].y, tb[d][3].y};
#pragma unroll
                    for (int gq = 0; gq < G; gq++) {
                        ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], be[gq], ae, 0, 0, 0);
                        ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gq], bo[gq], ao, 0, 0, 0);
                        a[gq] = aload1(s + 1, gq);
                    }
                    const __amdgpu_buffer_rsrc_t rt = band_rsrc(s);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        if (ok && i0 + 16 * s + lk + 4 * r < i1)
                            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, d2{ae[r], ao[r]}), rt, voffT,
                                                                   (int)(r * 4 * ld * 8), 2);
                        asm volatile("s_nop 1" ::: "memory");
                    }
                    if (s + DEP < nb) tload(tb[d], s + DEP);
                }
            }
        }
    }
    if (lane == 0 && touched) atomicAdd(&st->touched, touched);
}


}  // namespace lpg

using namespace lpg;

__global__ void k_fill(double *x, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * 0x1.0p-53 - 0.25;
    }
}

// P_q[j] = 0 for the slack block and the padding (the skipped columns)
__global__ void k_zero_cols(double *P, int64_t ld, int64_t j0, int k) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)k * ld; e += (int64_t)gridDim.x * blockDim.x)
        if (e % ld >= j0) P[e] = 0.0;
}

__global__ void k_cmp(const double *a, const double *b, int64_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += __double_as_longlong(a[i]) != __double_as_longlong(b[i]);
    if (c) atomicAdd(bad, c);
}

struct Lab {
    Geo g{};
    DevState *st = nullptr;
    double *T = nullptr, *T0 = nullptr, *Tref = nullptr, *Pbuf = nullptr, *Cbuf = nullptr, *zbuf = nullptr;
    int64_t n = 0, cs = 0;
    int K = 128;
    unsigned long long *bad = nullptr;
    hipEvent_t e0, e1;

    void reset_state(int np) {
        DevState h{};
        h.npend = np;
        CHK(hipMemcpy(st, &h, sizeof h, hipMemcpyHostToDevice));
    }
};

typedef void (*LaunchFn)(Lab &L);

// the engine's k_flushw<64> twice: slots 0..63, then 64..127 (same chain)
static void fn_ref(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128;
    const int64_t rows = 512, nitems = flush_nitems(ntiles, rows, L.g.nloc);
    for (int h = 0; h < L.K / 64; h++) {
        L.reset_state(64);
        hipLaunchKernelGGL((k_flushw<64, 2, 2, 4>), dim3(512), dim3(256), 0, 0, L.g.T, L.g, L.st,
                           L.Pbuf + (int64_t)h * 64 * L.g.ld, L.Cbuf + (int64_t)h * 64 * L.cs, L.cs, ntiles, nitems,
                           rows, 1);
    }
}

template <int KMAX, int NB, int LB, int R>
static void fn_w(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128;
    const int64_t nitems = flush_nitems(ntiles, R, L.g.nloc);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushw<KMAX, NB, LB, 4>), dim3((unsigned)std::min<int64_t>(nitems, 256 * LB)), dim3(256), 0,
                       0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, (int64_t)R, 1);
}

template <int KMAX, int NB, int WPB, int R>
static void fn_v(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 16 * WPB - 1) / (16 * WPB);
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushv<KMAX, NB, WPB>), dim3((unsigned)std::min<int64_t>(nitems, 256)), dim3(64 * WPB), 0,
                       0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, (int64_t)R, 1);
}

template <int KMAX, int NB, int WPB, int R, int MODE>
static void fn_vp(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 16 * WPB - 1) / (16 * WPB);
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushv_probe<KMAX, NB, WPB, MODE>), dim3((unsigned)std::min<int64_t>(nitems, 256)),
                       dim3(64 * WPB), 0, 0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, (int64_t)R, 1);
}

template <int KMAX, int MW, int LW, int DT, int R>
static void fn_s(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 16 * MW - 1) / (16 * MW);
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    const size_t lds = (size_t)(DT + 1) * (16 * 16 * MW + 16 * KMAX) * 8;
    static bool set = false;
    if (!set) {
        CHK(hipFuncSetAttribute((const void *)k_flushs<KMAX, MW, LW, DT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
        set = true;
    }
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushs<KMAX, MW, LW, DT>), dim3((unsigned)std::min<int64_t>(nitems, 256)),
                       dim3(64 * (MW + LW)), lds, 0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems,
                       (int64_t)R, 1, (const double *)L.zbuf);
}

template <int KMAX, int MW, int LW, int DT, int R, int MODE>
static void fn_sp(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 16 * MW - 1) / (16 * MW);
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    const size_t lds = (size_t)(DT + 1) * (16 * 16 * MW + 16 * KMAX) * 8;
    static bool set = false;
    if (!set) {
        CHK(hipFuncSetAttribute((const void *)k_flushs_probe<KMAX, MW, LW, DT, MODE>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        set = true;
    }
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushs_probe<KMAX, MW, LW, DT, MODE>), dim3((unsigned)std::min<int64_t>(nitems, 256)),
                       dim3(64 * (MW + LW)), lds, 0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems,
                       (int64_t)R, 1, (const double *)L.zbuf);
}

template <int KMAX, int SB, int LB, int R>
static void fn_x(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128;
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushx<KMAX, SB, LB>), dim3((unsigned)std::min<int64_t>(nitems, 256 * LB)), dim3(256), 0, 0,
                       L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, (int64_t)R, 1, L.zbuf);
}

template <int KMAX, int LB, int PF, int R, int MODE = 0>
static void fn_y(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 63) / 64;
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushy<KMAX, LB, PF, MODE>), dim3((unsigned)std::min<int64_t>(nitems, 256 * LB)), dim3(256), 0, 0,
                       L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, (int64_t)R, 1);
}


template <int KMAX, int DEP, int LB, int R>
static void fn_g(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 31) / 32;
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    L.reset_state(L.K);
    hipLaunchKernelGGL((k_flushg<KMAX, DEP, LB>), dim3(256 * LB), dim3(256), 0, 0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf,
                       L.cs, ntiles, nitems, (int64_t)R, 1);
}

// 96-slot reference: the product's k_flushw<96> (bitwise = the fma chain, tests/test_gpu_defer.py)
static void fn_ref96(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128, rows = 512;
    const int64_t nitems = flush_nitems(ntiles, rows, L.g.nloc);
    L.reset_state(96);
    hipLaunchKernelGGL((k_flushw<96, 2, 2, 4>), dim3((unsigned)std::min<int64_t>(nitems, 512)), dim3(256), 0, 0, L.g.T,
                       L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, rows, 1);
}

static bool g_nocheck = false;
static double run(Lab &L, LaunchFn fn, const char *name, int reps) {
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    fn(L);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipMemset(L.bad, 0, 8));
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, L.T, L.Tref, L.n, L.bad);
    unsigned long long nb = 0;
    CHK(hipMemcpy(&nb, L.bad, 8, hipMemcpyDeviceToHost));
    if (nb && !g_nocheck) {
        printf("%-28s MISMATCH: %llu doubles differ from the reference\n", name, nb);
        fflush(stdout);
        return -1;
    }
    double best = 1e30, sum = 0;
    for (int r = 0; r < reps; r++) {
        CHK(hipEventRecord(L.e0));
        fn(L);
        CHK(hipEventRecord(L.e1));
        CHK(hipEventSynchronize(L.e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, L.e0, L.e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    DevState h{};
    CHK(hipMemcpy(&h, L.st, sizeof h, hipMemcpyDeviceToHost));
    const double bytes = 16.0 * (double)h.touched;
    const double flops = 2.0 * L.K * (double)h.touched;
    printf("%-28s K=%d  best %.3f ms  mean %.3f ms  touched %.3f GB  %.0f GB/s  %.1f TFLOP/s (best)\n", name, L.K,
           best, sum / reps, bytes / 1e9, bytes / (best * 1e-3) / 1e9, flops / (best * 1e-3) / 1e12);
    fflush(stdout);
    return best;
}

int main(int argc, char **argv) {
    Lab L;
    const int64_t m = argc > 1 ? atoll(argv[1]) : 16384, nstruct = 2 * m;
    const int64_t ncols = nstruct + m + 1, ld = (ncols + 63) / 64 * 64;
    L.n = m * ld;
    L.cs = (m + 63) / 64 * 64;
    const int SL = 128;
    CHK(hipMalloc(&L.T, L.n * 8));
    CHK(hipMalloc(&L.T0, L.n * 8));
    CHK(hipMalloc(&L.Tref, L.n * 8));
    CHK(hipMalloc(&L.st, sizeof(DevState)));
    CHK(hipMalloc(&L.bad, 8));
    CHK(hipMalloc(&L.Pbuf, (size_t)SL * ld * 8));
    CHK(hipMalloc(&L.Cbuf, (size_t)SL * L.cs * 8));
    CHK(hipMalloc(&L.zbuf, 4096));
    CHK(hipMemset(L.zbuf, 0, 4096));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, L.T0, L.n, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, L.Pbuf, (int64_t)SL * ld, 2ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, L.Cbuf, (int64_t)SL * L.cs, 3ull);
    hipLaunchKernelGGL(k_zero_cols, dim3(1024), dim3(256), 0, 0, L.Pbuf, ld, nstruct + 1, SL);
    CHK(hipDeviceSynchronize());
    L.g.T = L.T;
    L.g.ld = ld;
    L.g.nloc = m;
    L.g.nobj = 1;
    L.g.ncols = ncols;
    L.g.nact = ncols - 1;
    L.g.m = m;
    CHK(hipEventCreate(&L.e0));
    CHK(hipEventCreate(&L.e1));
    printf("flush lab: %lld rows x %lld cols (ld %lld), K=%d, P zero for columns > %lld\n", (long long)m,
           (long long)ncols, (long long)ld, L.K, (long long)nstruct);
    if (getenv("LAB_K")) L.K = atoi(getenv("LAB_K"));
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    if (L.K == 96) {   // k_flushw<96> is the reference; then the global-A form against it, and stop
        fn_ref96(L);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
        run(L, fn_ref96, "w<96,2,2,512> (product)", 5);
        run(L, fn_g<96, 2, 1, 512>, "g<96,dep2,1 wave/SIMD,512>", 5);
        run(L, fn_g<96, 2, 2, 512>, "g<96,dep2,2 waves/SIMD,512>", 5);
        run(L, fn_g<96, 3, 1, 512>, "g<96,dep3,1 wave/SIMD,512>", 5);
        run(L, fn_g<96, 1, 2, 512>, "g<96,dep1,2 waves/SIMD,512>", 5);
        run(L, fn_g<96, 2, 2, 1024>, "g<96,dep2,2 waves/SIMD,1024>", 5);
        run(L, fn_g<96, 2, 2, 256>, "g<96,dep2,2 waves/SIMD,256>", 5);
        run(L, fn_ref96, "w<96,2,2,512> (product)", 5);
        return 0;
    }
    fn_ref(L);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
    const int reps = 5;
    const char *only = getenv("LAB_ONLY");
    auto want = [&](const char *nm) { return !only || strstr(nm, only); };
    if (want("ref 2x w<64>")) run(L, fn_ref, "ref 2x w<64>", reps);
#define W(KM, NB, LB, R) \
    if (want("w<" #KM "," #NB "," #LB "," #R ">")) run(L, fn_w<KM, NB, LB, R>, "w<" #KM "," #NB "," #LB "," #R ">", reps);
#define X(KM, SB, LB, R) \
    if (want("x<" #KM "," #SB "," #LB "," #R ">")) run(L, fn_x<KM, SB, LB, R>, "x<" #KM "," #SB "," #LB "," #R ">", reps);
    W(128, 2, 1, 512)
#define S(KM, MW, LW, DT, R) \
    if (want("s<" #KM "," #MW "," #LW "," #DT "," #R ">")) run(L, fn_s<KM, MW, LW, DT, R>, "s<" #KM "," #MW "," #LW "," #DT "," #R ">", reps);
    S(128, 8, 4, 3, 512)
    S(128, 8, 4, 2, 512)
    S(128, 8, 4, 3, 1024)
    S(128, 8, 2, 3, 512)
    S(128, 8, 8, 3, 512)
#define V(KM, NB, WPB, R) \
    if (want("v<" #KM "," #NB "," #WPB "," #R ">")) run(L, fn_v<KM, NB, WPB, R>, "v<" #KM "," #NB "," #WPB "," #R ">", reps);
    V(128, 2, 8, 512)
    V(128, 2, 8, 256)
    V(128, 3, 8, 512)
    V(128, 2, 16, 512)
    V(128, 2, 4, 512)
    W(128, 3, 1, 512)
    X(128, 2, 1, 512)
#define Y(KM, LB, PF, R) \
    if (want("y<" #KM "," #LB "," #PF "," #R ">")) run(L, fn_y<KM, LB, PF, R>, "y<" #KM "," #LB "," #PF "," #R ">", reps);
    Y(128, 1, 1, 2048)
    g_nocheck = true;   // timing-only probes: no MFMA (memory alone), no tableau traffic (matrix cores alone)
    if (want("ymem")) run(L, fn_y<128, 1, 1, 2048, 1>, "ymem<128> (no MFMA)", reps);
    if (want("ymfma")) run(L, fn_y<128, 1, 1, 2048, 2>, "ymfma<128> (no T traffic)", reps);
    if (want("sp")) run(L, fn_sp<128, 8, 4, 3, 1024, 1>, "sp1 (no MFMA)", reps);
    if (want("sp")) run(L, fn_sp<128, 8, 4, 3, 1024, 2>, "sp2 (no DMA)", reps);
    if (want("vp")) run(L, fn_vp<128, 2, 16, 512, 1>, "vp1 (no C staging)", reps);
    if (want("vp")) run(L, fn_vp<128, 2, 16, 512, 2>, "vp2 (no T traffic)", reps);
    if (want("vp")) run(L, fn_vp<128, 2, 16, 512, 3>, "vp3 (no band barrier)", reps);
    if (want("vp")) run(L, fn_vp<128, 2, 8, 512, 1>, "vp1 w8 (no C staging)", reps);
    if (want("vp")) run(L, fn_vp<128, 2, 8, 512, 2>, "vp2 w8 (no T traffic)", reps);
    return 0;
}
