// flush64_lab.hip — the 64-pivot block pass at config 3 (16384 x 49153, ld
// 49216, fp64): the product's k_flushw<64> against a form whose tableau bands
// and multipliers arrive by LDS-DMA (global_load_lds, no registers), DT bands
// ahead, so that a CU keeps 2-3x the bytes in flight that k_flushw's
// one-band-ahead register prefetch holds (k_flushw moves
// 5.1 TB/s; the in-flight bytes per CU, 32 KB, are below what the guide says
// hides an HBM miss, ~72 KB). Every design is checked bitwise against the
// product kernel before it is timed. Tools only.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/flush64_lab tools/flush64_lab.hip
//   tools/flush64_lab [reps]
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

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// k_flushd (measured slower than k_flushw, not in the product: profiles/r04_flush64_lab.log):
// k_flushw's wave tile (16 rows x 32 columns, lane (lk, lc) holds
// column pair 2 lc and rows lk + 4 r; even / odd-column MFMA chains, B in
// VGPRs) with the tableau band and the band's multipliers brought into an LDS
// ring by LDS-DMA DT bands ahead. Per wave and band: 4 tableau DMAs (1 KB
// each, the wave's own 16 x 32 piece, read back by the same lanes) and CPW
// multiplier DMAs (the block's 8 KB band of C, shared: one barrier per band).
// Multipliers are raw C with B = -P: fma(c, -p, x) == fma(-c, p, x) bit for
// bit; padding slots read A = +0 from the zero row against B = -0, and
// x + (+0)(-0) == x for every x -- the same chain as k_flushw. Every wave
// issues the same number of memory instructions per band (sources past the
// item or outside the live columns read the zero row, stores of such lanes
// go to a sink), so the counted vmcnt waits are exact. All LDS is one dynamic
// array (a second __shared__ object makes hipcc wait vmcnt(0) before LDS
// reads, cdna_hip_programming.md "Projection GEMM" item 4(a)).
template <int KMAX, int WPB, int DT, int MINB = 1>
__global__ __launch_bounds__(64 * WPB, MINB) void k_flushd(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                        const double *__restrict__ Pbuf,
                                                        const double *__restrict__ Cbuf, int64_t cs, int64_t ntiles,
                                                        int64_t nitems, int64_t rows, int skip,
                                                        const double *__restrict__ zrow, double *__restrict__ sink) {
    constexpr int G = KMAX / 4;
    constexpr int RING = DT + 1;
    constexpr int TWV = 512;                        // doubles of tableau per wave per band
    constexpr int CB = 16 * KMAX;                   // doubles of multipliers per band
    constexpr int CPW = CB / 128 / WPB;             // multiplier DMAs (1 KB) per wave per band
    static_assert(CPW >= 1 && CB / 128 % WPB == 0, "multiplier band = whole DMAs per wave");
    constexpr int NI = 4 + CPW;                     // DMAs per wave per band
    constexpr int NS = 4;                           // stores per wave per band
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double *sT = lds;                               // [RING][WPB][TWV]
    double *sC = lds + RING * WPB * TWV;            // [RING][CB]
    int64_t *sx = (int64_t *)(sC + RING * CB);      // [0] next item, [1 ..] per-wave counts
    const int np = (int)st->npend;
    if (np <= 0) return;
    const int64_t ld = g.ld;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    unsigned long long touched = 0;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) sx[0] = (int64_t)atomicAdd(&st->fwork, 1ull);
        __syncthreads();
        const int64_t item = sx[0];
        if (item >= nitems) break;
        int64_t tile, i0, i1;
        flush_item(item, ntiles, rows, g.nloc, tile, i0, i1);
        const int64_t cl = tile * (32 * WPB) + wave * 32 + 2 * lc;
        const bool in = cl < g.ncols;
        double be[G], bo[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            d2 v = d2{0.0, 0.0};
            if (in && q < np) v = *(const d2 *)(Pbuf + (int64_t)q * ld + cl);
            be[gq] = -v.x;
            bo[gq] = -v.y;
            live = live || v.x != 0.0 || v.y != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        int mine = (lk == 0 && ok) ? (cl + 1 < g.ncols ? 2 : 1) : 0;
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        if (lane == 0) sx[1 + wave] = mine;
        if (__syncthreads_count(mine > 0 && lane == 0) == 0) continue;   // the whole tile is skipped
        if (threadIdx.x == 0) {
            int64_t sum = 0;
#pragma unroll
            for (int w = 0; w < WPB; w++) sum += sx[1 + w];
            touched += (unsigned long long)sum * (unsigned long long)(i1 - i0);
        }
        const int nb = (int)((i1 - i0 + 15) / 16);
        auto issue = [&](int s) {
            double *ts = sT + ((s % RING) * WPB + wave) * TWV;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                const double *src = (ok && s < nb && row < i1) ? T + row * ld + cl : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(ts + r * 128), 16, 0, 0);
            }
            double *cslot = sC + (s % RING) * CB;
#pragma unroll
            for (int u = 0; u < CPW; u++) {
                const int blk = u * WPB + wave;               // 1 KB block of the band's multiplier image
                const int e = blk * 64 + lane;                // 16-byte piece: slot e >> 3, rows 2 (e & 7) .. +1
                const int q = e >> 3;
                const int64_t row = i0 + 16 * s + 2 * (e & 7);
                const double *src = (q < np && s < nb && row < i1) ? Cbuf + (int64_t)q * cs + row : zrow + 2 * lane;
                __builtin_amdgcn_global_load_lds((const void *)src, (void *)(cslot + blk * 128), 16, 0, 0);
            }
        };
#pragma unroll
        for (int s = 0; s < DT; s++) issue(s);
        for (int s = 0; s < nb; s++) {
            // band s has landed: the younger memory instructions are the
            // DMAs and stores issued after it (exact: every band issues NI
            // DMAs and NS stores per wave)
            if (s >= DT) vm_wait<NS + (DT - 1) * (NI + NS)>();
            else if (s == 0) vm_wait<(DT - 1) * NI>();
            else if (s == 1) vm_wait<(DT - 1) * NI + NS>();
            else vm_wait<(DT - 1) * NI + 2 * NS>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();                     // every wave's DMAs of band s are in; slot (s-1) % RING is free
            asm volatile("" ::: "memory");
            issue(s + DT);
            const double *ts = sT + ((s % RING) * WPB + wave) * TWV;
            d4 ae, ao;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const d2 t = *(const d2 *)(ts + r * 128 + 2 * lane);
                ae[r] = t.x;
                ao[r] = t.y;
            }
            const double *sa = sC + (s % RING) * CB + lk * 16 + lc;
#pragma unroll
            for (int gq = 0; gq < G; gq++) {
                const double a = sa[gq * 64];
                ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a, be[gq], ae, 0, 0, 0);
                ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bo[gq], ao, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int64_t row = i0 + 16 * s + lk + 4 * r;
                d2 *dst = (ok && row < i1) ? (d2 *)(T + row * ld + cl) : (d2 *)(sink + 2 * lane);
                __builtin_nontemporal_store(d2{ae[r], ao[r]}, dst);
            }
        }
        vm_wait<0>();                                         // the dummy DMAs past the item (zero row) land
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

template <int KMAX, int WPB, int DT>
constexpr size_t flushd_lds() {
    return (size_t)(DT + 1) * (WPB * 512 + 16 * KMAX) * sizeof(double) + (1 + WPB) * sizeof(int64_t);
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
    double *T = nullptr, *T0 = nullptr, *Tref = nullptr, *Pbuf = nullptr, *Cbuf = nullptr, *zbuf = nullptr,
           *sink = nullptr;
    int64_t n = 0, cs = 0;
    int K = 64;
    unsigned long long *bad = nullptr;
    hipEvent_t e0, e1;

    void reset_state(int np) {
        DevState h{};
        h.npend = np;
        CHK(hipMemcpy(st, &h, sizeof h, hipMemcpyHostToDevice));
    }
};
typedef void (*LaunchFn)(Lab &L);
static bool g_tail = true;   // the short tail items (flush_item); false: whole items throughout

// the product's launch of k_flushw<64> (lpg_kernels.hip launch_flush_main)
static void fn_ref(Lab &L) {
    const int64_t tw = 256, ntiles = (L.g.ncols + tw - 1) / tw, rows = g_tail ? 512 : -512;
    const int64_t nitems = flush_nitems(ntiles, rows, L.g.nloc);
    const int64_t nblocks = std::min<int64_t>(nitems, 512);
    L.reset_state(64);
    hipLaunchKernelGGL((k_flushw<64, 2, 2, 8>), dim3((unsigned)((nblocks + 1) / 2)), dim3(512), 0, 0, L.g.T, L.g,
                       L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, rows, 1);
}

template <int WPB, int DT, int R, int BPC, int KM = 64, int MINB = 1>
static void fn_d(Lab &L) {
    const int64_t tw = 32 * WPB, ntiles = (L.g.ncols + tw - 1) / tw;
    const int64_t rows = g_tail ? R : -R;
    const int64_t nitems = flush_nitems(ntiles, rows, L.g.nloc);
    const size_t lds = flushd_lds<KM, WPB, DT>();
    static bool set = false;
    if (!set) {
        CHK(hipFuncSetAttribute((const void *)k_flushd<KM, WPB, DT, MINB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
        set = true;
    }
    L.reset_state(KM);
    hipLaunchKernelGGL((k_flushd<KM, WPB, DT, MINB>), dim3((unsigned)std::min<int64_t>(nitems, 256 * BPC)), dim3(64 * WPB),
                       lds, 0, L.g.T, L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, rows, 1,
                       (const double *)L.zbuf, L.sink);
}

// the product's launch of k_flushw<96> (launch_flush_main: 4-wave blocks, 128-column tiles, 2 per CU)
template <int R = 512>
static void fn_ref96(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128, rows = g_tail ? R : -R;
    const int64_t nitems = flush_nitems(ntiles, rows, L.g.nloc);
    L.reset_state(96);
    hipLaunchKernelGGL((k_flushw<96, 2, 2, 4>), dim3((unsigned)std::min<int64_t>(nitems, 512)), dim3(256), 0, 0, L.g.T,
                       L.g, L.st, L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, rows, 1);
}

static double run(Lab &L, LaunchFn fn, const char *name, int reps) {
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    fn(L);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipMemset(L.bad, 0, 8));
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, L.T, L.Tref, L.n, L.bad);
    unsigned long long nb = 0;
    CHK(hipMemcpy(&nb, L.bad, 8, hipMemcpyDeviceToHost));
    if (nb) {
        printf("%-34s MISMATCH: %llu doubles differ from the reference\n", name, nb);
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
    printf("%-34s best %.3f ms  mean %.3f ms  touched %.3f GB  %.0f GB/s (best)  %.1f TFLOP/s\n", name, best,
           sum / reps, bytes / 1e9, bytes / (best * 1e-3) / 1e9, 2.0 * L.K * (double)h.touched / (best * 1e-3) / 1e12);
    fflush(stdout);
    return best;
}

int main(int argc, char **argv) {
    Lab L;
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int64_t m = 16384, nstruct = 2 * m;
    const int64_t ncols = nstruct + m + 1, ld = (ncols + 63) / 64 * 64;
    L.n = m * ld;
    L.cs = (m + 63) / 64 * 64;
    const int K = getenv("LAB_K") ? atoi(getenv("LAB_K")) : 64;   // 64 (config 3's block) or 96 (config 4's)
    const int SL = K;
    L.K = K;
    CHK(hipMalloc(&L.T, L.n * 8));
    CHK(hipMalloc(&L.T0, L.n * 8));
    CHK(hipMalloc(&L.Tref, L.n * 8));
    CHK(hipMalloc(&L.st, sizeof(DevState)));
    CHK(hipMalloc(&L.bad, 8));
    CHK(hipMalloc(&L.Pbuf, (size_t)SL * ld * 8));
    CHK(hipMalloc(&L.Cbuf, (size_t)SL * L.cs * 8));
    CHK(hipMalloc(&L.zbuf, (size_t)ld * 8));
    CHK(hipMalloc(&L.sink, 64 * 1024));
    CHK(hipMemset(L.zbuf, 0, (size_t)ld * 8));
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
    printf("flush64 lab: %lld rows x %lld cols (ld %lld), K=%d, P zero for columns > %lld\n", (long long)m,
           (long long)ncols, (long long)ld, K, (long long)nstruct);
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    if (K == 96) {
        fn_ref96<512>(L);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
        for (int rep = 0; rep < 2; rep++) {
            run(L, fn_ref96<512>, "w<96,2,2,4> (product, 512 rows)", reps);
            run(L, fn_ref96<1024>, "w<96,2,2,4> 1024 rows", reps);
            run(L, fn_ref96<2048>, "w<96,2,2,4> 2048 rows", reps);
            run(L, fn_d<12, 1, 512, 1, 96>, "d<96: 12 waves x1, DT 1, 512 rows>", reps);
            run(L, fn_d<12, 1, 1024, 1, 96>, "d<96: 12 waves x1, DT 1, 1024 rows>", reps);
            run(L, fn_d<12, 1, 2048, 1, 96>, "d<96: 12 waves x1, DT 1, 2048 rows>", reps);
            run(L, fn_d<4, 1, 512, 2, 96>, "d<96: 4 waves x2, DT 1, 512 rows>", reps);
            run(L, fn_d<4, 1, 1024, 2, 96>, "d<96: 4 waves x2, DT 1, 1024 rows>", reps);
            run(L, fn_d<4, 1, 2048, 2, 96>, "d<96: 4 waves x2, DT 1, 2048 rows>", reps);
        }
        return 0;
    }
    fn_ref(L);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
    run(L, fn_ref, "w<64,2,2,8> (product, tail)", reps);
    g_tail = false;
    run(L, fn_ref, "w<64,2,2,8> (no tail)", reps);
    run(L, fn_d<8, 2, 512, 1>, "d<8 waves, DT 2, 512 rows> no tail", reps);
    g_tail = true;
    run(L, fn_d<8, 2, 512, 1>, "d<8 waves, DT 2, 512 rows>", reps);
    run(L, fn_d<8, 1, 512, 1>, "d<8 waves, DT 1, 512 rows>", reps);
    run(L, fn_d<4, 2, 512, 2>, "d<4 waves x2, DT 2, 512 rows>", reps);
    run(L, fn_d<4, 3, 512, 1>, "d<4 waves x1, DT 3, 512 rows>", reps);
    run(L, fn_d<4, 1, 512, 3, 64, 3>, "d<4 waves x3, DT 1, 512 rows>", reps);
    run(L, fn_d<8, 2, 1024, 1>, "d<8 waves, DT 2, 1024 rows>", reps);
    run(L, fn_d<4, 2, 1024, 2>, "d<4 waves x2, DT 2, 1024 rows>", reps);
    run(L, fn_ref, "w<64,2,2,8> (product, tail)", reps);
    g_tail = false;
    run(L, fn_ref, "w<64,2,2,8> (no tail)", reps);
    return 0;
}
