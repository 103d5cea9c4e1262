// flush_lab.hip — standalone bench of deferred-flush kernel designs at the
// config-3 shape (16384 constraint rows x 49153 columns, ld 49216, fp64), on
// random T / Pbuf / Cbuf with the slack block's P entries zero (skipped, as in
// the first blocks of a solve). Every design is checked bitwise against the
// engine's default flush (launch_flush) before it is timed. Tools only: the
// product never links this file.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/flush_lab tools/flush_lab.hip
//   tools/flush_lab [K] [rows]
#include "../linearprogramming_amd/csrc/lpg_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

// k_flushr: 16 columns per wave (8-byte accesses), NSUB independent 16-row
// MFMA chains per iteration sharing the B fragments, multipliers staged
// negated in a padded LDS tile, the next iteration's rows loaded ahead.
template <int KMAX, int SR, int NSUB>
__global__ __launch_bounds__(kBlock) void k_flushr(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                   const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                   int64_t cs, int64_t ntiles, int64_t nitems, int skip) {
    constexpr int G = KMAX / 4;
    constexpr int SRP = SR + 16;
    constexpr int RI = 16 * NSUB;
    static_assert(SR % RI == 0, "strip must hold whole iterations");
    __shared__ __attribute__((aligned(16))) double sC[KMAX * SRP];
    __shared__ int64_t next_item;
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
        const int64_t i0 = strip * SR;
        const int64_t i1 = i0 + SR < g.nloc ? i0 + SR : g.nloc;
        const int64_t col = tile * 64 + wave * 16 + lc;
        const bool in = col < g.ncols;
        double b[G];
        bool live = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const int q = 4 * gq + lk;
            b[gq] = (in && q < np) ? Pbuf[(int64_t)q * ld + col] : 0.0;
            live = live || b[gq] != 0.0;
        }
        live = (__shfl_xor((int)live, 16, 64) | (int)live) != 0;
        live = (__shfl_xor((int)live, 32, 64) | (int)live) != 0;
        const bool ok = in && (!skip || live);
        const int cnt = __syncthreads_count(ok);
        if (cnt == 0) continue;
        if (threadIdx.x == 0) touched += (unsigned long long)(cnt / 4) * (unsigned long long)(i1 - i0);
        for (int e = threadIdx.x; e < KMAX * SR / 2; e += kBlock) {
            const int q = e / (SR / 2), rr = 2 * (e % (SR / 2));
            d2 v = d2{0.0, 0.0};
            if (q < np && i0 + rr < i1) v = *(const d2 *)(Cbuf + (int64_t)q * cs + i0 + rr);
            *(d2 *)(sC + q * SRP + rr) = -v;
        }
        __syncthreads();
        double *cp = T + col;
        double t[NSUB][4];
        auto load = [&](double (&x)[NSUB][4], int64_t i) {
#pragma unroll
            for (int s = 0; s < NSUB; s++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i + 16 * s + lk + 4 * r;
                    x[s][r] = (ok && row < i1) ? __builtin_nontemporal_load(cp + row * ld) : 0.0;
                }
        };
        int64_t i = i0;
        load(t, i);
        for (;;) {
            const bool more = i + RI < i1;
            double tn[NSUB][4];
            if (more) load(tn, i + RI);
            d4 acc[NSUB];
#pragma unroll
            for (int s = 0; s < NSUB; s++) acc[s] = d4{t[s][0], t[s][1], t[s][2], t[s][3]};
            const double *sa = sC + lk * SRP + (int)(i - i0) + lc;
#pragma unroll
            for (int gq = 0; gq < G; gq++) {
#pragma unroll
                for (int s = 0; s < NSUB; s++)
                    acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[4 * gq * SRP + 16 * s], b[gq], acc[s], 0, 0, 0);
            }
#pragma unroll
            for (int s = 0; s < NSUB; s++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = i + 16 * s + lk + 4 * r;
                    if (ok && row < i1) __builtin_nontemporal_store(acc[s][r], cp + row * ld);
                }
            if (!more) break;
            i += RI;
#pragma unroll
            for (int s = 0; s < NSUB; s++)
#pragma unroll
                for (int r = 0; r < 4; r++) t[s][r] = tn[s][r];
        }
    }
    if (threadIdx.x == 0 && touched) atomicAdd(&st->touched, touched);
}

template <int KMAX, int NB, int LB>
__global__ __launch_bounds__(kBlock, LB) void k_flushw2(double *__restrict__ T, Geo g, DevState *__restrict__ st,
                                                       const double *__restrict__ Pbuf, const double *__restrict__ Cbuf,
                                                       int64_t cs, int64_t ntiles, int64_t nitems, int64_t rows,
                                                       int skip) {
    constexpr int G = KMAX / 4;
    constexpr int BAND = KMAX * 16;                 // doubles per band
    constexpr int PER = BAND / 2 / kBlock;          // 16-byte multiplier pieces per thread per band
    static_assert(PER >= 1 && BAND / 2 % kBlock == 0, "band staging");
    __shared__ __attribute__((aligned(16))) double sC[NB][BAND];
    __shared__ int64_t next_item;
    __shared__ int wsum[kBlock / 64];
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
        const int64_t cl = tile * 128 + wave * 32 + 2 * lc;   // this lane's column pair
        const bool in = cl < g.ncols;                         // cl even, ld even: cl + 1 < ld
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
        // per-chain liveness: the even (odd) chain runs if any even (odd) column of the wave is live
        bool le = false, lo = false;
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            le = le || be[gq] != 0.0;
            lo = lo || bo[gq] != 0.0;
        }
        const bool run_e = !skip || __ballot(in && le) != 0, run_o = !skip || __ballot(in && lo && cl + 1 < g.ncols) != 0;
        int mine = (lk == 0 && ok) ? (cl + 1 < g.ncols ? 2 : 1) : 0;   // live doubles per row, pairs counted once
        for (int mask = 32; mask > 0; mask >>= 1) mine += __shfl_xor(mine, mask, 64);
        const bool wlive = mine > 0;                                   // wave-uniform
        if (lane == 0) wsum[wave] = mine;
        if (__syncthreads_count(wlive && lane == 0) == 0) continue;    // the whole tile is skipped
        if (threadIdx.x == 0)
            touched += (unsigned long long)(wsum[0] + wsum[1] + wsum[2] + wsum[3]) * (unsigned long long)(i1 - i0);
        const int nb = (int)((i1 - i0 + 15) / 16);
        // multiplier piece e of band s: slot q = e / 8, band rows 2 (e % 8) .. +1
        // (zeros past np and past i1: A = -0 there, x + -0 == x)
        auto cload = [&](d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int e = threadIdx.x + u * kBlock;
                const int q = e >> 3, rr = 2 * (e & 7);
                const int64_t row = i0 + 16 * s + rr;
                d2 v = d2{0.0, 0.0};
                if (s < nb && q < np && row < i1) v = *(const d2 *)(Cbuf + (int64_t)q * cs + row);   // row + 1 < cs
                cr[u] = -v;
            }
        };
        auto cstore = [&](const d2 (&cr)[PER], int s) {
#pragma unroll
            for (int u = 0; u < PER; u++) *(d2 *)(&sC[s % NB][2 * (threadIdx.x + u * kBlock)]) = cr[u];
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
            d2 tn[4];
            if (s + 1 < nb) tload(tn, s + 1);
            __syncthreads();                  // band s is staged; ring slot (s - 1) % NB is free
            cstore(cn, s + NB - 1);
            cload(cn, s + NB);
            if (wlive) {
                d4 ae = d4{t[0].x, t[1].x, t[2].x, t[3].x};
                d4 ao = d4{t[0].y, t[1].y, t[2].y, t[3].y};
                const double *sa = &sC[s % NB][lk * 16 + lc];
                if (run_e && run_o) {
#pragma unroll
                    for (int gq = 0; gq < G; gq++) {
                        const double a = sa[gq * 64];
                        ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a, be[gq], ae, 0, 0, 0);
                        ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bo[gq], ao, 0, 0, 0);
                    }
                } else if (run_e) {
#pragma unroll
                    for (int gq = 0; gq < G; gq++) ae = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], be[gq], ae, 0, 0, 0);
                } else {
#pragma unroll
                    for (int gq = 0; gq < G; gq++) ao = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[gq * 64], bo[gq], ao, 0, 0, 0);
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

}  // namespace lpg

using namespace lpg;

__global__ void k_fill(double *x, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * 0x1.0p-53;
    }
}

// P_q[j] = 0 for the slack block and the padding (the skipped columns),
// except every `every`-th slack column (0: none), which stays live: the
// slacks that left the basis, scattered over the block as in a real solve
__global__ void k_zero_cols(double *P, int64_t ld, int64_t j0, int64_t j1, int k, int64_t every) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)k * ld; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e % ld;
        if (j >= j0 && !(every > 0 && j < j1 && (j - j0) % every == 0)) P[e] = 0.0;
    }
}

__global__ void k_cmp(const double *a, const double *b, int64_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += __double_as_longlong(a[i]) != __double_as_longlong(b[i]);
    if (c) atomicAdd(bad, c);
}

struct Lab {
    Geo g{};
    Defer D{};
    DevState *st = nullptr;
    double *T = nullptr, *T0 = nullptr, *Tref = nullptr;
    int64_t n = 0;
    int K = 32;
    unsigned long long *bad = nullptr;
    hipEvent_t e0, e1;

    void reset_state() {
        DevState h{};
        h.npend = K;
        h.fwork = 0;
        CHK(hipMemcpy(st, &h, sizeof h, hipMemcpyHostToDevice));
    }
};

typedef void (*LaunchFn)(Lab &L);

static double run(Lab &L, LaunchFn fn, const char *name, bool check, int reps) {
    if (check) {
        CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
        L.reset_state();
        fn(L);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
        CHK(hipMemset(L.bad, 0, 8));
        hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, L.T, L.Tref, L.n, L.bad);
        unsigned long long nb = 0;
        CHK(hipMemcpy(&nb, L.bad, 8, hipMemcpyDeviceToHost));
        if (nb) {
            printf("%-34s MISMATCH: %llu doubles differ from the engine flush\n", name, nb);
            return -1;
        }
    }
    double best = 1e30, sum = 0;
    for (int r = 0; r < reps; r++) {
        L.reset_state();
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
    printf("%-34s K=%d  best %.3f ms  mean %.3f ms  touched %.3f GB  %.0f GB/s (best)\n", name, L.K, best, sum / reps,
           bytes / 1e9, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
    return best;
}

static int g_variant = 8;
static void fn_engine(Lab &L) {
    Launch la{nullptr};
    if (launch_flush(la, L.g, L.st, L.D, L.K, 1, g_variant)) {
        printf("launch_flush failed\n");
        exit(1);
    }
}

template <int KMAX, int SR, int NSUB, int PERCU>
static void fn_r(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 63) / 64;
    const int64_t nitems = ntiles * ((L.g.nloc + SR - 1) / SR);
    const int64_t nblocks = std::min<int64_t>(nitems, 256 * PERCU);
    hipLaunchKernelGGL((k_flushr<KMAX, SR, NSUB>), dim3((unsigned)nblocks), dim3(kBlock), 0, 0, L.g.T, L.g, L.st,
                       L.D.Pbuf, L.D.Cbuf, L.D.cs, ntiles, nitems, 1);
}

template <int KMAX, int R, int NB, int LB, int PERCU>
static void fn_w(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128;
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    const int64_t nblocks = std::min<int64_t>(nitems, 256 * PERCU);
    hipLaunchKernelGGL((k_flushw<KMAX, NB, LB>), dim3((unsigned)nblocks), dim3(kBlock), 0, 0, L.g.T, L.g, L.st,
                       L.D.Pbuf, L.D.Cbuf, L.D.cs, ntiles, nitems, (int64_t)R, 1);
}

template <int KMAX, int R, int NB, int LB, int PERCU>
static void fn_w2(Lab &L) {
    const int64_t ntiles = (L.g.ncols + 127) / 128;
    const int64_t nitems = ntiles * ((L.g.nloc + R - 1) / R);
    const int64_t nblocks = std::min<int64_t>(nitems, 256 * PERCU);
    hipLaunchKernelGGL((k_flushw2<KMAX, NB, LB>), dim3((unsigned)nblocks), dim3(kBlock), 0, 0, L.g.T, L.g, L.st,
                       L.D.Pbuf, L.D.Cbuf, L.D.cs, ntiles, nitems, (int64_t)R, 1);
}

int main(int argc, char **argv) {
    Lab L;
    L.K = argc > 1 ? atoi(argv[1]) : 32;
    const int64_t m = argc > 2 ? atoll(argv[2]) : 16384, nstruct = 2 * m;
    const int64_t ncols = nstruct + m + 1, ld = (ncols + 63) / 64 * 64;
    L.n = m * ld;
    CHK(hipMalloc(&L.T, L.n * 8));
    CHK(hipMalloc(&L.T0, L.n * 8));
    CHK(hipMalloc(&L.Tref, L.n * 8));
    CHK(hipMalloc(&L.st, sizeof(DevState)));
    CHK(hipMalloc(&L.bad, 8));
    double *Pbuf, *Cbuf;
    int64_t *rq;
    const int64_t cs = (m + 63) / 64 * 64;
    const int SL = 128;                                  // slots (blocks up to 128 pivots)
    CHK(hipMalloc(&Pbuf, (size_t)SL * ld * 8));
    CHK(hipMalloc(&Cbuf, (size_t)SL * cs * 8));
    CHK(hipMalloc(&rq, SL * 8));
    CHK(hipMemset(rq, 0xff, SL * 8));                 // -1: no pivot row of the block is local
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, L.T0, L.n, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, Pbuf, (int64_t)SL * ld, 2ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, Cbuf, (int64_t)SL * cs, 3ull);
    const int64_t every = getenv("LAB_SCATTER") ? atoll(getenv("LAB_SCATTER")) : 0;
    hipLaunchKernelGGL(k_zero_cols, dim3(1024), dim3(256), 0, 0, Pbuf, ld, nstruct + 1, ncols, SL, every);
    CHK(hipDeviceSynchronize());
    L.g.T = L.T;
    L.g.ld = ld;
    L.g.nloc = m;
    L.g.nobj = 1;
    L.g.ncols = ncols;
    L.g.nact = ncols - 1;
    L.g.m = m;
    L.D.Pbuf = Pbuf;
    L.D.Cbuf = Cbuf;
    L.D.cs = cs;
    L.D.rq = rq;
    CHK(hipMalloc(&L.D.mul, (size_t)LPG_DEFER_MAX * LPG_DEFER_MAX * 8));
    L.D.on = 1;
    CHK(hipEventCreate(&L.e0));
    CHK(hipEventCreate(&L.e1));
    printf("flush lab: %lld rows x %lld cols (ld %lld), K=%d, P zero for columns > %lld except every %lld-th\n",
           (long long)m, (long long)ncols, (long long)ld, L.K, (long long)nstruct, (long long)every);
    const int reps = 5;
    const char *only = getenv("LAB_ONLY");
    auto want = [&](const char *nm) { return !only || strstr(nm, only); };
    if (L.K > 64) {   // beyond the engine's blocks: timing only (no reference flush to compare with)
#define WB(KM, R, NB, LB, PC)                                                                      \
        if (L.K <= KM && want("w<" #KM "," #R "," #NB "," #LB "," #PC ">"))                        \
            run(L, fn_w<KM, R, NB, LB, PC>, "w<" #KM "," #R "," #NB "," #LB "," #PC ">", false, reps);
        WB(96, 512, 2, 2, 2) WB(96, 512, 2, 1, 1) WB(128, 512, 2, 1, 1) WB(128, 512, 2, 2, 2) WB(128, 1024, 2, 1, 1)
        return 0;
    }
    // reference result: the engine's default flush
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    L.reset_state();
    fn_engine(L);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
    for (int v : {8, 19, 20, 14, 16}) {
        g_variant = v;
        char nm[64];
        snprintf(nm, sizeof nm, "engine variant %d", v);
        if (want(nm)) run(L, fn_engine, nm, true, reps);
    }
#define R(KM, SR, NS, PC)                                                       \
    if (L.K <= KM && want("r<" #KM "," #SR "," #NS "," #PC ">"))               \
        run(L, fn_r<KM, SR, NS, PC>, "r<" #KM "," #SR "," #NS "," #PC ">", true, reps);
    if (L.K <= 32) {
        R(32, 64, 1, 4) R(32, 64, 2, 4) R(32, 128, 2, 4) R(32, 64, 4, 4) R(32, 128, 4, 2)
    } else {
        R(64, 64, 1, 4) R(64, 64, 2, 4) R(64, 32, 2, 6) R(64, 64, 4, 4) R(64, 32, 1, 6)
    }
#define W(KM, R, NB, LB, PC)                                                            \
    if (L.K <= KM && want("w<" #KM "," #R "," #NB "," #LB "," #PC ">"))                  \
        run(L, fn_w<KM, R, NB, LB, PC>, "w<" #KM "," #R "," #NB "," #LB "," #PC ">", true, reps);
    if (L.K <= 32) {
        W(32, 512, 2, 3, 3) W(32, 512, 3, 3, 3) W(32, 256, 2, 3, 3) W(32, 1024, 2, 3, 3) W(32, 512, 2, 4, 4)
    } else {
        W(64, 512, 2, 2, 2) W(64, 512, 3, 2, 2) W(64, 256, 2, 2, 2) W(64, 1024, 2, 2, 2)
    }
    if (L.K > 32 && want("w2<64,512,2,2,2>")) run(L, fn_w2<64, 512, 2, 2, 2>, "w2<64,512,2,2,2>", true, reps);
    return 0;
}
