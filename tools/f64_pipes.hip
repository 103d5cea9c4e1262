// Round 6 lab: do the f64 matrix pipe and the f64 VALU run at the same time
// on gfx950? The block pass (k_flushw) is all v_mfma_f64_16x16x4_f64 (MFMA
// busy 0.70-0.79 of its cycles); an element's chain
// fma(-C_q[i], P_q[j], x) is also exactly v_fma_f64, so if the two pipes add,
// a share of each tile's columns could run on the VALU bitwise unchanged.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/f64_pipes tools/f64_pipes.hip
//   tools/f64_pipes [iters]
//
// Every block: 512 threads = 8 waves = 2 per SIMD. Modes:
//   M   all waves MFMA (4 independent 16x16x4 chains per wave)
//   V   all waves v_fma_f64 (16 independent chains per lane)
//   MV  waves 0-3 MFMA, waves 4-7 VALU (one of each per SIMD)
//   I/r every wave interleaves: 4 MFMAs then r*4 v_fma_f64, repeated
//   Mc  all waves MFMA, c = 1, 2, 4 independent chains per wave
//   band/...  k_band: k_flushw's per-band MFMA loop without HBM (see there)
// Prints TFLOP/s per mode (MFMA 2048 flops per instruction per wave, VALU 128).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

template <int MODE, int R>
__global__ __launch_bounds__(512, 1) void k_pipes(double *out, int iters, double s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const double a = s * (1 + lane), b = s * 0.5;
    d4 acc[4];
    double v[16];
#pragma unroll
    for (int u = 0; u < 4; u++) acc[u] = d4{s, s, s, s};
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = s * u;
    const bool do_m = MODE == 0 || (MODE == 2 && wave < 4) || MODE == 3;
    const bool do_v = MODE == 1 || (MODE == 2 && wave >= 4) || MODE == 3;
    if (MODE == 3) {
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
#pragma unroll
                for (int k = 0; k < R; k++)
#pragma unroll
                    for (int w = 0; w < 4; w++) v[4 * (k & 3) + w] = __builtin_fma(a, b + w, v[4 * (k & 3) + w]);
            }
        }
    } else if (MODE >= 4) {
        // MODE 4 + c: c = 0, 1, 2 -> 1, 2, 4 independent MFMA chains per wave,
        // 4 MFMAs per iteration either way
        constexpr int NC = MODE >= 4 ? 1 << (MODE - 4) : 1;
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int u = 0; u < 4; u++) acc[u % NC] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u % NC], 0, 0, 0);
        }
    } else {
        if (do_m) {
            for (int it = 0; it < iters; it++) {
#pragma unroll
                for (int u = 0; u < 4; u++) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
            }
        }
        if (do_v) {
            // 16 v_fma_f64 per iteration per lane = 4 cycles each at 16 lanes/clk:
            // 64 cycles, one MFMA's worth; x4 to match the MFMA loop's 4 MFMAs
            for (int it = 0; it < iters; it++) {
#pragma unroll
                for (int rep = 0; rep < 4; rep++)
#pragma unroll
                    for (int u = 0; u < 16; u++) v[u] = __builtin_fma(a, b + u, v[u]);
            }
        }
    }
    double r = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) r += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
#pragma unroll
    for (int u = 0; u < 16; u++) r += v[u];
    out[blockIdx.x * 512 + threadIdx.x] = r;
}


// k_band<VAR>: the block pass's inner loop without HBM (k_flushw's matrix side):
// per 16-row band, 24 k-steps x 2 chains (even / odd columns) with B fragments
// be/bo in registers. VAR bits: 1 = __syncthreads per band, 2 = A operands read
// from an LDS ring (one ds_read_b64 per k-step, one pair ahead, as k_flushw),
// else from registers; 4 = no sched_barrier around the MFMA groups; 8 = A read as
// one 16-byte LDS read per pair of k-steps (ring laid out [pair][lane][2]).
template <int VAR>
__global__ __launch_bounds__(512, 1) void k_band(double *out, int nbands, double s) {
    constexpr int G = 24;
    __shared__ __attribute__((aligned(16))) double sC[2][96 * 16];
    const int lane = threadIdx.x & 63;
    const int lc = lane & 15, lk = lane >> 4;
    for (int e = threadIdx.x; e < 2 * 96 * 16; e += 512) (&sC[0][0])[e] = s * (e & 31);
    __syncthreads();
    double be[G], bo[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
        be[g] = s * (g + lane);
        bo[g] = s * (g - lane);
    }
    double res = 0.0;
    for (int b = 0; b < nbands; b++) {
        if (VAR & 1) __syncthreads();
        d4 ae = d4{res, s, s, s}, ao = d4{s, res, s, s};
        if (VAR & 2) {
            if (VAR & 8) {
                const d2 *sp = (const d2 *)&sC[b & 1][0] + lane;
                d2 a = sp[0];
#pragma unroll
                for (int gq = 0; gq < G; gq += 2) {
                    d2 n = d2{0.0, 0.0};
                    if (gq + 2 < G) n = sp[(gq / 2 + 1) * 64];
                    if (!(VAR & 4)) __builtin_amdgcn_sched_barrier(0);
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, be[gq], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, bo[gq], ao, 0, 0, 0);
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, be[gq + 1], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, bo[gq + 1], ao, 0, 0, 0);
                    if (!(VAR & 4)) __builtin_amdgcn_sched_barrier(0);
                    a = n;
                }
            } else {
                const double *sa = &sC[b & 1][lk * 16 + lc];
                double a0 = sa[0], a1 = sa[64];
#pragma unroll
                for (int gq = 0; gq < G; gq += 2) {
                    double n0 = 0.0, n1 = 0.0;
                    if (gq + 2 < G) {
                        n0 = sa[(gq + 2) * 64];
                        n1 = sa[(gq + 3) * 64];
                    }
                    if (!(VAR & 4)) __builtin_amdgcn_sched_barrier(0);
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, be[gq], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bo[gq], ao, 0, 0, 0);
                    ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, be[gq + 1], ae, 0, 0, 0);
                    ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bo[gq + 1], ao, 0, 0, 0);
                    if (!(VAR & 4)) __builtin_amdgcn_sched_barrier(0);
                    a0 = n0;
                    a1 = n1;
                }
            }
        } else {
            const double a0 = s * lane, a1 = s * lk;
#pragma unroll
            for (int gq = 0; gq < G; gq += 2) {
                ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, be[gq], ae, 0, 0, 0);
                ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bo[gq], ao, 0, 0, 0);
                ae = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, be[gq + 1], ae, 0, 0, 0);
                ao = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bo[gq + 1], ao, 0, 0, 0);
            }
        }
        res += ae[0] + ae[1] + ae[2] + ae[3] + ao[0] + ao[1] + ao[2] + ao[3];
    }
    out[blockIdx.x * 512 + threadIdx.x] = res;
}

template <int VAR>
static void run_band(const char *name, double *out, int grid, int nbands) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_band<VAR>), dim3(grid), dim3(512), 0, 0, out, nbands, 1e-3);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_band<VAR>), dim3(grid), dim3(512), 0, 0, out, nbands, 1e-3);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double mf = (double)grid * 8 * nbands * 48 * 2048;
    printf("band/%-9s grid %4d  %8.3f ms  mfma %6.1f TF\n", name, grid, best, mf / best / 1e9);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

template <int MODE, int R>
static void run(const char *name, double *out, int grid, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_pipes<MODE, R>), dim3(grid), dim3(512), 0, 0, out, iters, 1e-3);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((k_pipes<MODE, R>), dim3(grid), dim3(512), 0, 0, out, iters, 1e-3);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    // flops per wave per iteration
    double mf = 0, vf = 0;
    const double waves = (double)grid * 8;
    if (MODE == 0) mf = waves * 4 * 2048;
    if (MODE == 1) vf = waves * 64 * 64 * 2;
    if (MODE == 2) { mf = waves / 2 * 4 * 2048; vf = waves / 2 * 64 * 64 * 2; }
    if (MODE == 3) { mf = waves * 4 * 2048; vf = waves * 4 * R * 4 * 64 * 2; }
    if (MODE >= 4) mf = waves * 4 * 2048;
    mf *= iters;
    vf *= iters;
    printf("%-6s grid %4d  %8.3f ms  mfma %6.1f TF  valu %6.1f TF  total %6.1f TF\n", name, grid, best,
           mf / best / 1e9, vf / best / 1e9, (mf + vf) / best / 1e9);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int grid = p.multiProcessorCount;
    printf("%s, %d CUs, iters %d\n", p.gcnArchName, grid, iters);
    double *out;
    CHECK(hipMalloc(&out, (size_t)grid * 2 * 512 * sizeof(double)));
    for (int g = grid; g <= 2 * grid; g += grid) {
        run<0, 0>("M", out, g, iters);
        run<1, 0>("V", out, g, iters);
        run<2, 0>("MV", out, g, iters);
        run<3, 1>("I/1", out, g, iters);
        run<3, 2>("I/2", out, g, iters);
        run<3, 4>("I/4", out, g, iters);
        run<4, 0>("M1ch", out, g, iters);
        run<5, 0>("M2ch", out, g, iters);
        run<6, 0>("M4ch", out, g, iters);
    }
    const int nb = 4 * iters / 48;
    run_band<0>("reg", out, grid, nb);
    run_band<1>("reg+bar", out, grid, nb);
    run_band<2>("lds", out, grid, nb);
    run_band<3>("lds+bar", out, grid, nb);
    run_band<6>("lds-sb", out, grid, nb);
    run_band<7>("lds-sb+bar", out, grid, nb);
    run_band<10>("lds128", out, grid, nb);
    run_band<11>("lds128+bar", out, grid, nb);
    run_band<15>("lds128-sb+b", out, grid, nb);
    CHECK(hipFree(out));
    return 0;
}
