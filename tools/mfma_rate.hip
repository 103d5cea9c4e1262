// mfma_rate.hip — issue rate of v_mfma_f64_16x16x4_f64 and v_fma_f64 on one
// MI355X (all CUs busy, W waves per SIMD, 4 independent accumulators). Tools only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int NACC>
__global__ void k_mfma(double *out, int iters, double a, double b) {
    d4 acc[NACC];
    for (int k = 0; k < NACC; k++) acc[k] = d4{threadIdx.x * 1.0, 1.0, 2.0, 3.0};
    double av = a + threadIdx.x, bv = b - threadIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < NACC; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[k], 0, 0, 0);
    }
    double s = 0;
    for (int k = 0; k < NACC; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma(double *out, int iters, double a, double b) {
    double x0 = threadIdx.x, x1 = 1, x2 = 2, x3 = 3, x4 = 4, x5 = 5, x6 = 6, x7 = 7;
    for (int it = 0; it < iters; it++) {
        x0 = fma(a, x0, b); x1 = fma(a, x1, b); x2 = fma(a, x2, b); x3 = fma(a, x3, b);
        x4 = fma(a, x4, b); x5 = fma(a, x5, b); x6 = fma(a, x6, b); x7 = fma(a, x7, b);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

// 16 independent fma chains per lane (does the VALU reach its f64 peak?)
__global__ void k_fma16(double *out, int iters, double a, double b) {
    double x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = threadIdx.x + k;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 16; k++) x[k] = fma(a, x[k], b);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA and VALU waves side by side on every SIMD: 512-thread blocks, waves 0-3
// (one per SIMD) run MFMA chains, waves 4-7 run v_fma_f64 chains. `vit`
// scales the VALU waves' work so both halves take about as long.
__global__ __launch_bounds__(512) void k_mixed(double *out, int iters, int vit, double a, double b) {
    const int w = threadIdx.x >> 6;
    double s = 0;
    if (w < 4) {
        d4 acc[4];
        for (int k = 0; k < 4; k++) acc[k] = d4{threadIdx.x * 1.0, 1.0, 2.0, 3.0};
        double av = a + threadIdx.x, bv = b - threadIdx.x;
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[k], 0, 0, 0);
        }
        for (int k = 0; k < 4; k++) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    } else {
        double x[16];
#pragma unroll
        for (int k = 0; k < 16; k++) x[k] = threadIdx.x + k;
        for (int it = 0; it < vit; it++) {
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] = fma(a, x[k], b);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) s += x[k];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double *out;
    CHK(hipMalloc(&out, 256 * 8 * 1024 * 8));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    const int iters = 4096;
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps;          // 256 threads = 4 waves per block, one per SIMD
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_mfma<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 0.999);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            const double mfmas = (double)blocks * 4 * iters * 4;   // waves x iters x NACC
            if (rep) printf("mfma_f64_16x16x4: %d waves/SIMD: %.1f TFLOP/s, %.1f ns per MFMA per SIMD\n", wps,
                            mfmas * 2048 / (ms * 1e-3) / 1e12, ms * 1e6 / (mfmas / 1024));
        }
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 0.999);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            const double fmas = (double)blocks * 256 * iters * 8;
            if (rep) printf("v_fma_f64:        %d waves/SIMD: %.1f TFLOP/s\n", wps, fmas * 2 / (ms * 1e-3) / 1e12);
        }
    }
    // VALU with 16 independent chains
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps;
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_fma16, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001, 0.999);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            const double fmas = (double)blocks * 256 * iters * 16;
            if (rep) printf("v_fma_f64 x16:    %d waves/SIMD: %.1f TFLOP/s\n", wps, fmas * 2 / (ms * 1e-3) / 1e12);
        }
    }
    // MFMA + VALU waves together; vit = VALU iterations (16 fmas each) per MFMA iteration count
    for (int vit : {0, 512, 1024, 2048, 4096, 8192}) {
        const int blocks = 256 * 2;
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_mixed, dim3(blocks), dim3(512), 0, 0, out, iters, vit, 1.0000001, 0.999);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
            const double mf = (double)blocks * 4 * iters * 4 * 2048;       // MFMA flops
            const double vf = (double)blocks * 256 * (double)vit * 16 * 2;  // VALU flops
            if (rep) printf("mixed (1 MFMA + 1 VALU wave/SIMD, vit %5d): %.3f ms  MFMA %.1f + VALU %.1f = %.1f TFLOP/s\n",
                            vit, ms, mf / (ms * 1e-3) / 1e12, vf / (ms * 1e-3) / 1e12, (mf + vf) / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
