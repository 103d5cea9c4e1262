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
    return 0;
}
