// mfma_rate2.hip — what holds the block pass's f64 MFMA loop at ~47 TFLOP/s
// when the pipe reaches 72-75 with constant operands (mfma_rate.hip)? Every
// CU busy, W waves per SIMD, v_mfma_f64_16x16x4_f64 chains of 32 steps per
// "band" (the pass's shape at 128 slots) with:
//   NACC independent accumulators per wave (1 = k_flushv, 2 = k_flushw),
//   B from a per-lane array of 32 doubles (the pass's P fragments) or constant,
//   A from LDS (one ds_read_b64 per step, the pass's multipliers) or constant.
// Tools only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int NACC, bool BARR, bool ALDS>
__global__ void k_band(double *out, int bands, double a0, double b0) {
    __shared__ double sA[32 * 64 * 2];
    for (int e = threadIdx.x; e < 32 * 64 * 2; e += blockDim.x) sA[e] = a0 + e * 1e-9;
    __syncthreads();
    double b[BARR ? 32 : 1];
#pragma unroll
    for (int k = 0; k < (BARR ? 32 : 1); k++) b[k] = b0 + threadIdx.x * 1e-7 + k;
    d4 acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; k++) acc[k] = d4{threadIdx.x * 1.0, 1.0, 2.0, 3.0};
    const int lane = threadIdx.x & 63;
    for (int s = 0; s < bands; s++) {
        const double *sa = &sA[(s & 1) * 2048 + lane];
#pragma unroll
        for (int g = 0; g < 32; g++) {
            const double a = ALDS ? sa[g * 64] : a0;
#pragma unroll
            for (int k = 0; k < NACC; k++)
                acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[BARR ? g : 0], acc[k], 0, 0, 0);
        }
    }
    double r = 0;
#pragma unroll
    for (int k = 0; k < NACC; k++) r += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NACC, bool BARR, bool ALDS>
static void run(const char *name, double *out, int cus, int w) {
    const int bands = 400;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_band<NACC, BARR, ALDS>), dim3(cus), dim3(256 * w), 0, 0, out, 4, 0.5, 0.25);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_band<NACC, BARR, ALDS>), dim3(cus), dim3(256 * w), 0, 0, out, bands, 0.5, 0.25);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double flops = 2.0 * 1024 * 32 * NACC * (double)bands * 4 * w * cus;   // per MFMA 16x16x4 = 1024 FMA
    printf("%-34s %d waves/SIMD: %.1f TFLOP/s\n", name, w, flops / (ms * 1e-3) / 1e12);
}

// MFMA waves (0-3) and HBM read-modify-write waves (4-7, MEM) in the same
// blocks: does the matrix-core rate hold while the memory stream runs?
template <bool MEM>
__global__ __launch_bounds__(512) void k_mix(double *out, double *buf, int64_t per_block, int bands, double *gbps) {
    __shared__ double sA[2 * 2048];
    __shared__ int done;
    if (threadIdx.x == 0) done = 0;
    for (int e = threadIdx.x; e < 4096; e += blockDim.x) sA[e] = 0.5 + e * 1e-9;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ double msum;
    if (threadIdx.x == 0) msum = 0;
    __syncthreads();
    if (wave < 4) {
        double b[32];
#pragma unroll
        for (int k = 0; k < 32; k++) b[k] = 0.25 + threadIdx.x * 1e-7 + k;
        d4 acc = d4{threadIdx.x * 1.0, 1.0, 2.0, 3.0};
        for (int s = 0; s < bands; s++) {
            const double *sa = &sA[(s & 1) * 2048 + lane];
#pragma unroll
            for (int g = 0; g < 32; g++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sa[g * 64], b[g], acc, 0, 0, 0);
        }
        out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
        if (lane == 0) __hip_atomic_fetch_add(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MEM) {   // 64 KB chunks (4 x 16 B per thread), the flag checked between chunks
        double *p = buf + (int64_t)blockIdx.x * per_block;
        const int t = threadIdx.x - 256;
        double moved = 0;
        for (int64_t c0 = 0; __hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4;
             c0 = (c0 + 8192) % per_block) {
            d2 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load((const d2 *)(p + c0 + 2 * (t + 256 * u)));
#pragma unroll
            for (int u = 0; u < 4; u++) {
                v[u].x = v[u].x * 1.0000001;
                v[u].y = v[u].y * 1.0000001;
                __builtin_nontemporal_store(v[u], (d2 *)(p + c0 + 2 * (t + 256 * u)));
            }
            moved += 2 * 4 * 16;   // bytes read + written by this thread
        }
        atomicAdd(&msum, moved);
    }
    __syncthreads();
    if (threadIdx.x == 0) gbps[blockIdx.x] = msum;
}

template <bool MEM>
static void run_mix(const char *name, double *out, double *buf, int64_t per_block, double *gb, int cus) {
    const int bands = 400;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_mix<MEM>), dim3(cus), dim3(512), 0, 0, out, buf, per_block, 4, gb);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_mix<MEM>), dim3(cus), dim3(512), 0, 0, out, buf, per_block, bands, gb);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    double *h = (double *)malloc(cus * 8), bytes = 0;
    CHK(hipMemcpy(h, gb, cus * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < cus; i++) bytes += h[i];
    free(h);
    const double flops = 2.0 * 1024 * 32 * (double)bands * 4 * cus;
    printf("%-34s MFMA %.1f TFLOP/s, HBM read+write %.0f GB/s (%.3f ms)\n", name, flops / (ms * 1e-3) / 1e12,
           bytes / (ms * 1e-3) / 1e9, ms);
}

int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double *out;
    CHK(hipMalloc(&out, (size_t)cus * 1024 * 8));
    for (int w = 1; w <= 4; w *= 2) {
        run<4, false, false>("4 acc, B const, A const", out, cus, w);
        run<2, false, false>("2 acc, B const, A const", out, cus, w);
        run<1, false, false>("1 acc, B const, A const", out, cus, w);
        run<2, true, false>("2 acc, B array, A const", out, cus, w);
        run<1, true, false>("1 acc, B array, A const", out, cus, w);
        run<2, true, true>("2 acc, B array, A LDS (k_flushw)", out, cus, w);
        run<1, true, true>("1 acc, B array, A LDS (k_flushv)", out, cus, w);
        run<4, true, true>("4 acc, B array, A LDS", out, cus, w);
    }
    double *buf, *gb;
    const int64_t per_block = ((int64_t)24 << 20) / 8;   // 24 MB per block: 6 GB in all, well past the caches
    CHK(hipMalloc(&buf, (size_t)per_block * cus * 8));
    CHK(hipMalloc(&gb, (size_t)cus * 8));
    CHK(hipMemset(buf, 0, (size_t)per_block * cus * 8));
    run_mix<false>("mix: MFMA waves alone", out, buf, per_block, gb, cus);
    run_mix<true>("mix: MFMA waves + HBM RMW waves", out, buf, per_block, gb, cus);
    run_mix<false>("mix: MFMA waves alone", out, buf, per_block, gb, cus);
    run_mix<true>("mix: MFMA waves + HBM RMW waves", out, buf, per_block, gb, cus);
    return 0;
}
