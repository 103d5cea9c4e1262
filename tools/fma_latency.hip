// fma_latency.hip — dependent-issue latency of v_fma_f64 on gfx950 (tools only):
// one wave per SIMD runs N dependent fmas (1, 2, 4 or 8 independent chains
// interleaved per lane); cycles per chain step from s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int CH>
__global__ void k_chain(double *out, long long *cyc, int n, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = fma(a, x[c], b);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the same through an LDS operand per step (the pivot chains' form)
__global__ void k_chain_lds(double *out, long long *cyc, int n, double b) {
    __shared__ double sl[256 * 8];
    for (int i = threadIdx.x; i < 256 * 8; i += blockDim.x) sl[i] = 1.0 + 1e-9 * i;
    __syncthreads();
    double x = threadIdx.x;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = sl[threadIdx.x * 8 + j];
#pragma unroll
        for (int j = 0; j < 8; j++) x = fma(-v[j], b, x);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double *out; long long *cyc;
    CHK(hipMalloc(&out, 1 << 24)); CHK(hipMalloc(&cyc, 1 << 16));
    const int n = 4096;
    long long h[64];
    for (int threads : {64, 256, 512, 1024}) {
#define RUN(CH)                                                                                       \
        hipLaunchKernelGGL(k_chain<CH>, dim3(1), dim3(threads), 0, 0, out, cyc, n, 0.999, 1e-3);       \
        CHK(hipDeviceSynchronize());                                                                  \
        hipLaunchKernelGGL(k_chain<CH>, dim3(1), dim3(threads), 0, 0, out, cyc, n, 0.999, 1e-3);       \
        CHK(hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost));                                             \
        printf("threads %4d (waves/SIMD %d) chains/lane %d: %6.1f cycles per step\n", threads, threads / 256 ? threads / 256 : 1, CH, (double)h[0] / n);
        RUN(1) RUN(2) RUN(4) RUN(8)
    }
    hipLaunchKernelGGL(k_chain_lds, dim3(1), dim3(256), 0, 0, out, cyc, n, 0.999);
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_chain_lds, dim3(1), dim3(256), 0, 0, out, cyc, n, 0.999);
    CHK(hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost));
    printf("LDS operand chain, 1 wave/SIMD: %6.1f cycles per step\n", (double)h[0] / n);
    int clk = 0; CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    printf("s_memtime counts shader clocks? clockRate attribute %d kHz\n", clk);
    return 0;
}
