// hbm_calib2.hip — in-place read-modify-write stream under different load /
// store cache policies and batch depths (tools only; decides k_update's
// memory instructions). 3.2 GB buffer (32-bit buffer offsets), 1-D grid-stride,
// x = fma(-c, p, x) on 16 B per lane, U loads in flight before the stores.
// Policies use raw buffer loads/stores with the aux cache bits
// (gfx950: bit0 sc0, bit1 nt, bit4 sc1; cdna_hip_programming.md G16 R1).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void k_rmw(double *base, unsigned n16, double c) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0xffffffffu, 0x00020000);
    const d2 p = {0.5, 0.25};
    unsigned i = blockIdx.x * 256u + threadIdx.x;
    const unsigned st = gridDim.x * 256u;
    for (; i + (U - 1) * st < n16; i += U * st) {
        v4i t[U];
#pragma unroll
        for (int u = 0; u < U; u++) t[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (i + u * st) * 16u, 0, LAUX);
#pragma unroll
        for (int u = 0; u < U; u++) {
            d2 x = __builtin_bit_cast(d2, t[u]);
            x.x = fma(-c, p.x, x.x);
            x.y = fma(-c, p.y, x.y);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, x), rs, (i + u * st) * 16u, 0, SAUX);
        }
    }
}

template <int U, int LAUX, int SAUX>
static float run(double *A, unsigned n16, int grid, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_rmw<U, LAUX, SAUX>), dim3(grid), dim3(256), 0, 0, A, n16, 1e-3);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_rmw<U, LAUX, SAUX>), dim3(grid), dim3(256), 0, 0, A, n16, 1e-3);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

#define RUN(U, L, S, name)                                                                                  \
    do {                                                                                                    \
        for (int g = 0; g < 3; g++) {                                                                       \
            float ms = run<U, L, S>(A, n16, grids[g], reps);                                                \
            printf("%-22s U=%2d grid %5d : %7.1f GB/s\n", name, U, grids[g], 2.0 * bytes / ms / 1e6);        \
        }                                                                                                   \
    } while (0)

int main(int argc, char **argv) {
    const size_t bytes = (size_t)3200 << 20;   // 3.2 GiB: 32-bit buffer offsets
    const unsigned n16 = (unsigned)(bytes / 16);
    double *A;
    CHK(hipMalloc(&A, bytes));
    CHK(hipMemset(A, 0, bytes));
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    int grids[] = {2048, 4096, 8192};
    RUN(8, 0, 0, "plain/plain");
    RUN(8, 2, 2, "nt/nt");
    RUN(8, 0, 16, "plain/sc1");
    RUN(8, 2, 16, "nt/sc1");
    RUN(8, 2, 18, "nt/sc1+nt");
    RUN(8, 0, 17, "plain/sc0+sc1");
    RUN(8, 2, 3, "nt/sc0+nt");
    RUN(4, 2, 2, "nt/nt");
    RUN(16, 2, 2, "nt/nt");
    RUN(16, 2, 16, "nt/sc1");
    return 0;
}
