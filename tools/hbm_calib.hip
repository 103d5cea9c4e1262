// hbm_calib.hip — HBM ceilings for the access patterns of k_update (tools only).
//
// On one buffer of the config-3 tableau size (16385 x 49216 fp64 = 6.45 GB):
//   read      sum of every element (16 B/lane, grid-stride)
//   write     fill
//   copy      A -> B (two buffers)
//   rmw1d     x = fma(-c, p, x) in place, contiguous 1-D grid-stride
//   rmw1d_nt  same with non-temporal loads/stores
//   rmw2d     x = fma(-c[i], p[j], x) in place with k_update's 2-D tiling
//             (4 KB column tile x 64-row strip per block, row pitch ld)
// Each is timed with hipEvents over several launches; prints GB/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_read(const d2 *__restrict__ a, size_t n2, double *out) {
    d2 acc = {0, 0};
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) acc += a[i];
    if (acc.x == 12345.678) out[0] = acc.y;   // keep the loads alive
}
__global__ void k_write(d2 *__restrict__ a, size_t n2) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) a[i] = d2{1.0, 2.0};
}
__global__ void k_copy(const d2 *__restrict__ a, d2 *__restrict__ b, size_t n2) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
template <bool NT>
__global__ void k_rmw1d(d2 *__restrict__ a, size_t n2, double c) {
    const d2 p = {0.5, 0.25};
    size_t i = blockIdx.x * 256ull + threadIdx.x;
    const size_t st = (size_t)gridDim.x * 256;
    for (; i + 3 * st < n2; i += 4 * st) {
        d2 t[4];
#pragma unroll
        for (int u = 0; u < 4; u++) t[u] = NT ? __builtin_nontemporal_load(a + i + u * st) : a[i + u * st];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            t[u].x = fma(-c, p.x, t[u].x);
            t[u].y = fma(-c, p.y, t[u].y);
            if (NT) __builtin_nontemporal_store(t[u], a + i + u * st); else a[i + u * st] = t[u];
        }
    }
    for (; i < n2; i += st) { d2 t = a[i]; t.x = fma(-c, p.x, t.x); t.y = fma(-c, p.y, t.y); a[i] = t; }
}
__global__ void k_rmw2d(d2 *__restrict__ T, const double *__restrict__ C, const d2 *__restrict__ P, long ld2,
                        long nrows, long nvec, long ntiles) {
    const long tile = blockIdx.x % ntiles, strip = blockIdx.x / ntiles;
    const long cb = tile * 256 + threadIdx.x;
    if (cb >= nvec) return;
    const d2 p = P[cb];
    const long i0 = strip * 64, i1 = i0 + 64 < nrows ? i0 + 64 : nrows;
    long i = i0;
    for (; i + 8 <= i1; i += 8) {
        d2 t[8];
#pragma unroll
        for (int u = 0; u < 8; u++) t[u] = T[(i + u) * ld2 + cb];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const double c = -C[i + u];
            t[u].x = fma(c, p.x, t[u].x);
            t[u].y = fma(c, p.y, t[u].y);
            T[(i + u) * ld2 + cb] = t[u];
        }
    }
    for (; i < i1; i++) { d2 t = T[i * ld2 + cb]; t.x = fma(-C[i], p.x, t.x); t.y = fma(-C[i], p.y, t.y); T[i * ld2 + cb] = t; }
}

static float time_it(void (*f)(void *), void *arg, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    f(arg);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f(arg);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

struct Args { d2 *A, *B; double *C, *out; d2 *P; size_t n2; long ld2, nrows, nvec, ntiles; int grid; };
static Args G;
static void run_read(void *) { hipLaunchKernelGGL(k_read, dim3(G.grid), dim3(256), 0, 0, G.A, G.n2, G.out); }
static void run_write(void *) { hipLaunchKernelGGL(k_write, dim3(G.grid), dim3(256), 0, 0, G.A, G.n2); }
static void run_copy(void *) { hipLaunchKernelGGL(k_copy, dim3(G.grid), dim3(256), 0, 0, G.A, G.B, G.n2 / 2); }
static void run_rmw1d(void *) { hipLaunchKernelGGL(k_rmw1d<false>, dim3(G.grid), dim3(256), 0, 0, G.A, G.n2, 1e-3); }
static void run_rmw1d_nt(void *) { hipLaunchKernelGGL(k_rmw1d<true>, dim3(G.grid), dim3(256), 0, 0, G.A, G.n2, 1e-3); }
static void run_rmw2d(void *) {
    hipLaunchKernelGGL(k_rmw2d, dim3((unsigned)(G.ntiles * ((G.nrows + 63) / 64))), dim3(256), 0, 0, G.A, G.C, G.P,
                       G.ld2, G.nrows, G.nvec, G.ntiles);
}

int main(int argc, char **argv) {
    const long nrows = 16385, ncols = 49153, ld = 49216;
    G.ld2 = ld / 2; G.nrows = nrows; G.nvec = (ncols + 1) / 2; G.ntiles = (G.nvec + 255) / 256;
    G.n2 = (size_t)nrows * ld / 2;
    const size_t bytes = G.n2 * 16;
    CHK(hipMalloc(&G.A, bytes)); CHK(hipMalloc(&G.B, bytes / 2));
    CHK(hipMalloc(&G.C, nrows * 8)); CHK(hipMalloc(&G.P, ld * 8)); CHK(hipMalloc(&G.out, 8));
    CHK(hipMemset(G.A, 0, bytes)); CHK(hipMemset(G.C, 0, nrows * 8)); CHK(hipMemset(G.P, 0, ld * 8));
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    int grids[] = {1024, 2048, 4096, 8192};
    for (int gi = 0; gi < 4; gi++) {
        G.grid = grids[gi];
        float r = time_it(run_read, 0, reps), w = time_it(run_write, 0, reps), c = time_it(run_copy, 0, reps);
        float m1 = time_it(run_rmw1d, 0, reps), m1n = time_it(run_rmw1d_nt, 0, reps);
        printf("grid %5d  read %7.1f  write %7.1f  copy %7.1f  rmw1d %7.1f  rmw1d_nt %7.1f GB/s\n", G.grid,
               bytes / r / 1e6, bytes / w / 1e6, bytes / c / 1e6, 2 * bytes / m1 / 1e6, 2 * bytes / m1n / 1e6);
    }
    const double alg = 16.0 * nrows * ncols;
    float m2 = time_it(run_rmw2d, 0, reps);
    printf("rmw2d (k_update tiling, 4 KB x 64 rows)  %7.1f GB/s algorithmic, %.3f ms\n", alg / m2 / 1e6, m2);
    return 0;
}
