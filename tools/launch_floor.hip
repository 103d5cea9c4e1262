// launch_floor.hip — per-kernel floor of a dependent chain on one stream
// (eager and hipGraph), and the cost of an in-kernel grid barrier, to size
// the pivot loop's per-pivot overhead. Tools only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_empty() {}
__global__ void k_touch(double *a, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = a[i] * 1.0000001 + 1.0;
}
// dependent loads: each thread reads a value then uses it as an index
__global__ void k_chain(const int *idx, int *out, int hops) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int v = i;
    for (int h = 0; h < hops; h++) v = idx[v];
    out[i] = v;
}
// MODE 0: poll with an agent-scope acquire load; 1: poll with atomicAdd(0);
// 2: poll with a system-scope load; each with a release fence before arriving
// and an acquire fence after leaving. A data word written by every block
// before the barrier is checked by block 0 after it (stale reads counted).
// The words are double-buffered by round parity: a block that has left
// round r's barrier writes round r+1's word into the other half, so block
// 0's check of round r can only see round r's value or an older (stale) one.
// (Round 1 used one buffer, so faster blocks' round r+1 writes were counted
// as "stale" -- they were too new; profiles/r01_launch_floor.log.)
template <int MODE>
__global__ void k_barrier(unsigned long long *bar, int rounds, int nb, unsigned long long *data, unsigned long long *bad) {
    for (int r = 0; r < rounds; r++) {
        unsigned long long *dr = data + (r & 1) * nb;
        if (threadIdx.x == 0) dr[blockIdx.x] = (unsigned long long)r * 1000003ull + blockIdx.x;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            unsigned long long t = atomicAdd(bar, 1ull);
            unsigned long long target = (t / nb + 1) * nb;
            long long t0 = clock64();
            for (;;) {
                unsigned long long v;
                if (MODE == 0) v = __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                else if (MODE == 1) v = atomicAdd(bar, 0ull);
                else v = __hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (v >= target) break;
                __builtin_amdgcn_s_sleep(1);
                if (clock64() - t0 > 2000000000ll) break;
            }
            __threadfence();
        }
        __syncthreads();
        if (blockIdx.x == 0 && threadIdx.x < nb) {
            unsigned long long v = __hip_atomic_load(&dr[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v != (unsigned long long)r * 1000003ull + threadIdx.x) atomicAdd(bad, 1ull);
        }
        __syncthreads();
    }
}

template <typename F>
static double graph_time(hipStream_t s, int n, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; i++) launch();
    CHK(hipStreamEndCapture(s, &g));
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHK(hipGraphLaunch(ge, s));
    CHK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    CHK(hipEventRecord(a, s));
    for (int r = 0; r < 10; r++) CHK(hipGraphLaunch(ge, s));
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / (10.0 * n);
}

template <typename F>
static double eager_time(hipStream_t s, int n, F launch) {
    for (int i = 0; i < n; i++) launch();
    CHK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    CHK(hipEventRecord(a, s));
    for (int i = 0; i < 10 * n; i++) launch();
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms; CHK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / (10.0 * n);
}

int main() {
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double *a; int *idx, *out; unsigned long long *bar;
    const int n = 97 * 256;
    CHK(hipMalloc(&a, n * 8)); CHK(hipMemset(a, 0, n * 8));
    CHK(hipMalloc(&idx, (size_t)64 << 20)); CHK(hipMalloc(&out, n * 4));
    CHK(hipMalloc(&bar, 8)); CHK(hipMemset(bar, 0, 8));
    {   // random permutation-ish index over 64 MB (misses L2, hits MALL)
        int N = 16 << 20;
        int *h = (int *)malloc((size_t)N * 4);
        unsigned x = 12345;
        for (int i = 0; i < N; i++) { x = x * 1664525u + 1013904223u; h[i] = (int)(x % (unsigned)N); }
        CHK(hipMemcpy(idx, h, (size_t)N * 4, hipMemcpyHostToDevice));
        free(h);
    }
    const int N = 200;
    printf("empty kernel, 1 block:     graph %6.2f us  eager %6.2f us\n",
           graph_time(s, N, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }),
           eager_time(s, N, [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); }));
    printf("empty kernel, 97 blocks:   graph %6.2f us  eager %6.2f us\n",
           graph_time(s, N, [&] { hipLaunchKernelGGL(k_empty, dim3(97), dim3(256), 0, s); }),
           eager_time(s, N, [&] { hipLaunchKernelGGL(k_empty, dim3(97), dim3(256), 0, s); }));
    printf("touch 97x256 doubles:      graph %6.2f us  eager %6.2f us\n",
           graph_time(s, N, [&] { hipLaunchKernelGGL(k_touch, dim3(97), dim3(256), 0, s, a, n); }),
           eager_time(s, N, [&] { hipLaunchKernelGGL(k_touch, dim3(97), dim3(256), 0, s, a, n); }));
    for (int hops = 1; hops <= 8; hops *= 2)
        printf("dependent loads x%d:        graph %6.2f us\n", hops,
               graph_time(s, N, [&] { hipLaunchKernelGGL(k_chain, dim3(97), dim3(256), 0, s, idx, out, hops); }));
    unsigned long long *data, *bad;
    CHK(hipMalloc(&data, 2 * 1024 * 8)); CHK(hipMalloc(&bad, 8));
    for (int mode = 1; mode < 3; mode++)
    for (int nb = 4; nb <= 256; nb *= 4) {
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        const int rounds = 200;
        CHK(hipMemset(bar, 0, 8)); CHK(hipMemset(bad, 0, 8));
        CHK(hipEventRecord(e0, s));
        if (mode == 1) hipLaunchKernelGGL(k_barrier<1>, dim3(nb), dim3(256), 0, s, bar, rounds, nb, data, bad);
        else hipLaunchKernelGGL(k_barrier<2>, dim3(nb), dim3(256), 0, s, bar, rounds, nb, data, bad);
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long hb = 0;
        CHK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("grid barrier mode %d (%s), %3d blocks: %7.2f us per barrier, stale reads %llu\n", mode,
               mode == 1 ? "atomicAdd poll" : "system-scope load poll", nb, ms * 1e3 / rounds, hb);
    }
    return 0;
}
