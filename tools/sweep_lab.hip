// sweep_lab.hip -- the all-to-all decision of k_pivot_block in isolation
// ("prototype a two-level sweep"). Experiments only.
//
// One persistent launch of nwg workgroups (one per CU); per iteration every
// workgroup's wave 0 waits `work` + (hash % skew) ticks of s_memrealtime
// (the per-pivot chain work and its spread over the grid), publishes one
// 16-byte {key, wg, tag} record with an sc1 store (the product's granule),
// and the workgroup learns the grid's minimum key by:
//   mode 0  flat: wave 0 of EVERY workgroup sweeps all nwg records (the product);
//   mode 1  two-level: group g = wg % 8 (one XCD under round-robin placement;
//           speed only); workgroup g (< 8) sweeps its group's ~nwg/8 records and
//           publishes the group's minimum; every workgroup sweeps the 8 group
//           records;
//   mode 2  R readers: workgroups 0..R-1 sweep all nwg records and publish the
//           decision; workgroup w reads reader w % R's.
// Records are double-buffered by iteration parity (as the product alternates
// its ratio / pricing arrays), so no record is overwritten while a slow
// reader may still want it. Every spin is bounded (1 s): a workgroup that
// gives up sets *fail and leaves, and the others follow.
// The host checks every iteration's decision against the true argmin.
// Round 5 (XCD1): the flat sweep with the grid confined to ONE XCD (8 x nwg
// blocks launched, those with b % 8 != 0 leave at once, so the rest share one
// L2 under round-robin placement -- speed only, correctness is checked), with
// the records' sc1 policy on both sides (the product's: an sc1 store drops
// the line from L2, so readers fetch it at the cross-XCD rate), or plain / nt
// stores, which keep the line in that L2, with sc1 loads (L1 bypassed, L2
// served; MI355X_MICROARCH.md: sc0 loads hit L1 and never see the store):
// what a rank whose pivot slices fit one XCD (a column-sliced rank at P = 8:
// 3.1 MB) would pay per sweep.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../linearprogramming_amd/csrc/lpg_device.h"

using namespace lpg;
typedef unsigned u4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr long long kSpin = 100000000ll;   // 1 s at 100 MHz

__host__ __device__ inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__host__ __device__ inline uint64_t keyof(int wg, int it) { return mix(((uint64_t)it << 20) | (uint64_t)wg) >> 20; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, bytes, 0x00020000);
}
template <int AUX = 16>
__device__ __forceinline__ void rst(__amdgpu_buffer_rsrc_t r, int off, u4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}
template <int AUX = 16>
__device__ __forceinline__ u4 rld(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}
__device__ __forceinline__ uint64_t lo64(const u4 &v) { return ((uint64_t)v.y << 32) | v.x; }

// wave 0: sweep records idx = first + stride * (lane + 64 p), p < 4, for the
// n entries, until every tag matches; the minimum {key, wg}; false on timeout
template <int AUX = 16>
__device__ bool sweep_min(__amdgpu_buffer_rsrc_t r, int first, int stride, int n, uint32_t tag, uint64_t &h,
                          uint32_t &l) {
    const int lane = threadIdx.x & 63;
    const long long t0 = (long long)wall_clock64();
    u4 v[4];
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int i = lane + 64 * p;
            if (i < n) v[p] = rld<AUX>(r, (first + stride * i) * 16);
        }
#pragma unroll
        for (int p = 0; p < 4; p++)
            if (lane + 64 * p < n && v[p].w != tag) ok = false;
        if (__all(ok)) break;
        if ((long long)wall_clock64() - t0 > kSpin) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    h = ~0ull;
    l = ~0u;
#pragma unroll
    for (int p = 0; p < 4; p++)
        if (lane + 64 * p < n && key_less(lo64(v[p]), v[p].z, h, l)) {
            h = lo64(v[p]);
            l = v[p].z;
        }
    wave_min_key(h, l);
    return true;
}

__global__ __launch_bounds__(256, 1) void k_lab(int mode, int R, u4 *rec, u4 *aux, int nwg, int iters, int work,
                                                int skew, uint32_t tag0, int *dec, unsigned long long *stamp,
                                                int *fail) {
    __shared__ int sdec;
    const int wg = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int ng = nwg < 8 ? nwg : 8;
    for (int it = 0; it < iters; it++) {
        const uint32_t tag = tag0 + 1 + it;
        const __amdgpu_buffer_rsrc_t rr = rsrc(rec + (it & 1) * nwg, nwg * 16);
        const __amdgpu_buffer_rsrc_t ra = rsrc(aux + (it & 1) * 256, 256 * 16);
        if (tid < 64) {
            const uint64_t k = keyof(wg, it);
            const long long s = (long long)wall_clock64();
            const long long dur = work + (skew > 0 ? (long long)(mix(k) % (uint64_t)skew) : 0);
            while ((long long)wall_clock64() - s < dur) {}
            if (lane == 0) rst(rr, wg * 16, u4{(uint32_t)k, (uint32_t)(k >> 32), (uint32_t)wg, tag});
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint64_t h;
            uint32_t l;
            bool ok = true;
            if (mode == 0) {
                ok = sweep_min(rr, 0, 1, nwg, tag, h, l);
            } else if (mode == 1) {
                if (wg < ng) {   // group leader: members wg, wg + 8, ...
                    ok = sweep_min(rr, wg, ng, (nwg - wg + ng - 1) / ng, tag, h, l);
                    if (ok && lane == 0) rst(ra, wg * 16, u4{(uint32_t)h, (uint32_t)(h >> 32), l, tag});
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (ok) ok = sweep_min(ra, 0, 1, ng, tag, h, l);
            } else {
                if (wg < R) {
                    ok = sweep_min(rr, 0, 1, nwg, tag, h, l);
                    if (ok && lane == 0) rst(ra, wg * 16, u4{(uint32_t)h, (uint32_t)(h >> 32), l, tag});
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (ok) ok = sweep_min(ra, wg % R, 1, 1, tag, h, l);
            }
            if (lane == 0) {
                sdec = ok ? (int)l : -1;
                if (!ok) atomicAdd(fail, 1);
            }
        }
        __syncthreads();
        const int d = sdec;
        if (d < 0) break;
        if (tid == 0 && (wg == 0 || wg == nwg - 1)) {
            dec[(wg == 0 ? 0 : iters) + it] = d;
            if (wg == 0) stamp[it] = (unsigned long long)wall_clock64();
        }
        __syncthreads();
    }
}

// the flat sweep on a grid confined to one XCD (see the header)
template <int SAUX, int LAUX>
__global__ __launch_bounds__(256, 1) void k_lab1(u4 *rec, int nwg, int iters, int work, int skew, uint32_t tag0,
                                                 int *dec, unsigned long long *stamp, int *fail) {
    __shared__ int sdec;
    if (blockIdx.x % 8) return;
    const int wg = blockIdx.x / 8, tid = threadIdx.x, lane = tid & 63;
    for (int it = 0; it < iters; it++) {
        const uint32_t tag = tag0 + 1 + it;
        const __amdgpu_buffer_rsrc_t rr = rsrc(rec + (it & 1) * nwg, nwg * 16);
        if (tid < 64) {
            const uint64_t k = keyof(wg, it);
            const long long s = (long long)wall_clock64();
            const long long dur = work + (skew > 0 ? (long long)(mix(k) % (uint64_t)skew) : 0);
            while ((long long)wall_clock64() - s < dur) {}
            if (lane == 0) rst<SAUX>(rr, wg * 16, u4{(uint32_t)k, (uint32_t)(k >> 32), (uint32_t)wg, tag});
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint64_t h;
            uint32_t l;
            const bool ok = sweep_min<LAUX>(rr, 0, 1, nwg, tag, h, l);
            if (lane == 0) {
                sdec = ok ? (int)l : -1;
                if (!ok) atomicAdd(fail, 1);
            }
        }
        __syncthreads();
        const int d = sdec;
        if (d < 0) break;
        if (tid == 0 && (wg == 0 || wg == nwg - 1)) {
            dec[(wg == 0 ? 0 : iters) + it] = d;
            if (wg == 0) stamp[it] = (unsigned long long)wall_clock64();
        }
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    printf("sweep lab: %s, %d CUs, %d iterations per run, s_memrealtime 100 MHz\n", pr.gcnArchName,
           pr.multiProcessorCount, iters);
    u4 *rec, *aux;
    int *dec, *fail;
    unsigned long long *stamp;
    CK(hipMalloc(&rec, 2 * 256 * 16));
    CK(hipMalloc(&aux, 2 * 256 * 16));
    CK(hipMalloc(&dec, 2 * iters * sizeof(int)));
    CK(hipMalloc(&fail, sizeof(int)));
    CK(hipMalloc(&stamp, iters * sizeof(unsigned long long)));
    CK(hipMemset(rec, 0, 2 * 256 * 16));
    CK(hipMemset(aux, 0, 2 * 256 * 16));
    uint32_t tag0 = 0;
    std::vector<int> hd(2 * iters);
    std::vector<unsigned long long> hs(iters);
    if (getenv("LAB_XCD1")) {   // round 5: spread vs one-XCD flat sweeps at small grids
        for (int rep = 0; rep < 2; rep++)
            for (int nw : {16, 22, 32})
                for (int wi = 0; wi < 2; wi++)
                    for (int v = 0; v < 4; v++) {
                        const int work = wi ? 200 : 100, skew = wi ? 100 : 0;
                        CK(hipMemset(fail, 0, sizeof(int)));
                        CK(hipMemset(dec, 0xff, 2 * iters * sizeof(int)));
                        const char *name = v == 0 ? "spread, sc1 (product)" : v == 1 ? "one XCD, sc1" :
                                           v == 2 ? "one XCD, plain st + sc1 ld" : "one XCD, nt st + sc1 ld";
                        if (v == 0)
                            hipLaunchKernelGGL(k_lab, dim3(nw), dim3(256), 0, 0, 0, 0, rec, aux, nw, iters, work, skew,
                                               tag0, dec, stamp, fail);
                        else if (v == 1)
                            hipLaunchKernelGGL((k_lab1<16, 16>), dim3(8 * nw), dim3(256), 0, 0, rec, nw, iters, work, skew,
                                               tag0, dec, stamp, fail);
                        else if (v == 2)
                            hipLaunchKernelGGL((k_lab1<0, 16>), dim3(8 * nw), dim3(256), 0, 0, rec, nw, iters, work, skew,
                                               tag0, dec, stamp, fail);
                        else
                            hipLaunchKernelGGL((k_lab1<2, 16>), dim3(8 * nw), dim3(256), 0, 0, rec, nw, iters, work, skew,
                                               tag0, dec, stamp, fail);
                        CK(hipGetLastError());
                        CK(hipDeviceSynchronize());
                        tag0 += iters;
                        int hf = 0;
                        CK(hipMemcpy(&hf, fail, sizeof(int), hipMemcpyDeviceToHost));
                        CK(hipMemcpy(hd.data(), dec, 2 * iters * sizeof(int), hipMemcpyDeviceToHost));
                        CK(hipMemcpy(hs.data(), stamp, iters * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                        int bad = 0;
                        for (int it = 0; it < iters; it++) {
                            int best = 0;
                            for (int w = 1; w < nw; w++)
                                if (keyof(w, it) < keyof(best, it)) best = w;
                            bad += hd[it] != best || hd[iters + it] != best;
                        }
                        const double us = (double)(hs[iters - 1] - hs[iters / 2]) / (iters - 1 - iters / 2) / 100.0;
                        printf("rep %d nwg %3d work %.1f us skew %.1f us  %-22s %6.3f us/iter  (sweep ~%6.3f)  %s\n", rep,
                               nw, work / 100.0, skew / 100.0, name, us,
                               us - work / 100.0 - (skew > 0 ? (skew - 1) / 100.0 : 0.0), hf ? "TIMEOUT" : bad ? "WRONG" : "ok");
                        fflush(stdout);
                        if (hf) return 1;
                    }
        return 0;
    }
    struct Case { int mode, R; const char *name; };
    const Case cases[] = {{0, 0, "flat (product)"}, {1, 0, "two-level, 8 groups"}, {2, 32, "32 readers + bcast"},
                          {2, 8, "8 readers + bcast"}};
    const int nwgs[] = {227, 256};
    const int works[] = {100, 100, 200};
    const int skews[] = {0, 60, 100};
    for (int rep = 0; rep < 2; rep++)
        for (int nw : nwgs)
            for (int wi = 0; wi < 3; wi++)
                for (const Case &c : cases) {
                    CK(hipMemset(fail, 0, sizeof(int)));
                    CK(hipMemset(dec, 0xff, 2 * iters * sizeof(int)));
                    hipLaunchKernelGGL(k_lab, dim3(nw), dim3(256), 0, 0, c.mode, c.R, rec, aux, nw, iters, works[wi],
                                       skews[wi], tag0, dec, stamp, fail);
                    CK(hipGetLastError());
                    CK(hipDeviceSynchronize());
                    tag0 += iters;
                    int hf = 0;
                    CK(hipMemcpy(&hf, fail, sizeof(int), hipMemcpyDeviceToHost));
                    CK(hipMemcpy(hd.data(), dec, 2 * iters * sizeof(int), hipMemcpyDeviceToHost));
                    CK(hipMemcpy(hs.data(), stamp, iters * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                    int bad = 0;
                    for (int it = 0; it < iters; it++) {
                        int best = 0;
                        for (int w = 1; w < nw; w++)
                            if (keyof(w, it) < keyof(best, it)) best = w;
                        bad += hd[it] != best || hd[iters + it] != best;
                    }
                    // per-iteration time over the second half (steady state), us
                    const double us = (double)(hs[iters - 1] - hs[iters / 2]) / (iters - 1 - iters / 2) / 100.0;
                    printf("rep %d nwg %3d work %.1f us skew %.1f us  %-22s %6.3f us/iter  (sweep ~%6.3f)  %s\n", rep,
                           nw, works[wi] / 100.0, skews[wi] / 100.0, c.name, us,
                           us - works[wi] / 100.0 - (skews[wi] > 0 ? (skews[wi] - 1) / 100.0 : 0.0),
                           hf ? "TIMEOUT" : bad ? "WRONG" : "ok");
                    if (hf || bad) return 1;
                }
    return 0;
}
