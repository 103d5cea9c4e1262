// overlap_lab.hip — can the block pass run UNDER the pivot loop? (lab only;
// the product never links this file)
//
// Overlapping block b's pass with block b+1's pivots (VERDICT round 2, next
// #3) needs the pass to run on CUs where a pivot workgroup already sits: the
// persistent pivot kernel holds one workgroup per CU with ~136-150 KB of LDS
// and, today, 468-512 VGPRs per lane (k_pivot_block: 1 wave per SIMD fills
// the register file), so a pass kernel launched beside it on a second stream
// finds no registers and no LDS on 227 of the 256 CUs. The only overlap that
// can exist is a MERGED persistent kernel: per CU one workgroup with NPV
// pivot waves (each <= 256 VGPRs, the slices in LDS) and 4 pass waves (one
// per SIMD, <= 256 VGPRs, no LDS: B fragments = P in VGPRs, A = -C loaded
// straight from the Infinity Cache / L2, tableau bands prefetched DEP ahead).
//
// This lab measures the two numbers that decide whether that kernel can pay:
//   1. the pass alone at ONE wave per SIMD under a 136 KB LDS reservation
//      (NPV = 0) against the product's k_flushw<64> (2 waves per SIMD);
//   2. the same pass while NPV pivot-like waves run beside it (MODE 1: idle
//      spin on an LDS flag; MODE 2: wave 0 sweeps 256 tagged 16-byte records
//      with sc1 loads and every pivot wave runs a 64-step LDS-fed fma chain
//      between sweeps, i.e. the pivot loop's memory and VALU footprint).
// Every pass variant is checked bitwise against k_flushw<64> first (same
// chain, same MFMA), then timed.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/overlap_lab tools/overlap_lab.hip
//   tools/overlap_lab
#include "../linearprogramming_amd/csrc/lpg_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace lpg {

constexpr int kLabLds = 136 * 1024;   // the pivot kernel's slices at 256 workgroups (config 3)

// NPV pivot-like waves + 4 pass waves per workgroup, one workgroup per CU.
// Pass wave v (of 4 * gridDim.x) owns the 32-column tile v of the live
// columns over every row (k_flushw's lane map: lane (lk, lc) holds the column
// pair 2 lc, 2 lc + 1 and rows lk + 4 r of each 16-row band), 64 slots.
template <int NPV, int DEP, int MODE, int ST = 0>
__global__ __launch_bounds__(64 * (NPV + 4), 1) void k_opass(double *__restrict__ T, Geo g,
                                                              const double *__restrict__ Pbuf,
                                                              const double *__restrict__ Cbuf, int64_t cs,
                                                              int64_t ntiles, uint4 *rec, unsigned long long *spins) {
    constexpr int G = 16;                        // 64 slots / 4
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int done;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    if (wave < NPV) {
        // ---- pivot-like waves
        // MODE 0: exit at once; 1: f64-divide LDS init, then spin on the flag;
        // 2: 1 + a record sweep (wave 0, sc1 loads) and a 64-step LDS-fed fma
        // chain per loop; 3: spin only; 4: register-only v_fma_f64 chains;
        // 5: integer VALU chains; 6: LDS reads only; 7: v_add_f64 chains;
        // 8: v_mul_f64 chains
        if (MODE == 0) return;
        unsigned long long n = 0;
        double x = (double)lane, y = 1.0 + lane;
        uint32_t iv = lane;
        if (MODE == 1 || MODE == 2)
            for (int u = lane; u < 64 * 66; u += 64) lds[wave * 64 * 66 + u] = 1.0 / (1 + u);
        if (MODE == 6)
            for (int u = lane; u < 64 * 66; u += 64) lds[wave * 64 * 66 + u] = (double)u;
        while (__hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4) {
            if (MODE == 2) {
                if (wave == 0) {   // one sweep of 256 records (sc1 loads), as the pivot loop's phase P / S
                    uint32_t acc = 0;
                    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(rec, (short)0, 256 * 16, 0x00020000);
#pragma unroll
                    for (int p = 0; p < 4; p++) {
                        typedef unsigned u4v __attribute__((ext_vector_type(4)));
                        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (lane + 64 * p) * 16, 0, 16);
                        acc ^= v[3];
                    }
                    if (acc == 0xdeadbeef) rec[0].x = acc;   // never: keeps the loads
                }
            }
            if (MODE == 2 || MODE == 6) {
                // a 64-step chain fed from LDS (the pending chain of one pivot row)
                const double *sp = lds + (size_t)wave * 64 * 66 + (size_t)lane * 66 % 4096;
#pragma unroll 16
                for (int u = 0; u < 64; u++) {
                    if (MODE == 2) x = fma(sp[u], 0.999, x);
                    else iv ^= (uint32_t)__double_as_longlong(sp[u]);
                }
            }
            if (MODE == 4) {
#pragma unroll 16
                for (int u = 0; u < 64; u++) x = fma(x, 0.999, y);
            }
            if (MODE == 5) {
#pragma unroll 16
                for (int u = 0; u < 64; u++) iv = iv * 1664525u + 1013904223u;
            }
            if (MODE == 7) {
#pragma unroll 16
                for (int u = 0; u < 64; u++) x = x + y;
            }
            if (MODE == 8) {
#pragma unroll 16
                for (int u = 0; u < 64; u++) x = x * 0.999;
            }
            __builtin_amdgcn_s_sleep(MODE == 3 ? 32 : 8);
            n++;
        }
        if (lane == 0 && (x == -1.0 || iv == 7u)) spins[1] = n;   // never: keeps the chains
        if (lane == 0) atomicAdd(spins, n);
        return;
    }
    // ---- pass waves
    const int pw = (int)blockIdx.x * 4 + (wave - NPV);
    const int lc = lane & 15, lk = lane >> 4;
    if (pw < ntiles) {
        const int64_t ld = g.ld;
        const int64_t cl = (int64_t)pw * 32 + 2 * lc;
        double be[G], bo[G];
#pragma unroll
        for (int gq = 0; gq < G; gq++) {
            const d2 v = *(const d2 *)(Pbuf + (int64_t)(4 * gq + lk) * ld + cl);
            be[gq] = v.x;
            bo[gq] = v.y;
        }
        const int nb = (int)((g.nloc + 15) / 16);
        // buffer loads / stores: one VGPR offset per stream, the rest in SGPRs
        // (64-bit addresses for 16 A loads + 4 T loads cost ~40 VGPRs)
        const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(Cbuf), (short)0,
                                                                            (int)(64 * cs * 8), 0x00020000);
        const int voffT = (int)(((int64_t)lk * ld + cl) * 8);
        const int voffA = (int)(((int64_t)lk * cs + lc) * 8);
        auto band_rsrc = [&](int s) {
            return __builtin_amdgcn_make_buffer_rsrc(T + (int64_t)16 * s * ld, (short)0, (int)(16 * ld * 8), 0x00020000);
        };
        auto tload = [&](d2 (&x)[4], int s) {
            const __amdgpu_buffer_rsrc_t rt = band_rsrc(s);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rt, voffT, (int)(r * 4 * ld * 8), 2);
                x[r] = __builtin_bit_cast(d2, v);
            }
        };
        auto aload = [&](double (&a)[G], int s) {
#pragma unroll
            for (int gq = 0; gq < G; gq++) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rc, voffA + s * 16 * 8, (int)(gq * 4 * cs * 8), 0);
                a[gq] = s < nb ? -__builtin_bit_cast(double, v) : -0.0;
            }
        };
        d2 tb[DEP][4];
        double ab[2][G];
#pragma unroll
        for (int d = 0; d < DEP; d++) tload(tb[d], d);
        aload(ab[0], 0);
        for (int s0 = 0; s0 < nb; s0 += DEP) {
#pragma unroll
            for (int d = 0; d < DEP; d++) {
                const int s = s0 + d;
                if (s < nb) {
                    aload(ab[(d + 1) & 1], s + 1);
                    d4 ae = d4{tb[d][0].x, tb[d][1].x, tb[d][2].x, tb[d][3].x};
                    d4 ao = d4{tb[d][0].y, tb[d][1].y, tb[d][2].y, tb[d][3].y};
#pragma unroll
                    for (int gq = 0; gq < G; gq++) {
                        ae = __builtin_amdgcn_mfma_f64_16x16x4f64(ab[d & 1][gq], be[gq], ae, 0, 0, 0);
                        ao = __builtin_amdgcn_mfma_f64_16x16x4f64(ab[d & 1][gq], bo[gq], ao, 0, 0, 0);
                    }
                    const __amdgpu_buffer_rsrc_t rt = band_rsrc(s);
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        typedef unsigned u4v __attribute__((ext_vector_type(4)));
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, d2{ae[r], ao[r]}), rt, voffT,
                                                               (int)(r * 4 * ld * 8), 2);
                        // ST = 1: two wait states before anything may rewrite the
                        // store's data VGPRs (hipcc emits none after raw buffer
                        // stores; see tools/store_hazard_scan.py)
                        if (ST == 1) asm volatile("s_nop 1" ::: "memory");
                    }
                    if (s + DEP < nb) tload(tb[d], s + DEP);
                }
            }
        }
    }
    if (lane == 0) __hip_atomic_fetch_add(&done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

}  // namespace lpg

using namespace lpg;

__global__ void k_fill(double *x, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * 0x1.0p-53 - 0.25;
    }
}
// P_q[j] = 0 for the non-live columns (the basic region and the padding)
__global__ void k_zero_cols(double *P, int64_t ld, int64_t j0, int k) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)k * ld; e += (int64_t)gridDim.x * blockDim.x)
        if (e % ld >= j0) P[e] = 0.0;
}
// bad[0]: mismatching doubles; bad[1..8]: some of their indices
__global__ void k_cmp(const double *a, const double *b, int64_t n, unsigned long long *bad) {
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (__double_as_longlong(a[i]) != __double_as_longlong(b[i])) {
            c++;
            const unsigned long long k = atomicAdd(&bad[9], 1ull);
            if (k < 8) bad[1 + k] = (unsigned long long)i;
        }
    if (c) atomicAdd(bad, c);
}

struct Lab {
    Geo g{};
    DevState *st = nullptr;
    double *T = nullptr, *T0 = nullptr, *Tref = nullptr, *Pbuf = nullptr, *Cbuf = nullptr;
    uint4 *rec = nullptr;
    unsigned long long *spins = nullptr, *bad = nullptr;
    int64_t n = 0, cs = 0, nlive = 0;
    hipEvent_t e0, e1;
};
typedef void (*Fn)(Lab &);

static void fn_ref(Lab &L) {   // the product's launch (launch_flush_main, 64 slots)
    DevState h{};
    h.npend = 64;
    CHK(hipMemcpyAsync(L.st, &h, sizeof h, hipMemcpyHostToDevice, 0));
    const int64_t ntiles = (L.g.ncols + 255) / 256, rows = 512;
    const int64_t nitems = flush_nitems(ntiles, rows, L.g.nloc);
    const int64_t nblocks = std::min<int64_t>(nitems, 512);
    hipLaunchKernelGGL((k_flushw<64, 2, 2, 8>), dim3((unsigned)((nblocks + 1) / 2)), dim3(512), 0, 0, L.g.T, L.g, L.st,
                       L.Pbuf, L.Cbuf, L.cs, ntiles, nitems, rows, 1);
}

template <int NPV, int DEP, int MODE, int ST = 0>
static void fn_o(Lab &L) {
    static bool set = false;
    if (!set) {
        CHK(hipFuncSetAttribute((const void *)k_opass<NPV, DEP, MODE, ST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kLabLds));
        set = true;
    }
    const int64_t ntiles = L.nlive / 32;
    hipLaunchKernelGGL((k_opass<NPV, DEP, MODE, ST>), dim3((unsigned)((ntiles + 3) / 4)), dim3(64 * (NPV + 4)), kLabLds, 0,
                       L.g.T, L.g, L.Pbuf, L.Cbuf, L.cs, ntiles, L.rec, L.spins);
}

static void run(Lab &L, Fn fn, const char *name, int reps) {
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    fn(L);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipMemset(L.bad, 0, 10 * 8));
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, L.T, L.Tref, L.n, L.bad);
    unsigned long long bd[10];
    CHK(hipMemcpy(bd, L.bad, sizeof bd, hipMemcpyDeviceToHost));
    const unsigned long long nb = bd[0];
    if (nb) {
        printf("%-38s MISMATCH: %llu doubles differ from k_flushw<64>; e.g. (row, col):", name, nb);
        for (int k = 0; k < 8 && k < (int)nb; k++) printf(" (%lld, %lld)", (long long)(bd[1 + k] / L.g.ld), (long long)(bd[1 + k] % L.g.ld));
        printf("\n");
        fflush(stdout);
        return;
    }
    CHK(hipMemset(L.spins, 0, 8));
    double best = 1e30, sum = 0;
    for (int r = 0; r < reps; r++) {
        CHK(hipEventRecord(L.e0));
        fn(L);
        CHK(hipEventRecord(L.e1));
        CHK(hipEventSynchronize(L.e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, L.e0, L.e1));
        best = ms < best ? ms : best;
        sum += ms;
    }
    unsigned long long sp = 0;
    CHK(hipMemcpy(&sp, L.spins, 8, hipMemcpyDeviceToHost));
    const double bytes = 16.0 * (double)L.nlive * (double)L.g.nloc;
    printf("%-38s best %.3f ms  mean %.3f ms  %.0f GB/s  %.1f TFLOP/s  pivot-wave loop iterations %.0f per launch\n",
           name, best, sum / reps, bytes / (best * 1e-3) / 1e9, 2.0 * 64 * bytes / 16 / (best * 1e-3) / 1e12,
           (double)sp / reps);
    fflush(stdout);
}

int main(int argc, char **argv) {
    Lab L;
    const int64_t m = argc > 1 ? atoll(argv[1]) : 16384, nstruct = 2 * m;
    const int64_t ncols = nstruct + m + 1, ld = (ncols + 63) / 64 * 64;
    L.nlive = nstruct;                 // 32768 live columns = 1024 tiles of 32: one per pass wave at 256 CUs
    L.n = m * ld;
    L.cs = (m + 63) / 64 * 64;
    CHK(hipMalloc(&L.T, L.n * 8));
    CHK(hipMalloc(&L.T0, L.n * 8));
    CHK(hipMalloc(&L.Tref, L.n * 8));
    CHK(hipMalloc(&L.st, sizeof(DevState)));
    CHK(hipMalloc(&L.bad, 10 * 8));
    CHK(hipMalloc(&L.spins, 16));
    CHK(hipMalloc(&L.rec, 256 * sizeof(uint4)));
    CHK(hipMemset(L.rec, 0, 256 * sizeof(uint4)));
    CHK(hipMalloc(&L.Pbuf, (size_t)64 * ld * 8));
    CHK(hipMalloc(&L.Cbuf, (size_t)64 * L.cs * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, L.T0, L.n, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, L.Pbuf, (int64_t)64 * ld, 2ull);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, L.Cbuf, (int64_t)64 * L.cs, 3ull);
    hipLaunchKernelGGL(k_zero_cols, dim3(1024), dim3(256), 0, 0, L.Pbuf, ld, L.nlive, 64);
    CHK(hipDeviceSynchronize());
    L.g.T = L.T;
    L.g.ld = ld;
    L.g.nloc = m;
    L.g.nobj = 1;
    L.g.ncols = ncols;
    L.g.nact = ncols - 1;
    L.g.m = m;
    CHK(hipEventCreate(&L.e0));
    CHK(hipEventCreate(&L.e1));
    printf("overlap lab: %lld rows x %lld live columns (ld %lld), 64 slots, %.3f GB read+write per pass\n",
           (long long)m, (long long)L.nlive, (long long)ld, 16.0 * L.nlive * m / 1e9);
    CHK(hipMemcpy(L.T, L.T0, L.n * 8, hipMemcpyDeviceToDevice));
    fn_ref(L);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(L.Tref, L.T, L.n * 8, hipMemcpyDeviceToDevice));
    const int reps = 5;
    run(L, fn_ref, "k_flushw<64,2,2,8> (product)", reps);
    run(L, fn_o<0, 2, 0, 1>, "opass npv0 dep2", reps);
    run(L, fn_o<0, 4, 0, 1>, "opass npv0 dep4", reps);
    run(L, fn_o<4, 4, 0, 1>, "opass npv4 dep4 exit", reps);
    run(L, fn_o<4, 4, 3, 0>, "opass npv4 spin (no s_nop)", reps);
    run(L, fn_o<4, 4, 3, 1>, "opass npv4 spin", reps);
    run(L, fn_o<4, 4, 5, 0>, "opass npv4 int VALU (no s_nop)", reps);
    run(L, fn_o<4, 4, 5, 1>, "opass npv4 int VALU", reps);
    run(L, fn_o<4, 4, 4, 1>, "opass npv4 v_fma_f64", reps);
    run(L, fn_o<4, 4, 2, 0>, "opass npv4 sweeps+chains (no s_nop)", reps);
    run(L, fn_o<4, 4, 2, 1>, "opass npv4 sweeps+chains", reps);
    run(L, fn_o<4, 2, 2, 1>, "opass npv4 dep2 sweeps+chains", reps);
    run(L, fn_ref, "k_flushw<64,2,2,8> (product)", reps);
    return 0;
}
