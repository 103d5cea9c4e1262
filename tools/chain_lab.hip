// Chain lab: k_pivot_block's pending chains alone (lab only). Every
// workgroup (227, one per CU, 150 KB of slices like config 3) runs the
// pivot-row chain of its 217 columns over q slots `reps` times, a barrier
// between runs as in the kernel, and thread 0 stamps the run (s_memrealtime,
// 10 ns). Forms: the product's batched chain (lpg_block.hip chain<>), the
// same with only the waves holding columns, and an LDS-read-only pass (no
// fma), an fma-only pass (operands from registers) to split the cost, and
// a form that reads the uniform operand by v_readlane instead of LDS.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/chain_lab tools/chain_lab.hip
#include "../linearprogramming_amd/csrc/lpg_block.hip"

#include <stdio.h>
#include <stdlib.h>

using namespace lpg;

namespace {
// FORM 3: the chains with the uniform operand taken from a register instead of
// LDS (measured 2x slower than chain<>, not in the product): lane u of `uv` holds slot u's multiplier (row) or P_u[k] (column), and
// each step reads it with two v_readlane into SGPRs. Half the LDS reads of
// chain<>, and the readlanes run in the fma chain's latency shadow.
__device__ __forceinline__ double lane_val(double v, int u) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), u);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), u);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <bool ROW, bool SEL>
__device__ __forceinline__ double chain_rl_batch(const d2 (&o)[8], double uv, int base, int lim, double x) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const bool l0 = !SEL || base + 2 * j > lim, l1 = !SEL || base + 2 * j + 1 > lim;
        const double w0 = lane_val(uv, base + 2 * j), w1 = lane_val(uv, base + 2 * j + 1);
        if (ROW) {
            x = fma(l0 ? w0 : -0.0, l0 ? o[j].x : 0.0, x);
            x = fma(l1 ? w1 : -0.0, l1 ? o[j].y : 0.0, x);
        } else {
            x = fma(-(l0 ? o[j].x : 0.0), l0 ? w0 : 0.0, x);
            x = fma(-(l1 ? o[j].y : 0.0), l1 ? w1 : 0.0, x);
        }
    }
    return x;
}
template <bool ROW, bool SEL>
__device__ __forceinline__ double chain_rl(const double *own, double uv, int nb, int lim, double x) {
    if (nb <= 0) return x;
    d2 o0[8], o1[8];
    auto load = [&](d2 (&o)[8], int bb) {
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = ((const d2 *)own)[8 * bb + j];
    };
    load(o0, 0);
#pragma unroll 1
    for (int bb = 0; bb < nb; bb += 2) {
        if (bb + 1 < nb) load(o1, bb + 1);
        x = chain_rl_batch<ROW, SEL>(o0, uv, 16 * bb, lim, x);
        if (bb + 1 >= nb) break;
        if (bb + 2 < nb) load(o0, bb + 2);
        x = chain_rl_batch<ROW, SEL>(o1, uv, 16 * (bb + 1), lim, x);
    }
    return x;
}


constexpr int kCW = 217, kS = 66, kNWG = 227, kReps = 64;

template <int FORM>
__global__ __launch_bounds__(256, 1) void k_chain_lab(double *out, unsigned long long *ticks, int q) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ __attribute__((aligned(16))) double wm[4][72];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double *sPt = lds + (size_t)(tid < kCW ? tid : kCW - 1) * kS;
    for (int u = 0; u < kS; u++)
        if (tid < kCW) sPt[u] = u < q ? 1.0 + 1e-3 * (tid + u) : 0.0;
    wm[wave][lane] = lane < q ? -1e-2 * (lane + 1) : -0.0;
    if (lane < 8) wm[wave][64 + lane] = -0.0;
    __syncthreads();
    double x = 1.0 + tid;
    const int nb = (q + 15) >> 4;
    unsigned long long t0 = 0, c0 = 0;
    for (int r = 0; r < kReps; r++) {
        __syncthreads();
        if (r == 1 && tid == 0) {
            t0 = __builtin_amdgcn_s_memrealtime();
            c0 = clock64();
        }
        if (FORM == 0) {
            x = chain<true, false>(sPt, &wm[wave][0], nb, -1, x);
        } else if (FORM == 3) {                  // the uniform operand by readlane (lane u holds slot u)
            x = chain_rl<true, false>(sPt, wm[wave][lane], nb, -1, x);
        } else if (FORM == 1) {                  // LDS reads only: sum of the operands
            d2 acc = d2{0.0, 0.0};
            for (int b = 0; b < nb; b++) {
#pragma unroll
                for (int j = 0; j < 8; j++) acc += ((const d2 *)sPt)[8 * b + j] + ((const d2 *)&wm[wave][0])[8 * b + j];
            }
            x += acc.x + acc.y;
        } else {                                 // the dependent fmas only, operands in registers
            const double a0 = sPt[0], w0 = wm[wave][0];
            for (int b = 0; b < nb; b++) {
#pragma unroll
                for (int j = 0; j < 16; j++) x = fma(w0 + j, a0, x);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        ticks[blockIdx.x] = __builtin_amdgcn_s_memrealtime() - t0;
        ticks[kNWG + blockIdx.x] = clock64() - c0;
    }
    out[(size_t)blockIdx.x * 256 + tid] = x;
}

double g_ghz = 0;   // shader clock of the last run (clock64 / s_memrealtime)

template <int FORM>
double run(double *out, unsigned long long *ticks, int q) {
    (void)hipFuncSetAttribute((const void *)k_chain_lab<FORM>, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds);
    const size_t lds = (size_t)kS * (kCW + 73) * sizeof(double);
    hipLaunchKernelGGL(k_chain_lab<FORM>, dim3(kNWG), dim3(256), lds, 0, out, ticks, q);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(k_chain_lab<FORM>, dim3(kNWG), dim3(256), lds, 0, out, ticks, q);
    (void)hipDeviceSynchronize();
    unsigned long long h[2 * kNWG];
    (void)hipMemcpy(h, ticks, sizeof h, hipMemcpyDeviceToHost);
    double s = 0, c = 0;
    for (int w = 0; w < kNWG; w++) s += (double)h[w], c += (double)h[kNWG + w];
    g_ghz = c / (s * 10.0);
    return s / kNWG * 10.0 / (kReps - 1);   // ns per run
}
}  // namespace

int main() {
    double *out;
    unsigned long long *ticks;
    if (hipMalloc(&out, (size_t)kNWG * 256 * sizeof(double)) != hipSuccess ||
        hipMalloc(&ticks, 2 * kNWG * sizeof(unsigned long long)) != hipSuccess)
        return 1;
    printf("# chain lab: %d workgroups x 256 threads, %d columns per slice, stride %d; ns per chain run (mean over workgroups)\n",
           kNWG, kCW, kS);
    for (int q : {8, 16, 24, 32, 40, 48, 56, 64}) {
        const double a = run<0>(out, ticks, q);
        const double ghz = g_ghz;
        const double b = run<1>(out, ticks, q), c = run<2>(out, ticks, q);
        const double d = run<3>(out, ticks, q);
        printf("q=%2d batches=%d  chain %7.1f ns (%.2f GHz)   readlane chain %7.1f ns   LDS reads only %7.1f ns   fmas only %7.1f ns\n",
               q, (q + 15) >> 4, a, ghz, d, b, c);
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
