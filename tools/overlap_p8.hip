// overlap_p8.hip -- round 6 lab for DESIGN.md §5.1: the
// sliding-window overlap needs a P = 8 rank's pivot launch and the previous
// block's pass to run AT THE SAME TIME on disjoint CUs. This measures exactly
// that on one MI355X, with the product's own code on both sides:
//   * the pivot loop: liblpg.so (dlopen'ed with RTLD_DEEPBIND, so its symbols
//     stay its own) on a P = 8 rank's stand-in, m = 2048 rows x 32768
//     structural columns, dense LP, K pending pivots per block (LPG_DEFER);
//   * the pass beside it: this file's copy of lpg::k_flushw (the product
//     source, included) over a separate tableau of the same shape (the 32769
//     live columns of a rank), K slots, the product's XCD item map, launched
//     back to back from a second host thread on a CU-masked stream of BG CUs.
// Three phases: the loop alone, the loop with the pass beside it, the pass
// alone on its CUs. Run it under rocprofv3 --kernel-trace --stats for the
// per-kernel averages (the pass beside it is the <K, 2, 2, 4> instance, the
// library's own pass the <K, 2, 3, 4> one, so the two stay apart).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/overlap_p8 tools/overlap_p8.hip -ldl -lpthread
//   tools/overlap_p8 [K=32] [blocks=60] [bg_cus=126] [bg_first_cu=130]   (env OV_PHASE=alone|beside, OV_BG_LDS=1)
#include "../linearprogramming_amd/csrc/lpg_kernels.hip"

#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../include/lpg.h"

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

namespace lpg {
__global__ void k_fillr_ov(double *p, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (seed + (uint64_t)i) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = ((double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5) * 1e-3;
    }
}
__global__ void k_zero_cols_ov(double *P, int64_t ld, int64_t c0, int K) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)K * ld; i += (int64_t)gridDim.x * blockDim.x)
        if (i % ld >= c0) P[i] = 0.0;
}
}  // namespace lpg
using namespace lpg;

struct Api {
    int (*create)(lpg_ctx **, int, int64_t, int64_t, uint32_t);
    int (*generate)(lpg_ctx *, int64_t, uint64_t, int);
    int (*solve)(lpg_ctx *, int64_t, int, lpg_result *);
    int (*enqueue)(lpg_ctx *, int64_t, int);
    int (*sync)(lpg_ctx *, lpg_result *);
    int (*prepare)(lpg_ctx *, int);
    int (*reserve_log)(lpg_ctx *, int64_t);
    int (*info)(const lpg_ctx *, lpg_info_t *);
    const char *(*last_error)(const lpg_ctx *);
    const char *(*stamp)(void);
    void (*destroy)(lpg_ctx *);
};

template <typename F>
static void sym(void *h, const char *name, F &f) {
    f = (F)dlsym(h, name);
    if (!f) {
        printf("dlsym %s: %s\n", name, dlerror());
        exit(1);
    }
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 32;
    const int nblk = argc > 2 ? atoi(argv[2]) : 60;
    const int bg = argc > 3 ? atoi(argv[3]) : 126;
    const int bg0 = argc > 4 ? atoi(argv[4]) : 130;
    if (K != 32 && K != 64) {
        printf("K must be 32 or 64\n");
        return 2;
    }
    char kenv[16];
    snprintf(kenv, sizeof kenv, "%d", K);
    setenv("LPG_DEFER", kenv, 1);
    const char *so = getenv("LPG_SO") ? getenv("LPG_SO") : "linearprogramming_amd/liblpg.so";
    void *h = dlopen(so, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    if (!h) {
        printf("dlopen %s: %s\n", so, dlerror());
        return 1;
    }
    Api A;
    sym(h, "lpg_create", A.create);
    sym(h, "lpg_generate", A.generate);
    sym(h, "lpg_solve", A.solve);
    sym(h, "lpg_enqueue", A.enqueue);
    sym(h, "lpg_sync", A.sync);
    sym(h, "lpg_prepare", A.prepare);
    sym(h, "lpg_reserve_log", A.reserve_log);
    sym(h, "lpg_info", A.info);
    sym(h, "lpg_last_error", A.last_error);
    sym(h, "lpg_build_stamp", A.stamp);
    sym(h, "lpg_destroy", A.destroy);

    const int64_t m = 2048, nstruct = 32768, ncols = 1 + nstruct + m;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    if (bg < 1 || bg0 < 0 || bg0 + bg > cus) {
        printf("bad CU range %d + %d of %d\n", bg0, bg, cus);
        return 2;
    }

    // the pivot loop (the library)
    lpg_ctx *ctx = nullptr;
    if (A.create(&ctx, 0, m, ncols, LPG_FLAG_NO_LOG) || A.generate(ctx, nstruct, 20220518ull, LPG_GEN_DENSE)) {
        printf("create/generate failed: %s\n", ctx ? A.last_error(ctx) : "?");
        return 1;
    }
    lpg_result res{};
    if (A.solve(ctx, 4 * K, LPG_RULE_DANTZIG, &res) || A.prepare(ctx, LPG_RULE_DANTZIG) ||
        A.reserve_log(ctx, 3 * (int64_t)nblk * K)) {
        printf("warm-up failed: %s\n", A.last_error(ctx));
        return 1;
    }
    lpg_info_t inf{};
    A.info(ctx, &inf);
    printf("# overlap_p8: liblpg %s, %lld x %lld (ld %lld), K = %d, pivot workgroups %d, region %d, trade %d; "
           "the pass beside it on CUs %d..%d (%d of %d)\n",
           A.stamp(), (long long)m, (long long)ncols, (long long)inf.ld, inf.defer_k, inf.pivot_wg, inf.region,
           inf.column_trade, bg0, bg0 + bg - 1, bg, cus);
    if (inf.defer_k != K || inf.pivot_wg <= 0) {
        printf("not the persistent launch at K = %d\n", K);
        return 1;
    }

    // the pass beside it: its own tableau of the same shape, K slots
    const int64_t ld = (ncols + 63) / 64 * 64, n = m * ld, cs = m;
    double *T, *Pbuf, *Cbuf;
    DevState *st;
    CHK(hipMalloc(&T, n * 8));
    CHK(hipMalloc(&Pbuf, (size_t)K * ld * 8));
    CHK(hipMalloc(&Cbuf, (size_t)K * cs * 8));
    CHK(hipMalloc(&st, sizeof(DevState)));
    hipLaunchKernelGGL(k_fillr_ov, dim3(4096), dim3(256), 0, 0, T, n, 1ull);
    hipLaunchKernelGGL(k_fillr_ov, dim3(1024), dim3(256), 0, 0, Pbuf, (int64_t)K * ld, 2ull);
    hipLaunchKernelGGL(k_fillr_ov, dim3(1024), dim3(256), 0, 0, Cbuf, (int64_t)K * cs, 3ull);
    hipLaunchKernelGGL(k_zero_cols_ov, dim3(1024), dim3(256), 0, 0, Pbuf, ld, nstruct + 1, K);
    CHK(hipDeviceSynchronize());
    Geo g{};
    g.T = T;
    g.ld = ld;
    g.nloc = m;
    g.nobj = 1;
    g.ncols = ncols;
    g.nact = ncols - 1;
    g.m = m;
    // launch_flush_main's geometry at K = 32 / 64 on bg CUs: 128-column tiles x
    // 3 blocks per CU (K = 32) or 256-column tiles x 1 block of 8 waves (K = 64)
    const int tw = K == 64 ? 256 : 128;
    const int64_t ntiles = (ncols + tw - 1) / tw;
    const int64_t rows = 2048, nitems = flush_nitems(ntiles, rows, m);
    const int bpc = K == 64 ? 1 : 3;
    const FlushX X = flushx_plan(ntiles, m, K, (int64_t)bg * bpc, -1);
    const unsigned grid = (unsigned)(bg * bpc);
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int c = bg0; c < bg0 + bg; c++) mask[c / 32] |= 1u << (c % 32);
    hipStream_t bs;
    CHK(hipExtStreamCreateWithCUMask(&bs, (uint32_t)mask.size(), mask.data()));
    DevState *hst;
    CHK(hipHostMalloc((void **)&hst, sizeof(DevState)));
    *hst = DevState{};
    hst->npend = K;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    // OV_BG_LDS=1: every pass block also reserves dynamic LDS so that its CU has no
    // room left for a pivot-launch workgroup (~150 KB): the dispatcher cannot put
    // the launch beside the pass, the CU sets stay disjoint without a mask on the
    // library's stream (K = 32: 3 x (8 + 44) KB per CU; K = 64: 16 + 140 KB)
    const bool pad = getenv("OV_BG_LDS") && atoi(getenv("OV_BG_LDS")) != 0;
    const size_t dyn = !pad ? 0 : K == 64 ? 140 * 1024 : 44 * 1024;
    if (dyn) {
        CHK(hipFuncSetAttribute((const void *)k_flushw<64, 2, 1, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                140 * 1024));
        CHK(hipFuncSetAttribute((const void *)k_flushw<32, 2, 2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                44 * 1024));
    }
    auto bg_launch = [&]() {
        CHK(hipMemcpyAsync(st, hst, sizeof(DevState), hipMemcpyHostToDevice, bs));
        if (K == 64)
            hipLaunchKernelGGL((k_flushw<64, 2, 1, 8>), dim3(grid), dim3(512), dyn, bs, T, g, st, Pbuf, Cbuf, cs, ntiles,
                               nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        else
            hipLaunchKernelGGL((k_flushw<32, 2, 2, 4>), dim3(grid), dim3(256), dyn, bs, T, g, st, Pbuf, Cbuf, cs, ntiles,
                               nitems, rows, 1, X, (const int32_t *)nullptr, (const int64_t *)nullptr,
                               (const int32_t *)nullptr);
        CHK(hipGetLastError());
    };
    // the pass alone on its CUs (also the warm-up of its instance)
    auto bg_alone = [&](int reps) {
        for (int r = 0; r < 3; r++) bg_launch();
        CHK(hipStreamSynchronize(bs));
        CHK(hipEventRecord(e0, bs));
        for (int r = 0; r < reps; r++) bg_launch();
        CHK(hipEventRecord(e1, bs));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    const float bg_ms0 = bg_alone(50);
    printf("pass alone on %d CUs: %.3f ms per %d-slot pass (%.0f GB/s, %d blocks)\n", bg, bg_ms0, K,
           16.0 * m * (nstruct + 1) / (bg_ms0 * 1e-3) / 1e9, grid);

    auto loop = [&](const char *name, bool beside) {
        std::atomic<bool> stop{false};
        std::atomic<long> launched{0};
        std::thread th;
        if (beside) {
            th = std::thread([&]() {
                // keep a few passes queued; the stream runs them back to back
                while (!stop.load()) {
                    for (int r = 0; r < 4; r++) bg_launch();
                    launched += 4;
                    CHK(hipStreamSynchronize(bs));
                }
            });
            std::this_thread::sleep_for(std::chrono::milliseconds(30));
        }
        // the same LP and pivots in every phase: regenerate, warm up (the replayed graph, 4 blocks)
        lpg_result r0{}, r1{};
        if (A.generate(ctx, nstruct, 20220518ull, LPG_GEN_DENSE) || A.solve(ctx, 4 * K, LPG_RULE_DANTZIG, &r0) ||
            A.prepare(ctx, LPG_RULE_DANTZIG) || A.sync(ctx, &r0)) {
            printf("%s: regenerate / warm-up: %s\n", name, A.last_error(ctx));
            exit(1);
        }
        const long l0 = launched.load();
        const auto t0 = std::chrono::steady_clock::now();
        if (A.enqueue(ctx, (int64_t)nblk * K, LPG_RULE_DANTZIG) || A.sync(ctx, &r1)) {
            printf("%s: %s\n", name, A.last_error(ctx));
            exit(1);
        }
        const auto t1 = std::chrono::steady_clock::now();
        const long l1 = launched.load();
        if (beside) {
            stop = true;
            th.join();
        }
        const double s = std::chrono::duration<double>(t1 - t0).count();
        const int64_t piv = r1.pivots - r0.pivots;
        lpg_info_t in{};
        A.info(ctx, &in);
        printf("%-34s %lld pivots in %.2f ms: %.0f pivots/s, %.3f ms per %d-pivot block; status %d, residency "
               "fallbacks %d, pivot workgroups %d%s\n",
               name, (long long)piv, s * 1e3, piv / s, s * 1e3 / ((double)piv / K), K, r1.status,
               in.residency_fallbacks, in.pivot_wg,
               beside ? (" (passes beside it: " + std::to_string(l1 - l0) + "+ launched)").c_str() : "");
        fflush(stdout);
        return piv / s;
    };
    // OV_PHASE=alone | beside: one kind of phase only (a rocprofv3 --stats run per kind)
    const char *ph = getenv("OV_PHASE");
    const bool run_alone = !ph || strcmp(ph, "beside") != 0, run_beside = !ph || strcmp(ph, "alone") != 0;
    for (int rep = 0; rep < 2; rep++) {
        if (run_alone) loop("the loop alone", false);
        if (run_beside) loop("the loop with the pass beside it", true);
    }
    const float bg_ms1 = bg_alone(50);
    printf("pass alone on %d CUs (again): %.3f ms\n", bg, bg_ms1);
    A.destroy(ctx);
    CHK(hipFree(T));
    CHK(hipFree(Pbuf));
    CHK(hipFree(Cbuf));
    CHK(hipFree(st));
    return 0;
}
