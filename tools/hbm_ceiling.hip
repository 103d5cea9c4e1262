// hbm_ceiling.hip — what the HBM of this box streams, for the block pass's
// question: is an in-place read-modify-write held below
// a copy, and does an out-of-place RMW reach the copy's rate?
//
// Five streams over 16-byte lanes, byte counts as the pass counts them (read +
// written bytes):
//   read   sum of every element (one store per thread at the end)
//   write  a constant into every element
//   copy   dst = src                       (two buffers)
//   rmw    x = fma(-c, p, x) in place      (k_flushw's traffic shape)
//   rmwo   dst = fma(-c, p, src)           (an out-of-place pass)
// Two address layouts: grid-stride (consecutive workgroups on consecutive
// 4 KB) and chunked (each workgroup one contiguous span of n / grid), U
// 16-byte loads in flight per lane, plain or non-temporal loads and stores,
// grids of 1-8 workgroups of 256 per CU. 4 GiB per buffer (config 3's live
// region is 4.3 GB). tools only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                                     \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

enum { OP_READ, OP_WRITE, OP_COPY, OP_RMW, OP_RMWO };

template <bool NT>
__device__ __forceinline__ d2 ld(const d2 *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(d2 *p, d2 v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// n: 16-byte elements (a multiple of 256 * U * grid for both layouts)
template <int OP, int U, bool CHUNK, bool NT>
__global__ __launch_bounds__(256) void k_stream(const d2 *__restrict__ src, d2 *__restrict__ dst, size_t n, double c,
                                                d2 *__restrict__ sink) {
    const d2 p = {0.5, 0.25};
    size_t base, step, end;
    if (CHUNK) {
        const size_t span = n / gridDim.x;
        base = (size_t)blockIdx.x * span + threadIdx.x;
        step = 256;
        end = (size_t)(blockIdx.x + 1) * span;
    } else {
        base = (size_t)blockIdx.x * 256 + threadIdx.x;
        step = (size_t)gridDim.x * 256;
        end = n;
    }
    d2 acc = {0.0, 0.0};
    for (size_t i = base; i + (U - 1) * step < end; i += U * step) {
        d2 v[U];
        if (OP != OP_WRITE) {
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = ld<NT>(src + i + u * step);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (OP == OP_READ) {
                acc += v[u];
            } else if (OP == OP_WRITE) {
                st<NT>(dst + i + u * step, d2{c, c});
            } else if (OP == OP_COPY) {
                st<NT>(dst + i + u * step, v[u]);
            } else {
                d2 x = v[u];
                x.x = fma(-c, p.x, x.x);
                x.y = fma(-c, p.y, x.y);
                st<NT>(dst + i + u * step, x);
            }
        }
    }
    if (OP == OP_READ && acc.x == 12345.678) sink[threadIdx.x] = acc;
}


// The block pass's access shape without its arithmetic: a row-major tableau
// (config 3: 16384 rows, pitch 49216 doubles), the first `live` columns of
// every row read and written in place, in items of TW columns x IR rows
// (column tile fastest, like k_flushw's dequeue order), a 256-thread
// workgroup covering 256 / (TW / 2) rows per access, U accesses in flight
// per lane. Grid-stride over items (no dequeue).
template <int TW, int U>
__global__ __launch_bounds__(256) void k_tile_rmw(double *__restrict__ T, long ld, long rows, long live, long ir,
                                                  double c) {
    constexpr int LPR = TW / 2;                 // lanes per row (16 B each)
    constexpr int RPA = 256 / LPR;              // rows per access
    const d2 p = {0.5, 0.25};
    const long ntiles = (live + TW - 1) / TW;
    const long nitems = ntiles * ((rows + ir - 1) / ir);
    const int lc = threadIdx.x % LPR, lr = threadIdx.x / LPR;
    for (long item = blockIdx.x; item < nitems; item += gridDim.x) {
        const long tile = item % ntiles, strip = item / ntiles;
        const long c0 = tile * TW + 2 * lc;
        const bool in = c0 + 1 < live;
        const long r0 = strip * ir, r1 = r0 + ir < rows ? r0 + ir : rows;
        for (long rb = r0; rb < r1; rb += RPA * U) {
            d2 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const long r = rb + lr + u * RPA;
                v[u] = (in && r < r1) ? __builtin_nontemporal_load((const d2 *)(T + r * ld + c0)) : d2{0.0, 0.0};
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const long r = rb + lr + u * RPA;
                d2 x = v[u];
                x.x = fma(-c, p.x, x.x);
                x.y = fma(-c, p.y, x.y);
                if (in && r < r1) __builtin_nontemporal_store(x, (d2 *)(T + r * ld + c0));
            }
        }
    }
}

// k_flushw's own access shape without its arithmetic (round 4, layout
// question): 8-wave blocks over 256-column x IR-row items (column tile
// fastest), wave tile 16 rows x 32 columns, lane (lk, lc) = column pair 2 lc,
// rows lk + 4 r, one 16-row band loaded ahead. BLK = 0: row-major with pitch
// ld; BLK = 1: a blocked layout where every 16-row x 256-column tile is one
// contiguous 32 KB block (band-major within a column tile), so an item is
// one contiguous stream.
template <int BLK>
__global__ __launch_bounds__(512) void k_wtile_rmw(double *__restrict__ T, long ld, long rows, long live, long ir,
                                                   double c) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    const long ntiles = (live + 255) / 256, nbands = (rows + 15) / 16;
    const long nitems = ntiles * ((rows + ir - 1) / ir);
    const d2 p = {0.5, 0.25};
    auto addr = [&](long row, long col) -> double * {
        if (!BLK) return T + row * ld + col;
        const long t = col >> 8, b = row >> 4;
        return T + (((t * nbands + b) << 4) + (row & 15)) * 256 + (col & 255);
    };
    for (long item = blockIdx.x; item < nitems; item += gridDim.x) {
        const long tile = item % ntiles, strip = item / ntiles;
        const long cl = tile * 256 + wave * 32 + 2 * lc;
        const bool in = cl + 1 < live;
        const long i0 = strip * ir, i1 = i0 + ir < rows ? i0 + ir : rows;
        const int nb = (int)((i1 - i0 + 15) / 16);
        auto tload = [&](d2 (&x)[4], int sb) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const long row = i0 + 16 * sb + lk + 4 * r;
                x[r] = (in && row < i1) ? __builtin_nontemporal_load((const d2 *)addr(row, cl)) : d2{0.0, 0.0};
            }
        };
        d2 t[4];
        tload(t, 0);
        for (int sb = 0; sb < nb; sb++) {
            d2 tn[4];
            if (sb + 1 < nb) tload(tn, sb + 1);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const long row = i0 + 16 * sb + lk + 4 * r;
                d2 x = t[r];
                x.x = fma(-c, p.x, x.x);
                x.y = fma(-c, p.y, x.y);
                if (in && row < i1) __builtin_nontemporal_store(x, (d2 *)addr(row, cl));
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
}

typedef void (*TFn)(double *, long, long, long, long, double);
template <int TW>
static TFn tile_u(int u) {
    switch (u) {
        case 2: return k_tile_rmw<TW, 2>;
        case 4: return k_tile_rmw<TW, 4>;
        case 8: return k_tile_rmw<TW, 8>;
        default: return k_tile_rmw<TW, 16>;
    }
}
static TFn tile_kernel(int tw, int u) {
    switch (tw) {
        case 128: return tile_u<128>(u);
        case 256: return tile_u<256>(u);
        default: return tile_u<512>(u);
    }
}

typedef void (*KFn)(const d2 *, d2 *, size_t, double, d2 *);

template <int OP, int U, bool CHUNK, bool NT>
static KFn pick() {
    return k_stream<OP, U, CHUNK, NT>;
}

template <int OP, bool CHUNK, bool NT>
static KFn pick_u(int u) {
    switch (u) {
        case 1: return pick<OP, 1, CHUNK, NT>();
        case 2: return pick<OP, 2, CHUNK, NT>();
        case 4: return pick<OP, 4, CHUNK, NT>();
        default: return pick<OP, 8, CHUNK, NT>();
    }
}
template <int OP>
static KFn pick_all(int u, bool chunk, bool nt) {
    if (chunk) return nt ? pick_u<OP, true, true>(u) : pick_u<OP, true, false>(u);
    return nt ? pick_u<OP, false, true>(u) : pick_u<OP, false, false>(u);
}
static KFn kernel(int op, int u, bool chunk, bool nt) {
    switch (op) {
        case OP_READ: return pick_all<OP_READ>(u, chunk, nt);
        case OP_WRITE: return pick_all<OP_WRITE>(u, chunk, nt);
        case OP_COPY: return pick_all<OP_COPY>(u, chunk, nt);
        case OP_RMW: return pick_all<OP_RMW>(u, chunk, nt);
        default: return pick_all<OP_RMWO>(u, chunk, nt);
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    if (getenv("LAB_LAYOUT")) {   // the pass's wave-tile shape: pitch paddings and the blocked layout
        int cus = 0;
        CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        const long rows = 16384, live = 32770, ld0 = 49216;
        const long maxpad = 1024;
        double *T;
        const size_t bytes = (size_t)(rows + 16) * (ld0 + maxpad) * 8;
        CHK(hipMalloc(&T, bytes));
        CHK(hipMemset(T, 0, bytes));
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0));
        CHK(hipEventCreate(&e1));
        const double moved = 16.0 * rows * live;
        printf("# layout lab: %ld x %ld live columns, GB/s = bytes read + written / time, best and median of %d\n", rows,
               live, reps);
        for (int rep2 = 0; rep2 < 2; rep2++)
            for (long ir : {1024L, 2048L})
                for (int blk = 0; blk < 2; blk++)
                    for (long pad : {0L, 8L, 32L, 64L, 128L, 256L, 512L, 1024L}) {
                        if (blk && pad) continue;
                        const long ld = ld0 + pad;
                        const TFn k = blk ? k_wtile_rmw<1> : k_wtile_rmw<0>;
                        const int grid = 2 * cus;
                        hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, 0, T, ld, rows, live, ir, 1e-3);
                        CHK(hipDeviceSynchronize());
                        std::vector<float> t;
                        for (int r = 0; r < reps; r++) {
                            CHK(hipEventRecord(e0));
                            hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, 0, T, ld, rows, live, ir, 1e-3);
                            CHK(hipEventRecord(e1));
                            CHK(hipEventSynchronize(e1));
                            float ms;
                            CHK(hipEventElapsedTime(&ms, e0, e1));
                            t.push_back(ms);
                        }
                        std::sort(t.begin(), t.end());
                        printf("%-9s pitch %6ld (+%4ld) rows/item %5ld : best %7.1f  median %7.1f GB/s  (%.3f ms)\n",
                               blk ? "blocked" : "row-major", blk ? 0L : ld, pad, ir, moved / t[0] / 1e6,
                               moved / t[t.size() / 2] / 1e6, t[0]);
                        fflush(stdout);
                    }
        CHK(hipFree(T));
        return 0;
    }
    const size_t bytes = (size_t)4 << 30;
    const size_t n = bytes / 16;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    d2 *A, *B, *S;
    CHK(hipMalloc(&A, bytes));
    CHK(hipMalloc(&B, bytes));
    CHK(hipMalloc(&S, 256 * sizeof(d2)));
    CHK(hipMemset(A, 0, bytes));
    CHK(hipMemset(B, 0, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const char *names[] = {"read", "write", "copy", "rmw", "rmwo"};
    printf("# hbm_ceiling: %d CUs, %zu MiB per buffer, best and median of %d launches; GB/s = (read + written bytes) / time\n",
           cus, bytes >> 20, reps);
    const int wpcs[] = {1, 2, 4, 8};
    const int us[] = {1, 2, 4, 8};
    for (int op = 0; op < 5; op++) {
        double best_all = 0;
        char best_cfg[128] = "";
        for (int chunk = 0; chunk < 2; chunk++)
            for (int nt = 0; nt < 2; nt++)
                for (int wpc : wpcs)
                    for (int u : us) {
                        const int grid = wpc * cus;
                        // both layouts need n divisible by grid * 256 * u: trim the tail (< 0.1%)
                        const size_t unit = (size_t)grid * 256 * u;
                        const size_t nn = n / unit * unit;
                        KFn k = kernel(op, u, chunk, nt);
                        const d2 *src = A;
                        d2 *dst = (op == OP_RMW) ? A : B;
                        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, src, dst, nn, 1e-3, S);
                        CHK(hipDeviceSynchronize());
                        std::vector<float> t;
                        for (int r = 0; r < reps; r++) {
                            CHK(hipEventRecord(e0));
                            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, src, dst, nn, 1e-3, S);
                            CHK(hipEventRecord(e1));
                            CHK(hipEventSynchronize(e1));
                            float ms;
                            CHK(hipEventElapsedTime(&ms, e0, e1));
                            t.push_back(ms);
                        }
                        std::sort(t.begin(), t.end());
                        const double moved = (double)nn * 16 * ((op == OP_READ || op == OP_WRITE) ? 1 : 2);
                        const double gbs = moved / t[0] / 1e6, gbm = moved / t[t.size() / 2] / 1e6;
                        printf("%-5s %-6s %-5s wg/CU %d U %d : best %7.1f  median %7.1f GB/s  (%.3f ms)\n", names[op],
                               chunk ? "chunk" : "stride", nt ? "nt" : "plain", wpc, u, gbs, gbm, t[0]);
                        if (gbs > best_all) {
                            best_all = gbs;
                            snprintf(best_cfg, sizeof best_cfg, "%s %s wg/CU %d U %d", chunk ? "chunk" : "stride",
                                     nt ? "nt" : "plain", wpc, u);
                        }
                    }
        printf("## %s best %.1f GB/s (%s)\n", names[op], best_all, best_cfg);
        fflush(stdout);
    }
    // the block pass's shape: config 3's tableau, its 32770 live columns
    CHK(hipFree(A));
    CHK(hipFree(B));
    {
        const long rows = 16384, ld = 49216, live = 32770;
        double *T;
        CHK(hipMalloc(&T, (size_t)(rows + 1) * ld * 8));
        CHK(hipMemset(T, 0, (size_t)(rows + 1) * ld * 8));
        const double moved = 16.0 * rows * live;
        double best_all = 0;
        char best_cfg[128] = "";
        for (int tw : {128, 256, 512})
            for (long ir : {64L, 512L, 16384L})
                for (int wpc : {1, 2, 4, 8})
                    for (int u : {2, 4, 8, 16}) {
                        const int grid = wpc * cus;
                        TFn k = tile_kernel(tw, u);
                        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, T, ld, rows, live, ir, 1e-3);
                        CHK(hipDeviceSynchronize());
                        std::vector<float> t;
                        for (int r = 0; r < reps; r++) {
                            CHK(hipEventRecord(e0));
                            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, T, ld, rows, live, ir, 1e-3);
                            CHK(hipEventRecord(e1));
                            CHK(hipEventSynchronize(e1));
                            float ms;
                            CHK(hipEventElapsedTime(&ms, e0, e1));
                            t.push_back(ms);
                        }
                        std::sort(t.begin(), t.end());
                        const double gbs = moved / t[0] / 1e6, gbm = moved / t[t.size() / 2] / 1e6;
                        printf("tile  TW %3d rows/item %5ld wg/CU %d U %2d : best %7.1f  median %7.1f GB/s  (%.3f ms)\n",
                               tw, ir, wpc, u, gbs, gbm, t[0]);
                        if (gbs > best_all) {
                            best_all = gbs;
                            snprintf(best_cfg, sizeof best_cfg, "TW %d rows/item %ld wg/CU %d U %d", tw, ir, wpc, u);
                        }
                    }
        printf("## tile best %.1f GB/s (%s)\n", best_all, best_cfg);
        CHK(hipFree(T));
    }
    return 0;
}
