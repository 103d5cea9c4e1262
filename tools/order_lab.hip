// order_lab.hip — does the ORDER in which the block pass sweeps its items move
// its HBM stream? (round 6; lab only, the product never links this file)
//
// k_flushw's access shape without its arithmetic (tools/hbm_ceiling.hip
// k_wtile_rmw: 8-wave blocks, 256-column tiles, wave tile 16 rows x 32
// columns, one 16-row band loaded ahead, in-place non-temporal RMW) over
// config 3's tableau (16384 rows x 32770 live columns, pitch 49216), with the
// items of IR rows handed out in three orders:
//   ORD 0  column tile fastest over the whole tableau (round 4's global queue)
//   ORD 1  XCD x (= block % 8) owns row band x (2048 rows) and sweeps its
//          tiles within it, IR-row sub-strips (the product's FlushX at H = 1)
//   ORD 2  XCD x owns the column tiles t = x (mod 8) and all XCDs sweep the
//          rows top to bottom together, IR rows at a time: at any moment the
//          chip streams one IR-row strip across every column (the linear
//          RMW stream's shape, 5.84 TB/s in r04_hbm_ceiling.log, vs 5.23 for
//          the tile shape); the pass's P tiles would then stay in their XCD's L2
//   ORD 3  per-tile queues: block b starts on tile b mod ntiles and takes that
//          tile's IR-row strips in row order from the tile's own counter (so its
//          P tile -- B fragments -- would be loaded once, not per item); a
//          block whose tile is exhausted moves on to the next tile with strips
//          left. Every tile's blocks work on adjacent strips.
//   ORD 4  static, no queue: block b keeps tile b mod T (J = ceil(G / ntiles)
//          blocks per tile, T = G / J tiles: 128 of config 3's 129 at G = 512,
//          J = 4) and takes the strips
//          s = j, j + J, j + 2 J, ... (j = b / T): every block's B fragments would
//          be loaded once, and the blocks' fronts start together and drift freely;
//          only those T tiles are swept (bytes counted accordingly)
// Items are dequeued per XCD from an atomic counter (like the product).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/order_lab tools/order_lab.hip
//   tools/order_lab [reps] [rows] [cus]   (rows: 16384 = config 3; 2048 = one rank of it at P = 8;
//                                          cus: the CUs the grid may fill, 2 blocks each -- e.g. the 126
//                                          CUs a P = 8 rank's pivot launch leaves free)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>

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

template <int ORD>
__global__ __launch_bounds__(512) void k_order_rmw(double *__restrict__ T, long ld, long rows, long live, long ir,
                                                   double c, unsigned long long *__restrict__ q) {
    __shared__ long next;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lc = lane & 15, lk = lane >> 4;
    const long ntiles = (live + 255) / 256;
    const int x = (int)(blockIdx.x & 7);
    const d2 p = {0.5, 0.25};
    // items per queue
    long nq;
    if (ORD == 0) nq = ntiles * ((rows + ir - 1) / ir);
    else if (ORD == 1) nq = ntiles * ((rows / 8 + ir - 1) / ir);
    else nq = ((ntiles - x + 7) / 8) * ((rows + ir - 1) / ir);
    unsigned long long *qq = q + (ORD == 0 ? 0 : x);
    long tq = (long)blockIdx.x % ntiles, moved = 0;          // ORD 3: this block's tile, tiles tried
    const long nstrip = (rows + ir - 1) / ir;
    const long J4 = ((long)gridDim.x + ntiles - 1) / ntiles, T4 = std::min(ntiles, (long)gridDim.x / J4);
    long k4 = 0;                                             // ORD 4: this block's strips done
    if (ORD == 4 && (long)blockIdx.x >= T4 * J4) return;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            if (ORD == 4) {
                const long sidx = (long)blockIdx.x / T4 + J4 * k4++;
                next = sidx < nstrip ? ((long)blockIdx.x % T4) * nstrip + sidx : -1;
            } else if (ORD == 3) {
                long v = -1;
                while (moved < ntiles) {
                    const long s = (long)atomicAdd(q + 8 + tq, 1ull);
                    if (s < nstrip) {
                        v = tq * nstrip + s;
                        break;
                    }
                    tq = (tq + 1) % ntiles;
                    moved++;
                }
                next = v;
            } else {
                next = (long)atomicAdd(qq, 1ull);
            }
        }
        __syncthreads();
        const long it = next;
        if (ORD >= 3 ? it < 0 : it >= nq) break;
        long tile, i0, i1;
        if (ORD >= 3) {
            tile = it / nstrip;
            i0 = (it % nstrip) * ir;
            i1 = std::min(i0 + ir, rows);
        } else if (ORD == 0) {
            tile = it % ntiles;
            i0 = (it / ntiles) * ir;
            i1 = std::min(i0 + ir, rows);
        } else if (ORD == 1) {
            const long b0 = x * (rows / 8);
            tile = it % ntiles;
            i0 = b0 + (it / ntiles) * ir;
            i1 = std::min(i0 + ir, b0 + rows / 8);
        } else {
            const long ntx = (ntiles - x + 7) / 8;
            tile = x + 8 * (it % ntx);
            i0 = (it / ntx) * ir;
            i1 = std::min(i0 + ir, rows);
        }
        const long cl = tile * 256 + wave * 32 + 2 * lc;
        const bool in = cl + 1 < live;
        const int nb = (int)((i1 - i0 + 15) / 16);
        auto tload = [&](d2 (&v)[4], int sb) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const long row = i0 + 16 * sb + lk + 4 * r;
                v[r] = (in && row < i1) ? __builtin_nontemporal_load((const d2 *)(T + row * ld + cl)) : d2{0.0, 0.0};
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
                d2 v = t[r];
                v.x = fma(-c, p.x, v.x);
                v.y = fma(-c, p.y, v.y);
                if (in && row < i1) __builtin_nontemporal_store(v, (d2 *)(T + row * ld + cl));
            }
#pragma unroll
            for (int r = 0; r < 4; r++) t[r] = tn[r];
        }
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const long rows = argc > 2 ? atol(argv[2]) : 16384, live = 32770, ld = 49216;
    const int use = argc > 3 ? atoi(argv[3]) : 0;
    double *T;
    unsigned long long *q;
    CHK(hipMalloc(&T, (size_t)(rows + 16) * ld * 8));
    CHK(hipMemset(T, 0, (size_t)(rows + 16) * ld * 8));
    const long nq = 8 + (live + 255) / 256;
    CHK(hipMalloc(&q, nq * sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double moved = 16.0 * rows * live;
    // a CU-masked stream (hipExtStreamCreateWithCUMask): the grid may only use `use` CUs, as a pass
    // beside a pivot launch that holds the others would
    hipStream_t sm = 0;
    if (use > 0 && use < cus) {
        std::vector<uint32_t> mask((cus + 31) / 32, 0u);
        for (int c = 0; c < use; c++) mask[c / 32] |= 1u << (c % 32);
        CHK(hipExtStreamCreateWithCUMask(&sm, (uint32_t)mask.size(), mask.data()));
        cus = use;
    }
    printf("# order lab: %ld rows x %ld live columns (pitch %ld), 8-wave blocks x 2 per CU on %d CUs, GB/s = read + "
           "written / time, best and median of %d\n", rows, live, ld, cus, reps);
    for (int rep2 = 0; rep2 < 2; rep2++)
        for (int ord = 0; ord < 5; ord++)
            for (long ir : {16L, 64L, 128L, 256L, 1024L, 2048L}) {
                if (ord == 1 && ir > rows / 8) continue;
                if (ord < 4 && getenv("LAB_ORD4_ONLY")) continue;
                // LAB_ORD=o LAB_IR=r: one configuration only (for rocprofv3 --pmc passes)
                if (getenv("LAB_ORD") && atoi(getenv("LAB_ORD")) != ord) continue;
                if (getenv("LAB_IR") && atol(getenv("LAB_IR")) != ir) continue;
                auto k = ord == 0 ? k_order_rmw<0> : ord == 1 ? k_order_rmw<1> : ord == 2 ? k_order_rmw<2>
                       : ord == 3 ? k_order_rmw<3> : k_order_rmw<4>;
                std::vector<float> t;
                for (int r = 0; r <= reps; r++) {
                    CHK(hipMemsetAsync(q, 0, nq * sizeof(unsigned long long), sm));
                    CHK(hipEventRecord(e0, sm));
                    hipLaunchKernelGGL(k, dim3(2 * cus), dim3(512), 0, sm, T, ld, rows, live, ir, 1e-3, q);
                    CHK(hipEventRecord(e1, sm));
                    CHK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHK(hipEventElapsedTime(&ms, e0, e1));
                    if (r) t.push_back(ms);          // the first launch warms up
                }
                std::sort(t.begin(), t.end());
                double mv = moved;
                if (ord == 4) {   // only T4 full tiles are swept
                    const long ntl = (live + 255) / 256, J = (2L * cus + ntl - 1) / ntl, T4 = std::min(ntl, 2L * cus / J);
                    mv = 16.0 * rows * std::min(live, T4 * 256);
                }
                printf("ORD %d rows/item %5ld : best %7.1f  median %7.1f GB/s  (%.3f ms)\n", ord, ir,
                       mv / (t[0] * 1e-3) / 1e9, mv / (t[t.size() / 2] * 1e-3) / 1e9, t[0]);
                fflush(stdout);
            }
    return 0;
}
