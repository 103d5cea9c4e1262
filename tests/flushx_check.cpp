// Host check of k_flushw's XCD-grouped item map (FlushX, flushx_group /
// flushx_item in linearprogramming_amd/csrc/lpg_internal.h): over a sweep of
// tableau shapes, column classes, sub-band heights and tail sizes, the items
// of the 8 group queues cover every (column tile, row) exactly once (tail
// pieces per tile tq = 1 .. 16), start on
// 16-row boundaries and stay inside the rows. Built and run by
// tests/test_item_map.py with g++ (no GPU, no HIP headers).
#define __host__
#define __device__
#include "lpg_internal.h"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace lpg;

static int check(int64_t ntiles, int64_t nloc, int H, int64_t rs_div, int tt, int tq) {
    FlushX X{};
    X.ntiles = ntiles;
    X.nloc = nloc;
    X.H = H;
    const int64_t rb = ((nloc + 8 / H - 1) / (8 / H) + 15) / 16 * 16;
    X.rb = (int32_t)rb;
    X.rs = (int32_t)std::max<int64_t>(16, ((rb + rs_div - 1) / rs_div + 15) / 16 * 16);
    if (X.rs > rb) X.rs = (int32_t)rb;
    X.tt = tt;
    X.tq = tq;
    X.on = 1;
    std::vector<unsigned char> seen((size_t)(ntiles * nloc), 0);
    for (int g = 0; g < 8; g++) {
        const FlushXGroup G = flushx_group(X, g);
        for (int64_t it = 0; it < G.count; it++) {
            int64_t tile, i0, i1;
            flushx_item(X, G, g, it, tile, i0, i1);
            if (tile < 0 || tile >= ntiles || i0 < 0 || i1 > nloc || i0 >= i1 || i0 % 16) {
                printf("bad item: ntiles %ld nloc %ld H %d rs %d tt %d tq %d g %d it %ld -> tile %ld rows %ld..%ld\n",
                       (long)ntiles, (long)nloc, H, X.rs, tt, tq, g, (long)it, (long)tile, (long)i0, (long)i1);
                return 1;
            }
            for (int64_t i = i0; i < i1; i++)
                if (seen[(size_t)(tile * nloc + i)]++) {
                    printf("twice: ntiles %ld nloc %ld H %d rs %d tt %d tile %ld row %ld\n", (long)ntiles, (long)nloc,
                           H, X.rs, tt, (long)tile, (long)i);
                    return 1;
                }
        }
    }
    for (size_t e = 0; e < seen.size(); e++)
        if (!seen[e]) {
            printf("missed: ntiles %ld nloc %ld H %d rs %d tt %d tile %ld row %ld\n", (long)ntiles, (long)nloc, H,
                   X.rs, tt, (long)(e / nloc), (long)(e % nloc));
            return 1;
        }
    return 0;
}

int main() {
    long n = 0;
    for (int64_t ntiles : {1, 3, 7, 8, 9, 64, 65, 385})
        for (int64_t nloc : {1, 15, 16, 17, 100, 127, 600, 1024, 2047, 2048, 5000, 16384})
            for (int H : {1, 2, 4, 8})
                for (int64_t rs_div : {1, 2, 3, 5})
                    for (int tt : {0, 1, 4, 32, 1000})
                        for (int tq : {0, 1, 3, 8, 16}) {
                            if (check(ntiles, nloc, H, rs_div, tt, tq)) return 1;
                            n++;
                        }
    printf("flushx map ok: %ld configurations\n", n);
    return 0;
}
