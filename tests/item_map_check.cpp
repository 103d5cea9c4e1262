// Host-side check of the block pass's item map (lpg_internal.h flush_nitems /
// flush_item, used by k_flushw on the device): for every (ntiles, rows, nloc)
// in the sweep, the items cover every (column tile, constraint row) exactly
// once, each item is a non-empty row range of one tile, whole items are
// `rows` tall, and with the tail on the last two strips are cut into items of
// rows / 4. Built and run by tests/test_item_map.py (g++ on the CPU).
#define __host__
#define __device__
#include <stdio.h>

#include <vector>

#include "lpg_internal.h"

using lpg::flush_item;
using lpg::flush_nitems;
using lpg::flush_tail_rows;

static int check(int64_t ntiles, int64_t rows, int64_t nloc) {
    const int64_t n = flush_nitems(ntiles, rows, nloc);
    const int64_t h = rows < 0 ? -rows : rows;
    const int64_t tr = flush_tail_rows(rows, nloc);
    std::vector<unsigned char> seen((size_t)(ntiles * nloc), 0);
    for (int64_t it = 0; it < n; it++) {
        int64_t t, i0, i1;
        flush_item(it, ntiles, rows, nloc, t, i0, i1);
        if (t < 0 || t >= ntiles || i0 < 0 || i0 >= i1 || i1 > nloc) {
            printf("bad item: ntiles %ld rows %ld nloc %ld item %ld -> tile %ld [%ld, %ld)\n", (long)ntiles,
                   (long)rows, (long)nloc, (long)it, (long)t, (long)i0, (long)i1);
            return 1;
        }
        const int64_t want = (tr && i0 >= ((nloc + h - 1) / h - 2) * h) ? tr : h;
        if (i1 - i0 != want && i1 != nloc) {
            printf("item height: ntiles %ld rows %ld nloc %ld item %ld [%ld, %ld) want %ld\n", (long)ntiles, (long)rows,
                   (long)nloc, (long)it, (long)i0, (long)i1, (long)want);
            return 1;
        }
        for (int64_t i = i0; i < i1; i++) {
            unsigned char &s = seen[(size_t)(t * nloc + i)];
            if (s) {
                printf("covered twice: ntiles %ld rows %ld nloc %ld tile %ld row %ld\n", (long)ntiles, (long)rows,
                       (long)nloc, (long)t, (long)i);
                return 1;
            }
            s = 1;
        }
    }
    for (size_t k = 0; k < seen.size(); k++)
        if (!seen[k]) {
            printf("not covered: ntiles %ld rows %ld nloc %ld tile %ld row %ld\n", (long)ntiles, (long)rows, (long)nloc,
                   (long)(k / nloc), (long)(k % nloc));
            return 1;
        }
    return 0;
}

int main() {
    long cases = 0;
    for (int64_t ntiles : {1, 2, 3, 7, 64, 129, 193})
        for (int64_t rows : {64, 128, 256, 512, 1024, 2048, 4096, 8192})
            for (int sign : {1, -1})
                for (int64_t nloc : {1, 15, 16, 17, 63, 64, 65, 200, 511, 512, 513, 1000, 2048, 4095, 4096, 4097, 16384,
                                     16385, 65536})
                    if (ntiles * nloc <= (int64_t)30000000) {
                        if (check(ntiles, sign * rows, nloc)) return 1;
                        cases++;
                    }
    printf("ok %ld\n", cases);
    return 0;
}
