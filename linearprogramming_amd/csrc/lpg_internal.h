// lpg_internal.h — device-side data structures shared by the kernels
// (lpg_kernels.hip) and the context / C-ABI layer (lpg_ctx.hip).
//
// Per pivot t the device keeps everything the host would otherwise have to
// read back, so the host enqueues pivots without synchronising:
//   slot[t & 1]   entering column k_t (chosen by select_{t-1}), leaving row
//                 r_t (chosen by prep_t from the gathered ratio candidates),
//                 and a status that, once non-RUNNING, turns every later
//                 kernel into a no-op and is copied forward slot to slot.
//   C[t & 1]      column k_t of T_t (the pivot-column snapshot), written by
//                 select_{t-1} and read by update_t.
//   P             the normalised pivot row of T_t, written by prep_t.
//
// Deferred (blocked) updates, the default for large tableaus: the constraint
// rows of T lag behind by up to K pending pivots whose P rows, C columns and
// pivot rows are kept (Defer); the objective row(s) stay current. Any entry
// of the current tableau is the per-element chain
//   x = T_base[i][j];  for q in pending order:
//       x = (i == r_q) ? P_q[j] : fma(-C_q[i], P_q[j], x)
// which is, operation for operation, what K eager updates compute; prep
// evaluates it for the pivot row, select for columns 0 and k, and k_flush
// applies it to the whole block of constraint rows in one HBM pass.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace lpg {

constexpr int kBlock = 256;          // threads per block everywhere (4 waves of 64)
constexpr int kMaxSelBlocks = 512;   // ratio-test partials per rank
#ifndef LPG_DEFER_MAX
#define LPG_DEFER_MAX 128            // include/lpg.h
#endif

enum : int32_t { RUNNING = 0, OPTIMAL = 1, UNBOUNDED = 2, INFEASIBLE = 3, ITER_LIMIT = 4, NUMERIC = 5 };
enum : int { RULE_DANTZIG = 0, RULE_BLAND = 1 };

struct Slot {                 // 32 B
    int64_t k;                // entering column (1-based)
    int64_t r;                // leaving row (global)
    int32_t status;
    int32_t pad0;
    int64_t dpend;            // dual deferred path: the objective row owes the previous pivot's update (lpg_dual.hip)
};

struct DevState {
    Slot    slot[2];
    int64_t pivots;           // pivots applied (update kernels that ran)
    int64_t last_k, last_r;
    int64_t logcap;
    unsigned long long touched;   // tableau doubles the update / flush read+wrote (column skipping accounting)
    unsigned long long work[2];   // k_update work-item dequeue heads, per pivot parity (reset by k_prep)
    int64_t npend;                // deferred pivots applied but not yet flushed (prep_t sets q + 1)
    unsigned long long fwork;     // k_flush work-item dequeue head (reset with npend after each flush)
    int64_t stall;                // set by k_pivot_block when a workgroup gave up waiting (lpg_block.hip);
                                  // kStallResidency: a launch found its grid not co-resident and did nothing;
                                  // kStallPending: k_swap_plan found the pending block inconsistent
    int64_t stall_info[4];        // its view then: phase (1 P, 2 S), expected tag, record index, tag seen
    uint32_t rcnt;                // k_pivot_block residency census: arrivals (launch L's count from L * nwg)
    uint32_t rdec;                // its decision word: (L << 2) | kGo / kAbort (single rank)
    uint32_t rbad;                // region mode invalid: 1 a block's column trade was incomplete (k_swap_plan),
                                  // 2 the region build found no m distinct basic columns; 0 once rebuilt
    uint32_t pad1;
    unsigned long long gwork[8];  // k_flushw's per-XCD-group dequeue heads (FlushX; reset with fwork)
};
constexpr int64_t kStallResidency = 4;
constexpr int64_t kStallPending = 5;
constexpr int64_t kStallRegion = 6;   // a region-mode launch found rbad set and ran no pivot
// rq of a pending slot no pivot of the current block has filled (k_swap_plan
// refuses it: a local row is in [-1, nloc))
constexpr int64_t kNoSlot = INT64_MIN;

// Pending-pivot buffers of the deferred update (Defer::on == 0: eager mode).
struct Defer {
    double  *Pbuf;            // K x ld: P_q (slot q = q-th pivot since the last flush)
    double  *Cbuf;            // K x cs: C_q (column-major per pivot, rows 0..nloc-1)
    int64_t  cs;              // Cbuf pitch (>= nloc)
    int64_t *rq;              // K: local pivot row of pivot q, -1 on a non-owner rank
    int64_t *rqg;             // K: global pivot row of pivot q (region mode on a rank of a partition), or null
    int64_t *basis, *logk, *logr;   // bookkeeping done by prep_t in deferred mode
    const double *zrow;       // ld zeros (the padding slots of the prefetching pivot kernels)
    int64_t *kq, *lv;         // K: entering / leaving variable of pending pivot q (logical; k_swap_plan)
    const int32_t *colmap;    // ld: logical column held by physical column p (k_prep_d's pricing keys)
    const int32_t *inv;       // ld: physical column of logical column j (k_select_d when npp > its block)
    double  *mul;             // K x K: -C_u[r_q] (k_flush_pivot_rows' multipliers, built by k_swap_plan)
    double  *pv;              // K: pivot element of pending pivot q (replicated on every rank; k_swap_plan)
    int      q;               // pending index of this pivot
    int      on;
};

// Owner-push exchange of the multi-rank deferred path (k_prep_d / k_select_d
// MODE 2, lpg_kernels.hip). Every rank owns one exchange buffer, mapped into
// every rank's process (IPC between processes, plain device pointers between
// ranks that share one), laid out as
//   [0, offF)      xP[2][ld]             the pivot row its owner pushed (by tag parity)
//   [offF, offC)   xF[2][nblk] (u32)     per prep block: the tag of the P chunk that landed
//   [offC, ...)    xC[2][world][nx][6]   every rank's ratio candidates, 6 {payload, tag} words each
// Tags come from a host counter that never repeats within a context; the
// P chunks are published by a flag behind a system-scope release, the
// candidates are self-validating 8-byte {payload, tag} words.
struct Xch {
    char *const *base;            // device array: the world buffers ([rank] = this rank's own)
    int world, rank;
    int nblk, nx;                 // prep blocks (P chunks) and ratio candidates per rank
    int from_cand;                // 1: this pivot's candidates are in `cand` (after a bootstrap), not in xC
    uint32_t tag;                 // this pivot's tag (its candidates, its P flags); select publishes tag + 1
    int64_t offF, offC;           // byte offsets of xF and xC (xP at 0)
    int64_t offG;                 // byte offset of the residency census words {gcnt, gdec} (rank 0's are used)
};

// The census words use [offG, offG + 72); the buffer owner's identity (PCI
// bus id, 48 bytes, then its process id) sits at offG + kXchIdOff, read by
// every peer when the push is attached (lpg_ctx.hip push_shares_device).
constexpr int kXchIdOff = 128, kXchIdBytes = 64;

// Ratio-test candidate: lexicographic (theta, key); row < 0 = none.
struct Cand {                 // 32 B
    double  theta;
    double  piv;              // the pivot element T_t[row][k_t] (replicated check)
    int64_t key;              // row (Dantzig) or basic column (Bland)
    int64_t row;              // global row
};

// Pricing partial of an eligible column: Dantzig (cls, v, j) lexicographic,
// Bland smallest j. One objective row: cls 0, v = d_j < -eps. Big-M (two
// objective rows, M part first): cls 0 if dM_j < -eps (v = dM_j); cls 1 if
// |dM_j| <= eps and dR_j < -eps (v = dR_j), i.e. d_j = dM_j M + dR_j < 0.
struct PricePart {            // 24 B
    double  v;
    int64_t j;                // -1 = none
    int32_t cls;
    int32_t pad;
};

// Geometry of this rank's slice of the tableau.
struct Geo {
    double *T;                // (nloc + nobj) x ld, row-major; objective row(s) last
    int64_t ld;               // row pitch in doubles (multiple of 64)
    int64_t nloc;             // local constraint rows
    int64_t nobj;             // objective rows (1)
    int64_t ncols;            // N + 1
    int64_t nact;             // price columns 1..nact
    int64_t row0;             // global index of local row 0
    int64_t m;                // global constraint rows
    double  eps_piv, eps_opt;
};

// ---- launchers (lpg_kernels.hip) ----
struct Launch {
    void   *stream;           // hipStream_t
};

int launch_generate(const Launch &L, const Geo &g, int64_t n, uint64_t seed, int kind, int64_t *basis_dev);
int launch_objective_chain(const Launch &L, const Geo &g, const double *cb, const double *acc_in, double *acc_out);
int launch_objective_finish(const Launch &L, const Geo &g, const double *acc, const double *cost, int64_t orow);
int launch_price(const Launch &L, const Geo &g, int rule, int mode, const DevState *st, int s,
                 const double *P, const double *Cs, PricePart *pp, int *pc, int npp, bool defer = false,
                 const int32_t *colmap = nullptr, const int32_t *inv = nullptr);
int launch_prep(const Launch &L, const Geo &g, int rule, bool fuse_price, DevState *st, int s,
                const Cand *cand, int ncand, double *P, const double *Cs, PricePart *pp, int *pc, int npp,
                const Defer &D);
int launch_select(const Launch &L, const Geo &g, int rule, bool first, DevState *st, int s, int s1,
                  const double *P, const double *Cs, double *Cs1, const PricePart *pp, int npp,
                  const int64_t *basis, Cand *part, int nsel, int64_t force_k, int64_t force_r,
                  const int *pc, int skip, const Defer &D);
// One deferred-mode pivot without a communicator: k_prep_d + k_select_d
// (prefetching forms of prep + select; candidates in and out through part).
// Their grids: pivot_d_blocks(g, 0, nt) prep blocks (= pricing partials),
// pivot_d_blocks(g, 1, nt) select blocks (= ratio candidates) of nt = 256
// threads.
constexpr int kPivotThreads = 256;
int pivot_d_blocks(const Geo &g, int which, int nt);
int launch_pivot_d(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, Cand *part, int nsel,
                   double *P, const double *Cs, double *Cs1, PricePart *pp, int npp, const int64_t *basis,
                   const Defer &D, int nt);
// The same pair with a communicator: launch_prep_dm, then the caller's
// allreduce of P and launch_price(mode 1), then launch_select_dm.
int launch_prep_dm(const Launch &L, const Geo &g, int rule, DevState *st, int s, const Cand *cand, int ncand,
                   double *P, const double *Cs, int npp_d, const Defer &D);
// ... or, with the owner-push exchange, these two alone per pivot: prep takes
// the candidates from every rank's push (or `cand` after a bootstrap), the
// owner pushes P to every rank, every rank prices (k_price's work fused);
// select pushes its candidates to every rank.
int launch_prep_x(const Launch &L, const Geo &g, int rule, DevState *st, int s, const Cand *cand, int ncand,
                  double *P, const double *Cs, PricePart *pp, int npp_d, const Defer &D, const Xch &X);
int launch_select_x(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, const double *Cs,
                    double *Cs1, const PricePart *pp, int npp, const int64_t *basis, Cand *part, int nsel,
                    const Defer &D, const Xch &X);
int64_t xch_bytes(int64_t ld, int world, int nblk, int nx, int64_t *offF, int64_t *offC, int64_t *offG);
int launch_select_dm(const Launch &L, const Geo &g, int rule, DevState *st, int s, int s1, const double *Cs,
                     double *Cs1, const PricePart *pp, int npp, const int64_t *basis, Cand *part, int nsel,
                     const Defer &D);
// The deferred pivot loop as one persistent launch of n pivots starting at
// pending index q0 (lpg_block.hip): nwg workgroups, one per CU, each owning
// cw physical columns and rw constraint rows, with ks pending slots of their
// P / C slices in lds bytes of LDS. block_geometry picks the split (-1: the
// slices do not fit, use k_prep_d / k_select_d); the records buffer holds
// block_records_bytes(nwg) zero-initialised bytes; tags start after tag0.
int block_records_bytes(int nwg);
int block_geometry(const Geo &g, int ks, int cus, int want, int *nwg, int *cw, int *rw, size_t *lds);
// cin / ncin: the first pivot's ratio candidates (part itself on one rank).
// X != nullptr: multi-rank over the owner-push exchange (the same nwg / cw / rw
// on every rank), exchange tags xtag0, xtag0 + 1, ...
// Residency: every launch first counts its workgroups in (census launch
// index `cl`, DevState::rcnt / rdec; with X, every rank's through rank 0's
// exchange words): if the whole grid is not resident within a bound, the
// launch does nothing, stops the loop (both slots non-RUNNING) and sets
// DevState::stall = kStallResidency; the host then continues on the pair.
// Region mode (single rank, one objective row, column trade on): the slices
// hold only the columns whose pending P entries can be nonzero -- the nonbasic
// columns of the block start (live, column 0 excluded) plus per pending pivot
// one spare slot for the column leaving the basis then, and column 0 (lpg_block.hip
// k_pivot_block). block_geometry_region picks the split; launch_region_build
// (one workgroup) writes live, bcol0 and the 64-column liveness map tlive
// (ld / 64 ints: the block pass skips tiles without a nonbasic column, see
// launch_flush_main) from the basis and clears rbad;
// launch_region_check clears ok[0] unless every basic column is an exact unit
// vector with a zero reduced cost (the region's precondition).
struct RegionGeo {
    int nwg, cw, rw, nsp, cwx;
    size_t lds;
};
struct RegionArgs {
    const int32_t *live;
    int64_t nlive;
    const int64_t *bcol0;
    int nsp, cwx;
};
int block_geometry_region(const Geo &g, int ks, int cus, int want, int64_t nlive, RegionGeo *out);
int launch_region_build(const Launch &L, const Geo &g, DevState *st, const int64_t *basis, const int32_t *inv,
                        int32_t *mark, int32_t *live, int64_t *bcol0, int64_t nlive, int32_t *tlive);
int launch_region_check(const Launch &L, const Geo &g, const int64_t *basis, const int32_t *inv, int *ok);
int launch_pivot_block(const Launch &L, const Geo &g, int rule, DevState *st, int s0, int q0, int n, Cand *part,
                       int ncand, const Cand *cin, int ncin, const double *Cs0, double *Cs1, const Defer &D,
                       void *rec, uint32_t tag0, int nwg, int cw, int rw, int ks, size_t lds, uint32_t cl,
                       const Xch *X = nullptr, uint32_t xtag0 = 0, const RegionArgs *R = nullptr);
// Apply the pending pivots (st->npend <= kmax) to constraint rows 0..nloc-1.
int launch_flush(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, int skip, int which);
// ... in two parts: the block pass itself (k_flushw / k_flushm / k_flush), then
// the pivot-row rewrite and the pending-counter reset (the rewrite's
// multipliers come from launch_swap_plan, launched before either part)
// xcd: k_flushw's item map, -1 auto, 0 the global queue, 1 the XCD-grouped one (FlushX),
// 10 + H the latter with H column classes.
// tlive (region mode, launch_region_build's map, or null): a tile none of
// whose 64-column chunks holds a block-start nonbasic column and none of whose
// columns is a leaving column of the block (D.lv through D.inv, after the
// trade) has all-zero pending P entries and is skipped without reading them.
// Valid only for a block whose P entries of other columns are +-0: the basic
// columns were exact unit vectors at the block start (region mode's check)
// and every pivot recorded its leaving variable in D.lv.
int launch_flush_main(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, int skip, int which,
                      int xcd = -1, const int32_t *tlive = nullptr);
// reset = false: the caller ends the block itself (launch_fill_cols with st)
int launch_flush_tail(const Launch &L, const Geo &g, DevState *st, const Defer &D, int kmax, bool reset = true);
// Item map of the banded block pass (k_flushw): column tile
// fastest, `rows`-row strips; when the rows hold >= 8 strips the last two are
// cut into items of rows / 4 (a multiple of 16), so that the dynamic queue
// ends on short items (the last round of whole items left most CUs idle while
// a few finished theirs). flush_nitems is the host's count for the launch.
// rows < 0: |rows|-row items throughout, no tail (LPG_FLUSH_TAIL=0, A/B)
__host__ __device__ inline int64_t flush_tail_rows(int64_t rows, int64_t nloc) {
    return (rows > 0 && nloc >= 8 * rows && rows >= 64) ? rows / 4 : 0;
}
__host__ __device__ inline int64_t flush_nitems(int64_t ntiles, int64_t rows, int64_t nloc) {
    const int64_t tr = flush_tail_rows(rows, nloc);
    if (rows < 0) rows = -rows;
    if (!tr) return ntiles * ((nloc + rows - 1) / rows);
    const int64_t t0 = ((nloc + rows - 1) / rows - 2) * rows;
    return ntiles * (t0 / rows) + ntiles * ((nloc - t0 + tr - 1) / tr);
}
__host__ __device__ inline void flush_item(int64_t item, int64_t ntiles, int64_t rows, int64_t nloc, int64_t &tile,
                                           int64_t &i0, int64_t &i1) {
    const int64_t tr = flush_tail_rows(rows, nloc);
    if (rows < 0) rows = -rows;
    const int64_t t0 = tr ? ((nloc + rows - 1) / rows - 2) * rows : nloc;
    const int64_t nbig = ntiles * (t0 / rows);
    tile = item % ntiles;
    if (!tr || item < nbig) {
        i0 = (item / ntiles) * rows;
        i1 = i0 + rows;
    } else {
        i0 = t0 + ((item - nbig) / ntiles) * tr;
        i1 = i0 + tr;
    }
    if (i1 > nloc) i1 = nloc;
}
// XCD-grouped item map of k_flushw: the persistent blocks b with the same
// b % 8 share one XCD (one L2), and group g = b % 8 dequeues from its own
// queue (DevState::gwork[g]) the items of one row band x column class: band
// g / H of 8 / H bands, tiles t = h + H j of class h = g % H. Within a group the
// items run sub-band by sub-band (rs rows, the band's multipliers C held in
// that XCD's L2), tiles in descending order, and the last sub-band's lowest tt
// tiles are cut into nq row pieces each, one tile's pieces in a row (its P
// tile stays in L2), so the queue ends on short items where the column trade
// keeps the live columns. A group whose queue is empty takes items from the
// others (g + 1, g + 2, ...): every item is run once whatever the placement.
struct FlushX {
    int64_t ntiles, nloc;
    int32_t H;        // column classes (1, 2, 4, 8)
    int32_t rb;       // band rows (multiple of 16)
    int32_t rs;       // sub-band rows (multiple of 16, <= rb)
    int32_t tt;       // tail tiles per group
    int32_t on;
    int32_t tq;       // row pieces per tail tile (flushx_plan: 8; 0 reads as 4)
};
struct FlushXGroup {
    int64_t r0, r1, ntg, nsb, ttg, nq, qrows, count;
};
__host__ __device__ inline FlushXGroup flushx_group(const FlushX &f, int g) {
    FlushXGroup o{};
    const int b = g / f.H, h = g % f.H;
    o.r0 = (int64_t)b * f.rb;
    o.r1 = o.r0 + f.rb < f.nloc ? o.r0 + f.rb : f.nloc;
    o.ntg = h < f.ntiles ? (f.ntiles - h + f.H - 1) / f.H : 0;
    if (o.r0 >= f.nloc || o.ntg == 0) return o;
    o.nsb = (o.r1 - o.r0 + f.rs - 1) / f.rs;
    const int64_t ls = (o.r1 - o.r0) - (o.nsb - 1) * f.rs;   // last sub-band's rows
    const int64_t tq = f.tq > 0 ? f.tq : 4;
    o.qrows = ((ls + tq - 1) / tq + 15) / 16 * 16;
    o.nq = (ls + o.qrows - 1) / o.qrows;
    o.ttg = f.tt < o.ntg ? f.tt : o.ntg;
    o.count = (o.nsb - 1) * o.ntg + (o.ntg - o.ttg) + o.nq * o.ttg;
    return o;
}
__host__ __device__ inline void flushx_item(const FlushX &f, const FlushXGroup &G, int g, int64_t it, int64_t &tile,
                                            int64_t &i0, int64_t &i1) {
    const int h = g % f.H;
    int64_t j;
    const int64_t full = (G.nsb - 1) * G.ntg;
    const int64_t base = G.r0 + (G.nsb - 1) * f.rs;
    if (it < full) {
        j = G.ntg - 1 - it % G.ntg;
        i0 = G.r0 + (it / G.ntg) * f.rs;
        i1 = i0 + f.rs;
    } else if (it - full < G.ntg - G.ttg) {
        j = G.ntg - 1 - (it - full);
        i0 = base;
        i1 = G.r1;
    } else {
        const int64_t k = it - full - (G.ntg - G.ttg);
        j = G.ttg - 1 - k / G.nq;
        i0 = base + (k % G.nq) * G.qrows;
        i1 = i0 + G.qrows;
    }
    if (i1 > G.r1) i1 = G.r1;
    tile = h + (int64_t)f.H * j;
}
int flush_kmax_supported(int k);     // smallest compiled pending bound >= k (0: k too large)
// Basis-partitioned column order (single-rank deferred path): after a block,
// every column that went nonbasic -> basic during it swaps its physical
// position with one that went basic -> nonbasic, so the nonbasic columns keep
// the physical positions the nonbasic columns had at the start of the solve
// (for the synthetic LPs: one contiguous block) and a flush never meets
// scattered live columns. launch_swap_plan (before the flush: reads npend)
// pairs them and updates colmap / inv when plan != 0, and always builds the
// pivot-row multipliers D.mul; launch_move_cols (before the block
// pass) moves the leaving columns' data and P entries into place;
// launch_fill_cols (after the pivot-row rewrite) writes the entering
// columns' unit vectors (lpg_kernels.hip, above k_swap_plan).
// kmax: the pending block's bound (npend above it, or a slot's kq / lv / rq
// out of range, stops the loop with kStallPending instead of indexing).
int launch_swap_plan(const Launch &L, const Geo &g, DevState *st, const Defer &D, int32_t *colmap, int32_t *inv,
                     int32_t *pairs, int plan, int kmax);   // reads D.pv (replicated pivot elements)
// pairs: count, then kPairW ints per pair {E's position a, L's position b,
// E's row, L's row at the block start (-1: another rank's)}. unit: L's base
// column is known to be its unit vector (region mode checked it), so the
// constraint rows write it without reading it.
constexpr int kPairW = 4;
int launch_move_cols(const Launch &L, const Geo &g, const DevState *st, const Defer &D, const int32_t *pairs,
                     int unit);
// st != nullptr: also ends the pending block (npend, fwork, and D's kmax slots
// back to their never-filled sentinels), in place of launch_flush_tail's
// k_end_block (one dispatch fewer per block)
// bcol0 != nullptr (region mode, one rank): also the spares' Pbuf columns
// zeroed and every row's basic column of the next block written
int launch_fill_cols(const Launch &L, const Geo &g, const int32_t *pairs, DevState *st = nullptr,
                     const Defer *D = nullptr, int kmax = 0, int64_t *bcol0 = nullptr);
// Canonical order again: rows [i0, i0 + nr) gathered through inv into tmp
// (nr x ld), then copied back; launch_iota resets colmap / inv.
int launch_gather_rows(const Launch &L, const Geo &g, const int32_t *inv, double *tmp, int64_t i0, int64_t nr);
int launch_iota(const Launch &L, int32_t *a, int64_t n);
int launch_update(const Launch &L, const Geo &g, DevState *st, int s, const double *P, const double *Cs,
                  int64_t *basis, int64_t *logk, int64_t *logr, int variant, int skip);

int launch_dual_rows(const Launch &L, const Geo &g, Cand *part, int nsel);
// The dual on the deferred tableau (lpg_dual.hip), one pivot = row_d, then
// (row partition) the host's sum of R over the ranks and ratio, then col_d.
// rc: row candidates in (nrc: every rank's after an allgather) / out
// (nrc_out >= this rank's rows + objective rows, 256 per block), cp: the
// ratio-test partials (one per column block), R: the current pivot row,
// Pprev / Cprev: the previous pivot's P and column (its objective update),
// Cs: this pivot's column. mr: row partition (R from the owner, -0 elsewhere;
// the partials left to launch_dual_ratio).
int launch_dual_row_d(const Launch &L, const Geo &g, DevState *st, int s, const Cand *rc, int nrc, Cand *cp,
                      double *R, const double *Pprev, const double *Cprev, const Defer &D, bool mr);
int launch_dual_ratio(const Launch &L, const Geo &g, const DevState *st, int s, const double *R, Cand *cp);
int launch_dual_col_d(const Launch &L, const Geo &g, DevState *st, int s, const Cand *cp, const double *R, double *Cs,
                      Cand *rc, int nrc_out, const Defer &D);
int launch_dual_pivot(const Launch &L, const Geo &g, DevState *st, int s, Cand *part, int nsel, PricePart *pp,
                      int *pc, int npp, int skip, double *P, double *Cs, bool price_only = false);

#ifdef LPG_PHASES
int debug_phases(unsigned long long *out, int reset);   // tools/phase_probe.py
int debug_block_phases(unsigned long long *out);        // tools/block_probe.py
#endif
int price_blocks(const Geo &g);      // number of pricing partials (= prep / price grid)
int update_variants();               // entries of the update-kernel variant table
int update_auto_variant(const Geo &g);   // default variant for this geometry

}  // namespace lpg
