// lpg_ctx.hip — context, memory layout, pivot-loop driver and the extern "C"
// entry points of include/lpg.h.
//
// The host side of one pivot is a fixed sequence of launches on one stream
// (prep -> [allreduce P] -> [price] -> select -> [allgather candidates] ->
// update); nothing is read back per pivot, so the host runs ahead of the
// device and lpg_solve only synchronises every `batch` pivots to check the
// device-side status (SURVEY.md §3 call stack (3)).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types only: RCCL itself is opened at the first communicator (rccl_api())

#include <dlfcn.h>
#include <unistd.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/lpg.h"
#include "lpg_internal.h"

using namespace lpg;

namespace {

thread_local char g_err[512];

struct TimingRing {
    std::vector<hipEvent_t> ev;   // 3 per pivot: before prep, before update, after update
    std::vector<char> upd;        // per pivot: an update / flush kernel ran between marks 1 and 2
    int used = 0;
    double update_ms = 0, select_ms = 0, comm_ms = 0;
    int64_t count = 0;
};

}  // namespace

struct lpg_ctx {
    int device = 0, world = 1, rank = 0;
    int64_t m = 0, ncols = 0, ld = 0, row0 = 0, nloc = 0, nobj = 1, nact = 0;
    double eps_piv = 1e-9, eps_opt = 1e-9;
    uint32_t flags = 0;
    // device buffers
    double *T = nullptr;          // (nloc + nobj) x ld
    double *P = nullptr;          // ld
    double *C[2] = {nullptr, nullptr};
    double *acc = nullptr;        // ld (objective chain)
    double *cb = nullptr;         // nloc
    double *cost = nullptr;       // ncols
    PricePart *pp = nullptr;
    int *pc = nullptr;            // npp live-slice counts of P (column-skipping accounting)
    Cand *part = nullptr;         // nsel (this rank's select partials)
    Cand *cand = nullptr;         // world * nsel (gathered); == part when world == 1
    Cand *drc = nullptr, *dcp = nullptr;   // deferred dual: row candidates, ratio-test partials (lazy)
    Cand *drc_all = nullptr;               // ... every rank's row candidates (row partition)
    int64_t *basis = nullptr;     // m (replicated)
    int64_t *logk = nullptr, *logr = nullptr;
    int64_t logcap = 0;
    DevState *st = nullptr;
    int npp = 0, nsel = 0;
    int npp_d = 0, nsel_d = 0;    // the same partial counts for the single-rank deferred pair (k_prep_d / k_select_d)
    int pivot_nt = kPivotThreads; // threads per block of that pair
    // the persistent block kernel (lpg_block.hip): single rank, deferred, the
    // default where its slices fit (LPG_PERSIST=0 turns it off)
    bool persist = false;         // single rank, no communicator: k_pivot_block
    bool pmr = false;             // k_pivot_block's geometry also holds for the multi-rank form (same on every rank)
    bool persist_x = false;       // multi-rank k_pivot_block over the owner-push exchange (attach_push)
    bool no_reorder = false;      // LPG_NO_REORDER=1: keep the caller's column order (no block-end column trade)
    int pb_nwg = 0, pb_cw = 0, pb_rw = 0;
    size_t pb_lds = 0;
    // region mode of the single-rank persistent launch (lpg_block.hip REG): the
    // slices hold the block start's nonbasic columns only; needs one objective
    // row, the column trade, and basic columns that are exact unit vectors with
    // zero reduced costs (units_known: true after lpg_generate, or once
    // region_setup's check passed; the engine's own pivots keep it)
    bool reg = false;             // the persistent launch runs in region mode (one rank, or every rank of a push exchange)
    bool reg_valid = false;       // live / bcol0 describe the current column order and basis
    bool units_known = false;
    RegionGeo rg{};
    int32_t *live = nullptr, *mark = nullptr;
    int32_t *tlive = nullptr;     // region: 64-column chunks holding a block-start nonbasic column (k_flushw skips the rest)
    bool block_region = false;    // the pending block's pivots ran in region mode (its flush may use tlive)
    bool tlive_on = true;         // LPG_FLUSH_TLIVE=0: the pass reads every tile's P entries (A/B)
    bool move_unit = true;        // LPG_MOVE_UNIT=0: k_move_cols reads the leaving columns (A/B)
    int64_t *bcol0 = nullptr;
    int *rok = nullptr;           // region_check's flag (+ every rank's, world > 1)
    void *rec = nullptr;          // its records (zeroed once; tags never repeat within a context)
    uint32_t tag = 0;
    uint32_t pb_launch = 0;       // persistent launches since the DevState was reset (the census index)
    int64_t lost = 0;             // pivots enqueued on launches a residency census stopped (lpg_sync re-runs them)
    int res_fallbacks = 0;        // residency censuses that failed (lpg_info: the pair took over)
    int reg_recoveries = 0;       // region-mode launches stopped by rbad and re-run (recover_region)
    // owner-push exchange of the multi-rank deferred path (Xch, lpg_internal.h)
    char *xbuf = nullptr;         // this rank's exchange buffer
    int64_t xbytes = 0, xoffF = 0, xoffC = 0, xoffG = 0;
    int xnblk = 0, xnx = 0;
    bool xuncached = false;
    char **xbase = nullptr;       // device array of the world buffers
    std::vector<void *> xpeer;    // IPC-opened peer buffers (closed at destroy)
    bool xmode = false;           // attached: per pivot k_prep_d / k_select_d MODE 2, no collective
    uint32_t xtag = 1;            // next pivot's tag (never repeats within the context)
    bool x_from_cand = true;      // the next pivot's candidates are in `cand` (after a bootstrap)
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // pivot-loop host state
    bool booted = false;
    int boot_rule = 0;
    int par = 0;                  // parity of the next pivot's slot
    int64_t enq = 0;              // pivots enqueued since the last reset (log bound)
    int update_variant = 0;
    // deferred (blocked) updates: defer_k pivots per flush (0 = eager)
    int defer_k = 0;
    int pend = 0;                 // pivots enqueued since the last flush (host view)
    int flush_variant = -1;       // launch_flush_main `which`: -1 default, 0 k_flushm, 1 k_flushw
    int flush_xcd = -1;           // launch_flush_main `xcd`: -1 auto, 0 global queue, 1 XCD-grouped
    bool capture_block = false;   // capturing a deferred block's pivots (its flush stays outside the graph)
    bool fast_pivot = true;       // deferred single-rank pivots through k_prep_d / k_select_d (LPG_SLOW_PIVOT=1: generic pair)
    double *Pbuf = nullptr, *Cbuf = nullptr;
    double *zrow = nullptr;       // ld zeros (padding slots of the prefetching pivot kernels)
    // basis-partitioned column order (single-rank deferred path, lpg_internal.h)
    int64_t *kq = nullptr, *lv = nullptr;   // per pending pivot: entering / leaving variable
    int32_t *colmap = nullptr, *inv = nullptr, *pairs = nullptr;
    double *mul = nullptr;        // pivot-row multipliers of a flush (LPG_DEFER_MAX^2)
    double *pv = nullptr;         // pivot elements of the pending block (replicated)
    double *tmp = nullptr;        // row chunk for canonicalize()
    int64_t tmp_rows = 0;
    bool permuted = false;        // colmap may differ from the identity
    int64_t cs = 0;
    int64_t *rq = nullptr;
    int64_t *rqg = nullptr;       // region mode on ranks: the global pivot row of each pending slot
    int skip = 1;                 // column skipping in the update (LPG_FLAG_NO_SKIP turns it off)
    // the test-hook build only (LPG_TEST_HOOKS; env LPG_TEST_PENDING_FAULT=F:W):
    // before flush F, make the pending block inconsistent (W = npend | kq | lv |
    // rq | ahead) to exercise k_swap_plan's guard
    int inject_flush = -1, inject_what = 0;
    // (test hooks) env LPG_TEST_REGION_BAD=F: after flush F's swap plan, set
    // DevState::rbad as an incomplete column trade would, so that the next
    // region-mode launch -- inside the same lpg_enqueue -- stops with
    // kStallRegion and recover_region / lpg_sync re-run its pivots
    int inject_rbad = -1;
    // k_swap_plan refused a pending block (pending_fault): the basis already
    // holds the block's pivots while the constraint rows do not, so every
    // pivoting entry point refuses until the LP is reloaded or regenerated
    bool poisoned = false;
    int64_t nflush = 0;           // flush_launch calls so far
    unsigned long long touched_mark = 0;
    // communication
    ncclComm_t nccl = nullptr;
    lpg_host_comm_ops hops{};
    bool have_hops = false;
    std::vector<unsigned char> hsend, hrecv;
    // hipGraph of kGraphPivots pivots (starting at parity 0), replayed by
    // enqueue when no communicator and no per-pivot timing is active
    hipGraphExec_t graph[2] = {nullptr, nullptr};   // by parity of the first pivot
    int graph_rule[2] = {-1, -1};
    bool use_graphs = true;
    bool graph_comm = false;      // RCCL collectives captured into the replayed graphs (LPG_GRAPH_RCCL=1;
                                  // cleared if capture fails). Off by default: on one GPU (1-rank
                                  // communicator) it measured no gain, and the 8-GPU path is untested here
    // timing
    bool timing = false;
    TimingRing tr;
    char err[512] = {0};
};

static int fail(lpg_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) snprintf(c->err, sizeof c->err, "%s", buf);
    snprintf(g_err, sizeof g_err, "%s", buf);
    return code;
}

#define HIPCHK(c, x)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            (void)hipGetLastError(); /* a failed call (e.g. an OOM hipMalloc) must not fail the next launch check */ \
            return fail((c), LPG_ERR_DEVICE, "%s: %s", #x, hipGetErrorString(e_));           \
        }                                                                                    \
    } while (0)

static Geo geo(const lpg_ctx *c) {
    Geo g;
    g.T = c->T;
    g.ld = c->ld;
    g.nloc = c->nloc;
    g.nobj = c->nobj;
    g.ncols = c->ncols;
    g.nact = c->nact;
    g.row0 = c->row0;
    g.m = c->m;
    g.eps_piv = c->eps_piv;
    g.eps_opt = c->eps_opt;
    return g;
}

static Launch lau(const lpg_ctx *c) { return Launch{(void *)c->stream}; }

static int use_device(lpg_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    return 0;
}

// ---------------------------------------------------------------------------
// collectives: RCCL on device buffers, or caller-provided host-staged ops
// ---------------------------------------------------------------------------

static bool has_comm(const lpg_ctx *c) { return c->world > 1 || c->nccl || c->have_hops; }

// RCCL is not a link-time dependency of liblpg.so. A process that already
// holds an RCCL (torch's bundled librccl.so, SONAME librccl.so.1) keeps using
// that one; otherwise the system ROCm's librccl.so.1 is opened here. Linking
// it made every liblpg user map the system RCCL (and its librocm_smi64) at
// load time, which aborted at exit next to torch's copies
// (profiles/r01_runtime_order.log, linearprogramming_amd/_lib.py bind_runtime).
struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    const char *(*GetErrorString)(ncclResult_t);
};

static const RcclApi *rccl_api() {
    static RcclApi api;
    static int state = 0;   // 0 untried, 1 ok, -1 unavailable
    if (state) return state > 0 ? &api : nullptr;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    state = -1;
    if (!h) return nullptr;
    api.GetUniqueId = (decltype(api.GetUniqueId))dlsym(h, "ncclGetUniqueId");
    api.CommInitRank = (decltype(api.CommInitRank))dlsym(h, "ncclCommInitRank");
    api.CommDestroy = (decltype(api.CommDestroy))dlsym(h, "ncclCommDestroy");
    api.AllGather = (decltype(api.AllGather))dlsym(h, "ncclAllGather");
    api.AllReduce = (decltype(api.AllReduce))dlsym(h, "ncclAllReduce");
    api.GetErrorString = (decltype(api.GetErrorString))dlsym(h, "ncclGetErrorString");
    if (api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.AllGather && api.AllReduce && api.GetErrorString)
        state = 1;
    return state > 0 ? &api : nullptr;
}

static int comm_allgather(lpg_ctx *c, const void *send, void *recv, size_t bytes) {
    if (!has_comm(c)) return 0;
    if (c->nccl) {
        const RcclApi *R = rccl_api();
        ncclResult_t r = R->AllGather(send, recv, bytes, ncclUint8, c->nccl, c->stream);
        if (r != ncclSuccess) return fail(c, LPG_ERR_COMM, "ncclAllGather: %s", R->GetErrorString(r));
        return 0;
    }
    if (!c->have_hops) return fail(c, LPG_ERR_STATE, "world > 1 but no communicator attached");
    c->hsend.resize(bytes);
    c->hrecv.resize(bytes * c->world);
    HIPCHK(c, hipMemcpyAsync(c->hsend.data(), send, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->hops.allgather(c->hops.user, c->hsend.data(), c->hrecv.data(), bytes) != 0)
        return fail(c, LPG_ERR_COMM, "host allgather callback failed");
    HIPCHK(c, hipMemcpyAsync(recv, c->hrecv.data(), bytes * c->world, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

static int comm_allreduce_sum(lpg_ctx *c, double *buf, size_t count) {
    if (!has_comm(c)) return 0;
    if (c->nccl) {
        const RcclApi *R = rccl_api();
        ncclResult_t r = R->AllReduce(buf, buf, count, ncclFloat64, ncclSum, c->nccl, c->stream);
        if (r != ncclSuccess) return fail(c, LPG_ERR_COMM, "ncclAllReduce: %s", R->GetErrorString(r));
        return 0;
    }
    if (!c->have_hops) return fail(c, LPG_ERR_STATE, "world > 1 but no communicator attached");
    c->hsend.resize(count * sizeof(double));
    HIPCHK(c, hipMemcpyAsync(c->hsend.data(), buf, count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->hops.allreduce_sum_f64(c->hops.user, (double *)c->hsend.data(), count) != 0)
        return fail(c, LPG_ERR_COMM, "host allreduce callback failed");
    HIPCHK(c, hipMemcpyAsync(buf, c->hsend.data(), count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------
// timing ring
// ---------------------------------------------------------------------------

static int timing_flush(lpg_ctx *c) {
    TimingRing &t = c->tr;
    if (t.used == 0) return 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int q = 0; q < t.used; q++) {
        float a = 0, b = 0;
        HIPCHK(c, hipEventElapsedTime(&a, t.ev[3 * q], t.ev[3 * q + 1]));
        HIPCHK(c, hipEventElapsedTime(&b, t.ev[3 * q + 1], t.ev[3 * q + 2]));
        if (t.upd[q] != 2) t.select_ms += a;   // 2: a flush-only entry (marks 0 and 1 adjacent)
        if (t.upd[q]) {
            t.update_ms += b;
            t.count++;
        } else {
            t.select_ms += b;
        }
    }
    t.used = 0;
    return 0;
}

static int timing_mark(lpg_ctx *c, int which, int updated = 1) {
    TimingRing &t = c->tr;
    if (which == 0 && t.used * 3 + 3 > (int)t.ev.size()) {
        int rc = timing_flush(c);
        if (rc) return rc;
    }
    HIPCHK(c, hipEventRecord(t.ev[3 * t.used + which], c->stream));
    if (which == 2) t.upd[t.used++] = (char)updated;
    return 0;
}

// ---------------------------------------------------------------------------
// deferred updates
// ---------------------------------------------------------------------------

static Defer defer_of(const lpg_ctx *c, int q) {
    Defer d;
    d.Pbuf = c->Pbuf;
    d.Cbuf = c->Cbuf;
    d.cs = c->cs;
    d.rq = c->rq;
    d.rqg = c->rqg;
    d.basis = c->basis;
    d.logk = c->logk;
    d.logr = c->logr;
    d.zrow = c->zrow;
    d.kq = c->kq;
    d.lv = c->lv;
    d.colmap = c->colmap;
    d.inv = c->inv;
    d.mul = c->mul;
    d.pv = c->pv;
    d.q = q;
    d.on = c->defer_k > 0 ? 1 : 0;
    return d;
}

// Apply the pending block (its size on the device is st->npend <= pend).
// In deferred mode the timing ring brackets exactly this (k_flush +
// k_flush_pivot_rows + the counter reset).
// Reordered columns need the prefetching pivot pair (k_prep_d / k_select_d;
// with a communicator k_price mode 1 between them prices logical keys): every
// rank runs the same plan from replicated data (kq, lv, pv), so the physical
// order, and with it the exchanged P, is the same on every rank.
static bool reorders(const lpg_ctx *c) { return c->defer_k > 0 && c->fast_pivot && c->colmap && !c->no_reorder; }

// The timing ring brackets the block pass alone (k_flushw / k_flushm), the
// kernel the roofline reports; the swap plan, pivot-row rewrite and column
// swaps around it count as "other" time per pivot.
#ifdef LPG_TEST_HOOKS
// The test hook's corruptions, one hipMemsetAsync each: npend = 0x7f7f.. (far
// above any block), kq[0] = lv[0] = -1 (no column), rq[0] = 0x7f7f.. (no row).
// "ahead" (5): npend one past the slots the block filled (what a block stopped
// mid-way can leave), so the plan meets a slot no pivot of this block wrote.
static int inject_pending_fault(lpg_ctx *c) {
    switch (c->inject_what) {
        case 1: HIPCHK(c, hipMemsetAsync(&c->st->npend, 0x7f, sizeof(int64_t), c->stream)); break;
        case 2: HIPCHK(c, hipMemsetAsync(c->kq, 0xff, sizeof(int64_t), c->stream)); break;
        case 3: HIPCHK(c, hipMemsetAsync(c->lv, 0xff, sizeof(int64_t), c->stream)); break;
        case 4: HIPCHK(c, hipMemsetAsync(c->rq, 0x7f, sizeof(int64_t), c->stream)); break;
        case 5: {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            int64_t np = 0;
            HIPCHK(c, hipMemcpy(&np, &c->st->npend, sizeof np, hipMemcpyDeviceToHost));
            np += 1;
            HIPCHK(c, hipMemcpy(&c->st->npend, &np, sizeof np, hipMemcpyHostToDevice));
            break;
        }
        default: break;
    }
    return 0;
}

#endif

static int flush_launch(lpg_ctx *c) {
    int rc;
    const bool re = reorders(c);
#ifdef LPG_TEST_HOOKS
    if (c->inject_flush >= 0 && c->nflush == c->inject_flush && (rc = inject_pending_fault(c))) return rc;
#endif
    c->nflush++;
    // unit: the leaving columns' base data is their unit vector (a region block:
    // the basic columns were checked exact unit vectors, and the trade, the
    // pass and k_fill_cols keep them so), written without reading it
    const int unit = (c->block_region && c->reg_valid && c->move_unit) ? 1 : 0;
    if (launch_swap_plan(lau(c), geo(c), c->st, defer_of(c, 0), c->colmap, c->inv, c->pairs, re ? 1 : 0, c->defer_k) ||
        (re && launch_move_cols(lau(c), geo(c), c->st, defer_of(c, 0), c->pairs, unit)))
        return fail(c, LPG_ERR_DEVICE, "swap plan launch failed");
#ifdef LPG_TEST_HOOKS
    if (c->inject_rbad >= 0 && c->nflush == c->inject_rbad + 1)
        HIPCHK(c, hipMemsetAsync(&c->st->rbad, 0x01, sizeof(uint32_t), c->stream));
#endif
    if (c->timing && ((rc = timing_mark(c, 0)) || (rc = timing_mark(c, 1)))) return rc;
    // tlive: region blocks only (every pivot recorded its leaving column, the
    // basic columns were exact unit vectors at the block start); LPG_FLUSH_TLIVE=0 off (A/B)
    const int32_t *tl = (c->block_region && c->reg_valid && re && c->tlive_on && c->skip) ? c->tlive : nullptr;
    c->block_region = false;
    if (launch_flush_main(lau(c), geo(c), c->st, defer_of(c, 0), c->pend, c->skip, c->flush_variant, c->flush_xcd, tl))
        return fail(c, LPG_ERR_DEVICE, "flush launch failed");
    if (c->timing && (rc = timing_mark(c, 2, 2))) return rc;
    if (launch_flush_tail(lau(c), geo(c), c->st, defer_of(c, 0), c->pend, !re))
        return fail(c, LPG_ERR_DEVICE, "flush launch failed");
    if (re) {   // k_fill_cols also clears the pending block
        const Defer D = defer_of(c, 0);
        if (launch_fill_cols(lau(c), geo(c), c->pairs, c->st, &D, flush_kmax_supported(c->defer_k),
                             c->reg ? c->bcol0 : nullptr))
            return fail(c, LPG_ERR_DEVICE, "fill launch failed");
        c->permuted = true;
    }
    c->pend = 0;
    return 0;
}

// Bring the constraint rows up to date (no-op in eager mode or with nothing pending).
static int materialize(lpg_ctx *c) {
    if (c->defer_k == 0 || c->pend == 0) return 0;
    return flush_launch(c);
}

// Up to date AND in the caller's column order (every entry point other than
// the pivot loop itself: host reads and writes, generic kernels).
static int canonicalize(lpg_ctx *c) {
    int rc = materialize(c);
    c->reg_valid = false;      // region mode rebuilds its live columns for the order and basis of the next launch
    if (rc || !c->permuted) return rc;
    const int64_t rows = c->nloc + c->nobj;
    if (!c->tmp) {
        c->tmp_rows = std::min<int64_t>(rows, 512);
        HIPCHK(c, hipMalloc(&c->tmp, (size_t)c->tmp_rows * c->ld * sizeof(double)));
    }
    const Geo g = geo(c);
    for (int64_t i0 = 0; i0 < rows; i0 += c->tmp_rows) {
        const int64_t nr = std::min(c->tmp_rows, rows - i0);
        if (launch_gather_rows(lau(c), g, c->inv, c->tmp, i0, nr)) return fail(c, LPG_ERR_DEVICE, "gather launch failed");
        HIPCHK(c, hipMemcpy2DAsync(c->T + i0 * c->ld, c->ld * sizeof(double), c->tmp, c->ld * sizeof(double),
                                   c->ncols * sizeof(double), nr, hipMemcpyDeviceToDevice, c->stream));
    }
    if (launch_iota(lau(c), c->colmap, c->ld) || launch_iota(lau(c), c->inv, c->ld))
        return fail(c, LPG_ERR_DEVICE, "iota launch failed");
    c->permuted = false;
    return 0;
}

// ---------------------------------------------------------------------------
// pivot loop
// ---------------------------------------------------------------------------

// Ratio candidates per rank: the deferred prefetching pair (single rank or
// not) works with nsel_d, the generic kernels with nsel.
static int cand_per_rank(const lpg_ctx *c) { return (c->defer_k > 0 && c->fast_pivot) ? c->nsel_d : c->nsel; }

// Doubles of the pivot row the allreduce exchanges: the columns the prep
// kernels write, [0, ncols) plus the even padding column k_flushw reads in
// pairs -- never the rest of the ld pitch, which no kernel writes (round 2
// summed that uninitialised padding across ranks: the overflow warning of
// tests/test_gpu_dist.py's host transport).
static int64_t prow_count(const lpg_ctx *c) { return (c->ncols + 1) & ~(int64_t)1; }

static int exchange_candidates(lpg_ctx *c) {
    if (!has_comm(c)) return 0;
    return comm_allgather(c, c->part, c->cand, sizeof(Cand) * (size_t)cand_per_rank(c));
}

// The generic select of a bootstrap writes nsel ratio candidates, and the
// deferred pair's k_prep_d reads nsel_d: the rest must read as "none".
static int clear_candidates(lpg_ctx *c) {
    if (c->nsel_d > c->nsel)
        HIPCHK(c, hipMemsetAsync(c->part + c->nsel, 0xff, (size_t)(c->nsel_d - c->nsel) * sizeof(Cand), c->stream));
    return 0;
}

static int region_setup(lpg_ctx *c);

static int bootstrap(lpg_ctx *c, int rule) {
    int rc = canonicalize(c);
    if (rc || (rc = region_setup(c)) || (rc = clear_candidates(c))) return rc;
    HIPCHK(c, hipMemsetAsync(c->st->slot, 0, sizeof(c->st->slot), c->stream));
    const Geo g = geo(c);
    if (launch_price(lau(c), g, rule, 0, c->st, 0, c->P, c->C[0], c->pp, c->pc, c->npp))
        return fail(c, LPG_ERR_DEVICE, "price launch failed");
    if (launch_select(lau(c), g, rule, true, c->st, 0, 0, c->P, c->C[1], c->C[0], c->pp, c->npp, c->basis,
                      c->part, c->nsel, 0, -1, c->pc, c->skip, defer_of(c, 0)))
        return fail(c, LPG_ERR_DEVICE, "select launch failed");
    if ((rc = exchange_candidates(c))) return rc;
    c->par = 0;
    c->booted = true;
    c->boot_rule = rule;
    c->x_from_cand = true;
    return 0;
}

// Bootstrap onto a caller-chosen pivot (k, r): no pricing, the ratio test
// admits only row r (either sign, |T[r][k]| > eps_piv).
static int bootstrap_forced(lpg_ctx *c, int rule, int64_t k, int64_t r) {
    int rc = canonicalize(c);
    if (rc || (rc = region_setup(c)) || (rc = clear_candidates(c))) return rc;
    HIPCHK(c, hipMemsetAsync(c->st->slot, 0, sizeof(c->st->slot), c->stream));
    if (launch_select(lau(c), geo(c), rule, true, c->st, 0, 0, c->P, c->C[1], c->C[0], c->pp, c->npp, c->basis,
                      c->part, c->nsel, k, r, c->pc, c->skip, defer_of(c, 0)))
        return fail(c, LPG_ERR_DEVICE, "select launch failed");
    if ((rc = exchange_candidates(c))) return rc;
    c->par = 0;
    c->booted = true;
    c->boot_rule = rule;
    c->x_from_cand = true;
    return 0;
}

static constexpr int kGraphPivots = 32;
static constexpr int kDefaultDeferHuge = 96;    // pivots per flush (LPG_DEFER), tableaus >= 16 GB per rank
static constexpr int kDefaultDefer = 64;        // pivots per flush, large tableaus
static constexpr int kDefaultDeferSmall = 32;   // tableaus below 200 MB per rank

static int enqueue_eager(lpg_ctx *c, int64_t npiv, int rule);

// Ratio candidates in `part` that a consumer reads: every producer writes
// its own count and the bootstraps clear the rest (clear_candidates).
static int cand_cap(const lpg_ctx *c) { return std::max(c->nsel, c->nsel_d); }

// Region mode's precondition on a tableau the engine did not generate
// (lpg_load_rows / lpg_set_basis): every basic column an exact unit vector
// with a zero reduced cost. Checked once (synchronously) at the next
// bootstrap; the engine's own pivots keep it (an entering column becomes
// exactly e_r: P_q[E] = piv / piv = 1, every other row fma(-x, 1, x) = +0, its
// reduced cost fma(-d, 1, d) = 0). Where it fails the context leaves region
// mode for good: the all-column slices if they fit this block size, else the
// two-kernel pair.
// With world > 1 (region mode on the ranks of a push exchange) the ranks
// decide together: each checks its rows (or knows them), the flags are
// allgathered, and region mode stays only if every rank's passed -- a rank
// alone in region mode would run another kernel than its peers.
static int region_setup(lpg_ctx *c) {
    if (!c->reg) return 0;
    if (c->world > 1 && !(c->persist_x && c->xmode)) return 0;   // the collectives' pair: region mode unused
    if (c->world == 1 && c->units_known) return 0;
    int ok = 1;
    if (!c->units_known) {
        HIPCHK(c, hipMemsetAsync(c->rok, 0xff, sizeof(int), c->stream));
        if (launch_region_check(lau(c), geo(c), c->basis, c->inv, c->rok))
            return fail(c, LPG_ERR_DEVICE, "region check failed");
    } else {
        HIPCHK(c, hipMemsetAsync(c->rok, 0xff, sizeof(int), c->stream));   // known: nonzero
    }
    if (c->world > 1) {
        int rc = comm_allgather(c, c->rok, c->rok + 1, sizeof(int));
        if (rc) return rc;
        std::vector<int> all((size_t)c->world);
        HIPCHK(c, hipMemcpyAsync(all.data(), c->rok + 1, all.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (int v : all) ok = ok && v != 0;
    } else {
        HIPCHK(c, hipMemcpyAsync(&ok, c->rok, sizeof ok, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (ok) {
        c->units_known = true;
        return 0;
    }
    c->reg = false;
    if (c->world > 1) {                // the all-column slices where they fit, else the pair
        if (!c->pmr) c->persist_x = false;
        return 0;
    }
    if (c->pmr && !has_comm(c)) {
        c->nsel_d = c->pb_nwg;
    } else {
        c->persist = false;
        c->nsel_d = pivot_d_blocks(geo(c), 1, c->pivot_nt);   // <= the allocation
    }
    return 0;
}

// live columns and block-start basic columns for the current order and basis
// (one workgroup, on the stream: no host sync); also clears DevState::rbad.
// Always at a block boundary (a rebuild follows canonicalize / a bootstrap),
// where Pbuf holds nothing pending: it is zeroed, because region mode keeps
// the Pbuf entries of every column it does not hold at +0 (the block pass
// skips all-zero tiles and reads the rest), and a column order restored by
// canonicalize() leaves other columns' entries at the positions basic columns
// now hold.
static int region_build(lpg_ctx *c) {
    HIPCHK(c, hipMemsetAsync(c->Pbuf, 0, (size_t)flush_kmax_supported(c->defer_k) * c->ld * sizeof(double), c->stream));
    if (launch_region_build(lau(c), geo(c), c->st, c->basis, c->inv, c->mark, c->live, c->bcol0, c->ncols - 1 - c->m,
                            c->tlive))
        return fail(c, LPG_ERR_DEVICE, "region build failed");
    c->reg_valid = true;
    return 0;
}

// Persistent path: one k_pivot_block launch per run of pivots inside a
// block, the block's flush after its last pivot.
static int enqueue_blocks(lpg_ctx *c, int64_t npiv, int rule) {
    const Geo g = geo(c);
    const bool mr = c->persist_x && c->xmode;
    const bool reg = c->reg && (mr || !has_comm(c));
    const int nwg = reg ? c->rg.nwg : c->pb_nwg;
    if (reg && !c->reg_valid) {
        int rc = region_build(c);
        if (rc) return rc;
    }
    RegionArgs R{c->live, c->ncols - 1 - c->m, c->bcol0, c->rg.nsp, c->rg.cwx};
    while (npiv > 0) {
        const int n = (int)std::min<int64_t>(npiv, c->defer_k - c->pend);
        const int s0 = c->par, s1 = (s0 + n) & 1;
        // the first pivot's ratio candidates: the previous launch's (one per
        // workgroup, this rank's) or, after a bootstrap on a communicator, the
        // gathered ones of every rank
        const Cand *cin = c->part;
        int ncin = cand_cap(c), ncand = cand_cap(c);
        Xch X;
        if (mr) {
            ncand = std::max(ncand, nwg);
            ncin = c->x_from_cand ? cand_per_rank(c) * c->world : nwg;
            if (c->x_from_cand) cin = c->cand;
            X.base = c->xbase;
            X.world = c->world;
            X.rank = c->rank;
            X.nblk = c->xnblk;
            X.nx = c->xnx;
            X.from_cand = 0;
            X.tag = c->xtag;
            X.offF = c->xoffF;
            X.offC = c->xoffC;
            X.offG = c->xoffG;
        }
        const bool ok = reg ? launch_pivot_block(lau(c), g, rule, c->st, s0, c->pend, n, c->part, ncand, cin, ncin,
                                                 c->C[s0], c->C[s1], defer_of(c, c->pend), c->rec, c->tag, c->rg.nwg,
                                                 c->rg.cw, c->rg.rw, c->defer_k, c->rg.lds, c->pb_launch + 1,
                                                 mr ? &X : nullptr, c->xtag, &R) == 0
                            : launch_pivot_block(lau(c), g, rule, c->st, s0, c->pend, n, c->part, ncand, cin, ncin,
                                                 c->C[s0], c->C[s1], defer_of(c, c->pend), c->rec, c->tag, c->pb_nwg,
                                                 c->pb_cw, c->pb_rw, c->defer_k, c->pb_lds, c->pb_launch + 1,
                                                 mr ? &X : nullptr, c->xtag) == 0;
        if (!ok)
            return fail(c, LPG_ERR_DEVICE, "pivot block launch failed");
        if (reg) c->block_region = true;
        c->pb_launch++;
        if (mr) {
            c->xtag += (uint32_t)n;
            c->x_from_cand = false;
        }
        c->tag += (uint32_t)n;
        c->pend += n;
        c->par = s1;
        c->enq += n;
        npiv -= n;
        if (c->pend == c->defer_k) {
            int rc = flush_launch(c);
            if (rc) return rc;
        }
    }
    return 0;
}

static void graph_drop(lpg_ctx *c) {
    for (int p = 0; p < 2; p++) {
        if (c->graph[p]) (void)hipGraphExecDestroy(c->graph[p]);
        c->graph[p] = nullptr;
        c->graph_rule[p] = -1;
    }
}

// Pivots per graph: eager mode kGraphPivots; deferred mode the defer_k pivots
// of one block (prep + select); the block's flush is launched after each
// replay, outside the graph, so that it alone can be timed with events.
static int graph_len(const lpg_ctx *c) { return c->defer_k > 0 ? c->defer_k : kGraphPivots; }

// Capture graph_len pivots starting at the current parity (the launches read
// every per-pivot choice from device memory, so one graph serves every
// replay at that parity and block position 0).
static int graph_build(lpg_ctx *c, int rule) {
    const int par = c->par;
    if (c->graph[par]) (void)hipGraphExecDestroy(c->graph[par]);
    c->graph[par] = nullptr;
    c->graph_rule[par] = -1;
    hipGraph_t g = nullptr;
    HIPCHK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    const int64_t enq = c->enq;
    const int pend = c->pend;
    c->capture_block = true;
    int rc = enqueue_eager(c, graph_len(c), rule);
    c->capture_block = false;
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    c->par = par;
    c->enq = enq;
    c->pend = pend;
    if (rc) return rc;
    if (e != hipSuccess) return fail(c, LPG_ERR_DEVICE, "hipStreamEndCapture: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(&c->graph[par], g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        c->graph[par] = nullptr;
        return fail(c, LPG_ERR_DEVICE, "hipGraphInstantiate: %s", hipGetErrorString(e));
    }
    c->graph_rule[par] = rule;
    return 0;
}

static int enqueue(lpg_ctx *c, int64_t npiv, int rule) {
    if (!c->booted || c->boot_rule != rule) {
        int rc = bootstrap(c, rule);
        if (rc) return rc;
    }
    if (c->persist && !has_comm(c)) return enqueue_blocks(c, npiv, rule);
    if (c->persist_x && c->xmode) return enqueue_blocks(c, npiv, rule);
    const int G = graph_len(c);
    // eager-mode timing brackets every update, which a graph cannot; deferred
    // timing brackets only the flushes, which stay outside the graph
    const bool timed = c->timing && c->defer_k == 0;
    // a host-callback communicator cannot be captured; RCCL's collectives can
    // (the push exchange's tags are launch arguments: never replayed)
    const bool comm_ok = !has_comm(c) || (c->nccl && !c->have_hops && c->graph_comm && !c->xmode);
    if (!c->use_graphs || timed || !comm_ok || npiv < 2 * G || (G & 1)) return enqueue_eager(c, npiv, rule);
    int rc;
    if (c->pend) {                           // finish the open block first
        const int64_t a = G - c->pend;
        if ((rc = enqueue_eager(c, a, rule))) return rc;
        npiv -= a;
    }
    const int par = c->par;                  // G is even: every block starts at this parity
    if (npiv >= G && (!c->graph[par] || c->graph_rule[par] != rule)) {
        if ((rc = graph_build(c, rule))) {
            if (!has_comm(c)) return rc;
            c->graph_comm = false;           // this RCCL build does not capture: launch eagerly from now on
            c->err[0] = 0;
            return enqueue_eager(c, npiv, rule);
        }
    }
    for (; npiv >= G; npiv -= G) {
        HIPCHK(c, hipGraphLaunch(c->graph[par], c->stream));
        c->enq += G;
        if (c->defer_k) {                    // the block's flush
            c->pend = G;
            if ((rc = flush_launch(c))) return rc;
        }
    }
    return enqueue_eager(c, npiv, rule);
}

static int enqueue_eager(lpg_ctx *c, int64_t npiv, int rule) {
    const Geo g = geo(c);
    const Launch L = lau(c);
    // Without a communicator the pricing of d_{t+1} is fused into prep; with
    // one (any world size) P must be exchanged first.
    const bool fuse = !has_comm(c);
    const int ncand = c->nsel * c->world;
    const int ncand_d = c->nsel_d * c->world;
    for (int64_t q = 0; q < npiv; q++) {
        const int s = c->par, s1 = s ^ 1;
        const Defer D = defer_of(c, c->pend);
        double *P = D.on ? c->Pbuf + (int64_t)c->pend * c->ld : c->P;
        int rc;
        const bool mark = c->timing && !D.on;   // deferred mode times the flushes only
        if (mark && (rc = timing_mark(c, 0))) return rc;
        if (D.on && fuse && c->fast_pivot) {    // deferred, single rank: the prefetching pair
            if (launch_pivot_d(L, g, rule, c->st, s, s1, c->part, c->nsel_d, P, c->C[s], c->C[s1], c->pp, c->npp_d,
                               c->basis, D, c->pivot_nt))
                return fail(c, LPG_ERR_DEVICE, "pivot launch failed");
            if (++c->pend == c->defer_k && !c->capture_block)
                if ((rc = flush_launch(c))) return rc;
            c->par = s1;
            c->enq++;
            continue;
        }
        if (D.on && c->fast_pivot && c->xmode) {   // deferred, owner-push exchange: two kernels, no collective
            Xch X;
            X.base = c->xbase;
            X.world = c->world;
            X.rank = c->rank;
            X.nblk = c->xnblk;
            X.nx = c->xnx;
            X.from_cand = c->x_from_cand ? 1 : 0;
            X.tag = c->xtag;
            X.offF = c->xoffF;
            X.offC = c->xoffC;
            X.offG = c->xoffG;
            if (launch_prep_x(L, g, rule, c->st, s, c->cand, ncand_d, P, c->C[s], c->pp, c->npp_d, D, X))
                return fail(c, LPG_ERR_DEVICE, "prep launch failed");
            if (launch_select_x(L, g, rule, c->st, s, s1, c->C[s], c->C[s1], c->pp, c->npp_d, c->basis, c->part,
                                c->nsel_d, D, X))
                return fail(c, LPG_ERR_DEVICE, "select launch failed");
            c->xtag++;
            c->x_from_cand = false;
            if (++c->pend == c->defer_k && !c->capture_block)
                if ((rc = flush_launch(c))) return rc;
            c->par = s1;
            c->enq++;
            continue;
        }
        if (D.on && c->fast_pivot) {            // deferred, with a communicator: the pair around the exchange
            if (launch_prep_dm(L, g, rule, c->st, s, c->cand, ncand_d, P, c->C[s], c->npp_d, D))
                return fail(c, LPG_ERR_DEVICE, "prep launch failed");
            if ((rc = comm_allreduce_sum(c, P, (size_t)prow_count(c)))) return rc;
            if (launch_price(L, g, rule, 1, c->st, s, P, c->C[s], c->pp, c->pc, c->npp, true, c->colmap, c->inv))
                return fail(c, LPG_ERR_DEVICE, "price launch failed");
            if (launch_select_dm(L, g, rule, c->st, s, s1, c->C[s], c->C[s1], c->pp, c->npp, c->basis, c->part,
                                 c->nsel_d, D))
                return fail(c, LPG_ERR_DEVICE, "select launch failed");
            if ((rc = exchange_candidates(c))) return rc;
            if (++c->pend == c->defer_k && !c->capture_block)
                if ((rc = flush_launch(c))) return rc;
            c->par = s1;
            c->enq++;
            continue;
        }
        if (launch_prep(L, g, rule, fuse, c->st, s, c->cand, ncand, P, c->C[s], c->pp, c->pc, c->npp, D))
            return fail(c, LPG_ERR_DEVICE, "prep launch failed");
        if (!fuse) {
            if ((rc = comm_allreduce_sum(c, P, (size_t)prow_count(c)))) return rc;
            if (launch_price(L, g, rule, 1, c->st, s, P, c->C[s], c->pp, c->pc, c->npp, D.on != 0))
                return fail(c, LPG_ERR_DEVICE, "price launch failed");
        }
        if (launch_select(L, g, rule, false, c->st, s, s1, P, c->C[s], c->C[s1], c->pp, c->npp, c->basis,
                          c->part, c->nsel, 0, -1, c->pc, c->skip, D))
            return fail(c, LPG_ERR_DEVICE, "select launch failed");
        if ((rc = exchange_candidates(c))) return rc;
        if (mark && (rc = timing_mark(c, 1))) return rc;
        if (!D.on) {
            if (launch_update(L, g, c->st, s, c->P, c->C[s], c->basis, c->logk, c->logr, c->update_variant, c->skip))
                return fail(c, LPG_ERR_DEVICE, "update launch failed");
        } else if (++c->pend == c->defer_k && !c->capture_block) {
            if ((rc = flush_launch(c))) return rc;
        }
        if (mark && (rc = timing_mark(c, 2))) return rc;
        c->par = s1;
        c->enq++;
    }
    return 0;
}

// A persistent launch found its grid (every rank's, on a communicator) not
// resident at once -- another kernel or process held CUs -- and stopped
// before its first pivot; every pivot launch after it did nothing (both
// slots non-RUNNING), the flushes applied the pivots that had run. The loop
// continues on the two-kernel pair, which needs no co-residency: the next
// enqueue bootstraps (flush, then price and ratio test from the current
// tableau, i.e. the choices the persistent launch would have made), so the
// pivot sequence is unchanged. Every rank sees the same census decision
// (rank 0's word, lpg_block.hip), so on a communicator every rank recovers
// at the same launch and the bootstrap's collectives match.
static int recover_residency(lpg_ctx *c, const DevState &h) {
    c->persist = false;
    c->persist_x = false;
    c->pmr = false;
    if (!has_comm(c)) c->nsel_d = pivot_d_blocks(geo(c), 1, c->pivot_nt);   // <= the allocation (max(nsel_d, nwg))
    c->lost += std::max<int64_t>(c->enq - h.pivots, 0);
    c->enq = h.pivots;
    c->pend = (int)h.npend;
    c->booted = false;
    c->res_fallbacks++;
    HIPCHK(c, hipMemsetAsync(&c->st->stall, 0, sizeof(int64_t), c->stream));
    return 0;
}

// A region-mode launch found DevState::rbad set (a block's column trade was
// incomplete, so the block start's nonbasic columns moved) and ran no pivot,
// nor did any launch after it: the next enqueue bootstraps (restoring the
// caller's column order, then rebuilding the region, which clears rbad) and
// lpg_sync re-runs the lost pivots, as after a residency abort.
static int recover_region(lpg_ctx *c, const DevState &h) {
    c->reg_recoveries++;
    c->lost += std::max<int64_t>(c->enq - h.pivots, 0);
    c->enq = h.pivots;
    c->pend = (int)h.npend;
    c->booted = false;
    c->reg_valid = false;
    HIPCHK(c, hipMemsetAsync(&c->st->stall, 0, sizeof(int64_t), c->stream));
    return 0;
}

// k_swap_plan refused the pending block (lpg_kernels.hip): the loop was
// stopped with NUMERIC and nothing of the block was applied.
static int pending_fault(lpg_ctx *c, const DevState &h) {
    static const char *const what[] = {"?", "npend", "kq", "lv", "rq"};
    const int64_t w = h.stall_info[0] >= 1 && h.stall_info[0] <= 4 ? h.stall_info[0] : 0;
    c->poisoned = true;   // the basis holds the block's pivots, the constraint rows do not
    return fail(c, LPG_ERR_STATE,
                "pending block inconsistent at the flush (%s[%lld] = %lld, npend %lld): the loop was stopped with "
                "NUMERIC instead of indexing with it; the constraint rows were not brought up to date",
                what[w], (long long)h.stall_info[1], (long long)h.stall_info[2], (long long)h.stall_info[3]);
}

// Every pivoting entry point: a context whose pending block was refused
// (pending_fault) stays refused until the basis is replaced (lpg_set_basis,
// normally after lpg_load_rows) or the LP regenerated (lpg_generate)
// (continuing would pivot on a basis and constraint rows that
// disagree; ADVICE r5: a row reload alone no longer clears it).
static int usable(lpg_ctx *c) {
    if (!c->poisoned) return 0;
    return fail(c, LPG_ERR_STATE, "context unusable: an earlier flush refused an inconsistent pending block, so the "
                "basis and the constraint rows disagree; reload the rows and the basis (lpg_load_rows, lpg_set_basis) or "
                "regenerate (lpg_generate) the LP");
}

static int read_result(lpg_ctx *c, lpg_result *out, int rule) {
    DevState h;
    HIPCHK(c, hipMemcpyAsync(&h, c->st, sizeof h, hipMemcpyDeviceToHost, c->stream));
    double z = 0;
    HIPCHK(c, hipMemcpyAsync(&z, c->T + (c->nloc + c->nobj - 1) * c->ld, sizeof z, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (h.stall == kStallResidency) {
        int rc = recover_residency(c, h);
        if (rc) return rc;
        h.stall = 0;
    }
    if (h.stall == kStallRegion) {
        int rc = recover_region(c, h);
        if (rc) return rc;
        h.stall = 0;
    }
    if (h.stall == kStallPending) return pending_fault(c, h);
    if (h.stall == 2 || h.stall == 3)
        return fail(c, LPG_ERR_COMM, "owner-push exchange: rank %d waited > 2 s for the %s (a rank stopped, or the "
                    "buffers are not shared; LPG_EXCHANGE=rccl keeps the collectives)", c->rank,
                    h.stall == 2 ? "other ranks' ratio candidates" : "pivot row");
    if (h.stall)
        return fail(c, LPG_ERR_DEVICE,
                    "k_pivot_block: a workgroup waited > 2 s for the others (phase %lld, tag %lld, record %lld "
                    "showed tag %lld; is another kernel holding CUs? LPG_PERSIST=0 uses the two-kernel pivot)",
                    (long long)h.stall_info[0], (long long)h.stall_info[1], (long long)h.stall_info[2],
                    (long long)h.stall_info[3]);
    if (out) {
        const int32_t s = c->booted ? h.slot[c->par].status : RUNNING;
        out->status = s == RUNNING ? LPG_ITER_LIMIT : s;
        out->rule = rule;
        out->pivots = h.pivots;
        out->objective = z;
        out->entering = h.pivots ? h.last_k : -1;
        out->leaving = h.pivots ? h.last_r : -1;
    }
    return 0;
}

static int reset_state(lpg_ctx *c) {
    DevState h;
    memset(&h, 0, sizeof h);
    h.logcap = c->logcap;
    h.last_k = h.last_r = -1;
    HIPCHK(c, hipMemcpyAsync(c->st, &h, sizeof h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->booted = false;
    c->par = 0;
    c->enq = 0;
    c->pend = 0;
    c->touched_mark = 0;
    c->pb_launch = 0;      // the census counts from 0 again (DevState::rcnt / rdec are zero)
    c->lost = 0;
    return 0;
}

static void graph_drop(lpg_ctx *c);

static int ensure_log(lpg_ctx *c, int64_t need) {
    if (c->flags & LPG_FLAG_NO_LOG) return 0;
    if (need <= c->logcap) return 0;
    graph_drop(c);   // a captured graph holds the old log pointers
    int64_t cap = std::max<int64_t>(need, 2 * c->logcap);
    int64_t *nk = nullptr, *nr = nullptr;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMalloc(&nk, cap * sizeof(int64_t)));
    HIPCHK(c, hipMalloc(&nr, cap * sizeof(int64_t)));
    if (c->logk) {
        HIPCHK(c, hipMemcpy(nk, c->logk, c->logcap * sizeof(int64_t), hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(nr, c->logr, c->logcap * sizeof(int64_t), hipMemcpyDeviceToDevice));
        HIPCHK(c, hipFree(c->logk));
        HIPCHK(c, hipFree(c->logr));
    }
    c->logk = nk;
    c->logr = nr;
    c->logcap = cap;
    HIPCHK(c, hipMemcpy(&c->st->logcap, &cap, sizeof cap, hipMemcpyHostToDevice));
    return 0;
}

static int64_t device_pivots(lpg_ctx *c) {
    int64_t n = 0;
    if (hipMemcpy(&n, &c->st->pivots, sizeof n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return n;
}

// ---------------------------------------------------------------------------
// extern "C" API
// ---------------------------------------------------------------------------

extern "C" {

const char *lpg_last_error(const lpg_ctx *c) { return c ? c->err : g_err; }

int lpg_device_count(int *count) {
    if (!count) return fail(nullptr, LPG_ERR_ARG, "count is NULL");
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return fail(nullptr, LPG_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    return 0;
}

int lpg_create_dist(lpg_ctx **out, int device, int world, int rank, int64_t m, int64_t ncols, uint32_t flags) {
    if (!out) return fail(nullptr, LPG_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (m < 1 || ncols < 2 || world < 1 || rank < 0 || rank >= world || world > m)
        return fail(nullptr, LPG_ERR_ARG, "bad shape m=%lld ncols=%lld world=%d rank=%d", (long long)m,
                    (long long)ncols, world, rank);
    lpg_ctx *c = new lpg_ctx();
    c->device = device;
    c->world = world;
    c->rank = rank;
    c->m = m;
    c->ncols = ncols;
    c->ld = (ncols + 63) & ~(int64_t)63;   // 512-byte aligned rows
    c->nobj = (flags & LPG_FLAG_BIG_M) ? 2 : 1;
    c->row0 = m * rank / world;
    c->nloc = m * (rank + 1) / world - c->row0;
    c->nact = ncols - 1;
    c->flags = flags;
    const char *uv = getenv("LPG_UPDATE_VARIANT");
    c->update_variant = uv ? atoi(uv) : -1;   // -1: size-adaptive default (launch_update)
    const char *ng = getenv("LPG_NO_GRAPH");
    c->use_graphs = !(ng && atoi(ng));
    const char *gr = getenv("LPG_GRAPH_RCCL");
    c->graph_comm = gr && atoi(gr);
    const char *ns = getenv("LPG_NO_SKIP");
    c->skip = ((flags & LPG_FLAG_NO_SKIP) || (ns && atoi(ns))) ? 0 : 1;
    const char *dk = getenv("LPG_DEFER");
    // default block: 64 pivots once this rank's tableau is >= 200 MB (the
    // flush dominates; k_flushw keeps 64-pivot flushes memory-bound), 32 below
    // (the per-pivot work dominates: m = 2048, n = 4096 (100 MB) 100k pivots/s
    // at 32, 99k at 64; m = 4096, n = 8192 (403 MB) 77k / 82k,
    // profiles/r02_k32_64.log)
    const int64_t nloc_max = (m + world - 1) / world;    // the largest row block: every rank decides alike
    // 96 once it is >= 16 GB (too big for the persistent pivot kernel's
    // slices, so the pair runs the pivots): the 96- and 128-pivot passes both
    // sit at ~47 TFLOP/s on the matrix cores (the same cost per pivot, 23%
    // below 64-pivot passes), and the pair's chains are shorter at 96 --
    // config 4: 2,424 vs 2,347 pivots/s (profiles/r03_bench_config4_k96.json)
    const double tbytes = (double)nloc_max * (double)ncols * 8.0;
    // the block-end column trade (§3.3 of DESIGN.md) pays where the block pass
    // is long; below 2 GB on one rank its kernels cost more than scattered
    // live columns do (config 2: 105k -> 112k pivots/s without it, config 5:
    // 67k -> 69k, config 3: 25k -> 21k). LPG_NO_REORDER=0/1 decides instead.
    const char *nr = getenv("LPG_NO_REORDER");
    c->no_reorder = nr ? atoi(nr) != 0 : (world == 1 && tbytes < 2e9);
    const char *sp = getenv("LPG_SLOW_PIVOT");
    c->fast_pivot = !(sp && atoi(sp));
    // the persistent pivot launch (LPG_PERSIST=0: the two-kernel pair) and its
    // region mode (one rank, one objective row, the column trade on;
    // LPG_REGION=0: the all-column slices)
    const char *pe = getenv("LPG_PERSIST"), *pw = getenv("LPG_PERSIST_WG"), *pr = getenv("LPG_REGION");
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 0;
    const bool persist_ok = c->fast_pivot && !(pe && atoi(pe) == 0) && cus > 0;
    // (with world > 1 region mode runs on the ranks of a push exchange)
    const bool reg_ok = persist_ok && c->nobj == 1 && !c->no_reorder && !(pr && atoi(pr) == 0);
    const int64_t nlive = ncols - 1 - m;                 // nonbasic columns other than column 0 (any basis)
    Geo g0{};
    g0.nloc = nloc_max;
    g0.nobj = c->nobj;
    g0.ncols = ncols;
    g0.m = m;
    int kdef = tbytes >= 16e9 ? kDefaultDeferHuge : tbytes >= 200e6 ? kDefaultDefer : kDefaultDeferSmall;
    // region mode at 96-pivot blocks where the pass dominates (>= 2 GB) and the
    // region's slices hold 96 slots: the 96-pivot pass costs ~12% less per
    // pivot than the 64-pivot one (config-3 shape: 2.15 vs 1.625 ms per pass,
    // profiles/r04_flush96_lab.log, r04_ab_k72_*), which the all-column
    // slices could not hold (config 3: 49,153 columns at 96 slots = 37 MB of LDS).
    // On the ranks of a row partition from 1 GB: config 3's P = 4 rank (4096
    // rows, stand-in with the push and the trade) 48.8k pivots/s at 64, 54.6k
    // at 96; P = 8 (0.8 GB) 60.8k vs 59.5k (profiles/r05_ab_mrreg_p48.log)
    RegionGeo rg96{};
    if (reg_ok && tbytes >= (world > 1 ? 1e9 : 2e9) && tbytes < 16e9 && nlive > 0 &&
        block_geometry_region(g0, 96, cus, pw ? atoi(pw) : 0, nlive, &rg96) == 0)
        kdef = 96;
    c->defer_k = (flags & LPG_FLAG_EAGER) ? 0 : (dk ? atoi(dk) : kdef);
    if (c->defer_k < 0 || c->defer_k > LPG_DEFER_MAX || (c->defer_k && !flush_kmax_supported(c->defer_k))) {
        fail(c, LPG_ERR_ARG, "LPG_DEFER=%d out of range [0, %d]", c->defer_k, LPG_DEFER_MAX);
        snprintf(g_err, sizeof g_err, "%s", c->err);
        delete c;
        return LPG_ERR_ARG;
    }
#ifdef LPG_TEST_HOOKS
    // the test-hook build only (linearprogramming_amd/liblpg_testhooks.so,
    // Makefile): the product library never reads this variable
    if (const char *pf = getenv("LPG_TEST_PENDING_FAULT")) {
        char w[16] = {0};
        int f = -1;
        if (sscanf(pf, "%d:%15s", &f, w) == 2) {
            static const char *const names[] = {"", "npend", "kq", "lv", "rq", "ahead"};
            for (int u = 1; u <= 5; u++)
                if (!strcmp(w, names[u])) c->inject_what = u;
            c->inject_flush = c->inject_what ? f : -1;
        }
    }
    if (const char *rb = getenv("LPG_TEST_REGION_BAD")) c->inject_rbad = atoi(rb);
#endif
    const char *fv = getenv("LPG_FLUSH_KERNEL");   // m | w: force k_flushm / k_flushw (tests); default by block size
    c->flush_variant = fv ? (fv[0] == 'w' ? 1 : fv[0] == 'm' ? 0 : -1) : -1;
    // 0 | 1 | h1, h2, h4, h8: k_flushw's global / XCD-grouped item queue, the
    // latter with H column classes (tests, A/B); unset: by size
    const char *ft = getenv("LPG_FLUSH_TLIVE");
    c->tlive_on = !(ft && ft[0] == '0');
    {
        const char *mu = getenv("LPG_MOVE_UNIT");
        c->move_unit = !(mu && mu[0] == '0');
    }
    const char *fx = getenv("LPG_FLUSH_XCD");
    c->flush_xcd = -1;
    if (fx && fx[0] == '0') c->flush_xcd = 0;
    if (fx && fx[0] == '1') c->flush_xcd = 1;
    if (fx && fx[0] == 'h' && (fx[1] == '1' || fx[1] == '2' || fx[1] == '4' || fx[1] == '8')) c->flush_xcd = 10 + (fx[1] - '0');
    int rc;
    if ((rc = use_device(c))) { lpg_destroy(c); return rc; }
    const int64_t rows = c->nloc + c->nobj;
    const Geo g = geo(c);
    c->npp = price_blocks(g);
    const int64_t maxloc = (m + world - 1) / world + c->nobj;   // identical on every rank
    c->nsel = (int)std::min<int64_t>((maxloc + kBlock - 1) / kBlock, kMaxSelBlocks);
    c->npp_d = pivot_d_blocks(g, 0, c->pivot_nt);
    // k_select_d: one row per thread; with world > 1 the count must be the
    // same on every rank (the candidates are allgathered)
    c->nsel_d = world == 1 ? pivot_d_blocks(g, 1, c->pivot_nt) : (int)((maxloc + 255) / 256);
    {
        // the split is computed for the largest row block, so every rank of a
        // row partition gets the same workgroups, columns and rows per slice
        // (the multi-rank form exchanges P slice by slice)
        Geo gm = g;
        gm.nloc = (m + world - 1) / world;
        if (c->defer_k > 0 && persist_ok &&
            block_geometry(gm, c->defer_k, cus, pw ? atoi(pw) : 0, &c->pb_nwg, &c->pb_cw, &c->pb_rw, &c->pb_lds) == 0) {
            c->pmr = true;
            if (world == 1) {
                c->persist = true;
                c->nsel_d = c->pb_nwg;      // one ratio candidate per workgroup
            }
        }
        // region mode where its slices fit (preferred over the all-column form);
        // on ranks (largest row block) it runs once a push exchange is attached
        if (c->defer_k > 0 && reg_ok && nlive > 0 &&
            block_geometry_region(gm, c->defer_k, cus, pw ? atoi(pw) : 0, nlive, &c->rg) == 0) {
            c->reg = true;
            if (world == 1) {
                c->persist = true;
                c->nsel_d = c->rg.nwg;
            }
        }
    }
#define ALLOC(p, bytes)                                                                    \
    do {                                                                                   \
        hipError_t e_ = hipMalloc((void **)&(p), (bytes));                                 \
        if (e_ != hipSuccess) {                                                            \
            fail(c, LPG_ERR_OOM, "hipMalloc(%s, %zu): %s", #p, (size_t)(bytes), hipGetErrorString(e_)); \
            snprintf(g_err, sizeof g_err, "%s", c->err);                                   \
            lpg_destroy(c);                                                                \
            return LPG_ERR_OOM;                                                            \
        }                                                                                  \
    } while (0)
    ALLOC(c->T, (size_t)rows * c->ld * sizeof(double));
    ALLOC(c->P, (size_t)c->ld * sizeof(double));
    ALLOC(c->C[0], (size_t)rows * sizeof(double));
    ALLOC(c->C[1], (size_t)rows * sizeof(double));
    ALLOC(c->acc, (size_t)c->ld * world * sizeof(double));
    ALLOC(c->cb, (size_t)std::max<int64_t>(c->nloc, 1) * sizeof(double));
    ALLOC(c->cost, (size_t)ncols * sizeof(double));
    ALLOC(c->pp, (size_t)std::max(c->npp, c->npp_d) * sizeof(PricePart));
    ALLOC(c->pc, (size_t)c->npp * sizeof(int));
    const int nwg_rec = std::max(c->pmr ? c->pb_nwg : 0, c->reg ? c->rg.nwg : 0);
    ALLOC(c->part, (size_t)std::max({c->nsel, c->nsel_d, nwg_rec}) * sizeof(Cand));
    if (nwg_rec) ALLOC(c->rec, (size_t)block_records_bytes(nwg_rec));
    if (c->reg) {
        ALLOC(c->live, (size_t)ncols * sizeof(int32_t));
        ALLOC(c->mark, (size_t)c->ld * sizeof(int32_t));
        ALLOC(c->tlive, (size_t)(c->ld / 64 + 1) * sizeof(int32_t));
        ALLOC(c->bcol0, (size_t)m * sizeof(int64_t));
        ALLOC(c->rok, (size_t)(1 + world) * sizeof(int));
    }
    if (world > 1) ALLOC(c->cand, (size_t)std::max(c->nsel, c->nsel_d) * world * sizeof(Cand));
    else c->cand = c->part;
    ALLOC(c->basis, (size_t)m * sizeof(int64_t));
    ALLOC(c->st, sizeof(DevState));
    if (c->defer_k > 0) {
        c->cs = std::max<int64_t>((c->nloc + 63) & ~(int64_t)63, 64);
        // slots up to the flush kernel's compiled bound (it reads C of every slot)
        const int64_t slots = flush_kmax_supported(c->defer_k);
        ALLOC(c->Pbuf, (size_t)slots * c->ld * sizeof(double));
        ALLOC(c->Cbuf, (size_t)slots * c->cs * sizeof(double));
        ALLOC(c->rq, (size_t)slots * sizeof(int64_t));
        if (c->reg) ALLOC(c->rqg, (size_t)slots * sizeof(int64_t));
        ALLOC(c->zrow, (size_t)c->ld * sizeof(double));
        ALLOC(c->kq, (size_t)slots * sizeof(int64_t));
        ALLOC(c->lv, (size_t)slots * sizeof(int64_t));
        ALLOC(c->colmap, (size_t)c->ld * sizeof(int32_t));
        ALLOC(c->inv, (size_t)c->ld * sizeof(int32_t));
        ALLOC(c->pairs, (size_t)(1 + kPairW * LPG_DEFER_MAX) * sizeof(int32_t));
        ALLOC(c->mul, (size_t)LPG_DEFER_MAX * LPG_DEFER_MAX * sizeof(double));
        ALLOC(c->pv, (size_t)slots * sizeof(double));
    }
#undef ALLOC
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        fail(c, LPG_ERR_DEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
        lpg_destroy(c);
        return LPG_ERR_DEVICE;
    }
    c->own_stream = true;
    if (hipMemset(c->T, 0, (size_t)rows * c->ld * sizeof(double)) != hipSuccess ||
        hipMemset(c->P, 0, (size_t)c->ld * sizeof(double)) != hipSuccess ||
        hipMemset(c->basis, 0, (size_t)m * sizeof(int64_t)) != hipSuccess ||
        (c->Cbuf && hipMemset(c->Cbuf, 0, (size_t)flush_kmax_supported(c->defer_k) * c->cs * sizeof(double)) != hipSuccess) ||
        (c->Pbuf && hipMemset(c->Pbuf, 0, (size_t)flush_kmax_supported(c->defer_k) * c->ld * sizeof(double)) != hipSuccess) ||
        (c->zrow && hipMemset(c->zrow, 0, (size_t)c->ld * sizeof(double)) != hipSuccess) ||
        // slots no pivot of the current block filled read as out of range
        // (kq = lv = 0: no column; rq 0x8080.. < -1: no row), which k_swap_plan
        // refuses; every block's end writes the same sentinels back (end_block)
        (c->kq && hipMemset(c->kq, 0, (size_t)flush_kmax_supported(c->defer_k) * sizeof(int64_t)) != hipSuccess) ||
        (c->lv && hipMemset(c->lv, 0, (size_t)flush_kmax_supported(c->defer_k) * sizeof(int64_t)) != hipSuccess) ||
        (c->rq && hipMemset(c->rq, 0x80, (size_t)flush_kmax_supported(c->defer_k) * sizeof(int64_t)) != hipSuccess) ||
        (c->pv && hipMemset(c->pv, 0, (size_t)flush_kmax_supported(c->defer_k) * sizeof(double)) != hipSuccess) ||
        (c->rec && hipMemset(c->rec, 0, (size_t)block_records_bytes(nwg_rec)) != hipSuccess) ||
        (c->colmap && (launch_iota(lau(c), c->colmap, c->ld) || launch_iota(lau(c), c->inv, c->ld)))) {
        fail(c, LPG_ERR_DEVICE, "hipMemset failed");
        lpg_destroy(c);
        return LPG_ERR_DEVICE;
    }
    if ((rc = ensure_log(c, 1024)) || (rc = reset_state(c))) {
        lpg_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

int lpg_create(lpg_ctx **out, int device, int64_t m, int64_t ncols, uint32_t flags) {
    return lpg_create_dist(out, device, 1, 0, m, ncols, flags);
}

int lpg_comm_unique_id(void *uid, size_t len) {
    if (!uid || len < sizeof(ncclUniqueId)) return fail(nullptr, LPG_ERR_ARG, "uid buffer too small");
    const RcclApi *R = rccl_api();
    if (!R) return fail(nullptr, LPG_ERR_COMM, "RCCL (librccl.so.1) not loadable");
    ncclUniqueId id;
    ncclResult_t r = R->GetUniqueId(&id);
    if (r != ncclSuccess) return fail(nullptr, LPG_ERR_COMM, "ncclGetUniqueId: %s", R->GetErrorString(r));
    memcpy(uid, &id, sizeof id);
    return 0;
}

// With a communicator the deferred pair runs in 256-thread blocks (its
// candidate count must match across ranks): drop a 128-thread choice.
static void comm_pivot_blocks(lpg_ctx *c) {
    if (c->persist) {   // the single-rank form; the multi-rank one comes with the push exchange (attach_push)
        c->persist = false;
        c->nsel_d = pivot_d_blocks(geo(c), 1, 256);    // <= the allocation (sized for max(nsel, nwg))
        c->booted = false;
    }
    if (c->pivot_nt == 256) return;
    c->pivot_nt = 256;
    c->npp_d = pivot_d_blocks(geo(c), 0, 256);    // buffers were sized for the larger 128-thread counts
    c->nsel_d = pivot_d_blocks(geo(c), 1, 256);
    c->booted = false;
    graph_drop(c);
}

int lpg_comm_init_rccl(lpg_ctx *c, const void *uid, size_t len) {
    if (!c || !uid || len < sizeof(ncclUniqueId)) return fail(c, LPG_ERR_ARG, "bad uid");
    if (c->nccl || c->have_hops) return fail(c, LPG_ERR_STATE, "communicator already attached");
    const RcclApi *R = rccl_api();
    if (!R) return fail(c, LPG_ERR_COMM, "RCCL (librccl.so.1) not loadable");
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;   // the generic kernels work in caller order
    ncclUniqueId id;
    memcpy(&id, uid, sizeof id);
    comm_pivot_blocks(c);
    ncclResult_t r = R->CommInitRank(&c->nccl, c->world, id, c->rank);
    if (r != ncclSuccess) {
        c->nccl = nullptr;
        return fail(c, LPG_ERR_COMM, "ncclCommInitRank: %s", R->GetErrorString(r));
    }
    return 0;
}

int lpg_comm_init_host(lpg_ctx *c, const lpg_host_comm_ops *ops) {
    if (!c || !ops || !ops->allgather || !ops->allreduce_sum_f64) return fail(c, LPG_ERR_ARG, "bad host comm ops");
    if (c->nccl || c->have_hops) return fail(c, LPG_ERR_STATE, "communicator already attached");
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    comm_pivot_blocks(c);
    c->hops = *ops;
    c->have_hops = true;
    return 0;
}

// ---- owner-push exchange ----
static int ensure_xbuf(lpg_ctx *c) {
    if (c->xbuf) return 0;
    if (!(c->defer_k > 0 && c->fast_pivot)) return fail(c, LPG_ERR_STATE, "push exchange needs the deferred pivot pair");
    // P chunk flags: prep blocks / k_pivot_block slices (all-column or region)
    c->xnblk = std::max({c->npp_d, c->pmr ? c->pb_nwg : 0, c->reg ? c->rg.nwg : 0});
    c->xnx = c->nsel_d;
    c->xbytes = xch_bytes(c->ld, c->world, c->xnblk, c->xnx, &c->xoffF, &c->xoffC, &c->xoffG);
    // uncached: a peer's stores over xGMI land in this GPU's HBM behind its
    // L2; with L2 out of the path the system-scope loads cannot hit a stale line
    void *p = nullptr;
    if (hipExtMallocWithFlags(&p, (size_t)c->xbytes, hipDeviceMallocUncached) == hipSuccess) {
        c->xuncached = true;
    } else {
        (void)hipGetLastError();
        HIPCHK(c, hipMalloc(&p, (size_t)c->xbytes));
    }
    c->xbuf = (char *)p;
    HIPCHK(c, hipMemset(c->xbuf, 0, (size_t)c->xbytes));
    // identity of the GPU this buffer lives on, read by every peer at attach
    // (push_shares_device): PCI bus id, then the owning process id
    char id[kXchIdBytes] = {0};
    HIPCHK(c, hipDeviceGetPCIBusId(id, 48, c->device));
    const int32_t pid = (int32_t)getpid();
    memcpy(id + 48, &pid, sizeof pid);
    HIPCHK(c, hipMemcpy(c->xbuf + c->xoffG + kXchIdOff, id, sizeof id, hipMemcpyHostToDevice));
    return 0;
}

// the push's kernels spin-wait on a peer's kernel, so
// two ranks must never depend on each other for CUs or hardware queues. Two
// refusals at attach time, each with a named error, instead of a 2 s
// exchange timeout in the middle of a solve:
//  * ranks of ONE process (lpg_comm_init_push_local, world > 1) share its
//    hardware queues (GPU_MAX_HW_QUEUES): a rank's waiting kernel can sit in
//    front of the peer kernel it waits for (tools/soak_dist.py measured 108
//    such timeouts in 784 cases with 4 queues, 14 in 2,721 with 16);
//  * ranks of several processes on ONE GPU (the same PCI bus id in their
//    exchange buffers) share its CUs: a non-owner's spinning grid can hold
//    the CUs the owner's grid needs.
// The deployment layout (one process per GPU: bench.py under
// torch.distributed, lpgcli --gpus P on a P-GPU node) passes both checks.
// Tests that exercise the protocol on the one GPU of this pool, at sizes
// whose grids co-reside, acknowledge the sharing with LPG_PUSH_SHARED_QUEUES=1
// / LPG_PUSH_SHARED_DEVICE=1.
static bool env_on(const char *name) {
    const char *v = getenv(name);
    return v && atoi(v) != 0;
}

static int push_shares_device(lpg_ctx *c, const std::vector<char *> &bases) {
    if (env_on("LPG_PUSH_SHARED_DEVICE")) return 0;
    char mine[kXchIdBytes], peer[kXchIdBytes];
    HIPCHK(c, hipMemcpy(mine, c->xbuf + c->xoffG + kXchIdOff, sizeof mine, hipMemcpyDeviceToHost));
    for (int r = 0; r < c->world; r++) {
        if (r == c->rank) continue;
        HIPCHK(c, hipMemcpy(peer, bases[r] + c->xoffG + kXchIdOff, sizeof peer, hipMemcpyDeviceToHost));
        if (peer[0] && !strncmp(mine, peer, 48)) {
            int32_t pid_mine, pid_peer;      // the owning processes, named in the message
            memcpy(&pid_mine, mine + 48, sizeof pid_mine);
            memcpy(&pid_peer, peer + 48, sizeof pid_peer);
            return fail(c, LPG_ERR_STATE,
                        "owner-push exchange refused: ranks %d (pid %d) and %d (pid %d) share GPU %.48s, so a rank's "
                        "spin-waiting exchange kernel can hold the CUs its peer needs; use one GPU per rank, or the "
                        "collectives (LPG_PUSH_SHARED_DEVICE=1 acknowledges the sharing for small co-resident tests)",
                        c->rank, (int)pid_mine, r, (int)pid_peer, mine);
        }
    }
    return 0;
}

static int attach_push(lpg_ctx *c, std::vector<char *> &bases) {
    HIPCHK(c, hipMalloc((void **)&c->xbase, bases.size() * sizeof(char *)));
    HIPCHK(c, hipMemcpy(c->xbase, bases.data(), bases.size() * sizeof(char *), hipMemcpyHostToDevice));
    graph_drop(c);
    c->xmode = true;
    c->booted = false;               // the next pivot bootstraps (its candidates through the communicator)
    // the pivot loop as one launch per block on every rank (LPG_PERSIST=0 or
    // LPG_PERSIST_MR=0: the two-kernel pair)
    const char *pe = getenv("LPG_PERSIST"), *pm = getenv("LPG_PERSIST_MR");
    c->persist_x = (c->pmr || c->reg) && !(pe && atoi(pe) == 0) && !(pm && atoi(pm) == 0);
    return 0;
}

int lpg_comm_push_handle(lpg_ctx *c, void *handle, size_t len) {
    if (!c || !handle || len < sizeof(hipIpcMemHandle_t)) return fail(c, LPG_ERR_ARG, "push handle buffer too small");
    if (!has_comm(c)) return fail(c, LPG_ERR_STATE, "attach a communicator before the push exchange");
    int rc;
    if ((rc = use_device(c)) || (rc = ensure_xbuf(c))) return rc;
    hipIpcMemHandle_t h;
    HIPCHK(c, hipIpcGetMemHandle(&h, c->xbuf));
    memcpy(handle, &h, sizeof h);
    return 0;
}

int lpg_comm_push_base(lpg_ctx *c, void **base) {
    if (!c || !base) return fail(c, LPG_ERR_ARG, "base is NULL");
    if (!has_comm(c)) return fail(c, LPG_ERR_STATE, "attach a communicator before the push exchange");
    int rc;
    if ((rc = use_device(c)) || (rc = ensure_xbuf(c))) return rc;
    *base = c->xbuf;
    return 0;
}

int lpg_comm_init_push(lpg_ctx *c, const void *handles, size_t len) {
    if (!c || !handles || len != (size_t)c->world * sizeof(hipIpcMemHandle_t))
        return fail(c, LPG_ERR_ARG, "need world x %zu handle bytes", sizeof(hipIpcMemHandle_t));
    if (c->xmode) return fail(c, LPG_ERR_STATE, "push exchange already attached");
    int rc;
    if ((rc = use_device(c)) || (rc = ensure_xbuf(c))) return rc;
    std::vector<char *> bases((size_t)c->world, nullptr);
    for (int r = 0; r < c->world; r++) {
        if (r == c->rank) {
            bases[r] = c->xbuf;
            continue;
        }
        hipIpcMemHandle_t h;
        memcpy(&h, (const char *)handles + (size_t)r * sizeof h, sizeof h);
        void *p = nullptr;
        HIPCHK(c, hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        c->xpeer.push_back(p);
        bases[r] = (char *)p;
    }
    if ((rc = push_shares_device(c, bases))) {
        for (void *p : c->xpeer) (void)hipIpcCloseMemHandle(p);
        c->xpeer.clear();
        return rc;
    }
    return attach_push(c, bases);
}

int lpg_comm_init_push_local(lpg_ctx *c, void *const *bases_in, int world) {
    if (!c || !bases_in || world != c->world) return fail(c, LPG_ERR_ARG, "need world device pointers");
    if (c->xmode) return fail(c, LPG_ERR_STATE, "push exchange already attached");
    int rc;
    if ((rc = use_device(c)) || (rc = ensure_xbuf(c))) return rc;
    if (bases_in[c->rank] != c->xbuf) return fail(c, LPG_ERR_ARG, "bases[rank] is not this rank's buffer");
    if (world > 1 && !env_on("LPG_PUSH_SHARED_QUEUES"))
        return fail(c, LPG_ERR_STATE,
                    "owner-push exchange refused: the %d ranks are threads of one process and share its hardware "
                    "queues, so a rank's spin-waiting exchange kernel can sit in front of the peer kernel it waits "
                    "for; use one process per GPU, or the collectives (LPG_PUSH_SHARED_QUEUES=1 acknowledges the "
                    "sharing for tests)", world);
    std::vector<char *> bases((size_t)world);
    for (int r = 0; r < world; r++) bases[r] = (char *)bases_in[r];
    return attach_push(c, bases);
}

void lpg_destroy(lpg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    graph_drop(c);
    if (c->nccl) rccl_api()->CommDestroy(c->nccl);
    for (void *p : c->xpeer) (void)hipIpcCloseMemHandle(p);
    if (c->xbase) (void)hipFree(c->xbase);
    if (c->xbuf) (void)hipFree(c->xbuf);
    for (hipEvent_t e : c->tr.ev) (void)hipEventDestroy(e);
    if (c->cand && c->cand != c->part) (void)hipFree(c->cand);
    void *bufs[] = {c->T, c->P, c->C[0], c->C[1], c->acc, c->cb, c->cost, c->pp, c->pc, c->part, c->basis, c->logk, c->logr, c->st,
                    c->Pbuf, c->Cbuf, c->rq, c->rqg, c->zrow, c->kq, c->lv, c->colmap, c->inv, c->pairs, c->mul, c->pv, c->tmp,
                    c->rec, c->drc, c->dcp, c->drc_all, c->live, c->mark, c->bcol0, c->rok, c->tlive};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int lpg_info(const lpg_ctx *c, lpg_info_t *o) {
    if (!c || !o) return fail(const_cast<lpg_ctx *>(c), LPG_ERR_ARG, "NULL argument");
    o->m = c->m;
    o->ncols = c->ncols;
    o->ld = c->ld;
    o->row0 = c->row0;
    o->nrows = c->nloc;
    o->world = c->world;
    o->rank = c->rank;
    o->device = c->device;
    o->nobj = (int32_t)c->nobj;
    o->defer_k = c->defer_k;
    const bool pb = (c->persist && !has_comm(c)) || (c->persist_x && c->xmode);
    o->pivot_wg = pb ? (c->reg ? c->rg.nwg : c->pb_nwg) : 0;
    o->bytes_per_pivot = 16.0 * (double)(c->nloc + c->nobj) * (double)c->ncols;
    o->exchange = c->xmode ? (c->xuncached ? 2 : 1) : 0;
    o->column_trade = reorders(c) ? 1 : 0;
    o->residency_fallbacks = c->res_fallbacks;
    o->region_recoveries = c->reg_recoveries;
    o->region = (o->pivot_wg > 0 && c->reg) ? 1 : 0;
    return 0;
}

int lpg_load_rows(lpg_ctx *c, int64_t row0, int64_t nrows, const double *rows, int64_t ld) {
    if (!c || !rows || row0 < 0 || nrows < 0 || row0 + nrows > c->m + c->nobj || ld < c->ncols)
        return fail(c, LPG_ERR_ARG, "lpg_load_rows: bad arguments");
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    // canonicalize() queues work on c->stream (non-blocking): the synchronous
    // copies below go through the null stream and must not overtake it
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // constraint rows inside this rank's block
    const int64_t a = std::max(row0, c->row0), b = std::min(row0 + nrows, c->row0 + c->nloc);
    if (a < b)
        HIPCHK(c, hipMemcpy2D(c->T + (a - c->row0) * c->ld, c->ld * sizeof(double), rows + (a - row0) * ld,
                              ld * sizeof(double), c->ncols * sizeof(double), b - a, hipMemcpyHostToDevice));
    // objective row(s): global index m + q, replicated on every rank
    for (int64_t q = 0; q < c->nobj; q++) {
        const int64_t gi = c->m + q;
        if (gi >= row0 && gi < row0 + nrows)
            HIPCHK(c, hipMemcpy(c->T + (c->nloc + q) * c->ld, rows + (gi - row0) * ld, c->ncols * sizeof(double),
                                hipMemcpyHostToDevice));
    }
    // (a refused context stays refused: rows alone, even all of them, do not
    // replace the basis that holds the refused block's pivots -- lpg_set_basis
    // or lpg_generate clears it)
    c->units_known = false;   // region mode checks the basic columns first (region_setup)
    return reset_state(c);
}

int lpg_set_basis(lpg_ctx *c, const int64_t *basis) {
    if (!c || !basis) return fail(c, LPG_ERR_ARG, "basis is NULL");
    for (int64_t i = 0; i < c->m; i++)
        if (basis[i] < 1 || basis[i] >= c->ncols) return fail(c, LPG_ERR_ARG, "basis[%lld] out of range", (long long)i);
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(c->basis, basis, c->m * sizeof(int64_t), hipMemcpyHostToDevice));
    c->units_known = false;
    c->poisoned = false;   // the caller's basis replaces the one holding a refused block's pivots
    return reset_state(c);
}

static int set_objective_row(lpg_ctx *c, const double *cost, int64_t orow);

int lpg_set_objective(lpg_ctx *c, const double *cost) {
    if (!c || !cost) return fail(c, LPG_ERR_ARG, "cost is NULL");
    return set_objective_row(c, cost, c->nloc + c->nobj - 1);
}

int lpg_set_objective_m(lpg_ctx *c, const double *costM) {
    if (!c || !costM) return fail(c, LPG_ERR_ARG, "cost is NULL");
    if (c->nobj != 2) return fail(c, LPG_ERR_STATE, "lpg_set_objective_m needs a context created with LPG_FLAG_BIG_M");
    return set_objective_row(c, costM, c->nloc);
}

static int set_objective_row(lpg_ctx *c, const double *cost, int64_t orow) {
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<int64_t> hb(c->m);
    HIPCHK(c, hipMemcpy(hb.data(), c->basis, c->m * sizeof(int64_t), hipMemcpyDeviceToHost));
    std::vector<double> hcb(std::max<int64_t>(c->nloc, 1));
    for (int64_t i = 0; i < c->nloc; i++) {
        const int64_t col = hb[c->row0 + i];
        if (col < 1 || col >= c->ncols) return fail(c, LPG_ERR_STATE, "basis not set (row %lld)", (long long)(c->row0 + i));
        hcb[i] = cost[col - 1];
    }
    HIPCHK(c, hipMemcpy(c->cb, hcb.data(), c->nloc * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->cost, cost, (c->ncols - 1) * sizeof(double), hipMemcpyHostToDevice));
    const Geo g = geo(c);
    // Chain the fma sum over ranks in global row order: round p, rank p
    // extends the chain; everybody receives it through a sum with zeros.
    double *chain = c->acc;
    for (int p = 0; p < c->world; p++) {
        if (c->rank == p) {
            if (launch_objective_chain(lau(c), g, c->cb, p == 0 ? nullptr : chain, chain))
                return fail(c, LPG_ERR_DEVICE, "objective chain launch failed");
        } else {
            HIPCHK(c, hipMemsetAsync(chain, 0, c->ncols * sizeof(double), c->stream));
        }
        if ((rc = comm_allreduce_sum(c, chain, (size_t)c->ncols))) return rc;
    }
    if (launch_objective_finish(lau(c), g, chain, c->cost, orow))
        return fail(c, LPG_ERR_DEVICE, "objective finish failed");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->booted = false;   // re-price from the new objective row; the pivot count and log carry on
    return 0;
}

int lpg_set_tolerances(lpg_ctx *c, double eps_piv, double eps_opt) {
    if (!c || !(eps_piv >= 0) || !(eps_opt >= 0)) return fail(c, LPG_ERR_ARG, "bad tolerances");
    c->eps_piv = eps_piv;
    c->eps_opt = eps_opt;
    c->booted = false;
    graph_drop(c);
    return 0;
}

int lpg_set_active_columns(lpg_ctx *c, int64_t nact) {
    if (!c || nact < 1 || nact > c->ncols - 1) return fail(c, LPG_ERR_ARG, "bad active column count");
    c->nact = nact;
    c->booted = false;
    graph_drop(c);
    return 0;
}

int lpg_generate(lpg_ctx *c, int64_t n, uint64_t seed, int kind) {
    if (!c || n < 1 || c->ncols != n + c->m + 1 || kind < LPG_GEN_DENSE || kind > LPG_GEN_DUAL)
        return fail(c, LPG_ERR_ARG, "lpg_generate: need ncols == n + m + 1 and a known kind");
    int rc;
    if ((rc = use_device(c))) return rc;
    if (c->colmap && (launch_iota(lau(c), c->colmap, c->ld) || launch_iota(lau(c), c->inv, c->ld)))
        return fail(c, LPG_ERR_DEVICE, "iota launch failed");
    c->permuted = false;
    c->pend = 0;                 // the generator overwrites the whole tableau: nothing pending survives
    if (launch_generate(lau(c), geo(c), n, seed, kind, c->basis)) return fail(c, LPG_ERR_DEVICE, "generate launch failed");
    c->poisoned = false;   // the whole tableau and the basis are rewritten
    c->units_known = true; // the generator writes exact unit columns for the slack / artificial basis
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return reset_state(c);
}

int lpg_enqueue(lpg_ctx *c, int64_t npiv, int rule) {
    if (!c || npiv < 0 || (rule != LPG_RULE_DANTZIG && rule != LPG_RULE_BLAND))
        return fail(c, LPG_ERR_ARG, "lpg_enqueue: bad arguments");
    int rc;
    if ((rc = use_device(c))) return rc;
    if ((rc = usable(c))) return rc;
    if ((rc = ensure_log(c, c->enq + npiv))) return rc;
    return enqueue(c, npiv, rule);
}

int lpg_reserve_log(lpg_ctx *c, int64_t npivots) {
    if (!c || npivots < 0) return fail(c, LPG_ERR_ARG, "lpg_reserve_log: bad arguments");
    int rc;
    if ((rc = use_device(c))) return rc;
    return ensure_log(c, c->enq + npivots);
}

int lpg_prepare(lpg_ctx *c, int rule) {
    if (!c || (rule != LPG_RULE_DANTZIG && rule != LPG_RULE_BLAND)) return fail(c, LPG_ERR_ARG, "lpg_prepare: bad arguments");
    int rc;
    if ((rc = usable(c))) return rc;
    if ((rc = use_device(c)) || (rc = materialize(c))) return rc;
    if (!c->booted || c->boot_rule != rule)
        if ((rc = bootstrap(c, rule))) return rc;
    if ((c->persist && !has_comm(c)) || (c->persist_x && c->xmode)) return 0;   // one launch per block: nothing to capture
    // the conditions under which enqueue replays graphs (enqueue, above)
    const int G = graph_len(c);
    const bool timed = c->timing && c->defer_k == 0;
    const bool comm_ok = !has_comm(c) || (c->nccl && !c->have_hops && c->graph_comm && !c->xmode);
    if (!c->use_graphs || timed || !comm_ok || (G & 1)) return 0;
    if (c->graph[c->par] && c->graph_rule[c->par] == rule) return 0;
    if ((rc = graph_build(c, rule))) {
        if (!has_comm(c)) return rc;
        c->graph_comm = false;                  // as in enqueue: this RCCL build does not capture
        c->err[0] = 0;
    }
    return 0;
}

int lpg_sync(lpg_ctx *c, lpg_result *out) {
    if (!c) return fail(c, LPG_ERR_ARG, "ctx is NULL");
    int rc;
    if ((rc = use_device(c)) || (rc = materialize(c))) return rc;
    lpg_result r;
    if ((rc = read_result(c, &r, c->boot_rule))) return rc;
    // pivots a residency census dropped run now, on the pair (at most once:
    // the persistent form is off after a recovery)
    if (c->lost > 0 && r.status == LPG_ITER_LIMIT) {
        const int64_t n = c->lost;
        c->lost = 0;
        if ((rc = lpg_enqueue(c, n, c->boot_rule)) || (rc = materialize(c)) || (rc = read_result(c, &r, c->boot_rule)))
            return rc;
    }
    c->lost = 0;
    if (out) *out = r;
    return 0;
}

int lpg_solve(lpg_ctx *c, int64_t max_pivots, int rule, lpg_result *out) {
    if (!c || max_pivots < 0 || (rule != LPG_RULE_DANTZIG && rule != LPG_RULE_BLAND))
        return fail(c, LPG_ERR_ARG, "lpg_solve: bad arguments");
    int rc;
    if ((rc = use_device(c))) return rc;
    if ((rc = usable(c))) return rc;
    lpg_result r;
    if (c->booted && c->boot_rule == rule) {
        if ((rc = read_result(c, &r, rule))) return rc;
        if (r.status != LPG_ITER_LIMIT) {
            if (out) *out = r;
            return 0;
        }
    }
    // max_pivots counts pivots the device applies: a launch a residency census
    // stopped (recover_residency) applied none, and its pivots are re-run
    int64_t have = device_pivots(c), batch = 8;
    if (have < 0) return fail(c, LPG_ERR_DEVICE, "reading pivot count failed");
    const int64_t target = max_pivots > INT64_MAX - have ? INT64_MAX : have + max_pivots;
    if (max_pivots == 0) {
        if (!c->booted || c->boot_rule != rule)
            if ((rc = enqueue(c, 0, rule))) return rc;
    }
    while (have < target) {
        const int64_t n = std::min(batch, target - have);
        if ((rc = lpg_enqueue(c, n, rule))) return rc;
        if ((rc = read_result(c, &r, rule))) return rc;
        if (r.status != LPG_ITER_LIMIT) break;
        have = r.pivots;
        batch = std::min<int64_t>(batch * 2, 256);
    }
    c->lost = 0;
    if ((rc = materialize(c))) return rc;
    return read_result(c, out, rule);
}

int lpg_pivot(lpg_ctx *c, int64_t k, int64_t r) {
    if (!c || k < 1 || k >= c->ncols || r < 0 || r >= c->m) return fail(c, LPG_ERR_ARG, "lpg_pivot: bad (k, r)");
    int rc;
    if ((rc = use_device(c))) return rc;
    if ((rc = usable(c))) return rc;
    if ((rc = ensure_log(c, c->enq + 1))) return rc;
    const int rule = c->booted ? c->boot_rule : LPG_RULE_DANTZIG;
    lpg_result before, after;
    if ((rc = read_result(c, &before, rule))) return rc;
    if ((rc = bootstrap_forced(c, rule, k, r))) return rc;
    if ((rc = enqueue(c, 1, rule))) return rc;
    if ((rc = read_result(c, &after, rule))) return rc;
    c->booted = false;   // the next solve prices from scratch
    if (after.pivots != before.pivots + 1)
        return fail(c, LPG_ERR_STATE, "lpg_pivot: |T[%lld][%lld]| <= eps_piv, pivot not applied", (long long)r, (long long)k);
    return 0;
}

// Sums of host values over ranks: count doubles through the device scratch
// `acc` and the attached communicator (no-op on one rank).
static int host_allreduce_sum(lpg_ctx *c, double *v, size_t count) {
    if (!has_comm(c)) return 0;
    if (count > (size_t)c->ncols) return fail(c, LPG_ERR_ARG, "host_allreduce_sum: %zu > ncols", count);
    HIPCHK(c, hipMemcpyAsync(c->acc, v, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    int rc;
    if ((rc = comm_allreduce_sum(c, c->acc, count))) return rc;
    HIPCHK(c, hipMemcpyAsync(v, c->acc, count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

// sum |b_i| over every constraint row in global row order, the same double
// on every rank: rank p continues rank p - 1's running sum (the others add
// +0), so the rounding is the single rank's
static int abs_b_sum(lpg_ctx *c, double *out) {
    std::vector<double> xb(std::max<int64_t>(c->nloc, 1));
    int rc;
    if ((rc = lpg_get_column0(c, xb.data()))) return rc;
    double s = 0.0;
    for (int p = 0; p < c->world; p++) {
        double v = 0.0;
        if (p == c->rank) {
            v = s;
            for (int64_t i = 0; i < c->nloc; i++) v += fabs(xb[i]);
        }
        if (c->world > 1 && (rc = host_allreduce_sum(c, &v, 1))) return rc;
        s = v;
    }
    *out = s;
    return 0;
}

int lpg_solve_two_phase(lpg_ctx *c, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                        lpg_result *out) {
    if (!c || art_first < 2 || art_first >= c->ncols || max_pivots < 0)
        return fail(c, LPG_ERR_ARG, "lpg_solve_two_phase: bad arguments");
    if (c->world > 1 && !has_comm(c)) return fail(c, LPG_ERR_STATE, "lpg_solve_two_phase: no communicator attached");
    int rc;
    if ((rc = use_device(c))) return rc;
    if ((rc = usable(c))) return rc;
    const int64_t N = c->ncols - 1;
    std::vector<double> own;
    if (!cost) {   // costs = -1 x the objective row as loaded (slack-form -c row, replicated)
        own.resize(c->ncols);
        if ((rc = lpg_get_rows(c, c->m, 1, own.data(), c->ncols))) return rc;
        for (int64_t j = 1; j <= N; j++) own[j - 1] = -own[j];
        cost = own.data();
    }
    // Phase I: max -sum(artificials) over all columns.
    std::vector<double> c1(N, 0.0);
    for (int64_t j = art_first; j <= N; j++) c1[j - 1] = -1.0;
    if ((rc = lpg_set_active_columns(c, N)) || (rc = lpg_set_objective(c, c1.data()))) return rc;
    lpg_result r1;
    if ((rc = lpg_solve(c, max_pivots, rule, &r1))) return rc;
    int64_t used = r1.pivots;
    if (r1.status == LPG_ITER_LIMIT || r1.status == LPG_NUMERIC || r1.status == LPG_UNBOUNDED) {
        if (out) { *out = r1; if (r1.status == LPG_UNBOUNDED) out->status = LPG_NUMERIC; }
        return 0;
    }
    // infeasible when the artificials cannot all reach zero
    double bsum = 0;
    if ((rc = abs_b_sum(c, &bsum))) return rc;
    if (r1.objective < -1e-9 * std::max(1.0, bsum)) {
        if (out) { *out = r1; out->status = LPG_INFEASIBLE; }
        return 0;
    }
    // Drive artificials still basic (at zero) out of the basis with forced
    // degenerate pivots on the first usable original column of their row; a
    // row with no such column is redundant and keeps its artificial at zero.
    // Row i lives on one rank: its owner finds the column and every rank
    // learns it through a sum (the others add 0), then every rank pivots.
    std::vector<int64_t> basis(c->m);
    if ((rc = lpg_get_basis(c, basis.data()))) return rc;
    std::vector<double> row(c->ncols);
    for (int64_t i = 0; i < c->m; i++) {
        if (basis[i] < art_first) continue;
        double jv = 0.0;
        if (i >= c->row0 && i < c->row0 + c->nloc) {
            if ((rc = lpg_get_rows(c, i, 1, row.data(), c->ncols))) return rc;
            for (int64_t j = 1; j < art_first; j++)
                if (fabs(row[j]) > c->eps_piv) {
                    jv = (double)j;
                    break;
                }
        }
        if (c->world > 1 && (rc = host_allreduce_sum(c, &jv, 1))) return rc;
        if (jv > 0.0) {
            if ((rc = lpg_pivot(c, (int64_t)jv, i))) return rc;
            used++;
        }
    }
    // Phase II: original costs, artificial columns barred from entering.
    if ((rc = lpg_set_active_columns(c, art_first - 1)) || (rc = lpg_set_objective(c, cost))) return rc;
    lpg_result r2;
    if ((rc = lpg_solve(c, std::max<int64_t>(max_pivots - used, 0), rule, &r2))) return rc;
    if (out) *out = r2;
    return 0;
}

int lpg_solve_big_m(lpg_ctx *c, int64_t art_first, const double *cost, int64_t max_pivots, int rule,
                    lpg_result *out) {
    if (!c || art_first < 2 || art_first >= c->ncols || max_pivots < 0)
        return fail(c, LPG_ERR_ARG, "lpg_solve_big_m: bad arguments");
    if (c->nobj != 2) return fail(c, LPG_ERR_STATE, "lpg_solve_big_m needs a context created with LPG_FLAG_BIG_M");
    int rc;
    if ((rc = usable(c))) return rc;
    if ((rc = use_device(c))) return rc;
    const int64_t N = c->ncols - 1;
    std::vector<double> cr(N), cm(N, 0.0), row(c->ncols);
    if (cost) {
        for (int64_t j = 0; j < N; j++) cr[j] = cost[j];
    } else {   // costs = -1 x the (real) objective row as loaded (slack-form -c row)
        if ((rc = lpg_get_rows(c, c->m + c->nobj - 1, 1, row.data(), c->ncols))) return rc;
        for (int64_t j = 1; j <= N; j++) cr[j - 1] = -row[j];
    }
    for (int64_t j = art_first; j <= N; j++) {   // artificial: cost -M (max form) = M part -1, real part 0
        cr[j - 1] = 0.0;
        cm[j - 1] = -1.0;
    }
    if ((rc = lpg_set_active_columns(c, N)) || (rc = lpg_set_objective_m(c, cm.data())) ||
        (rc = lpg_set_objective(c, cr.data())))
        return rc;
    lpg_result r;
    if ((rc = lpg_solve(c, max_pivots, rule, &r))) return rc;
    if (r.status == LPG_OPTIMAL || r.status == LPG_UNBOUNDED) {
        // artificials still positive (M-part objective < 0) -> infeasible; also
        // at UNBOUNDED: the pricing takes a negative M part first and such a
        // column is never a ray (every basic artificial would grow along it),
        // so a ray found while the M objective is negative cannot reach
        // feasibility (as oracle/lpo.c lpo_solve_big_m)
        double zM = 0, bsum = 0;
        std::vector<double> xb(c->nloc);
        if ((rc = lpg_get_rows(c, c->m, 1, row.data(), c->ncols)) || (rc = lpg_get_column0(c, xb.data()))) return rc;
        zM = row[0];
        for (double v : xb) bsum += fabs(v);
        if (zM < -1e-9 * std::max(1.0, bsum)) r.status = LPG_INFEASIBLE;
    }
    if (out) *out = r;
    return 0;
}

// The dual on the deferred tableau (lpg_dual.hip): two kernels per pivot,
// the block's flush (no column trade: the ratio test's keys are the caller's
// column order) every defer_k pivots, and a final k_dual_row_d for the
// objective row's owed update and the optimality peek (as oracle/lpo.c).
static int solve_dual_deferred(lpg_ctx *c, int64_t max_pivots, lpg_result *out) {
    const Geo g = geo(c);
    const Launch L = lau(c);
    const bool mr = has_comm(c);
    // row-candidate blocks: the same count on every rank (the largest row block)
    int64_t maxloc = 0;
    for (int p = 0; p < c->world; p++) maxloc = std::max(maxloc, c->m * (p + 1) / c->world - c->m * p / c->world);
    const int nrc = (int)((maxloc + c->nobj + 255) / 256), ncp = pivot_d_blocks(g, 0, 256);
    if (!c->drc) HIPCHK(c, hipMalloc(&c->drc, (size_t)nrc * sizeof(Cand)));
    if (!c->dcp) HIPCHK(c, hipMalloc(&c->dcp, (size_t)ncp * sizeof(Cand)));
    if (mr && !c->drc_all) HIPCHK(c, hipMalloc(&c->drc_all, (size_t)nrc * c->world * sizeof(Cand)));
    HIPCHK(c, hipMemsetAsync(c->st->slot, 0, sizeof(c->st->slot), c->stream));
    if (launch_dual_rows(L, g, c->drc, nrc)) return fail(c, LPG_ERR_DEVICE, "dual rows launch failed");
    c->par = 0;
    c->booted = false;
    // the column trade stays off for the dual's whole run and comes back on
    // every exit, the HIPCHK early returns included
    struct ReorderGuard {
        lpg_ctx *c;
        bool keep;
        ~ReorderGuard() { c->no_reorder = keep; }
    } guard{c, c->no_reorder};
    c->no_reorder = true;
    int rc = 0;
    // one pivot: (MR: every rank's row candidates) row_d, (MR: R summed over
    // the ranks, the ratio partials) col_d; row_only: row_d alone
    auto pivot = [&](bool row_only) -> int {
        const int s = c->par;
        const Defer D = defer_of(c, c->pend);
        const double *Pprev = c->Pbuf + (int64_t)((c->pend + c->defer_k - 1) % c->defer_k) * c->ld;
        int r2;
        if (mr && (r2 = comm_allgather(c, c->drc, c->drc_all, (size_t)nrc * sizeof(Cand)))) return r2;
        if (launch_dual_row_d(L, g, c->st, s, mr ? c->drc_all : c->drc, mr ? nrc * c->world : nrc, c->dcp, c->P,
                              Pprev, c->C[s ^ 1], D, mr))
            return fail(c, LPG_ERR_DEVICE, "dual row launch failed");
        if (row_only) return 0;
        if (mr) {
            if ((r2 = comm_allreduce_sum(c, c->P, (size_t)prow_count(c)))) return r2;
            if (launch_dual_ratio(L, g, c->st, s, c->P, c->dcp)) return fail(c, LPG_ERR_DEVICE, "dual ratio launch failed");
        }
        if (launch_dual_col_d(L, g, c->st, s, c->dcp, c->P, c->C[s], c->drc, nrc, D))
            return fail(c, LPG_ERR_DEVICE, "dual column launch failed");
        return 0;
    };
    int64_t done = 0, batch = 8;
    while (done < max_pivots) {
        const int64_t n = std::min(batch, max_pivots - done);
        if ((rc = ensure_log(c, c->enq + n))) break;
        for (int64_t q = 0; q < n && !rc; q++) {
            if (!(rc = pivot(false)) && ++c->pend == c->defer_k) rc = flush_launch(c);
            c->par ^= 1;
            c->enq++;
        }
        if (rc) break;
        done += n;
        DevState h;
        HIPCHK(c, hipMemcpyAsync(&h, c->st, sizeof h, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (h.stall == kStallPending) return pending_fault(c, h);
        if (h.slot[c->par].status != LPG_RUNNING) break;
        batch = std::min<int64_t>(batch * 2, 256);
    }
    if (!rc) rc = pivot(true);
    if (!rc && hipMemsetAsync(&c->st->slot[c->par].dpend, 0, sizeof(int64_t), c->stream) != hipSuccess)
        rc = fail(c, LPG_ERR_DEVICE, "hipMemsetAsync failed");
    if (!rc) rc = materialize(c);
    if (rc) return rc;
    DevState h;
    double z = 0;
    HIPCHK(c, hipMemcpyAsync(&h, c->st, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&z, c->T + (c->nloc + c->nobj - 1) * c->ld, sizeof z, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (h.stall == kStallPending) return pending_fault(c, h);
    const int32_t st = h.slot[c->par].status;
    lpg_result r;
    // the final row-only k_dual_row_d publishes its optimality peek as r = -1
    // on a RUNNING slot (it never writes the status its own blocks read)
    r.status = st != LPG_RUNNING ? st : h.slot[c->par].r < 0 ? LPG_OPTIMAL : LPG_ITER_LIMIT;
    r.rule = LPG_RULE_DANTZIG;
    r.pivots = h.pivots;
    r.objective = z;
    r.entering = h.pivots ? h.last_k : -1;
    r.leaving = h.pivots ? h.last_r : -1;
    if (out) *out = r;
    return 0;
}

int lpg_solve_dual(lpg_ctx *c, int64_t max_pivots, lpg_result *out) {
    if (!c || max_pivots < 0) return fail(c, LPG_ERR_ARG, "lpg_solve_dual: bad arguments");
    if (c->world > 1 && !has_comm(c)) return fail(c, LPG_ERR_STATE, "lpg_solve_dual: no communicator attached");
    if (has_comm(c) && !(c->defer_k > 0 && c->nobj == 1))
        return fail(c, LPG_ERR_STATE, "lpg_solve_dual: a row partition runs the deferred form only (not LPG_FLAG_EAGER)");
    int rc;
    if ((rc = usable(c))) return rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    // the dual simplex starts from a dual-feasible basis: every d_j >= -eps
    std::vector<double> obj(c->ncols);
    if ((rc = lpg_get_rows(c, c->m + c->nobj - 1, 1, obj.data(), c->ncols))) return rc;
    for (int64_t j = 1; j <= c->nact; j++)
        if (obj[j] < -c->eps_opt)
            return fail(c, LPG_ERR_STATE, "lpg_solve_dual: basis not dual feasible (d_%lld = %g)", (long long)j, obj[j]);
    if (c->defer_k > 0 && c->nobj == 1) return solve_dual_deferred(c, max_pivots, out);
    const Geo g = geo(c);
    const Launch L = lau(c);
    HIPCHK(c, hipMemsetAsync(c->st->slot, 0, sizeof(c->st->slot), c->stream));
    if (launch_dual_rows(L, g, c->part, c->nsel)) return fail(c, LPG_ERR_DEVICE, "dual rows launch failed");
    c->par = 0;
    c->booted = false;   // the primal loop must re-price after a dual solve
    int64_t done = 0, batch = 8;
    lpg_result r;
    while (done < max_pivots) {
        const int64_t n = std::min(batch, max_pivots - done);
        if ((rc = ensure_log(c, c->enq + n))) return rc;   // grown per batch (doubling), not to max_pivots up front
        for (int64_t q = 0; q < n; q++) {
            const int s = c->par;
            if (launch_dual_pivot(L, g, c->st, s, c->part, c->nsel, c->pp, c->pc, c->npp, c->skip, c->P, c->C[s]))
                return fail(c, LPG_ERR_DEVICE, "dual pivot launch failed");
            if (launch_update(L, g, c->st, s, c->P, c->C[s], c->basis, c->logk, c->logr, c->update_variant, c->skip))
                return fail(c, LPG_ERR_DEVICE, "update launch failed");
            c->par = s ^ 1;
            c->enq++;
        }
        done += n;
        DevState h;
        HIPCHK(c, hipMemcpyAsync(&h, c->st, sizeof h, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (h.stall == kStallPending) return pending_fault(c, h);
        if (h.slot[c->par].status != LPG_RUNNING) break;
        batch = std::min<int64_t>(batch * 2, 256);
    }
    // the budget ran out: k_dual_price alone says whether the last pivot was optimal
    if (launch_dual_pivot(L, g, c->st, c->par, c->part, c->nsel, c->pp, c->pc, c->npp, c->skip, c->P, c->C[c->par], true))
        return fail(c, LPG_ERR_DEVICE, "dual price launch failed");
    DevState h;
    double z = 0;
    HIPCHK(c, hipMemcpyAsync(&h, c->st, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&z, c->T + (c->nloc + c->nobj - 1) * c->ld, sizeof z, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int32_t st = h.slot[c->par].status;
    r.status = st == LPG_RUNNING ? LPG_ITER_LIMIT : st;
    r.rule = LPG_RULE_DANTZIG;
    r.pivots = h.pivots;
    r.objective = z;
    r.entering = h.pivots ? h.last_k : -1;
    r.leaving = h.pivots ? h.last_r : -1;
    if (out) *out = r;
    return 0;
}

int lpg_get_rows(lpg_ctx *c, int64_t row0, int64_t nrows, double *out, int64_t ld) {
    if (!c || !out || row0 < 0 || nrows < 0 || row0 + nrows > c->m + c->nobj || ld < c->ncols)
        return fail(c, LPG_ERR_ARG, "lpg_get_rows: bad arguments");
    int rc;
    if ((rc = use_device(c)) || (rc = canonicalize(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t a = std::max(row0, c->row0), b = std::min(row0 + nrows, c->row0 + c->nloc);
    if (a < b)
        HIPCHK(c, hipMemcpy2D(out + (a - row0) * ld, ld * sizeof(double), c->T + (a - c->row0) * c->ld,
                              c->ld * sizeof(double), c->ncols * sizeof(double), b - a, hipMemcpyDeviceToHost));
    for (int64_t q = 0; q < c->nobj; q++) {
        const int64_t gi = c->m + q;
        if (gi >= row0 && gi < row0 + nrows)
            HIPCHK(c, hipMemcpy(out + (gi - row0) * ld, c->T + (c->nloc + q) * c->ld, c->ncols * sizeof(double),
                                hipMemcpyDeviceToHost));
    }
    return 0;
}

int lpg_get_basis(lpg_ctx *c, int64_t *basis) {
    if (!c || !basis) return fail(c, LPG_ERR_ARG, "basis is NULL");
    int rc;
    if ((rc = use_device(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(basis, c->basis, c->m * sizeof(int64_t), hipMemcpyDeviceToHost));
    return 0;
}

int lpg_get_column0(lpg_ctx *c, double *xB) {
    if (!c || !xB) return fail(c, LPG_ERR_ARG, "xB is NULL");
    int rc;
    if ((rc = use_device(c)) || (rc = materialize(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->nloc)
        HIPCHK(c, hipMemcpy2D(xB, sizeof(double), c->T, c->ld * sizeof(double), sizeof(double), c->nloc,
                              hipMemcpyDeviceToHost));
    return 0;
}

int64_t lpg_get_log(lpg_ctx *c, int64_t *k, int64_t *r, int64_t max) {
    if (!c || max < 0) return fail(c, LPG_ERR_ARG, "lpg_get_log: bad arguments");
    if (use_device(c)) return LPG_ERR_DEVICE;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(c, LPG_ERR_DEVICE, "sync failed");
    const int64_t n = device_pivots(c);
    if (n < 0) return fail(c, LPG_ERR_DEVICE, "reading pivot count failed");
    if (c->flags & LPG_FLAG_NO_LOG) return n;
    const int64_t cnt = std::min(std::min(n, max), c->logcap);
    if (cnt > 0) {
        if (k && hipMemcpy(k, c->logk, cnt * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(c, LPG_ERR_DEVICE, "log copy failed");
        if (r && hipMemcpy(r, c->logr, cnt * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(c, LPG_ERR_DEVICE, "log copy failed");
    }
    return n;
}

int lpg_set_timing(lpg_ctx *c, int enable) {
    if (!c) return fail(c, LPG_ERR_ARG, "ctx is NULL");
    int rc;
    if ((rc = use_device(c))) return rc;
    if (enable && c->tr.ev.empty()) {
        c->tr.ev.resize(3 * 1024);
        c->tr.upd.assign(1024, 0);
        for (auto &e : c->tr.ev) HIPCHK(c, hipEventCreate(&e));
    }
    c->timing = enable != 0;
    return 0;
}

int lpg_get_timing(lpg_ctx *c, lpg_timing *out) {
    if (!c || !out) return fail(c, LPG_ERR_ARG, "NULL argument");
    int rc;
    if ((rc = use_device(c))) return rc;
    if ((rc = timing_flush(c))) return rc;
    unsigned long long touched = 0;
    HIPCHK(c, hipMemcpy(&touched, &c->st->touched, sizeof touched, hipMemcpyDeviceToHost));
    out->update_bytes = 16.0 * (double)(touched - c->touched_mark);
    c->touched_mark = touched;
    out->update_ms = c->tr.update_ms;
    out->select_ms = c->tr.select_ms;
    out->comm_ms = c->tr.comm_ms;
    out->update_count = c->tr.count;
    c->tr.update_ms = c->tr.select_ms = c->tr.comm_ms = 0;
    c->tr.count = 0;
    return 0;
}

int lpg_device_sync(lpg_ctx *c) {
    if (!c) return fail(c, LPG_ERR_ARG, "ctx is NULL");
    int rc;
    if ((rc = use_device(c)) || (rc = materialize(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

#ifdef LPG_PHASES
// tools/phase_probe.py only (not part of include/lpg.h; absent from liblpg.so)
int lpg_debug_phases(unsigned long long *out, int reset) { return lpg::debug_phases(out, reset); }
int lpg_debug_block_phases(unsigned long long *out) { return lpg::debug_block_phases(out); }
#endif

}  // extern "C"
