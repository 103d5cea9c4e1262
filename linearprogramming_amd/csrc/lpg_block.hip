// lpg_block.hip — the deferred pivot loop as ONE persistent launch per run of
// pivots: k_pivot_block (single rank; and, with MR, every rank of a row
// partition over the owner-push exchange -- see the note above the kernel).
//
// What it replaces. Without it every pivot t is two kernels (k_prep_d, then
// k_select_d, lpg_kernels.hip), and the kernel boundary between them is the
// grid-wide step where the block partials meet. Each of those kernels then
// reloads, from the Infinity Cache, the pending-pivot data its chain needs:
// up to 64 P rows (25 MB at config 3) for the pivot row and 64 C columns
// (8.4 MB) for the entering column -- at 64 pending pivots that reload, not
// the arithmetic, is most of the 10-11 us each kernel takes.
//
// Here workgroup w (one per CU) owns a fixed slice of the tableau for the
// whole launch: physical columns [w cw, (w+1) cw) and constraint rows
// [w rw, (w+1) rw). The slices of the pending P rows and C columns it
// produces stay in its LDS (sP: KS x cw, sC: KS x rw doubles; 131 KB at
// config 3), so a chain reads LDS, and only the pivot row's base entries,
// the entering column's base entries and 64 multipliers per step come from
// memory. The reference loop this restates is absent upstream
// (Source/simplex.c:40 -> :65).
//
// Per pivot t (pending index q), two phases, each ending in an all-to-all of
// one record per workgroup ("granules": 16-byte write-through stores whose
// last word is the pivot's tag, swept by one wave per workgroup until every
// tag matches -- the data is its own flag, MI355X_MICROARCH.md
// "allgather" / cdna_hip_programming.md Guideline 16 R2):
//   P (prep):   ratio records -> leaving row r, pivot element; row r of the
//               current tableau on this slice's columns = the pending chain
//               over sP; P_q = row / piv -> sP[q] and Pbuf[q]; the objective
//               row(s) d = fma(-C_t[obj], P_q, d) (kept in registers for the
//               launch); the slice's pricing argmin -> pricing record
//   S (select): pricing records -> entering column k; column k of the
//               current tableau on this slice's rows = the chain over sC;
//               column 0 (b) kept current in registers; C_{t+1} -> sC[q+1]
//               and Cbuf[q+1]; the slice's min-ratio -> ratio record.
// The arithmetic and every tie-break are k_prep_d / k_select_d's, so the
// pivot log, the basis and every tableau value are bitwise the same
// (tests/test_gpu_block.py).
//
// Inter-workgroup data: records, P_q entries (read by every slice as the
// entering column's P_u[k] and P_q[0]) and C_q entries (read as the pivot
// row's multipliers C_u[r]) are written with sc1 (write-through) stores and
// read with sc1 loads, after the reading wave saw the record tags that were
// published behind the writing waves' s_waitcnt vmcnt(0) and a workgroup
// barrier (MI355X_MICROARCH.md, "Valid forms", first table row). Everything
// else a workgroup reads was written before the launch. Spins are bounded
// (~2 s): a workgroup that gives up writes NUMERIC and the flag word
// DevState::stall, and the launch drains.
//
// Residency: one workgroup per CU (the LDS slices force it), as many
// workgroups as CUs; the launch needs the whole GPU to itself (multi-rank:
// each rank its own GPU, or launches small enough to be resident together).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "lpg_device.h"
#include "lpg_internal.h"

namespace lpg {

typedef unsigned u4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kNT = 256;            // threads per workgroup
constexpr int kMaxWG = 256;         // records swept per phase: 4 per lane of one wave
constexpr int kPer = kMaxWG / 64;
constexpr int kRecPMax = 5;         // pricing record granules (k_pivot_block's NGP), space reserved per workgroup
constexpr int kRecR = 2;            // ratio record:   {theta, key, tag} {piv, row, tag}
constexpr int kMaxLds = 150 * 1024;  // dynamic LDS cap (the slices)
constexpr long long kSpinTicks = 200000000ll;   // s_memrealtime runs at 100 MHz: 2 s
constexpr int kSweepSleep = 1;      // s_sleep between record polls (64 clocks each)

// doubles per thread row of the LDS slices: the unrolled chains read 16, 32,
// 48 or 64 slots, so >= ks rounded up to 16; = 2 mod 4 (16-byte reads at this
// stride from 16 lanes cover the 64 banks once)
__host__ __device__ constexpr int slot_stride(int ks) { return ((ks + 15) & ~15) + 2; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, bytes, 0x00020000);
}
// ONE 16-byte write-through store / load (aux 16 = sc1)
constexpr int kRecAux = 16;
__device__ __forceinline__ void rec_store(__amdgpu_buffer_rsrc_t r, int off, u4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kRecAux);
}
__device__ __forceinline__ u4 rec_load(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kRecAux);
}
// 8-byte write-through store / load of a double (global_store/load_dwordx2 sc1)
__device__ __forceinline__ void st_wt(double *p, double v) {
    __hip_atomic_store((unsigned long long *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double *p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((unsigned long long *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ u4 pack(uint64_t a, uint32_t b, uint32_t tag) {
    return u4{(uint32_t)a, (uint32_t)(a >> 32), b, tag};
}
__device__ __forceinline__ uint64_t lo64(const u4 &v) { return ((uint64_t)v.y << 32) | v.x; }

// One wave sweeps the NG-granule records of nwg workgroups until every tag
// equals `tag`; lane l holds records l, l + 64, l + 128, l + 192. XG: lane 0
// also holds the one extra granule xidx (workgroup 0's P_q[0]) in xg.
// False on timeout (the caller stops the launch).
template <int NG, bool XG = false>
__device__ bool sweep(__amdgpu_buffer_rsrc_t r, int nwg, uint32_t tag, u4 (&rec)[kPer][NG], int phase,
                      DevState *st, u4 *xg = nullptr, int xidx = 0) {
    const int lane = threadIdx.x & 63;
    const long long t0 = (long long)wall_clock64();
    for (;;) {
        bool ok = true;
        int bad = -1;
        uint32_t seen = 0;
#pragma unroll
        for (int p = 0; p < kPer; p++) {
            const int w = lane + 64 * p;
            if (w < nwg) {
#pragma unroll
                for (int k = 0; k < NG; k++) rec[p][k] = rec_load(r, (w * NG + k) * 16);
            }
        }
        if (XG && lane == 0) {
            *xg = rec_load(r, xidx * 16);
            if (xg->w != tag) {
                ok = false;
                bad = xidx;
                seen = xg->w;
            }
        }
#pragma unroll
        for (int p = 0; p < kPer; p++) {
            const int w = lane + 64 * p;
            if (w < nwg) {
#pragma unroll
                for (int k = 0; k < NG; k++)
                    if (rec[p][k].w != tag) {
                        ok = false;
                        if (bad < 0) {
                            bad = w * NG + k;
                            seen = rec[p][k].w;
                        }
                    }
            }
        }
        if (__all(ok)) return true;
        if ((long long)wall_clock64() - t0 > kSpinTicks) {
            const int wl = winner_lane(!ok);
            const int bi = (int)rdl32((uint32_t)bad, wl);
            const uint32_t sv = rdl32(seen, wl);
            if (lane == 0) {
                st->stall_info[0] = phase;
                st->stall_info[1] = tag;
                st->stall_info[2] = bi;
                st->stall_info[3] = sv;
            }
            return false;
        }
        __builtin_amdgcn_s_sleep(kSweepSleep);
    }
}

// lexicographic min over this lane's records, then over the wave; src = the
// winner's workgroup (uniform), -1 if every key is (~0, ~0); pay[k] = its
// granule k + 1 (uniform)
template <int NG>
__device__ __forceinline__ void rec_min(const u4 (&rec)[kPer][NG], int nwg, uint64_t &h, uint32_t &l, int &src,
                                        u4 (&pay)[NG > 1 ? NG - 1 : 1]) {
    const int lane = threadIdx.x & 63;
    h = ~0ull;
    l = ~0u;
    int mine = -1;
    u4 mp[NG > 1 ? NG - 1 : 1];
#pragma unroll
    for (int k = 0; k + 1 < NG; k++) mp[k] = u4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int p = 0; p < kPer; p++) {
        const int w = lane + 64 * p;
        if (w < nwg) {
            const uint64_t a = lo64(rec[p][0]);
            const uint32_t b = rec[p][0].z;
            if (key_less(a, b, h, l)) {
                h = a;
                l = b;
                mine = w;
#pragma unroll
                for (int k = 0; k + 1 < NG; k++) mp[k] = rec[p][k + 1];
            }
        }
    }
    const uint64_t mh = h;
    const uint32_t ml = l;
    wave_min_key(h, l);
    const int wl = winner_lane(mine >= 0 && mh == h && ml == l);
    src = (wl < 0 || (h == ~0ull && l == ~0u)) ? -1 : (int)rdl32((uint32_t)mine, wl);
#pragma unroll
    for (int k = 0; k + 1 < NG; k++)
        pay[k] = wl < 0 ? u4{0u, 0u, 0u, 0u}
                        : u4{rdl32(mp[k].x, wl), rdl32(mp[k].y, wl), rdl32(mp[k].z, wl), rdl32(mp[k].w, wl)};
}

struct Bcast {            // one phase's decision, from wave 0 to the workgroup
    uint64_t h;
    uint32_t l;
    int32_t ok;           // 1: decided, 0: none (OPTIMAL / UNBOUNDED), -1: timeout, -2: exchange timeout
    uint64_t p0, p1, p2, p3;   // winner payload
    uint64_t z;           // P_q[0]
    uint64_t pv;          // phase P, RPIV: the pivot element, fetched after the sweep
    int32_t okv;          //   1: fetched, -1: timeout
};

// Multi-rank (owner-push exchange, Xch, lpg_internal.h). Workgroup 0 of every
// rank stores its rank's best ratio candidate {theta bits, key, piv bits,
// row} as 6 self-validating 8-byte words {payload, tag} into slot 0 of its
// rank in every rank's xC (system-scope stores; lane 0 only) ...
__device__ __forceinline__ void xpush_best(const Xch &X, uint32_t tag, uint64_t h, uint32_t l, uint64_t p0,
                                           uint64_t p1) {
    const uint32_t w[6] = {(uint32_t)h, (uint32_t)(h >> 32), (uint32_t)p0, (uint32_t)(p0 >> 32), l, (uint32_t)p1};
    for (int rk = 0; rk < X.world; rk++) {
        uint64_t *d = xch_cand(X, rk, tag & 1, X.rank, 0);
#pragma unroll
        for (int k = 0; k < 6; k++) st_sys64(d + k, ((uint64_t)tag << 32) | w[k]);
    }
}
// ... and wave 0 of every workgroup polls its own xC (lane l: rank l) until
// every rank's words carry the tag, then takes the lexicographic min. False
// on timeout.
__device__ bool xpoll_best(const Xch &X, uint32_t tag, uint64_t &h, uint32_t &l, uint64_t &p0, uint64_t &p1,
                           DevState *st) {
    const int lane = threadIdx.x & 63;
    const long long t0 = (long long)wall_clock64();
    uint64_t v[6] = {0, 0, 0, 0, 0, 0};
    for (;;) {
        bool ok = true;
        if (lane < X.world) {
            const uint64_t *w = xch_cand(X, X.rank, tag & 1, lane, 0);
#pragma unroll
            for (int k = 0; k < 6; k++) v[k] = ld_sys64(w + k);
#pragma unroll
            for (int k = 0; k < 6; k++) ok = ok && (uint32_t)(v[k] >> 32) == tag;
        }
        if (__all(ok)) break;
        if ((long long)wall_clock64() - t0 > kSpinTicks) {
            if (lane == 0) {
                st->stall_info[0] = 4;
                st->stall_info[1] = tag;
            }
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t lo = 0xffffffffull;
    uint64_t mh = ~0ull, m0 = 0, m1 = 0;
    uint32_t ml = ~0u;
    if (lane < X.world) {
        mh = (v[0] & lo) | ((v[1] & lo) << 32);
        m0 = (v[2] & lo) | ((v[3] & lo) << 32);
        ml = (uint32_t)v[4];
        m1 = v[5] & lo;
    }
    h = mh;
    l = ml;
    wave_min_key(h, l);
    const int wl = winner_lane(lane < X.world && mh == h && ml == l);
    p0 = wl < 0 ? 0 : rdl64(m0, wl);
    p1 = wl < 0 ? 0 : rdl64(m1, wl);
    return true;
}

// ---- residency census (the persistent launch needs every workgroup resident
// at once; nothing guarantees it when another kernel or process holds CUs) --
constexpr long long kResTicks = 100000ll;       // 1 ms for one rank's grid (normally resident within ~1 us)
constexpr long long kResTicksMR = 2000000ll;    // 20 ms for every rank's (ranks drift apart by up to a block pass)
constexpr uint64_t kGo = 1, kAbort = 2;

// The first decision for launch `cl` wins: a word from an earlier launch is
// replaced by (cl << 2) | d with a compare-and-swap; returns the decided word.
template <typename W, int SCOPE>
__device__ W decide(W *w, W cl, W d) {
    W v = __hip_atomic_load(w, __ATOMIC_RELAXED, SCOPE);
    while ((v >> 2) != cl)
        if (__hip_atomic_compare_exchange_strong(w, &v, (cl << 2) | d, __ATOMIC_RELAXED, __ATOMIC_RELAXED, SCOPE))
            return (cl << 2) | d;
    return v;
}

// Thread 0 of every workgroup: count in, then wait for the decision. One
// rank: the last of nwg arrivals decides GO (DevState::rcnt counts from
// (cl - 1) * nwg: every earlier launch's workgroups all arrived, aborted or
// not, before this one started); a workgroup that waits kResTicks decides
// ABORT. Several ranks (X): each rank's last local arrival adds the rank to
// rank 0's global count (tagged with this launch's exchange tag, the same on
// every rank), the arrival that completes it decides GO in rank 0's global
// decision word, and any workgroup of any rank that waits kResTicksMR
// decides ABORT there: one word, so every rank takes the same decision.
template <bool MR>
__device__ bool census(DevState *st, int nwg, uint32_t cl, const Xch &X, uint32_t xtag) {
    const uint32_t n =
        __hip_atomic_fetch_add(&st->rcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (cl - 1u) * (uint32_t)nwg + 1u;
    uint64_t *gc = MR ? (uint64_t *)(X.base[0] + X.offG) : nullptr;   // {count tagged (xtag << 8)} ...
    uint64_t *gd = MR ? gc + 8 : nullptr;                             // ... and the decision, a line apart
    if (n == (uint32_t)nwg) {
        if (!MR) {
            decide<uint32_t, __HIP_MEMORY_SCOPE_AGENT>(&st->rdec, cl, (uint32_t)kGo);
        } else {
            uint64_t v = __hip_atomic_load(gc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), nv;
            for (;;) {
                nv = (v >> 8) == (uint64_t)xtag ? v + 1 : (((uint64_t)xtag << 8) | 1u);
                if (__hip_atomic_compare_exchange_strong(gc, &v, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_SYSTEM))
                    break;
            }
            if ((int)(nv & 0xff) == X.world) decide<uint64_t, __HIP_MEMORY_SCOPE_SYSTEM>(gd, xtag, kGo);
        }
    }
    const long long t0 = (long long)wall_clock64();
    for (;;) {
        uint64_t v;
        if (MR) v = __hip_atomic_load(gd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else v = __hip_atomic_load(&st->rdec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 2) == (MR ? (uint64_t)xtag : (uint64_t)cl)) return (v & 3) == kGo;
        if ((long long)wall_clock64() - t0 > (MR ? kResTicksMR : kResTicks)) {
            v = MR ? decide<uint64_t, __HIP_MEMORY_SCOPE_SYSTEM>(gd, xtag, kAbort)
                   : decide<uint32_t, __HIP_MEMORY_SCOPE_AGENT>(&st->rdec, cl, (uint32_t)kAbort);
            return (v & 3) == kGo;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

}  // namespace

#ifdef LPG_PHASES
// Phase probe (tools/block_probe.py; tools/liblpg_phases.so only): s_memrealtime
// stamps of thread 0 of workgroups 0 and nwg / 2 at the phase boundaries of
// every pivot of the launch (LPG_PHASES_PUBONLY: none of those, only every
// workgroup's publish and decision-seen stamps, which cost each workgroup alike).
__device__ unsigned long long g_bph[2][64][16];
#ifdef LPG_PHASES_NOWAIT   // issue-time stamps: no wait for outstanding vector memory ops
#define LPG_BPH_WAIT() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#else                      // completion stamps: everything issued so far has landed
#define LPG_BPH_WAIT() asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory")
#endif
__device__ unsigned long long g_bclk[64];   // shader clock (clock64) beside workgroup 0's stamp 0
#ifdef LPG_PHASES_PUBONLY
#define LPG_BPH(t, k) do { } while (0)
#else
#define LPG_BPH(t, k)                                                                          \
    do {                                                                                       \
        LPG_BPH_WAIT();                                                                        \
        if (tid == 0 && (wg == 0 || wg == nwg / 2) && (t) < 64) {                              \
            g_bph[wg == 0 ? 0 : 1][(t)][(k)] = __builtin_amdgcn_s_memrealtime();               \
            if ((k) == 0 && wg == 0) g_bclk[(t)] = clock64();                                  \
        }                                                                                      \
    } while (0)
#endif
__device__ unsigned long long g_bpub[2][64][256];   // every workgroup's publish stamp, phase P / S
__device__ unsigned long long g_bseen[2][64][256];  // ... and when its wave 0 had swept the decision
#define LPG_BPUB(ph, t)                                                                        \
    do {                                                                                       \
        if (tid == 0 && (t) < 64 && wg < 256) g_bpub[ph][(t)][wg] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define LPG_BSEEN(ph, t)                                                                       \
    do {                                                                                       \
        if (tid == 0 && (t) < 64 && wg < 256) g_bseen[ph][(t)][wg] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
int debug_block_phases(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bph), sizeof g_bph) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + sizeof g_bph / 8, HIP_SYMBOL(g_bpub), sizeof g_bpub) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + (sizeof g_bph + sizeof g_bpub) / 8, HIP_SYMBOL(g_bclk), sizeof g_bclk) != hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(out + (sizeof g_bph + sizeof g_bpub + sizeof g_bclk) / 8, HIP_SYMBOL(g_bseen),
                               sizeof g_bseen) == hipSuccess
               ? 0
               : -1;
}
#else
#define LPG_BPH(t, k) do { } while (0)
#define LPG_BPUB(ph, t) do { } while (0)
#define LPG_BSEEN(ph, t) do { } while (0)
#endif

// The pending chains of one thread over nb batches of 16 slots, software-
// pipelined: batch b+1's LDS reads are in flight while batch b's 16 dependent
// fmas run (one wave per SIMD cannot hide an LDS round trip per step; loading
// all 64 slots before the first fma, round 3's form, held 256 VGPRs of
// operands and spilled into AGPRs). Slots past the chain read as exact no-ops:
// past q the slices hold +0 and the multiplier / P_u[k] rows hold -0 / +0, so
// a step fma(-0, +0, x) is exactly x (and nb = 0 leaves x as it is).
// Pivot row, column j (ROW): x = fma(m_u, P_u[j], x) for u < q; with SEL the
// steps u <= lim (the row's restart point, uniform) are (-0, +0) no-ops.
// Entering column, row i (!ROW): x = fma(-C_v[i], P_v[k], x) for v <= q; with
// SEL the steps v <= lim (this lane's restart point, -1 if none) are (+0, +0)
// no-ops. own: this thread's slice slots; uni: the wave's uniform row.
template <bool ROW, bool SEL>
__device__ __forceinline__ double chain_batch(const d2 (&o)[8], const d2 (&w)[8], int base, int lim, double x) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const bool l0 = !SEL || base + 2 * j > lim, l1 = !SEL || base + 2 * j + 1 > lim;
        if (ROW) {
            x = fma(l0 ? w[j].x : -0.0, l0 ? o[j].x : 0.0, x);
            x = fma(l1 ? w[j].y : -0.0, l1 ? o[j].y : 0.0, x);
        } else {
            x = fma(-(l0 ? o[j].x : 0.0), l0 ? w[j].x : 0.0, x);
            x = fma(-(l1 ? o[j].y : 0.0), l1 ? w[j].y : 0.0, x);
        }
    }
    return x;
}
// NB batches, fully unrolled: batch b+1's reads are issued before batch b's
// fmas (a runtime loop over the batches measured slower from the third batch
// on: its back-edge carried the prefetched operands through spills)
template <bool ROW, bool SEL, int NB>
__device__ __forceinline__ double chain_n(const double *own, const double *uni, int lim, double x) {
    d2 o[2][8], w[2][8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        o[0][j] = ((const d2 *)own)[j];
        w[0][j] = ((const d2 *)uni)[j];
    }
#pragma unroll
    for (int bb = 0; bb < NB; bb++) {
        if (bb + 1 < NB) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                o[(bb + 1) & 1][j] = ((const d2 *)own)[8 * (bb + 1) + j];
                w[(bb + 1) & 1][j] = ((const d2 *)uni)[8 * (bb + 1) + j];
            }
        }
        x = chain_batch<ROW, SEL>(o[bb & 1], w[bb & 1], 16 * bb, lim, x);
    }
    return x;
}
template <bool ROW, bool SEL, bool B2>
__device__ __forceinline__ double chain(const double *own, const double *uni, int nb, int lim, double x) {
#ifndef LPG_CHAIN_UNROLL96
#ifdef LPG_CHAIN_UNROLL64
    if (B2) {
#else
    if (true) {
#endif
        // a loop over pairs of batches (then one), not a fully unrolled form
        // per batch count: at 96 slots those six bodies per chain kind made the
        // launch's code (77 KB) larger than the instruction cache two CUs share
        // (64 KB); at <= 64 slots the four bodies held 400-470 registers with
        // spills, the loop 280-360 and none (config 5 68.7k -> 72.1k pivots/s,
        // config 2 +0.9%, profiles/r05_ab_chain_loop64.log). Each pair restarts
        // the operand prefetch (one LDS round trip per 32 slots)
        int b = 0;
#pragma unroll 1
        for (; b + 2 <= nb; b += 2) x = chain_n<ROW, SEL, 2>(own + 16 * b, uni + 16 * b, lim - 16 * b, x);
        if (b < nb) x = chain_n<ROW, SEL, 1>(own + 16 * b, uni + 16 * b, lim - 16 * b, x);
        return x;
    }
#endif
    switch (nb) {      // nb <= KB / 16: blocks of <= 64 or <= 96 pivots (block_geometry)
        case 0: return x;
        case 1: return chain_n<ROW, SEL, 1>(own, uni, lim, x);
        case 2: return chain_n<ROW, SEL, 2>(own, uni, lim, x);
        case 3: return chain_n<ROW, SEL, 3>(own, uni, lim, x);
        case 4: return chain_n<ROW, SEL, 4>(own, uni, lim, x);
        case 5: return B2 ? chain_n<ROW, SEL, 5>(own, uni, lim, x) : x;
        default: return B2 ? chain_n<ROW, SEL, 6>(own, uni, lim, x) : x;
    }
}

struct BlockArgs {
    double *T;
    Geo g;
    DevState *st;
    int s0, q0, n;               // parity and pending index of the first pivot; pivots in this launch
    Cand *part;                  // out: one ratio candidate per workgroup, none up to ncand
    int ncand;
    const Cand *cin;             // in: the first pivot's ratio candidates (ncin; == part on one rank)
    int ncin;
    Xch X;                       // multi-rank: the owner-push exchange
    uint32_t xtag0;              // multi-rank: exchange tag of pivot i of this launch = xtag0 + i
    const double *Cs0;           // C[s0]: the first pivot's column snapshot (incl. objective rows)
    double *Cs1;                 // C[(s0 + n) & 1]: the snapshot the launch leaves behind
    Defer D;
    u4 *rec;                     // nwg * (kRecPMax + kRecR) granules
    uint32_t tag0;               // tag of pivot i of this launch = tag0 + 1 + i (never repeats per context)
    int nwg, cw, rw, ks;         // workgroups, columns / rows per slice, LDS slots
    uint32_t cl;                 // residency census: this launch's index since the DevState was reset (1-based)
    int xcd1;                    // 1: a grid of 8 x nwg blocks of which blocks b % 8 == 0 work (one XCD, below)
    // REG (region mode): the slices hold the live columns only (below)
    const int32_t *live;         // nlive physical columns, nonbasic at the block start, column 0 excluded
    int64_t nlive;
    const int64_t *bcol0;        // m: (logical << 32) | physical column of row r's basic variable at the block start
    int nsp, cwx;                // spare column slots per workgroup; thread rows of the sP slice
};

// MR (multi-rank, row partition; Xch attached): the leaving row is the
// minimum over every rank's best ratio candidate (xpush_best / xpoll_best);
// the owner of row r computes the pivot row on each slice and stores it into
// every other rank's xP behind a per-workgroup flag, the other ranks'
// workgroups wait for their slice's flag and read it. Pricing needs no
// exchange: P and the objective rows are replicated, so every rank takes the
// same entering column from its own records. rq holds LOCAL rows (-1: another
// rank's), the replicated basis / lv are kept by workgroup 0 of every rank.
// KB: the pending slots a block may hold, 64 or 96. Pending pivot u's per-slot
// scalars (its row r_u, the multipliers -C_u[r], the entering column's P_u[k])
// sit in lane u of every wave -- for KB = 96 a second bank of registers holds
// slots 64..95 in lanes 0..31 (B2).
//
// REG (region mode, one objective row): the column slices hold only the
// columns whose pending P entries can be nonzero. A column basic at the block
// start has P_u = +0 at every pivot until it leaves the basis (its column is
// the unit vector e_r, so the pivot row's entry is +0 unless the pivot row is
// r), so the slices hold the nonbasic columns of the block start (a.live:
// with the column trade these keep their physical positions from block to
// block) and, per pending pivot sq, one spare slot (workgroup sq mod nwg,
// thread cw + sq / nwg) that takes over the column leaving the basis at pivot
// sq when row r_sq was not pivoted earlier in the block (otherwise the leaving
// variable entered during the block and is a live column already). At its
// leaving pivot the spare evaluates the chain from the base value 1.0 (row
// r_sq of e_r) over its +0 slots -- the value every column thread of the
// all-column form computes -- while it looks up the column (a.bcol0[r_sq]);
// it stores that slot and applies its objective update at the next pivot, before
// any reader (never priced at its own leaving pivot: d_L = -d_k P_q[L] >= 0,
// so not eligible). Workgroup 0's thread cw + nsp holds column 0 (b).
// On a rank of a row partition (MR): the spare of pivot sq is decided from the
// global pivot rows of the block (rgv, D.rqg) so that every rank agrees; the
// owner of the leaving row computes its entry as above and pushes it with its
// pivot row's slice, the other ranks read it behind that slice's flag (bcol0 holds
// every row of the LP, not only this rank's).
// Preconditions kept by the host (lpg_ctx.hip region_setup): basic columns
// are exact unit vectors with zero reduced costs, every block's column trade
// was complete (k_swap_plan sets DevState::rbad otherwise and the launch
// stops with kStallRegion), end_block zeroes the spares' Pbuf columns.
template <int RULE, int NOBJ, bool MR, int KB, bool REG>
__global__ __launch_bounds__(kNT, 1) void k_pivot_block(BlockArgs a) {
    static_assert(!REG || NOBJ == 1, "region mode: one objective row");
    constexpr bool B2 = KB > 64;
    constexpr int WS = B2 ? 104 : 72;                // per-wave slot rows of wm / wp
    // pricing record granules: {key, j} {P_q[phys], phys} [{dR}] [{dM}], and one
    // extra granule {P_q[0]} after the nwg records (workgroup 0's). Dantzig on
    // one objective row carries no dR: the key holds it (cls 0, ~bits(dR) in the
    // low 63 bits), so the record a sweep reads is 32 bytes, not 64.
    constexpr bool KDR = RULE != RULE_BLAND && NOBJ == 1;    // dR recovered from the key
    constexpr int GDR = KDR ? 0 : 2;                         // granule of dR (0: none)
    constexpr int NGP = 2 + (KDR ? 0 : 1) + (NOBJ == 2 ? 1 : 0);
    // ratio records: {theta, key} {piv, row}; one rank under Dantzig (key ==
    // row) sweeps only {theta, row} and fetches the winner's {piv, row} granule
    // (granule nwg + w) while the pivot row's base entries load -- the pivot
    // element is first needed after the chain
    constexpr bool RPIV = !MR && RULE != RULE_BLAND;
    constexpr int NGR = RPIV ? 1 : kRecR;
    static_assert(NGP < kRecPMax, "pricing records (nwg * NGP + 1 granules) exceed their reservation");
    // PK1 (KDR): the sweep reads one granule per workgroup, {key, physical
    // column}; the winner's {P_q[phys], j} granule (nwg + w) is fetched after
    // the sweep while the entering column's base entries load (j, the tie-break,
    // is read for every record that shares the least key -- rare)
    // Bland on one objective row (round 5): the same one-granule sweep with the
    // key = j (Bland's entering column is the least eligible j, and j is
    // unique: no ties), and the winner's dR in a third granule (2 nwg + w),
    // fetched after the sweep beside {P_q[k], j} -- the sweep read 3 granules
    // per workgroup before
    constexpr bool PK1 = NOBJ == 1;
    constexpr bool PKD = PK1 && !KDR;                        // PK1 with the dR granule (Bland)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ Bcast bc;
    __shared__ int xok;
    // per wave, by pending slot: the pivot row's multipliers -C_u[r] (phase P)
    // and the entering column's P_u[k] (phase S); slots 64..71 are the
    // padding a batch of 8 may reach: -0 and +0, so a padded step
    // fma(-0, +0, x) / fma(-(+0), +0, x) is exactly x
    __shared__ __attribute__((aligned(16))) double wm[kNT / 64][WS], wp[kNT / 64][WS];
    const Geo &g = a.g;
    const Defer &D = a.D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // xcd1: blocks b and b + 8 share an XCD and its L2, so workgroup w runs as
    // block 8 w and the other blocks leave at once: every record's store and
    // load then stays on one XCD (0.98-1.21 us per sweep vs 1.33-1.50 over the
    // chip at 16-32 workgroups, profiles/r05_sweep_lab_one_xcd.log). Speed only:
    // the records keep their sc1 stores and loads, correct on any placement.
    if (a.xcd1 && (blockIdx.x & 7)) return;
    const int wg = a.xcd1 ? (int)(blockIdx.x >> 3) : (int)blockIdx.x, nwg = a.nwg, cw = a.cw, rw = a.rw, ks = a.ks;
    // thread-major slices: sP[col][slot], sC[row][slot], a row of S = slot_stride(ks)
    // doubles (>= ks + 8, = 2 mod 4: 16-byte reads of 16 consecutive lanes hit all
    // 64 banks once). Slots past the pending block stay +0, so the chains'
    // padding steps (a batch of 8 past q) are exact no-ops.
    const int S = slot_stride(ks);
    const int cwx = REG ? a.cwx : cw;                  // thread rows of sP (REG: + spares + column 0)
    double *sP = lds;
    double *sC = lds + (size_t)S * cwx;
    double *sPt = sP + (size_t)(tid < cwx ? tid : cwx - 1) * S;   // this thread's slots (clamped: in bounds)
    double *sCt = sC + (size_t)(tid < rw ? tid : rw - 1) * S;
    const int64_t ncp = (g.ncols + 1) & ~(int64_t)1;   // columns incl. the even padding one (k_flushw reads pairs)
    int64_t c = (int64_t)wg * cw + tid;                // this thread's physical column
    bool hc = tid < cw && c < ncp;
    int sq = -1;                                       // REG spare slot: the pending index it serves
    if (REG) {
        if (tid < cw) {
            const int64_t k = (int64_t)wg * cw + tid;
            hc = k < a.nlive;
            c = hc ? a.live[k] : 0;
        } else if (tid < cw + a.nsp) {
            sq = wg + (tid - cw) * nwg;
            if (sq >= ks) sq = -1;
            hc = false;
            c = 0;
        } else {
            hc = wg == 0 && tid == cw + a.nsp;         // column 0
            c = 0;
        }
    }
    const bool colwave = wave * 64 < cwx;              // this wave holds column threads (phase P's chain)
    // REG spare state: at its leaving pivot (actq) the spare keeps P_actq there and
    // that pivot's objective multiplier; its column ({logical, physical}) and the
    // objective entry there land while the block goes on
    int actq = -1;
    double pql = 0.0, cobl = 0.0, dR0 = 0.0;
    int64_t bc0 = 0;
    const int64_t i = (int64_t)wg * rw + tid;          // this thread's local constraint row
    const bool hr = tid < rw && i < g.nloc;
    const int64_t rM = g.nloc, rR = g.nloc + NOBJ - 1;
    const __amdgpu_buffer_rsrc_t recP = rsrc(a.rec, (nwg * NGP + 1) * 16);
    const int xidx = PK1 ? (PKD ? 3 : 2) * nwg : nwg * NGP;     // workgroup 0's {P_q[0]} granule
    const __amdgpu_buffer_rsrc_t recR = rsrc(a.rec + nwg * kRecPMax, nwg * kRecR * 16);
    DevState *st = a.st;

    // ---- residency census: the whole grid (every rank's) resident, or nothing
    {
        __shared__ int go;
        if (tid == 0) go = census<MR>(st, nwg, a.cl, a.X, a.xtag0);
        __syncthreads();
        if (!go) {
            if (tid == 0) {               // every workgroup alike: no pivot ran; the loop stops until the host
                // has switched to the pair (lpg_ctx.hip recover_residency). Only a
                // RUNNING slot is stopped: a terminal status (a launch enqueued
                // after the loop had ended) is the result and stays
                for (int u = 0; u < 2; u++)
                    if (st->slot[u].status == RUNNING) st->slot[u].status = ITER_LIMIT;
                st->stall = kStallResidency;
            }
            return;
        }
    }
    // ---- region mode: the live columns are the block start's nonbasic ones
    // only while every block's column trade was complete (k_swap_plan clears
    // nothing and sets rbad otherwise, e.g. after a forced pivot with a
    // negative element); then no pivot runs and the host rebuilds the region
    if (REG && st->rbad) {
        if (wg == 0 && tid == 0) {
            for (int u = 0; u < 2; u++)
                if (st->slot[u].status == RUNNING) st->slot[u].status = ITER_LIMIT;
            st->stall = kStallRegion;
        }
        return;
    }

    // ---- launch start: everything here was written before the launch
    int s = a.s0;
    const int32_t status0 = st->slot[s].status;
    const int64_t np0 = st->pivots, logcap = st->logcap;   // pivots before this launch (workgroup 0 counts on)
    int64_t kt = st->slot[s].k;                        // entering column (logical) of the first pivot
    double cobjM = NOBJ == 2 ? a.Cs0[rM] : 0.0, cobjR = a.Cs0[rR];
    double dM = 0.0, dR = 0.0;
    int32_t lj = 0;
    if (REG && sq >= 0 && sq < a.q0) {
        // a spare of an earlier launch of this block: active iff the variable that
        // left at pivot sq had not entered earlier in the block (then its row had
        // not been pivoted); the earlier launch stored its slots and objective entry
        const int64_t L = D.lv[sq];
        bool fresh = L > 0;
        for (int u = 0; u < sq; u++) fresh = fresh && D.kq[u] != L;
        if (fresh) {
            c = D.inv[L];
            hc = true;
        }
    }
    if (hc) {
        if (NOBJ == 2) dM = g.T[rM * g.ld + c];
        dR = g.T[rR * g.ld + c];
        lj = D.colmap[c];
    }
    int64_t rqv = lane < a.q0 ? D.rq[lane] : -1;       // lane u: r_u of pending pivot u
    int64_t rqv1 = B2 && 64 + lane < a.q0 ? D.rq[64 + lane] : -1;   // bank 1: r_{64 + lane}
    // MR + REG, lane u: the GLOBAL row of pending pivot u (rqv holds local rows,
    // -1 off this rank): whether a spare takes over the leaving column must be
    // decided alike on every rank
    int64_t rgv = (MR && REG && lane < a.q0) ? D.rqg[lane] : -1;
    int64_t rgv1 = (MR && REG && B2 && 64 + lane < a.q0) ? D.rqg[64 + lane] : -1;
    for (int u = 0; u < S; u++) {
        if (tid < cwx) sPt[u] = (u < a.q0 && hc) ? D.Pbuf[(int64_t)u * g.ld + c] : 0.0;
        if (tid < rw) sCt[u] = (u < a.q0 && hr) ? D.Cbuf[(int64_t)u * D.cs + i] : 0.0;
    }
    double b = 0.0;                                    // column 0 of the current tableau, this thread's row
    int64_t mybasis = 0;
    int lastpiv = -1;                                  // last pending pivot on this thread's row
    if (hr) {
        const double cq = a.Cs0[i];
        sCt[a.q0] = cq;
        st_wt(D.Cbuf + (int64_t)a.q0 * D.cs + i, cq);   // read as a multiplier by other slices later
        b = g.T[i * g.ld];
        mybasis = D.basis[g.row0 + i];
    }
    {
        const double p0l = lane < a.q0 ? D.Pbuf[(int64_t)lane * g.ld] : 0.0;
        const double p0l1 = B2 && 64 + lane < a.q0 ? D.Pbuf[(int64_t)(64 + lane) * g.ld] : 0.0;
        const uint64_t p0b = (uint64_t)__double_as_longlong(p0l), p0b1 = (uint64_t)__double_as_longlong(p0l1);
        for (int u = 0; u < a.q0; u++) {               // b = the pending chain over the earlier pivots
            const bool hi = B2 && u >= 64;
            const double p0 = __longlong_as_double((long long)(hi ? rdl64(p0b1, u - 64) : rdl64(p0b, u)));
            const int64_t ru = (int64_t)(hi ? rdl64((uint64_t)rqv1, u - 64) : rdl64((uint64_t)rqv, u));
            if (hr) {
                b = (i == ru) ? p0 : fma(-sCt[u], p0, b);
                if (i == ru) lastpiv = u;
            }
        }
    }
    if (lane < WS - 64) {
        wm[wave][64 + lane] = -0.0;
        wp[wave][64 + lane] = 0.0;
    }
    __syncthreads();
    bool stop = status0 != RUNNING;
    if (stop && wg == 0 && tid == 0) st->slot[s ^ 1].status = status0;
    double p0q = 0.0;                                  // P_q[0] of the current pivot (workgroup 0's record)

    for (int t = 0; t < a.n && !stop; t++) {
        const int q = a.q0 + t;
        const uint32_t tag = a.tag0 + 1 + (uint32_t)t;
        LPG_BPH(t, 0);
        // ================= phase P: the leaving row and the pivot row
        // MR: this rank's best ratio candidate goes to every rank, and while
        // the grid's best is awaited every workgroup computes the pivot row
        // of this rank's best row -- which is the grid's whenever this rank
        // holds the grid's (the global minimum is one of the ranks' minima)
        u4 pvg{0u, 0u, 0u, 0u};                         // RPIV, wave 0 lane 0: the winner's {piv, row} granule
        bool pvneed = false;                            // RPIV, wave 0: it is still to be checked
        int psrc = -1;
        if (wave == 0) {
            uint64_t h = ~0ull, p0 = 0, p1 = 0;
            uint32_t l = ~0u;
            int src = -1;
            bool ok = true;
            if (t == 0) {
                // candidates of the previous select (k_select_d, a bootstrap or the previous launch)
                uint64_t mh = ~0ull, mp0 = 0, mp1 = 0;
                uint32_t ml = ~0u;
                for (int e = lane; e < a.ncin; e += 64) {
                    const Cand cd = a.cin[e];
                    if (cd.row < 0) continue;
                    const uint64_t ch = (uint64_t)__double_as_longlong(cd.theta);
                    const uint32_t cl = (uint32_t)cd.key;
                    if (key_less(ch, cl, mh, ml)) {
                        mh = ch;
                        ml = cl;
                        mp0 = (uint64_t)__double_as_longlong(cd.piv);
                        mp1 = (uint64_t)cd.row;
                    }
                }
                h = mh;
                l = ml;
                wave_min_key(h, l);
                const int wl = winner_lane(mh == h && ml == l && mh != ~0ull);
                if (wl >= 0 && !(h == ~0ull && l == ~0u)) {
                    src = 0;
                    p0 = rdl64(mp0, wl);
                    p1 = rdl64(mp1, wl);
                }
            } else {
                u4 rec[kPer][NGR], pay[NGR > 1 ? NGR - 1 : 1];
                ok = sweep<NGR>(recR, nwg, tag - 1, rec, 1, st);
                if (ok) {
                    rec_min<NGR>(rec, nwg, h, l, src, pay);
                    if (RPIV) {
                        p1 = l;                 // leaving row (the key)
                        if (src >= 0 && lane == 0) pvg = rec_load(recR, (nwg + src) * 16);   // checked below
                        pvneed = src >= 0;
                    } else {
                        p0 = lo64(pay[0]);      // pivot element
                        p1 = pay[0].z;          // leaving row
                    }
                }
            }
            if (MR && wg == 0 && ok && lane == 0)   // this rank's best -> every rank
                xpush_best(a.X, a.xtag0 + (uint32_t)t, src >= 0 ? h : ~0ull, src >= 0 ? l : ~0u, p0, p1);
            psrc = src;
            if (lane == 0) {
                bc.h = h;
                bc.l = l;
                bc.ok = !ok ? -1 : (src >= 0 ? 1 : 0);
                bc.p0 = p0;
                bc.p1 = p1;
                bc.pv = p0;
                bc.okv = 1;
            }
        }
        __syncthreads();
        LPG_BPH(t, 1);
        LPG_BSEEN(1, t);                                // the ratio decision (records of phase S, t - 1)
        int okP = bc.ok;
        int64_t r = (int64_t)bc.p1;                     // leaving row (MR: this rank's candidate so far)
        const int64_t rs = r;                           // MR: the row computed ahead of the decision
        const bool owns = okP > 0 && (!MR || (rs >= g.row0 && rs < g.row0 + g.nloc));
        // this slice's base entries of row rs and the multipliers -C_u[rs]
        // (lane u < q; -0 past q): in flight across the barrier below
        const int64_t rloc = owns ? rs - g.row0 : -1;
        // REG: an active spare's first pivot after its leave (actq) completes it
        // here, before the drain below: the leave's slot into Pbuf (a reader
        // meets it at the earliest in this pivot's phase S, behind the pricing
        // records) and its objective update; and the spare of this pivot takes
        // the leaving column if row r was not pivoted earlier in the block
        bool actnow = false;
        if (REG) {
            if (actq >= 0 && !hc) {
                c = (int64_t)(uint32_t)bc0;
                lj = (int32_t)(bc0 >> 32);
                hc = true;
                dR = fma(-cobl, pql, dR0);
                st_wt(D.Pbuf + (int64_t)actq * g.ld + c, pql);
            }
            // MR: this rank's candidate row, before the decision (speculative, as the pivot row)
            const unsigned long long h0 = __ballot(lane < q && (MR ? rgv : rqv) == rs);
            const unsigned long long h1 = B2 ? __ballot(64 + lane < q && (MR ? rgv1 : rqv1) == rs) : 0ull;
            actnow = sq == q && owns && (h0 | h1) == 0ull;
            if (actnow) bc0 = a.bcol0[rs];               // {logical, physical}: needed from the next pivot on
        }
        const double xrow = (owns && hc) ? g.T[rloc * g.ld + c] : (actnow ? 1.0 : 0.0);
        // (unconditional loads from clamped addresses, negated and selected at
        // their use: a load behind the condition was waited for on the spot)
        const double mraw = ld_wt(D.Cbuf + (int64_t)(lane < q ? lane : 0) * D.cs + (owns ? rloc : 0));
        const double mraw1 = B2 ? ld_wt(D.Cbuf + (int64_t)(64 + lane < q ? 64 + lane : 0) * D.cs + (owns ? rloc : 0)) : 0.0;
        if (RPIV && pvneed) {
            // the winner's {piv, row} granule: stored with its {theta, row}, so
            // normally already visible; re-polled (bounded) if not
            const long long t0 = (long long)wall_clock64();
            int okv = 1;
            if (lane == 0) {
                while (pvg.w != tag - 1 || (int64_t)pvg.z != r) {
                    if ((long long)wall_clock64() - t0 > kSpinTicks) {
                        okv = -1;
                        st->stall_info[0] = 7;
                        st->stall_info[1] = tag - 1;
                        st->stall_info[2] = nwg + psrc;
                        st->stall_info[3] = pvg.w;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    pvg = rec_load(recR, (nwg + psrc) * 16);
                }
                bc.pv = lo64(pvg);
                bc.okv = okv;
            }
        }
        __syncthreads();                                // bc is rewritten below / by the next phase
        double piv = __longlong_as_double((long long)bc.pv);
        if (RPIV && bc.okv < 0) okP = -1;
        auto fail_p = [&](int ok) {                     // the oracle's NUMERIC rule (k_prep_d), UNBOUNDED, timeouts
            if (wg == 0 && tid == 0) {
                const int32_t sv = ok < 0 ? NUMERIC : (ok == 0 ? UNBOUNDED : NUMERIC);
                st->slot[s].status = sv;
                st->slot[s].r = -1;
                st->slot[s ^ 1].status = sv;
                if (ok < 0) st->stall = ok == -2 ? 2 : 1;
            }
        };
        if (!MR && (okP <= 0 || !isfinite(piv))) {
            fail_p(okP);
            break;
        }
        // row rr of the current tableau on this slice (on: this rank holds it):
        // the multipliers -C_u[rr] (lane u < q; -0 past q), the restart point
        // (the last pending pivot on rr), the base entries, the pending chain
        auto pivot_row = [&](bool on, int64_t rr) -> double {
            wm[wave][lane] = (owns && lane < q) ? -mraw : -0.0;
            if (B2 && lane < 32) wm[wave][64 + lane] = (owns && 64 + lane < q) ? -mraw1 : -0.0;
            const unsigned long long hit = __ballot(on && lane < q && rqv == rr);
            const unsigned long long hit1 = B2 ? __ballot(on && 64 + lane < q && rqv1 == rr) : 0ull;
            const int qs = hit1 ? 127 - __clzll((long long)hit1) : (hit ? 63 - __clzll((long long)hit) : -1);
            double x = xrow;
            if (qs >= 0) x = sPt[qs];
            const double *wmw = &wm[wave][0];
            if (!on || !colwave) {
                // another rank's row: its P slice arrives below (or no column in this wave)
            } else if (qs < 0) {
                x = chain<true, false, B2>(sPt, wmw, (q + 15) >> 4, qs, x);      // slots u < q
            } else {
                x = chain<true, true, B2>(sPt, wmw, (q + 15) >> 4, qs, x);
            }
            return x;
        };
        LPG_BPH(t, 15);
        double x = pivot_row(owns, rloc);
        LPG_BPH(t, 2);
        const uint32_t xt = a.xtag0 + (uint32_t)t;      // MR: this pivot's exchange tag
        const int xpar = (int)(xt & 1);
        if (MR && owns && a.X.world > 1) {
            // every rank with a candidate sends ITS pivot row slice to every
            // other rank (into the sender's own region, behind a per-slice
            // flag) before the decision is known: the owner's copy, the one
            // the others will read, is then already on its way while the
            // decision travels (the other copies are never read)
            if (hc) {
                const uint64_t v = (uint64_t)__double_as_longlong(x / piv);
                for (int rk = 0; rk < a.X.world; rk++)
                    if (rk != a.X.rank) st_sys64(xch_row(a.X, rk, xpar, a.X.rank, g.ld) + c, v);
            }
            if (REG && actnow) {                        // the spare's entry, at the leaving column
                const uint64_t v = (uint64_t)__double_as_longlong(x / piv);
                for (int rk = 0; rk < a.X.world; rk++)
                    if (rk != a.X.rank) st_sys64(xch_row(a.X, rk, xpar, a.X.rank, g.ld) + (uint32_t)bc0, v);
            }
            drain();
            __syncthreads();
            if (tid == 0) {
                release_system();
                for (int rk = 0; rk < a.X.world; rk++)
                    if (rk != a.X.rank)
                        __hip_atomic_store(xch_flag(a.X, rk, xpar, wg, a.X.rank), xt, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (MR) {                                       // every rank's best -> the grid's
            if (wave == 0) {
                uint64_t h = ~0ull, p0 = 0, p1 = 0;
                uint32_t l = ~0u;
                const bool ok = okP >= 0 && xpoll_best(a.X, a.xtag0 + (uint32_t)t, h, l, p0, p1, st);
                if (lane == 0) {
                    bc.ok = okP < 0 ? -1 : (!ok ? -2 : ((h == ~0ull && l == ~0u) ? 0 : 1));
                    bc.p0 = p0;
                    bc.p1 = p1;
                }
            }
            __syncthreads();
            okP = bc.ok;
            piv = __longlong_as_double((long long)bc.p0);
            r = (int64_t)bc.p1;
            __syncthreads();
            if (okP <= 0 || !isfinite(piv)) {
                fail_p(okP);
                break;
            }
        }
        const bool own = !MR || (r >= g.row0 && r < g.row0 + g.nloc);   // uniform: this rank holds row r
        const int64_t rl = MR ? (own ? r - g.row0 : -1) : r;           // its local index (-1: another rank's)
        if (MR && REG) {
            // the decision, row r (global): a spare takes over the leaving column
            // iff r was not pivoted earlier in the block -- on every rank alike.
            // The owner computed its entry above (r == rs) and pushed it with its
            // slice; the others read it behind the slice's flag below
            const unsigned long long ga = __ballot(lane < q && rgv == r);
            const unsigned long long gb = B2 ? __ballot(64 + lane < q && rgv1 == r) : 0ull;
            const bool act = sq == q && (ga | gb) == 0ull;
            if (act && !own) bc0 = a.bcol0[r];
            actnow = act;
        }
        if (MR && own && !(owns && r == rs)) {
            // cannot happen: the grid's minimum, if this rank holds it, is this
            // rank's minimum (unique keys). Stop loudly rather than guess.
            if (tid == 0) {
                st->slot[s].status = NUMERIC;
                st->slot[s ^ 1].status = NUMERIC;
                st->stall_info[0] = 6;
                st->stall = 1;
            }
            break;
        }
        int64_t lvv = 0;                                // MR: the leaving variable, from the replicated basis
        // k_prep_d's bookkeeping, stores only (a dependent load here would hold
        // back workgroup 0, and every sweep waits for the slowest workgroup):
        // the row's owner records the leaving variable it holds. One rank:
        // both after this pivot's pricing record (book_late below) -- here they
        // sat in front of the drain that gates the record, and workgroup 0 was
        // the last to publish in 43 of 64 pivots (profiles/r04_block_probe_clock.log)
        const bool own_row = hr && i == rl;             // this thread holds the leaving row
        const int64_t lv_old = mybasis;
        if (MR && wg == 0 && tid == 0) {
            st->slot[s].r = r;
            D.rq[q] = rl;
            if (REG) D.rqg[q] = r;                      // global: later launches of the block restore rgv
            if (MR) lvv = D.basis[r];                   // stored after the P exchange: its latency hides there
            st->npend = q + 1;
            D.kq[q] = kt;
            D.pv[q] = piv;
            const int64_t np = np0 + t;
            if (D.logk && np < logcap) {
                D.logk[np] = kt;
                D.logr[np] = r;
            }
            st->pivots = np + 1;
            st->last_k = kt;
            st->last_r = r;
        }
        if (own_row) {
            mybasis = kt;
            lastpiv = q;
        }
        if (lane == q) rqv = rl;
        if (B2 && 64 + lane == q) rqv1 = rl;
        if (MR && REG && lane == q) rgv = r;
        if (MR && REG && B2 && 64 + lane == q) rgv1 = r;
        LPG_BPH(t, 8);
        drain();                                        // the previous phase's C stores, before this record
        LPG_BPH(t, 9);
        PricePart pb{0.0, -1, 0, 0};
        double pq = 0.0;
        int xowner = -1;                                // MR: the rank that pushed this pivot's row
        if (own && hc) pq = x / piv;
        if (MR) {
            if (!own) {                                 // wait for this slice of P from the owner
                // the owner: rows [floor(m p / W), floor(m (p + 1) / W)) are rank p's
                int owner = (int)((r * (int64_t)a.X.world) / g.m);
                while (owner + 1 < a.X.world && (g.m * (int64_t)(owner + 1)) / a.X.world <= r) owner++;
                xowner = owner;
                if (tid == 0) {
                    const long long t0 = (long long)wall_clock64();
                    int okx = 1;
                    while (__hip_atomic_load(xch_flag(a.X, a.X.rank, xpar, wg, owner), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM) != xt) {
                        if ((long long)wall_clock64() - t0 > kSpinTicks) {
                            okx = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    xok = okx;                          // the slice is read with system-scope loads: no acquire
                }
                __syncthreads();
                if (!xok) {
                    if (tid == 0) {
                        st->slot[s].status = NUMERIC;
                        st->slot[s ^ 1].status = NUMERIC;
                        st->stall_info[0] = 5;
                        st->stall_info[1] = xt;
                        st->stall = 3;
                    }
                    break;
                }
                if (hc) pq = __longlong_as_double((long long)ld_sys64(xch_row(a.X, a.X.rank, xpar, owner, g.ld) + c));
            }
            if (wg == 0 && tid == 0) {                  // the replicated basis and the block's leaving variables
                D.lv[q] = lvv;
                D.basis[r] = kt;
            }
        }
        if (REG && actnow) {                           // the spare's slot q; Pbuf and d at the next pivot
            // MR, another rank's row: the owner's entry, behind the flag awaited above
            pql = (MR && !own) ? __longlong_as_double((long long)ld_sys64(xch_row(a.X, a.X.rank, xpar, xowner, g.ld) +
                                                                          (uint32_t)bc0))
                               : x / piv;
            sPt[q] = pql;
            cobl = cobjR;
            actq = q;
        }
        if (hc) {
            sPt[q] = pq;
            st_wt(D.Pbuf + (int64_t)q * g.ld + c, pq);  // drained in phase S, before the ratio record
            if (NOBJ == 2) dM = fma(-cobjM, pq, dM);
            dR = fma(-cobjR, pq, dR);
            price_one<RULE>(pb, dM, dR, lj, g, c);
            pb.pad = (int32_t)c;
        }
        LPG_BPH(t, 10);
        pb = block_argmin_pp<RULE, kNT / 64, false>(pb);   // barriers since the previous call: no lead
        LPG_BPH(t, 11);
        if (tid == 0) {
            uint64_t h = ~0ull;
            uint32_t l = ~0u;
            if (pb.j >= 0) {
                h = RULE == RULE_BLAND ? 0ull
                                       : (((uint64_t)(uint32_t)pb.cls << 63) |
                                          (~(uint64_t)__double_as_longlong(pb.v) & 0x7fffffffffffffffull));
                l = (uint32_t)pb.j;
            }
            if (!PK1) rec_store(recP, (wg * NGP + 0) * 16, pack(h, l, tag));
            else if (pb.j < 0) {
                rec_store(recP, wg * 16, pack(h, l, tag));
                rec_store(recP, (nwg + wg) * 16, pack(0ull, ~0u, tag));
            }
        }
        // P_q[0] for every slice's column 0 (workgroup 0 holds column 0: thread 0, REG thread cw + nsp)
        if (wg == 0 && hc && c == 0) rec_store(recP, xidx * 16, pack((uint64_t)__double_as_longlong(pq), 0u, tag));
        // the slice winner's objective entries and P_q entry ride along (C_{t+1}[obj]
        // and P_q[k] if it wins the grid); the thread of that column holds them
        if (PK1 && pb.j >= 0 && hc && (int64_t)lj == pb.j) {
            // the slice winner's thread: {key, physical column} and {P_q there, j}
            // (PKD: key j, and {dR} in the third granule)
            const uint64_t h = PKD ? (uint64_t)(uint32_t)pb.j
                                   : (((uint64_t)(uint32_t)pb.cls << 63) |
                                      (~(uint64_t)__double_as_longlong(pb.v) & 0x7fffffffffffffffull));
            rec_store(recP, wg * 16, pack(h, (uint32_t)c, tag));
            rec_store(recP, (nwg + wg) * 16, pack((uint64_t)__double_as_longlong(pq), (uint32_t)pb.j, tag));
            if (PKD) rec_store(recP, (2 * nwg + wg) * 16, pack((uint64_t)__double_as_longlong(dR), 0u, tag));
        }
        if (!PK1 && pb.j >= 0 && hc && (int64_t)lj == pb.j) {
            rec_store(recP, (wg * NGP + 1) * 16, pack((uint64_t)__double_as_longlong(pq), (uint32_t)c, tag));
            if (!KDR) rec_store(recP, (wg * NGP + GDR) * 16, pack((uint64_t)__double_as_longlong(dR), 0u, tag));
            if (NOBJ == 2) rec_store(recP, (wg * NGP + NGP - 1) * 16, pack((uint64_t)__double_as_longlong(dM), 0u, tag));
        }
        if (!PK1 && pb.j < 0 && tid == 0) {
#pragma unroll
            for (int k = 1; k < NGP; k++) rec_store(recP, (wg * NGP + k) * 16, pack(0ull, 0u, tag));
        }
        LPG_BPUB(0, t);
        if (!MR) {                                      // book_late: nobody in this launch reads these
            if (wg == 0 && tid == 64) {
                st->slot[s].r = r;
                D.rq[q] = rl;
                st->npend = q + 1;
                D.kq[q] = kt;
                D.pv[q] = piv;
                const int64_t np = np0 + t;
                if (D.logk && np < logcap) {
                    D.logk[np] = kt;
                    D.logr[np] = r;
                }
                st->pivots = np + 1;
                st->last_k = kt;
                st->last_r = r;
            }
            if (own_row) {
                D.lv[q] = lv_old;
                D.basis[r] = kt;
            }
        }
        LPG_BPH(t, 3);

        // ================= phase S: the entering column and the ratio test
        u4 g1{0u, 0u, 0u, 0u};                          // PK1, wave 0 lane 0: the winner's {P_q[k], j}
        u4 g2{0u, 0u, 0u, 0u};                          // PKD, wave 0 lane 0: the winner's {dR}
        int g1src = -1;                                 // PK1, wave 0: its workgroup, -1 if fetched already / none
        if (wave == 0 && PK1) {
            u4 rec[kPer][1], xg{0u, 0u, 0u, 0u};
            const bool ok = sweep<1, true>(recP, nwg, tag, rec, 2, st, &xg, xidx);
            uint64_t hmin = ~0ull, p1 = 0, p2 = 0;
            uint32_t l = ~0u;
            int src = -1, okd = ok ? 1 : -1;
            if (ok) {
                // the least key over this lane's records (branch-free), then the wave's
                uint64_t mh = ~0ull;
                uint32_t mphys = 0;
                int mw = -1, cnt = 0;
#pragma unroll
                for (int p = 0; p < kPer; p++) {
                    const int w = lane + 64 * p;
                    const uint64_t hh = w < nwg ? lo64(rec[p][0]) : ~0ull;
                    const bool lt = hh < mh, eq = hh == mh;
                    cnt = lt ? 1 : (eq ? cnt + 1 : cnt);
                    mw = lt ? w : mw;
                    mphys = lt ? rec[p][0].z : mphys;
                    mh = lt ? hh : mh;
                }
                hmin = wave_min_u64(mh);
                const bool has = hmin != ~0ull && mh == hmin;
                const unsigned long long bal = __ballot(has);
                const bool tie = (__ballot(has && cnt > 1) != 0ull) || __popcll(bal) > 1;
                if (hmin == ~0ull) {
                    okd = 0;                            // no eligible column: OPTIMAL
                } else if (!tie) {
                    const int wl = __ffsll((long long)bal) - 1;
                    src = (int)rdl32((uint32_t)mw, wl);
                    p1 = rdl32(mphys, wl);
                    if (lane == 0) {
                        g1 = rec_load(recP, (nwg + src) * 16);   // checked after the barrier
                        if (PKD) g2 = rec_load(recP, (2 * nwg + src) * 16);
                    }
                    g1src = src;
                } else if (PKD) {
                    okd = -1;                           // Bland's keys are the columns' j: unique, never tied
                } else {
                    // several records share the least key: j decides; fetch {P_q, j}
                    // of each (bounded polls), the least j wins
                    uint32_t bj = ~0u, bphys = 0;
                    uint64_t bpq = 0;
                    int bw = -1;
                    const long long t0 = (long long)wall_clock64();
#pragma unroll
                    for (int p = 0; p < kPer; p++) {
                        const int w = lane + 64 * p;
                        if (w < nwg && lo64(rec[p][0]) == hmin) {
                            u4 v = rec_load(recP, (nwg + w) * 16);
                            while (v.w != tag && (long long)wall_clock64() - t0 <= kSpinTicks) {
                                __builtin_amdgcn_s_sleep(1);
                                v = rec_load(recP, (nwg + w) * 16);
                            }
                            if (v.w != tag) okd = -1;
                            const bool better = v.z < bj;
                            bj = better ? v.z : bj;
                            bphys = better ? rec[p][0].z : bphys;
                            bpq = better ? lo64(v) : bpq;
                            bw = better ? w : bw;
                        }
                    }
                    okd = __ballot(okd < 0) ? -1 : okd;
                    const uint32_t jm = wave_min_u32(bj);
                    const int wl = winner_lane(bw >= 0 && bj == jm);
                    src = wl < 0 ? -1 : (int)rdl32((uint32_t)bw, wl);
                    p1 = wl < 0 ? 0 : rdl32(bphys, wl);
                    p2 = wl < 0 ? 0 : rdl64(bpq, wl);
                    l = jm;
                }
                if (lane == 0) bc.z = lo64(xg);
            }
            if (lane == 0) {
                bc.h = hmin;
                bc.l = l;
                bc.ok = okd < 0 ? -1 : (okd == 0 ? 0 : (src >= 0 ? 1 : -1));
                bc.p0 = (1ull << 63) | (~hmin & 0x7fffffffffffffffull);   // dR at the entering column
                bc.p1 = p1;
                bc.p2 = p2;
                bc.p3 = 0;
            }
        }
        if (wave == 0 && !PK1) {
            u4 rec[kPer][NGP], pay[NGP - 1], xg{0u, 0u, 0u, 0u};
            const bool ok = sweep<NGP, true>(recP, nwg, tag, rec, 2, st, &xg, xidx);
            uint64_t h = ~0ull, p0 = 0, p1 = 0, p2 = 0, p3 = 0;
            uint32_t l = ~0u;
            int src = -1;
            if (ok) {
                rec_min<NGP>(rec, nwg, h, l, src, pay);
                // dR at the entering column: from the key (v < 0: sign bit set,
                // ~bits(v) in the low 63 bits) or its own granule
                p0 = KDR ? ((1ull << 63) | (~h & 0x7fffffffffffffffull)) : lo64(pay[GDR - 1]);
                p1 = pay[0].z;                  // its physical column
                p2 = lo64(pay[0]);              // P_q at the entering column
                if (NOBJ == 2) p3 = lo64(pay[NGP - 2]);   // dM
                // P_q[0]: workgroup 0's extra granule, held by lane 0
                if (lane == 0) bc.z = lo64(xg);
            }
            if (lane == 0) {
                bc.h = h;
                bc.l = l;
                bc.ok = !ok ? -1 : (src >= 0 ? 1 : 0);
                bc.p0 = p0;
                bc.p1 = p1;
                bc.p2 = p2;
                bc.p3 = p3;
            }
        }
        __syncthreads();
        LPG_BPH(t, 4);
        LPG_BSEEN(0, t);                                // the pricing decision (records of phase P, t)
        int okS = bc.ok;
        const int64_t kp = (int64_t)bc.p1;              // physical column of the entering column
        double nR = __longlong_as_double((long long)bc.p0);   // PKD: the fetched granule's, read below
        const double nM = __longlong_as_double((long long)bc.p3);
        p0q = __longlong_as_double((long long)bc.z);
        // column k's base entries on this slice's rows (HBM) and P_u[k] for
        // u < q (Pbuf): in flight across the barrier below
        double xa = (okS > 0 && hr) ? g.T[i * g.ld + kp] : 0.0;
        double pu = (okS > 0 && wave * 64 < rw && lane < q) ? ld_wt(D.Pbuf + (int64_t)lane * g.ld + kp) : 0.0;
        double pu1 = (B2 && okS > 0 && wave * 64 < rw && 64 + lane < q) ? ld_wt(D.Pbuf + (int64_t)(64 + lane) * g.ld + kp)
                                                                         : 0.0;
        // REG: the objective entry of the column that left at this pivot (as
        // stored: a basic column's entry does not change while it stays basic)
        if (REG && actq == q) dR0 = g.T[rR * g.ld + (int64_t)(uint32_t)bc0];
        if (PK1 && wave == 0 && g1src >= 0) {
            // the winner's {P_q[k], j}: stored with its key, so normally visible
            if (lane == 0) {
                const long long t0 = (long long)wall_clock64();
                while (g1.w != tag && (long long)wall_clock64() - t0 <= kSpinTicks) {
                    __builtin_amdgcn_s_sleep(1);
                    g1 = rec_load(recP, (nwg + g1src) * 16);
                }
                if (g1.w != tag) {
                    bc.ok = -1;
                    st->stall_info[0] = 8;
                    st->stall_info[1] = tag;
                    st->stall_info[2] = nwg + g1src;
                    st->stall_info[3] = g1.w;
                } else {
                    bc.l = g1.z;
                    bc.p2 = lo64(g1);
                }
                if (PKD) {                              // the winner's dR, stored with the other two
                    while (g2.w != tag && (long long)wall_clock64() - t0 <= kSpinTicks) {
                        __builtin_amdgcn_s_sleep(1);
                        g2 = rec_load(recP, (2 * nwg + g1src) * 16);
                    }
                    if (g2.w != tag) {
                        bc.ok = -1;
                        st->stall_info[0] = 9;
                        st->stall_info[1] = tag;
                        st->stall_info[2] = 2 * nwg + g1src;
                        st->stall_info[3] = g2.w;
                    } else {
                        bc.p0 = lo64(g2);
                    }
                }
            }
        }
        __syncthreads();
        okS = bc.ok;
        if (PKD) nR = __longlong_as_double((long long)bc.p0);
        const int64_t kn = (int64_t)bc.l;               // logical entering column of pivot t + 1
        const double pkq = __longlong_as_double((long long)bc.p2);   // P_q at the entering column
        const int s1 = s ^ 1;
        if (okS <= 0) {
            if (wg == 0 && tid == 0) {
                const int32_t sv = okS < 0 ? NUMERIC : OPTIMAL;
                st->slot[s1].status = sv;
                st->slot[s1].k = -1;
                st->slot[s1].r = -1;
                st->slot[s].status = sv;
                if (okS < 0) st->stall = 1;
            }
            break;
        }
        if (wg == 0 && tid == 0) {
            st->slot[s1].status = RUNNING;
            st->slot[s1].k = kn;
        }
        // column k of the current tableau; P_u[k] (lane u < q from Pbuf, P_q[k]
        // from the record; +0 past q)
        if (wave * 64 < rw)                             // waves holding rows
            wp[wave][lane] = lane == q ? pkq : pu;
        if (B2 && wave * 64 < rw && lane < 32)
            wp[wave][64 + lane] = 64 + lane == q ? pkq : pu1;
        LPG_BPH(t, 6);
        if (hr) b = (i == rl) ? p0q : fma(-sCt[q], p0q, b);
        // the chain over slots v <= q (q / 16 + 1 batches). A row pivoted earlier in this
        // block restarts at its last pivot lp: x = P_lp[k] and the steps up to
        // lp become no-ops (the select form, for waves holding such a row).
        if (hr && lastpiv >= 0) xa = wp[wave][lastpiv];
        if (wave * 64 < rw) {                           // waves holding rows (xa is used under hr only)
            const double *wpw = &wp[wave][0];
            const bool sel = __ballot(hr && lastpiv >= 0) != 0ull;
            if (!sel) xa = chain<false, false, B2>(sCt, wpw, (q >> 4) + 1, lastpiv, xa);   // slots v <= q
            else xa = chain<false, true, B2>(sCt, wpw, (q >> 4) + 1, lastpiv, xa);
        }
        LPG_BPH(t, 7);
        drain();                                        // this pivot's P stores, before the ratio record
        LPG_BPH(t, 12);
        const bool last = t + 1 == a.n;
        Cand cd{0.0, 0.0, 0, -1};
        if (hr) {
            if (!last) {
                sCt[q + 1] = xa;
                st_wt(D.Cbuf + (int64_t)(q + 1) * D.cs + i, xa);   // drained in the next phase P
            } else {
                a.Cs1[i] = xa;
            }
            if (xa > g.eps_piv) {
                cd.theta = b > 0.0 ? b / xa : 0.0;
                cd.piv = isfinite(b) ? xa : __longlong_as_double(0x7ff8000000000000ll);   // NUMERIC at phase P
                cd.row = g.row0 + i;
                cd.key = RULE == RULE_BLAND ? mybasis : g.row0 + i;
            }
        }
        LPG_BPH(t, 13);
        // all rows in wave 0 (rw <= 64, config 3): its own wave min, no LDS
        // exchange and no barrier (the other waves hold no candidate)
        if (rw <= 64) cd = wave == 0 ? block_argmin_cand<1, false>(cd) : cd;
        else cd = block_argmin_cand<kNT / 64, false>(cd);
        LPG_BPH(t, 14);
        if (tid == 0) {
            uint64_t h = ~0ull;
            uint32_t l = ~0u;
            if (cd.row >= 0) {
                h = (uint64_t)__double_as_longlong(cd.theta);
                l = (uint32_t)cd.key;
            }
            rec_store(recR, (wg * NGR + 0) * 16, pack(h, l, tag));
            rec_store(recR, ((RPIV ? nwg : 0) + wg * NGR + (RPIV ? 0 : 1)) * 16,
                      pack((uint64_t)__double_as_longlong(cd.piv), (uint32_t)cd.row, tag));
            if (last) a.part[wg] = cd;
        }
        if (last && wg == 0 && tid == 0) {
            a.Cs1[rR] = nR;
            if (NOBJ == 2) a.Cs1[rM] = nM;
            for (int e = nwg; e < a.ncand; e++) a.part[e] = Cand{0.0, 0.0, -1, -1};
        }
        LPG_BPUB(1, t);
        LPG_BPH(t, 5);
        kt = kn;
        cobjR = nR;
        cobjM = nM;
        s = s1;
    }
    // REG: a spare whose leave was the launch's last applied pivot completes it here
    if (REG && actq >= 0 && !hc) {
        c = (int64_t)(uint32_t)bc0;
        hc = true;
        dR = fma(-cobl, pql, g.T[rR * g.ld + c]);
        D.Pbuf[(int64_t)actq * g.ld + c] = pql;
    }
    // the objective row(s) of this slice, current after the last applied pivot
    if (hc) {
        if (NOBJ == 2) g.T[rM * g.ld + c] = dM;
        g.T[rR * g.ld + c] = dR;
    }
}

// ---- host side -------------------------------------------------------------

int block_records_bytes(int nwg) { return nwg * (kRecPMax + kRecR) * 16; }

// Default split: the FEWEST workgroups whose slices fit (one column and one
// row per thread at most, both slices in LDS). Every per-pivot all-to-all
// sweeps one record per workgroup, and its cost grows with their number
// (config 2: 77.6k pivots/s on 256 workgroups, 99.8k on 16; config 5: 58.6k
// on 256, 65.2k on 128; config 3 needs all 256 for the LDS).
int block_geometry(const Geo &g, int ks, int cus, int want, int *nwg, int *cw, int *rw, size_t *lds) {
    if (ks < 1 || ks > 96) return -1;                      // blocks of <= 96 pivots (the slices' chains, two lane banks)
    const int64_t ncp = (g.ncols + 1) & ~(int64_t)1;
    const int64_t S = slot_stride(ks);
    const int64_t per_wg = kMaxLds / (S * (int64_t)sizeof(double));   // columns + rows one workgroup holds
    int64_t w = want;
    if (w <= 0) {
        w = std::max<int64_t>({(ncp + kNT - 1) / kNT, (g.nloc + kNT - 1) / kNT, (ncp + g.nloc + per_wg - 1) / per_wg, 1});
        while (w <= kMaxWG && w <= cus && ((ncp + w - 1) / w + (g.nloc + w - 1) / w) > per_wg) w++;
        // one wave of rows: when the fewest workgroups that fit already fill
        // most of the chip and leave more than 64 rows each, take 64 rows per
        // workgroup if the CUs allow (the entering-column chain then runs on
        // one wave; config 3: 256 workgroups instead of 227, +0.6%,
        // profiles/r04_ab_wg256.log)
        const int64_t w64 = (g.nloc + 63) / 64;
        if (w >= 192 && w64 > w && w64 <= kMaxWG && w64 <= cus && (ncp + w64 - 1) / w64 + 64 <= per_wg) w = w64;
    }
    if (w > kMaxWG || w > cus || w < 1) return -1;
    const int64_t c = (ncp + w - 1) / w, r = (g.nloc + w - 1) / w;
    if (c > kNT || r > kNT || c + r > per_wg) return -1;
    *nwg = (int)w;
    *cw = (int)c;
    *rw = (int)r;
    *lds = (size_t)(S * (c + r)) * sizeof(double);
    return 0;
}

// Region mode (REG, see k_pivot_block): the slices hold the nlive nonbasic
// columns of the block start (column 0 excluded), nsp = ceil(ks / nwg) spare
// slots per workgroup and column 0; the FEWEST workgroups whose slices fit
// (threads cw + nsp + 1 <= 256 and rows <= 256, LDS within kMaxLds), then the
// one-wave-of-rows rule of block_geometry.
int block_geometry_region(const Geo &g, int ks, int cus, int want, int64_t nlive, RegionGeo *out) {
    if (ks < 1 || ks > 96 || nlive < 1 || g.nobj != 1) return -1;
    const int64_t S = slot_stride(ks);
    const int64_t per_wg = kMaxLds / (S * (int64_t)sizeof(double));
    auto fits = [&](int64_t w) {
        const int64_t c = (nlive + w - 1) / w, r = (g.nloc + w - 1) / w, x = c + (ks + w - 1) / w + 1;
        return w >= 1 && w <= kMaxWG && w <= cus && x <= kNT && r <= kNT && x + r <= per_wg;
    };
    int64_t w = want;
    if (w <= 0) {
        for (w = 1; w <= kMaxWG && w <= cus && !fits(w); w++) {
        }
        const int64_t w64 = (g.nloc + 63) / 64;
        if (w >= 192 && w64 > w && fits(w64) && (g.nloc + w64 - 1) / w64 <= 64) w = w64;
    }
    if (!fits(w)) return -1;
    out->nwg = (int)w;
    out->cw = (int)((nlive + w - 1) / w);
    out->rw = (int)((g.nloc + w - 1) / w);
    out->nsp = (int)((ks + w - 1) / w);
    out->cwx = out->cw + out->nsp + 1;
    out->lds = (size_t)(S * (out->cwx + out->rw)) * sizeof(double);
    return 0;
}

// ---- region-mode bookkeeping kernels (one workgroup each; bootstrap / rebuild only)

// live: the physical columns in [1, ncols) holding no basic variable, ascending;
// bcol0[r] = (basis[r] << 32) | its physical column; rbad cleared. mark: ld ints.
// tlive[c] = 1 iff the 64 physical columns 64c .. 64c+63 hold a nonbasic one
// (column 0 included): the block pass skips a tile with none without reading
// its pending P entries (k_flushw), checking only the block's leaving columns.
__global__ __launch_bounds__(1024) void k_region_build(DevState *st, const int64_t *basis, const int32_t *inv,
                                                        int64_t m, int64_t ncols, int64_t ld, int32_t *mark,
                                                        int32_t *live, int64_t *bcol0, int64_t nlive, int32_t *tlive) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int64_t p = tid; p < ncols; p += nt) mark[p] = 0;
    __syncthreads();
    for (int64_t r = tid; r < m; r += nt) {
        const int64_t v = basis[r];
        const int32_t p = inv[v];
        mark[p] = 1;
        bcol0[r] = (v << 32) | (int64_t)(uint32_t)p;
    }
    __syncthreads();
    for (int64_t c = tid; c < ld / 64; c += nt) {
        int any = 0;
        for (int64_t p = 64 * c; p < 64 * c + 64 && p < ncols; p++) any |= mark[p] == 0;
        tlive[c] = any;
    }
    // stable compaction of the unmarked columns 1..ncols-1: each thread a contiguous chunk
    const int64_t per = (ncols - 1 + nt - 1) / nt, p0 = 1 + (int64_t)tid * per, p1 = std::min<int64_t>(p0 + per, ncols);
    int cnt = 0;
    for (int64_t p = p0; p < p1; p++) cnt += mark[p] == 0;
    __shared__ int part[1024];
    part[tid] = cnt;
    __syncthreads();
    for (int d = 1; d < nt; d <<= 1) {           // inclusive scan (Hillis-Steele)
        const int v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int64_t o = part[tid] - cnt;
    for (int64_t p = p0; p < p1; p++)
        if (mark[p] == 0 && o < nlive) live[o++] = (int32_t)p;
    if (tid == 0) st->rbad = (part[nt - 1] == nlive) ? 0u : 2u;   // 2: the basis is not m distinct columns
}

// the region's preconditions on this tableau: every basic column an exact unit
// vector (1.0 in its row, +0 elsewhere) with a zero reduced cost; ok[0] = 0
// on the first violation (this rank's rows: the host combines the ranks').
// Grid: (rows / 64, basic variables / 256).
__global__ __launch_bounds__(256) void k_region_check(const double *T, Geo g, const int64_t *basis,
                                                       const int32_t *inv, int *ok) {
    const int64_t r = (int64_t)blockIdx.y * 256 + threadIdx.x;     // basic variable of row r
    if (r >= g.m) return;
    const int64_t p = inv[basis[r]];
    bool good = true;
    const int64_t i0 = (int64_t)blockIdx.x * 64, i1 = std::min<int64_t>(i0 + 64, g.nloc + g.nobj);
    for (int64_t i = i0; i < i1; i++) {
        const double v = T[i * g.ld + p];
        // bit for bit (+0, not -0: k_move_cols writes a leaving column's base data as +0 / 1.0)
        const uint64_t want = g.row0 + i == r ? 0x3ff0000000000000ull : 0ull;
        good = good && (i < g.nloc ? (uint64_t)__double_as_longlong(v) == want : v == 0.0);
    }
    if (!good) ok[0] = 0;
}

int launch_region_build(const Launch &L, const Geo &g, DevState *st, const int64_t *basis, const int32_t *inv,
                        int32_t *mark, int32_t *live, int64_t *bcol0, int64_t nlive, int32_t *tlive) {
    if (g.ld % 64) return -1;
    hipLaunchKernelGGL(k_region_build, dim3(1), dim3(1024), 0, (hipStream_t)L.stream, st, basis, inv, g.m, g.ncols,
                       g.ld, mark, live, bcol0, nlive, tlive);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_region_check(const Launch &L, const Geo &g, const int64_t *basis, const int32_t *inv, int *ok) {
    const int64_t rows = g.nloc + g.nobj;
    hipLaunchKernelGGL(k_region_check, dim3((unsigned)((rows + 63) / 64), (unsigned)((g.m + 255) / 256)), dim3(256), 0,
                       (hipStream_t)L.stream, g.T, g, basis, inv, ok);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_pivot_block(const Launch &L, const Geo &g, int rule, DevState *st, int s0, int q0, int n, Cand *part,
                       int ncand, const Cand *cin, int ncin, const double *Cs0, double *Cs1, const Defer &D,
                       void *rec, uint32_t tag0, int nwg, int cw, int rw, int ks, size_t lds, uint32_t cl,
                       const Xch *X, uint32_t xtag0, const RegionArgs *R) {
    if (n < 1 || q0 < 0 || q0 + n > ks || ks > 96 || nwg < 1 || nwg > kMaxWG || ncand < nwg || cl < 1) return -1;
    if (X && (X->world < 1 || X->world > 64 || X->nblk < nwg || X->nx < 1)) return -1;
    if (!R && ((int64_t)nwg * cw < ((g.ncols + 1) & ~(int64_t)1) || (int64_t)nwg * rw < g.nloc)) return -1;
    if (R && (g.nobj != 1 || (int64_t)nwg * cw < R->nlive || (int64_t)nwg * rw < g.nloc ||
              (int64_t)nwg * R->nsp < ks || R->cwx != cw + R->nsp + 1 || R->cwx > kNT || !R->live || !R->bcol0))
        return -1;
    if (g.nobj != 1 && g.nobj != 2) return -1;
    BlockArgs a;
    a.T = g.T;
    a.g = g;
    a.st = st;
    a.s0 = s0;
    a.q0 = q0;
    a.n = n;
    a.part = part;
    a.ncand = ncand;
    a.cin = cin;
    a.ncin = ncin;
    a.X = X ? *X : Xch{};
    a.xtag0 = xtag0;
    a.Cs0 = Cs0;
    a.Cs1 = Cs1;
    a.D = D;
    a.rec = (u4 *)rec;
    a.tag0 = tag0;
    a.nwg = nwg;
    a.cw = cw;
    a.rw = rw;
    a.ks = ks;
    a.cl = cl;
    a.live = R ? R->live : nullptr;
    a.nlive = R ? R->nlive : 0;
    a.bcol0 = R ? R->bcol0 : nullptr;
    a.nsp = R ? R->nsp : 0;
    a.cwx = R ? R->cwx : cw;
    hipStream_t stream = (hipStream_t)L.stream;
    // one XCD for grids that fit its CUs (one rank; LPG_PIVOT_XCD1=0 spreads them)
    static const bool xcd1_on = [] {
        const char *e = getenv("LPG_PIVOT_XCD1");
        return !(e && e[0] == '0');
    }();

    // the dynamic-LDS limit is a per-device attribute: set once per device
    // (bit `dev` of a per-kernel mask; ranks as threads may race to set it,
    // which is harmless)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    static std::atomic<int> cus_of[64];   // CUs per device, read once (0: not yet)
    int cus = cus_of[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = -1;
        cus_of[dev].store(cus, std::memory_order_relaxed);
    }
    a.xcd1 = (xcd1_on && !X && cus >= 8 * 32 && nwg <= cus / 8) ? 1 : 0;
    const unsigned grid = (unsigned)(a.xcd1 ? 8 * nwg : nwg);
#define LPG_PB(RU, NO, M, KB, RG)                                                                       \
    do {                                                                                                \
        static std::atomic<unsigned long long> attr{0};                                                 \
        if (!((attr.load(std::memory_order_acquire) >> dev) & 1ull)) {                                   \
            if (hipFuncSetAttribute((const void *)k_pivot_block<RU, NO, M, KB, RG>,                     \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds) != hipSuccess) \
                return -1;                                                                              \
            attr.fetch_or(1ull << dev, std::memory_order_acq_rel);                                      \
        }                                                                                               \
        hipLaunchKernelGGL((k_pivot_block<RU, NO, M, KB, RG>), dim3(grid), dim3(kNT), lds, stream, a); \
    } while (0)
#define LPG_PB_K(RU, NO, M, RG)                 \
    do {                                        \
        if (ks > 64) LPG_PB(RU, NO, M, 96, RG); \
        else LPG_PB(RU, NO, M, 64, RG);         \
    } while (0)
#define LPG_PB_M(RU, NO)                      \
    do {                                      \
        if (X) LPG_PB_K(RU, NO, true, false); \
        else LPG_PB_K(RU, NO, false, false);  \
    } while (0)
    if (R && X) {              // region mode on a rank of a row partition (D.rqg: global pivot rows)
        if (!D.rqg) return -1;
        if (rule == RULE_BLAND) LPG_PB_K(RULE_BLAND, 1, true, true);
        else LPG_PB_K(RULE_DANTZIG, 1, true, true);
    } else if (R) {
        if (rule == RULE_BLAND) LPG_PB_K(RULE_BLAND, 1, false, true);
        else LPG_PB_K(RULE_DANTZIG, 1, false, true);
    } else if (rule == RULE_BLAND) {
        if (g.nobj == 2) LPG_PB_M(RULE_BLAND, 2);
        else LPG_PB_M(RULE_BLAND, 1);
    } else {
        if (g.nobj == 2) LPG_PB_M(RULE_DANTZIG, 2);
        else LPG_PB_M(RULE_DANTZIG, 1);
    }
#undef LPG_PB_M
#undef LPG_PB_K
#undef LPG_PB
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lpg
