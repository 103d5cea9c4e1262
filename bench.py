"""Benchmark: simplex pivots/s and HBM-roofline fraction of the gfx950 engine.

Workload (BASELINE.json `metric`, config 3): dense synthetic LP m=16384,
n=32768 (tableau 16385 x 49153 fp64 = 6.44 GB), Dantzig pricing, generated on
the device (splitmix64, seed 20220518). Each simplex pivot is price (argmin
over the reduced-cost row) -> ratio test (min over the entering column) ->
Gauss-Jordan rank-1 update of the whole tableau. The update is deferred:
prep / select evaluate the pending chain for the entries they need and
k_flushw applies each block of K pivots to the constraint rows in one pass,
bitwise identical to K eager updates (LPG_DEFER; default K = 96 in region
mode from 2 GB on one rank / 1 GB per rank of a partition -- config 3 --, 96
from 16 GB with the two-kernel pair -- config 4 --, 64 from 200 MB, else 32;
include/lpg.h).

A "step" is one such block: K pivots and the one pass over the tableau that
applies them (with --defer 0, eager updates, a step is one pivot). `value` is
pivots/s = steps x K / time; `ms_per_step` is the time of one block. Warm-up
steps are whole blocks too, so every timed pass applies exactly K pending
pivots (the kernel and K named in `roofline`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

With N > 1 the tableau is row-block partitioned over N processes (one per
GPU; strong scaling: the LP is the same for every N). Per pivot the owner of
the pivot row stores it, with the ratio candidates, into every peer's
IPC-mapped exchange buffer (the owner push, default); `--exchange rccl`
allgathers the candidates and allreduces the pivot row over RCCL instead, and
the bench falls back to those collectives (or to gloo host collectives when
RCCL cannot start) if the push cannot attach or fails in the warm-up.

Rank 0 prints ONE JSON line. `roofline.achieved` = algorithmic bytes of one
launch of the dominant kernel on rank 0 (k_flushw: 16 B x local constraint
rows x columns not skipped, one read + one write of every entry the block
changes; eager k_update: the same over all rows for one pivot) / its mean
device time, timed with HIP events around that kernel alone on the engine's
own stream over the timed region. `cpu_baseline` =
the CPU oracle (oracle/liblpo.so, same pivot rules, OpenMP) on the same LP,
rank 0 at N=1 only, for a bounded number of pivots; its pivot sequence is
compared with the GPU's.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def spawn_ranks_if_needed() -> None:
    """`python3 bench.py --gpus N` with N > 1 and no WORLD_SIZE in the
    environment: start N rank processes of this same command (RANK /
    LOCAL_RANK / WORLD_SIZE set, rendezvous through a file in a fresh
    temporary directory, so no port can collide), relay rank 0's one JSON line
    on stdout and exit with the first failing rank's code. Runs before this
    process imports the engine, torch or anything that could touch the GPU
    (VERDICT r5 missing #3); the torch.distributed.run launch is unchanged."""
    if "WORLD_SIZE" in os.environ:
        return
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args()[0].gpus
    if n <= 1:
        return
    import ctypes
    import signal
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp(prefix="lpg_bench_")
    out_path = os.path.join(tmp, "rank0.out")
    procs = []

    def die_with_parent():            # in the child, before exec: no rank outlives this launcher
        try:
            ctypes.CDLL(None).prctl(1, signal.SIGKILL)    # PR_SET_PDEATHSIG
        except Exception:
            pass

    def stop(signum, frame):          # a time limit on this launcher ends the ranks too
        for p in procs:
            if p.poll() is None:
                p.kill()
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    with open(out_path, "wb") as out0:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", LPG_BENCH_INIT_FILE=os.path.join(tmp, "rendezvous"))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=out0 if r == 0 else subprocess.DEVNULL, preexec_fn=die_with_parent))
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:                      # one rank failed: the others would wait on it in a collective
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    with open(out_path, "rb") as f:
        sys.stdout.buffer.write(f.read())
    sys.stdout.flush()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    raise SystemExit(rc)


if __name__ == "__main__":
    spawn_ranks_if_needed()

import linearprogramming_amd as lpg   # first: binds the process to the system ROCm runtime (_lib.bind_runtime)
import torch  # noqa: E402  (torch.distributed gloo plumbing only; reuses that runtime)
import torch.distributed as dist  # noqa: E402
from linearprogramming_amd import _lib as lpg_lib  # noqa: E402
from linearprogramming_amd._stamp import source_stamp  # noqa: E402

METRIC = "Simplex pivots/sec + HBM GB/s fraction, dense m=16384×n=32768 fp64, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# dense f64 matrix-core peak of MI355X (AMD's published FP64 matrix figure, no
# sparsity; 256 CUs x 4 SIMDs x 32 flop/clk x 2.4 GHz); the box's f64 MFMA pipe
# measures 73-75 TFLOP/s in isolation (profiles/r01_mfma_rate.log)
MFMA_F64_PEAK_TFS = 78.6


def roofline_bound(touched, defer, upd_ms):
    """The block pass against both rooflines: HBM (16 B per live element,
    touched = bytes per launch) and the f64 matrix cores (2 flops per live
    element per pending pivot). `bound` is the one whose ideal time is longer
    (HBM below ~78 pending pivots, the matrix cores above: 16 x 78.6 / 8000 x 8
    ~ 77 flop per byte pair); `achieved` / `frac` are that roofline's."""
    flops = touched / 16.0 * 2.0 * max(defer, 1)
    t = upd_ms * 1e-3 if upd_ms > 0 else float("inf")
    hbm = {"achieved": touched / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s"}
    hbm["frac"] = hbm["achieved"] / HBM_PEAK_GBS
    mf = {"achieved": flops / t / 1e12, "peak": MFMA_F64_PEAK_TFS, "unit": "TFLOP/s",
          "algorithmic_flops_per_launch": flops}
    mf["frac"] = mf["achieved"] / MFMA_F64_PEAK_TFS
    t_hbm, t_mf = touched / (HBM_PEAK_GBS * 1e9), flops / (MFMA_F64_PEAK_TFS * 1e12)
    main, bound = (mf, "mfma") if t_mf > t_hbm else (hbm, "hbm")
    return {"bound": bound, "achieved": main["achieved"], "peak": main["peak"], "unit": main["unit"],
            "frac": main["frac"], "hbm": hbm, "mfma": mf}
SEED = 20220518
CONFIGS = {
    2: dict(m=1024, n=2048, name="BASELINE config 2: random dense LP m=1024 n=2048 fp64"),
    3: dict(m=16384, n=32768, name="BASELINE config 3: random dense LP m=16384 n=32768 fp64"),
    4: dict(m=65536, n=131072, name="BASELINE config 4: random dense LP m=65536 n=131072 fp64"),
    5: dict(m=8192, n=8192, name="BASELINE config 5: two-phase (artificials) on a KM-style degenerate LP m=8192 n=8192, "
                                 "Bland rule, pivot cap 20000"),
}


def pmc_traffic(a, kname, defer, m, n, world, stamp):
    """The PMC traffic of profiles/pmc_config{C}.json, or None and the reason:
    the file must carry this build's source stamp and this run's kernel,
    pending-pivot count and LP shape (a stand-in
    --shape run or a changed pass never inherits a stale figure)."""
    pmc = os.path.join(ROOT, "profiles", f"pmc_config{a.config}.json")
    if not defer:
        return None, "eager updates: no PMC file"
    if world != 1 or a.shape:
        return None, "PMC files are captured for the single-GPU BASELINE configs only"
    if not os.path.exists(pmc):
        return None, f"no {os.path.relpath(pmc, ROOT)}"
    with open(pmc) as f:
        p = json.load(f)
    want = {"kernel": kname, "pending_pivots": defer, "m": m, "n": n, "source_stamp": stamp}
    diff = {k: (p.get(k), v) for k, v in want.items() if p.get(k) != v}
    if diff:
        return None, (f"{os.path.relpath(pmc, ROOT)} does not match this run (field: file vs run): "
                      + ", ".join(f"{k}: {x!r} vs {y!r}" for k, (x, y) in diff.items()))
    return p, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)    # deferred blocks (K pivots each) timed
    ap.add_argument("--warmup", type=int, default=2)    # blocks before the timed region (page-in, graph build)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--cpu-1core-seconds", type=float, default=6.0, help="1-core CPU baseline time budget")
    ap.add_argument("--variant", type=int, default=None, help="eager update-kernel form (LPG_UPDATE_VARIANT 0|1)")
    ap.add_argument("--no-skip", action="store_true", help="update every column (disable column skipping)")
    ap.add_argument("--force-rccl", action="store_true", help="attach a 1-rank RCCL communicator at N=1 (times the exchange)")
    ap.add_argument("--exchange", choices=["push", "rccl"], default=os.environ.get("LPG_EXCHANGE", "push"),
                    help="per-pivot exchange with N>1 (or --force-*): owner push through IPC-mapped buffers "
                         "(default), or RCCL allreduce + allgather")
    ap.add_argument("--host-comm", action="store_true",
                    help="N>1: set up through gloo host collectives instead of RCCL (ranks sharing one GPU, "
                         "which RCCL refuses)")
    ap.add_argument("--force-push", action="store_true", help="N=1: attach the owner-push exchange to a 1-rank "
                                                              "host communicator (times the push kernels)")
    ap.add_argument("--defer", type=int, default=None, help="pivots per deferred block (LPG_DEFER; 0 = eager updates)")
    ap.add_argument("--shape", default=None,
                    help="M,N: a labelled stand-in LP of M rows and N structural columns in place of --config's "
                         "(e.g. one rank's row block of config 3 at P ranks: M = 16384/P, N = 49152 - M; never the "
                         "headline line)")
    return ap.parse_args()


def cpu_baseline(m, n, gpu_log, budget_s, budget_1core_s):
    """Oracle leg: same LP, same rules, OpenMP on the host cores (rank 0, N=1
    only), then the same oracle on ONE core for a few more pivots of the same
    solve (BASELINE.md CPU-baseline plan)."""
    from oracle.lpo import GEN_DENSE, RULE_DANTZIG, Oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    o = Oracle(m, n + m + 1, nthreads=threads)
    o.generate(n, SEED, GEN_DENSE)
    o.solve(1, RULE_DANTZIG)                       # first pivot untimed (page faults)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s and done < 400:
        o.solve(1, RULE_DANTZIG)
        done += 1
    dt = time.perf_counter() - t0
    k, r = o.get_log()
    n_cmp = min(len(k), len(gpu_log[0]))
    same = bool((k[:n_cmp] == gpu_log[0][:n_cmp]).all() and (r[:n_cmp] == gpu_log[1][:n_cmp]).all())
    one = None
    if budget_1core_s > 0:
        o.set_threads(1)
        t1 = time.perf_counter()
        d1 = 0
        while d1 < 2 or (time.perf_counter() - t1 < budget_1core_s and d1 < 50):
            o.solve(1, RULE_DANTZIG)
            d1 += 1
        s1 = time.perf_counter() - t1
        one = {"value": d1 / s1, "unit": "pivots/s", "cores": 1, "kind": "port", "pivots": d1, "seconds": s1,
               "sample": f"pivots {done + 2}..{done + 1 + d1} of the same solve, oracle/liblpo.so on 1 thread"}
    o.close()
    return {"value": done / dt, "unit": "pivots/s", "cores": threads, "kind": "port",
            "sample": f"{done} timed pivots (after 1 untimed) of the same {m}x{n} LP, oracle/liblpo.so "
                      f"(C fp64, OpenMP {threads} threads)",
            "seconds": dt, "single_core": one}, {"pivots_compared": int(n_cmp), "identical_pivot_sequence": same}


def trajectory_parity(a, eng, world, rank):
    """The whole run -- warm-up and timed pivots -- against the oracle's pinned
    trajectory of config 3 (tests/golden/config3_2400.json, VERDICT r5 missing
    #2): the (entering, leaving) log pivot by pivot, and at the run's last
    pivot (a multiple of 96 up to 2,400: the default and the driver's forms
    both end on one) the objective's bits, the basis and the digests of column
    0, the objective row and 16 fixed rows (rows at N = 1 only). Read after
    the timed region. None for other configs / shapes."""
    if a.config != 3 or a.shape:
        return None
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    try:
        import trajectory as T
    finally:
        sys.path.pop(0)
    if not os.path.exists(T.FIXTURE):
        return {"error": "tests/golden/config3_2400.json missing"}
    import numpy as np
    fix = T.load()
    k, r = eng.get_log()
    res = eng.sync()
    snaps = {}
    key = str(res.pivots)
    if key in fix["checkpoints"]:
        if world == 1:
            rows = np.concatenate([eng.get_rows(i, 1) for i in T.ROWS])
            snaps[res.pivots] = T.snapshot(res.objective, eng.get_basis(), eng.get_column0(),
                                           eng.get_rows(T.M, 1)[0], rows)
        else:                                        # the replicated parts only; rows live on their owners
            snaps[res.pivots] = {"objective_hex": float(res.objective).hex(), "basis": T.digest(eng.get_basis())}
    cmp = T.compare(fix, k, r, snaps)
    cmp.update({"fixture": "tests/golden/config3_2400.json (oracle/liblpo.so, tests/golden/make_config3_golden.py)",
                "pivots_run": int(res.pivots),
                "covers_timed_region": bool(cmp["pivots_compared"] >= res.pivots and cmp["pivots_compared"] > 0),
                "rows_checked": world == 1 and bool(snaps)})
    if world > 1:
        cmp["note"] = "N > 1: log, objective and basis (replicated) checked; row digests at N = 1"
    return cmp if rank == 0 else None


def host_ops(world):
    """gloo host collectives for lpg_comm_init_host (setup and bootstrap only once the push exchange is attached)."""
    import numpy as np

    def allgather(b: bytes) -> bytes:
        if world == 1:
            return b
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.numpy()) for o in outs)

    def allreduce(arr: "np.ndarray") -> "np.ndarray":
        if world == 1:
            return arr
        t = torch.from_numpy(arr)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    return allgather, allreduce


def config5(a):
    """Config 5: the whole two-phase solve (phase I, artificial clean-up, phase II) under Bland."""
    cfg = CONFIGS[5]
    m, n, cap = cfg["m"], cfg["n"], 20000
    art_first = 1 + n + (m + 1) // 2
    eng = lpg.Engine(m, n + m + 1)
    eng.generate(n, SEED, lpg.GEN_ARTIFICIAL)
    eng.reserve_log(cap + 8)
    eng.set_timing(True)
    eng.get_timing()
    eng.device_sync()
    t0 = time.perf_counter()
    res = eng.solve_two_phase(art_first, None, cap, lpg.RULE_BLAND)
    eng.device_sync()
    elapsed = time.perf_counter() - t0
    timing = eng.get_timing()
    upd_ms = timing.update_ms / max(timing.update_count, 1)
    touched = timing.update_bytes / max(timing.update_count, 1)
    achieved = touched / (upd_ms * 1e-3) / 1e9 if upd_ms > 0 else 0.0
    line = {"metric": METRIC + " [config 5 variant: pivots/s of a full two-phase solve]", "value": res.pivots / elapsed,
            "unit": "pivots/s", "n_gpus": 1, "steps": res.pivots, "warmup": 0,
            "ms_per_step": elapsed / max(res.pivots, 1) * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": f"synthetic KM-style degenerate LP with equality rows (splitmix64 seed {SEED}), generated on device",
            "config": {"workload": cfg["name"], "m": m, "n": n, "rule": "bland", "art_first": art_first},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": ("lpg::" + ("k_flushw" if lpg.flush_kernel_for(eng.info.defer_k) == "w" else "k_flushm"))
                                   if eng.info.defer_k else "lpg::k_update",
                         "launches_timed": timing.update_count,
                         "algorithmic_bytes_per_launch": touched,
                         "full_tableau_bytes_per_launch": eng.info.bytes_per_pivot, "update_ms_mean": upd_ms},
            "status": lpg.STATUS_NAMES.get(res.status, res.status), "pivots_total": res.pivots,
            "objective": res.objective, "seconds": elapsed, "build_stamp": lpg_lib.build_stamp}
    # the whole solve against the oracle's (tests/golden/config5_solve.json), read after the timed region
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    try:
        import make_config5_golden as G5
        import trajectory as T
    finally:
        sys.path.pop(0)
    if os.path.exists(G5.FIXTURE):
        fix = T.load(G5.FIXTURE)
        ek, er = eng.get_log()
        line["parity_fixture"] = {
            "fixture": "tests/golden/config5_solve.json (oracle/liblpo.so, tests/golden/make_config5_golden.py)",
            "pivots_compared": int(min(len(ek), len(fix["log_k"]))),
            "identical_log": ek.tolist() == fix["log_k"] and er.tolist() == fix["log_r"],
            "status": lpg.STATUS_NAMES.get(res.status) == fix["status"],
            "objective_bits": float(res.objective).hex() == fix["objective_hex"],
            "basis": T.digest(eng.get_basis()) == fix["basis"],
            "rows": [T.digest(eng.get_rows(i, 1)[0]) for i in fix["rows"]] == fix["row_digests"]}
        line["parity_fixture"]["ok"] = all(v for k, v in line["parity_fixture"].items()
                                           if k not in ("fixture", "pivots_compared"))
    if not a.no_cpu:
        from oracle.lpo import Oracle
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        o = Oracle(m, n + m + 1, nthreads=threads)
        o.generate(n, SEED, 2)
        k_cpu = 400
        t0 = time.perf_counter()
        ro = o.solve_two_phase(art_first, None, k_cpu, lpg.RULE_BLAND)
        dt = time.perf_counter() - t0
        ok, orr = o.get_log()
        ek, er = eng.get_log()
        ncmp = min(len(ok), len(ek))
        line["cpu_baseline"] = {"value": ro.pivots / dt, "unit": "pivots/s", "cores": threads, "kind": "port",
                                "sample": f"first {ro.pivots} pivots of the same two-phase solve (oracle/liblpo.so, "
                                          f"OpenMP {threads} threads)", "seconds": dt}
        line["parity"] = {"pivots_compared": int(ncmp),
                          "identical_pivot_sequence": bool((ok[:ncmp] == ek[:ncmp]).all() and
                                                           (orr[:ncmp] == er[:ncmp]).all())}
    print(json.dumps(line), flush=True)


def main():
    a = parse()
    if a.defer is not None:
        os.environ["LPG_DEFER"] = str(a.defer)
    if a.config == 5:
        if a.gpus != 1:
            raise SystemExit("config 5 (two-phase) is single-GPU")
        if a.no_skip:
            os.environ["LPG_NO_SKIP"] = "1"
        return config5(a)
    if a.variant is not None:
        os.environ["LPG_UPDATE_VARIANT"] = str(a.variant)
    if a.no_skip:
        os.environ["LPG_NO_SKIP"] = "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    result_fd = 1
    if world > 1:
        # gloo (and RCCL) print connection banners on fd 1; stdout carries exactly
        # one JSON line, so everything else goes to stderr and the line is
        # written to the saved descriptor
        sys.stdout.flush()
        result_fd = os.dup(1)
        os.dup2(2, 1)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        init = os.environ.get("LPG_BENCH_INIT_FILE")      # the self-spawned ranks (spawn_ranks_if_needed)
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                init_method=f"file://{init}" if init else None)
    cfg = CONFIGS[a.config]
    m, n = cfg["m"], cfg["n"]
    if a.shape:                                        # a stand-in shape, labelled as such in the line
        m, n = (int(x) for x in a.shape.split(","))
        cfg = dict(m=m, n=n, name=f"STAND-IN (not a BASELINE config): dense LP m={m} n={n} fp64, generated like "
                                  f"config {a.config}")
    ndev = lpg.device_count()
    if ndev < 1:
        raise SystemExit("no GPU visible")
    dev = local % ndev

    host_comm = [a.host_comm]

    def make_engine(push):
        e = lpg.Engine(m, n + m + 1, device=dev, world=world, rank=rank)
        if world > 1 and not host_comm[0]:
            # RCCL for setup (and the collectives); if its init fails on any rank
            # (an error, not a hang), every rank rebuilds on the gloo host collectives
            ok = True
            try:
                uid = [lpg.Engine.rccl_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                e.comm_init_rccl(uid[0])
            except lpg.LPGError as ex:
                print(f"bench: rank {rank}: RCCL communicator failed ({ex}); using the host collectives",
                      file=sys.stderr)
                ok = False
            t = torch.tensor([1 if ok else 0], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            if not t.item():
                e.close()
                host_comm[0] = True
                return make_engine(push)
        elif world > 1 or a.force_push:
            e.comm_init_host(*host_ops(world))
        elif a.force_rccl:
            e.comm_init_rccl(lpg.Engine.rccl_unique_id())
        if push:                                       # every rank attaches it, or none does
            def agree(ok):
                if world == 1:
                    return ok
                t = torch.tensor([1 if ok else 0], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
                return bool(t.item())
            try:
                h = e.push_handle()
            except lpg.LPGError as ex:
                print(f"bench: no owner-push buffer ({ex})", file=sys.stderr)
                h = None
            hs = [h]
            if world > 1:
                hs = [None] * world
                dist.all_gather_object(hs, h)
            ok = agree(all(x is not None for x in hs))
            if ok:
                try:
                    e.comm_init_push(hs)
                except lpg.LPGError as ex:
                    print(f"bench: owner-push attach failed ({ex})", file=sys.stderr)
                    ok = False
                ok = agree(ok)
            if not ok:
                e.close()
                return make_engine(False)
        e.generate(n, SEED, lpg.GEN_DENSE)
        return e

    use_push = (world > 1 or a.force_push) and a.exchange == "push"
    eng = make_engine(use_push)
    use_push = use_push and eng.info.exchange > 0
    K = eng.info.defer_k or 1                           # pivots per step (one block; eager: one pivot)
    warm, timed = a.warmup * K, a.steps * K
    # the push exchange is proven on untimed pivots before the timed region:
    # the warm-up, or one block of its own when --warmup 0
    warm_run = warm if (warm > 0 or not use_push) else K
    eng.reserve_log(warm_run + timed + 8)
    failed = 0
    try:
        eng.enqueue(warm_run, lpg.RULE_DANTZIG)
        before = eng.sync().pivots
    except lpg.LPGError as ex:                          # the push exchange did not work here: collectives instead
        if not use_push:
            raise
        print(f"bench: owner-push exchange failed in warm-up ({ex}); using the collectives", file=sys.stderr)
        failed = 1
    if world > 1:
        if not failed:                                 # every rank must have taken the same pivots (replicated log)
            import hashlib
            lk, lr = eng.get_log()
            hs = [None] * world
            dist.all_gather_object(hs, hashlib.sha1(lk.tobytes() + lr.tobytes()).hexdigest())
            if len(set(hs)) != 1:
                print("bench: ranks diverged in warm-up; using the collectives", file=sys.stderr)
                failed = 1
        ft = torch.tensor([failed], dtype=torch.int64)
        dist.all_reduce(ft, op=dist.ReduceOp.MAX)
        failed = int(ft.item())
    if failed:
        eng.close()
        use_push = False
        eng = make_engine(False)
        eng.reserve_log(warm + timed + 8)
        eng.enqueue(warm, lpg.RULE_DANTZIG)
        before = eng.sync().pivots

    # HIP events around the block pass inside the timed region (the roofline
    # numerator's kernel time). For config 2 the events would forbid the
    # hipGraph replay that hides its launch overhead, so config 2 times the
    # pass in an event-instrumented run of 3 blocks before the timed region.
    live_events = a.config != 2
    if not live_events:
        eng.set_timing(True)
        eng.get_timing()
        eng.enqueue(3 * K, lpg.RULE_DANTZIG)
        eng.sync()
        timing = eng.get_timing()
        eng.set_timing(False)
        eng.enqueue(4 * K, lpg.RULE_DANTZIG)           # builds the replayed hipGraph outside the timed region
        before = eng.sync().pivots
    eng.set_timing(live_events)
    if live_events:
        eng.get_timing()                               # reset sums
    eng.prepare(lpg.RULE_DANTZIG)                      # the replayed graph is built here, not in the timed region
    if world > 1:
        dist.barrier()
    eng.device_sync()
    t0 = time.perf_counter()
    eng.enqueue(timed, lpg.RULE_DANTZIG)
    res = eng.sync()
    eng.device_sync()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if live_events:
        timing = eng.get_timing()
    info = eng.info
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    done = res.pivots - before          # pivots really applied (an LP that finishes early turns the rest into no-ops)
    if world > 1:
        dd = torch.tensor([done], dtype=torch.int64)
        dist.all_reduce(dd, op=dist.ReduceOp.MIN)
        done = int(dd.item())
    upd_ms = timing.update_ms / max(timing.update_count, 1)
    # bytes the block pass actually read + wrote (columns whose K pending P
    # entries are all zero are not counted, SURVEY.md §8(d) restated per block
    # in DESIGN.md §6); the events bracket the pass alone, so this agrees with
    # rocprofv3's average for that kernel
    touched = timing.update_bytes / max(timing.update_count, 1)
    defer = info.defer_k
    achieved = touched / (upd_ms * 1e-3) / 1e9 if upd_ms > 0 else 0.0
    kname = ("k_flushw" if lpg.flush_kernel_for(defer) == "w" else "k_flushm") if defer else "k_update"
    ms_block = elapsed * 1e3 / max(done, 1) * K
    roof = roofline_bound(touched, defer, upd_ms)
    roof.update({"traffic": None,
            "kernel": f"lpg::{kname}" + (f" (Gauss-Jordan block pass, {defer} pending pivots per launch; HIP events "
                                         f"around this kernel alone)" if defer else " (Gauss-Jordan rank-1)"),
            "pending_pivots_per_launch": defer or 1,
            "launches_timed": timing.update_count,
            "algorithmic_bytes_per_launch": touched,
            "full_tableau_bytes_per_launch": info.bytes_per_pivot,
            "column_skipping": not a.no_skip,
            "update_ms_mean": upd_ms})
    if defer and live_events:
        # per-block ceiling: the pass at the HBM spec peak plus the measured rest of the block (pivot kernels,
        # column trade, pivot-row rewrite, launch gaps), i.e. what this design reaches with a perfect pass
        other_ms = ms_block - upd_ms
        pass_ideal_ms = max(touched / (HBM_PEAK_GBS * 1e9), roof["mfma"]["algorithmic_flops_per_launch"] /
                            (MFMA_F64_PEAK_TFS * 1e12)) * 1e3
        ceil_ms = pass_ideal_ms + other_ms
        roof.update({"ms_per_block": ms_block, "other_ms_per_block": other_ms, "pass_ideal_ms": pass_ideal_ms,
                     "block_ceiling_ms": ceil_ms, "block_ceiling_pivots_per_s": defer / (ceil_ms * 1e-3),
                     "pass_only_ceiling_pivots_per_s": defer / (pass_ideal_ms * 1e-3)})
    stamp = source_stamp()
    roof["source_stamp"] = stamp
    p, why = pmc_traffic(a, kname, defer, m, n, world, stamp)
    if p is not None:
        roof["traffic"] = p.get("hbm_bytes_per_launch")
        roof["traffic_source"] = (f"profiles/pmc_config{a.config}.json: separate rocprofv3 --pmc FETCH_SIZE / "
                                  f"WRITE_SIZE passes of this bench at source stamp {stamp} ({p.get('source')})")
    else:
        roof["traffic_note"] = why
    line = {
        "metric": METRIC,
        "value": done / elapsed,
        "unit": "pivots/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_block,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic dense LP generated on device (splitmix64 seed {SEED}): A_ij=u, b_i=n/8(1+u), c_j=1+u",
        "config": {"workload": cfg["name"], "m": m, "n": n, "tableau": [m + 1, n + m + 1],
                   "tableau_GB": (m + 1) * (n + m + 1) * 8 / 1e9, "rule": "dantzig",
                   "step": (f"one deferred block: {K} pivots + one block pass" if defer else "one pivot (eager)"),
                   "pivots_timed": done,
                   "parallelism": f"row-block x{world}" + (
                       (" (owner push per pivot: pivot row and candidates stored into IPC-mapped peer buffers"
                        + (", uncached" if info.exchange == 2 else "") + ")"
                        if use_push else (" (host gloo allgather + allreduce per pivot)" if host_comm[0]
                                          else " (RCCL allgather + allreduce per pivot)"))
                       if world > 1 or a.force_rccl or a.force_push else ""),
                   "update": (f"deferred blocks of {defer} pivots (one k_flush pass per block)" if defer
                              else "eager rank-1 update per pivot"),
                   "pivot_loop": (f"k_pivot_block: one persistent launch per block, {info.pivot_wg} workgroups"
                                  if info.pivot_wg else "k_prep_d + k_select_d per pivot"),
                   "update_variant": int(os.environ.get("LPG_UPDATE_VARIANT", "-1"))},
        "roofline": roof,
        "status": lpg.STATUS_NAMES.get(res.status, res.status),
        "pivots_total": res.pivots,
        "objective": res.objective,
    }
    line["build_stamp"] = lpg_lib.build_stamp
    traj = trajectory_parity(a, eng, world, rank)
    if traj is not None:
        line["parity_trajectory"] = traj
    if world == 1 and rank == 0 and not a.no_cpu:
        log = eng.get_log()
        eng.close()
        cb, parity = cpu_baseline(m, n, log, a.cpu_seconds, a.cpu_1core_seconds)
        line["cpu_baseline"] = cb
        line["parity"] = parity
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        if result_fd == 1:
            print(json.dumps(line), flush=True)
        else:
            os.write(result_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
