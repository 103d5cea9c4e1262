"""host/lpgcli: the plain-C host (north star: "the host stays plain C") on
the device, single rank and row-partitioned over P processes (--gpus P).

The reference host is one interactive process (Source/main.c:4-45); lpgcli is
its non-interactive counterpart (SURVEY.md §5 config / flags). --gpus P forks
P ranks before any HIP call; the parent relays the host-staged collectives
over socketpairs and never touches the GPU. On the one-GPU box all ranks
share the card (rank r -> device r mod 1), the layout the row partition
tests use; the 8-GPU node gives each its own.
"""
from __future__ import annotations

import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from oracle.lpo import Oracle

CLI = os.path.join(ROOT, "host", "lpgcli")
needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="host/lpgcli not built")


def _fnv(k, r):
    h = 1469598103934665603
    for a, b in zip(k.tolist(), r.tolist()):
        for byte in np.array([a, b], dtype=np.int64).tobytes():
            h = ((h ^ byte) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def _cli(args, env=None, timeout=120, ack_shared=True):
    # `--gpus P` forks P ranks onto the test box's ONE GPU: acknowledge that for
    # the owner push (refused at attach otherwise, lpg_ctx.hip push_shares_device)
    base = {k: v for k, v in os.environ.items() if k not in ("LPG_PUSH_SHARED_DEVICE", "LPG_PUSH_SHARED_QUEUES")}
    if ack_shared:
        base["LPG_PUSH_SHARED_DEVICE"] = "1"
    p = subprocess.run([CLI] + args, capture_output=True, text=True, timeout=timeout, env={**base, **(env or {})})
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p, lines


@needs_cli
def test_gpus_without_a_device_fails_cleanly():
    """Every rank fails (no GPU in the build container, or a bad device): the
    hub sees them all hang up, nothing blocks, the exit status is non-zero."""
    if os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible: the GPU tests below cover --gpus")
    p, lines = _cli(["--synthetic", "64", "64", "--gpus", "3"], timeout=60)
    assert p.returncode != 0 and not lines
    assert "ERROR: rank" in p.stderr


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("m,n,gpus,extra,env", [
    (1024, 2048, 2, [], {}),                                  # owner push, persistent launch on every rank
    (1024, 2048, 2, [], {"LPG_PERSIST_MR": "0"}),            # owner push, the two-kernel pair
    (1024, 2048, 2, ["--exchange", "host"], {}),             # the host collectives every pivot
    (701, 903, 3, [], {}),                                    # uneven row blocks
    (300, 500, 2, ["--kind", "degenerate", "--rule", "bland", "--pivots", "3000"], {}),   # capped: KM-style
])
def test_gpus_equals_one_rank_and_the_oracle(m, n, gpus, extra, env):
    p1, l1 = _cli(["--synthetic", str(m), str(n)] + extra, env)
    assert p1.returncode == 0, p1.stderr
    one = json.loads(l1[-1])
    pp, lp = _cli(["--synthetic", str(m), str(n), "--gpus", str(gpus)] + extra, env)
    assert pp.returncode == 0, pp.stderr
    assert len(lp) == 1, lp                      # rank 0 alone prints, one JSON line
    dist = json.loads(lp[0])
    assert dist["gpus"] == gpus and dist["status"] == one["status"]
    assert one["status"] in ("OPTIMAL", "UNBOUNDED", "ITER_LIMIT")
    assert dist["pivots"] == one["pivots"] and dist["objective"] == one["objective"]
    assert dist["log_fnv"] == one["log_fnv"]
    assert (dist["exchange"] == 0) if "host" in extra else (dist["exchange"] in (1, 2))
    kind = 1 if "degenerate" in extra else 0
    o = Oracle(m, n + m + 1)
    o.generate(n, 20220518, kind)
    res = o.solve(int(extra[extra.index("--pivots") + 1]) if "--pivots" in extra else 1 << 40, 1 if "bland" in extra else 0)
    assert res.pivots == one["pivots"] and res.objective == one["objective"]
    assert _fnv(*o.get_log()) == one["log_fnv"]


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 3])
def test_gpus_refused_push_falls_back_to_host_collectives(gpus):
    """the README's `lpgcli --synthetic 1024 2048 --gpus 2`
    on a node with fewer GPUs than ranks, without the test override. The
    owner push is refused at attach (ranks share a GPU); every rank must then
    continue on the host collectives (exchange 0), not exit -- also when the
    refusal would be asymmetric (3 ranks)."""
    m, n = 1024, 2048
    p1, l1 = _cli(["--synthetic", str(m), str(n)])
    assert p1.returncode == 0, p1.stderr
    one = json.loads(l1[-1])
    pp, lp = _cli(["--synthetic", str(m), str(n), "--gpus", str(gpus)], ack_shared=False)
    assert pp.returncode == 0, pp.stderr
    assert "using the host collectives" in pp.stderr and "share GPU" in pp.stderr, pp.stderr
    assert len(lp) == 1, lp
    dist = json.loads(lp[0])
    assert dist["exchange"] == 0 and dist["gpus"] == gpus
    assert dist["pivots"] == one["pivots"] and dist["objective"] == one["objective"]
    assert dist["log_fnv"] == one["log_fnv"]


@needs_cli
@pytest.mark.gpu
def test_gpus_config3_pair_path():
    """BASELINE config 3 from plain C over 2 processes on the one GPU with the
    pair (persistent launches of both ranks do not fit one GPU at once),
    200 pivots: the single-rank log, objective and pivot count."""
    args = ["--synthetic", "16384", "32768", "--pivots", "200"]
    p1, l1 = _cli(args, timeout=600)
    assert p1.returncode == 0, p1.stderr
    one = json.loads(l1[-1])
    pp, lp = _cli(args + ["--gpus", "2"], {"LPG_PERSIST_MR": "0"}, timeout=600)
    assert pp.returncode == 0, pp.stderr
    assert len(lp) == 1
    dist = json.loads(lp[0])
    assert dist["pivots"] == one["pivots"] == 200 and dist["objective"] == one["objective"]
    assert dist["log_fnv"] == one["log_fnv"] and dist["pivot_wg"] == 0


DUAL_LP = "OF {\n\tmin:z=2x1+3x2\n}\nST {\n\tx1+x2>=4;\n\tx1+3x2>=6;\n\tx1>=0;\n\tx2>=0\n}\n"


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("m,n", [(400, 300), (2000, 1500)])
def test_cli_dual_synthetic_equals_the_oracle(m, n):
    """lpgcli --synthetic M N --dual: LPG_GEN_DUAL through lpg_solve_dual (the
    deferred blocks at these sizes) from plain C, against the oracle's dual."""
    p, lines = _cli(["--synthetic", str(m), str(n), "--dual", "--seed", "3"])
    assert p.returncode == 0, p.stderr
    got = json.loads(lines[-1])
    assert got["method"] == "dual" and got["defer_k"] > 0
    o = Oracle(m, n + m + 1)
    o.generate(n, 3, 3)
    res = o.solve_dual(1 << 40)
    assert got["status"] == "OPTIMAL" and res.status == 1
    assert got["pivots"] == res.pivots and got["objective"] == res.objective
    assert got["log_fnv"] == _fnv(*o.get_log())


@needs_cli
@pytest.mark.gpu
def test_cli_dual_lp_model(tmp_path):
    """lpgcli --lp MODEL --dual: the dual form from the C front end, solved by the
    dual simplex on the device; the same optimum as the primal two-phase run and
    as the Python front end's dual."""
    from linearprogramming_amd import frontend as F
    f = tmp_path / "dual.txt"
    f.write_text(DUAL_LP)
    p, lines = _cli(["--lp", str(f), "--dual"])
    assert p.returncode == 0, p.stderr
    dual = json.loads(lines[-1])
    p, lines = _cli(["--lp", str(f)])
    primal = json.loads(lines[-1])
    assert dual["status"] == primal["status"] == "OPTIMAL"
    assert abs(dual["z"] - 9.0) < 1e-12 and abs(primal["z"] - 9.0) < 1e-12
    assert {v: dual["variables"][v] for v in ("x1", "x2")} == pytest.approx({"x1": 3.0, "x2": 1.0}, abs=1e-12)
    py = F.solve_text(DUAL_LP, method="dual")
    assert py.status == "OPTIMAL" and py.pivots == dual["pivots"] and py.z == dual["z"]
    # not dual feasible (a positive max-form cost): a clean error line
    g = tmp_path / "notdual.txt"
    g.write_text("OF {\n\tmax:z=x1\n}\nST {\n\tx1<=3;\n\tx1>=0\n}\n")
    p, lines = _cli(["--lp", str(g), "--dual"])
    assert p.returncode != 0 and "dual feasible" in json.loads(lines[-1])["error"]


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("m,n,gpus,extra", [
    (400, 300, 2, ["--dual"]),                                   # the deferred dual over the row partition
    (700, 500, 3, ["--dual", "--exchange", "host"]),
    (257, 300, 2, ["--kind", "artificial"]),                      # config 5's family, two-phase
    (640, 512, 3, ["--kind", "artificial", "--rule", "bland"]),
])
def test_gpus_dual_and_two_phase_equal_one_rank_and_the_oracle(m, n, gpus, extra):
    """--dual and --kind artificial (two-phase) from plain C, one rank and
    --gpus P (round 3: both methods run on a row partition): the same status,
    pivot count, objective and pivot-log hash, and the oracle's."""
    seed = 20220518
    p1, l1 = _cli(["--synthetic", str(m), str(n)] + extra)
    assert p1.returncode == 0, p1.stderr
    one = json.loads(l1[-1])
    pp, lp = _cli(["--synthetic", str(m), str(n), "--gpus", str(gpus)] + extra)
    assert pp.returncode == 0, pp.stderr
    assert len(lp) == 1, lp
    dist = json.loads(lp[0])
    method = "dual" if "--dual" in extra else "two-phase"
    assert one["method"] == dist["method"] == method and dist["gpus"] == gpus
    assert dist["status"] == one["status"] and dist["pivots"] == one["pivots"]
    assert dist["objective"] == one["objective"] and dist["log_fnv"] == one["log_fnv"]
    o = Oracle(m, n + m + 1)
    if method == "dual":
        o.generate(n, seed, 3)
        res = o.solve_dual(1 << 40)
    else:
        o.generate(n, seed, 2)
        res = o.solve_two_phase(1 + n + (m + 1) // 2, None, 1 << 40, 1 if "bland" in extra else 0)
    assert res.pivots == one["pivots"] and res.objective == one["objective"]
    assert _fnv(*o.get_log()) == one["log_fnv"]
