"""bench.py attaches a PMC traffic figure only to the build and run it
measured: the file's source stamp, kernel,
pending-pivot count and LP shape must all match, a --shape stand-in or a
multi-GPU line never takes one. CPU only (no kernel runs)."""
from __future__ import annotations

import json
import os
import types

import bench


def _args(config=3, shape=None):
    return types.SimpleNamespace(config=config, shape=shape)


def _write(tmp_path, monkeypatch, **kw):
    prof = tmp_path / "profiles"
    prof.mkdir()
    rec = {"hbm_bytes_per_launch": 9.2e9, "kernel": "k_flushw", "pending_pivots": 64, "m": 16384, "n": 32768,
           "source_stamp": bench.source_stamp(), "source": "profiles/rNN_pmc.json"}
    rec.update(kw)
    (prof / "pmc_config3.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    return rec


def test_source_stamp_is_stable_and_covers_the_sources():
    a, b = bench.source_stamp(), bench.source_stamp()
    assert a == b and len(a) == 16


def test_matching_file_is_attached(tmp_path, monkeypatch):
    stamp = bench.source_stamp()
    _write(tmp_path, monkeypatch)
    p, why = bench.pmc_traffic(_args(), "k_flushw", 64, 16384, 32768, 1, stamp)
    assert why is None and p["hbm_bytes_per_launch"] == 9.2e9


def test_stale_stamp_is_refused(tmp_path, monkeypatch):
    stamp = bench.source_stamp()
    _write(tmp_path, monkeypatch, source_stamp="0123456789abcdef")
    p, why = bench.pmc_traffic(_args(), "k_flushw", 64, 16384, 32768, 1, stamp)
    assert p is None and "source_stamp" in why


def test_unstamped_file_is_refused(tmp_path, monkeypatch):
    stamp = bench.source_stamp()
    rec = _write(tmp_path, monkeypatch)
    rec.pop("source_stamp")
    (tmp_path / "profiles" / "pmc_config3.json").write_text(json.dumps(rec))
    p, why = bench.pmc_traffic(_args(), "k_flushw", 64, 16384, 32768, 1, stamp)
    assert p is None and "source_stamp" in why


def test_other_shape_kernel_or_pending_refused(tmp_path, monkeypatch):
    stamp = bench.source_stamp()
    _write(tmp_path, monkeypatch)
    for kname, defer, m, n in (("k_flushw", 96, 16384, 32768), ("k_flushm", 64, 16384, 32768),
                               ("k_flushw", 64, 8192, 40960)):
        p, why = bench.pmc_traffic(_args(), kname, defer, m, n, 1, stamp)
        assert p is None and why


def test_stand_in_and_multi_gpu_lines_never_take_a_file(tmp_path, monkeypatch):
    stamp = bench.source_stamp()
    _write(tmp_path, monkeypatch)
    p, why = bench.pmc_traffic(_args(shape="8192,40960"), "k_flushw", 64, 16384, 32768, 1, stamp)
    assert p is None and "single-GPU" in why
    p, why = bench.pmc_traffic(_args(), "k_flushw", 64, 16384, 32768, 2, stamp)
    assert p is None and "single-GPU" in why


def test_committed_files_carry_a_stamp_or_are_refused():
    """Every committed pmc_config*.json is either stamped with the current
    sources or refused by bench.py (never attached silently)."""
    prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    stamp = bench.source_stamp()
    for name in sorted(os.listdir(prof)):
        if name.startswith("pmc_config") and name.endswith(".json"):
            cfg = int(name[len("pmc_config"):-len(".json")])
            rec = json.load(open(os.path.join(prof, name)))
            m, n = bench.CONFIGS[cfg]["m"], bench.CONFIGS[cfg]["n"]
            p, why = bench.pmc_traffic(_args(cfg), rec.get("kernel"), rec.get("pending_pivots"), m, n, 1, stamp)
            assert (p is not None) == (rec.get("source_stamp") == stamp), (name, why)


def test_roofline_names_the_binding_roofline():
    """The pass against both rooflines: at 64 pending pivots its bytes bind
    (HBM), at 96 its flops do (the f64 matrix cores); `achieved` / `frac` are
    the binding one's and both are reported."""
    touched = 8.59e9                                    # config 3: 16 B x 16384 rows x 32770 live columns
    r64 = bench.roofline_bound(touched, 64, 1.60)
    assert r64["bound"] == "hbm" and r64["unit"] == "GB/s"
    assert abs(r64["achieved"] - touched / 1.60e-3 / 1e9) < 1e-6 and r64["frac"] == r64["hbm"]["frac"]
    r96 = bench.roofline_bound(touched, 96, 2.20)
    assert r96["bound"] == "mfma" and r96["unit"] == "TFLOP/s" and r96["peak"] == bench.MFMA_F64_PEAK_TFS
    flops = touched / 16 * 2 * 96
    assert abs(r96["mfma"]["algorithmic_flops_per_launch"] - flops) < 1.0
    assert abs(r96["achieved"] - flops / 2.20e-3 / 1e12) < 1e-9 and r96["frac"] < 1.0
    assert r96["hbm"]["unit"] == "GB/s" and abs(r96["hbm"]["achieved"] - touched / 2.20e-3 / 1e9) < 1e-6
