"""The block pass's item map (lpg_internal.h flush_nitems / flush_item: whole
items, then the last two strips in quarter-height items) covers every
(column tile, constraint row) exactly once, for tiles / heights / row counts
around every boundary. Host-side: the same inline functions k_flushw runs,
compiled with g++ (tests/item_map_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_item_map_covers_every_tile_row_once(tmp_path):
    exe = tmp_path / "item_map_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "linearprogramming_amd", "csrc"),
                    "-o", str(exe), os.path.join(ROOT, "tests", "item_map_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok ")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_xcd_grouped_item_map_covers_every_tile_row_once(tmp_path):
    """k_flushw's XCD-grouped map (FlushX: 8 group queues of row bands x H
    column classes, sub-bands, short tail pieces; tests/flushx_check.cpp) over
    shapes, H, sub-band heights and tail sizes. GPU side, bitwise:
    tests/test_gpu_defer.py::test_flush_item_maps_agree."""
    exe = tmp_path / "flushx_check"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "linearprogramming_amd", "csrc"),
                    "-o", str(exe), os.path.join(ROOT, "tests", "flushx_check.cpp")], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("flushx map ok")
