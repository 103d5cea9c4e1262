"""The C-ABI library loads and exports exactly what include/lpg.h declares
(no GPU needed: nothing here launches a kernel)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "lpg.h")
LIB = os.path.join(ROOT, "linearprogramming_amd", "liblpg.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(lpg_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("lpg_create", "lpg_load_rows", "lpg_set_objective", "lpg_set_basis", "lpg_generate",
                     "lpg_solve", "lpg_enqueue", "lpg_get_basis", "lpg_get_column0", "lpg_last_error",
                     "lpg_destroy", "lpg_create_dist", "lpg_comm_init_rccl"):
        assert required in names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build first: make (or __graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from linearprogramming_amd import _lib
    bound = {name for name, _, _ in _lib.PROTOTYPES}
    assert bound == set(declared_functions())


def test_product_never_links_the_oracle():
    """liblpg.so must not depend on or contain the CPU oracle (no silent CPU path)."""
    nm = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True).stdout
    assert "lpo_" not in nm
    ldd = subprocess.run(["readelf", "-d", LIB], capture_output=True, text=True).stdout
    assert "liblpo" not in ldd
    assert "libamdhip64" in ldd
    # RCCL is opened at the first communicator (lpg_ctx.hip rccl_api), not linked: the symbols the
    # multi-rank path calls are looked up by name, so the library must carry those names
    assert "librccl" not in ldd
    strings = subprocess.run(["strings", LIB], capture_output=True, text=True).stdout
    for sym in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllGather", "ncclAllReduce", "librccl.so.1"):
        assert sym in strings, sym


def test_device_code_is_gfx950():
    """The embedded offload bundle carries a gfx950 code object (and no other GPU target)."""
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_errors_without_a_device_are_reported_not_raised():
    """Error behaviour mirrors the reference's `valid` flags: a negative code plus a message."""
    from linearprogramming_amd import _lib
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    rc = lib.lpg_create_dist(ctypes.byref(ctx), 0, 2, 5, 10, 20, 0)   # rank >= world
    assert rc == _lib.ERR_ARG
    assert b"bad shape" in lib.lpg_last_error(None)
    rc = lib.lpg_create(ctypes.byref(ctx), 0, 0, 20, 0)                # m = 0
    assert rc == _lib.ERR_ARG


def test_no_store_data_hazard_in_the_device_code():
    """No >8-byte VMEM store in liblpg.so's gfx950 code has its data VGPRs
    rewritten by VALU within two wait states (tools/store_hazard_scan.py:
    hipcc emits that sequence after raw buffer stores, and with other waves
    issuing on the SIMD the store then writes the new register values --
    profiles/r03_overlap_lab.log)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import store_hazard_scan
    finally:
        sys.path.pop(0)
    if not os.path.exists(store_hazard_scan.OBJDUMP):
        pytest.skip("llvm-objdump not installed")
    assert os.path.exists(LIB), "build first: make (or __graft_entry__.build())"
    hits = store_hazard_scan.scan(LIB)
    assert not hits, hits[:5]


def test_fault_hook_only_in_the_test_hook_build():
    """LPG_TEST_PENDING_FAULT (which corrupts the device's pending
    block on purpose) is compiled into linearprogramming_amd/liblpg_testhooks.so
    only; the product library carries no trace of it, and the hook build
    exports the same boundary."""
    hooks = os.path.join(ROOT, "linearprogramming_amd", "liblpg_testhooks.so")
    assert os.path.exists(LIB) and os.path.exists(hooks), "build first: make (or __graft_entry__.build())"
    assert b"LPG_TEST_PENDING_FAULT" not in open(LIB, "rb").read()
    assert b"LPG_TEST_PENDING_FAULT" in open(hooks, "rb").read()
    lib = ctypes.CDLL(hooks, mode=ctypes.RTLD_LOCAL)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
