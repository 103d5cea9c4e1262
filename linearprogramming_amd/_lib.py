"""ctypes binding of include/lpg.h (the C-ABI of the gfx950 pivot engine).

The shared library is built in-tree (``make`` -> linearprogramming_amd/liblpg.so)
so that it travels with the repository snapshot to the GPU box. There is no
fallback: if the library is missing or cannot be loaded, importing the engine
raises, so a GPU test can never pass on a silent CPU path.
"""
from __future__ import annotations

import ctypes
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblpg.so")

# include/lpg.h constants
OK, ERR_ARG, ERR_DEVICE, ERR_OOM, ERR_STATE, ERR_COMM = 0, -1, -2, -3, -4, -5
RUNNING, OPTIMAL, UNBOUNDED, INFEASIBLE, ITER_LIMIT, NUMERIC = 0, 1, 2, 3, 4, 5
STATUS_NAMES = {0: "RUNNING", 1: "OPTIMAL", 2: "UNBOUNDED", 3: "INFEASIBLE", 4: "ITER_LIMIT", 5: "NUMERIC"}
RULE_DANTZIG, RULE_BLAND = 0, 1
GEN_DENSE, GEN_DEGENERATE, GEN_ARTIFICIAL, GEN_DUAL = 0, 1, 2, 3
FLAG_NO_LOG = 0x1
FLAG_NO_SKIP = 0x2
FLAG_BIG_M = 0x4
FLAG_EAGER = 0x8
DEFER_MAX = 128

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int64_p = ctypes.POINTER(ctypes.c_int64)


class Result(ctypes.Structure):
    """lpg_result (same layout as oracle lpo_result)."""
    _fields_ = [("status", ctypes.c_int32), ("rule", ctypes.c_int32), ("pivots", ctypes.c_int64),
                ("objective", ctypes.c_double), ("entering", ctypes.c_int64), ("leaving", ctypes.c_int64)]


class Info(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("ncols", ctypes.c_int64), ("ld", ctypes.c_int64),
                ("row0", ctypes.c_int64), ("nrows", ctypes.c_int64),
                ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("device", ctypes.c_int32),
                ("nobj", ctypes.c_int32), ("defer_k", ctypes.c_int32), ("pivot_wg", ctypes.c_int32),
                ("bytes_per_pivot", ctypes.c_double), ("exchange", ctypes.c_int32), ("column_trade", ctypes.c_int32),
                ("residency_fallbacks", ctypes.c_int32), ("region", ctypes.c_int32),
                ("region_recoveries", ctypes.c_int32)]


class Timing(ctypes.Structure):
    _fields_ = [("update_ms", ctypes.c_double), ("select_ms", ctypes.c_double),
                ("comm_ms", ctypes.c_double), ("update_count", ctypes.c_int64), ("update_bytes", ctypes.c_double)]


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, c_double_p, ctypes.c_size_t)


class HostCommOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("allreduce_sum_f64", ALLREDUCE_FN)]


# (name, restype, argtypes) for every function include/lpg.h declares.
PROTOTYPES = [
    ("lpg_device_count", ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    ("lpg_create", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32]),
    ("lpg_create_dist", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_uint32]),
    ("lpg_comm_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    ("lpg_comm_init_rccl", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("lpg_comm_init_host", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(HostCommOps)]),
    ("lpg_comm_push_handle", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("lpg_comm_push_base", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    ("lpg_comm_init_push", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("lpg_comm_init_push_local", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
    ("lpg_destroy", None, [ctypes.c_void_p]),
    ("lpg_info", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Info)]),
    ("lpg_last_error", ctypes.c_char_p, [ctypes.c_void_p]),
    ("lpg_load_rows", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, c_double_p, ctypes.c_int64]),
    ("lpg_set_basis", ctypes.c_int, [ctypes.c_void_p, c_int64_p]),
    ("lpg_set_objective", ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    ("lpg_set_objective_m", ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    ("lpg_set_tolerances", ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]),
    ("lpg_set_active_columns", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("lpg_generate", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int]),
    ("lpg_solve", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(Result)]),
    ("lpg_enqueue", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]),
    ("lpg_sync", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Result)]),
    ("lpg_reserve_log", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("lpg_prepare", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("lpg_pivot", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]),
    ("lpg_solve_two_phase", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, c_double_p, ctypes.c_int64, ctypes.c_int,
                                           ctypes.POINTER(Result)]),
    ("lpg_solve_big_m", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, c_double_p, ctypes.c_int64, ctypes.c_int,
                                       ctypes.POINTER(Result)]),
    ("lpg_solve_dual", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(Result)]),
    ("lpg_get_rows", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, c_double_p, ctypes.c_int64]),
    ("lpg_get_basis", ctypes.c_int, [ctypes.c_void_p, c_int64_p]),
    ("lpg_get_column0", ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    ("lpg_get_log", ctypes.c_int64, [ctypes.c_void_p, c_int64_p, c_int64_p, ctypes.c_int64]),
    ("lpg_set_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("lpg_get_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Timing)]),
    ("lpg_device_sync", ctypes.c_int, [ctypes.c_void_p]),
    ("lpg_build_stamp", ctypes.c_char_p, []),
]


class StaleBuildError(RuntimeError):
    """The library's compiled-in source stamp is not the stamp of the sources beside it."""


def check_stamp(lib: ctypes.CDLL, path: str, src_root: str) -> str:
    """Refuse a library built from other sources than those under src_root
    (VERDICT r5 weak #9); returns the stamp."""
    from ._stamp import source_stamp
    built = lib.lpg_build_stamp().decode()
    if not os.path.isdir(os.path.join(src_root, "linearprogramming_amd", "csrc")):
        return built          # a library shipped without its sources: nothing to compare against
    want = source_stamp(src_root)
    if built != want:
        raise StaleBuildError(f"{path} is stale: built from sources at stamp {built}, the tree at {src_root} is "
                              f"{want} (run `make`)")
    return built

_lib = None
_runtime = None

# The unversioned names under which torch's bundled ROCm libraries NEED the
# runtime (torch/lib/libtorch_hip.so -> libamdhip64.so, librccl.so, ...).
# Dependencies first; every one of these is also bundled in torch/lib. RCCL
# (and the librocm_smi64 it pulls in) is deliberately absent: the system copy
# next to torch aborts at exit, so liblpg opens RCCL only when a communicator
# is attached, reusing torch's copy when torch is loaded (lpg_ctx.hip rccl_api).
_RUNTIME_NAMES = ("libnuma.so", "libelf.so", "libdrm.so", "libdrm_amdgpu.so", "librocm-core.so", "libroctx64.so",
                  "librocprofiler-register.so", "libamd_comgr.so", "libhsa-runtime64.so", "libamdhip64.so",
                  "libhiprtc.so")


def bind_runtime() -> str:
    """Make the whole process use ONE HIP runtime, whatever is imported next.

    liblpg.so NEEDs libamdhip64.so.7 (the system ROCm 7.2 the C host links);
    torch's bundled libraries NEED the unversioned names (libamdhip64.so,
    libhsa-runtime64.so, ...) and ship their own ROCm 7.0 copies. The dynamic loader reuses an already-loaded object when
    the requested name equals its SONAME or a name it was opened under, so:

    * torch already imported: liblpg's versioned NEEDED entry matches the
      SONAME of torch's copy (libamdhip64.so.7) -> torch's runtime serves
      both;
    * otherwise: open the system ROCm libraries here under exactly the
      unversioned names torch will ask for (resolved through ld.so.cache to
      /opt/rocm), RTLD_GLOBAL; liblpg then binds to them by SONAME and a
      later ``import torch`` binds to them by name -> one runtime, ROCm 7.2,
      the one lpgcli and the bridged reference CLI use.

    Before this, liblpg first and torch second mapped two libamdhip64 copies
    and aborted at exit (profiles/r01_runtime_order.log). Returns "torch" or
    "system"; tools/runtime_order.py checks /proc/self/maps for one copy of
    each library.
    """
    global _runtime
    if _runtime is not None:
        return _runtime
    if "torch" in sys.modules:
        _runtime = "torch"
        return _runtime
    for name in _RUNTIME_NAMES:
        try:
            ctypes.CDLL(name, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:   # no system ROCm: liblpg's own NEEDED entries decide (and fail loudly if absent)
            if name == "libamdhip64.so":
                raise RuntimeError(f"system ROCm runtime not loadable ({e}); liblpg.so needs libamdhip64.so.7") from e
    _runtime = "system"
    return _runtime


def mapped_runtimes() -> list:
    """Paths of every libamdhip64 mapped into this process (diagnostic)."""
    return sorted(p for p in mapped_libraries() if "libamdhip64" in p)


def mapped_libraries() -> list:
    """Real paths of every shared object mapped into this process."""
    out = set()
    with open("/proc/self/maps") as f:
        for line in f:
            p = line.split()[-1]
            if ".so" in p and p.startswith("/"):
                out.add(os.path.realpath(p))
    return sorted(out)


def duplicated_libraries() -> dict:
    """Library families mapped from more than one file (e.g. torch/lib and /opt/rocm copies)."""
    fam = {}
    for p in mapped_libraries():
        fam.setdefault(os.path.basename(p).split(".so")[0], []).append(p)
    return {k: v for k, v in fam.items() if len(v) > 1}


TESTHOOKS_PATH = os.path.join(_HERE, "liblpg_testhooks.so")
_private = {}


def load_testhooks(path: str = TESTHOOKS_PATH) -> ctypes.CDLL:
    """The engine built with its test-only fault hooks (LPG_TEST_HOOKS, the
    Makefile's liblpg_testhooks.so), loaded privately (RTLD_LOCAL, linked
    -Bsymbolic) next to liblpg.so for the tests that need a hook; pass it to
    Engine(lib=...). The product library has no hook."""
    if path in _private:
        return _private[path]
    if not os.path.exists(path):
        raise RuntimeError(f"test-hook engine not built: {path} is missing (run `make`)")
    bind_runtime()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if os.path.abspath(path) == TESTHOOKS_PATH:
        check_stamp(lib, path, _SRC_ROOT)
    _private[path] = lib
    return lib


# the sources the in-tree libraries are built from (linearprogramming_amd/csrc, include/lpg.h)
_SRC_ROOT = os.path.dirname(_HERE)
build_stamp = None


def load(path: str = LIB_PATH, src_root: str = None) -> ctypes.CDLL:
    """Load liblpg.so and declare every prototype. Raises if it is absent, or
    if the in-tree library's compiled-in stamp is not its sources' (a stale
    prebuilt binary never runs silently). Lab builds loaded from another path
    are not stamped against the tree."""
    global _lib, build_stamp
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"lpg HIP engine not built: {path} is missing (run `make` or __graft_entry__.build())")
    bind_runtime()
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if src_root is not None or os.path.abspath(path) == LIB_PATH:
        build_stamp = check_stamp(lib, path, src_root or _SRC_ROOT)
    else:
        build_stamp = lib.lpg_build_stamp().decode()
    _lib = lib
    return lib
