"""Python handle on one lpg context (include/lpg.h) — test and bench plumbing.

The product is the C-ABI library; this class only marshals numpy arrays and
turns negative return codes into exceptions carrying lpg_last_error(), the way
the reference turns ``valid == 0`` into an ``ERROR: ...`` line.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import sys
from dataclasses import dataclass

import numpy as np

from . import _lib as L


class LPGError(RuntimeError):
    pass


@dataclass
class SolveResult:
    status: int
    pivots: int
    objective: float
    entering: int
    leaving: int
    rule: int

    @property
    def status_name(self) -> str:
        return L.STATUS_NAMES.get(self.status, str(self.status))


def _res(r: L.Result) -> SolveResult:
    return SolveResult(r.status, r.pivots, r.objective, r.entering, r.leaving, r.rule)


@contextlib.contextmanager
def _stdout_to_stderr():
    """RCCL prints a version banner on the process's stdout at init; keep
    stdout for results (bench.py's one JSON line) by pointing fd 1 at fd 2."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        ctypes.CDLL(None).fflush(None)      # C stdio buffers go out through the redirected fd
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def flush_kernel_for(pending: int) -> str:
    """Which block-pass kernel the default configuration launches for `pending`
    pivots (lpg_kernels.hip launch_flush_main): k_flushw at every block size
    ("m" = k_flushm only when LPG_FLUSH_KERNEL=m asks for it, <= 32 slots)."""
    return "w"


def device_count() -> int:
    lib = L.load()
    n = ctypes.c_int(0)
    lib.lpg_device_count(ctypes.byref(n))
    return n.value


class Engine:
    """One rank's engine for an m x ncols (= N+1) tableau."""

    def __init__(self, m: int, ncols: int, device: int = 0, world: int = 1, rank: int = 0, flags: int = 0,
                 lib=None):
        self.lib = lib if lib is not None else L.load()
        self._ctx = ctypes.c_void_p()
        rc = self.lib.lpg_create_dist(ctypes.byref(self._ctx), device, world, rank, m, ncols, flags)
        if rc != 0:
            raise LPGError(f"lpg_create_dist rc={rc}: {self.lib.lpg_last_error(None).decode()}")
        self.m, self.ncols, self.world, self.rank = m, ncols, world, rank
        self.nobj = 2 if flags & L.FLAG_BIG_M else 1
        self._keep = []   # ctypes callbacks kept alive

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if self._ctx:
            self.lib.lpg_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc < 0:
            raise LPGError(f"{what} rc={rc}: {self.lib.lpg_last_error(self._ctx).decode()}")
        return rc

    @property
    def info(self) -> L.Info:
        i = L.Info()
        self._check(self.lib.lpg_info(self._ctx, ctypes.byref(i)), "lpg_info")
        return i

    # -- communication ---------------------------------------------------
    def comm_init_rccl(self, uid: bytes):
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        with _stdout_to_stderr():
            rc = self.lib.lpg_comm_init_rccl(self._ctx, buf, len(uid))
        self._check(rc, "lpg_comm_init_rccl")

    @staticmethod
    def rccl_unique_id() -> bytes:
        lib = L.load()
        buf = ctypes.create_string_buffer(128)
        with _stdout_to_stderr():
            rc = lib.lpg_comm_unique_id(buf, 128)
        if rc != 0:
            raise LPGError(f"lpg_comm_unique_id rc={rc}: {lib.lpg_last_error(None).decode()}")
        return buf.raw

    def comm_init_host(self, allgather, allreduce_sum):
        """allgather(send: bytes) -> bytes (world * len); allreduce_sum(np.ndarray f64) -> np.ndarray."""
        world = self.world

        def _ag(user, send, recv, nbytes):
            try:
                data = ctypes.string_at(send, nbytes)
                out = allgather(data)
                assert len(out) == nbytes * world
                ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:   # pragma: no cover - reported as LPG_ERR_COMM
                return -1

        def _ar(user, buf, count):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(count,))
                arr[:] = allreduce_sum(arr.copy())
                return 0
            except Exception:   # pragma: no cover
                return -1

        ops = L.HostCommOps(None, L.ALLGATHER_FN(_ag), L.ALLREDUCE_FN(_ar))
        self._keep += [ops, _ag, _ar]
        self._check(self.lib.lpg_comm_init_host(self._ctx, ctypes.byref(ops)), "lpg_comm_init_host")

    # owner-push exchange (include/lpg.h): after a communicator
    def push_handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        self._check(self.lib.lpg_comm_push_handle(self._ctx, buf, 64), "lpg_comm_push_handle")
        return buf.raw

    def push_base(self) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.lpg_comm_push_base(self._ctx, ctypes.byref(p)), "lpg_comm_push_base")
        return p.value

    def comm_init_push(self, handles):
        """handles: every rank's push_handle(), in rank order."""
        blob = b"".join(bytes(h) for h in handles)
        buf = ctypes.create_string_buffer(blob, len(blob))
        self._check(self.lib.lpg_comm_init_push(self._ctx, buf, len(blob)), "lpg_comm_init_push")

    def comm_init_push_local(self, bases):
        """bases: every rank's push_base() (ranks of one process), in rank order."""
        arr = (ctypes.c_void_p * len(bases))(*bases)
        self._check(self.lib.lpg_comm_init_push_local(self._ctx, arr, len(bases)), "lpg_comm_init_push_local")

    # -- loading ---------------------------------------------------------
    def load_rows(self, row0: int, rows: np.ndarray):
        rows = np.ascontiguousarray(rows, dtype=np.float64)
        self._check(self.lib.lpg_load_rows(self._ctx, row0, rows.shape[0],
                                           rows.ctypes.data_as(L.c_double_p), rows.shape[1]), "lpg_load_rows")

    def load_tableau(self, T: np.ndarray, basis=None):
        """T: (m+1) x ncols full tableau (objective row last)."""
        self.load_rows(0, T)
        if basis is not None:
            self.set_basis(basis)

    def set_basis(self, basis):
        b = np.ascontiguousarray(basis, dtype=np.int64)
        self._check(self.lib.lpg_set_basis(self._ctx, b.ctypes.data_as(L.c_int64_p)), "lpg_set_basis")

    def set_objective(self, c):
        c = np.ascontiguousarray(c, dtype=np.float64)
        self._check(self.lib.lpg_set_objective(self._ctx, c.ctypes.data_as(L.c_double_p)), "lpg_set_objective")

    def set_tolerances(self, eps_piv=1e-9, eps_opt=1e-9):
        self._check(self.lib.lpg_set_tolerances(self._ctx, eps_piv, eps_opt), "lpg_set_tolerances")

    def set_active_columns(self, nact: int):
        self._check(self.lib.lpg_set_active_columns(self._ctx, nact), "lpg_set_active_columns")

    def generate(self, n: int, seed: int = 20220518, kind: int = L.GEN_DENSE):
        self._check(self.lib.lpg_generate(self._ctx, n, seed, kind), "lpg_generate")

    # -- pivoting --------------------------------------------------------
    def solve(self, max_pivots: int = 1 << 40, rule: int = L.RULE_DANTZIG) -> SolveResult:
        r = L.Result()
        self._check(self.lib.lpg_solve(self._ctx, max_pivots, rule, ctypes.byref(r)), "lpg_solve")
        return _res(r)

    def enqueue(self, npivots: int, rule: int = L.RULE_DANTZIG):
        self._check(self.lib.lpg_enqueue(self._ctx, npivots, rule), "lpg_enqueue")

    def sync(self) -> SolveResult:
        r = L.Result()
        self._check(self.lib.lpg_sync(self._ctx, ctypes.byref(r)), "lpg_sync")
        return _res(r)

    def pivot(self, k: int, r: int):
        self._check(self.lib.lpg_pivot(self._ctx, k, r), "lpg_pivot")

    def solve_two_phase(self, art_first: int, cost=None, max_pivots: int = 1 << 40, rule: int = L.RULE_DANTZIG):
        cp = None if cost is None else np.ascontiguousarray(cost, dtype=np.float64).ctypes.data_as(L.c_double_p)
        r = L.Result()
        self._check(self.lib.lpg_solve_two_phase(self._ctx, art_first, cp, max_pivots, rule, ctypes.byref(r)),
                    "lpg_solve_two_phase")
        return _res(r)

    def set_objective_m(self, cM):
        c = np.ascontiguousarray(cM, dtype=np.float64)
        self._check(self.lib.lpg_set_objective_m(self._ctx, c.ctypes.data_as(L.c_double_p)), "lpg_set_objective_m")

    def solve_big_m(self, art_first: int, cost=None, max_pivots: int = 1 << 40, rule: int = L.RULE_DANTZIG):
        cp = None if cost is None else np.ascontiguousarray(cost, dtype=np.float64).ctypes.data_as(L.c_double_p)
        r = L.Result()
        self._check(self.lib.lpg_solve_big_m(self._ctx, art_first, cp, max_pivots, rule, ctypes.byref(r)),
                    "lpg_solve_big_m")
        return _res(r)

    def solve_dual(self, max_pivots: int = 1 << 40) -> SolveResult:
        r = L.Result()
        self._check(self.lib.lpg_solve_dual(self._ctx, max_pivots, ctypes.byref(r)), "lpg_solve_dual")
        return _res(r)

    def reserve_log(self, n: int):
        self._check(self.lib.lpg_reserve_log(self._ctx, n), "lpg_reserve_log")

    def prepare(self, rule: int = L.RULE_DANTZIG):
        """Build the replayed pivot graph now (no pivots run; include/lpg.h lpg_prepare)."""
        self._check(self.lib.lpg_prepare(self._ctx, rule), "lpg_prepare")

    def device_sync(self):
        self._check(self.lib.lpg_device_sync(self._ctx), "lpg_device_sync")

    # -- readout ---------------------------------------------------------
    def get_rows(self, row0: int, nrows: int) -> np.ndarray:
        out = np.zeros((nrows, self.ncols), dtype=np.float64)
        self._check(self.lib.lpg_get_rows(self._ctx, row0, nrows, out.ctypes.data_as(L.c_double_p), self.ncols),
                    "lpg_get_rows")
        return out

    def get_basis(self) -> np.ndarray:
        out = np.zeros(self.m, dtype=np.int64)
        self._check(self.lib.lpg_get_basis(self._ctx, out.ctypes.data_as(L.c_int64_p)), "lpg_get_basis")
        return out

    def get_column0(self) -> np.ndarray:
        out = np.zeros(self.info.nrows, dtype=np.float64)
        self._check(self.lib.lpg_get_column0(self._ctx, out.ctypes.data_as(L.c_double_p)), "lpg_get_column0")
        return out

    def get_log(self):
        n = self._check(self.lib.lpg_get_log(self._ctx, None, None, 0), "lpg_get_log")
        k = np.zeros(max(n, 1), dtype=np.int64)
        r = np.zeros(max(n, 1), dtype=np.int64)
        self._check(self.lib.lpg_get_log(self._ctx, k.ctypes.data_as(L.c_int64_p), r.ctypes.data_as(L.c_int64_p), n),
                    "lpg_get_log")
        return k[:n], r[:n]

    # -- timing ----------------------------------------------------------
    def set_timing(self, enable: bool):
        self._check(self.lib.lpg_set_timing(self._ctx, int(enable)), "lpg_set_timing")

    def get_timing(self) -> L.Timing:
        t = L.Timing()
        self._check(self.lib.lpg_get_timing(self._ctx, ctypes.byref(t)), "lpg_get_timing")
        return t
