"""ctypes handle on oracle/liblpo.so — TEST INFRASTRUCTURE ONLY.

The CPU fp64 restatement of the pivot loop (see lpo.h for what it restates
and what pins it). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker or the
timed CPU baseline; the product (linearprogramming_amd / liblpg.so) never
calls it.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblpo.so")

RULE_DANTZIG, RULE_BLAND = 0, 1
GEN_DENSE, GEN_DEGENERATE, GEN_ARTIFICIAL, GEN_DUAL = 0, 1, 2, 3
STATUS_NAMES = {0: "RUNNING", 1: "OPTIMAL", 2: "UNBOUNDED", 3: "INFEASIBLE", 4: "ITER_LIMIT", 5: "NUMERIC"}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int64)


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("rule", ctypes.c_int32), ("pivots", ctypes.c_int64),
                ("objective", ctypes.c_double), ("entering", ctypes.c_int64), ("leaving", ctypes.c_int64)]


@dataclass
class OracleResult:
    status: int
    pivots: int
    objective: float
    entering: int
    leaving: int


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        lib = ctypes.CDLL(LIB_PATH)
        sig = {
            "lpo_create": (ctypes.c_void_p, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]),
            "lpo_create2": (ctypes.c_void_p, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int]),
            "lpo_set_objective_m": (ctypes.c_int, [ctypes.c_void_p, _dp]),
            "lpo_solve_big_m": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, _dp, ctypes.c_int64, ctypes.c_int,
                                               ctypes.POINTER(_Result)]),
            "lpo_destroy": (None, [ctypes.c_void_p]),
            "lpo_set_threads": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
            "lpo_load_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _dp, ctypes.c_int64]),
            "lpo_set_basis": (ctypes.c_int, [ctypes.c_void_p, _ip]),
            "lpo_set_objective": (ctypes.c_int, [ctypes.c_void_p, _dp]),
            "lpo_generate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int]),
            "lpo_set_tolerances": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]),
            "lpo_set_active_columns": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
            "lpo_solve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(_Result)]),
            "lpo_get_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _dp, ctypes.c_int64]),
            "lpo_get_basis": (ctypes.c_int, [ctypes.c_void_p, _ip]),
            "lpo_get_log": (ctypes.c_int64, [ctypes.c_void_p, _ip, _ip, ctypes.c_int64]),
            "lpo_pivot": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]),
            "lpo_rows": (ctypes.c_int64, [ctypes.c_void_p]),
            "lpo_price_col": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]),
            "lpo_ratio": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, _dp]),
            "lpo_pivot_row": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _dp]),
            "lpo_apply": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _dp]),
            "lpo_solve_two_phase": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, _dp, ctypes.c_int64, ctypes.c_int,
                                                   ctypes.POINTER(_Result)]),
            "lpo_solve_dual": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(_Result)]),
            "lpo_uniform": (ctypes.c_double, [ctypes.c_uint64, ctypes.c_uint64]),
            "lpo_subkey": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


class Oracle:
    def __init__(self, m: int, ncols: int, nthreads: int = 1, nobj: int = 1):
        self.lib = load()
        self.m, self.ncols, self.nobj = m, ncols, nobj
        self.ctx = self.lib.lpo_create2(m, ncols, nthreads, nobj)
        if not self.ctx:
            raise RuntimeError("lpo_create failed")

    def set_threads(self, n: int):
        self._ok(self.lib.lpo_set_threads(self.ctx, n), "set_threads")

    def close(self):
        if self.ctx:
            self.lib.lpo_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        self.close()

    def _ok(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed rc={rc}")

    def load_tableau(self, T, basis=None):
        T = np.ascontiguousarray(T, dtype=np.float64)
        self._ok(self.lib.lpo_load_rows(self.ctx, 0, T.shape[0], T.ctypes.data_as(_dp), T.shape[1]), "load_rows")
        if basis is not None:
            self.set_basis(basis)

    def set_basis(self, basis):
        b = np.ascontiguousarray(basis, dtype=np.int64)
        self._ok(self.lib.lpo_set_basis(self.ctx, b.ctypes.data_as(_ip)), "set_basis")

    def set_objective(self, c):
        c = np.ascontiguousarray(c, dtype=np.float64)
        self._ok(self.lib.lpo_set_objective(self.ctx, c.ctypes.data_as(_dp)), "set_objective")

    def set_objective_m(self, c):
        c = np.ascontiguousarray(c, dtype=np.float64)
        self._ok(self.lib.lpo_set_objective_m(self.ctx, c.ctypes.data_as(_dp)), "set_objective_m")

    def solve_big_m(self, art_first: int, cost=None, max_pivots: int = 1 << 40, rule: int = RULE_DANTZIG):
        cp = None if cost is None else np.ascontiguousarray(cost, dtype=np.float64).ctypes.data_as(_dp)
        r = _Result()
        self._ok(self.lib.lpo_solve_big_m(self.ctx, art_first, cp, max_pivots, rule, ctypes.byref(r)), "solve_big_m")
        return OracleResult(r.status, r.pivots, r.objective, r.entering, r.leaving)

    def set_tolerances(self, eps_piv=1e-9, eps_opt=1e-9):
        self._ok(self.lib.lpo_set_tolerances(self.ctx, eps_piv, eps_opt), "set_tolerances")

    def set_active_columns(self, nact):
        self._ok(self.lib.lpo_set_active_columns(self.ctx, nact), "set_active_columns")

    def generate(self, n: int, seed: int = 20220518, kind: int = GEN_DENSE):
        self._ok(self.lib.lpo_generate(self.ctx, n, seed, kind), "generate")

    def solve(self, max_pivots: int = 1 << 40, rule: int = RULE_DANTZIG, nparts: int = 1) -> OracleResult:
        r = _Result()
        self._ok(self.lib.lpo_solve(self.ctx, max_pivots, rule, nparts, ctypes.byref(r)), "solve")
        return OracleResult(r.status, r.pivots, r.objective, r.entering, r.leaving)

    def solve_two_phase(self, art_first: int, cost=None, max_pivots: int = 1 << 40, rule: int = RULE_DANTZIG):
        cp = None if cost is None else np.ascontiguousarray(cost, dtype=np.float64).ctypes.data_as(_dp)
        r = _Result()
        self._ok(self.lib.lpo_solve_two_phase(self.ctx, art_first, cp, max_pivots, rule, ctypes.byref(r)),
                 "solve_two_phase")
        return OracleResult(r.status, r.pivots, r.objective, r.entering, r.leaving)

    def solve_dual(self, max_pivots: int = 1 << 40) -> OracleResult:
        r = _Result()
        self._ok(self.lib.lpo_solve_dual(self.ctx, max_pivots, ctypes.byref(r)), "solve_dual")
        return OracleResult(r.status, r.pivots, r.objective, r.entering, r.leaving)

    def pivot(self, k: int, r: int):
        self._ok(self.lib.lpo_pivot(self.ctx, k, r), "pivot")

    # -- row-block primitives (multi-rank protocol model) --
    def price_col(self, rule=RULE_DANTZIG) -> int:
        return self.lib.lpo_price_col(self.ctx, rule)

    def ratio(self, k: int, rule: int, row_offset: int):
        out = np.zeros(4)
        self._ok(self.lib.lpo_ratio(self.ctx, k, rule, row_offset, out.ctypes.data_as(_dp)), "ratio")
        return out

    def pivot_row(self, rl: int, k: int) -> np.ndarray:
        P = np.zeros(self.ncols)
        self._ok(self.lib.lpo_pivot_row(self.ctx, rl, k, P.ctypes.data_as(_dp)), "pivot_row")
        return P

    def apply(self, k: int, rl: int, P: np.ndarray):
        P = np.ascontiguousarray(P, dtype=np.float64)
        self._ok(self.lib.lpo_apply(self.ctx, k, rl, P.ctypes.data_as(_dp)), "apply")

    def get_rows(self, row0=0, nrows=None) -> np.ndarray:
        if nrows is None:
            nrows = self.m + self.nobj - row0
        out = np.zeros((nrows, self.ncols))
        self._ok(self.lib.lpo_get_rows(self.ctx, row0, nrows, out.ctypes.data_as(_dp), self.ncols), "get_rows")
        return out

    def get_basis(self) -> np.ndarray:
        out = np.zeros(self.m, dtype=np.int64)
        self._ok(self.lib.lpo_get_basis(self.ctx, out.ctypes.data_as(_ip)), "get_basis")
        return out

    def get_log(self):
        n = self.lib.lpo_get_log(self.ctx, None, None, 0)
        k = np.zeros(max(n, 1), dtype=np.int64)
        r = np.zeros(max(n, 1), dtype=np.int64)
        self.lib.lpo_get_log(self.ctx, k.ctypes.data_as(_ip), r.ctypes.data_as(_ip), n)
        return k[:n], r[:n]


def uniform(key: int, idx: int) -> float:
    return load().lpo_uniform(key, idx)


def subkey(seed: int, which: int) -> int:
    return load().lpo_subkey(seed, which)
