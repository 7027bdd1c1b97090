"""ctypes binding of the C oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the checker / CPU baseline. "parity unpinned" — see
oracle/tswap_oracle.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(
            os.path.join(HERE, "tswap_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER
        u32, i32, u64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
        L.orc_graph_create.argtypes = [P(ctypes.c_uint8), u32, u32]
        L.orc_graph_create.restype = ctypes.c_void_p
        L.orc_graph_destroy.argtypes = [ctypes.c_void_p]
        L.orc_get_path_next.argtypes = [ctypes.c_void_p, u32, u32, P(u32), P(u64)]
        L.orc_get_path_next.restype = i32
        L.orc_bfs_u16.argtypes = [ctypes.c_void_p, u32, P(ctypes.c_uint16)]
        L.orc_bfs_u16.restype = ctypes.c_int
        L.orc_next_codes.argtypes = [ctypes.c_void_p, u32, P(ctypes.c_uint8)]
        L.orc_next_codes.restype = ctypes.c_int
        L.orc_tswap_step.argtypes = [ctypes.c_void_p, P(u32), P(u32), u32]
        L.orc_tswap_mapd.argtypes = [ctypes.c_void_p, P(u32), u32, P(u32), u32, u32, P(u64), P(u32)]
        L.orc_tswap_mapd.restype = i32
        L.orc_decide.argtypes = [ctypes.c_void_p, u32, u32, P(u32), P(u32), u32, P(u32), P(u32), P(u32), P(u32),
                                 P(u32)]
        L.orc_decide.restype = ctypes.c_int
        L.orc_tswap_mapd_fast.argtypes = [P(ctypes.c_uint8), u32, u32, P(u32), u32, P(u32), u32, u32, P(u64),
                                          P(u32), u32, P(u64)]
        L.orc_tswap_mapd_fast.restype = i32
        L.orc_stat_calls.argtypes = [ctypes.c_void_p]
        L.orc_stat_calls.restype = u64
        L.orc_stat_pops.argtypes = [ctypes.c_void_p]
        L.orc_stat_pops.restype = u64
        _lib = L
    return _lib


def _u32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class OracleGraph:
    def __init__(self, cells: np.ndarray):
        self.cells = np.ascontiguousarray(cells, dtype=np.uint8)
        self.h, self.w = self.cells.shape
        L = lib()
        self.ptr = L.orc_graph_create(self.cells.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), self.w, self.h)
        if not self.ptr:
            raise ValueError("bad grid")

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().orc_graph_destroy(self.ptr)
            self.ptr = None

    def get_path_next(self, start: int, goal: int):
        nxt = ctypes.c_uint32(0)
        pops = ctypes.c_uint64(0)
        ln = lib().orc_get_path_next(self.ptr, start, goal, ctypes.byref(nxt), ctypes.byref(pops))
        return nxt.value, ln, pops.value

    def bfs(self, goal: int) -> np.ndarray:
        out = np.zeros(self.w * self.h, dtype=np.uint16)
        rc = lib().orc_bfs_u16(self.ptr, goal, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
        if rc != 0:
            raise ValueError("goal blocked")
        return out

    def next_codes(self, goal: int) -> np.ndarray:
        out = np.zeros(self.w * self.h, dtype=np.uint8)
        if lib().orc_next_codes(self.ptr, goal, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) != 0:
            raise ValueError("goal blocked")
        return out

    def step(self, v, g):
        v = np.ascontiguousarray(v, dtype=np.uint32).copy()
        g = np.ascontiguousarray(g, dtype=np.uint32).copy()
        lib().orc_tswap_step(self.ptr, _u32p(v), _u32p(g), v.size)
        return v, g

    def mapd(self, starts_xy: np.ndarray, tasks_xyxy: np.ndarray, max_t: int = 2000, trace_goals: bool = False):
        """Returns (rec (n,T) uint64 = x | y<<16 | state<<32, goals (n,T) or None)."""
        s = np.ascontiguousarray(starts_xy, dtype=np.uint32).reshape(-1)
        t = np.ascontiguousarray(tasks_xyxy, dtype=np.uint32).reshape(-1)
        n, m = s.size // 2, t.size // 4
        out = np.zeros((max(n, 1), max_t + 1), dtype=np.uint64)
        gout = np.zeros((max(n, 1), max_t + 1), dtype=np.uint32) if trace_goals else None
        T = lib().orc_tswap_mapd(self.ptr, _u32p(s), n, _u32p(t), m, max_t,
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                 _u32p(gout) if gout is not None else None)
        if T < 0:
            raise ValueError("invalid input (reference would panic)")
        return out[:n, :T], (gout[:n, :T] if gout is not None else None)

    def mapd_fast(self, starts_xy: np.ndarray, tasks_xyxy: np.ndarray, max_t: int = 2000, nthreads: int = 8):
        """Same plan as mapd(trace_goals=True) from the memoised, prefilled oracle loop
        (tswap_oracle_fast.c). Returns (rec, goals, stats) with stats = {inline, prefill, hits, memo}."""
        s = np.ascontiguousarray(starts_xy, dtype=np.uint32).reshape(-1)
        t = np.ascontiguousarray(tasks_xyxy, dtype=np.uint32).reshape(-1)
        n, m = s.size // 2, t.size // 4
        out = np.zeros((max(n, 1), max_t + 1), dtype=np.uint64)
        gout = np.zeros((max(n, 1), max_t + 1), dtype=np.uint32)
        st = np.zeros(4, dtype=np.uint64)
        T = lib().orc_tswap_mapd_fast(self.cells.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), self.w, self.h,
                                      _u32p(s), n, _u32p(t), m, max_t,
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _u32p(gout), nthreads,
                                      st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        if T < 0:
            raise ValueError("invalid input (reference would panic)")
        stats = dict(zip(("inline", "prefill", "hits", "memo"), (int(x) for x in st)))
        return out[:n, :T], gout[:n, :T], stats

    def decide(self, my_v: int, my_g: int, nb_v, nb_g):
        """compute_next_move_with_tswap (agent.rs:329-462) for one agent. Returns
        (act, cell, partner, participants) with act 0 Move, 1 WaitForGoalSwap, 2 WaitForRotation,
        3 Wait; partner / participants are indices into the nearby list."""
        nv = np.ascontiguousarray(nb_v, dtype=np.uint32)
        ng = np.ascontiguousarray(nb_g, dtype=np.uint32)
        act, cell, partner, npart = (ctypes.c_uint32(0) for _ in range(4))
        part = np.zeros(nv.size + 1, dtype=np.uint32)
        rc = lib().orc_decide(self.ptr, my_v, my_g, _u32p(nv), _u32p(ng), nv.size, ctypes.byref(act),
                              ctypes.byref(cell), ctypes.byref(partner), ctypes.byref(npart), _u32p(part))
        if rc != 0:
            raise ValueError("agent cell not free (reference panics)")
        return act.value, cell.value, partner.value, [int(x) for x in part[:npart.value]]

    def calls(self):
        return lib().orc_stat_calls(self.ptr)

    def pops(self):
        return lib().orc_stat_pops(self.ptr)
