"""MI355X-native TSWAP planning core — Python mirror of the reference interface.

Drop-in for the src/algorithm path of RenKoya1/p2p_distributed_tswap
(@ 2025-11-21). Everything here is a thin ctypes layer over the C ABI in
include/tswap.h (libtswap_hip.so: hand-written gfx950 HIP kernels + C++ host
runtime). There is NO CPU fallback: if the HIP library or a GPU is missing,
every call raises.

Reference interface mirrored (same names, argument meaning, error behaviour):
  tswap_mapd(grid, initial_positions, tasks)  src/algorithm/tswap.rs:39-43
      -> list[list[((x, y), AgentState)]]; panics become TswapError(EINVAL)
  AgentState                                  src/map/agent.rs:9-15
  Task(pickup, delivery, peer_id, task_id)    src/map/task_generator.rs:6-12
  Point = (x, y)                              src/map/map.rs:4
"""
from __future__ import annotations

import ctypes
import enum
import os
from dataclasses import dataclass
from typing import Iterable, Optional, Sequence

import numpy as np

__all__ = [
    "AgentState", "Task", "TswapError", "Planner", "tswap_mapd", "tswap_step",
    "load_library", "LIB_PATH", "grid_to_bytes", "build_id",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtswap_hip.so")
# diagnostic build (-DTSW_DIAG): the same kernels plus the TSW_* environment knobs (kernel A/B variants,
# instrumentation). Tests of the A/B variants and measurement scripts only; products load LIB_PATH.
DIAG_LIB_PATH = os.path.join(_HERE, "libtswap_hip_diag.so")

TSW_OK, TSW_EINVAL, TSW_ENOMEM, TSW_EHIP, TSW_EOVERFLOW = 0, -22, -12, -5, -75
TSW_ABI_VERSION = 6  # include/tswap.h
TSW_F_EAGER_NEXTHOP, TSW_F_LAZY_NEXTHOP, TSW_F_EXIT_MODE = 1, 2, 4
# TswapAction (bin/decentralized/agent.rs:321-326), include/tswap.h TSW_ACT_*
TSW_ACT_MOVE, TSW_ACT_GOAL_SWAP, TSW_ACT_ROTATION, TSW_ACT_WAIT = 0, 1, 2, 3
DIST_INF = 0xFFFF


class AgentState(enum.IntEnum):
    """src/map/agent.rs:9-15 (discriminants in declaration order)."""
    PICKING = 0
    CARRYING = 1
    DELIVERED = 2
    IDLE = 3


@dataclass
class Task:
    """src/map/task_generator.rs:6-12. peer_id/task_id are carried, never read by the planner."""
    pickup: tuple
    delivery: tuple
    peer_id: Optional[str] = None
    task_id: Optional[int] = None


class TswapError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"tswap error {code}: {msg}")
        self.code = code


class _Point(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32)]


class _Task(ctypes.Structure):
    _fields_ = [("pickup", _Point), ("delivery", _Point)]


class _Rec(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint16), ("y", ctypes.c_uint16), ("state", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 3)]


class _Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("table_budget_bytes", ctypes.c_uint64), ("watchdog_ms", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [
        ("bfs_goals", ctypes.c_uint64), ("bfs_launches", ctypes.c_uint64), ("bfs_ms", ctypes.c_double),
        ("astar_queries", ctypes.c_uint64), ("astar_launches", ctypes.c_uint64), ("astar_ms", ctypes.c_double),
        ("walker_launches", ctypes.c_uint64), ("walker_ms", ctypes.c_double),
        ("assign_launches", ctypes.c_uint64), ("assign_ms", ctypes.c_double),
        ("steps", ctypes.c_uint64), ("tables", ctypes.c_uint64), ("plan_ms", ctypes.c_double),
        ("plan_section_ms", ctypes.c_double * 8), ("rule_rounds", ctypes.c_uint64),
        ("plan_exits", ctypes.c_uint64 * 8), ("table_evictions", ctypes.c_uint64),
        ("coop_waits", ctypes.c_uint64), ("coop_wait_ms", ctypes.c_double),
        ("coop_wait_sec_ms", ctypes.c_double * 8), ("coop_waits_sec", ctypes.c_uint64 * 8),
        ("relabels_full", ctypes.c_uint64), ("relabels_inc", ctypes.c_uint64),
        ("move_rounds", ctypes.c_uint64), ("plan_block", ctypes.c_uint32),
        ("coop_workers", ctypes.c_uint32), ("coop_worker_busy_ms", ctypes.c_double * 3),
        ("watchdog_fires", ctypes.c_uint64), ("tableless_goals", ctypes.c_uint64),
        ("coop_worker_queries", ctypes.c_uint64 * 3), ("coop_worker_pops", ctypes.c_uint64 * 3),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["plan_section_ms"] = list(self.plan_section_ms)
        d["plan_exits"] = list(self.plan_exits)
        d["coop_wait_sec_ms"] = list(self.coop_wait_sec_ms)
        d["coop_waits_sec"] = list(self.coop_waits_sec)
        d["coop_worker_busy_ms"] = list(self.coop_worker_busy_ms)
        d["coop_worker_queries"] = list(self.coop_worker_queries)
        d["coop_worker_pops"] = list(self.coop_worker_pops)
        return d


# every symbol declared in include/tswap.h (tests check the .so exports them)
EXPORTED_SYMBOLS = (
    "tsw_create", "tsw_destroy", "tsw_last_error", "tsw_plan_mapd", "tsw_plan_mapd_trace",
    "tsw_step", "tsw_get_path_next", "tsw_decide", "tsw_dist_tables", "tsw_dist_tables_device",
    "tsw_import_tables_device", "tsw_next_hop_tables", "tsw_next_hop_tables_device", "tsw_import_next_hops_device",
    "tsw_clear_tables", "tsw_get_stats", "tsw_reset_stats", "tsw_set_timing", "tsw_probe_round_floors",
    "tsw_abi_version", "tsw_plan_mapd_resolved", "tsw_next_hop_codes", "tsw_build_id",
)

# tsw_resolve_fn (include/tswap.h): int (*)(void *user, uint32_t k, const uint32_t *start,
# const uint32_t *goal, uint8_t *code)
_RESOLVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                               ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint8))

_libs = {}


def load_library(path: str = LIB_PATH):
    """Load libtswap_hip.so (built by __graft_entry__.build()). Raises if absent."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise TswapError(TSW_EHIP, f"HIP library not built: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    # the ABI revision first: an older library lacks the newer symbols, and binding them
    # before this check would fail with a bare AttributeError instead of the rebuild message
    abi = None
    if hasattr(lib, "tsw_abi_version"):
        lib.tsw_abi_version.argtypes = []
        lib.tsw_abi_version.restype = ctypes.c_int
        abi = lib.tsw_abi_version()
    if abi != TSW_ABI_VERSION:
        raise TswapError(TSW_EINVAL, f"{path}: ABI {abi}, this binding mirrors {TSW_ABI_VERSION} "
                                     "(rebuild with __graft_entry__.build())")
    P = ctypes.POINTER
    u32, i32, u64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
    vp = ctypes.c_void_p
    lib.tsw_create.argtypes = [P(ctypes.c_uint8), u32, u32, P(_Opts)]
    lib.tsw_create.restype = vp
    lib.tsw_destroy.argtypes = [vp]
    lib.tsw_destroy.restype = None
    lib.tsw_last_error.argtypes = [vp]
    lib.tsw_last_error.restype = ctypes.c_char_p
    lib.tsw_plan_mapd.argtypes = [vp, P(_Point), u32, P(_Task), u32, u32, P(_Rec), P(u32)]
    lib.tsw_plan_mapd_trace.argtypes = [vp, P(_Point), u32, P(_Task), u32, u32, P(_Rec), P(u32), P(u32)]
    lib.tsw_step.argtypes = [vp, P(u32), P(u32), u32]
    lib.tsw_get_path_next.argtypes = [vp, P(u32), P(u32), u32, P(u32), P(i32)]
    lib.tsw_decide.argtypes = [vp, P(u32), P(u32), u32, P(u32), P(u32), P(u32), P(u32), P(u32), P(u32), P(u32),
                               P(u32)]
    lib.tsw_dist_tables.argtypes = [vp, P(u32), u32, P(ctypes.c_uint16)]
    lib.tsw_dist_tables_device.argtypes = [vp, P(u32), u32, vp]
    lib.tsw_import_tables_device.argtypes = [vp, P(u32), u32, vp]
    lib.tsw_clear_tables.argtypes = [vp]
    lib.tsw_next_hop_tables.argtypes = [vp, P(u32), u32, P(ctypes.c_uint8)]
    lib.tsw_next_hop_tables_device.argtypes = [vp, P(u32), u32, vp, vp]
    lib.tsw_import_next_hops_device.argtypes = [vp, P(u32), u32, vp, vp]
    lib.tsw_get_stats.argtypes = [vp, P(Stats)]
    lib.tsw_reset_stats.argtypes = [vp]
    lib.tsw_set_timing.argtypes = [vp, ctypes.c_int]
    lib.tsw_probe_round_floors.argtypes = [vp, ctypes.c_uint32, P(ctypes.c_double)]
    lib.tsw_plan_mapd_resolved.argtypes = [vp, P(_Point), u32, P(_Task), u32, u32, P(_Rec), P(u32), P(u32),
                                           _RESOLVE_FN, vp]
    lib.tsw_plan_mapd_resolved.restype = ctypes.c_int
    lib.tsw_next_hop_codes.argtypes = [vp, P(u32), P(u32), u32, P(ctypes.c_uint8)]
    lib.tsw_next_hop_codes.restype = ctypes.c_int
    lib.tsw_build_id.argtypes = []
    lib.tsw_build_id.restype = ctypes.c_uint64
    for name in ("tsw_plan_mapd", "tsw_plan_mapd_trace", "tsw_step", "tsw_get_path_next", "tsw_decide", "tsw_dist_tables",
                 "tsw_dist_tables_device", "tsw_import_tables_device", "tsw_clear_tables", "tsw_next_hop_tables",
                 "tsw_next_hop_tables_device", "tsw_import_next_hops_device", "tsw_get_stats", "tsw_reset_stats",
                 "tsw_set_timing", "tsw_probe_round_floors"):
        getattr(lib, name).restype = ctypes.c_int
    _libs[path] = lib
    return lib


def build_id(diag: bool = False) -> str:
    """tsw_build_id() of the loaded library as 16 hex digits: the sha1 of the sources it was built from
    (__graft_entry__.source_hash). Profiles record it; bench.py pairs a profile only with its build."""
    return f"{load_library(DIAG_LIB_PATH if diag else LIB_PATH).tsw_build_id():016x}"


def grid_to_bytes(grid) -> tuple:
    """grid: list[str] | list[list[str]] | np.ndarray(uint8, HxW). Returns (bytes_array, w, h).

    Mirrors the reference: h = len(grid), w = len(grid[0]) (tswap.rs:46-47).
    """
    if isinstance(grid, np.ndarray):
        a = np.ascontiguousarray(grid, dtype=np.uint8)
        return a, a.shape[1], a.shape[0]
    rows = ["".join(r) if not isinstance(r, str) else r for r in grid]
    h = len(rows)
    w = len(rows[0])
    if any(len(r) != w for r in rows):
        raise TswapError(TSW_EINVAL, "ragged grid rows (the reference indexes grid[y][x] for x < len(grid[0]))")
    a = np.frombuffer("".join(rows).encode("latin-1"), dtype=np.uint8).reshape(h, w).copy()
    return a, w, h


def _u32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class Planner:
    """One device context (tsw_ctx) bound to a grid."""

    def __init__(self, grid, device: int = 0, flags: int = 0, table_budget_bytes: int = 0, watchdog_ms: int = 0,
                 diag: bool = False):
        """flags: TSW_F_*; watchdog_ms: tsw_opts.watchdog_ms (0 = 10 s); diag: bind the diagnostic
        build (reads the TSW_* environment knobs at creation) instead of the production library."""
        self._lib = load_library(DIAG_LIB_PATH if diag else LIB_PATH)
        cells, w, h = grid_to_bytes(grid)
        self.w, self.h = int(w), int(h)
        opts = _Opts(device, flags, table_budget_bytes, watchdog_ms, 0)
        ptr = self._lib.tsw_create(cells.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), w, h,
                                   ctypes.byref(opts))
        if not ptr:
            raise TswapError(TSW_EHIP, self._lib.tsw_last_error(None).decode())
        self._ctx = ptr

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.tsw_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc):
        if rc != TSW_OK:
            raise TswapError(rc, self._lib.tsw_last_error(self._ctx).decode())

    # --- tswap_mapd -------------------------------------------------------
    def plan_mapd_arrays(self, starts_xy: np.ndarray, tasks_xyxy: np.ndarray, max_t: int = 2000,
                         trace_goals: bool = False):
        """starts_xy: (n,2) uint32; tasks_xyxy: (m,4) uint32 (pickup x,y, delivery x,y).

        Returns (rec (n, T) uint64 packed x | y<<16 | state<<32, goals (n, T) or None).
        """
        starts = np.ascontiguousarray(starts_xy, dtype=np.uint32).reshape(-1, 2)
        tasks = np.ascontiguousarray(tasks_xyxy, dtype=np.uint32).reshape(-1, 4)
        n, m = starts.shape[0], tasks.shape[0]
        stride = max_t + 1
        out = np.zeros((max(n, 1), stride), dtype=np.uint64)
        T = ctypes.c_uint32(0)
        sp = starts.ctypes.data_as(ctypes.POINTER(_Point))
        tp = tasks.ctypes.data_as(ctypes.POINTER(_Task))
        op = out.ctypes.data_as(ctypes.POINTER(_Rec))
        goals = None
        if trace_goals:
            goals = np.zeros((max(n, 1), stride), dtype=np.uint32)
            rc = self._lib.tsw_plan_mapd_trace(self._ctx, sp, n, tp, m, max_t, op, _u32p(goals), ctypes.byref(T))
        else:
            rc = self._lib.tsw_plan_mapd(self._ctx, sp, n, tp, m, max_t, op, ctypes.byref(T))
        self._check(rc)
        t = T.value
        rec = out[:n, :t] & np.uint64(0xFFFFFFFFFF)
        return rec, (goals[:n, :t] if goals is not None else None)

    def plan_mapd_resolved(self, starts_xy: np.ndarray, tasks_xyxy: np.ndarray, max_t: int, resolve,
                           trace_goals: bool = False):
        """tsw_plan_mapd_resolved: as plan_mapd_arrays, with every K3 batch answered by
        resolve(start u32[k], goal u32[k]) -> u8[k] codes (e.g. sharding.ShardedK3.resolve)."""
        starts = np.ascontiguousarray(starts_xy, dtype=np.uint32).reshape(-1, 2)
        tasks = np.ascontiguousarray(tasks_xyxy, dtype=np.uint32).reshape(-1, 4)
        n, m = starts.shape[0], tasks.shape[0]
        stride = max_t + 1
        out = np.zeros((max(n, 1), stride), dtype=np.uint64)
        goals = np.zeros((max(n, 1), stride), dtype=np.uint32) if trace_goals else None
        T = ctypes.c_uint32(0)
        failure = []

        def cb(user, k, sp, gp, cp):
            try:
                st = np.ctypeslib.as_array(sp, shape=(k,)).copy()
                gl = np.ctypeslib.as_array(gp, shape=(k,)).copy()
                codes = np.ascontiguousarray(resolve(st, gl), dtype=np.uint8)
                if codes.shape != (k,):
                    raise ValueError(f"resolver returned {codes.shape}, expected ({k},)")
                ctypes.memmove(cp, codes.ctypes.data, k)
                return 0
            except BaseException as e:  # noqa: BLE001 — re-raised after the call returns
                failure.append(e)
                return 1

        fn = _RESOLVE_FN(cb)
        rc = self._lib.tsw_plan_mapd_resolved(
            self._ctx, starts.ctypes.data_as(ctypes.POINTER(_Point)), n,
            tasks.ctypes.data_as(ctypes.POINTER(_Task)), m, max_t, out.ctypes.data_as(ctypes.POINTER(_Rec)),
            _u32p(goals) if goals is not None else None, ctypes.byref(T), fn, None)
        if failure:
            raise failure[0]
        self._check(rc)
        t = T.value
        rec = out[:n, :t] & np.uint64(0xFFFFFFFFFF)
        return rec, (goals[:n, :t] if goals is not None else None)

    def next_hop_codes(self, start, goal) -> np.ndarray:
        """tsw_next_hop_codes: u8 next-hop code of get_path(start[i], goal[i]) (0..3 S,E,N,W, 4 stay),
        from this context's table store (K1 / exact A* for what it does not hold yet)."""
        st = np.ascontiguousarray(start, dtype=np.uint32)
        gl = np.ascontiguousarray(goal, dtype=np.uint32)
        if st.shape != gl.shape:
            raise TswapError(TSW_EINVAL, "start and goal must have the same length")
        out = np.zeros(st.size, dtype=np.uint8)
        if st.size:
            self._check(self._lib.tsw_next_hop_codes(self._ctx, _u32p(st), _u32p(gl), st.size,
                                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def tswap_mapd(self, initial_positions: Sequence, tasks: Iterable, max_t: int = 2000):
        starts = np.array([[p[0], p[1]] for p in initial_positions], dtype=np.uint32).reshape(-1, 2)
        tl = []
        for t in tasks:
            pu, dl = (t.pickup, t.delivery) if isinstance(t, Task) else (t[0], t[1])
            tl.append([pu[0], pu[1], dl[0], dl[1]])
        tarr = np.array(tl, dtype=np.uint32).reshape(-1, 4)
        rec, _ = self.plan_mapd_arrays(starts, tarr, max_t)
        x = (rec & np.uint64(0xFFFF)).astype(np.int64)
        y = ((rec >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64)
        s = ((rec >> np.uint64(32)) & np.uint64(0xFF)).astype(np.int64)
        return [[((int(x[i, t]), int(y[i, t])), AgentState(int(s[i, t]))) for t in range(rec.shape[1])]
                for i in range(rec.shape[0])]

    # --- tswap_step (per tick, bin/centralized/manager.rs:101-144) ---------
    def step(self, v: np.ndarray, g: np.ndarray):
        v = np.ascontiguousarray(v, dtype=np.uint32).copy()
        g = np.ascontiguousarray(g, dtype=np.uint32).copy()
        if v.shape != g.shape:
            raise TswapError(TSW_EINVAL, "v and g must have the same length")
        self._check(self._lib.tsw_step(self._ctx, _u32p(v), _u32p(g), v.size))
        return v, g

    # --- decentralized decision (bin/decentralized/agent.rs:329-462) ----------
    def decide(self, my_v, my_g, nearby):
        """Batched compute_next_move_with_tswap. my_v, my_g: (n,) cell ids; nearby: list of n
        sequences of (cell, goal_cell) pairs (the agent's get_nearby list, self excluded, in
        order). Returns a list of (act, cell, partner, participants) with act one of
        TSW_ACT_MOVE / _GOAL_SWAP / _ROTATION / _WAIT and list indices for partner/participants."""
        my_v = np.ascontiguousarray(my_v, dtype=np.uint32)
        my_g = np.ascontiguousarray(my_g, dtype=np.uint32)
        n = my_v.size
        if my_g.size != n or len(nearby) != n:
            raise TswapError(TSW_EINVAL, "my_v, my_g and nearby must have the same length")
        off = np.zeros(n + 1, dtype=np.uint32)
        off[1:] = np.cumsum([len(x) for x in nearby]) if n else []
        flat = [p for x in nearby for p in x]
        nv = np.array([p[0] for p in flat], dtype=np.uint32)
        ng = np.array([p[1] for p in flat], dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        cell = np.zeros(n, dtype=np.uint32)
        partner = np.zeros(n, dtype=np.uint32)
        npart = np.zeros(n, dtype=np.uint32)
        part = np.zeros(int(off[-1]) + n + 1, dtype=np.uint32)
        self._check(self._lib.tsw_decide(self._ctx, _u32p(my_v), _u32p(my_g), n, _u32p(off), _u32p(nv),
                                         _u32p(ng), _u32p(act), _u32p(cell), _u32p(partner), _u32p(npart),
                                         _u32p(part)))
        out = []
        for i in range(n):
            b = int(off[i]) + i
            out.append((int(act[i]), int(cell[i]), int(partner[i]), [int(x) for x in part[b:b + npart[i]]]))
        return out

    # --- get_path -----------------------------------------------------------
    def get_path_next(self, start: np.ndarray, goal: np.ndarray):
        s = np.ascontiguousarray(start, dtype=np.uint32)
        g = np.ascontiguousarray(goal, dtype=np.uint32)
        nxt = np.zeros(s.size, dtype=np.uint32)
        ln = np.zeros(s.size, dtype=np.int32)
        self._check(self._lib.tsw_get_path_next(self._ctx, _u32p(s), _u32p(g), s.size, _u32p(nxt),
                                                ln.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return nxt, ln

    # --- K1 tables ----------------------------------------------------------
    def dist_tables(self, goals) -> np.ndarray:
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        out = np.zeros((g.size, self.h * self.w), dtype=np.uint16)
        self._check(self._lib.tsw_dist_tables(self._ctx, _u32p(g), g.size,
                                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))))
        return out

    def dist_tables_device(self, goals, dev_ptr: int):
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        self._check(self._lib.tsw_dist_tables_device(self._ctx, _u32p(g), g.size, ctypes.c_void_p(dev_ptr)))

    def import_tables_device(self, goals, dev_ptr: int):
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        self._check(self._lib.tsw_import_tables_device(self._ctx, _u32p(g), g.size, ctypes.c_void_p(dev_ptr)))

    def next_hop_tables(self, goals) -> np.ndarray:
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        out = np.zeros((g.size, self.h * self.w), dtype=np.uint8)
        self._check(self._lib.tsw_next_hop_tables(self._ctx, _u32p(g), g.size,
                                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def next_hop_tables_device(self, goals, dev_ptr: int, dist_ptr: int = 0):
        """Resolved next-hop codes of `goals` (eager A*) into device memory (len(goals) x w*h u8);
        dist_ptr (optional): their K1 distance tables too (len(goals) x w*h u16)."""
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        self._check(self._lib.tsw_next_hop_tables_device(self._ctx, _u32p(g), g.size, ctypes.c_void_p(dev_ptr),
                                                         ctypes.c_void_p(dist_ptr or None)))

    def import_next_hops_device(self, goals, dist_ptr: int, nh_ptr: int):
        """Ingest tables + next-hop codes from device memory (e.g. an all-gather of rank shards)."""
        g = np.ascontiguousarray(goals, dtype=np.uint32)
        self._check(self._lib.tsw_import_next_hops_device(self._ctx, _u32p(g), g.size, ctypes.c_void_p(dist_ptr),
                                                          ctypes.c_void_p(nh_ptr)))

    def clear_tables(self):
        self._check(self._lib.tsw_clear_tables(self._ctx))

    def stats(self) -> dict:
        s = Stats()
        self._check(self._lib.tsw_get_stats(self._ctx, ctypes.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        self._check(self._lib.tsw_reset_stats(self._ctx))

    def probe_round_floors(self, block: int = 0) -> tuple:
        """(us per wave-0 rules firing chain, us per block-wide pass) of the plan kernel's round
        shapes on a `block`-thread workgroup (0 = the last plan's): its latency floors (bench.py)."""
        out = (ctypes.c_double * 2)()
        self._check(self._lib.tsw_probe_round_floors(self._ctx, block, out))
        return float(out[0]), float(out[1])

    def set_timing(self, on: bool):
        self._check(self._lib.tsw_set_timing(self._ctx, 1 if on else 0))


def tswap_mapd(grid, initial_positions, tasks, max_t: int = 2000):
    """Drop-in for `pub fn tswap_mapd` (src/algorithm/tswap.rs:39-43)."""
    with Planner(grid) as p:
        return p.tswap_mapd(initial_positions, tasks, max_t)


def tswap_step(grid, agents_v, agents_g):
    """One `tswap_step` over cell ids (y*w+x) on a throw-away context (tests, one-off calls).

    For the centralized manager's per-tick use (plan_all_paths, bin/centralized/manager.rs:101-144)
    keep ONE `Planner` for the grid and call `Planner.step` every tick: its goal tables and resolved
    next hops persist across ticks (LRU-bounded by table_budget_bytes), where this function rebuilds
    the context — grid upload, BFS tables, A* scratch — on every call."""
    with Planner(grid) as p:
        return p.step(np.asarray(agents_v), np.asarray(agents_g))
