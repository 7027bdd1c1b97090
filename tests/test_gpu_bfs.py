"""K1 parity: the five BFS kernels (k_bfs_mg: one workgroup per group of <= 16 same-parity goals,
goal-bit-parallel; k_bfs_blk: one wavefront per goal over 8x8 blocks;
k_bfs_wave: one wavefront per goal over row words; k_bfs: one workgroup per goal over row words;
k_bfs_big: one workgroup per goal over 8x8 blocks, the large-grid kernel) against the oracle's BFS (oracle/tswap_oracle.c, cross-checked against A* path lengths in
test_oracle.py), bit-exact, on ragged widths, list-overflow paths and the full-size den520d-like
cave (BASELINE configs[3])."""
import os

import numpy as np
import pytest

from p2p_distributed_tswap_amd import Planner, maps
from oracle import OracleGraph

pytestmark = pytest.mark.gpu


class _env:
    """Kernel selection is read when a context of the DIAGNOSTIC build is created (TSW_BFS_KERNEL,
    TSW_BFS_LISTCAP, ...); the production library reads no environment and runs its default chain."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


GRIDS = {
    "open8": lambda: maps.open_map(8, 8),
    "line1x40": lambda: maps.open_map(1, 40),
    "row40x1": lambda: maps.open_map(40, 1),
    "rand33x17": lambda: maps.random_map(33, 17, 0.25, 11),
    "rand32": lambda: maps.random_map(32, 32, 0.20, 0x3232),
    "rand100x31": lambda: maps.random_map(100, 31, 0.35, 5),
    "warehouse": lambda: maps.warehouse_map(170, 84, 0x170084),
    "cave64": lambda: maps.cave_map(64, 65, 3),
    "bundled": maps.bundled_map,
    # isolated free cells at odd x: 16 run starts in every 32-cell word (decode worst case)
    "comb70x20": lambda: maps.to_rows(np.array([[(x % 2 == 0) or (y % 3 == 0) for x in range(70)]
                                                 for y in range(20)])),
}


def _check(rows, goals, **env):
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    with _env(**env), Planner(rows, diag=bool(env)) as p:
        got = p.dist_tables(goals)
    for k, g in enumerate(goals):
        ref = og.bfs(int(g))
        assert np.array_equal(got[k], ref), f"goal {g}: {np.count_nonzero(got[k] != ref)} cells differ"


def _goals(rows, n, seed):
    """Up to n distinct free cells (seeded)."""
    cells = maps.rows_to_array(rows)
    free = np.flatnonzero(cells.reshape(-1) != ord("@"))
    rng = np.random.default_rng(seed)
    return rng.choice(free, size=min(n, free.size), replace=False).astype(np.uint32)


@pytest.mark.parametrize("kernel", ["default", "mg", "blk", "wave", "block", "big"])
@pytest.mark.parametrize("name", sorted(GRIDS))
def test_bfs_kernels_bit_exact(kernel, name):
    rows = GRIDS[name]()
    if kernel == "default":  # the production library's own kernel choice
        _check(rows, _goals(rows, 40, 7))
    else:
        _check(rows, _goals(rows, 40, 7), TSW_BFS_KERNEL=kernel)


@pytest.mark.parametrize("name", sorted(GRIDS))
def test_bfs_blk_lds_west_steps(name):
    """k_bfs_blk with the west-step blocks in LDS (TSW_BFS_WLS=1: no global scratch atomics)."""
    rows = GRIDS[name]()
    _check(rows, _goals(rows, 40, 9), TSW_BFS_KERNEL="blk", TSW_BFS_WLS=1)


@pytest.mark.parametrize("wls", [0, 1])
@pytest.mark.parametrize("name", sorted(GRIDS))
def test_bfs_blk_pair(name, wls):
    """k_bfs_blk with two goals per wave, one per 32-lane half (TSW_BFS_PAIR=1). An odd goal count
    leaves the upper half of the last pair without a goal (it must write nothing)."""
    rows = GRIDS[name]()
    _check(rows, _goals(rows, 41, 13), TSW_BFS_KERNEL="blk", TSW_BFS_PAIR=1, TSW_BFS_WLS=wls)


@pytest.mark.parametrize("cap", [1, 3, 17])
def test_bfs_blk_pair_list_overflow(cap):
    """Two goals per wave with lists spilling to the per-goal-slot global overflow area; halves
    whose lists differ in length run different trip counts inside one level."""
    rows = maps.cave_map(128, 97, 9)
    _check(rows, _goals(rows, 25, 3), TSW_BFS_KERNEL="blk", TSW_BFS_BLKCAP=cap, TSW_BFS_PAIR=1)


@pytest.mark.parametrize("cap", [1, 3, 17])
def test_bfs_wave_list_overflow(cap):
    """Lists longer than the LDS capacity spill to the per-wave global overflow area."""
    rows = maps.cave_map(128, 97, 9)
    _check(rows, _goals(rows, 24, 3), TSW_BFS_KERNEL="wave", TSW_BFS_LISTCAP=cap)


@pytest.mark.parametrize("wls", [0, 1])
@pytest.mark.parametrize("cap", [1, 3, 17])
def test_bfs_blk_list_overflow(cap, wls):
    rows = maps.cave_map(128, 97, 9)
    _check(rows, _goals(rows, 24, 3), TSW_BFS_KERNEL="blk", TSW_BFS_BLKCAP=cap, TSW_BFS_WLS=wls)


@pytest.mark.parametrize("kernel", ["mg", "blk", "blk-pair", "wave", "big"])
def test_bfs_wave_unreachable_pockets(kernel):
    """Walled-off pockets stay 0xFFFF; goals inside a pocket see only the pocket."""
    a = np.zeros((40, 70), dtype=bool)
    a[10, :] = True          # full wall: two halves
    a[20:25, 30:35] = True   # closed box ...
    a[21:24, 31:34] = False  # ... with a hollow pocket
    rows = maps.to_rows(a)
    cells = maps.rows_to_array(rows)
    goals = np.array([0, 69, 11 * 70 + 5, 22 * 70 + 32, 39 * 70 + 69], dtype=np.uint32)
    assert all(cells.reshape(-1)[g] != ord("@") for g in goals)
    if kernel == "blk-pair":
        _check(rows, goals, TSW_BFS_KERNEL="blk", TSW_BFS_PAIR=1)
    else:
        _check(rows, goals, TSW_BFS_KERNEL=kernel)


class _DevBuf:
    """Device buffer from the HIP runtime the library itself links (/opt/rocm), not torch's
    bundled one: a second runtime in the process cannot open the device after the first."""

    def __init__(self, nbytes):
        import ctypes

        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.ptr = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(nbytes)) == 0
        self.nbytes = nbytes

    def to_host(self, arr):
        assert self.hip.hipDeviceSynchronize() == 0
        assert self.hip.hipMemcpy(arr.ctypes.data_as(self.ct.c_void_p), self.ptr,
                                  self.ct.c_size_t(arr.nbytes), 2) == 0  # hipMemcpyDeviceToHost
        return arr

    def __del__(self):
        self.hip.hipFree(self.ptr)


@pytest.mark.parametrize("kernel", ["mg", "blk", "blk-pair", "wave", "big"])
def test_bfs_den520d_full_size(kernel):
    """BASELINE configs[3] geometry: 256x257 cave, 1,000 distinct goals through the device-output
    entry point the bench times (16-B stores), every table bit-exact vs the oracle."""
    rows = maps.cave_map(256, 257, 0x520D)
    cells = maps.rows_to_array(rows)
    og = OracleGraph(cells)
    goals = np.sort(_goals(rows, 1000, 0x520D))
    ncell = 256 * 257
    env = dict(TSW_BFS_KERNEL="blk", TSW_BFS_PAIR=1) if kernel == "blk-pair" else dict(TSW_BFS_KERNEL=kernel)
    with _env(**env), Planner(rows, diag=True) as p:
        buf = _DevBuf(goals.size * ncell * 2)
        p.dist_tables_device(goals, buf.ptr.value)
        got = buf.to_host(np.empty((goals.size, ncell), dtype=np.uint16))
    for k, g in enumerate(goals):
        ref = og.bfs(int(g))
        assert np.array_equal(got[k], ref), f"goal {g}: {np.count_nonzero(got[k] != ref)} cells differ"


@pytest.mark.parametrize("kernel", ["mg", "blk", "wave", "big"])
def test_bfs_symmetry_full_goal_set(kernel):
    """Size-independent property at full size: d_g(c) == d_c(g) for every pair of goals, over all
    free cells of a 96x97 cave used as goals (the table matrix restricted to goals is symmetric),
    and blocked cells are 0xFFFF in every table."""
    rows = maps.cave_map(96, 97, 0x5EED)
    cells = maps.rows_to_array(rows).reshape(-1)
    free = np.flatnonzero(cells != ord("@")).astype(np.uint32)
    with _env(TSW_BFS_KERNEL=kernel), Planner(rows, diag=True) as p:
        t = p.dist_tables(free)
    sub = t[:, free].astype(np.int64)
    assert np.array_equal(sub, sub.T)
    assert np.all(t[:, cells == ord("@")] == 0xFFFF)
    assert np.all(t[np.arange(free.size), free] == 0)


def test_bfs_den520d_10k_goals_as_benched():
    """the exact launch bench.py times — 10,000 distinct den520d goals (configs[3]) in
    one tsw_dist_tables_device call of the production library — every table's sha1 against the
    oracle's (tests/golden/tables_den520d_10k.npz, made by make_digests.py den520d_10k)."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_digests import den520d_goals, table_digests

    ref = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tables_den520d_10k.npz"))
    rows, goals = den520d_goals(10000)
    assert np.array_equal(goals, ref["goals"])
    ncell = 256 * 257
    with Planner(rows) as p:
        buf = _DevBuf(goals.size * ncell * 2)
        p.dist_tables_device(goals, buf.ptr.value)
        got = buf.to_host(np.empty((goals.size, ncell), dtype=np.uint16))
    dig = table_digests(got)
    bad = np.flatnonzero(dig != ref["sha1_8"])
    assert bad.size == 0, f"{bad.size} of {goals.size} tables differ, first goal {goals[bad[0]]}"


@pytest.mark.parametrize("name,n", [("comb70x20", 300), ("rand100x31", 1500), ("cave64", 2000), ("warehouse", 700)])
def test_bfs_mg_many_groups(name, n):
    """k_bfs_mg with many groups per launch: both parities, partial groups, groups dequeued by more
    workgroups than CUs hold at once (scratch reuse across groups)."""
    rows = GRIDS[name]()
    _check(rows, _goals(rows, n, 21), TSW_BFS_KERNEL="mg")
