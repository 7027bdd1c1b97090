"""Seeded synthetic MovingAI-style grids and MAPD instances.

The reference draws starts/tasks with unseeded thread_rng (src/map/make_node.rs:22-49,
src/map/task_generator.rs:23); every instance here is reproducible from a seed
through a self-contained splitmix64 stream, so fixtures never depend on a
library's RNG version. '.' = passable, '@' = blocked (the only blocked char the
reference recognises, tswap.rs:53). Starts and tasks are drawn from the largest
4-connected component so that no task is unreachable.
"""
from __future__ import annotations

from collections import deque

import numpy as np

MASK64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next_u64(self) -> int:
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def uniform(self) -> float:
        return (self.next_u64() >> 11) * (1.0 / (1 << 53))

    def below(self, n: int) -> int:
        return self.next_u64() % n

    def shuffle(self, a: list) -> None:
        for i in range(len(a) - 1, 0, -1):
            j = self.below(i + 1)
            a[i], a[j] = a[j], a[i]


def to_rows(arr: np.ndarray) -> list:
    return ["".join("@" if b else "." for b in row) for row in arr]


def rows_to_blocked(rows) -> np.ndarray:
    return np.array([[c == "@" for c in r] for r in rows], dtype=bool)


def bundled_map() -> list:
    """src/map/map.rs MAP: 100 rows x 100 '.' (parse_map, bin/centralized/manager.rs:25-34)."""
    return ["." * 100 for _ in range(100)]


def open_map(w: int, h: int) -> list:
    return ["." * w for _ in range(h)]


def random_map(w: int, h: int, p: float, seed: int) -> list:
    """Bernoulli(p) obstacles (random-32-32-20 style)."""
    r = SplitMix64(seed)
    blocked = np.zeros((h, w), dtype=bool)
    for y in range(h):
        for x in range(w):
            blocked[y, x] = r.uniform() < p
    return to_rows(blocked)


def warehouse_map(w: int = 170, h: int = 84, seed: int = 0x170084) -> list:
    """Shelf blocks (2 rows x 10 cols) separated by 1-wide aisles, 2-cell border corridor."""
    r = SplitMix64(seed)
    blocked = np.zeros((h, w), dtype=bool)
    y = 2
    while y + 2 <= h - 2:
        x = 2
        while x + 10 <= w - 2:
            blocked[y:y + 2, x:x + 10] = True
            # occasional gap in a shelf row (cross aisle), seeded
            if r.uniform() < 0.1:
                gx = x + int(r.below(10))
                blocked[y:y + 2, gx] = False
            x += 11
        y += 3
    return to_rows(blocked)


def cave_map(w: int = 256, h: int = 257, seed: int = 0x520D, fill: float = 0.45, iters: int = 5) -> list:
    """den520d-like cave: cellular automaton (4-5 rule) on a seeded random fill."""
    r = SplitMix64(seed)
    a = np.zeros((h, w), dtype=bool)
    for y in range(h):
        for x in range(w):
            a[y, x] = r.uniform() < fill
    a[0, :] = a[-1, :] = True
    a[:, 0] = a[:, -1] = True
    for _ in range(iters):
        p = np.pad(a, 1, constant_values=True)
        cnt = sum(p[1 + dy:1 + dy + h, 1 + dx:1 + dx + w].astype(np.int32)
                  for dy in (-1, 0, 1) for dx in (-1, 0, 1) if (dy, dx) != (0, 0))
        a = np.where(a, cnt >= 4, cnt >= 5)
        a[0, :] = a[-1, :] = True
        a[:, 0] = a[:, -1] = True
    return to_rows(a)


def sortation_map(w: int = 1024, h: int = 1024) -> list:
    """Sortation floor: 1-cell chutes (blocked) on a 4-pitch lattice, open aisles between."""
    a = np.zeros((h, w), dtype=bool)
    a[2:h - 2:4, 2:w - 2:4] = True
    return to_rows(a)


def largest_component(rows) -> list:
    """Cells (x, y) of the largest 4-connected free component, row-major order (ties: the
    component met first in row-major order)."""
    blocked = rows_to_blocked(rows)
    h, w = blocked.shape
    try:
        from scipy import ndimage
    except ImportError:  # pragma: no cover - scipy is in the image; the loop below is the fallback
        ndimage = None
    if ndimage is not None:
        lab, nlab = ndimage.label(~blocked)  # default structure = 4-connectivity in 2-D
        if nlab == 0:
            return []
        sizes = np.bincount(lab.reshape(-1))[1:]
        best_id = int(np.argmax(sizes)) + 1  # labels are numbered in raster order of first cell
        ys, xs = np.nonzero(lab == best_id)
        return [(int(x), int(y)) for y, x in zip(ys, xs)]
    comp = -np.ones((h, w), dtype=np.int64)
    best, best_id, cid = 0, -1, 0
    for sy in range(h):
        for sx in range(w):
            if blocked[sy, sx] or comp[sy, sx] >= 0:
                continue
            q = deque([(sx, sy)])
            comp[sy, sx] = cid
            size = 0
            while q:
                x, y = q.popleft()
                size += 1
                for dx, dy in ((0, 1), (1, 0), (0, -1), (-1, 0)):
                    nx, ny = x + dx, y + dy
                    if 0 <= nx < w and 0 <= ny < h and not blocked[ny, nx] and comp[ny, nx] < 0:
                        comp[ny, nx] = cid
                        q.append((nx, ny))
            if size > best:
                best, best_id = size, cid
            cid += 1
    ys, xs = np.nonzero(comp == best_id)
    return [(int(x), int(y)) for y, x in zip(ys, xs)]


def make_instance(rows, n_agents: int, n_tasks: int, seed: int):
    """n distinct start cells and n_tasks (pickup != delivery) pairs, seeded.

    Returns (starts (n,2) uint32, tasks (m,4) uint32 [px,py,dx,dy]).
    """
    cells = largest_component(rows)
    r = SplitMix64(seed ^ 0xA5A5A5A5)
    pool = list(cells)
    r.shuffle(pool)
    if n_agents > len(pool):
        raise ValueError("more agents than free cells")
    starts = np.array(pool[:n_agents], dtype=np.uint32).reshape(-1, 2)
    tasks = np.zeros((n_tasks, 4), dtype=np.uint32)
    nc = len(cells)
    for k in range(n_tasks):
        a = r.below(nc)
        b = r.below(nc - 1)
        if b >= a:
            b += 1
        tasks[k] = (*cells[a], *cells[b])
    return starts, tasks


def rows_to_array(rows) -> np.ndarray:
    return np.frombuffer("".join(rows).encode("latin-1"), dtype=np.uint8).reshape(len(rows), len(rows[0])).copy()


# ---- map text / MovingAI I/O --------------------------
def parse_map(text: str) -> list:
    """The reference's parse_map (src/bin/centralized/manager.rs:25-34): every '\\r' removed,
    lines split, lines that are blank after trimming dropped, each kept line's characters as a
    row (no other trimming). Rows must come out equally long for the C ABI (the reference
    indexes grid[y][x] for x < grid[0].len(), tswap.rs:51-56, and panics on a short row)."""
    rows = [ln for ln in text.replace("\r", "").splitlines() if ln.strip()]
    if rows and any(len(r) != len(rows[0]) for r in rows):
        raise ValueError("ragged map: every row must be as long as the first (tswap.rs:51-56)")
    return rows


def read_scen(path: str):
    """MovingAI .scen (\"version 1\" header; per line: bucket map width height sx sy gx gy
    optimal). Returns (starts (n,2) uint32, goals (n,2) uint32, optimal (n,) float64) as
    (x, y) points — the Point convention of src/map/map.rs:4 (x = column, y = row)."""
    st, gl, opt = [], [], []
    with open(path) as f:
        for ln in f:
            parts = ln.split()
            if len(parts) < 9 or parts[0].lower() == "version":
                continue
            sx, sy, gx, gy = (int(v) for v in parts[4:8])
            st.append((sx, sy))
            gl.append((gx, gy))
            opt.append(float(parts[8]))
    return (np.array(st, dtype=np.uint32).reshape(-1, 2), np.array(gl, dtype=np.uint32).reshape(-1, 2),
            np.array(opt, dtype=np.float64))


def write_scen(path: str, map_name: str, rows, starts, goals, optimal=None) -> None:
    h, w = len(rows), len(rows[0])
    with open(path, "w") as f:
        f.write("version 1\n")
        for i, ((sx, sy), (gx, gy)) in enumerate(zip(starts, goals)):
            o = float(optimal[i]) if optimal is not None else 0.0
            f.write(f"0\t{map_name}\t{w}\t{h}\t{sx}\t{sy}\t{gx}\t{gy}\t{o:.8f}\n")


# ---- MovingAI .map files ------------------------------------------------------
def write_movingai(path: str, rows) -> None:
    with open(path, "w") as f:
        f.write("type octile\n")
        f.write(f"height {len(rows)}\n")
        f.write(f"width {len(rows[0])}\n")
        f.write("map\n")
        for r in rows:
            f.write(r + "\n")


def read_movingai(path: str, passable: str = ".GS") -> list:
    """Reads a MovingAI map; any char not in `passable` becomes '@' (blocked)."""
    with open(path) as f:
        lines = [ln.rstrip("\r\n") for ln in f]
    i = lines.index("map")
    rows = [ln for ln in lines[i + 1:] if ln.strip()]
    return ["".join(c if c in passable else "@" for c in r).replace("G", ".").replace("S", ".") for r in rows]


def make_window_instance(rows, n_agents: int, n_tasks: int, seed: int, x0: int, y0: int, w: int, h: int):
    """As make_instance, but starts and task cells are drawn from the window [x0, x0+w) x [y0, y0+h)
    of the largest component: dense traffic (C5 — "dense rotation cycles") on a large floor."""
    cells = [c for c in largest_component(rows) if x0 <= c[0] < x0 + w and y0 <= c[1] < y0 + h]
    r = SplitMix64(seed ^ 0x5A5A5A5A)
    pool = list(cells)
    r.shuffle(pool)
    if n_agents > len(pool):
        raise ValueError("more agents than free cells in the window")
    starts = np.array(pool[:n_agents], dtype=np.uint32).reshape(-1, 2)
    tasks = np.zeros((n_tasks, 4), dtype=np.uint32)
    nc = len(cells)
    for k in range(n_tasks):
        a = r.below(nc)
        b = r.below(nc - 1)
        if b >= a:
            b += 1
        tasks[k] = (*cells[a], *cells[b])
    return starts, tasks


def make_wf_instance(rows, n_agents: int, n_tasks: int, seed: int, window=None):
    """Well-formed MAPD instance (round 5): n distinct start (parking) cells, and
    n_tasks (pickup != delivery) pairs whose endpoints are drawn from the OTHER free cells of the
    largest component (optionally of the window (x0, y0, w, h)), so no task endpoint is a start cell.

    Why it matters for the reference loop: an Idle agent keeps g = v (tswap.rs:92-101, :119-121);
    an agent whose goal is the cell such an agent rests on gets a rule-3 swap of two EQUAL goals
    (tswap.rs:198-202), a no-op, and the plan spins to `timestep > 2000` (:167) with nothing moving.
    With endpoints disjoint from the parking cells and a task stream that outlasts the horizon (an
    agent that delivers takes its next task in the same ASSIGN pass, :119-139), no agent parks and
    every timestep moves agents. Returns (starts (n,2) uint32, tasks (m,4) uint32 [px,py,dx,dy])."""
    cells = largest_component(rows)
    if window is not None:
        x0, y0, w, h = window
        cells = [c for c in cells if x0 <= c[0] < x0 + w and y0 <= c[1] < y0 + h]
    r = SplitMix64(seed ^ 0xC3C3C3C3)
    pool = list(cells)
    r.shuffle(pool)
    if n_agents + 2 > len(pool):
        raise ValueError("more agents than free cells (two task endpoints must remain)")
    starts = np.array(pool[:n_agents], dtype=np.uint32).reshape(-1, 2)
    ep = pool[n_agents:]
    ne = len(ep)
    tasks = np.zeros((n_tasks, 4), dtype=np.uint32)
    for k in range(n_tasks):
        a = r.below(ne)
        b = r.below(ne - 1)
        if b >= a:
            b += 1
        tasks[k] = (*ep[a], *ep[b])
    return starts, tasks


C5_WINDOW = (432, 432, 160, 160)


def c5_instance(n_agents: int = 10000, n_tasks: int = 24000, seed: int = 0x1024):
    """C5 (BASELINE configs[4]): the 1024x1024 sortation floor, agents and task cells packed
    into the central 160x160 window (~24k free cells, 10k agents = ~42% occupancy): dense traffic,
    rule-3 swaps and rule-4 rotation cycles every step. Well-formed (make_wf_instance) with a
    24,000-task stream: ~10k deliveries in 2,001 steps, so the stream outlasts the horizon and every
    timestep moves agents. Returns (rows, starts, tasks)."""
    rows = sortation_map(1024, 1024)
    starts, tasks = make_wf_instance(rows, n_agents, n_tasks, seed, C5_WINDOW)
    return rows, starts, tasks


def wh10k_instance(n_agents: int = 10000, n_tasks: int = 40000, seed: int = 0x510220):
    """The north_star's "10k-agent warehouse": the warehouse generator at 510x220 (shelf blocks,
    1-wide aisles), 10,000 agents, a well-formed 40,000-task MAPD stream (outlasts 2,001 steps).
    Returns (rows, starts, tasks)."""
    rows = warehouse_map(510, 220, seed)
    starts, tasks = make_wf_instance(rows, n_agents, n_tasks, seed)
    return rows, starts, tasks


# ---- round-1..4 instances (kept as extra parity tests) -------------------------------------
# Task endpoints drawn from all free cells (start cells included) and streams shorter than the
# horizon: the plans freeze once the stream is spent (C3 from t = 446, C5 from t = 152, wh10k from
# t = 1,282 — VERDICT r4 missing #1). Their full-horizon digests stay committed.
def c5_legacy_instance(n_agents: int = 10000, n_tasks: int = 10000, seed: int = 0x1024):
    rows = sortation_map(1024, 1024)
    starts, tasks = make_window_instance(rows, n_agents, n_tasks, seed, *C5_WINDOW)
    return rows, starts, tasks


def wh10k_legacy_instance(n_agents: int = 10000, n_tasks: int = 30000, seed: int = 0x510220):
    rows = warehouse_map(510, 220, seed)
    starts, tasks = make_instance(rows, n_agents, n_tasks, seed)
    return rows, starts, tasks


def c2_legacy_instance():
    """Round 1-5 C2: 600 tasks drawn from all free cells (parking cells included); the plan spins to the
    cap with only 180 of its 2,000 transitions moving an agent (VERDICT r5 missing #3)."""
    rows = random_map(32, 32, 0.20, 0x3232)
    starts, tasks = make_instance(rows, 200, 600, 0x3232)
    return rows, starts, tasks


def c3_legacy_instance():
    rows = warehouse_map(170, 84, 0x170084)
    starts, tasks = make_instance(rows, 1000, 3000, 0x170084)
    return rows, starts, tasks


CONFIGS = {
    # name: (map factory, n_agents, n_tasks, instance seed)  — BASELINE.json configs
    "c1_bundled_10": (bundled_map, 10, 30, 1),
    # well-formed (round 6), 16,000-task stream: ~10.2k assignments in 2,001 steps, every
    # timestep moves agents (the round-1..5 600-task instance is c2_legacy_instance: 180 of 2,000 move)
    "c2_random_32_32_20": (lambda: random_map(32, 32, 0.20, 0x3232), 200, 16000, 0x3232),
    # well-formed, 32,000-task stream: ~24k deliveries in 2,001 steps, every timestep moves agents
    "c3_warehouse_170x84": (lambda: warehouse_map(170, 84, 0x170084), 1000, 32000, 0x170084),
    # K1-only config: 10,000 distinct goal cells (BFS tables), goal-sharded over 2/4/8 GPUs
    "c4_den520d_10k_goals": (lambda: cave_map(256, 257, 0x520D), 0, 0, 0x520D),
    # dense MAPD on the sortation floor: instance from c5_instance() (window-packed, not make_instance)
    "c5_sortation_1024_10k": (lambda: sortation_map(1024, 1024), 10000, 24000, 0x1024),
}
# configs whose instance is well-formed (make_wf_instance)
WELL_FORMED = {"c2_random_32_32_20", "c3_warehouse_170x84", "c5_sortation_1024_10k"}
# distinct K1 goals of the table-build configs
CONFIG_GOALS = {"c4_den520d_10k_goals": 10000, "c5_sortation_1024_10k": 10000}


def config_instance(name: str, seed_offset: int = 0):
    """(rows, starts, tasks) of a MAPD config of CONFIGS; seed_offset draws another instance of the same
    shape on the same map (bench.py's replicas: seed + rank)."""
    fac, n, m, seed = CONFIGS[name]
    if name == "c5_sortation_1024_10k":
        return c5_instance(n, m, seed + seed_offset)
    rows = fac()
    if name in WELL_FORMED:
        starts, tasks = make_wf_instance(rows, n, m, seed + seed_offset)
    else:
        starts, tasks = make_instance(rows, n, m, seed + seed_offset)
    return rows, starts, tasks


def moving_timesteps(rec: np.ndarray) -> int:
    """Timesteps t >= 1 of a plan (records (n, T), x | y<<16 | state<<32) in which at least one agent's
    position differs from t - 1 (report how much of a horizon actually plans)."""
    pos = np.asarray(rec, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    if pos.shape[1] < 2:
        return 0
    return int(np.count_nonzero((pos[:, 1:] != pos[:, :-1]).any(axis=0)))
