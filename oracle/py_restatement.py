"""Second, independent CPU restatement of the reference TSWAP path.

TEST INFRASTRUCTURE ONLY. Used by tests/ to cross-check the C oracle
(oracle/tswap_oracle.c) on small cases — pure-Python loops, so keep inputs
small. Parity status: "parity unpinned" (see tswap_oracle.h).

Written deliberately in a different shape from the C oracle so that a shared
misreading is less likely: it keeps the reference's own node numbering
(row-major over free cells, tswap.rs:51-59), dict-based g_score/came_from
(tswap.rs:324-325) and a class that mirrors Rust's std BinaryHeap method by
method (push/pop/sift_up/sift_down_to_bottom with the Hole semantics).
Points are (x, y) with y = row (grid[y][x], tswap.rs:53).
"""
from __future__ import annotations

PICKING, CARRYING, DELIVERED, IDLE = 0, 1, 2, 3  # src/map/agent.rs:9-15


class _Node:
    __slots__ = ("node_id", "g_cost", "f_cost")

    def __init__(self, node_id, g_cost, f_cost):
        self.node_id = node_id
        self.g_cost = g_cost
        self.f_cost = f_cost

    def cmp(self, other) -> int:
        """AstarNode::cmp (tswap.rs:314-321): other.f.cmp(self.f).then(other.g.cmp(self.g))."""
        if other.f_cost != self.f_cost:
            return -1 if other.f_cost < self.f_cost else 1
        if other.g_cost != self.g_cost:
            return -1 if other.g_cost < self.g_cost else 1
        return 0

    def le(self, other) -> bool:
        return self.cmp(other) <= 0


class RustBinaryHeap:
    """std::collections::BinaryHeap (max-heap) restated from its documented algorithm."""

    def __init__(self):
        self.data = []

    def push(self, item):
        old_len = len(self.data)
        self.data.append(item)
        self._sift_up(0, old_len)

    def pop(self):
        if not self.data:
            return None
        item = self.data.pop()
        if self.data:
            item, self.data[0] = self.data[0], item
            self._sift_down_to_bottom(0)
        return item

    def _sift_up(self, start, pos):
        data = self.data
        elem = data[pos]
        while pos > start:
            parent = (pos - 1) // 2
            if elem.le(data[parent]):
                break
            data[pos] = data[parent]
            pos = parent
        data[pos] = elem
        return pos

    def _sift_down_to_bottom(self, pos):
        data = self.data
        end = len(data)
        start = pos
        elem = data[pos]
        child = 2 * pos + 1
        while child <= max(end - 2, 0):
            if data[child].le(data[child + 1]):
                child += 1
            data[pos] = data[child]
            pos = child
            child = 2 * pos + 1
        if child == end - 1:
            data[pos] = data[child]
            pos = child
        data[pos] = elem
        self._sift_up(start, pos)


class Graph:
    """Node graph exactly as tswap.rs:44-77 builds it."""

    def __init__(self, grid):
        self.h = len(grid)
        self.w = len(grid[0])
        self.pos2id = {}
        self.id2pos = []
        for y in range(self.h):
            for x in range(self.w):
                if grid[y][x] != "@":
                    self.pos2id[(x, y)] = len(self.id2pos)
                    self.id2pos.append((x, y))
        self.neighbors = []
        for (x, y) in self.id2pos:
            nbs = []
            for dx, dy in ((0, 1), (1, 0), (0, -1), (-1, 0)):
                nx, ny = x + dx, y + dy
                if nx >= 0 and ny >= 0 and (nx, ny) in self.pos2id:
                    nbs.append(self.pos2id[(nx, ny)])
            self.neighbors.append(nbs)
        self.pops = 0

    def get_path(self, start, goal):
        """tswap.rs:288-390; returns the full path (list of node ids)."""
        if start == goal:
            return [start]
        gx, gy = self.id2pos[goal]

        def heuristic(nid):
            x, y = self.id2pos[nid]
            return abs(x - gx) + abs(y - gy)

        open_list = RustBinaryHeap()
        came_from = {}
        g_score = {start: 0}
        open_list.push(_Node(start, 0, heuristic(start)))
        while True:
            current = open_list.pop()
            if current is None:
                break
            self.pops += 1
            cid = current.node_id
            if cid == goal:
                path = [cid]
                node = cid
                while node in came_from:
                    node = came_from[node]
                    path.append(node)
                path.reverse()
                return path
            for nb in self.neighbors[cid]:
                tg = current.g_cost + 1
                if tg < g_score.get(nb, float("inf")):
                    came_from[nb] = cid
                    g_score[nb] = tg
                    open_list.push(_Node(nb, tg, tg + heuristic(nb)))
        best = start
        min_dist = heuristic(start)
        for nb in self.neighbors[start]:
            d = heuristic(nb)
            if d < min_dist:
                min_dist = d
                best = nb
        return [start, best]


def tswap_step(agents, graph: Graph):
    """tswap.rs:174-286. agents: list of [v, g] node ids (mutated in place)."""
    n = len(agents)

    def position(u):
        for k, a in enumerate(agents):
            if a[0] == u:
                return k
        return None

    for i in range(n):
        if agents[i][0] == agents[i][1]:
            continue
        path = graph.get_path(agents[i][0], agents[i][1])
        if len(path) < 2:
            continue
        u = path[1]
        j = position(u)
        if j is None or j == i:
            continue
        if agents[j][0] == agents[j][1]:
            agents[i][1], agents[j][1] = agents[j][1], agents[i][1]
        else:
            a_p = [i]
            cur = j
            found = False
            while True:
                bv, bg = agents[cur]
                if bv == bg:
                    break
                bpath = graph.get_path(bv, bg)
                if len(bpath) < 2:
                    break
                c = position(bpath[1])
                if c is None:
                    break
                if cur in a_p:
                    a_p.clear()
                    break
                a_p.append(cur)
                cur = c
                if cur == i:
                    found = True
                    break
            if found and len(a_p) > 1:
                first = a_p[0]
                last_goal = agents[a_p[-1]][1]
                for k in range(len(a_p) - 1, 0, -1):
                    agents[a_p[k]][1] = agents[a_p[k - 1]][1]
                agents[first][1] = last_goal
    for i in range(n):
        if agents[i][0] == agents[i][1]:
            continue
        path = graph.get_path(agents[i][0], agents[i][1])
        if len(path) < 2:
            continue
        u = path[1]
        j = position(u)
        if j is not None:
            if i != j:
                pj = graph.get_path(agents[j][0], agents[j][1])
                if len(pj) >= 2 and pj[1] == agents[i][0]:
                    agents[i][0], agents[j][0] = agents[j][0], agents[i][0]
        else:
            agents[i][0] = u


def tswap_mapd(grid, initial_positions, tasks, max_t=2000, trace_goals=None):
    """tswap.rs:39-172. tasks: list of ((px,py),(dx,dy)). Returns paths[i] = [((x,y), state)]."""
    graph = Graph(grid)
    n = len(initial_positions)
    paths = [[] for _ in range(n)]
    used = [False] * len(tasks)
    st = ["idle"] * n
    atask = [None] * n
    agents = [[graph.pos2id[p], graph.pos2id[p]] for p in initial_positions]
    t = 0
    while True:
        for i in range(n):
            if agents[i][0] == agents[i][1]:
                if st[i] == "pickup":
                    st[i] = "delivery"
                    if atask[i] is not None:
                        agents[i][1] = graph.pos2id[atask[i][1]]
                elif st[i] == "delivery":
                    st[i] = "idle"
                    atask[i] = None
            if st[i] == "idle":
                cx, cy = graph.id2pos[agents[i][0]]
                best = None
                for k, task in enumerate(tasks):
                    if used[k]:
                        continue
                    d = abs(cx - task[0][0]) + abs(cy - task[0][1])
                    if best is None or d < best[1]:
                        best = (k, d)
                if best is not None:
                    used[best[0]] = True
                    atask[i] = tasks[best[0]]
                    st[i] = "pickup"
                    agents[i][1] = graph.pos2id[tasks[best[0]][0]]
        tswap_step(agents, graph)
        for i in range(n):
            pos = graph.id2pos[agents[i][0]]
            if st[i] == "idle":
                s = IDLE
            elif st[i] == "pickup":
                s = PICKING
            else:
                s = DELIVERED if agents[i][0] == agents[i][1] else CARRYING
            paths[i].append((pos, s))
            if trace_goals is not None:
                trace_goals.setdefault(i, []).append(graph.id2pos[agents[i][1]])
        t += 1
        if (all(used) and all(s == "idle" for s in st)) or t > max_t:
            break
    return paths


def compute_next_move_with_tswap(my_pos, my_goal, nearby, graph: Graph):
    """src/bin/decentralized/agent.rs:329-462, with POSITIONS (x, y). nearby: list of
    (current_pos, goal_pos) in get_nearby order (self excluded). Returns (kind, payload):
    ("move", pos) | ("swap", list index) | ("rotation", [list indices]) | ("wait", None)."""
    def find(pos):  # nearby_agents.iter().find(|a| a.current_pos == pos)
        for k, a in enumerate(nearby):
            if a[0] == pos:
                return k
        return None

    if my_pos == my_goal:  # Rule 1
        return ("move", my_pos)
    path = graph.get_path(graph.pos2id[my_pos], graph.pos2id[my_goal])
    if len(path) < 2:
        return ("move", my_pos)
    next_pos = graph.id2pos[path[1]]
    b = find(next_pos)
    if b is None:  # Rule 2
        return ("move", next_pos)
    if nearby[b][0] == nearby[b][1]:  # Rule 3
        return ("swap", b)
    a_p = [my_pos]  # Rule 4
    cur = b
    found = False
    while True:
        cpos, cgoal = nearby[cur]
        if cpos == cgoal:
            break
        if cpos not in graph.pos2id or cgoal not in graph.pos2id:
            break
        ap = graph.get_path(graph.pos2id[cpos], graph.pos2id[cgoal])
        if len(ap) < 2:
            break
        nd = graph.id2pos[ap[1]]
        nx = find(nd)
        if nx is None:
            break
        if nearby[nx][0] in a_p:
            if nearby[nx][0] == my_pos:
                found = True
            else:
                a_p.clear()
            break
        a_p.append(cpos)
        cur = nx
    if found and len(a_p) > 1:
        parts = [find(p) for p in a_p]
        parts = [k for k in parts if k is not None]
        if len(parts) > 1:
            return ("rotation", parts)
        return ("wait", None)
    return ("wait", None)
