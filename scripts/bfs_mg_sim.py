"""CPU simulation of k_bfs_mg's ALGORITHM (not the HIP code), checked against the oracle BFS: 16 same-parity
goals per group, union-front levels, exact candidate-block marks, WL bits + run-start levels, row-word decode.
Test infrastructure (imports the oracle as the checker)."""
# CPU simulation of k_bfs_mg's algorithm (not the HIP code): per-level union processing of 16 same-parity goals,
# exact candidate marks, WL + run-start anchors, word decode. Checks against the oracle BFS.
import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/oracle')
from oracle import OracleGraph
from p2p_distributed_tswap_amd import maps

def run(rows, goals):
    cells = maps.rows_to_array(rows); H, W = cells.shape
    free = cells != ord('@')
    BW, BH = (W+7)//8, (H+7)//8; Bp = BW+1; nbp = (BH+2)*Bp
    FR = np.zeros(nbp, dtype=np.uint64)
    for y in range(H):
        for x in range(W):
            if free[y,x]: FR[((y>>3)+1)*Bp + (x>>3)] |= np.uint64(1) << np.uint64(((y&7)<<3)|(x&7))
    def isfree(p, bit): return (int(FR[p]) >> bit) & 1
    # run starts (x%32==0 or west blocked)
    def is_rs(x, y): return free[y,x] and (x % 32 == 0 or not free[y,x-1])
    out = {}
    gpar = None
    V = np.zeros((H+2, W+2), dtype=np.int64)
    WL = np.zeros((H, W), dtype=np.int64)
    AN = {}
    ng = len(goals)
    pars = {(g % W + g // W) & 1 for g in goals}; assert len(pars) == 1
    gpar = pars.pop()
    CB = [set(), set(), set()]
    for k, g in enumerate(goals):
        y, x = divmod(g, W)
        V[y+1, x+1] |= 1 << k
        if is_rs(x, y): AN[(x, y, k)] = 0
        p = ((y>>3)+1)*Bp + (x>>3)
        CB[1] |= {p, p-1, p+1, p-Bp, p+Bp}
    L = 1
    while True:
        cur = CB[L % 3]; nxt = CB[(L+1) % 3]; CB[(L+2) % 3].clear()
        lst = sorted(cur)
        if not lst: break
        P = (gpar + L) & 1
        writes = []
        for p in lst:
            by, bx = divmod(p, Bp)
            newmask = {}
            for r in range(8):
                for col in range(8):
                    if ((r + col) & 1) != P: continue
                    bit = r*8 + col
                    if not isfree(p, bit): continue
                    x = 8*bx + col; y = 8*by + r - 8
                    a = (y+1, x+1)
                    vc = V[a]; vw = V[y+1, x]; ve = V[y+1, x+2]; vn = V[y, x+1]; vs = V[y+2, x+1]
                    nw = (vw | ve | vn | vs) & ~vc & 0xFFFF
                    if nw:
                        writes.append((a, vc | nw))
                        WL[y, x] |= nw & vw
                        if is_rs(x, y):
                            for k in range(16):
                                if (nw >> k) & 1: AN[(x, y, k)] = L
                        newmask[(r, col)] = nw
            if newmask:
                nxt.add(p)
                if any(r == 0 for (r, c) in newmask): nxt.add(p - Bp)
                if any(r == 7 for (r, c) in newmask): nxt.add(p + Bp)
                if any(c == 0 for (r, c) in newmask): nxt.add(p - 1)
                if any(c == 7 for (r, c) in newmask): nxt.add(p + 1)
        for a, val in writes: V[a] = val
        L += 1
    # decode
    D = np.full((ng, H, W), 0xFFFF, dtype=np.int64)
    for y in range(H):
        for x in range(W):
            v = V[y+1, x+1]
            if not v: continue
            xr = x
            while not is_rs(xr, y): xr -= 1
            for k in range(ng):
                if not (v >> k) & 1: continue
                pc = sum((WL[y, j] >> k) & 1 for j in range(xr+1, x+1))
                D[k, y, x] = (AN[(xr, y, k)] + 2*pc - (x - xr)) & 0xFFFF
    return D, L

for name, rows in [("rand33x17", maps.random_map(33, 17, 0.25, 11)), ("cave64", maps.cave_map(64, 65, 3)),
                   ("comb", maps.to_rows(np.array([[(x % 2 == 0) or (y % 3 == 0) for x in range(70)] for y in range(20)])))]:
    cells = maps.rows_to_array(rows); H, W = cells.shape
    og = OracleGraph(cells)
    freec = np.flatnonzero(cells.reshape(-1) != ord('@'))
    rng = np.random.default_rng(3)
    for par in (0, 1):
        cand = [int(c) for c in freec if ((c % W) + (c // W)) % 2 == par]
        goals = [int(g) for g in rng.choice(cand, size=min(16, len(cand)), replace=False)]
        D, L = run(rows, goals)
        for k, g in enumerate(goals):
            ref = og.bfs(g).reshape(H, W).astype(np.int64)
            assert np.array_equal(D[k], ref), (name, par, k, np.argwhere(D[k] != ref)[:5])
    print(name, "ok, levels", L)
