"""Lane-level model of the wave-cooperative BinaryHeap operations in csrc/tsw_astar.h, checked
against Rust's std BinaryHeap semantics (push = sift_up; pop = swap the last element into the root,
sift_down_to_bottom, sift_up), which the reference's A* (src/algorithm/tswap.rs:323-374) relies on
for its tie-break.

The kernels cannot run here, so this test pins the round-4 rewrites at the level of the per-lane
arithmetic they perform (same address formulas, same ballots), with many equal keys:
  * wpop fused with the sift_up of the last element: the path below the first node the last
    element does not pass is left untouched, so the pop stops there and never re-reads the path;
  * a batched push (measured and not kept: A* relaxations average 1.04 pushes per pop, so
    batching had nothing to batch — profiles/r4/astar_latency.txt): up to four consecutive pushes
    from one read of all their root paths (lane group g = lane >> 4 holds push g's ancestors,
    lane & 15 = depth), the sift_ups applied in registers in push order, one write per node.
    Kept here as the model of that variant.
CPU only; pure Python.
"""
import random

import pytest


def key(e):
    return e[0]


# ---------------------------------------------------------------- Rust BinaryHeap (min on key)
def ref_sift_up(H, pos):
    elem = H[pos]
    while pos > 0:
        parent = (pos - 1) // 2
        if key(elem) >= key(H[parent]):  # hole.element() <= hole.get(parent) in Ord
            break
        H[pos] = H[parent]
        pos = parent
    H[pos] = elem


def ref_push(H, e):
    H.append(e)
    ref_sift_up(H, len(H) - 1)


def ref_pop(H):
    item = H.pop()
    if H:
        item, H[0] = H[0], item
        end = len(H)
        pos, elem = 0, H[0]
        child = 1
        while child <= max(end - 2, 0) and end >= 2:
            child += 1 if key(H[child]) >= key(H[child + 1]) else 0  # get(child) <= get(child+1)
            H[pos] = H[child]
            pos = child
            child = 2 * pos + 1
        if child == end - 1:
            H[pos] = H[child]
            pos = child
        H[pos] = elem
        ref_sift_up(H, pos)
    return item


# ---------------------------------------------------------------- lane model of wpop (fused)
def log2(x):
    return x.bit_length() - 1


def win_lane(lane):
    if lane >= 62:
        return None
    kk = log2(lane + 2)
    ki = lane + 2 - (1 << kk)
    one = zero = 0
    for a in range(kk):
        lc = (2 << a) - 2 + 2 * (ki >> (kk - a))
        if (ki >> (kk - a - 1)) & 1:
            one |= 1 << lc
        else:
            zero |= 1 << lc
    return one, zero


WL = [win_lane(l) for l in range(64)]


def model_wpop(H, length):
    """H has at least `length` entries (index `length - 1` = the last); returns (top, new length)."""
    end = length - 1
    last, top = H[end], H[0]
    if end == 0:
        return last, 0
    klast = key(last)
    pos = 0
    while True:
        node, val, ex = [0] * 64, [None] * 64, [False] * 64
        for l in range(62):
            kk = log2(l + 2)
            ki = l + 2 - (1 << kk)
            node[l] = ((pos + 1) << kk) - 1 + ki
            val[l] = H[min(node[l], end)]
            ex[l] = node[l] < end
        VL = sum(1 << l for l in range(62) if ex[l])
        CR = 0
        for l in range(0, 62, 2):  # left-child lanes: right child taken when left >= right and it exists
            if key(val[l]) >= key(val[l + 1]) and (VL >> (l + 1)) & 1:
                CR |= 1 << l
        on = [l < 62 and ex[l] and (CR & WL[l][0]) == WL[l][0] and (CR & WL[l][1]) == 0 for l in range(64)]
        PM = sum(1 << l for l in range(64) if on[l])
        if PM == 0:
            break
        LE = sum(1 << l for l in range(62) if key(val[l]) <= klast)
        PU = PM & LE
        if PU != PM:  # the last element stops inside this window
            tgt = pos
            if PU:
                lu = log2(PU)
                d = log2(lu + 2)
                tgt = ((pos + 1) << d) - 1 + (lu + 2 - (1 << d))
            for l in range(62):
                if (PU >> l) & 1:
                    H[(node[l] - 1) >> 1] = val[l]
            H[tgt] = last
            return top, end
        lt = log2(PM)
        d = log2(lt + 2)
        for l in range(62):
            if on[l]:
                H[(node[l] - 1) >> 1] = val[l]
        pos = ((pos + 1) << d) - 1 + (lt + 2 - (1 << d))
        if d < 5:
            break
    H[pos] = last
    return top, end


# ---------------------------------------------------------------- lane model of wpush_batch
def model_push_batch(H, length, elems):
    """Pushes elems (1..4, in order) at positions length.. from one read of their root paths."""
    np_ = len(elems)
    p0 = length
    a, addr, live = [None] * 64, [0] * 64, [False] * 64
    for l in range(64):
        g, j = l >> 4, l & 15
        pg = p0 + g
        dg = log2(pg + 1)
        live[l] = g < np_ and j <= dg
        addr[l] = ((pg + 1) >> (dg - j)) - 1 if live[l] else 0
        a[l] = H[addr[l]] if addr[l] < len(H) else ("hole",)  # a hole lane's read is garbage
    mod = [False] * 64
    for k, ek in enumerate(elems):
        pk = p0 + k
        dk = log2(pk + 1)
        G = 0
        for l in range(64):
            g, j = l >> 4, l & 15
            if g == k and j < dk and key(ek) < key(a[l]):
                G |= 1 << l
        t = dk - bin(G).count("1")
        new = list(a)
        for l in range(64):
            g, j = l >> 4, l & 15
            onk = live[l] and g >= k and j <= dk and ((pk + 1) >> (dk - j)) - 1 == addr[l]
            if not onk or j < t:
                continue
            up = a[l - 1] if j > 0 else None  # DPP row_shr:1 within the 16-lane row
            new[l] = ek if j == t else up
            mod[l] = True
        a = new
    while len(H) < p0 + np_:
        H.append(None)
    for l in range(64):
        g, j = l >> 4, l & 15
        if not (live[l] and mod[l]):
            continue
        last_holder = all(
            ((p0 + h + 1) >> (log2(p0 + h + 1) - j)) - 1 != addr[l] for h in range(g + 1, np_)
        )
        if last_holder:
            H[addr[l]] = a[l]
    return p0 + np_


def test_model_matches_binary_heap():
    rng = random.Random(1234)
    for trial in range(300):
        kr = rng.choice([2, 3, 5, 40])  # small key ranges: ties everywhere
        R, M = [], []
        uid = 0
        for op in range(rng.randrange(20, 600)):
            if R and rng.random() < 0.45:
                top_r = ref_pop(R)
                top_m, n = model_wpop(M, len(M))
                del M[n:]
                assert top_m == top_r, (trial, op)
                assert M == R, (trial, op)
            else:
                k = rng.randrange(1, 5) if rng.random() < 0.8 else 1
                elems = []
                for _ in range(k):
                    uid += 1
                    elems.append((rng.randrange(kr), uid))
                for e in elems:
                    ref_push(R, e)
                n = model_push_batch(M, len(M), elems)
                assert n == len(R) and M == R, (trial, op, k)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7])
def test_model_small_heaps(n):
    """Tiny heaps: a later push's hole can be an earlier push's parent (p0 <= 2)."""
    rng = random.Random(n)
    for trial in range(400):
        R = []
        for i in range(n):
            ref_push(R, (rng.randrange(3), i))
        M = list(R)
        elems = [(rng.randrange(3), 100 + i) for i in range(rng.randrange(1, 5))]
        for e in elems:
            ref_push(R, e)
        model_push_batch(M, len(M), elems)
        assert M == R
        while R:
            assert model_wpop(M, len(M))[0] == ref_pop(R)
            del M[len(R):]
            assert M == R


def test_model_deep_heap():
    """Depth up to 12 (the 4,096-entry LDS heap): three pop windows, 13-deep push paths."""
    rng = random.Random(7)
    R, M, uid = [], [], 0
    while len(R) < 4000:
        elems = []
        for _ in range(rng.randrange(1, 5)):
            uid += 1
            elems.append((rng.randrange(60), uid))
        for e in elems:
            ref_push(R, e)
        model_push_batch(M, len(M), elems)
        if rng.random() < 0.2:
            assert model_wpop(M, len(M))[0] == ref_pop(R)
            del M[len(R):]
    assert M == R
    while R:
        assert model_wpop(M, len(M))[0] == ref_pop(R)
        del M[len(R):]
    assert not M


# ---------------------------------------------------------------- register-resident heap (round 4)
# Heaps of <= 63 entries live in one 64-bit VGPR pair across the wave: node 0 (the root) in lane 63,
# node n in 1..62 in lane n - 1 — the first pop window's own layout, so siblings are lane pairs
# (2i, 2i + 1) and the path test is the same WinLane test. Values move along a path with one
# ds_bpermute (pull from the chosen child / from the parent), not an LDS round trip.
NONE = 0xFFFF


def lane_of(n):
    return 63 if n == 0 else n - 1


def reg_lane(lane):
    node = 0 if lane == 63 else (NONE if lane == 62 else lane + 1)
    depth = log2(node + 1) if node != NONE else 15
    plane = lane_of((node - 1) >> 1) if node not in (0, NONE) else lane
    cl = lane_of(2 * node + 1) if node != NONE and node <= 30 else 63
    return node, depth, plane, cl


RL = [reg_lane(l) for l in range(64)]
M62 = (1 << 62) - 1
EVEN = 0x5555555555555555


def ballot(pred):
    return sum(1 << l for l in range(64) if pred(l))


def model_rpop(R, length):
    end = length - 1
    top = R[63]
    last = R[lane_of(end)]
    if end == 0:
        return last, 0
    klast = key(last)
    keys = [key(v) if v is not None else 1 << 40 for v in R]
    sib = [keys[l ^ 1] for l in range(64)]  # DPP quad_perm [1,0,3,2]
    ex = [RL[l][0] != NONE and RL[l][0] < end for l in range(64)]
    VL = ballot(lambda l: ex[l]) & M62
    LE = ballot(lambda l: keys[l] <= klast)
    CR = ballot(lambda l: keys[l] >= sib[l]) & (VL >> 1) & EVEN
    on = [l < 62 and ex[l] and (CR & WL[l][0]) == WL[l][0] and (CR & WL[l][1]) == 0 for l in range(64)]
    PM = ballot(lambda l: on[l])
    PU = PM & LE
    land = 63 if PU == 0 else log2(PU)
    new = list(R)
    for l in range(64):
        node, _, _, cl = RL[l]
        src = cl + ((CR >> cl) & 1) if cl != 63 else 63
        recv = (PU >> src) & 1
        new[l] = last if l == land else (R[src] if recv else R[l])  # ds_bpermute from src
    R[:] = new
    return top, end


def model_rpush(R, length, e):
    p1 = length + 1
    dp = log2(p1)
    keys = [key(v) if v is not None else 1 << 40 for v in R]
    onp = [RL[l][1] <= dp and (p1 >> (dp - RL[l][1])) == RL[l][0] + 1 for l in range(64)]
    G = ballot(lambda l: onp[l] and RL[l][1] < dp and key(e) < keys[l])
    t = dp - bin(G).count("1")
    new = list(R)
    for l in range(64):
        if onp[l] and RL[l][1] == t:
            new[l] = e
        elif onp[l] and RL[l][1] > t:
            new[l] = R[RL[l][2]]  # ds_bpermute from the parent's lane
    R[:] = new
    return length + 1


def test_register_heap_matches_binary_heap():
    """Pops and pushes on the register layout, spilling to / reloading from the array model of the LDS
    heap at 63 / 40 entries as the kernel does."""
    rng = random.Random(99)
    for trial in range(200):
        kr = rng.choice([2, 3, 6, 50])
        Rf, H, R = [], [], [None] * 64
        reg, n, uid = True, 0, 0
        for op in range(rng.randrange(30, 500)):
            if Rf and rng.random() < 0.47:
                top_r = ref_pop(Rf)
                if reg:
                    top_m, n = model_rpop(R, n)
                else:
                    top_m, n = model_wpop(H, n)
                    del H[n:]
                    if n <= 40:  # reload
                        R = [H[RL[l][0]] if RL[l][0] != NONE and RL[l][0] < n else None for l in range(64)]
                        reg = True
                assert top_m == top_r, (trial, op)
            else:
                k = rng.randrange(1, 5)
                elems = []
                for _ in range(k):
                    uid += 1
                    elems.append((rng.randrange(kr), uid))
                for e in elems:
                    ref_push(Rf, e)
                if reg and n + k > 63:  # spill
                    H = [R[lane_of(i)] for i in range(n)]
                    reg = False
                for e in elems:
                    if reg:
                        n = model_rpush(R, n, e)
                    else:
                        H.append(None)
                        n += 1
                        H[n - 1] = e
                        ref_sift_up(H, n - 1)
            cur = [R[lane_of(i)] for i in range(n)] if reg else H[:n]
            assert cur == Rf, (trial, op, reg)
