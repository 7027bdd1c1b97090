// tsw_astar.h — exact A* next hop (get_path, tswap.rs:288-390) as device functions shared by
// the K3 kernels (tsw_kernels.hip) and the coop workers inside the plan dispatch (tsw_plan.hip).
// Rust std BinaryHeap semantics restated (push = sift_up; pop = swap last into the root,
// sift_down_to_bottom, sift_up), ordered by AstarNode::cmp (tswap.rs:314-321). gfx950 only.
#pragma once
#include <hip/hip_runtime.h>

#include "tsw_internal.h"

namespace tsw {

// neighbour directions S,E,N,W = (0,+1),(+1,0),(0,-1),(-1,0): tswap.rs:62
__device__ __forceinline__ uint32_t step_cell(uint32_t c, uint32_t code, uint32_t W) {
  switch (code) {
    case 0: return c + W;
    case 1: return c + 1;
    case 2: return c - W;
    case 3: return c - 1;
    default: return c;
  }
}

// Unreachable-goal fallback of get_path (tswap.rs:378-389): the first
// neighbour (S,E,N,W order) strictly closer in Manhattan distance; every
// improving neighbour is exactly 1 closer, so "first improving" == argmin.
__device__ __forceinline__ uint8_t fallback_code(uint8_t m, uint32_t x, uint32_t y, uint32_t gx,
                                                 uint32_t gy) {
  if ((m & 1) && gy > y) return 0;
  if ((m & 2) && gx > x) return 1;
  if ((m & 4) && gy < y) return 2;
  if ((m & 8) && gx < x) return 3;
  return NH_STAY;
}

// Next-hop classification from a distance table (any address space).
__device__ __forceinline__ uint8_t classify_cell(const uint16_t* D, uint32_t c, uint8_t m,
                                                 uint32_t W, uint32_t goal, uint32_t gx,
                                                 uint32_t gy) {
  if (!(m & NB_FREE)) return NH_UNKNOWN;
  if (c == goal) return NH_STAY;
  const uint16_t d = D[c];
  if (d == DIST_INF) return fallback_code(m, c % W, c / W, gx, gy);
  const uint16_t want = (uint16_t)(d - 1);
  uint32_t cntc = 0, best = 0;
#pragma unroll
  for (uint32_t dir = 0; dir < 4; ++dir) {
    if (m & (1u << dir)) {
      if (D[step_cell(c, dir, W)] == want) {
        ++cntc;
        best = dir;
      }
    }
  }
  return cntc == 1 ? (uint8_t)best : NH_UNKNOWN;
}

__device__ __forceinline__ uint32_t fast_div(uint32_t a, uint32_t b, float inv) {
  uint32_t q = (uint32_t)((float)a * inv);
  while (q * b > a) --q;
  while ((q + 1) * b <= a) ++q;
  return q;
}

// ----------------------------------------------------------------------------
// K3: exact A* next hop, one query per lane.
// Heap entry: f:21 | g:21 | x:11 | y:11; Rust "a <= b" == key(a) >= key(b).
// g_score word per cell: tag:10 | label:2 | g:20 where label = direction of
// path[1] from the start. label(child) = dir if parent is the start, else
// label(parent) at relaxation time; with a consistent heuristic (Manhattan on
// a 4-grid) a node's g, came_from and hence label are final when it is first
// popped, and stale pops relax nothing, so label(goal) at the goal's pop ==
// the direction of path[1] of the reference's came_from chain (tswap.rs:344-355).
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mk_entry(uint32_t f, uint32_t g, uint32_t x, uint32_t y) {
  return ((uint64_t)f << 43) | ((uint64_t)g << 22) | ((uint64_t)x << 11) | (uint64_t)y;
}
__device__ __forceinline__ uint64_t ekey(uint64_t e) { return e >> KEY_SHIFT; }

// BinaryHeap::sift_up(start = 0, pos) with `elem` in the hole.
__device__ __forceinline__ void heap_sift_up(uint64_t* Hp, uint32_t pos, uint64_t elem) {
  const uint64_t k = ekey(elem);
  while (pos > 0) {
    const uint32_t parent = (pos - 1u) >> 1;
    const uint64_t pe = Hp[parent];
    if (k >= ekey(pe)) break;  // elem <= parent
    Hp[pos] = pe;
    pos = parent;
  }
  Hp[pos] = elem;
}

// BinaryHeap::pop with sift_down_to_bottom(0).
__device__ __forceinline__ uint64_t heap_pop(uint64_t* Hp, uint32_t& len) {
  const uint32_t end = --len;
  const uint64_t last = Hp[end];
  if (end == 0) return last;
  const uint64_t top = Hp[0];
  uint32_t pos = 0, child = 1;
  while (child + 1u < end) {  // child <= end - 2
    uint64_t l = Hp[child];
    const uint64_t r = Hp[child + 1];
    if (ekey(l) >= ekey(r)) {  // left <= right: take the right child
      ++child;
      l = r;
    }
    Hp[pos] = l;
    pos = child;
    child = 2u * pos + 1u;
  }
  if (child == end - 1u) {
    Hp[pos] = Hp[child];
    pos = child;
  }
  heap_sift_up(Hp, pos, last);
  return top;
}

// err == nullptr: a heap overflow returns NH_UNKNOWN with *len_out = -2 (caller re-queues the
// query to a larger heap) instead of raising ERR_HEAP_OVERFLOW.
__device__ __forceinline__ uint8_t astar_one(const DevGrid& G, uint32_t v, uint32_t goal, uint32_t tag, uint64_t* Hp,
                                             uint32_t hcap, uint32_t* GS, int32_t* len_out, uint32_t* err) {
  const uint32_t W = G.W;
  const uint32_t vx = v % W, vy = v / W, gx = goal % W, gy = goal / W;
  if (v == goal) {
    *len_out = 1;
    return NH_STAY;
  }
  const uint32_t tagw = tag << 22;
  uint32_t len = 0;
  GS[v] = tagw;
  {
    const uint32_t h0 = (vx > gx ? vx - gx : gx - vx) + (vy > gy ? vy - gy : gy - vy);
    Hp[0] = mk_entry(h0, 0, vx, vy);
    len = 1;
  }
  while (len > 0) {
    const uint64_t e = heap_pop(Hp, len);
    const uint32_t cx = (uint32_t)(e >> 11) & 0x7FFu, cy = (uint32_t)e & 0x7FFu;
    const uint32_t cg = (uint32_t)(e >> 22) & 0x1FFFFFu;
    const uint32_t c = cy * W + cx;
    if (c == goal) {
      *len_out = (int32_t)cg + 1;
      return (uint8_t)((GS[goal] >> 20) & 3u);
    }
    const uint8_t m = G.nbmask[c];
    const uint32_t labc = (GS[c] >> 20) & 3u;
    const uint32_t tg = cg + 1u;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
      if (!(m & (1u << d))) continue;
      const uint32_t nx = d == 1 ? cx + 1 : (d == 3 ? cx - 1 : cx);
      const uint32_t ny = d == 0 ? cy + 1 : (d == 2 ? cy - 1 : cy);
      const uint32_t nc = ny * W + nx;
      const uint32_t old = GS[nc];
      const uint32_t oldg = ((old & 0xFFC00000u) == tagw) ? (old & GS_G_MASK) : 0xFFFFFFFFu;
      if (tg < oldg) {
        const uint32_t lab = cg == 0 ? d : labc;
        GS[nc] = tagw | (lab << 20) | tg;
        if (len >= hcap) {
          if (err) atomicOr(err, ERR_HEAP_OVERFLOW);
          *len_out = err ? -1 : -2;
          return NH_UNKNOWN;
        }
        const uint32_t h = (nx > gx ? nx - gx : gx - nx) + (ny > gy ? ny - gy : gy - ny);
        heap_sift_up(Hp, len, mk_entry(tg + h, tg, nx, ny));
        ++len;
      }
    }
  }
  *len_out = 2;
  return fallback_code(G.nbmask[v], vx, vy, gx, gy);
}

// ----------------------------------------------------------------------------
// Single-lane A* core for k_astar_wave. A lone lane is instruction-bound, so the heap entry
// keeps its ORDER KEY in the high dword: (f << 15 | g) << 32 | x << 16 | y — one 32-bit
// compare per sift step and no division to recover (x, y). Same order as mk_entry's key
// (f, then g; cell bits never compared). f >= 2^17 or g >= 2^15 hands the query off (-2).
// GSM 0/1: u32 tag | label | g words (global slot / LDS); GSM 2: byte words as astar_one_b8.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hk(uint64_t e) { return (uint32_t)(e >> 32); }

__device__ __forceinline__ void hk_sift_up(uint64_t* Hp, uint32_t pos, uint64_t elem) {
  const uint32_t k = hk(elem);
  while (pos > 0) {
    const uint32_t parent = (pos - 1u) >> 1;
    const uint64_t pe = Hp[parent];
    if (k >= hk(pe)) break;  // elem <= parent
    Hp[pos] = pe;
    pos = parent;
  }
  Hp[pos] = elem;
}

__device__ __forceinline__ uint64_t hk_pop(uint64_t* Hp, uint32_t& len) {
  const uint32_t end = --len;
  const uint64_t last = Hp[end];
  if (end == 0) return last;
  const uint64_t top = Hp[0];
  uint32_t pos = 0, child = 1;
  while (child + 1u < end) {
    uint64_t l = Hp[child];
    const uint64_t r = Hp[child + 1];
    if (hk(l) >= hk(r)) {  // left <= right: take the right child
      ++child;
      l = r;
    }
    Hp[pos] = l;
    pos = child;
    child = 2u * pos + 1u;
  }
  if (child == end - 1u) {
    Hp[pos] = Hp[child];
    pos = child;
  }
  hk_sift_up(Hp, pos, last);
  return top;
}

template <int GSM>
__device__ __forceinline__ uint8_t astar_wave_core(const DevGrid& G, uint32_t v, uint32_t goal, uint32_t tag,
                                                   uint64_t* Hp, uint32_t hcap, uint32_t* GS, uint8_t* GB,
                                                   int32_t* len_out) {
  const uint32_t W = G.W;
  const uint32_t vy = v / W, vx = v - vy * W, gy = goal / W, gx = goal - gy * W;
  if (v == goal) {
    *len_out = 1;
    return NH_STAY;
  }
  const uint32_t tagw = tag << 22;
  if constexpr (GSM == 2) GB[v] = 0x80u;
  else GS[v] = tagw;
  const uint32_t h0 = (vx > gx ? vx - gx : gx - vx) + (vy > gy ? vy - gy : gy - vy);
  if (h0 >= (1u << 17)) {
    *len_out = -2;
    return NH_UNKNOWN;
  }
  Hp[0] = ((uint64_t)(h0 << 15) << 32) | (vx << 16) | vy;
  uint32_t len = 1;
  while (len > 0) {
    const uint64_t e = hk_pop(Hp, len);
    const uint32_t cx = (uint32_t)(e >> 16) & 0xFFFFu, cy = (uint32_t)e & 0xFFFFu;
    const uint32_t cg = hk(e) & 0x7FFFu;
    const uint32_t c = cy * W + cx;
    if (c == goal) {
      *len_out = (int32_t)cg + 1;
      if constexpr (GSM == 2) return (uint8_t)((GB[goal] >> 5) & 3u);
      else return (uint8_t)((GS[goal] >> 20) & 3u);
    }
    const uint32_t m = G.nbmask[c];
    uint32_t labc;
    if constexpr (GSM == 2) labc = (GB[c] >> 5) & 3u;
    else labc = (GS[c] >> 20) & 3u;
    const uint32_t tg = cg + 1u;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
      if (!(m & (1u << d))) continue;
      const uint32_t nx = d == 1 ? cx + 1 : (d == 3 ? cx - 1 : cx);
      const uint32_t ny = d == 0 ? cy + 1 : (d == 2 ? cy - 1 : cy);
      const uint32_t nc = ny * W + nx;
      uint32_t oldg;
      uint32_t man = 0;
      if constexpr (GSM == 2) {
        man = (nx > vx ? nx - vx : vx - nx) + (ny > vy ? ny - vy : vy - ny);
        const uint32_t old = GB[nc];
        oldg = (old & 0x80u) ? man + 2u * (old & 31u) : 0xFFFFFFFFu;
      } else {
        const uint32_t old = GS[nc];
        oldg = ((old & 0xFFC00000u) == tagw) ? (old & GS_G_MASK) : 0xFFFFFFFFu;
      }
      if (tg < oldg) {
        const uint32_t lab = cg == 0 ? d : labc;
        const uint32_t h = (nx > gx ? nx - gx : gx - nx) + (ny > gy ? ny - gy : gy - ny);
        const uint32_t f = tg + h;
        bool ovf = len >= hcap || tg >= (1u << 15) || f >= (1u << 17);
        if constexpr (GSM == 2) {
          const uint32_t hh = (tg - man) >> 1;
          ovf = ovf || hh > 31u;
          if (!ovf) GB[nc] = (uint8_t)(0x80u | (lab << 5) | hh);
        } else {
          if (!ovf) GS[nc] = tagw | (lab << 20) | tg;
        }
        if (ovf) {
          *len_out = -2;
          return NH_UNKNOWN;
        }
        hk_sift_up(Hp, len, ((uint64_t)((f << 15) | tg) << 32) | (nx << 16) | ny);
        ++len;
      }
    }
  }
  *len_out = 2;
  return fallback_code(G.nbmask[v], vx, vy, gx, gy);
}

// ----------------------------------------------------------------------------
// Wave-cooperative A* core (k_astar_wave default; TSW_ASTAR_SERIAL=1 selects the lone-lane
// core above). Same BinaryHeap algorithm, same heap contents after every operation — only the
// way each sift touches its path changes, so the pop order (and every label) is identical:
//  * sift_down_to_bottom: the 62 descendants of the hole within 5 levels are read by one
//    ds_read (lane j -> depth k = log2(j + 2), index j + 2 - 2^k below the hole). Each left
//    child compares its key with its sibling's (DPP lane swap); "take the right child" bits and
//    the node-exists bits are balloted, and the path (left <= right -> right child, a lone left
//    child is taken, stop at a childless node) is found by every lane testing its own ancestors'
//    choices (WinLane masks) — one more ballot, no serial walk. The path's values move up one
//    level with one ds_write. A 4096-entry heap has depth 12: <= 3 LDS round trips per pop
//    instead of 12 dependent ones.
//  * sift_up (of the popped-last element and of every push): the hole's ancestors are read one
//    per lane. The root path is heap ordered, so the ancestors whose key exceeds the element's
//    (those the element passes: it stops at the first parent it is not smaller than) are a
//    suffix of it: one ballot gives the landing depth and one ds_write shifts them down.
//  * the four neighbours are relaxed by lanes 0..3 at once (distinct cells); the improved
//    ones are pushed in direction order (tswap.rs:337-360's loop order).
// LDS instructions of one wave complete in issue order, so a lane reads what another lane of
// the same wave wrote by an earlier instruction.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rl32(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t x, uint32_t l) {
  return ((uint64_t)rl32((uint32_t)(x >> 32), l) << 32) | rl32((uint32_t)x, l);
}
__device__ __forceinline__ void wave_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t ballot64(bool c) { return __builtin_amdgcn_ballot_w64(c); }

// BinaryHeap::sift_up(0, pos) with `elem` in the hole; wave-uniform arguments. Straight-line:
// every lane reads (lanes >= the hole's depth re-read the hole), one ballot, one store.
__device__ __forceinline__ void wsift_up(uint64_t* Hp, uint32_t pos, uint64_t elem, uint32_t lane) {
  const uint32_t p1 = pos + 1u;
  const uint32_t dp = 31u - (uint32_t)__builtin_clz(p1);  // depth of the hole (root = 0)
  const uint32_t k = hk(elem);
  const uint32_t sh = dp > lane ? dp - lane : 0u;
  const uint64_t a = Hp[(p1 >> sh) - 1u];  // ancestor at depth `lane`
  const uint64_t G = ballot64(k < hk(a)) & ((1ull << dp) - 1ull);  // ancestors elem moves past
  const uint32_t t = dp - (uint32_t)__popcll(G);                   // landing depth
  const bool isdp = lane == dp;
  // lanes t..dp-1 move their ancestor one level down the path; lane dp stores elem at depth t
  const uint32_t dst = isdp ? (p1 >> (dp - t)) - 1u : (p1 >> (sh - 1u)) - 1u;
  wave_order();
  if (lane >= t && lane <= dp) Hp[dst] = isdp ? elem : a;
  wave_order();
}

// Window lane constants for wpop's path test: lane j < 62 holds the node at depth kk = log2(j + 2)
// (1..5), index ki = j + 2 - 2^kk below the hole. The path reaches that node iff every ancestor in
// the window chose the child leading to it: for ancestor depth a < kk, the choice bit lives at the
// lane of that ancestor's left child, 2^(a+1) - 2 + 2 * (ki >> (kk - a)), and must equal bit
// (kk - a - 1) of ki. `one` / `zero` collect those lanes by the required bit. Loop-invariant.
struct WinLane {
  uint64_t one, zero;
};
__device__ __forceinline__ WinLane win_lane(uint32_t lane) {
  WinLane w{0ull, 0ull};
  if (lane >= 62u) {  // not window lanes: the path test fails (a required bit is both 0 and 1)
    w.one = w.zero = 1ull;
    return w;
  }
  const uint32_t kk = 31u - (uint32_t)__builtin_clz(lane + 2u), ki = lane + 2u - (1u << kk);
  for (uint32_t a = 0; a < kk; ++a) {
    const uint32_t lc = (2u << a) - 2u + 2u * (ki >> (kk - a));
    if ((ki >> (kk - a - 1u)) & 1u) w.one |= 1ull << lc;
    else w.zero |= 1ull << lc;
  }
  return w;
}

// BinaryHeap::pop (swap last into the root, sift_down_to_bottom(0), sift_up(0, hole)); len >= 1.
// Window lanes: lane j < 62 <-> depth kk = log2(j + 2) (1..5), index ki = j + 2 - 2^kk below the
// hole; the first window's lanes 62 / 63 fetch the last element / the root. The path is found
// lane-parallel (each lane tests its own ancestors' choices against WinLane masks; the deepest lane
// on the path gives the window's end) instead of a 5-step SALU walk: same path, fewer instructions
// on the pop's dependent chain.
// The trailing sift_up of the last element is fused in: it moves back down every path node whose key
// exceeds the last element's (a suffix of the path, which is heap ordered), so the net effect is that
// only the path nodes p_1..p_t with key <= last's move up one level and the last element takes p_t's
// old place. The pop therefore stops in the first window holding a path node the last element does
// not pass — no deeper window, no re-read of the path (tests/test_heap_lane_model.py models it).
// `at_top(top)` runs as soon as the popped entry is known (after the first window read), so the
// caller can issue the popped node's neighbour loads while the sift still runs.
template <class AtTop>
__device__ __forceinline__ uint64_t wpop(uint64_t* Hp, uint32_t& len, uint32_t lane, const WinLane& wl,
                                         AtTop&& at_top) {
  constexpr uint64_t M62 = (1ull << 62) - 1ull, EVEN = 0x5555555555555555ull;
  const uint32_t end = --len;
  uint32_t pos = 0, klast = 0;
  uint64_t last = 0, top = 0;
  const uint32_t kk = 31u - (uint32_t)__builtin_clz(lane + 2u);
  const uint32_t ki = lane + 2u - (1u << kk);
  for (bool first = true;; first = false) {
    const uint32_t node = ((pos + 1u) << kk) - 1u + ki;
    uint32_t addr = node < end ? node : end;  // Hp[end] is still allocated
    if (first) addr = lane == 62u ? end : (lane == 63u ? 0u : addr);
    const uint64_t val = Hp[addr];
    if (first) {
      last = rl64(val, 62);
      top = rl64(val, 63);
      if (end == 0) {
        at_top(last);
        return last;
      }
      klast = hk(last);
      at_top(top);
    }
    const uint32_t key = hk(val);
    const uint32_t sib = (uint32_t)__builtin_amdgcn_mov_dpp((int)key, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    const bool ex = node < end;
    const uint64_t VL = ballot64(ex) & M62;
    const uint64_t LE = ballot64(key <= klast);  // nodes the last element would not pass
    // left child lane (even) takes the right child when left <= right and the right exists
    const uint64_t CR = ballot64(key >= sib) & (VL >> 1) & EVEN;
    const bool on = ex & ((CR & wl.one) == wl.one) & ((CR & wl.zero) == 0ull);  // branch-free
    const uint64_t PM = ballot64(on);
    if (PM == 0ull) break;  // the hole has no child
    const uint64_t PU = PM & LE;
    if (PU != PM) {  // the last element lands in this window: below the deepest moving node, or at the hole
      uint32_t tgt = pos;
      if (PU != 0ull) {
        const uint32_t lu = 63u - (uint32_t)__builtin_clzll(PU);
        const uint32_t d = 31u - (uint32_t)__builtin_clz(lu + 2u);
        tgt = ((pos + 1u) << d) - 1u + (lu + 2u - (1u << d));
      }
      wave_order();
      if ((PU >> lane) & 1ull) Hp[(node - 1u) >> 1] = val;  // lanes >= 62 are never on the path
      if (lane == 63u) Hp[tgt] = last;
      wave_order();
      return top;
    }
    const uint32_t lt = 63u - (uint32_t)__builtin_clzll(PM);  // deepest node on the path
    const uint32_t d = 31u - (uint32_t)__builtin_clz(lt + 2u), idx = lt + 2u - (1u << d);
    wave_order();
    if (on) Hp[(node - 1u) >> 1] = val;  // move up into the parent
    wave_order();
    pos = ((pos + 1u) << d) - 1u + idx;
    if (d < 5) break;
  }
  // every path node moved up (the last element passes none of them): it fills the bottom hole
  wave_order();
  if (lane == 63u) Hp[pos] = last;
  wave_order();
  return top;
}

// ----------------------------------------------------------------------------
// Register-resident heap (round 4). A* heaps are small — on C3 the heap holds 31 entries at the median
// pop, 49 at p90 — so a heap of <= REG_HEAP_MAX = 63 entries lives in one 64-bit VGPR pair across the
// wave in the first pop window's own layout: node 0 (the root) in lane 63, node n in 1..62 in lane n - 1
// (siblings are lane pairs (2i, 2i + 1); lane 62 holds nothing). A pop is then the window's path test
// with no LDS read, and values move along a path with one ds_bpermute (pull from the chosen child; for a
// push, from the parent) instead of an LDS write / read round trip. The heap spills to the LDS array
// when a push would pass 63 entries and is reloaded once a pop leaves <= REG_HEAP_RELOAD; both forms
// hold the same BinaryHeap array, so the pop order is unchanged (tests/test_heap_lane_model.py models
// rpop / rpush with the spill and reload against the restated BinaryHeap).
// ----------------------------------------------------------------------------
constexpr uint32_t REG_HEAP_MAX = 63u, REG_HEAP_RELOAD = 40u, REG_NONE = 0xFFFFu;
struct RegLane {
  uint32_t node, depth, plane, src_child;  // src_child: lane of the left child (node <= 30), else 63
};
__device__ __forceinline__ uint32_t reg_lane_of(uint32_t n) { return n == 0u ? 63u : n - 1u; }
__device__ __forceinline__ RegLane reg_lane(uint32_t lane) {
  RegLane r;
  r.node = lane == 63u ? 0u : (lane == 62u ? REG_NONE : lane + 1u);
  r.depth = r.node == REG_NONE ? 15u : 31u - (uint32_t)__builtin_clz(r.node + 1u);
  r.plane = (r.node == 0u || r.node == REG_NONE) ? lane : reg_lane_of((r.node - 1u) >> 1);
  r.src_child = (r.node != REG_NONE && r.node <= 30u) ? reg_lane_of(2u * r.node + 1u) : 63u;
  return r;
}
__device__ __forceinline__ uint64_t bperm64(uint64_t x, uint32_t src) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// BinaryHeap::pop on the register heap (1 <= len <= 63), the last element's sift_up fused as in wpop:
// the path nodes with key <= last's move up (each path node above the landing pulls its chosen child's
// value), the last element takes the deepest one's place (the root when none moves).
template <class AtTop>
__device__ __forceinline__ uint64_t rpop(uint64_t& R, uint32_t& len, uint32_t lane, const WinLane& wl,
                                         const RegLane& rl, AtTop&& at_top) {
  constexpr uint64_t M62 = (1ull << 62) - 1ull, EVEN = 0x5555555555555555ull;
  const uint32_t end = --len;
  const uint64_t top = rl64(R, 63u);
  at_top(top);
  if (end == 0) return top;
  const uint64_t last = rl64(R, end - 1u);  // node end >= 1 sits in lane end - 1
  const uint32_t klast = hk(last), key = hk(R);
  const uint32_t sib = (uint32_t)__builtin_amdgcn_mov_dpp((int)key, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  const bool ex = rl.node < end;  // lane 62 (REG_NONE) never; lane 63 (the root) is masked below
  const uint64_t VL = ballot64(ex) & M62;
  const uint64_t LE = ballot64(key <= klast);
  const uint64_t CR = ballot64(key >= sib) & (VL >> 1) & EVEN;
  const bool on = ex & ((CR & wl.one) == wl.one) & ((CR & wl.zero) == 0ull);
  const uint64_t PU = ballot64(on) & LE;
  const uint32_t land = PU == 0ull ? 63u : 63u - (uint32_t)__builtin_clzll(PU);
  const uint32_t src = rl.src_child == 63u ? 63u : rl.src_child + (uint32_t)((CR >> rl.src_child) & 1ull);
  const uint64_t pulled = bperm64(R, src);
  const bool recv = (PU >> src) & 1ull;  // bit 63 of PU is never set
  R = lane == land ? last : (recv ? pulled : R);
  return top;
}

// BinaryHeap::push (sift_up(0, len)) on the register heap, len < 63: the ancestors the element passes
// (a suffix of its root path) pull their parent's value, the element lands at depth t.
__device__ __forceinline__ void rpush(uint64_t& R, uint32_t& len, uint64_t e, const RegLane& rl) {
  const uint32_t p1 = len + 1u, dp = 31u - (uint32_t)__builtin_clz(p1);
  const uint32_t sh = rl.depth <= dp ? dp - rl.depth : 0u;
  const bool onp = rl.depth <= dp && (p1 >> sh) == rl.node + 1u;  // the hole's root path (the hole included)
  const uint64_t G = ballot64(onp && rl.depth < dp && hk(e) < hk(R));
  const uint32_t t = dp - (uint32_t)__popcll(G);
  const uint64_t pulled = bperm64(R, rl.plane);
  R = (onp && rl.depth == t) ? e : ((onp && rl.depth > t) ? pulled : R);
  ++len;
}

// Detour bytes of a goal for astar_wave_par<*, *, 1>: DT[c] = (D[c] - |c - goal|_1) / 2 (D and the Manhattan
// distance share parity on a 4-grid), 255 when that is >= 255 or c is blocked / unreachable — the table
// store's format (round 6), copied from the goal's store slot DTg. Only the cells of the box [x0, x1] x
// [y0, y1] are copied: the caller passes the bounding box of the query's ellipse {x : |x - v| + |x - goal| <= d*},
// outside which every cell has f = g + h > d* and so can never pass the DAG test (g + D = d*) whatever
// DT holds there. Lanes walk the box's cells in row-major order, STAGE_INFLIGHT loads in flight per lane
// (the staging is a chain of global round trips in front of the query's first pop).
constexpr uint32_t STAGE_INFLIGHT = 8u;
__device__ __forceinline__ void stage_detour(uint8_t* DT, const uint8_t* DTg, uint32_t W, uint32_t x0, uint32_t x1,
                                             uint32_t y0, uint32_t y1, uint32_t lane) {
  const uint32_t bw = x1 - x0 + 1u, nb = bw * (y1 - y0 + 1u);
  const float inv = 1.0f / (float)bw;
  for (uint32_t i0 = lane; i0 < nb; i0 += 64u * STAGE_INFLIGHT) {
    uint32_t cell[STAGE_INFLIGHT], d[STAGE_INFLIGHT];
#pragma unroll
    for (uint32_t u = 0; u < STAGE_INFLIGHT; ++u) {
      const uint32_t i = i0 + 64u * u;
      const uint32_t r = fast_div(i < nb ? i : 0u, bw, inv);
      cell[u] = (y0 + r) * W + x0 + ((i < nb ? i : 0u) - r * bw);
      d[u] = DTg[cell[u]];
    }
#pragma unroll
    for (uint32_t u = 0; u < STAGE_INFLIGHT; ++u) {
      if (i0 + 64u * u >= nb) break;
      DT[cell[u]] = (uint8_t)d[u];
    }
  }
}

// FB: the grid's free-cell row bitmap (DevGrid::freebits) staged in LDS, so relaxing a node
// needs no global load.
// PROF: pr[0..4] = pops, clocks in pops, in relaxations, in pushes, pushes (TSW_ASTAR_PROF)
//
// DAG early exit (DAG = 1: the goal's detour bytes DT staged in LDS, see stage_detour; DAG = 2: the
// same bytes read from the goal's table-store slot DG beside the g-score words; 0: off). Exact, from these facts about this
// A* (consistent Manhattan heuristic, no closed set, keys (f, then smaller g)):
//  * a node n is relaxed at most once with its optimal g = d_s(n) (later relaxations need a strictly
//    smaller g), and that relaxation fixes came_from(n) — hence its label — for good;
//  * n lies on a shortest start -> goal path with g optimal iff g + D[n] == d* (D = the goal's K1
//    distance, d* = D[start]); every node of the final came_from chain is such a "DAG" node;
//  * take the chain's last node m that is already relaxed at some moment: its successor on the chain
//    is not relaxed yet, so m has not been expanded (its pop would have relaxed it optimally). So
//    label(goal) = label(m) for some DAG node relaxed but not yet popped.
// Hence once every DAG node relaxed-but-unpopped carries the same label — or the goal itself has been
// relaxed with g = d* — label(goal) = path[1]'s direction is decided and the search stops there.
// Those nodes are exactly the heap entries with g + D == d* (a stale entry has a larger g; an optimal
// entry leaves the heap at its pop, the node's first). Every (dag_mask + 1) pops the wave scans the heap
// (one ds_read per 64 entries plus a D gather, label ballots) after the pop's pushes: nothing is added
// to the per-pop chain, and the stop comes at most dag_mask pops late.
template <int GSM, bool PROF, int DAG = 0, bool REG = true>
__device__ __forceinline__ uint8_t astar_wave_par(const DevGrid& G, uint32_t v, uint32_t goal, uint32_t tag,
                                                  uint64_t* Hp, uint32_t hcap, uint32_t* GS, uint8_t* GB,
                                                  const uint32_t* FB, int32_t* len_out, unsigned long long* pr,
                                                  const uint8_t* DT = nullptr, const uint8_t* DG = nullptr,
                                                  uint32_t* npop = nullptr, uint32_t dag_mask = 15u,
                                                  uint32_t reg_max = REG_HEAP_MAX) {
  const uint32_t lane = threadIdx.x & 63u;
  unsigned long long pops = 0, c_pop = 0, c_nb = 0, c_push = 0, npush = 0, tk = 0;
  auto tick = [&](unsigned long long& acc) {
    if constexpr (PROF) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc += t - tk;
      tk = t;
    }
  };
  auto flush = [&]() {
    if (npop) *npop = (uint32_t)pops;
    if constexpr (PROF) {
      pr[0] = pops;
      pr[1] = c_pop;
      pr[2] = c_nb;
      pr[3] = c_push;
      pr[4] = npush;
    }
  };
  const uint32_t W = G.W, H = G.H, Ww = G.Ww;
  const uint32_t vy = v / W, vx = v - vy * W, gy = goal / W, gx = goal - gy * W;
  if (v == goal) {
    *len_out = 1;
    return NH_STAY;
  }
  const uint32_t tagw = tag << 22;
  const uint32_t h0 = (vx > gx ? vx - gx : gx - vx) + (vy > gy ? vy - gy : gy - vy);
  if (h0 >= (1u << 17)) {
    *len_out = -2;
    return NH_UNKNOWN;
  }
  // DAG early exit: d* = h0 + 2 * detour(v), applicable when the start reaches the goal with an exact
  // detour byte. A DAG node n lies on a shortest start -> goal path, and along such a path the detour
  // (D - h) / 2 never grows (D drops by 1 per hop, h changes by 1), so detour(n) <= detour(v) < 255: the
  // test below skips saturated bytes (255) without skipping any DAG node.
  uint32_t dstar = 0xFFFFFFFFu;
  bool ee = false;
  if constexpr (DAG != 0) {
    const uint32_t dv = DAG == 1 ? DT[v] : DG[v];
    dstar = h0 + 2u * dv;
    ee = dv != 255u;
  }
  // the heap starts in registers (see rpop): the start entry at the root (lane 63); reg_max = 0 keeps
  // it in the LDS array throughout (A/B). REG = false compiles the register heap out: on grids whose
  // heaps mostly outgrow 63 entries (wh10k: 103 at the median pop) its live registers only add
  // pressure to the LDS path (wh10k 11.3-11.5 -> 12.1 s with it compiled in, same box)
  const RegLane rl = reg_lane(lane);
  bool reg = REG && reg_max != 0u;
  uint64_t R = ((uint64_t)(h0 << 15) << 32) | (vx << 16) | vy;
  if (lane == 0) {
    if constexpr (GSM == 2) GB[v] = 0x80u;
    else GS[v] = tagw;
    if (!reg) Hp[0] = R;
  }
  wave_order();
  if constexpr (PROF) tk = __builtin_amdgcn_s_memtime();
  uint32_t len = 1;
  // lanes 0..3 own the neighbour in direction `lane` (S, E, N, W: tswap.rs:62-73)
  const uint32_t dd = lane & 3u;
  // lane dd's step (S, E, N, W) as unsigned deltas (wrapping -1): cell, x, y, bitmap row
  const uint32_t ddx = dd == 1 ? 1u : (dd == 3 ? 0xFFFFFFFFu : 0u), ddy = dd == 0 ? 1u : (dd == 2 ? 0xFFFFFFFFu : 0u);
  const uint32_t dcell = ddy * W + ddx, drow = ddy * Ww;
  const WinLane wl = win_lane(lane);
  while (len > 0) {
    ++pops;
    // entry low dword: x << 16 | label << 12 | y (y < 2^11): the popped node's label travels in its
    // entry — a node's first pop is its lowest-g entry, i.e. its latest (strictly improving)
    // relaxation, whose label is the one its g-score word holds — so no g-score read is needed.
    // The neighbour loads are issued from inside the pop, right after its first window read (the
    // g-score / bitmap regions are disjoint from the heap, so the sift's LDS traffic cannot alias).
    uint32_t cx = 0, cy = 0, c = 0, fx = 0, fy = 0, nc = 0, fw = 0, old = 0;
    bool inb = false;
    auto at_top = [&](uint64_t t) {
      cx = (uint32_t)(t >> 16) & 0xFFFFu;
      cy = (uint32_t)t & 0x7FFu;
      c = cy * W + cx;
      // neighbour of lane dd (unsigned wrap: x - 1 at x = 0 fails the bound test); every lane
      // reads (out-of-grid lanes re-read the popped cell), the LDS reads issue together
      const uint32_t nx = cx + ddx, ny = cy + ddy;
      inb = lane < 4u && nx < W && ny < H;
      fx = inb ? nx : cx;
      fy = inb ? ny : cy;
      // cell and bitmap-word indices from the popped cell's (scalar) ones: no per-lane multiply
      nc = c + (inb ? dcell : 0u);
      fw = FB[cy * Ww + (inb ? drow : 0u) + (fx >> 5)];
      if constexpr (GSM == 2) old = GB[nc];
      else old = GS[nc];
    };
    uint64_t e;
    if (reg) {
      e = rpop(R, len, lane, wl, rl, at_top);
    } else {
      e = wpop(Hp, len, lane, wl, at_top);
      if (REG && reg_max != 0u && len <= REG_HEAP_RELOAD) {  // back to registers (the LDS array is the heap as it stands)
        R = Hp[rl.node < len ? rl.node : 0u];
        reg = true;
      }
    }
    tick(c_pop);
    const uint32_t labc = ((uint32_t)e >> 12) & 3u;
    const uint32_t cg = hk(e) & 0x7FFFu;
    if (c == goal) {
      flush();
      *len_out = (int32_t)cg + 1;
      return (uint8_t)labc;
    }
    const uint32_t tg = cg + 1u;
    uint32_t oldg, man = 0;
    if constexpr (GSM == 2) {
      man = (fx > vx ? fx - vx : vx - fx) + (fy > vy ? fy - vy : vy - fy);
      oldg = (old & 0x80u) ? man + 2u * (old & 31u) : 0xFFFFFFFFu;
    } else {
      oldg = ((old & 0xFFC00000u) == tagw) ? (old & GS_G_MASK) : 0xFFFFFFFFu;
    }
    const bool imp = inb && ((fw >> (fx & 31u)) & 1u) && tg < oldg;
    uint64_t ent = 0;
    bool ovf = false;
    if (imp) {
      const uint32_t lab = cg == 0 ? dd : labc;
      const uint32_t h = (fx > gx ? fx - gx : gx - fx) + (fy > gy ? fy - gy : gy - fy);
      const uint32_t f = tg + h;
      ovf = tg >= (1u << 15) || f >= (1u << 17);
      if constexpr (GSM == 2) {
        const uint32_t hh = (tg - man) >> 1;
        ovf = ovf || hh > 31u;
        if (!ovf) GB[nc] = (uint8_t)(0x80u | (lab << 5) | hh);
      } else {
        if (!ovf) GS[nc] = tagw | (lab << 20) | tg;
      }
      ent = ((uint64_t)((f << 15) | tg) << 32) | (fx << 16) | (lab << 12) | fy;
    }
    uint64_t M = ballot64(imp);
    tick(c_nb);
    if (ballot64(ovf) != 0ull || len + (uint32_t)__popcll(M) > hcap) {
      flush();
      *len_out = -2;
      return NH_UNKNOWN;
    }
    if (reg && len + (uint32_t)__popcll(M) > reg_max) {  // spill the register heap to the LDS array
      wave_order();
      if (rl.node < len) Hp[rl.node] = R;
      reg = false;
    }
    wave_order();
    while (M) {
      const uint32_t d = (uint32_t)__builtin_ctzll(M);
      M &= M - 1ull;
      if (reg) {
        rpush(R, len, rl64(ent, d), rl);
      } else {
        wsift_up(Hp, len, rl64(ent, d), lane);
        ++len;
      }
      ++npush;
    }
    tick(c_push);
    if constexpr (DAG != 0) {
      // every (dag_mask + 1) pops: the labels of the heap's DAG entries (g + D == d*), and whether the
      // goal is among them. Off the per-pop chain: one read per 64 entries plus a D gather.
      if (ee && (pops & dag_mask) == 0u) {
        uint32_t labs = 0, glab = 4u;
        for (uint32_t j0 = 0; j0 < len; j0 += 64u) {
          const uint32_t j = reg ? rl.node : j0 + lane;  // a register heap is one pass (len <= 63)
          const uint64_t en = reg ? R : Hp[j < len ? j : 0u];
          const uint32_t lo = (uint32_t)en, ex = lo >> 16, ey = lo & 0x7FFu, eg = hk(en) & 0x7FFFu;
          const uint32_t ec = ey * W + ex;
          // D = Manhattan to the goal + 2 * detour (DAG 1: LDS-staged bytes, DAG 2: the store slot's)
          const uint32_t eh = (ex > gx ? ex - gx : gx - ex) + (ey > gy ? ey - gy : gy - ey);
          const uint32_t db = DAG == 1 ? (uint32_t)DT[ec] : (uint32_t)DG[ec];
          bool d = db != 255u && eg + eh + 2u * db == dstar;
          d = d && j < len;
          const uint32_t el = (lo >> 12) & 3u;
          const uint64_t gm = ballot64(d && ec == goal);
          if (gm) glab = rl32(el, (uint32_t)__builtin_ctzll(gm));
          labs |= (ballot64(d && el == 0u) ? 1u : 0u) | (ballot64(d && el == 1u) ? 2u : 0u) |
                  (ballot64(d && el == 2u) ? 4u : 0u) | (ballot64(d && el == 3u) ? 8u : 0u);
        }
        if (glab != 4u || __builtin_popcount(labs) == 1) {
          flush();
          *len_out = (int32_t)dstar + 1;
          return (uint8_t)(glab != 4u ? glab : (uint32_t)__builtin_ctz(labs));
        }
      }
    }
  }
  flush();
  *len_out = 2;
  return fallback_code(G.nbmask[v], vx, vy, gx, gy);
}

}  // namespace tsw
