// tsw_kernels.hip — gfx950 kernels of the TSWAP planning core.
//
//   K1 k_bfs        batched per-goal BFS distance tables (bit-parallel rows,
//                   LDS-resident frontier/visited bitmaps and u16 table,
//                   one coalesced 16-B-per-lane write-out) fused with the
//                   next-hop classification of every cell (unique optimal
//                   neighbour / unreachable fallback / needs-A*).
//   K3 k_astar      exact get_path() next hop (tswap.rs:288-390): one query
//                   per lane, Rust std BinaryHeap sift semantics restated.
//   k_classify      next-hop codes for tables imported from elsewhere.
//   k_enqueue_unknown  eager next-hop mode: queue every unresolved (cell, goal).
// K2 (step) and K4 (assignment) live in the persistent k_plan (tsw_plan.hip).
//
// Launch wrappers are plain C++ functions declared in tsw_launch.h.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tsw_internal.h"
#include "tsw_launch.h"
#include "tsw_plan.h"

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
// K1: batched BFS distance tables.
// One workgroup per goal (grid-stride). LDS holds the frontier bitmap (double
// buffered), the visited bitmap, the free-cell bitmap and — when LDS_TABLE —
// the whole u16 table. Each level expands the frontier with word-parallel
// shifts (east/west inside a row word with carries, north/south from the
// adjacent rows) over the Manhattan band |y - gy| <= level + 1 only. Newly
// reached cells get level+1 written into the table. The table then leaves
// LDS in one pass of 16-B stores together with the 8-B next-hop codes.
// ----------------------------------------------------------------------------
template <bool LDS_TABLE>
__global__ void __launch_bounds__(1024) k_bfs(DevGrid G, const uint32_t* __restrict__ goals,
                                              const uint32_t* __restrict__ slots, uint32_t k,
                                              uint16_t* __restrict__ dist_base, uint64_t dstride,
                                              uint8_t* __restrict__ nh_base, uint64_t nstride,
                                              uint32_t* __restrict__ err) {
  extern __shared__ __align__(16) uint32_t smem[];
  const uint32_t W = G.W, H = G.H, Ww = G.Ww, nw = H * Ww, nwp = (nw + 3u) & ~3u;
  const uint32_t ncell = G.ncell, ncp = (ncell + 7u) & ~7u;
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  uint32_t* bufA = smem;
  uint32_t* bufB = smem + nwp;
  uint32_t* V = smem + 2 * nwp;
  uint32_t* FR = smem + 3 * nwp;
  uint16_t* Dl = reinterpret_cast<uint16_t*>(smem + 4 * nwp);
  const float invWw = 1.0f / (float)Ww;
  const bool vec_ok = (dstride % 8u) == 0;

  for (uint32_t t = tid; t < nw; t += bd) FR[t] = G.freebits[t];

  for (uint32_t gi = blockIdx.x; gi < k; gi += gridDim.x) {
    const uint32_t goal = goals[gi];
    const uint64_t slot = slots ? slots[gi] : gi;
    uint16_t* Dg = dist_base + slot * dstride;
    uint16_t* D = LDS_TABLE ? Dl : Dg;
    for (uint32_t t = tid; t < nw; t += bd) {
      bufA[t] = 0u;
      bufB[t] = 0u;
      V[t] = 0u;
    }
    if (LDS_TABLE || vec_ok) {
      const uint4 inf4 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
      const uint32_t lim = LDS_TABLE ? ncp / 8u : ncell / 8u;
      for (uint32_t t = tid; t < lim; t += bd) reinterpret_cast<uint4*>(D)[t] = inf4;
      if (!LDS_TABLE)
        for (uint32_t c = (ncell & ~7u) + tid; c < ncell; c += bd) D[c] = DIST_INF;
    } else {
      for (uint32_t c = tid; c < ncell; c += bd) D[c] = DIST_INF;
    }
    __syncthreads();
    const uint32_t gx = goal % W, gy = goal / W;
    if (tid == 0) {
      const uint32_t wt = gy * Ww + (gx >> 5);
      bufA[wt] = 1u << (gx & 31u);
      V[wt] = 1u << (gx & 31u);
      D[goal] = 0;
    }
    __syncthreads();
    uint32_t* cur = bufA;
    uint32_t* nxt = bufB;
    uint32_t level = 0;
    for (;;) {
      const int lo = max(0, (int)gy - (int)level - 1);
      const int hi = min((int)H - 1, (int)gy + (int)level + 1);
      const uint32_t t0 = (uint32_t)lo * Ww, t1 = (uint32_t)(hi + 1) * Ww;
      const uint16_t dn = (uint16_t)(level + 1);
      int any = 0;
      for (uint32_t t = t0 + tid; t < t1; t += bd) {
        const uint32_t r = fast_div(t, Ww, invWw);
        const uint32_t w = t - r * Ww;
        const uint32_t f = cur[t];
        const uint32_t left = (w > 0) ? cur[t - 1] : 0u;
        const uint32_t right = (w + 1 < Ww) ? cur[t + 1] : 0u;
        const uint32_t up = (r > 0) ? cur[t - Ww] : 0u;
        const uint32_t down = (r + 1 < H) ? cur[t + Ww] : 0u;
        const uint32_t hz = (f << 1) | (left >> 31) | (f >> 1) | (right << 31);
        uint32_t nb = (hz | up | down) & FR[t] & ~V[t];
        nxt[t] = nb;
        if (nb) {
          V[t] |= nb;
          any = 1;
          const uint32_t base = r * W + (w << 5);
          while (nb) {
            const uint32_t b = __builtin_ctz(nb);
            D[base + b] = dn;
            nb &= nb - 1u;
          }
        }
      }
      any = __syncthreads_or(any);
      if (!any) break;
      ++level;
      if (level >= 0xFFFEu) {
        if (tid == 0) atomicOr(err, ERR_DIST_OVERFLOW);
        break;
      }
      uint32_t* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
    __syncthreads();
    // write-out (+ fused next-hop classification)
    uint8_t* NHg = nh_base ? nh_base + slot * nstride : nullptr;
    if (LDS_TABLE && vec_ok) {
      for (uint32_t c8 = tid; c8 < ncell / 8u; c8 += bd)
        reinterpret_cast<uint4*>(Dg)[c8] = reinterpret_cast<const uint4*>(Dl)[c8];
      for (uint32_t c = (ncell & ~7u) + tid; c < ncell; c += bd) Dg[c] = Dl[c];
    } else if (LDS_TABLE) {
      for (uint32_t c = tid; c < ncell; c += bd) Dg[c] = Dl[c];
    }
    if (NHg) {
      for (uint32_t c8 = tid; c8 < ncp / 8u; c8 += bd) {
        const uint64_t m8 = reinterpret_cast<const uint64_t*>(G.nbmask)[c8];
        uint64_t codes = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
          const uint32_t c = c8 * 8u + j;
          uint8_t code = NH_UNKNOWN;
          if (c < ncell) code = classify_cell(D, c, (uint8_t)(m8 >> (8 * j)), W, goal, gx, gy);
          codes |= (uint64_t)code << (8 * j);
        }
        reinterpret_cast<uint64_t*>(NHg)[c8] = codes;
      }
    }
    __syncthreads();
  }
}

// Next-hop classification for tables that arrived from elsewhere
// (tsw_import_tables_device): one thread per 8 cells.
__global__ void k_classify(DevGrid G, const uint32_t* __restrict__ goals,
                           const uint32_t* __restrict__ slots, uint32_t k,
                           const uint16_t* __restrict__ dist_base, uint64_t stride,
                           uint8_t* __restrict__ nh_base) {
  const uint32_t ncp8 = (G.ncell + 7u) / 8u;
  const uint64_t total = (uint64_t)k * ncp8;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t gi = (uint32_t)(idx / ncp8), c8 = (uint32_t)(idx % ncp8);
    const uint32_t goal = goals[gi];
    const uint64_t slot = slots[gi];
    const uint16_t* D = dist_base + slot * stride;
    const uint32_t gx = goal % G.W, gy = goal / G.W;
    const uint64_t m8 = reinterpret_cast<const uint64_t*>(G.nbmask)[c8];
    uint64_t codes = 0;
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t c = c8 * 8u + j;
      uint8_t code = NH_UNKNOWN;
      if (c < G.ncell) code = classify_cell(D, c, (uint8_t)(m8 >> (8 * j)), G.W, goal, gx, gy);
      codes |= (uint64_t)code << (8 * j);
    }
    reinterpret_cast<uint64_t*>(nh_base + slot * stride)[c8] = codes;
  }
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
// K3 (small grids, ncell <= 1024): the same exact A*, heap in LDS.
// Heap entry u32: f:11 | g:10 | cell:11 (key = entry >> 11, same order as above);
// each lane's heap is interleaved with its block-mates (element i of lane t at
// i*BLK + t), so lanes touching equal heap depths never share an LDS bank.
// g_score u16 per cell in HBM/L2 per slot: tag:4 | label:2 | g:10.
// A query whose heap would exceed HCAP is handed to k_astar via the overflow list.
// ----------------------------------------------------------------------------
constexpr uint32_t LDS_HCAP = 128;
constexpr uint32_t LDS_BLK = 256;

__device__ __forceinline__ void lheap_sift_up(uint32_t* Hs, uint32_t t, uint32_t pos, uint32_t elem) {
  const uint32_t k = elem >> 11;
  while (pos > 0) {
    const uint32_t parent = (pos - 1u) >> 1;
    const uint32_t pe = Hs[parent * LDS_BLK + t];
    if (k >= (pe >> 11)) break;
    Hs[pos * LDS_BLK + t] = pe;
    pos = parent;
  }
  Hs[pos * LDS_BLK + t] = elem;
}

__device__ __forceinline__ uint32_t lheap_pop(uint32_t* Hs, uint32_t t, uint32_t& len) {
  const uint32_t end = --len;
  const uint32_t last = Hs[end * LDS_BLK + t];
  if (end == 0) return last;
  const uint32_t top = Hs[t];
  uint32_t pos = 0, child = 1;
  while (child + 1u < end) {
    uint32_t l = Hs[child * LDS_BLK + t];
    const uint32_t r = Hs[(child + 1) * LDS_BLK + t];
    if ((l >> 11) >= (r >> 11)) {
      ++child;
      l = r;
    }
    Hs[pos * LDS_BLK + t] = l;
    pos = child;
    child = 2u * pos + 1u;
  }
  if (child == end - 1u) {
    Hs[pos * LDS_BLK + t] = Hs[child * LDS_BLK + t];
    pos = child;
  }
  lheap_sift_up(Hs, t, pos, last);
  return top;
}

__global__ void __launch_bounds__(LDS_BLK) k_astar_lds(DevGrid G, const AstarQuery* __restrict__ Q, uint32_t nq,
                                                        uint8_t* __restrict__ nh_base, uint64_t nstride,
                                                        uint8_t* __restrict__ res, int32_t* __restrict__ lens,
                                                        uint16_t* __restrict__ gs_all, uint32_t* __restrict__ epochs,
                                                        uint32_t nslots, AstarQuery* __restrict__ ovf,
                                                        uint32_t* __restrict__ novf, uint32_t* __restrict__ qnext) {
  __shared__ uint32_t Hs[LDS_HCAP * LDS_BLK];
  const uint32_t t = threadIdx.x;
  const uint32_t slot = blockIdx.x * LDS_BLK + t;
  if (slot >= nslots || slot >= nq) return;
  const uint32_t W = G.W, ncell = G.ncell;
  const float invW = 1.0f / (float)W;
  uint16_t* GS = gs_all + (uint64_t)slot * ncell;
  uint32_t ep = epochs[slot];
  // first query static (qi = slot), then dynamic dequeue: query times vary by orders of
  // magnitude, so lanes that finish early take the rest instead of a fixed stride
  for (uint32_t qi = slot; qi < nq; qi = nslots + atomicAdd(qnext, 1u)) {
    if (ep % 15u == 0u && ep > 0u)
      for (uint32_t c = 0; c < ncell; ++c) GS[c] = 0;
    const uint32_t tagw = (ep % 15u + 1u) << 12;
    ++ep;
    const AstarQuery q = Q[qi];
    const uint32_t v = q.v, goal = q.goal;
    const uint32_t vy = fast_div(v, W, invW), vx = v - vy * W;
    const uint32_t gy = fast_div(goal, W, invW), gx = goal - gy * W;
    uint8_t code = NH_STAY;
    int32_t L = 1;
    if (v != goal) {
      GS[v] = (uint16_t)tagw;
      Hs[t] = ((vx > gx ? vx - gx : gx - vx) + (vy > gy ? vy - gy : gy - vy)) << 21 | v;
      uint32_t len = 1;
      bool found = false, overflow = false;
      while (len > 0) {
        const uint32_t e = lheap_pop(Hs, t, len);
        const uint32_t c = e & 0x7FFu, cg = (e >> 11) & 0x3FFu;
        if (c == goal) {
          code = (uint8_t)((GS[goal] >> 10) & 3u);
          L = (int32_t)cg + 1;
          found = true;
          break;
        }
        const uint32_t cy = fast_div(c, W, invW), cx = c - cy * W;
        const uint8_t m = G.nbmask[c];
        const uint32_t labc = (GS[c] >> 10) & 3u;
        const uint32_t tg = cg + 1u;
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
          if (!(m & (1u << d))) continue;
          const uint32_t nx = d == 1 ? cx + 1 : (d == 3 ? cx - 1 : cx);
          const uint32_t ny = d == 0 ? cy + 1 : (d == 2 ? cy - 1 : cy);
          const uint32_t nc = ny * W + nx;
          const uint32_t old = GS[nc];
          const uint32_t oldg = ((old & 0xF000u) == tagw) ? (old & 0x3FFu) : 0xFFFFu;
          if (tg < oldg) {
            const uint32_t lab = cg == 0 ? d : labc;
            GS[nc] = (uint16_t)(tagw | (lab << 10) | tg);
            if (len >= LDS_HCAP) {
              overflow = true;
              break;
            }
            const uint32_t h = (nx > gx ? nx - gx : gx - nx) + (ny > gy ? ny - gy : gy - ny);
            lheap_sift_up(Hs, t, len, ((tg + h) << 21) | (tg << 11) | nc);
            ++len;
          }
        }
        if (overflow) break;
      }
      if (overflow) {
        ovf[atomicAdd(novf, 1u)] = q;  // resolved by k_astar (global-memory heap)
        continue;
      }
      if (!found) {
        code = fallback_code(G.nbmask[v], vx, vy, gx, gy);
        L = 2;
      }
    }
    if (res) res[q.out] = code;
    if (lens) lens[q.out] = L;
    if (nh_base && q.tab >= 0) nh_base[(uint64_t)q.tab * nstride + q.v] = code;
  }
  epochs[slot] = ep;
}

__global__ void __launch_bounds__(64) k_astar(DevGrid G, const AstarQuery* __restrict__ Q,
                                              const uint32_t* __restrict__ nq_dev, uint32_t nq_host,
                                              uint8_t* __restrict__ nh_base, uint64_t nstride,
                                              uint8_t* __restrict__ res, int32_t* __restrict__ lens,
                                              uint64_t* __restrict__ heaps, uint32_t hcap,
                                              uint32_t* __restrict__ gs_all, uint32_t* __restrict__ epochs,
                                              uint32_t nslots, uint32_t* __restrict__ err) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= nslots) return;
  const uint32_t nq = nq_dev ? *nq_dev : nq_host;
  if (slot >= nq) return;
  uint64_t* Hp = heaps + (uint64_t)slot * hcap;
  uint32_t* GS = gs_all + (uint64_t)slot * G.ncell;
  uint32_t ep = epochs[slot];
  for (uint32_t qi = slot; qi < nq; qi += nslots) {
    if (ep % 1023u == 0u && ep > 0u)
      for (uint32_t c = 0; c < G.ncell; ++c) GS[c] = 0u;
    const uint32_t tag = ep % 1023u + 1u;
    ++ep;
    const AstarQuery q = Q[qi];
    int32_t L = 0;
    const uint8_t code = astar_one(G, q.v, q.goal, tag, Hp, hcap, GS, &L, err);
    if (res) res[q.out] = code;
    if (lens) lens[q.out] = L;
    if (nh_base && q.tab >= 0) nh_base[(uint64_t)q.tab * nstride + q.v] = code;
  }
  epochs[slot] = ep;
}

// astar_one with a BYTE g_score per cell (LDS-resident on grids of up to ~120k cells):
// bit 7 valid | label:2 | h:5 with g = manhattan(start, cell) + 2h (g and the Manhattan
// distance from the start have the same parity on a 4-grid, and g >= it). A g that would
// need h > 31, or a heap longer than hcap, returns NH_UNKNOWN with *len_out = -2 (the caller
// hands the query to the u32 g_score kernel). Same heap, same relaxations, same labels.
__device__ __forceinline__ uint8_t astar_one_b8(const DevGrid& G, uint32_t v, uint32_t goal, uint64_t* Hp,
                                                uint32_t hcap, uint8_t* GB, int32_t* len_out) {
  const uint32_t W = G.W;
  const uint32_t vx = v % W, vy = v / W, gx = goal % W, gy = goal / W;
  if (v == goal) {
    *len_out = 1;
    return NH_STAY;
  }
  uint32_t len = 0;
  GB[v] = 0x80u;
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
      return (uint8_t)((GB[goal] >> 5) & 3u);
    }
    const uint8_t m = G.nbmask[c];
    const uint32_t labc = (GB[c] >> 5) & 3u;
    const uint32_t tg = cg + 1u;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
      if (!(m & (1u << d))) continue;
      const uint32_t nx = d == 1 ? cx + 1 : (d == 3 ? cx - 1 : cx);
      const uint32_t ny = d == 0 ? cy + 1 : (d == 2 ? cy - 1 : cy);
      const uint32_t nc = ny * W + nx;
      const uint32_t man = (nx > vx ? nx - vx : vx - nx) + (ny > vy ? ny - vy : vy - ny);
      const uint32_t old = GB[nc];
      const uint32_t oldg = (old & 0x80u) ? man + 2u * (old & 31u) : 0xFFFFFFFFu;
      if (tg < oldg) {
        const uint32_t hh = (tg - man) >> 1;
        if (hh > 31u || len >= hcap) {
          *len_out = -2;
          return NH_UNKNOWN;
        }
        const uint32_t lab = cg == 0 ? d : labc;
        GB[nc] = (uint8_t)(0x80u | (lab << 5) | hh);
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
//    child is taken, stop at a childless node) is walked in SALU. The path's values move up one
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

// BinaryHeap::pop (swap last into the root, sift_down_to_bottom(0), sift_up(0, hole)); len >= 1.
// Window lanes: lane j < 62 <-> depth kk = log2(j + 2) (1..5), index ki = j + 2 - 2^kk below the
// hole; the first window's lanes 62 / 63 fetch the last element / the root.
__device__ __forceinline__ uint64_t wpop(uint64_t* Hp, uint32_t& len, uint32_t lane) {
  constexpr uint64_t M62 = (1ull << 62) - 1ull, EVEN = 0x5555555555555555ull;
  const uint32_t end = --len;
  uint32_t pos = 0;
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
      if (end == 0) return last;
    }
    const uint32_t key = hk(val);
    const uint32_t sib = (uint32_t)__builtin_amdgcn_mov_dpp((int)key, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    const uint64_t VL = ballot64(node < end) & M62;
    // left child lane (even) takes the right child when left <= right and the right exists
    const uint64_t CR = ballot64(key >= sib) & (VL >> 1) & EVEN;
    uint32_t idx = 0, d = 0, live = 1;
#pragma unroll
    for (uint32_t k = 1; k <= 5; ++k) {  // branch-free SALU walk down the path
      const uint32_t ll = (1u << k) - 2u + 2u * idx;
      live &= (uint32_t)(VL >> ll) & 1u;
      idx = live ? 2u * idx + ((uint32_t)(CR >> ll) & 1u) : idx;
      d += live;
    }
    if (d == 0) break;
    const bool on = kk <= d && ki == (idx >> (d - kk));
    wave_order();
    if (on) Hp[(node - 1u) >> 1] = val;  // move up into the parent
    wave_order();
    pos = ((pos + 1u) << d) - 1u + idx;
    if (d < 5) break;
  }
  wsift_up(Hp, pos, last, lane);
  return top;
}

// FB: the grid's free-cell row bitmap (DevGrid::freebits) staged in LDS, so relaxing a node
// needs no global load.
// PROF: pr[0..4] = pops, clocks in pops, in relaxations, in pushes, pushes (TSW_ASTAR_PROF)
template <int GSM, bool PROF>
__device__ __forceinline__ uint8_t astar_wave_par(const DevGrid& G, uint32_t v, uint32_t goal, uint32_t tag,
                                                  uint64_t* Hp, uint32_t hcap, uint32_t* GS, uint8_t* GB,
                                                  const uint32_t* FB, int32_t* len_out, unsigned long long* pr) {
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
  if (lane == 0) {
    if constexpr (GSM == 2) GB[v] = 0x80u;
    else GS[v] = tagw;
    Hp[0] = ((uint64_t)(h0 << 15) << 32) | (vx << 16) | vy;
  }
  wave_order();
  if constexpr (PROF) tk = __builtin_amdgcn_s_memtime();
  uint32_t len = 1;
  // lanes 0..3 own the neighbour in direction `lane` (S, E, N, W: tswap.rs:62-73)
  const uint32_t dd = lane & 3u;
  while (len > 0) {
    ++pops;
    const uint64_t e = wpop(Hp, len, lane);
    tick(c_pop);
    const uint32_t cx = (uint32_t)(e >> 16) & 0xFFFFu, cy = (uint32_t)e & 0xFFFFu;
    const uint32_t cg = hk(e) & 0x7FFFu;
    const uint32_t c = cy * W + cx;
    if (c == goal) {
      flush();
      *len_out = (int32_t)cg + 1;
      if constexpr (GSM == 2) return (uint8_t)((GB[goal] >> 5) & 3u);
      else return (uint8_t)((GS[goal] >> 20) & 3u);
    }
    // neighbour of lane dd (unsigned wrap: x - 1 at x = 0 fails the bound test); every lane
    // reads (out-of-grid lanes re-read the popped cell), the LDS reads issue together
    const uint32_t nx = dd == 1 ? cx + 1 : (dd == 3 ? cx - 1 : cx);
    const uint32_t ny = dd == 0 ? cy + 1 : (dd == 2 ? cy - 1 : cy);
    const bool inb = lane < 4u && nx < W && ny < H;
    const uint32_t fx = inb ? nx : cx, fy = inb ? ny : cy;
    const uint32_t nc = fy * W + fx;
    const uint32_t fw = FB[fy * Ww + (fx >> 5)];
    uint32_t old, labc;
    if constexpr (GSM == 2) {
      old = GB[nc];
      labc = (GB[c] >> 5) & 3u;
    } else {
      old = GS[nc];
      labc = (GS[c] >> 20) & 3u;
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
      ent = ((uint64_t)((f << 15) | tg) << 32) | (fx << 16) | fy;
    }
    uint64_t M = ballot64(imp);
    tick(c_nb);
    if (ballot64(ovf) != 0ull || len + (uint32_t)__popcll(M) > hcap) {
      *len_out = -2;
      return NH_UNKNOWN;
    }
    wave_order();
    while (M) {
      const uint32_t d = (uint32_t)__builtin_ctzll(M);
      M &= M - 1ull;
      wsift_up(Hp, len, rl64(ent, d), lane);
      ++len;
      ++npush;
    }
    tick(c_push);
  }
  flush();
  *len_out = 2;
  return fallback_code(G.nbmask[v], vx, vy, gx, gy);
}

// ----------------------------------------------------------------------------
// K3 (grids of > 1024 cells): the same exact A* (astar_one), ONE QUERY PER WAVE with the heap
// in LDS and, when the grid fits (WAVE_GS_LDS_MAX cells), the g_score words in LDS too. The
// planner's lazy mode exits to the host whenever a step needs unresolved next hops, so K3
// runs in many small batches and its latency is the slowest query of a batch: a heap sift
// step here is an LDS round trip instead of a dependent global load. Queries whose heap
// outgrows the LDS heap go to the overflow list (k_astar, global-memory heap).
// ----------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_astar_wave(DevGrid G, const AstarQuery* __restrict__ Q, uint32_t nq,
                                                   uint8_t* __restrict__ nh_base, uint64_t nstride,
                                                   uint8_t* __restrict__ res, int32_t* __restrict__ lens,
                                                   uint32_t hcap, uint32_t gs_lds, uint32_t* __restrict__ gs_all,
                                                   uint32_t* __restrict__ epochs, AstarQuery* __restrict__ ovf,
                                                   uint32_t* __restrict__ novf, uint32_t serial,
                                                   unsigned long long* __restrict__ prof,
                                                   uint32_t* __restrict__ qnext) {
  extern __shared__ __align__(16) uint64_t wsm[];
  uint64_t* Hp = wsm;
  const uint32_t lane = threadIdx.x, ncell = G.ncell;
  // gs_lds: 0 = u32 g_scores in global slots, 1 = u32 in LDS, 2 = bytes in LDS (astar_one_b8)
  uint32_t* GS = gs_lds == 1u ? reinterpret_cast<uint32_t*>(wsm + hcap) : gs_all + (uint64_t)blockIdx.x * ncell;
  uint8_t* GB = reinterpret_cast<uint8_t*>(wsm + hcap);
  // free-cell bitmap after the heap and the LDS g_scores (wave_lds_bytes' carve)
  const uint32_t gsb = gs_lds == 1u ? ncell * 4u : gs_lds == 2u ? (ncell + 15u) / 16u * 16u : 0u;
  uint32_t* FB = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(wsm + hcap) + gsb);
  const uint32_t nfw = G.H * G.Ww;
  if (!serial)
    for (uint32_t t = lane; t < nfw; t += 64u) FB[t] = G.freebits[t];
  uint32_t ep = gs_lds ? 0u : epochs[blockIdx.x];
  if (gs_lds == 1u)
    for (uint32_t c = lane; c < ncell; c += 64u) GS[c] = 0u;
  __syncthreads();
  // first query static (qi = block), then dynamic dequeue (lane 0's atomic, read by the whole
  // wave): a batch's query times vary by orders of magnitude, a fixed stride idles waves
  auto next_q = [&](uint32_t qi) -> uint32_t {
    if (!qnext) return qi + gridDim.x;
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(qnext, 1u);
    return gridDim.x + (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
  };
  for (uint32_t qi = blockIdx.x; qi < nq; qi = next_q(qi)) {
    if (gs_lds == 2u) {
      uint4* g4 = reinterpret_cast<uint4*>(GB);
      for (uint32_t c = lane; c < (ncell + 15u) / 16u; c += 64u) g4[c] = make_uint4(0u, 0u, 0u, 0u);
    } else if (ep % 1023u == 0u && ep > 0u) {
      for (uint32_t c = lane; c < ncell; c += 64u) GS[c] = 0u;
      __threadfence_block();
    }
    __syncthreads();
    const uint32_t tag = ep % 1023u + 1u;
    ++ep;
    const AstarQuery q = Q[qi];
    int32_t L = 0;
    uint8_t code = NH_UNKNOWN;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long pr[5] = {0, 0, 0, 0, 0};
    if (!serial && prof) {
      code = gs_lds == 2u ? astar_wave_par<2, true>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, FB, &L, pr)
                          : astar_wave_par<1, true>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, FB, &L, pr);
    } else if (!serial) {
      code = gs_lds == 2u ? astar_wave_par<2, false>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, FB, &L, pr)
                          : astar_wave_par<1, false>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, FB, &L, pr);
    } else if (lane == 0) {
      code = gs_lds == 2u ? astar_wave_core<2>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, &L)
                          : astar_wave_core<1>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, &L);
    }
    if (prof && lane == 0) {  // TSW_ASTAR_PROF: pops, shader clocks, 100 MHz ticks per query
      prof[8ull * qi + 1] = __builtin_amdgcn_s_memtime() - t0;
      prof[8ull * qi + 2] = __builtin_amdgcn_s_memrealtime() - r0;
      prof[8ull * qi] = pr[0];
      for (int j = 1; j < 5; ++j) prof[8ull * qi + 2 + j] = pr[j];
    }
    if (lane == 0) {
      if (L == -2) {
        ovf[atomicAdd(novf, 1u)] = q;  // heap outgrew LDS: resolved by k_astar
      } else {
        if (res) res[q.out] = code;
        if (lens) lens[q.out] = L;
        if (nh_base && q.tab >= 0) nh_base[(uint64_t)q.tab * nstride + q.v] = code;
      }
    }
  }
  if (!gs_lds && lane == 0) epochs[blockIdx.x] = ep;
}

// Enqueue every unresolved (goal, cell) of the given table slots (eager mode).
__global__ void k_enqueue_unknown(DevGrid G, const uint32_t* __restrict__ goals,
                                  const uint32_t* __restrict__ slots, uint32_t k,
                                  uint8_t* __restrict__ nh, uint64_t nstride, AstarQuery* __restrict__ Q,
                                  uint32_t* __restrict__ qcount, uint32_t qcap) {
  const uint64_t total = (uint64_t)k * G.ncell;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t gi = (uint32_t)(idx / G.ncell), c = (uint32_t)(idx % G.ncell);
    const uint32_t slot = slots[gi];
    uint8_t* p = nh + (uint64_t)slot * nstride + c;
    if (*p != NH_UNKNOWN) continue;
    if (!(G.nbmask[c] & NB_FREE)) continue;
    const uint32_t qi = atomicAdd(qcount, 1u);
    if (qi >= qcap) continue;  // host sees count > cap and retries
    *p = NH_PENDING;
    AstarQuery q;
    q.v = c;
    q.goal = goals[gi];
    q.tab = (int32_t)slot;
    q.out = qi;
    Q[qi] = q;
  }
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------
size_t bfs_lds_bytes(const DevGrid& G, bool lds_table) {
  const size_t nwp = ((size_t)G.H * G.Ww + 3u) & ~(size_t)3u;
  size_t b = 4u * nwp * 4u;
  if (lds_table) b += (((size_t)G.ncell + 7u) & ~(size_t)7u) * 2u;
  return b;
}

hipError_t launch_bfs(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                      uint16_t* dist_base, uint64_t dstride, uint8_t* nh_base, uint64_t nstride,
                      uint32_t* err, int max_lds, int num_cu, hipStream_t s) {
  if (k == 0) return hipSuccess;
  size_t lds_tab = bfs_lds_bytes(G, true);
  size_t lds_no = bfs_lds_bytes(G, false);
  const bool use_tab = lds_tab <= (size_t)max_lds;
  const size_t lds = use_tab ? lds_tab : lds_no;
  if (lds > (size_t)max_lds) return hipErrorInvalidValue;
  const uint32_t nw = G.H * G.Ww;
  uint32_t bd;
  if (lds > 80 * 1024) bd = 1024;
  else if (nw <= 64) bd = 64;
  else if (nw <= 1024) bd = 256;
  else bd = 512;
  const uint32_t per_cu = (uint32_t)std::max<size_t>(1, (160 * 1024) / std::max<size_t>(lds, 1));
  uint32_t grid = std::min<uint32_t>(k, (uint32_t)num_cu * std::min<uint32_t>(per_cu, 16u) * 4u);
  if (grid == 0) grid = 1;
  if (use_tab) {
    hipFuncSetAttribute((const void*)k_bfs<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_bfs<true>, dim3(grid), dim3(bd), lds, s, G, goals, slots, k, dist_base, dstride,
                       nh_base, nstride, err);
  } else {
    hipFuncSetAttribute((const void*)k_bfs<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_bfs<false>, dim3(grid), dim3(bd), lds, s, G, goals, slots, k, dist_base, dstride,
                       nh_base, nstride, err);
  }
  return hipGetLastError();
}

hipError_t launch_classify(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                           const uint16_t* dist_base, uint64_t stride, uint8_t* nh_base, hipStream_t s) {
  if (k == 0) return hipSuccess;
  const uint64_t total = (uint64_t)k * ((G.ncell + 7u) / 8u);
  const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(k_classify, dim3(grid), dim3(256), 0, s, G, goals, slots, k, dist_base, stride, nh_base);
  return hipGetLastError();
}

hipError_t launch_astar(const DevGrid& G, const AstarQuery* Q, const uint32_t* nq_dev, uint32_t nq_host,
                        uint32_t launch_threads, uint8_t* nh_base, uint64_t nstride, uint8_t* res,
                        int32_t* lens, uint64_t* heaps, uint32_t hcap, uint32_t* gs_all, uint32_t* epochs,
                        uint32_t nslots, uint32_t* err, hipStream_t s) {
  if (launch_threads == 0) return hipSuccess;
  const uint32_t th = std::min(launch_threads, nslots);
  const uint32_t grid = (th + 63) / 64;
  hipLaunchKernelGGL(k_astar, dim3(grid), dim3(64), 0, s, G, Q, nq_dev, nq_host, nh_base, nstride, res, lens,
                     heaps, hcap, gs_all, epochs, th, err);
  return hipGetLastError();
}

hipError_t launch_astar_lds(const DevGrid& G, const AstarQuery* Q, uint32_t nq, uint8_t* nh_base, uint64_t nstride,
                            uint8_t* res, int32_t* lens, uint16_t* gs16, uint32_t* epochs, uint32_t nslots,
                            AstarQuery* ovf, uint32_t* novf, uint32_t* qnext, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  const uint32_t th = std::min(nq, nslots);
  const uint32_t grid = (th + LDS_BLK - 1) / LDS_BLK;
  hipLaunchKernelGGL(k_astar_lds, dim3(grid), dim3(LDS_BLK), 0, s, G, Q, nq, nh_base, nstride, res, lens, gs16,
                     epochs, th, ovf, novf, qnext);
  return hipGetLastError();
}

bool astar_lds_ok(const DevGrid& G) { return G.ncell <= 1024u; }

constexpr uint32_t WAVE_HCAP = 4096;              // LDS heap entries (32 KiB)
constexpr uint32_t WAVE_GS_LDS_MAX = 24u * 1024u;   // cells whose u32 g_score words fit LDS beside it
constexpr uint32_t WAVE_GB_LDS_MAX = 120u * 1024u;  // cells whose byte g_scores fit LDS beside it

static uint32_t wave_gs_mode(const DevGrid& G) {
  return G.ncell <= WAVE_GS_LDS_MAX ? 1u : G.ncell <= WAVE_GB_LDS_MAX ? 2u : 0u;
}

constexpr size_t WAVE_LDS_MAX = 160u * 1024u;

// heap + LDS g_scores + free-cell bitmap (k_astar_wave's carve)
static size_t wave_lds_bytes(const DevGrid& G, uint32_t hcap, uint32_t m) {
  return (size_t)hcap * 8u + (m == 1u ? (size_t)G.ncell * 4u : m == 2u ? ((size_t)G.ncell + 15u) / 16u * 16u : 0u) +
         (size_t)G.H * G.Ww * 4u;
}

// largest heap (<= want) whose carve fits the 160 KiB of LDS
static uint32_t wave_fit_hcap(const DevGrid& G, uint32_t want, uint32_t m) {
  const size_t rest = wave_lds_bytes(G, 0, m);
  const size_t room = rest < WAVE_LDS_MAX ? (WAVE_LDS_MAX - rest) / 8u : 0u;
  return (uint32_t)std::min<size_t>(want, room);
}

bool astar_wave_lds_gs(const DevGrid& G) { return wave_gs_mode(G) != 0u; }

uint32_t astar_wave_slots(const DevGrid& G, int num_cu, bool global_gs) {
  const uint32_t m = global_gs ? 0u : wave_gs_mode(G);
  const size_t lds = wave_lds_bytes(G, wave_fit_hcap(G, WAVE_HCAP, m), m);
  const uint32_t per_cu = (uint32_t)std::max<size_t>(1, (160u * 1024u) / lds);
  return (uint32_t)num_cu * std::min<uint32_t>(per_cu, 16u);
}

hipError_t launch_astar_wave(const DevGrid& G, const AstarQuery* Q, uint32_t nq, uint8_t* nh_base, uint64_t nstride,
                             uint8_t* res, int32_t* lens, uint32_t* gs_all, uint32_t* epochs, uint32_t nslots,
                             AstarQuery* ovf, uint32_t* novf, uint32_t hcap, bool global_gs, hipStream_t s,
                             uint32_t* qnext, uint32_t diag) {
  if (nq == 0) return hipSuccess;
  const uint32_t gs_lds = global_gs ? 0u : wave_gs_mode(G);
  hcap = hcap ? std::max<uint32_t>(4u, std::min(hcap, WAVE_HCAP)) : WAVE_HCAP;
  hcap = wave_fit_hcap(G, hcap, gs_lds);  // overflowing queries are handed on
  if (hcap < 4u) return hipErrorInvalidValue;
  const size_t lds = wave_lds_bytes(G, hcap, gs_lds);
  const uint32_t grid = std::min(nq, nslots);
  hipError_t e = hipFuncSetAttribute((const void*)k_astar_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const uint32_t serial = (diag & ASTAR_DIAG_SERIAL) ? 1u : 0u;  // A/B and tests: lone-lane core
  unsigned long long* prof = nullptr;
  if (diag & ASTAR_DIAG_PROF) {
    e = hipMalloc(&prof, (size_t)nq * 64u);
    if (e != hipSuccess) return e;
    hipMemsetAsync(prof, 0, (size_t)nq * 64u, s);
  }
  hipLaunchKernelGGL(k_astar_wave, dim3(grid), dim3(64), lds, s, G, Q, nq, nh_base, nstride, res, lens, hcap,
                     gs_lds, gs_all, epochs, ovf, novf, serial, prof, qnext);
  e = hipGetLastError();
  if (prof) {
    std::vector<unsigned long long> h((size_t)nq * 8u);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), prof, h.size() * 8u, hipMemcpyDeviceToHost);
    hipFree(prof);
    size_t worst = 0;
    for (size_t i = 0; i < nq; ++i)
      if (h[8 * i + 2] > h[8 * worst + 2]) worst = i;
    const unsigned long long* w = &h[8 * worst];
    const double np = (double)std::max(1ull, w[0]);
    fprintf(stderr,
            "[k_astar_wave] nq %u gs_mode %u hcap %u | slowest: pops %llu clocks %llu real_us %.1f -> %.1f clk/pop "
            "(pop %.0f, relax %.0f, push %.0f; %.2f pushes/pop), %.3f us/pop, %.0f MHz\n",
            nq, gs_lds, hcap, w[0], w[1], w[2] / 100.0, w[1] / np, w[3] / np, w[4] / np, w[5] / np, w[6] / np,
            w[2] / 100.0 / np, (double)w[1] / std::max(1.0, w[2] / 100.0));
  }
  return e;
}

// Error recovery: every NH_PENDING / NH_PENDING_S code of the store back to NH_UNKNOWN (a K3 pass that failed
// after its pairs were marked must not leave them pending for later calls). 8 codes per thread.
__global__ void k_reset_pending(uint64_t* __restrict__ nh8, uint64_t n8) {
  constexpr uint64_t ONES = 0x0101010101010101ull, HIGH = 0x8080808080808080ull;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t w = nh8[i];
    // bytes equal to 0xFE: x = w ^ 0xFE.. has a zero byte there (classic zero-byte test, exact
    // after masking out borrows with ~x)
    // bytes 0xFE / 0xFD: w ^ 0xFE.. / w ^ 0xFD.. has a zero byte there (classic zero-byte test,
    // may flag a byte above a match too — the loop below checks each byte exactly)
    const uint64_t x1 = w ^ (ONES * (uint64_t)NH_PENDING), x2 = w ^ (ONES * (uint64_t)NH_PENDING_S);
    const uint64_t z = ((x1 - ONES) & ~x1 & HIGH) | ((x2 - ONES) & ~x2 & HIGH);
    if (z) {
      uint64_t out = w;
      for (int b = 0; b < 8; ++b) {
        const uint32_t c = (uint32_t)((w >> (8 * b)) & 0xFFu);
        if (c == NH_PENDING || c == NH_PENDING_S) out |= 0xFFull << (8 * b);
      }
      nh8[i] = out;
    }
  }
}

hipError_t launch_reset_pending(uint8_t* nh, uint64_t nbytes, hipStream_t s) {
  const uint64_t n8 = nbytes / 8u;  // table strides are multiples of 8
  if (n8 == 0) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n8 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_reset_pending, dim3(grid), dim3(256), 0, s, reinterpret_cast<uint64_t*>(nh), n8);
  return hipGetLastError();
}

hipError_t launch_enqueue_unknown(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                                  uint8_t* nh, uint64_t nstride, AstarQuery* Q, uint32_t* qcount,
                                  uint32_t qcap, hipStream_t s) {
  if (k == 0) return hipSuccess;
  const uint64_t total = (uint64_t)k * G.ncell;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(k_enqueue_unknown, dim3(grid), dim3(256), 0, s, G, goals, slots, k, nh, nstride, Q, qcount,
                     qcap);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Coop mode: persistent K3 worker waves running CONCURRENTLY with the planner (k_plan, one block).
// The planner publishes queued (cell, goal) pairs in two queues of CoopCtl — needed pairs a step
// is waiting on, and speculative prefetches — and keeps planning; each worker wave claims one pair
// at a time (needed first, CAS on the claim counter), runs the same exact A* as k_astar_wave (same
// BinaryHeap order, same hand-off chain: LDS heap + LDS g-scores -> LDS heap + global u32 g-scores
// -> global heap), and stores the code into the next-hop table with an agent-scope store the
// planner polls. Replaces the exit -> host sync -> K3 launch -> relaunch cycle of the exit mode:
// speculative pairs resolve on the 255 otherwise idle CUs while the planner runs, and the planner
// waits only for what a step needs.
// Termination: when the planner sets `stop` the workers drain the needed queue and exit (unclaimed
// speculative pairs are abandoned — the host resets them to UNKNOWN); an idle worker also exits
// after 5 s without work, whatever the planner does.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t w_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool w_cas(uint32_t* p, uint32_t expect, uint32_t want) {
  return __hip_atomic_compare_exchange_strong(p, &expect, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0: claim the next pair (0: needed queue, 1: speculative queue, 2: task chain, -1: exit).
// Task chains (long, lowest priority) only go to workers with take_t: the others stay free for the
// pairs the planner needs or will need soon.
__device__ int worker_claim(CoopCtl* cc, uint32_t* idx, bool take_t, const uint32_t* hflags) {
  const unsigned long long t0 = wall_clock64();
  // one pass over the queues in priority order: >= 0 claimed (queue id), -1 nothing, -2 stop
  auto scan = [&]() -> int {
    for (;;) {
      const uint32_t hn = w_ld(&cc->head_n), cn = w_ld(&cc->claim_n);
      if (cn < hn) {
        if (w_cas(&cc->claim_n, cn, cn + 1u)) {
          *idx = cn;
          return 0;
        }
        continue;
      }
      // relaxed poll (an acquire here would invalidate this XCD's L2 on every idle spin)
      if (w_ld(&cc->stop)) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        // the final needed head was published before `stop`: drain what is left, then exit
        if (w_ld(&cc->claim_n) < w_ld(&cc->head_n)) continue;
        return -2;
      }
      const uint32_t hs = w_ld(&cc->head_s), cs = w_ld(&cc->claim_s);
      if (cs < hs) {
        if (w_cas(&cc->claim_s, cs, cs + 1u)) {
          *idx = cs;
          return 1;
        }
        continue;
      }
      if (take_t) {
        const uint32_t ht = w_ld(&cc->head_t), ct = w_ld(&cc->claim_t);
        if (ct < ht) {
          if (w_cas(&cc->claim_t, ct, ct + 1u)) {
            *idx = ct;
            return 2;
          }
          continue;
        }
      }
      return -1;
    }
  };
  // Idle: poll only the planner's publish count (one load) and rescan the queues when it moves, or
  // every 64 polls as a safety net. Idle waves polling every head and claim word kept a few lines of
  // the fabric hot and slowed the planner's own memory accesses (worse the more workers run).
  uint32_t seen = w_ld(&cc->pub);
  for (;;) {
    const int r = scan();
    if (r >= 0) return r;
    if (r == -2) return -1;
    for (uint32_t k = 0;; ++k) {
      // host watchdog abort (pinned host memory, read over the host link: rarely)
      if ((k & 255u) == 255u && hflags &&
          __hip_atomic_load(&hflags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
        return -1;
      if (wall_clock64() - t0 > 500000000ull) return -1;  // 5 s idle: safety exit
      if (k < 8) __builtin_amdgcn_s_sleep(2);
      else __builtin_amdgcn_s_sleep(16);
      const uint32_t p = w_ld(&cc->pub);
      if (p != seen || (k & 63u) == 63u) {
        seen = p;
        break;
      }
    }
  }
}

// lane 0, non-blocking: claim one pair of the needed or the speculative queue (0 / 1), else -1.
// A worker walking a task chain calls this between hops, so chains (lowest priority, up to ~100
// A* each) never hold a worker while pairs the planner needs or will need soon are queued.
__device__ int worker_try_claim(CoopCtl* cc, uint32_t* idx) {
  for (;;) {
    const uint32_t hn = w_ld(&cc->head_n), cn = w_ld(&cc->claim_n);
    if (cn < hn) {
      if (w_cas(&cc->claim_n, cn, cn + 1u)) {
        *idx = cn;
        return 0;
      }
      continue;
    }
    const uint32_t hs = w_ld(&cc->head_s), cs = w_ld(&cc->claim_s);
    if (cs < hs) {
      if (w_cas(&cc->claim_s, cs, cs + 1u)) {
        *idx = cs;
        return 1;
      }
      continue;
    }
    return -1;
  }
}

// global g-score slot tag (k_astar / tier-2 scheme: tag:10 | label:2 | g:20, cleared every 1023)
__device__ __forceinline__ uint32_t slot_tag(uint32_t* GS, uint32_t ncell, uint32_t& ep, uint32_t lane) {
  if (ep % 1023u == 0u && ep > 0u) {
    for (uint32_t c = lane; c < ncell; c += 64u) GS[c] = 0u;
    __threadfence_block();
  }
  __syncthreads();
  const uint32_t tag = ep % 1023u + 1u;
  ++ep;
  return tag;
}

__global__ void __launch_bounds__(64) k_astar_worker(WorkerArgs A) {
  extern __shared__ __align__(16) uint64_t wsm[];
  const DevGrid G = A.G;
  uint64_t* Hp = wsm;
  const uint32_t lane = threadIdx.x, ncell = G.ncell, hcap = A.hcap, gs_lds = A.gs_lds;
  uint32_t* GSl = reinterpret_cast<uint32_t*>(wsm + hcap);  // gs_lds == 1
  uint8_t* GB = reinterpret_cast<uint8_t*>(wsm + hcap);      // gs_lds == 2
  const uint32_t gsb = gs_lds == 1u ? ncell * 4u : gs_lds == 2u ? (ncell + 15u) / 16u * 16u : 0u;
  const uint32_t* FB = G.freebits;
  if (A.stage_fb) {
    uint32_t* fb = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(wsm + hcap) + gsb);
    const uint32_t nfw = G.H * G.Ww;
    for (uint32_t t = lane; t < nfw; t += 64u) fb[t] = G.freebits[t];
    FB = fb;
  }
  if (gs_lds == 1u)
    for (uint32_t c = lane; c < ncell; c += 64u) GSl[c] = 0u;
  uint32_t* GSg = A.gs_all + (uint64_t)blockIdx.x * ncell;
  uint64_t* Hg = A.heaps + (uint64_t)blockIdx.x * A.ghcap;
  uint32_t ep = A.epochs[blockIdx.x], epl = 0;
  // a worker on the planner's XCD leaves at once: the planner's agent arrays, occupancy and table
  // lines then share that XCD's 4 MB L2 with nobody's g-score slots (wave-uniform exit, before `alive`)
  if (A.avoid_xcc) {
    const uint32_t px = w_ld(&A.cc->planner_xcc);
    if (px != 0u && px - 1u == (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20)) return;
  }
  __syncthreads();
  if (lane == 0) __hip_atomic_fetch_add(&A.cc->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // exact A* for (v, goal): tier 1 LDS heap + LDS (or global) g-scores, tier 2 global u32
  // g-scores, tier 3 global heap (the k_astar_wave -> k_astar hand-off chain, in one wave)
  auto resolve_exact = [&](uint32_t v, uint32_t goal) -> uint8_t {
    int32_t L = 0;
    uint8_t code = NH_UNKNOWN;
    if (gs_lds == 2u) {
      uint4* g4 = reinterpret_cast<uint4*>(GB);
      for (uint32_t c = lane; c < (ncell + 15u) / 16u; c += 64u) g4[c] = make_uint4(0u, 0u, 0u, 0u);
      __syncthreads();
      code = astar_wave_par<2, false>(G, v, goal, 0u, Hp, hcap, nullptr, GB, FB, &L, nullptr);
    } else if (gs_lds == 1u) {
      if (epl % 1023u == 0u && epl > 0u) {
        for (uint32_t c = lane; c < ncell; c += 64u) GSl[c] = 0u;
      }
      __syncthreads();
      const uint32_t tag = epl % 1023u + 1u;
      ++epl;
      code = astar_wave_par<1, false>(G, v, goal, tag, Hp, hcap, GSl, nullptr, FB, &L, nullptr);
    } else {
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      code = astar_wave_par<1, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FB, &L, nullptr);
    }
    if (L == -2 && gs_lds != 0u) {
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      code = astar_wave_par<1, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FB, &L, nullptr);
    }
    if (L == -2) {
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      if (lane == 0) code = astar_one(G, v, goal, tag, Hg, A.ghcap, GSg, &L, &A.cc->err);
      code = (uint8_t)__builtin_amdgcn_readfirstlane(code);
    }
    return code;
  };
  uint32_t cur_q = 0;  // diagnostics: queue of the query being resolved (0 needed, 1 spec, 2 chain)
  auto resolve = [&](uint32_t v, uint32_t goal) -> uint8_t {
    const unsigned long long tr0 = wall_clock64();
    const uint8_t code = resolve_exact(v, goal);
    if (lane == 0) {
      __hip_atomic_fetch_add(&A.cc->wbusy[cur_q], wall_clock64() - tr0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&A.cc->wcount[cur_q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return code;
  };
  // the code (or NH_UNKNOWN after a global-heap overflow, flagged in cc->err): an agent-scope
  // store the planner's polling load sees
  auto publish_code = [&](uint32_t v, int32_t tab, uint8_t code, bool chain) {
    if (lane == 0 && tab >= 0) {
      __hip_atomic_store(A.nh + (uint64_t)tab * A.nstride + v, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&A.cc->worker_queries, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (chain) __hip_atomic_fetch_add(&A.cc->chain_queries, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  auto code_at = [&](uint32_t v, int32_t tab) -> uint8_t {  // current code, past stale caches
    const uint8_t* p = A.nh + (uint64_t)tab * A.nstride + v;
    const uint32_t w = w_ld(reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3u));
    return (uint8_t)(w >> (8u * (uint32_t)((uintptr_t)p & 3u)));
  };
  const bool take_t = (blockIdx.x & A.tmask) == A.tmask;
  for (;;) {
    int which = -1;
    uint32_t idx = 0;
    if (lane == 0) which = worker_claim(A.cc, &idx, take_t, A.hflags);
    which = __builtin_amdgcn_readfirstlane(which);
    if (which < 0) break;
    idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
    // the entry was published by the planner's release of the head (or by the host before the
    // launch): read it past stale caches
    const uint32_t* e = reinterpret_cast<const uint32_t*>((which == 0 ? A.QN : which == 1 ? A.QS : A.QT) + idx);
    const uint32_t v = w_ld(e), goal = w_ld(e + 1);
    const int32_t tab = (int32_t)w_ld(e + 2);
    cur_q = (uint32_t)which;
    if (which < 2) {
      publish_code(v, tab, resolve(v, goal), false);
      continue;
    }
    // task chain: the path an agent carrying this task walks from its pickup to the delivery
    // (every hop is get_path(cell, delivery)[1], tswap.rs:263-266): follow resolved codes and
    // resolve each unresolved hop in turn; stop at a pair someone else has queued, at a stay code,
    // or at the goal. Pairs are not marked pending, so an abandoned chain leaves nothing behind.
    if (tab < 0) continue;
    uint32_t c = v;
    for (uint32_t hop = 0; hop < ncell && c != goal; ++hop) {
      // the planner is done: abandon the rest of the chain (nothing is marked pending)
      if ((uint32_t)__builtin_amdgcn_readfirstlane(lane == 0 ? w_ld(&A.cc->stop) : 0u)) break;
      // pairs the planner queued meanwhile come first (A.preempt)
      while (A.preempt) {
        int w2 = -1;
        uint32_t i2 = 0;
        if (lane == 0) w2 = worker_try_claim(A.cc, &i2);
        w2 = __builtin_amdgcn_readfirstlane(w2);
        if (w2 < 0) break;
        i2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)i2);
        const uint32_t* e2 = reinterpret_cast<const uint32_t*>((w2 == 0 ? A.QN : A.QS) + i2);
        const uint32_t v2 = w_ld(e2), g2 = w_ld(e2 + 1);
        const int32_t t2 = (int32_t)w_ld(e2 + 2);
        cur_q = (uint32_t)w2;
        publish_code(v2, t2, resolve(v2, g2), false);
        cur_q = 2u;
      }
      uint8_t code = (uint8_t)__builtin_amdgcn_readfirstlane(lane == 0 ? code_at(c, tab) : 0u);
      if (code == NH_UNKNOWN) {
        code = resolve(c, goal);
        publish_code(c, tab, code, true);
      }
      if (code >= NH_STAY) break;  // stay (unreachable goal), pending elsewhere, or overflow
      c = step_cell(c, code, G.W);
    }
  }
  if (lane == 0) A.epochs[blockIdx.x] = ep;
}

WorkerCfg worker_config(const DevGrid& G, int num_cu, uint32_t n_agents, uint32_t hcap_want, int force_gs) {
  const size_t fbb = (size_t)G.H * G.Ww * 4u;
  const uint32_t want = hcap_want ? std::min(hcap_want, WAVE_HCAP) : WAVE_HCAP;
  auto make = [&](uint32_t m, bool fb) {
    WorkerCfg c{};
    c.gs_lds = m;
    c.stage_fb = fb ? 1u : 0u;
    const size_t gsb = m == 1u ? (size_t)G.ncell * 4u : m == 2u ? ((size_t)G.ncell + 15u) / 16u * 16u : 0u;
    const size_t rest = gsb + (fb ? fbb : 0u);
    c.hcap = rest < WAVE_LDS_MAX ? (uint32_t)std::min<size_t>(want, (WAVE_LDS_MAX - rest) / 8u) : 0u;
    c.lds = (size_t)c.hcap * 8u + rest;
    const uint32_t per_cu = c.lds ? (uint32_t)std::min<size_t>(16u, WAVE_LDS_MAX / c.lds) : 0u;
    c.waves = (uint32_t)num_cu * per_cu;
    return c;
  };
  const uint32_t m = wave_gs_mode(G);
  const bool fits = force_gs == 0 || (force_gs == 1 && G.ncell <= WAVE_GS_LDS_MAX) ||
                    (force_gs == 2 && G.ncell <= WAVE_GB_LDS_MAX);
  if (force_gs >= 0 && fits) {  // A/B: another g-score placement than the default
    WorkerCfg f = make((uint32_t)force_gs, true);
    if (f.hcap >= 64u) return f;
  }
  WorkerCfg c = make(m, true);
  // u32 LDS g-scores leave one wave per CU on a C3-sized grid; byte g-scores (tier-2 hand-off past a
  // 62-cell detour) run 3x the waves — A* latency is the same, the startup bursts drain faster
  // (C3 plan 585 -> 563 ms once idle workers stopped polling every queue word)
  if (m == 1u) {
    const WorkerCfg c2 = make(2u, true);
    if (c2.hcap >= 64u && c2.waves >= 2u * c.waves) c = c2;
  }
  // grids whose byte g-scores fit LDS (<= 120k cells): with many agents, trade the LDS g-scores for
  // 3x the waves (global u32 slots, L2-resident at this size)
  if (m != 0u && n_agents > 2000u && c.waves < 3u * (uint32_t)num_cu) c = make(0u, true);
  // larger grids keep one wave per CU with the bitmap in LDS: their 4 MB g-score slots would not
  // stay cache-resident with more waves, and the traffic slows the planner itself (C5: 3x)
  if (c.hcap < 64u) c = make(0u, false);
  return c;
}

hipError_t launch_astar_workers(const WorkerArgs& A0, const WorkerCfg& cfg, hipStream_t s) {
  WorkerArgs A = A0;
  A.gs_lds = cfg.gs_lds;
  A.stage_fb = cfg.stage_fb;
  A.hcap = cfg.hcap;
  const uint32_t waves = cfg.waves;
  if (A.hcap < 4u || waves == 0) return hipErrorInvalidValue;
  const size_t lds = cfg.lds;
  hipError_t e = hipFuncSetAttribute((const void*)k_astar_worker, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_astar_worker, dim3(waves), dim3(64), lds, s, A);
  return hipGetLastError();
}

}  // namespace tsw
