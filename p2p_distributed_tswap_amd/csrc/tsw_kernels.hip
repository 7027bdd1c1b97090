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
#include "tsw_astar.h"
#include "tsw_plan.h"

namespace tsw {


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
                                              uint32_t* __restrict__ err, uint8_t* __restrict__ govf) {
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
        if (tid == 0 && govf) govf[gi] = 1u;  // planned without a table (K3)
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
  // LDS and global g-scores are separate pointers for separate calls (a run-time selected pointer is
  // generic: flat loads on the pop's chain instead of ds_read)
  uint32_t* const GSl = reinterpret_cast<uint32_t*>(wsm + hcap);
  uint32_t* const GSg = gs_all + (uint64_t)blockIdx.x * ncell;
  uint32_t* GS = gs_lds == 1u ? GSl : GSg;
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
      code = gs_lds == 2u   ? astar_wave_par<2, true>(G, q.v, q.goal, tag, Hp, hcap, GSl, GB, FB, &L, pr)
             : gs_lds == 1u ? astar_wave_par<1, true>(G, q.v, q.goal, tag, Hp, hcap, GSl, GB, FB, &L, pr)
                            : astar_wave_par<1, true, 0, false>(G, q.v, q.goal, tag, Hp, hcap, GSg, GB, FB, &L, pr);
    } else if (!serial) {
      code = gs_lds == 2u   ? astar_wave_par<2, false>(G, q.v, q.goal, tag, Hp, hcap, GSl, GB, FB, &L, pr)
             : gs_lds == 1u ? astar_wave_par<1, false>(G, q.v, q.goal, tag, Hp, hcap, GSl, GB, FB, &L, pr)
                            : astar_wave_par<1, false, 0, false>(G, q.v, q.goal, tag, Hp, hcap, GSg, GB, FB, &L, pr);
    }
#ifdef TSW_DIAG
    else if (lane == 0) {  // lone-lane core (TSW_ASTAR_SERIAL A/B, diagnostic build only)
      code = gs_lds == 2u ? astar_wave_core<2>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, &L)
                          : astar_wave_core<1>(G, q.v, q.goal, tag, Hp, hcap, GS, GB, &L);
    }
#endif
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
                      uint32_t* err, int max_lds, int num_cu, hipStream_t s, uint8_t* govf) {
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
                       nh_base, nstride, err, govf);
  } else {
    hipFuncSetAttribute((const void*)k_bfs<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_bfs<false>, dim3(grid), dim3(bd), lds, s, G, goals, slots, k, dist_base, dstride,
                       nh_base, nstride, err, govf);
  }
  return hipGetLastError();
}

// The table store's format (round 6): per goal, u8 next-hop codes and u8 detour bytes
// DT[c] = min((D[c] - |c - goal|_1) / 2, 255), 255 also for blocked / unreachable cells (D and the
// Manhattan distance share parity on a 4-grid). A goal's u16 table D (index src[i], or i, of `dist`)
// goes into store slot slots[i]: codes (nh_base, unless null: imported codes are kept) and detour bytes.
__global__ void k_classify_dt(DevGrid G, const uint32_t* __restrict__ goals, const uint32_t* __restrict__ src,
                              const uint32_t* __restrict__ slots, uint32_t k, const uint16_t* __restrict__ dist,
                              uint64_t dstride, uint8_t* __restrict__ nh_base, uint8_t* __restrict__ dt_base,
                              uint64_t tstride) {
  const uint32_t ncp8 = (G.ncell + 7u) / 8u;
  const uint64_t total = (uint64_t)k * ncp8;
  for (uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t gi = (uint32_t)(idx / ncp8), c8 = (uint32_t)(idx % ncp8);
    const uint32_t goal = goals[gi];
    const uint64_t slot = slots[gi];
    const uint16_t* D = dist + (uint64_t)(src ? src[gi] : gi) * dstride;
    const uint32_t gx = goal % G.W, gy = goal / G.W;
    const uint64_t m8 = reinterpret_cast<const uint64_t*>(G.nbmask)[c8];
    uint64_t codes = 0, dts = 0;
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t c = c8 * 8u + j;
      uint8_t code = NH_UNKNOWN, db = DT_NONE;
      if (c < G.ncell) {
        if (nh_base) code = classify_cell(D, c, (uint8_t)(m8 >> (8 * j)), G.W, goal, gx, gy);
        const uint32_t d = D[c];
        if (d != DIST_INF) {
          const uint32_t y = c / G.W, x = c - y * G.W;
          const uint32_t man = (x > gx ? x - gx : gx - x) + (y > gy ? y - gy : gy - y);
          db = d < man ? DT_NONE : (uint8_t)min((d - man) >> 1, (uint32_t)DT_NONE);
        }
      }
      codes |= (uint64_t)code << (8 * j);
      dts |= (uint64_t)db << (8 * j);
    }
    if (nh_base) reinterpret_cast<uint64_t*>(nh_base + slot * tstride)[c8] = codes;
    reinterpret_cast<uint64_t*>(dt_base + slot * tstride)[c8] = dts;
  }
}

hipError_t launch_classify_dt(const DevGrid& G, const uint32_t* goals, const uint32_t* src, const uint32_t* slots,
                              uint32_t k, const uint16_t* dist, uint64_t dstride, uint8_t* nh_base, uint8_t* dt_base,
                              uint64_t tstride, hipStream_t s) {
  if (k == 0) return hipSuccess;
  const uint64_t total = (uint64_t)k * ((G.ncell + 7u) / 8u);
  const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(k_classify_dt, dim3(grid), dim3(256), 0, s, G, goals, src, slots, k, dist, dstride, nh_base,
                     dt_base, tstride);
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

// Caller-resolved K3 (tsw_plan_mapd_resolved / tsw_next_hop_codes): codes of queued (start, goal) pairs
// out of / into the next-hop store. Q[i].tab is the goal's table slot.
__global__ void k_gather_codes(const AstarQuery* __restrict__ Q, uint32_t nq, const uint8_t* __restrict__ nh,
                               uint64_t nstride, uint8_t* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += gridDim.x * blockDim.x) {
    const AstarQuery q = Q[i];
    out[i] = q.tab < 0 ? NH_UNKNOWN : nh[(uint64_t)q.tab * nstride + q.v];
  }
}
__global__ void k_put_codes(const AstarQuery* __restrict__ Q, uint32_t nq, const uint8_t* __restrict__ codes,
                            uint8_t* __restrict__ nh, uint64_t nstride) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += gridDim.x * blockDim.x) {
    const AstarQuery q = Q[i];
    if (q.tab >= 0) nh[(uint64_t)q.tab * nstride + q.v] = codes[i];
  }
}

hipError_t launch_gather_codes(const AstarQuery* Q, uint32_t nq, const uint8_t* nh, uint64_t nstride, uint8_t* out,
                               hipStream_t s) {
  if (nq == 0) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>((nq + 255u) / 256u, 4096u);
  hipLaunchKernelGGL(k_gather_codes, dim3(grid), dim3(256), 0, s, Q, nq, nh, nstride, out);
  return hipGetLastError();
}

hipError_t launch_put_codes(const AstarQuery* Q, uint32_t nq, const uint8_t* codes, uint8_t* nh, uint64_t nstride,
                            hipStream_t s) {
  if (nq == 0) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>((nq + 255u) / 256u, 4096u);
  hipLaunchKernelGGL(k_put_codes, dim3(grid), dim3(256), 0, s, Q, nq, codes, nh, nstride);
  return hipGetLastError();
}

// The pending markers of queue entries [from, to) back to NH_UNKNOWN (a coop plan's unclaimed
// speculative pairs): O(entries), where launch_reset_pending sweeps the whole store (C5: 18 GB).
__global__ void k_reset_queue(const AstarQuery* __restrict__ Q, uint32_t from, uint32_t to, uint8_t* __restrict__ nh,
                              uint64_t nstride) {
  for (uint32_t i = from + blockIdx.x * blockDim.x + threadIdx.x; i < to; i += gridDim.x * blockDim.x) {
    const AstarQuery q = Q[i];
    if (q.tab < 0) continue;
    uint8_t* p = nh + (uint64_t)q.tab * nstride + q.v;
    const uint8_t c = *p;
    if (c == NH_PENDING || c == NH_PENDING_S) *p = NH_UNKNOWN;
  }
}

hipError_t launch_reset_queue(const AstarQuery* Q, uint32_t from, uint32_t to, uint8_t* nh, uint64_t nstride,
                              hipStream_t s) {
  if (to <= from) return hipSuccess;
  const uint32_t grid = std::min<uint32_t>((to - from + 255u) / 256u, 4096u);
  hipLaunchKernelGGL(k_reset_queue, dim3(grid), dim3(256), 0, s, Q, from, to, nh, nstride);
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


WorkerCfg worker_config(const DevGrid& G, int num_cu, uint32_t n_agents, uint32_t hcap_want, int force_gs,
                        bool dag_exit, size_t lds_cap, int force_fb) {
  // the workers' LDS is the plan dispatch's per-workgroup request (the planner's, just under the
  // CU's 160 KiB): every carve below must fit THAT, not the CU (C5's bitmap + heap
  // came to 160 KiB, 2 KiB over the dispatch's request, and no worker fit — exit mode)
  const size_t WAVE_LDS_MAX = std::min<size_t>(lds_cap, ::tsw::WAVE_LDS_MAX);
  const size_t fbb = (size_t)G.H * G.Ww * 4u;
  const uint32_t want = hcap_want ? std::min(hcap_want, WAVE_HCAP) : WAVE_HCAP;
  // m: g-score placement; fb: free bitmap in LDS. With LDS g-scores the DAG early exit stages the
  // goal's detour bytes in LDS too (its reads then cost what a g-score read costs) and the heap gives
  // up entries past 1,024 for more waves per CU, up to one per SIMD (C3 queries peak below 300
  // entries; an overflowing query is handed to the next tier); with global g-scores it reads the
  // u16 table beside them.
  auto make = [&](uint32_t m, bool fb) {
    WorkerCfg c{};
    c.gs_lds = m;
    c.stage_fb = fb ? 1u : 0u;
    c.dag = !dag_exit ? 0u : m != 0u ? 1u : 2u;
    const size_t gsb = m == 1u ? (size_t)G.ncell * 4u : m == 2u ? ((size_t)G.ncell + 15u) / 16u * 16u : 0u;
    const size_t dtb = c.dag == 1u ? ((size_t)G.ncell + 15u) / 16u * 16u : 0u;
    const size_t rest = gsb + (fb ? fbb : 0u) + dtb;
    c.hcap = rest < WAVE_LDS_MAX ? (uint32_t)std::min<size_t>(want, (WAVE_LDS_MAX - rest) / 8u) : 0u;
    if (c.dag == 1u && c.hcap > 1024u && hcap_want == 0u) {
      const size_t pc = std::min<size_t>(4u, WAVE_LDS_MAX / (rest + 1024u * 8u));
      if (pc >= 1u) c.hcap = (uint32_t)std::min<size_t>(c.hcap, (WAVE_LDS_MAX / pc - rest) / 8u);
    }
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
  if (c.hcap < 64u) c = make(0u, false);
  // global g-score workers: the staged free bitmap saves one L2 read per relaxation but costs LDS; drop
  // it when that at least doubles the waves per CU (C5's 128 KiB bitmap left one wave per CU: plan
  // 8.6 s with 255 workers, 3.97 s with 910 without it, planner sections unchanged — round 4,
  // profiles/r4/c5_workers_ab.jsonl; round 3 measured the opposite in exit mode, before the coop
  // workers stopped with the planner). TSW_WORKER_FB=0 / 1 forces either.
  if (c.gs_lds == 0u && c.stage_fb != 0u && force_fb != 1) {
    const WorkerCfg nf = make(0u, false);
    if (nf.hcap >= 64u && (force_fb == 0 || nf.waves >= 2u * c.waves)) c = nf;
  }
  // heap-only workers (the bitmap-less global-g-score case, C5's 2^20 cells): a 2,048-entry LDS heap
  // doubles the waves per CU — C5 3.64-3.67 s with 1,020 workers -> 3.44-3.51 s with 2,295, no query
  // outgrowing it (profiles/r4/c5_slots_ab.txt); a larger heap would go to the global tier-3 heap
  if (c.gs_lds == 0u && c.stage_fb == 0u && hcap_want == 0u && c.hcap > 2048u) {
    const uint32_t h = 2048u;
    c.hcap = h;
    c.lds = (size_t)h * 8u;
    c.waves = (uint32_t)num_cu * (uint32_t)std::min<size_t>(16u, WAVE_LDS_MAX / c.lds);
  }
  // global g-score workers that keep the staged bitmap (wh10k's 112k cells: 14 KiB of bitmap): a 2,048-entry
  // heap too when that raises the waves per CU by half or more — round 5, busy wh10k: 765 -> 1,275 workers,
  // 11.07-11.13 -> 10.55 s, no query outgrowing the heap (profiles/r5/worker_cfg_ab.txt; round 4 measured
  // it neutral on the frozen instance)
  if (c.gs_lds == 0u && c.stage_fb != 0u && hcap_want == 0u && c.hcap > 2048u) {
    WorkerCfg h2 = c;
    const size_t rest = c.lds - (size_t)c.hcap * 8u;
    h2.hcap = 2048u;
    h2.lds = (size_t)h2.hcap * 8u + rest;
    h2.waves = (uint32_t)num_cu * (uint32_t)std::min<size_t>(16u, WAVE_LDS_MAX / h2.lds);
    if (2u * h2.waves >= 3u * c.waves) c = h2;
  }
  // invariant the workers rely on (tsw_worker.h): LDS g-scores always come with the staged bitmap
  if (c.gs_lds != 0u) c.stage_fb = 1u;
  return c;
}

}  // namespace tsw
