// tsw_bfs.hip — K1 v2: k_bfs_wave, batched per-goal BFS distance tables with ONE
// WAVEFRONT PER GOAL and no workgroup barrier on the level loop.
//
// What it computes: for goal g, dist[c] = BFS distance from g to every cell c of the
// 4-connected grid (tswap.rs:44-77 graph), 0xFFFF for blocked/unreachable cells — the same
// table k_bfs (tsw_kernels.hip) writes; get_path's path length - 1 (tswap.rs:288-390).
//
// Why a new kernel: on a den520d-like 256x257 cave a BFS runs ~380 levels but its
// frontier touches only ~100 of the 2056 row words per level, and a u16 table does not
// fit LDS beside the bitmaps (131 KB), so k_bfs scattered 2-byte stores to HBM and swept
// the whole Manhattan band every level behind a 1024-thread barrier (1.7 % of HBM peak).
//
// Design (gfx950, 64-lane waves, 160 KiB LDS):
//  * LDS per workgroup: the padded free-cell bitmap FR (shared by its waves) and, per wave,
//    the visited bitmap V, the west-step plane WL, two dedup flag bitmaps and two
//    active-word lists. Padding = one zero guard word per row + a zero guard row above and
//    below, so neighbour words are plain index arithmetic (p-1, p+1, p-Wp, p+Wp).
//  * Level lvl processes exactly the words that gain cells at distance lvl (the list).
//    new = expand(V & parity(lvl-1)) & FR & ~V. Parity masks make the level loop
//    race-free inside the wave: every cell at distance lvl has grid parity == parity of
//    (goal + lvl) (the 4-grid is bipartite), so bits written during the level are never
//    read as sources in the same level.
//  * Pushes are EXACT: a neighbour word is queued for lvl+1 only if one of this word's new
//    cells has a free unvisited neighbour in it (that neighbour's distance is then lvl+1),
//    so every list entry gains >= 1 cell; dedup = LDS test-and-set (ds_or_rtn) on a flag
//    bitmap, appends = ballot + mbcnt prefix (wave-synchronous, no atomics on a counter).
//  * Distances are never stored per cell during the BFS. Adjacent cells on a 4-grid differ
//    by exactly 1, so along a row run d(x) = d(x-1) +/- 1; WL[c] = 1 iff c's west
//    neighbour was reached first (d(west) = d(c) - 1), recorded at visit time from V.
//    One anchor per run start (cell whose west is blocked, or bit 0 of a word) holds the
//    level at which it was reached (a u32 in per-wave global scratch, ~4.8k per goal).
//  * Decode: each lane rebuilds the 32 u16 distances of a word from (anchor, WL, V) and
//    writes them with 16-B stores (row-major u16 table, one pass, no read-back).
// Algorithmic bytes per goal: 2*W*H table write + ceil(W*H/8) bitmap read.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

namespace {

constexpr uint32_t EVEN_BITS = 0x55555555u;
constexpr uint32_t ODD_BITS = 0xAAAAAAAAu;

// Everything the wave wrote to LDS (and, for the anchor scratch, issued to global memory)
// is visible to every lane of the wave after this point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// global scratch written by this wave earlier: bypass the (non-coherent) vector L1
__device__ __forceinline__ uint32_t ld_nc(const uint32_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ uint16_t ld_nc16(const uint16_t* p) { return __builtin_nontemporal_load(p); }

struct WaveLds {
  uint32_t* V;
  uint32_t* WL;
  uint32_t* FL;   // 2 * nfw flag words
  uint16_t* LS;   // 2 * cap list entries
};

}  // namespace

// per-wave LDS words (u32 units); must match the carve in k_bfs_wave
__host__ __device__ __forceinline__ uint32_t wave_bfs_words(uint32_t npw, uint32_t nfw, uint32_t cap) {
  const uint32_t npw4 = (npw + 3u) & ~3u;
  return 2u * npw4 + ((2u * nfw + 3u) & ~3u) + ((cap + 3u) & ~3u);
}

__global__ void __launch_bounds__(1024) k_bfs_wave(WaveBfsArgs A) {
  extern __shared__ __align__(16) uint32_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  const uint32_t W = A.W, Ww = A.Ww, Wp = A.Wp, npw = A.npw, nfw = A.nfw, cap = A.cap;
  const uint32_t npw4 = (npw + 3u) & ~3u;
  uint32_t* FRs = smem;
  WaveLds S;
  {
    uint32_t* b = smem + npw4 + wv * wave_bfs_words(npw, nfw, cap);
    S.V = b;
    S.WL = b + npw4;
    S.FL = b + 2u * npw4;
    S.LS = reinterpret_cast<uint16_t*>(S.FL + ((2u * nfw + 3u) & ~3u));
  }
  for (uint32_t t = tid; t < npw; t += blockDim.x) FRs[t] = A.frp[t];
  __syncthreads();  // the only workgroup barrier: waves run their goals independently

  const uint32_t gw = blockIdx.x * nwv + wv;
  uint32_t* anch = A.anch + (uint64_t)gw * A.nanch;
  uint16_t* lovf = A.lovf + (uint64_t)gw * 2u * npw;
  const uint32_t idle_p = Wp + Ww;  // a guard word: FR = 0, every neighbour in bounds
  const float invWw = 1.0f / (float)Ww;

  for (;;) {
    uint32_t gi = 0;
    if (lane == 0) gi = atomicAdd(A.work, 1u);
    gi = __builtin_amdgcn_readfirstlane(gi);
    if (gi >= A.k) break;
    const uint32_t goal = A.goals[gi];
    const uint64_t slot = A.slots ? A.slots[gi] : gi;
    const uint32_t gy = goal / W, gx = goal - gy * W;
    const uint32_t gpar = (gx + gy) & 1u;

    for (uint32_t t = lane; t < npw; t += 64u) {
      S.V[t] = 0u;
      S.WL[t] = 0u;
    }
    for (uint32_t t = lane; t < 2u * nfw; t += 64u) S.FL[t] = 0u;
    wave_sync();

    // ---- level 0: the goal cell, and the words that gain cells at distance 1 ----------
    uint32_t ncur = 0;
    {
      const uint32_t gp = (gy + 1u) * Wp + (gx >> 5), gbit = 1u << (gx & 31u);
      if (lane == 0) {
        S.V[gp] = gbit;
        const uint32_t f0 = FRs[gp], rsw = f0 & ~(f0 << 1);
        if (rsw & gbit) anch[A.rb[gp] + __popc(rsw & (gbit - 1u))] = 0u;
      }
      wave_sync();
      // lanes 0..4 = self, west, east, north, south
      const uint32_t rpar = gy & 1u;
      uint32_t t = gp, tpar = rpar;
      bool want = false;
      if (lane == 0) {
        want = (((gbit << 1) | (gbit >> 1)) & FRs[gp] & ~gbit) != 0u;
      } else if (lane == 1) {
        t = gp - 1u;
        want = (gbit & 1u) && (FRs[gp - 1u] >> 31);
      } else if (lane == 2) {
        t = gp + 1u;
        want = (gbit >> 31) && (FRs[gp + 1u] & 1u);
      } else if (lane == 3) {
        t = gp - Wp;
        tpar ^= 1u;
        want = (gbit & FRs[gp - Wp]) != 0u;
      } else if (lane == 4) {
        t = gp + Wp;
        tpar ^= 1u;
        want = (gbit & FRs[gp + Wp]) != 0u;
      }
      const uint64_t m = __ballot(want);
      if (want) {
        const uint32_t pos = lane_rank(m);
        if (pos < cap) S.LS[pos] = (uint16_t)(t | (tpar << 15));
        else lovf[pos - cap] = (uint16_t)(t | (tpar << 15));
        atomicOr(&S.FL[t >> 5], 1u << (t & 31u));
      }
      ncur = (uint32_t)__popcll(m);
      wave_sync();
    }

    // ---- levels 1, 2, ...: process the words that gain cells at distance lvl ----------
    uint32_t cur = 0;
    uint32_t lvl = 1;
    while (ncur != 0u) {
      if (lvl >= 0xFFFFu) {
        if (lane == 0) atomicOr(A.err, ERR_DIST_OVERFLOW);
        break;
      }
      const uint32_t nxt = cur ^ 1u;
      const uint16_t* Lc = S.LS + cur * cap;
      uint16_t* Ln = S.LS + nxt * cap;
      const uint16_t* Oc = lovf + cur * npw;
      uint16_t* On = lovf + nxt * npw;
      uint32_t* Fc = S.FL + cur * nfw;
      uint32_t* Fn = S.FL + nxt * nfw;
      const uint32_t qlvl = (gpar + lvl) & 1u;
      uint32_t nn = 0;
      for (uint32_t b0 = 0; b0 < ncur; b0 += 64u) {
        const uint32_t i = b0 + lane;
        const bool act = i < ncur;
        uint32_t e = idle_p;
        if (act) e = i < cap ? (uint32_t)Lc[i] : (uint32_t)ld_nc16(Oc + (i - cap));
        const uint32_t p = e & 0x7FFFu, rpar = e >> 15;
        const uint32_t v0 = S.V[p], vw = S.V[p - 1u], ve = S.V[p + 1u], vn = S.V[p - Wp], vs = S.V[p + Wp];
        const uint32_t f0 = FRs[p], fw = FRs[p - 1u], fe = FRs[p + 1u], fn = FRs[p - Wp], fs = FRs[p + Wp];
        const uint32_t pnew = ((qlvl ^ rpar) & 1u) ? ODD_BITS : EVEN_BITS;  // cells at distance lvl
        const uint32_t psrc = ~pnew;                                           // cells at lvl-1 in row r
        const uint32_t a = v0 & psrc;
        const uint32_t hz = (a << 1) | (a >> 1) | ((vw & psrc) >> 31) | ((ve & psrc) << 31);
        const uint32_t nw = (hz | ((vn | vs) & pnew)) & f0 & ~v0;
        bool w_self = false, w_w = false, w_e = false, w_n = false, w_s = false;
        if (nw != 0u) {
          const uint32_t vv = v0 | nw;
          S.V[p] = vv;
          const uint32_t wl = nw & ((v0 << 1) | (vw >> 31));
          if (wl) atomicOr(&S.WL[p], wl);
          const uint32_t rsw = f0 & ~(f0 << 1);
          uint32_t rsn = nw & rsw;
          if (rsn) {
            const uint32_t base = A.rb[p];
            do {
              const uint32_t bb = __builtin_ctz(rsn);
              anch[base + __popc(rsw & ((1u << bb) - 1u))] = lvl;
              rsn &= rsn - 1u;
            } while (rsn);
          }
          // exact pushes: a neighbour word gains a cell at lvl+1
          w_self = (((nw << 1) | (nw >> 1)) & f0 & ~vv) != 0u;
          w_w = (nw & 1u) && ((fw & ~vw) >> 31);
          w_e = (nw >> 31) && ((fe & ~ve) & 1u);
          w_n = (nw & fn & ~vn) != 0u;
          w_s = (nw & fs & ~vs) != 0u;
        } else if (act) {
          atomicOr(A.err, ERR_BFS_LIST);  // every list entry must gain a cell
        }
        // dedup (test-and-set on the next level's flags)
        const uint32_t tw = p - 1u, te = p + 1u, tn = p - Wp, ts = p + Wp;
        if (w_self) w_self = !(atomicOr(&Fn[p >> 5], 1u << (p & 31u)) & (1u << (p & 31u)));
        if (w_w) w_w = !(atomicOr(&Fn[tw >> 5], 1u << (tw & 31u)) & (1u << (tw & 31u)));
        if (w_e) w_e = !(atomicOr(&Fn[te >> 5], 1u << (te & 31u)) & (1u << (te & 31u)));
        if (w_n) w_n = !(atomicOr(&Fn[tn >> 5], 1u << (tn & 31u)) & (1u << (tn & 31u)));
        if (w_s) w_s = !(atomicOr(&Fn[ts >> 5], 1u << (ts & 31u)) & (1u << (ts & 31u)));
        // append (ballot + mbcnt; nn stays wave-uniform)
        auto append = [&](bool c, uint32_t entry) {
          const uint64_t m = __ballot(c);
          if (c) {
            const uint32_t pos = nn + lane_rank(m);
            if (pos < cap) Ln[pos] = (uint16_t)entry;
            else On[pos - cap] = (uint16_t)entry;
          }
          nn += (uint32_t)__popcll(m);
        };
        append(w_self, p | (rpar << 15));
        append(w_w, tw | (rpar << 15));
        append(w_e, te | (rpar << 15));
        append(w_n, tn | ((rpar ^ 1u) << 15));
        append(w_s, ts | ((rpar ^ 1u) << 15));
      }
      // the flags of this level's list are reused two levels later
      for (uint32_t t = lane; t < nfw; t += 64u) Fc[t] = 0u;
      wave_sync();
      cur = nxt;
      ncur = nn;
      ++lvl;
    }
    wave_sync();

    // ---- decode + write-out: 32 cells per lane per iteration, row-major words ----------
    uint16_t* D = A.dist + slot * A.dstride;
    const uint32_t nwords = A.H * Ww;
    for (uint32_t k = lane; k < nwords; k += 64u) {
      uint32_t r = (uint32_t)((float)k * invWw);
      while (r * Ww > k) --r;
      while ((r + 1u) * Ww <= k) ++r;
      const uint32_t c = k - r * Ww;
      const uint32_t p = (r + 1u) * Wp + c;
      const uint32_t vis = S.V[p], wl = S.WL[p], f0 = FRs[p];
      uint32_t pk[16];
      if (vis == 0u) {
#pragma unroll
        for (int j = 0; j < 16; ++j) pk[j] = 0xFFFFFFFFu;
      } else {
        const uint32_t rsw = f0 & ~(f0 << 1);
        const uint32_t* ap = anch + A.rb[p];
        const uint32_t nr = __popc(rsw);
        uint32_t a0 = ld_nc(ap), a1 = 0, a2 = 0, a3 = 0;
        if (nr > 1u) a1 = ld_nc(ap + 1);
        if (nr > 2u) a2 = ld_nc(ap + 2);
        if (nr > 3u) a3 = ld_nc(ap + 3);
        uint32_t d = 0, j = 0;
#pragma unroll
        for (int b = 0; b < 32; ++b) {
          const uint32_t bit = 1u << b;
          if (rsw & bit) {
            d = j == 0 ? a0 : j == 1 ? a1 : j == 2 ? a2 : j == 3 ? a3 : ld_nc(ap + j);
            ++j;
          } else {
            d = (wl & bit) ? d + 1u : d - 1u;
          }
          const uint32_t v = (vis & bit) ? (d & 0xFFFFu) : 0xFFFFu;
          if (b & 1) pk[b >> 1] |= v << 16;
          else pk[b >> 1] = v;
        }
      }
      const uint32_t x0 = c << 5;
      const uint32_t cnt = min(32u, W - x0);
      uint16_t* dst = D + (uint64_t)r * W + x0;
      if (A.vec16 && cnt == 32u) {
        uint4* q = reinterpret_cast<uint4*>(dst);
        q[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        q[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
        q[2] = make_uint4(pk[8], pk[9], pk[10], pk[11]);
        q[3] = make_uint4(pk[12], pk[13], pk[14], pk[15]);
      } else {
#pragma unroll
        for (uint32_t b = 0; b < 32u; ++b)
          if (b < cnt) dst[b] = (uint16_t)(pk[b >> 1] >> ((b & 1u) * 16u));
      }
    }
    wave_sync();  // the next goal re-initialises this wave's LDS
  }
}

uint32_t bfs_wave_waves_per_block(uint32_t npw, uint32_t nfw, uint32_t cap, int max_lds) {
  const size_t per_wave = (size_t)wave_bfs_words(npw, nfw, cap) * 4u;
  const size_t shared = (size_t)((npw + 3u) & ~3u) * 4u;
  if (max_lds <= 0 || shared + per_wave > (size_t)max_lds) return 0;
  return (uint32_t)std::min<size_t>(16u, ((size_t)max_lds - shared) / per_wave);
}

hipError_t launch_bfs_wave(const WaveBfsArgs& A, int max_lds, int num_cu, hipStream_t s) {
  if (A.k == 0) return hipSuccess;
  const size_t per_wave = (size_t)wave_bfs_words(A.npw, A.nfw, A.cap) * 4u;
  const size_t shared = (size_t)((A.npw + 3u) & ~3u) * 4u;
  uint32_t nwv = std::min<uint32_t>(A.max_waves, bfs_wave_waves_per_block(A.npw, A.nfw, A.cap, max_lds));
  if (nwv == 0 || A.npw > 0x8000u) return hipErrorInvalidValue;
  const uint32_t grid = std::max<uint32_t>(
      1u, std::min<uint32_t>((uint32_t)num_cu, (A.k + nwv - 1u) / nwv));
  if ((uint64_t)grid * nwv > A.scratch_waves) return hipErrorInvalidValue;
  const size_t lds = shared + nwv * per_wave;
  hipError_t e = hipFuncSetAttribute((const void*)k_bfs_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bfs_wave, dim3(grid), dim3(nwv * 64u), lds, s, A);
  return hipGetLastError();
}

size_t bfs_wave_lds_one(uint32_t npw, uint32_t nfw, uint32_t cap) {
  return (size_t)(((npw + 3u) & ~3u) + wave_bfs_words(npw, nfw, cap)) * 4u;
}

}  // namespace tsw
