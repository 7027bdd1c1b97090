// tsw_bfs_mg.hip — K1 v5: k_bfs_mg, GOAL-BIT-PARALLEL batched BFS distance tables.
//
// What it computes: for every goal g, dist[c] = BFS distance from g to every cell c of the
// 4-connected grid (tswap.rs:44-77 graph), 0xFFFF for blocked/unreachable cells — the table
// every other K1 kernel writes; get_path's path length - 1 (tswap.rs:288-390).
//
// Why bit-parallel over goals: one goal's BFS front is thin (~110 cells per level
// on den520d spread over ~30 8x8 blocks), so a wave per goal spends ~270 instructions per level on
// ~3.7 new cells per block and is bound by that level's dependent chain (k_bfs_blk, 6.6 % of HBM
// peak). Here one WORKGROUP runs a GROUP of up to 16 goals at once: every grid cell holds a u16
// visited mask (bit k = goal k) in LDS, and one level processes the union of the 16 fronts. Goals
// are grouped on the host by (checkerboard parity, Morton order), so a group's goals are spatial
// neighbours and their fronts nearly coincide: on den520d a 16-goal group touches ~82 blocks per
// level where 16 separate BFS touch ~16 x 30 — the per-level instruction stream is shared ~6x.
//
// Level L (all goals of a group share the cell parity p of their goal cells, so the new cells of
// level L are exactly the cells of parity p + L; the grid is bipartite):
//    new[c] = (V[w] | V[e] | V[n] | V[s]) & ~V[c]       for free cells c of parity p + L
// A neighbour's bits are goals that reached it at level <= L-1 with its parity; a goal that
// reached it at L-3 or earlier reached c by L-2 already (|d(c) - d(n)| = 1), so ~V[c] removes it.
// Reads (parity p+L-1) and writes (parity p+L) never touch the same cell in a level: no races.
//  * Candidate blocks (8x8, padded numbering of k_bfs_blk: p = (by+1)*Bp + bx, zero guard blocks):
//    a block is processed at level L+1 iff it or a neighbour gained a cell on the shared edge at
//    L (exact marks from the wave ballot of the new masks, LDS atomic OR into a 3-deep ring of
//    block bitmaps); wave 0 turns the level's bitmap into a list, the 16 waves take two blocks
//    per task (lanes 0-31 / 32-63: the 32 cells of the level's parity of each block).
//  * Distances are not stored during the BFS (the 16 tables are 2 MB per group): a cell's west
//    step bits WL (bit k: d_k(c) = d_k(west) + 1, i.e. new & V[west]) go to per-workgroup global
//    scratch with fire-and-forget workgroup-scope atomic ORs, and each run start (free cell whose
//    west is blocked or whose x is a multiple of 32 — k_bfs_blk's compact numbering `abase`)
//    records its level per goal bit (per-workgroup scratch, [run start][16] u16).
//  * Decode (same launch, after the group's BFS): a lane per cell of a 32-cell row word, the
//    word's 16 goal bitmaps are transposed by 32 ballots (V from LDS, WL from global), and
//    d_k(x) = A_k(rs) + 2 * popc(WL_k in (rs, x]) - (x - rs) with rs the run start of x.
// LDS (den520d 256x257): V 133.6 KB + free blocks 9.2 KB + run numbering 4.6 KB + lists 2.8 KB,
// one workgroup (16 waves) per CU. Grids whose V does not fit, or with more than 65535 free cells
// (u16 levels), use k_bfs_blk / k_bfs_big.
// Algorithmic bytes per goal: 2*W*H table write + ceil(W*H/8) bitmap read.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

#ifdef TSW_DIAG
// The kernel is compiled into the diagnostic build only: it is a measured null result
// (5.5 ms vs k_bfs_blk's 2.7 ms on den520d's 10k goals) that the production path never selects.

namespace {

constexpr uint32_t MG_G = 16;  // goals per group (bits of the u16 visited mask)
constexpr uint64_t COL0 = 0x0101010101010101ull;

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

__device__ __forceinline__ void wl_or(uint32_t* p, uint32_t v) {
  (void)__hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// run-start mask of padded block p (free cells whose west is blocked, or with x % 32 == 0):
// the numbering k_bfs_blk's `abase` counts, in block bit order
__device__ __forceinline__ uint64_t rs_mask(const uint64_t* FR, uint32_t p, uint32_t bx) {
  const uint64_t f0 = FR[p];
  const uint64_t wf = ((f0 << 1) & ~COL0) | ((bx & 3u) ? ((FR[p - 1u] >> 7) & COL0) : 0ull);
  return f0 & ~wf;
}

}  // namespace

// LDS bytes of k_bfs_mg for a grid (0 if the layout's indices overflow)
__host__ __device__ __forceinline__ uint32_t mg_vbytes(uint32_t W, uint32_t H) {
  return (((W + 2u) * (H + 2u) * 2u) + 15u) & ~15u;
}
__host__ __device__ __forceinline__ uint32_t mg_nwc(uint32_t nbp) { return ((nbp + 31u) / 32u + 3u) & ~3u; }

size_t bfs_mg_lds_bytes(uint32_t W, uint32_t H, uint32_t nbp) {
  return (size_t)mg_vbytes(W, H) + (size_t)nbp * 8u + (size_t)nbp * 4u + 3u * mg_nwc(nbp) * 4u +
         (((size_t)nbp * 2u + 15u) & ~(size_t)15u);
}

__global__ void __launch_bounds__(1024) k_bfs_mg(MgBfsArgs A) {
  extern __shared__ __align__(16) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6, bd = blockDim.x;
  const uint32_t W = A.W, H = A.H, Wp = W + 2u, Bp = A.Bp, nbp = A.nbp, nwc = mg_nwc(nbp);
  uint16_t* V = reinterpret_cast<uint16_t*>(smem);
  uint64_t* FR = reinterpret_cast<uint64_t*>(smem + mg_vbytes(W, H));
  uint32_t* AB = reinterpret_cast<uint32_t*>(FR + nbp);
  uint32_t* CB = AB + nbp;  // 3 x nwc block bitmaps (level L reads CB[L % 3])
  uint16_t* LIST = reinterpret_cast<uint16_t*>(CB + 3u * nwc);
  __shared__ uint32_t s_gi, s_n, s_ng, s_gpar, s_gcell[MG_G], s_gslot[MG_G];

  for (uint32_t t = tid; t < nbp; t += bd) {
    FR[t] = A.frb[t];
    AB[t] = A.abase[t];
  }
  uint32_t* WL = A.wl + (uint64_t)blockIdx.x * A.wlw;
  uint16_t* AN = A.anch + (uint64_t)blockIdx.x * A.nrs * MG_G;
  const uint32_t vwords = mg_vbytes(W, H) / 4u;
  // lane roles in a BFS task: half hf (block A / B of the task), cell i of the block's 32 cells of one
  // parity (row r); mark lanes 0-9: direction dir (self, N, S, W, E) of block A (0-4) / B (5-9)
  const uint32_t wvu = __builtin_amdgcn_readfirstlane(wv);
  const uint32_t hf = lane >> 5, i = lane & 31u, r = i >> 2;
  const uint32_t dir = lane < 5u ? lane : (lane < 10u ? lane - 5u : 0u);
  const uint32_t toff = dir == 0u ? 0u : dir == 1u ? 0u - Bp : dir == 2u ? Bp : dir == 3u ? 0xFFFFFFFFu : 1u;
  const uint32_t Ww = (W + 31u) >> 5, nwords = H * Ww;
  uint64_t t_bfs = 0, t_dec = 0, n_lvl = 0, n_blk = 0, t_list = 0, t_task = 0;

  for (;;) {
    __syncthreads();  // the previous group's decode is done with V before it is cleared
    if (tid == 0) s_gi = atomicAdd(A.work, 1u);
    __syncthreads();
    const uint32_t gi = s_gi;
    if (gi >= A.ngroups) break;
    const uint64_t t0 = clk();
    const uint32_t g0 = A.grp[gi], ng = min(A.grp[gi + 1u] - g0, MG_G);
    // ---- init: V = 0, bitmaps = 0, WL scratch = 0 ------------------------------------------
    uint32_t* V32 = reinterpret_cast<uint32_t*>(V);
    for (uint32_t t = tid; t < vwords; t += bd) V32[t] = 0u;
    for (uint32_t t = tid; t < 3u * nwc; t += bd) CB[t] = 0u;
    for (uint32_t t = tid; t < A.wlw; t += bd) WL[t] = 0u;
    if (tid < ng) {
      s_gcell[tid] = A.goals[g0 + tid];
      s_gslot[tid] = A.slots ? A.slots[g0 + tid] : g0 + tid;
    }
    if (tid == 0) {
      s_ng = ng;
      const uint32_t c0 = A.goals[g0], y0 = c0 / W;
      s_gpar = (c0 - y0 * W + y0) & 1u;
    }
    // the WL zero stores reach L2 before any wave's atomics: wait for them, then the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // ---- level 0: the goal cells; candidates of level 1 = their blocks and the 4 neighbours ---
    if (tid < ng) {
      const uint32_t c = s_gcell[tid], y = c / W, x = c - y * W;
      V[(y + 1u) * Wp + x + 1u] = (uint16_t)(1u << tid);
      const uint32_t bx = x >> 3, p = ((y >> 3) + 1u) * Bp + bx, bit = ((y & 7u) << 3) | (x & 7u);
      const uint64_t rsm = rs_mask(FR, p, bx);
      if ((rsm >> bit) & 1ull) AN[(AB[p] + (uint32_t)__popcll(rsm & ((1ull << bit) - 1ull))) * MG_G + tid] = 0;
      uint32_t* CBn = CB + 1u * nwc;
      const uint32_t tg[5] = {p, p - 1u, p + 1u, p - Bp, p + Bp};
#pragma unroll
      for (int j = 0; j < 5; ++j) atomicOr(&CBn[tg[j] >> 5], 1u << (tg[j] & 31u));
    }
    __syncthreads();
    const uint32_t gpar = s_gpar;
    uint32_t L = 1;
    for (;; ++L) {
      const uint32_t* CBc = CB + (L % 3u) * nwc;
      uint32_t* CBn = CB + ((L + 1u) % 3u) * nwc;
      uint32_t* CBo = CB + ((L + 2u) % 3u) * nwc;  // read at level L-1: free to clear now
      const uint64_t tl0 = A.prof ? clk() : 0ull;
      if (wv == 0) {
        uint32_t n = 0;
        for (uint32_t base = 0; base < nwc; base += 64u) {
          const uint32_t d = base + lane;
          uint32_t bits = d < nwc ? CBc[d] : 0u;
          const uint32_t cnt = (uint32_t)__popc(bits);
          uint32_t incl = cnt;
#pragma unroll
          for (uint32_t off = 1; off < 64u; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off);
            if (lane >= off) incl += t;
          }
          uint32_t pos = n + incl - cnt;
          while (bits) {
            LIST[pos++] = (uint16_t)(d * 32u + (uint32_t)__builtin_ctz(bits));
            bits &= bits - 1u;
          }
          n += (uint32_t)__shfl(incl, 63);
        }
        if (lane == 0) s_n = n;
      } else {
        for (uint32_t t = tid - 64u; t < nwc; t += bd - 64u) CBo[t] = 0u;
      }
      __syncthreads();
      const uint32_t n = __builtin_amdgcn_readfirstlane(s_n);
      const uint64_t tl1 = A.prof ? clk() : 0ull;
      t_list += tl1 - tl0;
      n_blk += n;
      if (n == 0u) break;
      if (L >= 0xFFFFu) {  // cannot happen with <= 65535 free cells (checked on the host)
        if (tid == 0) atomicOr(A.err, ERR_DIST_OVERFLOW);
        break;
      }
      // per-lane constants of this level's parity: the lane's cell inside its block (row r, column
      // col of parity P), its V offset, and its mark target (lanes 0-4: block A's self, N, S, W, E;
      // lanes 5-9: block B's)
      const uint32_t P = (gpar + L) & 1u;
      const uint32_t col = 2u * (i & 3u) + ((r + P) & 1u);
      const uint32_t bitc = r * 8u + col, loff = r * Wp + col;
      const uint32_t mW = P ? 0x10101010u : 0x01010101u, mE = P ? 0x08080808u : 0x80808080u;
      const uint32_t mmask = dir == 0u ? 0xFFFFFFFFu : dir == 1u ? 0xFu : dir == 2u ? 0xF0000000u : dir == 3u ? mW : mE;
      for (uint32_t t = wvu; 2u * t < n; t += nwv) {
        const uint32_t e = 2u * t + hf;
        const uint32_t p = e < n ? (uint32_t)LIST[e] : 0u;  // block 0 is a guard (FR = 0)
        const uint32_t by = __umulhi(p, A.bp_magic), bx = p - by * Bp;  // p / Bp, p % Bp
        const uint64_t fr = FR[p];
        const bool fre = (fr >> bitc) & 1ull;  // guard blocks and off-grid cells are not free
        // V index of the lane's cell; other lanes use the guard word V[Wp] (west of cell (0, 0), always
        // 0: reads see no goal, the store below rewrites 0) — the store is then branch-free
        const uint32_t a = fre ? (8u * by - 7u) * Wp + 8u * bx + 1u + loff : Wp;
        const uint32_t vn = V[a - Wp], vw = V[a - 1u], vc = V[a], ve = V[a + 1u], vs = V[a + Wp];
        const uint32_t nw = fre ? ((vn | vw | ve | vs) & ~vc) & 0xFFFFu : 0u;  // the guard word stays 0
        V[a] = (uint16_t)(vc | nw);
        const uint32_t wl = nw & vw;
        if (wl) {
          const uint32_t cell = (8u * by - 8u + r) * W + 8u * bx + col;
          wl_or(WL + (cell >> 1), wl << ((cell & 1u) * 16u));
        }
        if (nw) {  // a run start records the level of every new goal bit
          const uint64_t rsm = rs_mask(FR, p, bx);
          if ((rsm >> bitc) & 1ull) {
            uint16_t* an = AN + (AB[p] + (uint32_t)__popcll(rsm & ((1ull << bitc) - 1ull))) * MG_G;
            uint32_t b = nw;
            while (b) {
              an[__builtin_ctz(b)] = (uint16_t)L;
              b &= b - 1u;
            }
          }
        }
        // exact marks for level L+1: the block itself, and a neighbour across an edge with new cells
        const uint64_t m = __ballot(nw != 0u);
        const uint32_t pA = __builtin_amdgcn_readlane(p, 0), pB = __builtin_amdgcn_readlane(p, 32);
        const uint32_t mh = lane < 5u ? (uint32_t)m : (uint32_t)(m >> 32);
        const bool want = lane < 10u && (mh & mmask) != 0u && (lane < 5u || 2u * t + 1u < n);
        if (want) {
          const uint32_t tg = (lane < 5u ? pA : pB) + toff;
          atomicOr(&CBn[tg >> 5], 1u << (tg & 31u));
        }
      }
      if (A.prof) t_task += clk() - tl1;
      __syncthreads();
    }
    n_lvl += L;
    // every wave's WL atomics and run-start stores have reached L2 before anyone decodes
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint64_t t1 = clk();
    // ---- decode: 16 tables of this group -------------------------------------------------
    // this CU's L1 may hold WL / anchor lines of the previous group (the atomics and the run-start
    // stores went to L2): invalidate before reading them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t gng = __builtin_amdgcn_readfirstlane(s_ng);
    uint32_t gslot[MG_G];
#pragma unroll
    for (uint32_t k = 0; k < MG_G; ++k) gslot[k] = __builtin_amdgcn_readfirstlane(s_gslot[k < gng ? k : 0u]);
    // one task = two consecutive 32-cell row words (lanes 0-31 / 32-63); the next task's loads are
    // issued before the current one is decoded (global latency off the per-task chain)
    struct Dw {
      uint32_t v, w, cell, rs;
      bool valid;
      uint4 a0, a1;
    };
    const uint32_t l = lane & 31u;
    auto fetch = [&](uint32_t t, Dw& o) {
      const uint32_t q = 2u * t + (lane >> 5);
      const uint32_t y = q / Ww, x = 32u * (q - y * Ww) + l;
      o.valid = q < nwords && x < W;
      o.cell = y * W + x;
      o.v = 0u;
      o.w = 0u;
      o.rs = 0u;
      o.a0 = o.a1 = make_uint4(0, 0, 0, 0);
      bool fre = false;
      uint32_t p = 0, bit = 0;
      if (o.valid) {
        o.v = V[(y + 1u) * Wp + x + 1u];
        p = ((y >> 3) + 1u) * Bp + (x >> 3);
        bit = ((y & 7u) << 3) | (x & 7u);
        fre = (FR[p] >> bit) & 1ull;
      }
      // run start of this lane's cell inside its 32-cell word (x % 32 == 0 or west blocked)
      const uint64_t fm = __ballot(fre);
      const uint32_t fh = (uint32_t)(fm >> (lane & 32u));
      const uint32_t rsw = fh & ~(fh << 1);
      const uint32_t below = rsw & (l == 31u ? 0xFFFFFFFFu : (2u << l) - 1u);
      o.rs = below ? 31u - (uint32_t)__builtin_clz(below) : 0u;
      if (o.v) {
        o.w = WL[o.cell >> 1];
        const uint32_t xr = x - l + o.rs, bxr = xr >> 3, pr = ((y >> 3) + 1u) * Bp + bxr;
        const uint32_t bitr = ((y & 7u) << 3) | (xr & 7u);
        const uint64_t rsm = rs_mask(FR, pr, bxr);
        const uint32_t ai = AB[pr] + (uint32_t)__popcll(rsm & ((1ull << bitr) - 1ull));
        const uint4* ap = reinterpret_cast<const uint4*>(AN + (uint64_t)ai * MG_G);
        o.a0 = ap[0];
        o.a1 = ap[1];
      }
    };
    const uint32_t ntask = (nwords + 1u) / 2u;
    Dw cur, nxt;
    if (wvu < ntask) fetch(wvu, cur);
    for (uint32_t t = wvu; t < ntask; t += nwv) {
      if (t + nwv < ntask) fetch(t + nwv, nxt);
      const uint32_t w = (cur.w >> ((cur.cell & 1u) * 16u)) & 0xFFFFu;
      const uint32_t upto = l == 31u ? 0xFFFFFFFFu : (2u << l) - 1u;
      const uint32_t mrun = upto & ~((2u << cur.rs) - 1u);  // bits (rs, l]
      const uint32_t an[8] = {cur.a0.x, cur.a0.y, cur.a0.z, cur.a0.w, cur.a1.x, cur.a1.y, cur.a1.z, cur.a1.w};
      const int32_t base = -(int32_t)(l - cur.rs);
#pragma unroll
      for (uint32_t k = 0; k < MG_G; ++k) {  // unrolled: an[] and gslot[] stay in registers
        if (k < gng) {
          const uint64_t wk = __ballot((w >> k) & 1u);
          const uint32_t pc = (uint32_t)__popc((uint32_t)(wk >> (lane & 32u)) & mrun);
          const uint32_t ak = (an[k >> 1] >> ((k & 1u) * 16u)) & 0xFFFFu;
          const uint32_t d = (uint32_t)((int32_t)(ak + 2u * pc) + base) & 0xFFFFu;
          if (cur.valid) A.dist[(uint64_t)gslot[k] * A.dstride + cur.cell] = (uint16_t)(((cur.v >> k) & 1u) ? d : 0xFFFFu);
        }
      }
      cur = nxt;
    }
    if (A.prof) {
      t_bfs += t1 - t0;
      t_dec += clk() - t1;
    }
  }
  if (A.prof && tid == 0) {
    atomicAdd((unsigned long long*)&A.prof[0], (unsigned long long)t_bfs);
    atomicAdd((unsigned long long*)&A.prof[1], (unsigned long long)t_dec);
    atomicAdd((unsigned long long*)&A.prof[2], (unsigned long long)n_lvl);
    atomicAdd((unsigned long long*)&A.prof[3], (unsigned long long)n_blk);
  }
  if (A.prof && lane == 0) {  // per wave: list build + barrier, own task loop (summed over waves)
    atomicAdd((unsigned long long*)&A.prof[4], (unsigned long long)t_list);
    atomicAdd((unsigned long long*)&A.prof[5], (unsigned long long)t_task);
  }
}

hipError_t launch_bfs_mg(const MgBfsArgs& A, int max_lds, int num_cu, hipStream_t s) {
  if (A.ngroups == 0) return hipSuccess;
  const size_t lds = bfs_mg_lds_bytes(A.W, A.H, A.nbp);
  if (max_lds <= 0 || lds > (size_t)max_lds) return hipErrorInvalidValue;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((uint32_t)num_cu, A.ngroups));
  if (grid > A.scratch_wgs) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)k_bfs_mg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bfs_mg, dim3(grid), dim3(1024), lds, s, A);
  return hipGetLastError();
}

#else   // production build: no k_bfs_mg (TSW_BFS_KERNEL is a diagnostic knob)

size_t bfs_mg_lds_bytes(uint32_t, uint32_t, uint32_t) { return ~(size_t)0; }

hipError_t launch_bfs_mg(const MgBfsArgs&, int, int, hipStream_t) { return hipErrorInvalidValue; }

#endif  // TSW_DIAG

}  // namespace tsw
