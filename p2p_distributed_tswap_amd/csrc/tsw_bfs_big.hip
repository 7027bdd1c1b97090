// tsw_bfs_big.hip — K1 v4: k_bfs_big, batched per-goal BFS distance tables for LARGE grids (up to
// the 2^20-cell limit, e.g. the 1024x1024 sortation floor of BASELINE configs[4]), ONE WORKGROUP
// per goal over 8x8 cell blocks.
//
// What it computes: the same table as every K1 kernel — dist[c] = BFS distance from the goal to
// cell c over the 4-connected graph of tswap.rs:44-77 (get_path's path length - 1,
// tswap.rs:288-390), 0xFFFF for blocked / unreachable cells.
//
// Why a workgroup per goal: k_bfs_blk keeps one goal per WAVE with the free-cell blocks, the
// visited blocks and its lists all in LDS. On 1024x1024 the visited bitmap alone is 131 KB (one
// bit per cell), so only one goal fits a CU, and its BFS front is ~1000 blocks wide: one wave would
// walk that list 16 chunks at a time for ~2000 levels. Here the eight waves of one workgroup share
// the goal's state and split each level's block list; one barrier separates levels.
//
// Layout (gfx950, 160 KiB LDS, 8 waves x 64 lanes):
//  * block (bx, by) at p = (by + 1) * Bp + bx, Bp = BW + 1 (zero guard block per block row, zero
//    guard block rows), bit r*8 + c = cell (8bx + c, 8by + r) — as k_bfs_blk (tsw_bfs_blk.hip).
//  * LDS: visited blocks V (nbp u64), two interleaved dedup-flag bitmaps, two block lists (u16).
//  * HBM/L2 (read-only, shared by every workgroup, L2-resident): free-cell blocks FR, the per-block
//    run-start numbering AB. Per-workgroup scratch (reused goal after goal): west-step blocks WL
//    (nbp u64, fire-and-forget workgroup-scope ORs, performed in L2), compact run-start anchors
//    (nrs u16), list overflow (2 x nbp u16).
//  * Level lvl processes exactly the blocks gaining cells at distance lvl:
//    new = expand(V & parity(lvl-1)) & FR & ~V; a neighbour's concurrent update adds only
//    parity-lvl bits, which this level never reads (the grid is bipartite), so V needs no locks.
//  * Decode (after the BFS): one thread per 32-cell row word rebuilds the u16 distances from the
//    row's run anchors and west-step bits (d(x) = d(x-1) +- 1 inside a free run) and writes them
//    with 16-B stores: the 2 B/cell table leaves the chip exactly once.
// Algorithmic bytes per goal: 2*W*H table write + ceil(W*H/8) bitmap read.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

namespace {

constexpr uint64_t BCOL0 = 0x0101010101010101ull;
constexpr uint64_t BCOL7 = 0x8080808080808080ull;
constexpr uint64_t BCB_EVEN = 0xAA55AA55AA55AA55ull;  // cells with (r + c) even
constexpr uint32_t BIG_THREADS = 512;
constexpr uint32_t BIG_RT_ROWS = 9;  // decode run table: 17 u16 rows = 9 dword rows per thread

__device__ __forceinline__ uint32_t big_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// u16 slot of decode run-table row j of thread t: rows j, j+1 of one thread share a dword, threads
// use distinct dwords, so a wave's access to one row j is bank-conflict-free.
__device__ __forceinline__ uint32_t rt_slot(uint32_t t, uint32_t j, uint32_t bd) {
  return 2u * ((j >> 1) * bd + t) + (j & 1u);
}

}  // namespace

__host__ __device__ __forceinline__ uint32_t big_bfs_klog(uint32_t nbp) {
  uint32_t kl = 5;
  while ((32u << kl) < nbp) ++kl;
  return kl;
}

// LDS bytes of one workgroup (must match the carve in k_bfs_big)
__host__ __device__ __forceinline__ size_t big_bfs_lds(uint32_t nbp, uint32_t cap) {
  const uint32_t nfk = 1u << big_bfs_klog(nbp);
  const size_t lists = (size_t)2u * cap * 2u;
  const size_t rt = (size_t)BIG_RT_ROWS * BIG_THREADS * 4u;  // reuses the flag + list area
  const size_t tail = (size_t)2u * nfk * 4u + lists;
  return (size_t)nbp * 8u + (tail > rt ? tail : rt);
}

__global__ void __launch_bounds__(512) k_bfs_big(BigBfsArgs A) {
  extern __shared__ __align__(16) uint64_t smb[];
  __shared__ uint32_t s_cnt[3], s_gi, s_bad;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, bd = blockDim.x;
  const uint32_t W = A.W, Bp = A.Bp, BW = A.BW, nbp = A.nbp, cap = A.cap, klog = A.klog;
  const uint32_t nfk = 1u << klog, kmask = nfk - 1u;
  uint64_t* V = smb;
  uint32_t* FL = reinterpret_cast<uint32_t*>(smb + nbp);  // 2 * nfk
  uint16_t* LS = reinterpret_cast<uint16_t*>(FL + 2u * nfk);  // 2 * cap
  uint16_t* RT = reinterpret_cast<uint16_t*>(FL);          // decode run table (after the BFS)
  const uint64_t* __restrict__ FR = A.frb;
  const uint32_t* __restrict__ AB = A.abase;
  uint16_t* anch = A.anch + (uint64_t)blockIdx.x * A.nrs;
  uint16_t* lovf = A.lovf + (uint64_t)blockIdx.x * 2u * nbp;
  uint64_t* WL = A.wlg + (uint64_t)blockIdx.x * nbp;
  const uint32_t idle_p = Bp + BW;  // guard block of block row 0: FR = 0, all neighbours in range

  for (;;) {
    if (tid == 0) s_gi = atomicAdd(A.work, 1u);
    __syncthreads();
    const uint32_t gi = s_gi;
    if (gi >= A.k) break;
    const uint32_t goal = A.goals[gi];
    const uint64_t slot = A.slots ? A.slots[gi] : gi;
    const uint32_t gy = goal / W, gx = goal - gy * W;
    const uint32_t gpar = (gx + gy) & 1u;
    for (uint32_t t = tid; t < nbp; t += bd) {
      V[t] = 0ull;
      WL[t] = 0ull;
    }
    for (uint32_t t = tid; t < 2u * nfk; t += bd) FL[t] = 0u;
    if (tid == 0) {
      s_cnt[0] = s_cnt[1] = s_cnt[2] = 0u;
      s_bad = 0u;
    }
    __syncthreads();

    // run starts of block p among cells nw (free cells whose west is blocked, or x % 32 == 0):
    // their level goes to the compact anchor slot AB[p] + rank inside the block
    auto anchors = [&](uint32_t p, uint64_t nw, uint64_t f0, uint64_t fw, uint32_t lvl) {
      const uint32_t bx = p - __umulhi(p, A.bp_magic) * Bp;
      const uint64_t wf = ((f0 << 1) & ~BCOL0) | ((bx & 3u) ? ((fw >> 7) & BCOL0) : 0ull);
      const uint64_t rs = f0 & ~wf;
      uint64_t rsn = nw & rs;
      if (rsn) {
        const uint32_t base = AB[p];
        while (rsn) {
          const uint32_t bb = (uint32_t)__builtin_ctzll(rsn);
          anch[base + (uint32_t)__popcll(rs & ((1ull << bb) - 1ull))] = (uint16_t)lvl;
          rsn &= rsn - 1ull;
        }
      }
    };
    // exact pushes of block p whose new cells (distance lvl) are nw: queue the blocks that gain a
    // cell at lvl + 1, deduplicated by test-and-set on flags Fn, appended to list Ln (overflow On)
    // through counter *cn. Wave-uniform call; lanes without work pass nw = 0.
    auto push = [&](uint32_t p, uint64_t nw, uint64_t vv, uint64_t f0, uint64_t fw, uint64_t fe, uint64_t fn,
                    uint64_t fs, uint64_t vw, uint64_t ve, uint64_t vn, uint64_t vs, uint32_t* Fn, uint16_t* Ln,
                    uint16_t* On, uint32_t* cn) {
      const uint64_t in = ((nw << 1) & ~BCOL0) | ((nw >> 1) & ~BCOL7) | (nw << 8) | (nw >> 8);
      bool w_self = (in & f0 & ~vv) != 0ull;
      bool w_w = (((nw & BCOL0) << 7) & fw & ~vw) != 0ull;
      bool w_e = (((nw & BCOL7) >> 7) & fe & ~ve) != 0ull;
      bool w_n = ((nw << 56) & fn & ~vn) != 0ull;
      bool w_s = ((nw >> 56) & fs & ~vs) != 0ull;
      const uint32_t tw = p - 1u, te = p + 1u, tn = p - Bp, ts = p + Bp;
      auto tas = [&](bool w, uint32_t t) -> bool {
        if (!w) return false;
        const uint32_t m = 1u << (t >> klog);
        return (atomicOr(&Fn[t & kmask], m) & m) == 0u;
      };
      w_self = tas(w_self, p);
      w_w = tas(w_w, tw);
      w_e = tas(w_e, te);
      w_n = tas(w_n, tn);
      w_s = tas(w_s, ts);
      // one counter update per wave for all five targets
      const uint64_t m0 = __ballot(w_self), m1 = __ballot(w_w), m2 = __ballot(w_e), m3 = __ballot(w_n),
                     m4 = __ballot(w_s);
      const uint32_t c0 = (uint32_t)__popcll(m0), c1 = (uint32_t)__popcll(m1), c2 = (uint32_t)__popcll(m2),
                     c3 = (uint32_t)__popcll(m3), c4 = (uint32_t)__popcll(m4);
      const uint32_t tot = c0 + c1 + c2 + c3 + c4;
      if (tot == 0u) return;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(cn, tot);
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      auto put = [&](bool c, uint64_t m, uint32_t off, uint32_t entry) {
        if (!c) return;
        const uint32_t pos = base + off + big_rank(m);
        if (pos < cap) Ln[pos] = (uint16_t)entry;
        else On[pos - cap] = (uint16_t)entry;
      };
      put(w_self, m0, 0u, p);
      put(w_w, m1, c0, tw);
      put(w_e, m2, c0 + c1, te);
      put(w_n, m3, c0 + c1 + c2, tn);
      put(w_s, m4, c0 + c1 + c2 + c3, ts);
    };

    // ---- level 0: the goal cell (wave 0); queues the blocks that gain cells at distance 1 ----
    if (tid < 64u) {
      const uint32_t gp = ((gy >> 3) + 1u) * Bp + (gx >> 3);
      const uint64_t gm = 1ull << (((gy & 7u) << 3) | (gx & 7u));
      const bool act = tid == 0u;
      const uint32_t p = act ? gp : idle_p;
      const uint64_t nw = act ? gm : 0ull;
      const uint64_t f0 = FR[p], fw = FR[p - 1u], fe = FR[p + 1u], fn = FR[p - Bp], fs = FR[p + Bp];
      if (act) {
        V[p] = gm;
        anchors(p, nw, f0, fw, 0u);
      }
      push(p, nw, nw, f0, fw, fe, fn, fs, 0ull, 0ull, 0ull, 0ull, FL, LS, lovf, &s_cnt[0]);
    }
    __syncthreads();

    // ---- levels 1, 2, ...: list (L-1)&1 -> list L&1; counters rotate over three slots ---------
    bool bad = false;
    uint32_t lvl = 1;
    for (;; ++lvl) {
      const uint32_t ncur = s_cnt[(lvl - 1u) % 3u];
      if (ncur == 0u) break;
      if (lvl >= 0xFFFFu) {
        if (tid == 0) atomicOr(A.err, ERR_DIST_OVERFLOW);
        if (tid == 0 && A.govf) A.govf[gi] = 1u;  // planned without a table (K3)
        break;
      }
      if (tid == 0) s_cnt[(lvl + 1u) % 3u] = 0u;  // the counter of the level after next
      const uint32_t cur = (lvl - 1u) & 1u, nxt = lvl & 1u;
      const uint16_t* Lc = LS + cur * cap;
      uint16_t* Ln = LS + nxt * cap;
      const uint16_t* Oc = lovf + cur * nbp;
      uint16_t* On = lovf + nxt * nbp;
      uint32_t* Fc = FL + cur * nfk;
      uint32_t* Fn = FL + nxt * nfk;
      uint32_t* cn = &s_cnt[lvl % 3u];
      const uint64_t pnew = ((gpar + lvl) & 1u) ? ~BCB_EVEN : BCB_EVEN;  // cells at distance lvl
      const uint64_t psrc = ~pnew;                                       // cells at distance lvl-1
      for (uint32_t b0 = 0; b0 < ncur; b0 += bd) {  // wave-uniform trip count
        const uint32_t i = b0 + tid;
        const bool act = i < ncur;
        const uint32_t p = !act ? idle_p : i < cap ? (uint32_t)Lc[i] : (uint32_t)Oc[i - cap];
        const uint64_t v0 = V[p], vw = V[p - 1u], ve = V[p + 1u], vn = V[p - Bp], vs = V[p + Bp];
        const uint64_t f0 = FR[p], fw = FR[p - 1u], fe = FR[p + 1u], fn = FR[p - Bp], fs = FR[p + Bp];
        const uint64_t a = v0 & psrc, aw = vw & psrc, ae = ve & psrc, an = vn & psrc, as = vs & psrc;
        const uint64_t ex = ((a << 1) & ~BCOL0) | ((a >> 1) & ~BCOL7) | ((aw >> 7) & BCOL0) | ((ae << 7) & BCOL7) |
                            (a << 8) | (a >> 8) | (an >> 56) | (as << 56);
        const uint64_t nw = ex & f0 & ~v0;  // 0 for idle lanes (FR of the guard block is 0)
        const uint64_t vv = v0 | nw;
        if (act) {
          V[p] = vv;  // owner-exclusive within the level (the list is deduplicated)
          const uint64_t wln = nw & (((v0 << 1) & ~BCOL0) | ((vw >> 7) & BCOL0));
          // fire-and-forget OR at workgroup scope (the scratch is this workgroup's; performed in
          // L2, no load on the level's critical path)
          if (wln) (void)__hip_atomic_fetch_or(WL + p, wln, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          bad |= nw == 0ull;  // a queued block must gain a cell
          anchors(p, nw, f0, fw, lvl);
        }
        push(p, nw, vv, f0, fw, fe, fn, fs, vw, ve, vn, vs, Fn, Ln, On, cn);
      }
      for (uint32_t t = tid; t < nfk; t += bd) Fc[t] = 0u;  // reused by the level after next
      __syncthreads();
    }
    if (bad) s_bad = 1u;
    __syncthreads();  // anchors / WL (global) complete before the decode reads them
    if (tid == 0 && s_bad) atomicOr(A.err, ERR_BFS_LIST);

    // ---- decode + write-out: one 32-cell row word per thread per iteration --------------------
    // d(b) = F(b) + C(run(b)): F(b) = 2*popc(WL & bits<=b) - (b+1) is the +-1 walk from bit 0,
    // C(j) = A(j) - F(s_j) for run j starting at bit s_j with anchor A(j) (mod 2^16).
    const uint8_t* V8 = reinterpret_cast<const uint8_t*>(V);
    const uint8_t* WL8 = reinterpret_cast<const uint8_t*>(WL);
    const uint8_t* FR8 = reinterpret_cast<const uint8_t*>(FR);
    uint16_t* D = A.dist + slot * A.dstride;
    const uint32_t Ww = (W + 31u) >> 5, nwords = A.H * Ww;
    for (uint32_t k = tid; k < nwords; k += bd) {
      const uint32_t y = k / Ww, cw = k - y * Ww, r = y & 7u;
      const uint32_t p0 = ((y >> 3) + 1u) * Bp + 4u * cw;
      uint32_t vis = 0u, wl = 0u, f0 = 0u;
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j)
        if (4u * cw + j < BW) {
          const uint32_t off = (p0 + j) * 8u + r;
          vis |= (uint32_t)V8[off] << (8u * j);
          wl |= (uint32_t)WL8[off] << (8u * j);
          f0 |= (uint32_t)FR8[off] << (8u * j);
        }
      uint32_t pk[16];
      if (vis != 0u) {
        const uint32_t rsw = f0 & ~(f0 << 1);
        uint32_t rs = rsw;
        for (uint32_t j = 1; rs != 0u; ++j) {
          const uint32_t sj = (uint32_t)__builtin_ctz(rs);
          rs &= rs - 1u;
          const uint32_t pb = p0 + (sj >> 3), cb = r * 8u + (sj & 7u);
          const uint64_t f = FR[pb];
          const uint64_t wf = ((f << 1) & ~BCOL0) | ((sj >> 3) ? ((FR[pb - 1u] >> 7) & BCOL0) : 0ull);
          const uint32_t Aj = anch[AB[pb] + (uint32_t)__popcll(f & ~wf & ((1ull << cb) - 1ull))];
          const uint32_t Fs = 2u * __popc(wl & (0xFFFFFFFFu >> (31u - sj))) - (sj + 1u);
          RT[rt_slot(tid, j, bd)] = (uint16_t)(Aj - Fs);  // own slots: program order suffices
        }
#pragma unroll
        for (int b = 0; b < 32; ++b) {
          const uint32_t m = 0xFFFFFFFFu >> (31 - b);
          const uint32_t C = RT[rt_slot(tid, (uint32_t)__popc(rsw & m), bd)];
          const uint32_t F = 2u * __popc(wl & m) - (uint32_t)(b + 1);
          const uint32_t v = ((vis >> b) & 1u) ? ((F + C) & 0xFFFFu) : 0xFFFFu;
          if (b & 1) pk[b >> 1] |= v << 16;
          else pk[b >> 1] = v;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) pk[j] = 0xFFFFFFFFu;
      }
      const uint32_t x0 = cw << 5;
      const uint32_t cnt = min(32u, W - x0);
      uint16_t* dst = D + (uint64_t)y * W + x0;
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
    __syncthreads();  // the next goal re-initialises the shared state
  }
}

bool bfs_big_fits(uint32_t nbp, int max_lds, uint32_t* cap_out) {
  if (nbp > 0xFFFFu || max_lds <= 0) return false;
  // largest list capacity (<= 8192) whose carve fits
  for (uint32_t cap = 8192; cap >= 256; cap >>= 1)
    if (big_bfs_lds(nbp, cap) <= (size_t)max_lds) {
      if (cap_out) *cap_out = cap;
      return true;
    }
  return false;
}

hipError_t launch_bfs_big(const BigBfsArgs& A0, int max_lds, int num_cu, hipStream_t s) {
  if (A0.k == 0) return hipSuccess;
  BigBfsArgs A = A0;
  A.klog = big_bfs_klog(A.nbp);
  A.bp_magic = (uint32_t)((0xFFFFFFFFull + A.Bp) / A.Bp);  // ceil(2^32 / Bp): exact p / Bp for p*Bp < 2^32
  const size_t lds = big_bfs_lds(A.nbp, A.cap);
  if (lds > (size_t)max_lds || A.nbp > 0xFFFFu) return hipErrorInvalidValue;
  const uint32_t per_cu = (uint32_t)std::max<size_t>(1u, (160u * 1024u) / lds);
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((uint32_t)num_cu * per_cu, A.k));
  if (grid > A.scratch_wgs) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)k_bfs_big, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bfs_big, dim3(grid), dim3(BIG_THREADS), lds, s, A);
  return hipGetLastError();
}

uint32_t bfs_big_workgroups(uint32_t nbp, uint32_t cap, int num_cu) {
  const size_t lds = big_bfs_lds(nbp, cap);
  return (uint32_t)num_cu * (uint32_t)std::max<size_t>(1u, (160u * 1024u) / lds);
}

}  // namespace tsw
