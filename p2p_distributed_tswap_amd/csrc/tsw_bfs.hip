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
//    level at which it was reached: a u16 in per-wave global scratch indexed by the padded
//    cell (~4.8k writes per goal on den520d, fire-and-forget, never waited for in the loop).
//  * Dedup flags are bit-interleaved (word t -> dword t & (K-1), bit t >> log2 K) so the
//    spatially clustered targets of one chunk hit distinct dwords / banks (the plain layout
//    serialised up to ~30 same-address LDS atomics per instruction).
//  * Decode: each lane rebuilds the 32 u16 distances of a word from (anchors, WL, V) and
//    writes them with 16-B stores (row-major u16 table, one pass, no read-back).
// Algorithmic bytes per goal: 2*W*H table write + ceil(W*H/8) bitmap read.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

namespace {

constexpr uint32_t EVEN_BITS = 0x55555555u;
constexpr uint32_t ODD_BITS = 0xAAAAAAAAu;

// LDS written by any lane of the wave is visible to every lane after this point. DS
// instructions of one wave execute in order; the wait + memory clobber keep the compiler
// from moving LDS accesses across. Global stores (anchors) are NOT waited for here.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ... and the wave's global stores (anchor scratch, list overflow) have completed; the
// matching loads use ld_nc (L1-bypassing) so they read L2.
__device__ __forceinline__ void full_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// global scratch written by this wave earlier: bypass the (non-coherent) vector L1
__device__ __forceinline__ uint32_t ld_nc16(const uint16_t* p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

// Overflow-capable list store, kept out of line: inlined, the compiler merges the LDS and
// the global store into one FLAT store, whose completion every later LDS read then waits for.
__device__ __attribute__((noinline)) void list_put_slow(uint16_t* Ln, uint16_t* On, uint32_t cap, uint32_t pos,
                                                       uint32_t entry) {
  if (pos < cap) Ln[pos] = (uint16_t)entry;
  else __builtin_nontemporal_store((uint16_t)entry, On + (pos - cap));
}

}  // namespace

// LDS words (u32 units) of one wave; must match the carve in k_bfs_wave. The list area holds
// at least 17 x 64 u16 (the decode's C table).
__host__ __device__ __forceinline__ uint32_t wave_bfs_words(uint32_t npw, uint32_t nfk, uint32_t cap) {
  const uint32_t npw4 = (npw + 3u) & ~3u;
  const uint32_t ls = cap < 544u ? 544u : cap;
  return 2u * npw4 + 2u * nfk + ((ls + 3u) & ~3u);
}

__global__ void __launch_bounds__(1024) k_bfs_wave(WaveBfsArgs A) {
  extern __shared__ __align__(16) uint32_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  const uint32_t W = A.W, Ww = A.Ww, Wp = A.Wp, npw = A.npw, cap = A.cap;
  const uint32_t nfk = 1u << A.klog, kmask = nfk - 1u, klog = A.klog;
  const uint32_t npw4 = (npw + 3u) & ~3u;
  uint32_t* FRs = smem;
  uint32_t* V;
  uint32_t* WL;
  uint32_t* FL;   // 2 * nfk interleaved flag dwords
  uint16_t* LS;   // 2 * cap list entries (>= 17 x 64 for the decode)
  {
    uint32_t* b = smem + npw4 + wv * wave_bfs_words(npw, nfk, cap);
    V = b;
    WL = b + npw4;
    FL = b + 2u * npw4;
    LS = reinterpret_cast<uint16_t*>(FL + 2u * nfk);
  }
  for (uint32_t t = tid; t < npw; t += blockDim.x) FRs[t] = A.frp[t];
  __syncthreads();  // the only workgroup barrier: waves run their goals independently

  const uint32_t gw = blockIdx.x * nwv + wv;
  uint16_t* anch = A.anch + (uint64_t)gw * npw * 32u;  // anchor of padded cell (p, b) at p*32+b
  uint16_t* lovf = A.lovf + (uint64_t)gw * 2u * npw;
  const uint32_t idle_p = Wp + Ww;  // a guard word: FR = 0, every neighbour in bounds
  const float invWw = 1.0f / (float)Ww;
  uint64_t t_bfs = 0, t_dec = 0, n_lvl = 0, n_chunk = 0;

  for (;;) {
    uint32_t gi = 0;
    if (lane == 0) gi = atomicAdd(A.work, 1u);
    gi = __builtin_amdgcn_readfirstlane(gi);
    if (gi >= A.k) break;
    const uint64_t t0 = clk();
    const uint32_t goal = A.goals[gi];
    const uint64_t slot = A.slots ? A.slots[gi] : gi;
    const uint32_t gy = goal / W, gx = goal - gy * W;
    const uint32_t gpar = (gx + gy) & 1u;

    {
      const uint4 z = make_uint4(0u, 0u, 0u, 0u);
      for (uint32_t t = lane; t < npw4 / 2u; t += 64u) reinterpret_cast<uint4*>(V)[t] = z;  // V and WL
      for (uint32_t t = lane; t < 2u * nfk; t += 64u) FL[t] = 0u;
    }
    lds_sync();

    // ---- level 0: the goal cell, and the words that gain cells at distance 1 ----------
    uint32_t ncur = 0;
    {
      const uint32_t gp = (gy + 1u) * Wp + (gx >> 5), gb = gx & 31u, gbit = 1u << gb;
      if (lane == 0) {
        V[gp] = gbit;
        const uint32_t f0 = FRs[gp];
        if ((f0 & ~(f0 << 1)) & gbit) anch[gp * 32u + gb] = 0;
      }
      lds_sync();
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
        if (pos < cap) LS[pos] = (uint16_t)(t | (tpar << 15));
        else __builtin_nontemporal_store((uint16_t)(t | (tpar << 15)), lovf + (pos - cap));
        atomicOr(&FL[t & kmask], 1u << (t >> klog));
      }
      ncur = (uint32_t)__popcll(m);
      if (ncur > cap) full_sync();
      else lds_sync();
    }

    // ---- levels 1, 2, ...: process the words that gain cells at distance lvl ----------
    uint32_t cur = 0;
    uint32_t lvl = 1;
    while (ncur != 0u) {
      if (lvl >= 0xFFFFu) {
        if (lane == 0) atomicOr(A.err, ERR_DIST_OVERFLOW);
        if (lane == 0 && A.govf) A.govf[gi] = 1u;  // planned without a table (K3)
        break;
      }
      const uint32_t nxt = cur ^ 1u;
      const uint16_t* Lc = LS + cur * cap;
      uint16_t* Ln = LS + nxt * cap;
      const uint16_t* Oc = lovf + cur * npw;
      uint16_t* On = lovf + nxt * npw;
      uint32_t* Fc = FL + cur * nfk;
      uint32_t* Fn = FL + nxt * nfk;
      const uint32_t qlvl = (gpar + lvl) & 1u;
      uint32_t nn = 0;
      // list entry of chunk b0 (prefetched one chunk ahead). LDS-only fast path when the list
      // fits (wave-uniform): a global load here would make the compiler wait for every
      // outstanding global store of the wave (the anchors) before the ds_read.
      auto list_get = [&](uint32_t i) -> uint32_t {
        if (i >= ncur) return idle_p;
        if (ncur <= cap) return Lc[i];
        return i < cap ? (uint32_t)Lc[i] : ld_nc16(Oc + (i - cap));
      };
      uint32_t e_next = list_get(lane);
      for (uint32_t b0 = 0; b0 < ncur; b0 += 64u) {
        const uint32_t e = e_next;
        e_next = list_get(b0 + 64u + lane);
        const uint32_t p = e & 0x7FFFu, rpar = e >> 15;
        const uint32_t v0 = V[p], vw = V[p - 1u], ve = V[p + 1u], vn = V[p - Wp], vs = V[p + Wp];
        const uint32_t wl0 = WL[p];
        const uint32_t f0 = FRs[p], fw = FRs[p - 1u], fe = FRs[p + 1u], fn = FRs[p - Wp], fs = FRs[p + Wp];
        const uint32_t pnew = ((qlvl ^ rpar) & 1u) ? ODD_BITS : EVEN_BITS;  // cells at distance lvl
        const uint32_t psrc = ~pnew;                                           // cells at lvl-1 in row r
        const uint32_t a = v0 & psrc;
        const uint32_t hz = (a << 1) | (a >> 1) | ((vw & psrc) >> 31) | ((ve & psrc) << 31);
        const uint32_t nw = (hz | ((vn | vs) & pnew)) & f0 & ~v0;  // 0 for idle lanes (f0 = 0)
        const uint32_t vv = v0 | nw;
        // owner-exclusive within the level: plain stores (idle lanes rewrite the zero guard)
        V[p] = vv;
        WL[p] = wl0 | (nw & ((v0 << 1) | (vw >> 31)));
        uint32_t rsn = nw & f0 & ~(f0 << 1);  // run starts reached now: anchors
        while (rsn) {
          const uint32_t bb = __builtin_ctz(rsn);
          anch[p * 32u + bb] = (uint16_t)lvl;
          rsn &= rsn - 1u;
        }
        if (nw == 0u && e != idle_p) atomicOr(A.err, ERR_BFS_LIST);  // entries must gain a cell
        // exact pushes: a neighbour word gains a cell at lvl+1
        const uint32_t tw = p - 1u, te = p + 1u, tn = p - Wp, ts = p + Wp;
        bool w_self = (((nw << 1) | (nw >> 1)) & f0 & ~vv) != 0u;
        bool w_w = (nw & 1u) && ((fw & ~vw) >> 31);
        bool w_e = (nw >> 31) && ((fe & ~ve) & 1u);
        bool w_n = (nw & fn & ~vn) != 0u;
        bool w_s = (nw & fs & ~vs) != 0u;
        // dedup: test-and-set on the next level's (interleaved) flags, five atomics back to
        // back (value 0 = no-op for targets not wanted): one LDS round trip
        const uint32_t b_self = w_self ? 1u << (p >> klog) : 0u, b_w = w_w ? 1u << (tw >> klog) : 0u,
                       b_e = w_e ? 1u << (te >> klog) : 0u, b_n = w_n ? 1u << (tn >> klog) : 0u,
                       b_s = w_s ? 1u << (ts >> klog) : 0u;
        const uint32_t o_self = atomicOr(&Fn[p & kmask], b_self);
        const uint32_t o_w = atomicOr(&Fn[tw & kmask], b_w);
        const uint32_t o_e = atomicOr(&Fn[te & kmask], b_e);
        const uint32_t o_n = atomicOr(&Fn[tn & kmask], b_n);
        const uint32_t o_s = atomicOr(&Fn[ts & kmask], b_s);
        w_self = w_self && !(o_self & b_self);
        w_w = w_w && !(o_w & b_w);
        w_e = w_e && !(o_e & b_e);
        w_n = w_n && !(o_n & b_n);
        w_s = w_s && !(o_s & b_s);
        // append (ballot + mbcnt; nn stays wave-uniform). LDS-only unless this chunk could
        // cross the capacity (wave-uniform test).
        const bool lds_only = nn + 5u * 64u <= cap;
        auto append = [&](bool c, uint32_t entry) {
          const uint64_t m = __ballot(c);
          if (c) {
            const uint32_t pos = nn + lane_rank(m);
            if (lds_only) Ln[pos] = (uint16_t)entry;
            else list_put_slow(Ln, On, cap, pos, entry);
          }
          nn += (uint32_t)__popcll(m);
        };
        append(w_self, p | (rpar << 15));
        append(w_w, tw | (rpar << 15));
        append(w_e, te | (rpar << 15));
        append(w_n, tn | ((rpar ^ 1u) << 15));
        append(w_s, ts | ((rpar ^ 1u) << 15));
        ++n_chunk;
      }
      // the flags of this level's list are reused two levels later
      for (uint32_t t = lane; t < nfk; t += 64u) Fc[t] = 0u;
      if (nn > cap) full_sync();  // overflow entries went to global memory
      else lds_sync();
      cur = nxt;
      ncur = nn;
      ++lvl;
    }
    full_sync();  // anchors (global) complete before the decode reads them
    const uint64_t t1 = clk();

    // ---- decode + write-out: 32 cells per lane per iteration, row-major words ----------
    // d(b) = F(b) + C(run(b)): F(b) = 2*popc(WL & bits<=b) - (b+1) is the +-1 walk from bit 0,
    // C(j) = A(j) - F(s_j) for run j starting at bit s_j with anchor A(j) (mod 2^16 suffices:
    // the table is u16). Bit b belongs to run popc(rsw & bits<=b) - 1 (<= 16 runs per word);
    // C goes to row popc(...) of a per-lane column of an LDS table (the dead list area,
    // [row][lane] u16, 17 rows: conflict-free) and every bit reads its run's C with one
    // ds_read_u16 — branch-free for any run count. Anchors of the next word are loaded one
    // iteration ahead (L2 latency off the chain).
    uint16_t* CT = LS + lane;  // CT[row * 64]
    uint16_t* D = A.dist + slot * A.dstride;
    const uint32_t nwords = A.H * Ww;
    auto word_at = [&](uint32_t k, uint32_t& r, uint32_t& c) {
      r = (uint32_t)((float)k * invWw);
      while (r * Ww > k) --r;
      while ((r + 1u) * Ww <= k) ++r;
      c = k - r * Ww;
    };
    auto load_anch = [&](uint32_t p, uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3) {
      const uint32_t f0 = FRs[p];
      uint32_t rs = f0 & ~(f0 << 1);
      const uint16_t* ap = anch + p * 32u;
      a0 = a1 = a2 = a3 = 0u;
      if (rs) { a0 = ld_nc16(ap + __builtin_ctz(rs)); rs &= rs - 1u; }
      if (rs) { a1 = ld_nc16(ap + __builtin_ctz(rs)); rs &= rs - 1u; }
      if (rs) { a2 = ld_nc16(ap + __builtin_ctz(rs)); rs &= rs - 1u; }
      if (rs) { a3 = ld_nc16(ap + __builtin_ctz(rs)); }
    };
    uint32_t r = 0, c = 0, p = 0, a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (lane < nwords) {
      word_at(lane, r, c);
      p = (r + 1u) * Wp + c;
      load_anch(p, a0, a1, a2, a3);
    }
    for (uint32_t k = lane; k < nwords; k += 64u) {
      const uint32_t cr = r, cc = c, cp = p, A0 = a0, A1 = a1, A2 = a2, A3 = a3;
      if (k + 64u < nwords) {
        word_at(k + 64u, r, c);
        p = (r + 1u) * Wp + c;
        load_anch(p, a0, a1, a2, a3);
      }
      const uint32_t vis = V[cp], wl = WL[cp], f0 = FRs[cp];
      const uint32_t rsw = f0 & ~(f0 << 1);
      uint32_t pk[16];
      if (vis != 0u) {
        // C table rows 1..nr (row j = run j-1, starting at the j-th set bit of rsw); row 0
        // only serves bits before the first run start, which are blocked
        const uint16_t* ap = anch + cp * 32u;
        uint32_t rs = rsw;
        for (uint32_t j = 1; rs != 0u; ++j) {
          const uint32_t sj = __builtin_ctz(rs);
          rs &= rs - 1u;
          const uint32_t Aj = j == 1u ? A0 : j == 2u ? A1 : j == 3u ? A2 : j == 4u ? A3 : ld_nc16(ap + sj);
          const uint32_t Fs = 2u * __popc(wl & (0xFFFFFFFFu >> (31u - sj))) - (sj + 1u);
          CT[j * 64u] = (uint16_t)(Aj - Fs);
        }
#pragma unroll
        for (int b = 0; b < 32; ++b) {
          const uint32_t m = 0xFFFFFFFFu >> (31 - b);
          const uint32_t C = CT[__popc(rsw & m) * 64u];
          const uint32_t F = 2u * __popc(wl & m) - (uint32_t)(b + 1);
          const uint32_t v = ((vis >> b) & 1u) ? ((F + C) & 0xFFFFu) : 0xFFFFu;
          if (b & 1) pk[b >> 1] |= v << 16;
          else pk[b >> 1] = v;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) pk[j] = 0xFFFFFFFFu;
      }
      const uint32_t x0 = cc << 5;
      const uint32_t cnt = min(32u, W - x0);
      uint16_t* dst = D + (uint64_t)cr * W + x0;
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
    lds_sync();  // the next goal re-initialises this wave's LDS
    if (A.prof) {
      const uint64_t t2 = clk();
      t_bfs += t1 - t0;
      t_dec += t2 - t1;
      n_lvl += lvl;
    }
  }
  if (A.prof && lane == 0) {
    atomicAdd((unsigned long long*)&A.prof[0], (unsigned long long)t_bfs);
    atomicAdd((unsigned long long*)&A.prof[1], (unsigned long long)t_dec);
    atomicAdd((unsigned long long*)&A.prof[2], (unsigned long long)n_lvl);
    atomicAdd((unsigned long long*)&A.prof[3], (unsigned long long)n_chunk);
  }
}

// flag dwords per buffer: a power of two >= 64 with 32 * K >= npw
uint32_t bfs_wave_klog(uint32_t npw) {
  uint32_t kl = 6;
  while ((32u << kl) < npw) ++kl;
  return kl;
}

uint32_t bfs_wave_waves_per_block(uint32_t npw, uint32_t cap, int max_lds) {
  const size_t per_wave = (size_t)wave_bfs_words(npw, 1u << bfs_wave_klog(npw), cap) * 4u;
  const size_t shared = (size_t)((npw + 3u) & ~3u) * 4u;
  if (max_lds <= 0 || shared + per_wave > (size_t)max_lds) return 0;
  return (uint32_t)std::min<size_t>(16u, ((size_t)max_lds - shared) / per_wave);
}

hipError_t launch_bfs_wave(const WaveBfsArgs& A0, int max_lds, int num_cu, hipStream_t s) {
  if (A0.k == 0) return hipSuccess;
  WaveBfsArgs A = A0;
  A.klog = bfs_wave_klog(A.npw);
  const size_t per_wave = (size_t)wave_bfs_words(A.npw, 1u << A.klog, A.cap) * 4u;
  const size_t shared = (size_t)((A.npw + 3u) & ~3u) * 4u;
  const uint32_t nwv = std::min<uint32_t>(A.max_waves, bfs_wave_waves_per_block(A.npw, A.cap, max_lds));
  if (nwv == 0 || A.npw > 0x8000u) return hipErrorInvalidValue;
  const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((uint32_t)num_cu, (A.k + nwv - 1u) / nwv));
  if ((uint64_t)grid * nwv > A.scratch_waves) return hipErrorInvalidValue;
  const size_t lds = shared + nwv * per_wave;
  hipError_t e = hipFuncSetAttribute((const void*)k_bfs_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bfs_wave, dim3(grid), dim3(nwv * 64u), lds, s, A);
  return hipGetLastError();
}

}  // namespace tsw
