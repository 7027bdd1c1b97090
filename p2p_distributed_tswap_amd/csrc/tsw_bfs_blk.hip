// tsw_bfs_blk.hip — K1 v3: k_bfs_blk, batched per-goal BFS distance tables over 8x8 CELL
// BLOCKS, one wavefront per goal.
//
// What it computes: for goal g, dist[c] = BFS distance from g to every cell c of the
// 4-connected grid (tswap.rs:44-77 graph), 0xFFFF for blocked/unreachable cells — the same
// table k_bfs / k_bfs_wave write; get_path's path length - 1 (tswap.rs:288-390).
//
// Why blocks: k_bfs_wave works on 32x1 row words. A BFS frontier is a Manhattan ring, i.e.
// diagonal, so a row word gains about one cell per level and stays on the active list for
// ~32 levels; on den520d that is ~18 activations per word. An 8x8 block (one u64 per
// bitmap) is crossed by a diagonal front in ~16 levels and holds 64 cells, so activations
// per cell drop ~4x while the per-activation bit logic stays a handful of 64-bit ops.
//
// Layout (gfx950, 64-lane waves, 160 KiB LDS):
//  * block (bx, by) of the W x H grid sits at p = (by + 1) * Bp + bx, Bp = BW + 1: a zero
//    guard block ends every block row and a zero guard row lies above and below, so the
//    four neighbour blocks are p-1, p+1, p-Bp, p+Bp. Bit (r*8 + c) of a block word is cell
//    (8bx + c, 8by + r). Block origins are even, so the grid's checkerboard parity is a
//    fixed mask (CB_EVEN) inside every block.
//  * LDS: the free-cell blocks FR (shared by the workgroup's waves); per wave the visited
//    blocks V, two interleaved dedup flag bitmaps and two active-block lists. Goals in
//    flight per CU are bounded by LDS and the level loop is issue-bound, so by default the
//    west-step blocks WL (bit set = the west neighbour was reached one level earlier; written
//    once per activation, read only by the decode) live in per-wave global scratch, updated
//    with fire-and-forget 64-bit workgroup-scope atomic ORs. Measured cost (den520d, 10k goals,
//    PMC): the scratch of 384 waves per XCD outgrows the XCD's L2 and its lines are written
//    back ~18x per goal — 1.64 GB of WRITE_SIZE per launch on top of 1.31 GB of tables.
//    k_bfs_blk<true> (TSW_BFS_WLS=1) keeps WL in LDS instead (plain owner-exclusive RMW):
//    traffic 1.03x the algorithmic bytes and 15 % fewer cycles per goal, but 6 instead of 12
//    goals in flight per CU — 3.21 vs 2.71 ms per launch, so the default stays global.
//  * Level lvl processes exactly the blocks that gain cells at distance lvl:
//    new = expand(V & parity(lvl-1)) & FR & ~V (race-free inside the wave: the 4-grid is
//    bipartite, so bits written during a level are never sources in the same level).
//    Pushes are exact (a neighbour block is queued only if one of its free unvisited cells
//    touches a new cell), deduplicated with an LDS test-and-set, appended with ballot+mbcnt.
//  * Distances are not stored per cell during the BFS: along a row run d(x) = d(x-1) +- 1,
//    recorded by WL, plus one anchor (u16 level) per run start — a free cell whose west is
//    blocked or whose x is a multiple of 32. Anchors are stored COMPACTLY (per-wave global
//    scratch of nrs u16, run starts numbered in block order: AB[p] + rank inside the block), so
//    a goal dirties ~2*nrs bytes of cache lines instead of one line per anchor.
//  * Decode: one lane per 32-cell row word gathers its 4 blocks' row bytes and rebuilds the
//    u16 distances (run index table in LDS, bank-conflict-free), 16-B stores, row-major.
// Algorithmic bytes per goal: 2*W*H table write + ceil(W*H/8) bitmap read.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

namespace {

constexpr uint64_t COL0 = 0x0101010101010101ull;
constexpr uint64_t COL7 = 0x8080808080808080ull;
constexpr uint64_t CB_EVEN = 0xAA55AA55AA55AA55ull;  // cells with (r + c) even (row 0 = low byte)
constexpr uint32_t CT_U16 = 1152;                     // decode run table: 18 rows x 64 lanes u16

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void full_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t ld_nc16(const uint16_t* p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }

// WL scratch belongs to one wave: a WORKGROUP-scope no-return OR is performed in this XCD's L2.
// (Plain atomicOr is agent scope, which on a multi-XCD part bypasses the non-coherent L2 and runs
// memory-side: every activation became HBM-side atomic traffic, ~1.5x the table bytes per goal.)
__device__ __forceinline__ void wl_or(unsigned long long* p, unsigned long long v) {
  (void)__hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wl_or32(unsigned int* p, unsigned int v) {
  (void)__hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __attribute__((noinline)) void blk_list_put_slow(uint16_t* Ln, uint16_t* On, uint32_t cap, uint32_t pos,
                                                           uint32_t entry) {
  if (pos < cap) Ln[pos] = (uint16_t)entry;
  else __builtin_nontemporal_store((uint16_t)entry, On + (pos - cap));
}

// u16 slot of run-table row j for this lane: lane l's entries live in bank (l & 31), two rows
// per dword, so the 32 lanes of a group never share a bank whatever rows they read.
__device__ __forceinline__ uint32_t ct_slot(uint32_t lane, uint32_t j) {
  return 2u * ((lane & 31u) + 32u * ((j >> 1) + 9u * (lane >> 5))) + (j & 1u);
}

}  // namespace

// LDS dwords of one wave; must match the carve in k_bfs_blk: V (nbp rounded to even u64), flags,
// then the list / run-table / staging region LS, 16-B aligned (every part is a multiple of 4 dwords).
__host__ __device__ __forceinline__ uint32_t blk_bfs_words(uint32_t nbp, uint32_t nfk, uint32_t cap, bool wls) {
  const uint32_t ls = 2u * cap < CT_U16 ? CT_U16 : 2u * cap;  // u16 entries: two lists, run table, staging
  return (wls ? 4u : 2u) * ((nbp + 1u) & ~1u) + 2u * nfk + ((ls + 7u) >> 3) * 4u;
}
// u64 words of the workgroup's shared part (FR u64 + AB u32), rounded to 16 B
__host__ __device__ __forceinline__ uint32_t blk_shared_u64(uint32_t nbp) {
  return (nbp + (nbp + 1u) / 2u + 1u) & ~1u;
}

// WLS: the west-step blocks WL live in the wave's LDS (after V) instead of global scratch — no
// memory-side atomics, at the cost of ~nbp*8 more LDS bytes per goal in flight.
// PAIR (TSW_BFS_PAIR=1, A/B variant): each 32-lane half of a wave runs its own goal (two goals per
// wave, in lockstep: both halves start together, run levels until both BFS are done, then decode
// together), so one level's instruction stream advances two goals at the same LDS per goal; the
// global scratch (WL, anchors, list overflow) is per goal slot. Measured slower on den520d (3.66 vs
// 2.68 ms per 10k goals): per-half state moves to VGPRs and the larger of two fronts needs more
// chunk passes, lengthening the dependent level chain that bounds the loop.
template <bool WLS, bool PAIR>
__global__ void __launch_bounds__(1024) k_bfs_blk(BlkBfsArgs A) {
  extern __shared__ __align__(16) uint64_t smem64[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, nwv = blockDim.x >> 6;
  // goal slot of this lane: the half (PAIR) or the whole wave; NL lanes per goal, gl = lane in it
  constexpr uint32_t NL = PAIR ? 32u : 64u;
  const uint32_t hf = PAIR ? (lane >> 5) : 0u, gl = PAIR ? (lane & 31u) : lane;
  const uint64_t hmask = PAIR ? (hf ? 0xFFFFFFFF00000000ull : 0x00000000FFFFFFFFull) : ~0ull;
  const uint32_t gs = PAIR ? 2u * wv + hf : wv;  // goal slot in the workgroup
  const uint32_t W = A.W, Bp = A.Bp, nbp = A.nbp, cap = A.cap, BW = A.BW;
  const uint32_t nfk = 1u << A.klog, kmask = nfk - 1u, klog = A.klog;
  uint64_t* FRs = smem64;
  uint32_t* AB = reinterpret_cast<uint32_t*>(smem64 + nbp);  // [nbp] first run-start index of block p
  uint64_t* V;
  uint64_t* WLl = nullptr;  // WLS: the LDS west-step blocks
  uint32_t* FL;  // 2 * nfk interleaved flag dwords: block t -> dword t & kmask, bit t >> klog
  uint16_t* LS;  // 2 * cap list entries / decode run table
  uint16_t* CT;  // decode run table (PAIR: the wave's first goal slot's LS; ct_slot separates the halves)
  {
    uint32_t* b0 = reinterpret_cast<uint32_t*>(smem64 + blk_shared_u64(nbp));
    uint32_t* b = b0 + gs * blk_bfs_words(nbp, nfk, cap, WLS);
    uint32_t* bw = b0 + (PAIR ? 2u * wv : wv) * blk_bfs_words(nbp, nfk, cap, WLS);
    CT = reinterpret_cast<uint16_t*>(bw + (WLS ? 4u : 2u) * ((nbp + 1u) & ~1u) + 2u * nfk);
    V = reinterpret_cast<uint64_t*>(b);
    if constexpr (WLS) {
      WLl = V + ((nbp + 1u) & ~1u);
      b += 2u * ((nbp + 1u) & ~1u);
    }
    FL = b + 2u * ((nbp + 1u) & ~1u);
    LS = reinterpret_cast<uint16_t*>(FL + 2u * nfk);
  }
  for (uint32_t t = tid; t < nbp; t += blockDim.x) {
    FRs[t] = A.frb[t];
    AB[t] = A.abase[t];
  }
  __syncthreads();  // the only workgroup barrier: waves run their goals independently

  const uint32_t gw = PAIR ? 2u * (blockIdx.x * nwv + wv) + hf : blockIdx.x * nwv + wv;  // scratch slot
  uint16_t* anch = A.anch + (uint64_t)gw * A.nrs;  // compact anchors (run-start index)
  uint16_t* lovf = A.lovf + (uint64_t)gw * 2u * nbp;
  unsigned long long* WL = WLS ? reinterpret_cast<unsigned long long*>(WLl) : A.wlg + (uint64_t)gw * nbp;
  const uint32_t idle_p = Bp + BW;  // guard block of block row 0: FR = 0, all neighbours in range
  uint64_t t_bfs = 0, t_dec = 0, n_lvl = 0, n_chunk = 0;

  for (;;) {
    uint32_t gi = 0;
    if (lane == 0) gi = atomicAdd(A.work, PAIR ? 2u : 1u);
    gi = __builtin_amdgcn_readfirstlane(gi);
    if (gi >= A.k) break;
    gi += hf;                     // PAIR: the upper half takes the next goal
    const bool live = gi < A.k;   // PAIR: the upper half of the last pair may have none
    const uint64_t t0 = clk();
    const uint32_t goal = live ? A.goals[gi] : A.goals[gi - 1u];
    const uint64_t slot = !live ? 0ull : A.slots ? A.slots[gi] : gi;
    const uint32_t gy = goal / W, gx = goal - gy * W;
    const uint32_t gpar = (gx + gy) & 1u;

    for (uint32_t t = gl; t < nbp; t += NL) {
      V[t] = 0ull;
      WL[t] = 0ull;
    }
    for (uint32_t t = gl; t < 2u * nfk; t += NL) FL[t] = 0u;
    // the WL zeroing stores complete before this goal's atomics are issued
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();

    uint32_t nn = 0;
    bool bad = false;
    // exact pushes of block p whose new cells (distance lvl) are nw: queue the blocks that gain
    // a cell at lvl + 1 into list Ln (flags Fn). Wave-uniform call; inactive lanes pass nw = 0.
    auto push = [&](uint32_t p, uint64_t nw, uint64_t vv, uint64_t f0, uint64_t fw, uint64_t fe, uint64_t fn,
                    uint64_t fs, uint64_t vw, uint64_t ve, uint64_t vn, uint64_t vs, uint32_t* Fn, uint16_t* Ln,
                    uint16_t* On) {
      const uint64_t in = ((nw << 1) & ~COL0) | ((nw >> 1) & ~COL7) | (nw << 8) | (nw >> 8);
      bool w_self = (in & f0 & ~vv) != 0ull;
      bool w_w = (((nw & COL0) << 7) & fw & ~vw) != 0ull;
      bool w_e = (((nw & COL7) >> 7) & fe & ~ve) != 0ull;
      bool w_n = ((nw << 56) & fn & ~vn) != 0ull;
      bool w_s = ((nw >> 56) & fs & ~vs) != 0ull;
      const uint32_t tw = p - 1u, te = p + 1u, tn = p - Bp, ts = p + Bp;
      // dedup: test-and-set on the next level's interleaved flags. All five atomics issue back
      // to back and are waited for once; a lane that does not want a target ORs 0 into its own
      // dword (a no-op that conflicts with nobody).
      auto tas = [&](bool w, uint32_t t) -> uint32_t {
        const uint32_t m = w ? 1u << (t >> klog) : 0u;
        return atomicOr(&Fn[w ? (t & kmask) : lane], m) & m;
      };
      const uint32_t o_self = tas(w_self, p), o_w = tas(w_w, tw), o_e = tas(w_e, te), o_n = tas(w_n, tn),
                     o_s = tas(w_s, ts);
      w_self = w_self && !o_self;
      w_w = w_w && !o_w;
      w_e = w_e && !o_e;
      w_n = w_n && !o_n;
      w_s = w_s && !o_s;
      const bool lds_only = nn + 5u * NL <= cap;
      auto append = [&](bool c, uint32_t entry) {
        const uint64_t m = __ballot(c) & hmask;
        if (c) {
          const uint32_t pos = nn + lane_rank(m);
          if (lds_only) Ln[pos] = (uint16_t)entry;
          else blk_list_put_slow(Ln, On, cap, pos, entry);
        }
        nn += (uint32_t)__popcll(m);
      };
      append(w_self, p);
      append(w_w, tw);
      append(w_e, te);
      append(w_n, tn);
      append(w_s, ts);
    };
    // run starts of block p among cells nw: free cells whose west is blocked, or with x % 32 == 0
    auto anchors = [&](uint32_t p, uint64_t nw, uint64_t f0, uint64_t fw, uint32_t lvl) {
      const uint32_t bx = p - __umulhi(p, A.bp_magic) * Bp;
      const uint64_t wf = ((f0 << 1) & ~COL0) | ((bx & 3u) ? ((fw >> 7) & COL0) : 0ull);
      const uint64_t rs = f0 & ~wf;
      uint64_t rsn = (TSW_DIAG_BITS(A.dbg) & 4u) ? 0ull : nw & rs;
      while (rsn) {
        const uint32_t bb = (uint32_t)__builtin_ctzll(rsn);
        anch[AB[p] + (uint32_t)__popcll(rs & ((1ull << bb) - 1ull))] = (uint16_t)lvl;
        rsn &= rsn - 1ull;
      }
    };

    // ---- lane pairs: a block is processed by lanes (2j, 2j+1), lane h = lane & 1 owning its
    // rows 4h..4h+3 as one dword (rows of 8 cells = bytes). All bit logic is 32-bit; the two
    // halves exchange their rows with a DPP quad_perm swap (no LDS). A level's ~30 active
    // blocks fill the wave's 64 lanes instead of leaving half of them idle.
    const uint32_t h = lane & 1u;
    uint32_t* V32 = reinterpret_cast<uint32_t*>(V);
    const uint32_t* FR32 = reinterpret_cast<const uint32_t*>(FRs);
    unsigned int* WL32 = reinterpret_cast<unsigned int*>(WL);
    constexpr uint32_t C0 = 0x01010101u, C7 = 0x80808080u;
    auto partner = [](uint32_t x) -> uint32_t {  // value of the other lane of the pair
      return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    };
    // run-start anchors among this half's new cells (block's run starts numbered in block order)
    auto anchors2 = [&](uint32_t p, uint32_t nw, uint32_t f0, uint32_t fw, uint32_t lvl, uint32_t abp) {
      const uint32_t bx = p - __umulhi(p, A.bp_magic) * Bp;
      const uint32_t wf = ((f0 << 1) & ~C0) | ((bx & 3u) ? ((fw >> 7) & C0) : 0u);
      const uint32_t rs = f0 & ~wf;
      const uint32_t below = __popc(partner(rs));  // the low half's run starts precede ours
      uint32_t rsn = (TSW_DIAG_BITS(A.dbg) & 4u) ? 0u : nw & rs;
      const uint32_t base = abp + (h ? below : 0u);
      while (rsn) {
        const uint32_t bb = (uint32_t)__builtin_ctz(rsn);
        anch[base + __popc(rs & ((1u << bb) - 1u))] = (uint16_t)lvl;
        rsn &= rsn - 1u;
      }
    };
    // exact pushes of block p (this lane's half has new cells nw): the blocks gaining a cell at
    // lvl + 1 — self (either half, or across the halves), W / E (either half), N (row 0, even
    // lane), S (row 7, odd lane); dedup by test-and-set on the next level's flags, appends by
    // ballot + mbcnt. Even lanes own (self, W, N), odd lanes (E, S).
    // `overlap` runs after the three returning dedup atomics are issued and before their results are
    // used (the run-start anchor stores), so it hides under their LDS latency
    auto push2 = [&](uint32_t p, uint32_t nw, uint32_t vv, uint32_t f0, uint32_t fw, uint32_t fe, uint32_t fx,
                    uint32_t fp, uint32_t vw, uint32_t ve, uint32_t vx, uint32_t vp, uint32_t* Fn, uint16_t* Ln,
                    uint16_t* On, auto&& overlap) {
      const uint32_t in = ((nw << 1) & ~C0) | ((nw >> 1) & ~C7) | (nw << 8) | (nw >> 8);
      const uint32_t cross = h ? (nw << 24) : (nw >> 24);  // row 4 -> row 3 / row 3 -> row 4
      const bool s_self = ((in & f0 & ~vv) | (cross & fp & ~vp)) != 0u;
      const bool s_w = (((nw & C0) << 7) & fw & ~vw) != 0u;
      const bool s_e = (((nw & C7) >> 7) & fe & ~ve) != 0u;
      const bool s_x = ((h ? (nw >> 24) : (nw << 24)) & fx & ~vx) != 0u;  // S (odd) / N (even)
      const uint32_t both = (s_self ? 1u : 0u) | (s_w ? 2u : 0u) | (s_e ? 4u : 0u);
      const uint32_t pb = both | partner(both);
      const uint32_t tw = p - 1u, te = p + 1u, tx = h ? p + Bp : p - Bp;
      // even: self, W, N; odd: E, S
      bool w0 = h ? (pb & 4u) != 0u : (pb & 1u) != 0u;
      bool w1 = h ? s_x : (pb & 2u) != 0u;
      bool w2 = h ? false : s_x;
      const uint32_t t0 = h ? te : p, t1 = h ? tx : tw, t2 = tx;
      auto tas2 = [&](bool w, uint32_t t) -> uint32_t {
        const uint32_t m = w ? 1u << (t >> klog) : 0u;
        return atomicOr(&Fn[w ? (t & kmask) : lane], m) & m;
      };
      const uint32_t o0 = tas2(w0, t0), o1 = tas2(w1, t1), o2 = tas2(w2, t2);
      overlap();
      w0 = w0 && !o0;
      w1 = w1 && !o1;
      w2 = w2 && !o2;
      const bool lds_only = nn + 3u * NL <= cap;
      auto append2 = [&](bool c, uint32_t entry) {
        const uint64_t m = __ballot(c) & hmask;
        if (c) {
          const uint32_t pos = nn + lane_rank(m);
          if (lds_only) Ln[pos] = (uint16_t)entry;
          else blk_list_put_slow(Ln, On, cap, pos, entry);
        }
        nn += (uint32_t)__popcll(m);
      };
      append2(w0, t0);
      append2(w1, t1);
      append2(w2, t2);
    };

    // ---- level 0: the goal cell; queue the blocks that gain cells at distance 1 ----------
    uint32_t ncur = 0;
    {
      const uint32_t gp = ((gy >> 3) + 1u) * Bp + (gx >> 3);
      const uint64_t gm = 1ull << (((gy & 7u) << 3) | (gx & 7u));
      const bool act = gl == 0u && live;
      const uint32_t p = act ? gp : idle_p;
      const uint64_t nw = act ? gm : 0ull;
      const uint64_t f0 = FRs[p], fw = FRs[p - 1u], fe = FRs[p + 1u], fn = FRs[p - Bp], fs = FRs[p + Bp];
      if (act) {
        V[p] = gm;
        anchors(p, nw, f0, fw, 0u);
      }
      push(p, nw, nw, f0, fw, fe, fn, fs, 0ull, 0ull, 0ull, 0ull, FL, LS, lovf);
      ncur = nn;
      lds_sync();
    }

    // ---- levels 1, 2, ...: process the blocks that gain cells at distance lvl -------------
    uint32_t cur = 0;
    uint32_t lvl = 1;
    while (PAIR ? __ballot(ncur != 0u) != 0ull : ncur != 0u) {
      if (lvl >= 0xFFFFu) {
        if (lane == 0) atomicOr(A.err, ERR_DIST_OVERFLOW);
        // this goal's table cannot hold its distances (u16): the host plans it without one (K3)
        if (A.govf && (lane & 31u) == 0u && live) A.govf[gi] = 1u;
        break;
      }
      const uint32_t nxt = cur ^ 1u;
      const uint16_t* Lc = LS + cur * cap;
      uint16_t* Ln = LS + nxt * cap;
      const uint16_t* Oc = lovf + cur * nbp;
      uint16_t* On = lovf + nxt * nbp;
      uint32_t* Fc = FL + cur * nfk;
      uint32_t* Fn = FL + nxt * nfk;
      const uint64_t pnew = ((gpar + lvl) & 1u) ? ~CB_EVEN : CB_EVEN;  // cells at distance lvl
      const uint64_t psrc = ~pnew;                                      // cells at distance lvl-1
      const uint32_t psrc2 = (uint32_t)psrc;  // a half-block has the same checkerboard
      nn = 0;
      // one chunk: lane's list entry p (idle lanes: the guard block idle_p, act = false)
      auto chunk = [&](uint32_t p, bool act) {
        const uint64_t v0 = V[p], vw = V[p - 1u], ve = V[p + 1u], vn = V[p - Bp], vs = V[p + Bp];
        const uint64_t f0 = FRs[p], fw = FRs[p - 1u], fe = FRs[p + 1u], fn = FRs[p - Bp], fs = FRs[p + Bp];
        const uint64_t a = v0 & psrc, aw = vw & psrc, ae = ve & psrc, an = vn & psrc, as = vs & psrc;
        const uint64_t ex = ((a << 1) & ~COL0) | ((a >> 1) & ~COL7) | ((aw >> 7) & COL0) | ((ae << 7) & COL7) |
                            (a << 8) | (a >> 8) | (an >> 56) | (as << 56);
        const uint64_t nw = ex & f0 & ~v0;  // 0 for idle lanes (FR of the guard block is 0)
        const uint64_t vv = v0 | nw;
        // owner-exclusive within the level (the list is deduplicated); idle lanes rewrite the
        // zero guard block
        V[p] = vv;
        const uint64_t wln = nw & (((v0 << 1) & ~COL0) | ((vw >> 7) & COL0));
        if (wln && !(TSW_DIAG_BITS(A.dbg) & 2u)) {
          if constexpr (WLS) WL[p] |= wln;  // owner-exclusive within the level, program order across levels
          else wl_or(WL + p, (unsigned long long)wln);
        }
        bad |= act && nw == 0ull;  // entries must gain a cell
        anchors(p, nw, f0, fw, lvl);
        push(p, nw, vv, f0, fw, fe, fn, fs, vw, ve, vn, vs, Fn, Ln, On);
        ++n_chunk;
      };
      // one chunk of 32 blocks: this lane's half of entry p (idle lanes: the guard block)
      auto chunk2 = [&](uint32_t p, bool act) {
        const uint32_t o = 2u * p + h;
        const uint32_t ox = h ? 2u * (p + Bp) : 2u * (p - Bp) + 1u;  // vertical neighbour dword
        const uint32_t v0 = V32[o], vw = V32[o - 2u], ve = V32[o + 2u], vx = V32[ox];
        const uint32_t f0 = FR32[o], fw = FR32[o - 2u], fe = FR32[o + 2u], fx = FR32[ox];
        const uint32_t abp = AB[p];
        const uint32_t vp = partner(v0), fp = partner(f0);
        const uint32_t a = v0 & psrc2, aw = vw & psrc2, ae = ve & psrc2, ax = vx & psrc2, ap = vp & psrc2;
        const uint32_t up_in = h ? (ap >> 24) : (ax >> 24);   // row above the half's top row
        const uint32_t dn_in = h ? (ax << 24) : (ap << 24);   // row below the half's bottom row
        const uint32_t ex = ((a << 1) & ~C0) | ((a >> 1) & ~C7) | ((aw >> 7) & C0) | ((ae << 7) & C7) | (a << 8) |
                            (a >> 8) | up_in | dn_in;
        const uint32_t nw = ex & f0 & ~v0;  // 0 for idle lanes (FR of the guard block is 0)
        const uint32_t vv = v0 | nw;
        V32[o] = vv;  // owner-exclusive (deduplicated list, one lane per half); idle lanes rewrite 0
        const uint32_t wln = nw & (((v0 << 1) & ~C0) | ((vw >> 7) & C0));
        if (wln && !(TSW_DIAG_BITS(A.dbg) & 2u)) {
          if constexpr (WLS) WL32[o] |= wln;
          else wl_or32(WL32 + o, wln);
        }
        const uint32_t nwp = partner(nw);
        bad |= act && (nw | nwp) == 0u;  // entries must gain a cell
        push2(p, nw, vv, f0, fw, fe, fx, fp, vw, ve, vx, vp, Fn, Ln, On, [&]() { anchors2(p, nw, f0, fw, lvl, abp); });
        ++n_chunk;
      };
      // path choice and trip counts are wave-uniform (PAIR: over both halves' lists)
      const uint32_t nmax = PAIR ? max((uint32_t)__builtin_amdgcn_readlane((int)ncur, 0),
                                       (uint32_t)__builtin_amdgcn_readlane((int)ncur, 32))
                                 : ncur;
      if (nmax <= NL / 2u && nmax <= cap) {
        // few active blocks: lane pairs, one half-block per lane (a single chunk)
        const uint32_t j0 = gl >> 1;
        chunk2(j0 < ncur ? (uint32_t)Lc[j0] : idle_p, j0 < ncur);
      } else if (nmax <= cap) {
        // LDS-only list (wave-uniform): no global load in the loop, so nothing waits for the
        // wave's outstanding anchor stores; entries prefetched one chunk ahead
        uint32_t e_next = gl < ncur ? (uint32_t)Lc[gl] : idle_p;
        for (uint32_t b0 = 0; b0 < nmax; b0 += NL) {
          const uint32_t p = e_next;
          const uint32_t i = b0 + NL + gl;
          e_next = i < ncur ? (uint32_t)Lc[i] : idle_p;
          chunk(p, b0 + gl < ncur);
        }
      } else {
        for (uint32_t b0 = 0; b0 < nmax; b0 += NL) {
          const uint32_t i = b0 + gl;
          const uint32_t p = i >= ncur ? idle_p : i < cap ? (uint32_t)Lc[i] : ld_nc16(Oc + (i - cap));
          chunk(p, i < ncur);
        }
      }
      // the flags of this level's list are reused two levels later
      for (uint32_t t = gl; t < nfk; t += NL) Fc[t] = 0u;
      if (PAIR ? __ballot(nn > cap) != 0ull : nn > cap) full_sync();  // overflow entries went to global memory
      else lds_sync();
      cur = nxt;
      ncur = nn;
      ++lvl;
    }
    if (__ballot(bad) && lane == 0) atomicOr(A.err, ERR_BFS_LIST);
    full_sync();  // anchors (global) complete before the decode reads them
    const uint64_t t1 = clk();

    // ---- decode + write-out: one 32-cell row word per lane per iteration ------------------
    // d(b) = F(b) + C(run(b)): F(b) = 2*popc(WL & bits<=b) - (b+1) is the +-1 walk from bit 0,
    // C(j) = A(j) - F(s_j) for run j starting at bit s_j with anchor A(j) (mod 2^16: the table
    // is u16). Bit b belongs to run popc(rsw & bits<=b) - 1 (<= 16 runs per word); C goes to row
    // popc(...) of this lane's column of the run table.
    const uint8_t* V8 = reinterpret_cast<const uint8_t*>(V);
    const uint8_t* WL8 = reinterpret_cast<const uint8_t*>(WL);  // LDS (WLS) or global, L2-resident
    const uint8_t* FR8 = reinterpret_cast<const uint8_t*>(FRs);
    uint16_t* D = A.dist + slot * A.dstride;
    const uint32_t Ww = (W + 31u) >> 5, nwords = A.H * Ww;
    const float invWw = 1.0f / (float)Ww;
    // compact index of the anchor of run-start cell bit cb of block pb (bx & 3 = j): the block's
    // run-start mask as in `anchors`
    auto aidx = [&](uint32_t pb, uint32_t j, uint32_t cb) -> uint32_t {
      const uint64_t f = FRs[pb];
      const uint64_t wf = ((f << 1) & ~COL0) | (j ? ((FRs[pb - 1u] >> 7) & COL0) : 0ull);
      return AB[pb] + (uint32_t)__popcll(f & ~wf & ((1ull << cb) - 1ull));
    };
    // row word k -> (y, cw), its first block p0 and row-in-block r; bitmaps gathered from the 4
    // blocks' row bytes; the first 4 run anchors are loaded one iteration ahead (L2 latency)
    struct Word {
      uint32_t y, cw, r, p0, vis, wl, f0, a[4];
    };
    auto fetch = [&](uint32_t k, Word& o) {
      uint32_t y = (uint32_t)((float)k * invWw);
      while (y * Ww > k) --y;
      while ((y + 1u) * Ww <= k) ++y;
      o.y = y;
      o.cw = k - y * Ww;
      o.r = y & 7u;
      o.p0 = ((y >> 3) + 1u) * Bp + 4u * o.cw;
      o.vis = o.wl = o.f0 = 0u;
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        if (4u * o.cw + j < BW) {
          const uint32_t off = (o.p0 + j) * 8u + o.r;
          o.vis |= (uint32_t)V8[off] << (8u * j);
          if constexpr (WLS) o.wl |= (uint32_t)WL8[off] << (8u * j);
          else o.wl |= (uint32_t)__builtin_nontemporal_load(WL8 + off) << (8u * j);
          o.f0 |= (uint32_t)FR8[off] << (8u * j);
        }
      }
      // unconditional loads (a run-less slot reads the word's first cell, unused), so the
      // compiler can count them in vmcnt instead of draining at a branch merge
      uint32_t rs = o.f0 & ~(o.f0 << 1);
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        const uint32_t sj = rs ? (uint32_t)__builtin_ctz(rs) : 0u;
        o.a[j] = ld_nc16(anch + aidx(o.p0 + (sj >> 3), sj >> 3, o.r * 8u + (sj & 7u)));
        rs &= rs - 1u;
      }
    };
    // decode of this lane's word into pk (two u16 per dword); false when the word has no visited cell
    auto decode = [&](const Word& cu, uint32_t* pk) {
      const uint32_t r = cu.r, p0 = cu.p0, vis = cu.vis, wl = cu.wl, f0 = cu.f0;
      const uint32_t rsw = f0 & ~(f0 << 1);
      if (vis != 0u) {
        // runs 1..4: branch-free with the prefetched anchors (rows past the last run are never
        // looked up); runs 5..16 (rare) load their anchors here
        uint32_t rs = rsw;
#pragma unroll
        for (uint32_t j = 1; j <= 4u; ++j) {
          const uint32_t sj = rs ? (uint32_t)__builtin_ctz(rs) : 0u;
          rs &= rs - 1u;
          const uint32_t Fs = 2u * __popc(wl & (0xFFFFFFFFu >> (31u - sj))) - (sj + 1u);
          CT[ct_slot(lane, j)] = (uint16_t)(cu.a[j - 1u] - Fs);  // own column: program order suffices
        }
        for (uint32_t j = 5; rs != 0u; ++j) {
          const uint32_t sj = __builtin_ctz(rs);
          rs &= rs - 1u;
          const uint32_t Aj = ld_nc16(anch + aidx(p0 + (sj >> 3), sj >> 3, r * 8u + (sj & 7u)));
          const uint32_t Fs = 2u * __popc(wl & (0xFFFFFFFFu >> (31u - sj))) - (sj + 1u);
          CT[ct_slot(lane, j)] = (uint16_t)(Aj - Fs);
        }
#pragma unroll
        for (int b = 0; b < 32; ++b) {
          const uint32_t m = 0xFFFFFFFFu >> (31 - b);
          const uint32_t C = CT[ct_slot(lane, (uint32_t)__popc(rsw & m))];
          const uint32_t F = 2u * __popc(wl & m) - (uint32_t)(b + 1);
          const uint32_t v = ((vis >> b) & 1u) ? ((F + C) & 0xFFFFu) : 0xFFFFu;
          if (b & 1) pk[b >> 1] |= v << 16;
          else pk[b >> 1] = v;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) pk[j] = 0xFFFFFFFFu;
      }
    };
    // lane-strided write-out (tables not 16-B aligned): the row word goes straight to HBM
    auto put_direct = [&](const Word& cu, const uint32_t* pk) {
      const uint32_t x0 = cu.cw << 5;
      const uint32_t cnt = min(32u, W - x0);
      uint16_t* dst = D + (uint64_t)cu.y * W + x0;
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
    };
    // Staged write-out of the wave's 64 consecutive words kb..kb+63 (valid: this lane's word exists).
    // Consecutive row words tile the row-major table, so each half-wave's 32 words are ONE contiguous
    // cell range [cs, ce) (<= 1024 cells): the half's lanes put their cells into LS at (cell - base),
    // base = cs rounded down to 8 cells, then the whole wave stores 16-B chunks of that range — lane q
    // takes chunk q, so every store instruction covers 1 KB contiguous (a lane-strided 16-B pattern
    // measured 11x slower than coalesced stores on gfx950: scripts/calib_write.hip). Chunks cut by the
    // range ends (neighbouring halves own the rest) are written cell by cell.
    auto put_staged = [&](const Word& cu, const uint32_t* pk, bool valid, uint32_t kb) {
      const uint32_t x0 = cu.cw << 5;
      const uint32_t cnt = valid ? min(32u, W - x0) : 0u;
      const uint32_t cb = cu.y * W + x0;
      if constexpr (PAIR) {
        // each half stages its own goal's 32 words kb..kb+31 into its own LS and stores them with
        // its own 32 lanes (512 B per store instruction per half)
        if (kb >= nwords) return;  // wave-uniform
        const uint32_t ll = min(31u, nwords - 1u - kb);
        const uint32_t cs = hf ? (uint32_t)__builtin_amdgcn_readlane((int)cb, 32)
                               : (uint32_t)__builtin_amdgcn_readlane((int)cb, 0);
        const uint32_t ce = hf ? (uint32_t)__builtin_amdgcn_readlane((int)(cb + cnt), (int)(32u + ll))
                               : (uint32_t)__builtin_amdgcn_readlane((int)(cb + cnt), (int)ll);
        const uint32_t base = cs & ~7u;
        if (valid) {
          const uint32_t off = cb - base;
          if ((W & 31u) == 0u) {
            uint4* q = reinterpret_cast<uint4*>(LS + off);
            q[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            q[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
            q[2] = make_uint4(pk[8], pk[9], pk[10], pk[11]);
            q[3] = make_uint4(pk[12], pk[13], pk[14], pk[15]);
          } else {
#pragma unroll
            for (uint32_t b = 0; b < 32u; ++b)
              if (b < cnt) LS[off + b] = (uint16_t)(pk[b >> 1] >> ((b & 1u) * 16u));
          }
        }
        lds_sync();
        const uint32_t nch = live ? (ce - base + 7u) >> 3 : 0u;
        for (uint32_t q = gl; q < nch; q += 32u) {
          const uint32_t c0 = base + 8u * q;
          if (c0 >= cs && c0 + 8u <= ce) {
            *reinterpret_cast<uint4*>(D + c0) = *reinterpret_cast<const uint4*>(LS + 8u * q);
          } else {
#pragma unroll
            for (uint32_t b = 0; b < 8u; ++b)
              if (c0 + b >= cs && c0 + b < ce) D[c0 + b] = LS[8u * q + b];
          }
        }
        lds_sync();
        return;
      }
#pragma unroll
      for (uint32_t hh = 0; hh < 2u; ++hh) {
        const uint32_t fl = 32u * hh;
        if (kb + fl >= nwords) break;  // wave-uniform
        const uint32_t ll = min(fl + 31u, nwords - 1u - kb);
        const uint32_t cs = (uint32_t)__builtin_amdgcn_readlane((int)cb, (int)fl);
        const uint32_t ce = (uint32_t)__builtin_amdgcn_readlane((int)(cb + cnt), (int)ll);
        const uint32_t base = cs & ~7u;
        if (valid && (lane >> 5) == hh) {
          const uint32_t off = cb - base;
          if ((W & 31u) == 0u) {  // word starts 64-B aligned in the staging buffer
            uint4* q = reinterpret_cast<uint4*>(LS + off);
            q[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            q[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
            q[2] = make_uint4(pk[8], pk[9], pk[10], pk[11]);
            q[3] = make_uint4(pk[12], pk[13], pk[14], pk[15]);
          } else {
#pragma unroll
            for (uint32_t b = 0; b < 32u; ++b)
              if (b < cnt) LS[off + b] = (uint16_t)(pk[b >> 1] >> ((b & 1u) * 16u));
          }
        }
        lds_sync();  // one wave: the DS unit runs its instructions in order
        const uint32_t nch = (ce - base + 7u) >> 3;
        for (uint32_t q = lane; q < nch; q += 64u) {
          const uint32_t c0 = base + 8u * q;
          if (c0 >= cs && c0 + 8u <= ce) {
            const uint4 v4 = *reinterpret_cast<const uint4*>(LS + 8u * q);
            if (TSW_DIAG_BITS(A.dbg) & 1u) {
              typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
              const u32x4 vv = {v4.x, v4.y, v4.z, v4.w};
              __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(D + c0));
            } else {
              *reinterpret_cast<uint4*>(D + c0) = v4;
            }
          } else {
#pragma unroll
            for (uint32_t b = 0; b < 8u; ++b)
              if (c0 + b >= cs && c0 + b < ce) D[c0 + b] = LS[8u * q + b];
          }
        }
        lds_sync();  // staging reads issued before the next half / the next run table overwrites LS
      }
    };
    auto emit = [&](const Word& cu, bool valid, uint32_t kb) {
      uint32_t pk[16];
      if (valid) decode(cu, pk);
      if (A.stage) put_staged(cu, pk, valid, kb);
      else if (valid) put_direct(cu, pk);
    };
    // four words in flight per lane (ring w0..w3, fetch distance 4): a decode waits on loads
    // issued three decodes earlier, enough to cover L2 latency at this residency. The loop is
    // wave-uniform (the staged write-out is a wave-wide exchange); lanes past the end idle.
    // (PAIR: per half, NL = 32 lanes; a half without a goal decodes nothing and stores nothing)
    Word w0{}, w1{}, w2{}, w3{};
    const uint32_t nwl = live ? nwords : 0u;  // words of this lane's goal
    if (gl < nwl) fetch(gl, w0);
    if (gl + NL < nwl) fetch(gl + NL, w1);
    if (gl + 2u * NL < nwl) fetch(gl + 2u * NL, w2);
    if (gl + 3u * NL < nwl) fetch(gl + 3u * NL, w3);
    for (uint32_t kb = 0; kb < nwords; kb += 4u * NL) {
      const uint32_t k = kb + gl;
      emit(w0, k < nwl, kb);
      if (k + 4u * NL < nwl) fetch(k + 4u * NL, w0);
      if (kb + NL < nwords) emit(w1, k + NL < nwl, kb + NL);
      if (k + 5u * NL < nwl) fetch(k + 5u * NL, w1);
      if (kb + 2u * NL < nwords) emit(w2, k + 2u * NL < nwl, kb + 2u * NL);
      if (k + 6u * NL < nwl) fetch(k + 6u * NL, w2);
      if (kb + 3u * NL < nwords) emit(w3, k + 3u * NL < nwl, kb + 3u * NL);
      if (k + 7u * NL < nwl) fetch(k + 7u * NL, w3);
    }
    lds_sync();  // the next goal re-initialises this wave's LDS
    if (A.prof) {
      const uint64_t t2 = clk();
      t_bfs += t1 - t0;
      t_dec += t2 - t1;
      n_lvl += PAIR ? (uint64_t)lvl * (uint64_t)__popcll(__ballot(live && gl == 0u)) : lvl;
    }
  }
  if (A.prof && lane == 0) {
    atomicAdd((unsigned long long*)&A.prof[0], (unsigned long long)t_bfs);
    atomicAdd((unsigned long long*)&A.prof[1], (unsigned long long)t_dec);
    atomicAdd((unsigned long long*)&A.prof[2], (unsigned long long)n_lvl);
    atomicAdd((unsigned long long*)&A.prof[3], (unsigned long long)n_chunk);
  }
}

uint32_t bfs_blk_klog(uint32_t nbp) {
  uint32_t kl = 6;
  while ((32u << kl) < nbp) ++kl;
  return kl;
}

uint32_t bfs_blk_waves_per_block(uint32_t nbp, uint32_t cap, int max_lds, bool wls, bool pair) {
  const size_t per_wave = (size_t)blk_bfs_words(nbp, 1u << bfs_blk_klog(nbp), cap, wls) * 4u * (pair ? 2u : 1u);
  const size_t shared = (size_t)blk_shared_u64(nbp) * 8u;  // FR u64 + AB u32
  if (max_lds <= 0 || shared + per_wave > (size_t)max_lds) return 0;
  return (uint32_t)std::min<size_t>(16u, ((size_t)max_lds - shared) / per_wave);
}

hipError_t launch_bfs_blk(const BlkBfsArgs& A0, int max_lds, int num_cu, hipStream_t s) {
  if (A0.k == 0) return hipSuccess;
  BlkBfsArgs A = A0;
  A.klog = bfs_blk_klog(A.nbp);
  A.bp_magic = (uint32_t)((0xFFFFFFFFull + A.Bp) / A.Bp);  // ceil(2^32 / Bp): exact p / Bp for p*Bp < 2^32
  const bool wls = A.wls != 0u, pair = A.pair != 0u;
  const uint32_t gpw = pair ? 2u : 1u;  // goal slots per wave
  const size_t per_wave = (size_t)blk_bfs_words(A.nbp, 1u << A.klog, A.cap, wls) * 4u * gpw;
  const size_t shared = (size_t)blk_shared_u64(A.nbp) * 8u;  // FR u64 + AB u32
  const uint32_t nwv = std::min<uint32_t>(A.max_waves, bfs_blk_waves_per_block(A.nbp, A.cap, max_lds, wls, pair));
  if (nwv == 0 || A.nbp > 0x10000u || A.cap > 0x8000u) return hipErrorInvalidValue;
  const uint32_t grid =
      std::max<uint32_t>(1u, std::min<uint32_t>((uint32_t)num_cu, (A.k + gpw * nwv - 1u) / (gpw * nwv)));
  if ((uint64_t)grid * nwv * gpw > A.scratch_waves) return hipErrorInvalidValue;  // scratch per goal slot
  const size_t lds = shared + nwv * per_wave;
#ifdef TSW_DIAG
  // the WLS / PAIR A/B variants exist in the diagnostic build only (both measured slower)
  const void* fn = wls ? (pair ? (const void*)k_bfs_blk<true, true> : (const void*)k_bfs_blk<true, false>)
                       : (pair ? (const void*)k_bfs_blk<false, true> : (const void*)k_bfs_blk<false, false>);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (wls && pair) hipLaunchKernelGGL((k_bfs_blk<true, true>), dim3(grid), dim3(nwv * 64u), lds, s, A);
  else if (wls) hipLaunchKernelGGL((k_bfs_blk<true, false>), dim3(grid), dim3(nwv * 64u), lds, s, A);
  else if (pair) hipLaunchKernelGGL((k_bfs_blk<false, true>), dim3(grid), dim3(nwv * 64u), lds, s, A);
  else hipLaunchKernelGGL((k_bfs_blk<false, false>), dim3(grid), dim3(nwv * 64u), lds, s, A);
#else
  if (wls || pair) return hipErrorInvalidValue;
  hipError_t e = hipFuncSetAttribute((const void*)k_bfs_blk<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_bfs_blk<false, false>), dim3(grid), dim3(nwv * 64u), lds, s, A);
#endif
  return hipGetLastError();
}

}  // namespace tsw
