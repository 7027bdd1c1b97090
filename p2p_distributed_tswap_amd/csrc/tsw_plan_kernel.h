// tsw_plan_kernel.h — k_plan: the persistent MAPD planning kernel (K2 step + K4 assignment).
//
// One workgroup runs whole timesteps of tswap_mapd (tswap.rs:104-170) on the device
// without returning to the host:
//   ASSIGN  state machine + nearest-pickup assignment (tswap.rs:106-139): needy agents
//           compacted in index order, block-wide argmin over unused tasks per idle agent
//   PRE1    parallel next-hop lookup for agents whose (v, g) changed
//   RULES   rules phase (tswap.rs:180-252), exact, as rounds of
//             parallel: succ(k) = lowest agent at next(k) (tswap.rs:190-192), and for
//                       every agent k >= cursor whether it fires: rule 3 (succ at its
//                       goal, :198) or rule 4 (k on a cycle of length >= 2 of succ over
//                       not-at-goal agents — exactly when the chase of :205-238 gets
//                       back to k; Floyd walk on the LDS succ array)
//             block-min -> first firing agent; one lane applies its goal swap /
//             target rotation (:199-202, :241-249); cursor moves past it.
//           Agents that do not fire change nothing, so this equals the sequential scan. With
//           n <= wave_rules_max wave 0 runs the rounds alone, and a run of firings that touch
//           disjoint agents (rule-3 swaps, 2-cycle rotations, none closing a new cycle) is
//           applied as one batch (round 6).
//   PRE2    parallel lookup for agents whose goal changed
//   MOVE    movement phase (tswap.rs:257-285), exact, as decidability rounds: agent k
//           commits in a round iff no still-undecided agent a < k can change what k reads
//           at its turn in the sequential scan — a's target is neither k's target nor
//           k's cell and a is not the occupant of k's target (a mutual-swap partner of a
//           lower undecided agent is caught by the second test). Decisions read the
//           round-start state, commits are disjoint. Three passes per round: targets +
//           round-tagged MU (lowest undecided agent per target cell), decide, commit.
//           With duplicate start cells the phase runs as the serial scan instead.
//   RECORD  parallel (Point, AgentState) record (tswap.rs:144-158) + termination (:163-169)
// When a next hop is unresolved (lazy next-hop mode) the kernel enqueues every such
// (cell, goal) pair, saves its exact resume point and exits; the host runs K3 (k_astar)
// and relaunches.
// (Header: the kernel template and its launcher; each instantiation is compiled in its own translation
// unit, tsw_plan_v*.hip, so the build runs them in parallel — one instantiation takes ~4 min of hipcc.)
#pragma once
#include <hip/hip_runtime.h>

#include "tsw_astar.h"
#include "tsw_internal.h"
#include "tsw_plan.h"
#include "tsw_worker.h"

// Planner instrumentation (TSW_PLAN_DEBUG, diagnostic build: sub-phase ticks, change tags, wait classes).
// Round 6 note: the helpers below stay out of line (as in rounds 1-5). Force-inlining them all took
// PlanArgs off the stack (0 B scratch) but the fully inlined planner hung in its first rules phase
// whenever an instrumentation branch ran, and in a two-process run without them;
// scripts/exp_lib.sh + hang_probe.py reproduce it.
#define PLAN_DBG (P.dbg != 0u)
// Planner barrier. Built with -DTSW_PBAR (scripts/exp_lib.sh) and run with TSW_PLAN_DEBUG, every barrier
// also leaves per-wave breadcrumbs in the host-visible watchdog words (line reached / passed, barriers
// passed: the watchdog prints them) and checks that all waves arrived at the same one. Round 6: this is
// how the debug-mode hang was read — waves 1-15 kept passing barriers while wave 0's breadcrumbs stopped,
// i.e. wave 0 ran on with an empty EXEC mask.
#ifndef TSW_PBAR
#define PBAR() __syncthreads()
#else
#define PBAR()                                                                                            \
  do {                                                                                                    \
    if (PLAN_DBG) {                                                                                       \
      uint32_t* bid_ = bar_ids();                                                                         \
      if ((threadIdx.x & 63u) == 0u) {                                                                    \
        bid_[threadIdx.x >> 6] = __LINE__;                                                                \
        if (P.hflags)                                                                                     \
          __hip_atomic_store(&P.hflags[8u + (threadIdx.x >> 6)], (uint32_t)__LINE__, __ATOMIC_RELAXED,    \
                             __HIP_MEMORY_SCOPE_SYSTEM);                                                  \
      }                                                                                                   \
      __syncthreads();                                                                                    \
      if ((threadIdx.x & 63u) == 0u && P.hflags) {                                                        \
        __hip_atomic_store(&P.hflags[8u + (threadIdx.x >> 6)], 0x10000u | (uint32_t)__LINE__,             \
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                                  \
        __hip_atomic_fetch_add(&P.hflags[24u + (threadIdx.x >> 6)], 1u, __ATOMIC_RELAXED,                 \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                                \
      }                                                                                                   \
      if (threadIdx.x == 0u) {                                                                            \
        for (uint32_t w_ = 1; w_ < (blockDim.x >> 6); ++w_)                                               \
          if (bid_[w_] != bid_[0] && bid_[16] == 0u) {                                                    \
            bid_[16] = 1u;                                                                                \
            if (P.hflags)                                                                                 \
              __hip_atomic_store(&P.hflags[4], (bid_[0] << 16) | bid_[w_], __ATOMIC_RELAXED,              \
                                 __HIP_MEMORY_SCOPE_SYSTEM);                                              \
            printf("[k_plan] barrier mismatch: wave 0 at line %u, wave %u at line %u\n", bid_[0], w_, bid_[w_]); \
          }                                                                                               \
      }                                                                                                   \
      __syncthreads();                                                                                    \
    } else {                                                                                              \
      __syncthreads();                                                                                    \
    }                                                                                                     \
  } while (0)
#endif

namespace tsw {

namespace {

__device__ __forceinline__ uint32_t* bar_ids() {  // PBAR: per-wave barrier line, [16] = reported
  __shared__ uint32_t b[17];
  return b;
}

constexpr uint8_t NHC_DIRTY = 0xFE;  // per-agent next-hop code must be re-looked-up
constexpr uint32_t OCC_NONE = 0xFFFFFFFFu;
constexpr uint32_t OCC_FLAG = 0x80000000u;  // cell holds more than one agent (duplicate starts)
constexpr uint32_t OCC_IDX = 0x7FFFFFFFu;
constexpr uint32_t SUCC_TERM = 0xFFFFFFFFu;
constexpr uint32_t NO_AGENT = 0xFFFFFFFFu;
constexpr uint32_t NO_CELL = 0xFFFFFFFFu;
constexpr uint32_t ABATCH = 8;    // K4: idle agents whose nearest pickups one pass over the tasks computes
constexpr uint32_t KCH = 32;      // K4: tasks per spatial chunk (PlanArgs::kbox / kcnt), a multiple of 16
constexpr uint32_t KPT = 2;       // K4: chunks per thread whose count and box stay in registers across a batch
constexpr uint32_t LIST_CAP = 1024;  // entries of the kernel's LDS `list` (ASSIGN compaction, changed agents)
// movement-round decision states
constexpr uint8_t DEC_OPEN = 0, DEC_DONE = 1, DEC_STAY = 2, DEC_MOVE = 3, DEC_SWAP = 4;

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t y = __shfl_xor(x, off, 64);
    x = y < x ? y : x;
  }
  return x;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t y = __shfl_xor(x, off, 64);
    x = y < x ? y : x;
  }
  return x;
}

// Agent / occupancy arrays; the AG / OC template flags place them in LDS at compile time
// (ds_read/ds_write instead of flat accesses) when they fit.
struct Arrays {
  uint32_t* V;     // cell of agent
  uint32_t* G;     // goal cell of agent
  int32_t* GT;     // goal-table slot of G (goal_tab[G])
  uint32_t* SUCC;  // rules: successor agent; movement: target cell
  uint8_t* NHC;    // next-hop code of (V, G) or NHC_DIRTY
  uint8_t* DEC;    // movement-round state
  uint8_t* ONC;    // rules: agent lies on a cycle of succ
  uint8_t* CANDC;  // rules: next hop of succ(k)'s cell toward k's goal — what succ(k) needs when it takes
                   // k's goal (rule-3 swap, or the rotation of a cycle through both)
  uint32_t* MK;    // rules (wave rounds): lowest batch lane touching each agent, ~0 when clear
  uint32_t* F1;    // rules: pointer-doubling buffers (n + 1 entries, n = terminal sink)
  uint32_t* F2;
  uint32_t* OCC;   // per cell: lowest agent | OCC_FLAG, or OCC_NONE
  uint64_t* MU;    // per cell: (round << 32) | ~(lowest undecided agent targeting it), movement rounds
  uint32_t* MU32;  // the same in LDS (MUL, n < 2^16): round16 << 16 | (0xFFFF - agent), round16 in [1, 65535]
  uint32_t* LIVE;  // K4: pickup points in Morton order, TASK_TAKEN once assigned (PlanArgs::live)
  unsigned long long t0;  // wall clock at the launch (coop: "no worker has started" is measured from here)
};

// Next-hop code of (v, goal slot tab). A plain load may return a stale PENDING from this XCD's L2
// after a worker has stored the code (coop mode): then the word is read again at agent scope, so a
// code that is already known does not send the planner through a refresh pass and a wait. Codes never
// change once written, so either read is exact.
__device__ __forceinline__ uint8_t nh_code_at(const uint8_t* nh, uint64_t nstride, bool coop, int32_t tab, uint32_t v) {
  const uint8_t* p = nh + (uint64_t)tab * nstride + v;
  uint8_t c = *p;
  if (coop && (c == NH_PENDING || c == NH_PENDING_S)) {
    const uint32_t w = __hip_atomic_load(reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3u),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c = (uint8_t)(w >> (8u * (uint32_t)((uintptr_t)p & 3u)));
  }
  return c;
}
__device__ __forceinline__ uint8_t nh_code(const PlanArgs& P, int32_t tab, uint32_t v) {
  return nh_code_at(P.nh, P.nstride, P.coop != 0u, tab, v);
}

// next-hop code of agent k for its current (v, g); -1 unresolved, -2 goal has no table
__device__ __forceinline__ int lookup_code(const PlanArgs& P, const Arrays& S, uint32_t k) {
  const uint8_t c = S.NHC[k];
  if (c <= NH_STAY) return c;
  const int32_t tab = S.GT[k];
  if (tab < 0) return -2;
  const uint8_t code = nh_code(P, tab, S.V[k]);
  if (code <= NH_STAY) {
    S.NHC[k] = code;
    return code;
  }
  return -1;
}

__device__ void occ_rescan(const PlanArgs& P, const Arrays& S, uint32_t cell) {
  uint32_t lowest = OCC_NONE, cnt = 0;
  for (uint32_t k = 0; k < P.n; ++k)
    if (S.V[k] == cell) {
      if (cnt == 0) lowest = k;
      ++cnt;
    }
  S.OCC[cell] = cnt == 0 ? OCC_NONE : (lowest | (cnt > 1 ? OCC_FLAG : 0u));
}

// succ(k) = lowest-index agent at next(k) (position(), tswap.rs:192/223), or TERM when k is at
// its goal, its next cell is empty, or its next hop is not resolved yet (caller checks).
__device__ __forceinline__ uint32_t succ_of(const PlanArgs& P, const Arrays& S, uint32_t k) {
  const uint32_t v = S.V[k];
  if (v == S.G[k]) return SUCC_TERM;
  const uint8_t c = S.NHC[k];
  if (c > NH_STAY) return SUCC_TERM;
  const uint32_t o = S.OCC[step_cell(v, c, P.W)];
  return o == OCC_NONE ? SUCC_TERM : (o & OCC_IDX);
}

// Parallel (whole block): succ of every agent, the rule-4 labels and the rule-3 prefetch.
// The chase of tswap.rs:205-238 started at j = succ(i) returns to i exactly when i lies on
// a cycle (length >= 2) of succ over not-at-goal agents. Pointer doubling: after R rounds
// with 2^R > n, F(k) = succ^(2^R)(k) sits on the cycle k drains into (or the sink n), and
// succ^(2^R) permutes each cycle, so {F(k)} is exactly the set of cycle members.
// pf (phase start, wide prefetch): rules_prefetch fused into the first pass — the pair (cell of
// succ(k), goal of k) is the CANDC load itself, and k's own next pair is one more load — saving the
// separate block-wide pass and its repeated table reads.
__device__ __forceinline__ void prefetch_pair(const PlanArgs& P, uint32_t v, uint32_t g, int32_t tab, uint32_t* s_q);
__device__ __forceinline__ bool spec_full(const PlanArgs& P, const uint32_t* s_q);
__device__ void rules_init(const PlanArgs& P, const Arrays& S, uint32_t* pf = nullptr) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x, n = P.n;
  for (uint32_t k = tid; k < n; k += bd) {
    const uint32_t s = succ_of(P, S, k);
    S.SUCC[k] = s;
    S.F1[k] = s == SUCC_TERM ? n : s;
    S.ONC[k] = 0;
    uint8_t cc = NHC_DIRTY;
    const int32_t tab = S.GT[k];
    if (s != SUCC_TERM && s != k && tab >= 0)
      cc = P.nh[(uint64_t)tab * P.nstride + S.V[s]];
    S.CANDC[k] = cc;
    if (pf && tab >= 0 && !spec_full(P, pf)) {  // as rules_prefetch (wide mode: no ONC filter)
      const uint8_t c = S.NHC[k];
      const uint32_t g = S.G[k];
      if (c < NH_STAY && S.V[k] != g) {
        const uint32_t u = step_cell(S.V[k], c, P.W);
        if (u != g && P.nh[(uint64_t)tab * P.nstride + u] == NH_UNKNOWN) prefetch_pair(P, u, g, tab, pf);
      }
      if (cc == NH_UNKNOWN) prefetch_pair(P, S.V[s], g, tab, pf);
    }
  }
  if (tid == 0) {
    S.F1[n] = n;
    S.F2[n] = n;
  }
  PBAR();
  uint32_t* a = S.F1;
  uint32_t* b = S.F2;
  for (uint32_t r = 1; r <= n; r <<= 1) {
    for (uint32_t k = tid; k < n; k += bd) b[k] = a[a[k]];
    PBAR();
    uint32_t* t = a;
    a = b;
    b = t;
  }
  for (uint32_t k = tid; k < n; k += bd) {
    const uint32_t c = a[k];
    if (c != n) S.ONC[c] = 1;
  }
  PBAR();
}

// Incremental rules relabel (thread 0) after a firing changed the goals of the `cnt` agents in
// `lst` (rule-4 rotation: every member of the rotated cycle; rule-3 swap: b and s) and the refresh
// re-looked-up their next hops. In the rules phase nobody moves (OCC is fixed), so only these
// agents' successors changed: SUCC / CANDC are recomputed for them alone, and a cycle that appears
// must pass through one of them while a cycle that disappears contained one (all of a rotated
// cycle's members are in `lst`, and rule 3 only extends the chain of s, which was terminal). So
// each changed agent's cycle label is a walk along SUCC from it: back to itself = on a cycle (label
// the cycle), TERM / a self-loop / an agent on another cycle = not. Walks average ~2 hops on the
// warehouse grids, against a block-wide pointer doubling over every agent. Returns false (caller
// relabels in full) if a walk runs past `limit` hops.
// one changed agent's successor, cleared label and CANDC (independent per agent)
__device__ __forceinline__ void relabel_reset(const PlanArgs& P, const Arrays& S, uint32_t k) {
  const uint32_t s = succ_of(P, S, k);
  S.SUCC[k] = s;
  S.ONC[k] = 0;
  uint8_t cc = NHC_DIRTY;
  if (s != SUCC_TERM && s != k && S.GT[k] >= 0) cc = P.nh[(uint64_t)S.GT[k] * P.nstride + S.V[s]];
  S.CANDC[k] = cc;
}

// the walks of rules_relabel_changed, after relabel_reset of every agent in lst
__device__ bool relabel_walks(const PlanArgs& P, const Arrays& S, const uint32_t* lst, uint32_t cnt, uint32_t limit);

__device__ bool rules_relabel_changed(const PlanArgs& P, const Arrays& S, const uint32_t* lst, uint32_t cnt,
                                      uint32_t limit) {
  for (uint32_t i = 0; i < cnt; ++i) relabel_reset(P, S, lst[i]);
  return relabel_walks(P, S, lst, cnt, limit);
}

__device__ bool relabel_walks(const PlanArgs& P, const Arrays& S, const uint32_t* lst, uint32_t cnt, uint32_t limit) {
  for (uint32_t i = 0; i < cnt; ++i) {
    const uint32_t a = lst[i];
    if (S.ONC[a]) continue;  // labelled by an earlier walk of this loop
    uint32_t x = S.SUCC[a];
    uint32_t steps = 0;
    while (x != SUCC_TERM && x != a) {
      if (S.ONC[x]) {
        // x is labelled: a cycle that still stands (every member of a cycle that broke is in
        // `lst` and was cleared above). It may contain a itself — `lst` accumulates every agent
        // changed since the last labelling, including members of a cycle a rule-3 swap closed
        // and labelled in fire() — so go once around it: meeting a puts a on it, back at x
        // without a means a only drains into it. A walk that does neither means a stale label:
        // relabel in full.
        uint32_t y = S.SUCC[x];
        while (y != x && y != a) {
          if (y == SUCC_TERM || S.SUCC[y] == y || ++steps > limit) return false;
          y = S.SUCC[y];
        }
        x = y;  // == a: on the cycle (labelled below); == x: not
        break;
      }
      const uint32_t nx = S.SUCC[x];
      if (nx == x) break;    // self-loop (stay code): a chain end
      x = nx;
      if (++steps > limit) return false;
    }
    if (x == a) {
      uint32_t y = a;
      do {
        S.ONC[y] = 1;
        y = S.SUCC[y];
      } while (y != a);
    }
  }
  return true;
}

__device__ __forceinline__ void put_query(const PlanArgs& P, uint8_t* p, uint32_t qi, uint32_t v, uint32_t g,
                                          int32_t tab) {
  *p = NH_PENDING;  // only once the slot is ours: a pending code is always really queued
  AstarQuery q;
  q.v = v;
  q.goal = g;
  q.tab = tab;
  // coop mode reads no result index: the entry carries its enqueue time (wall clock, low 32 bits)
  q.out = P.coop ? (uint32_t)wall_clock64() : qi;
  P.Q[qi] = q;
}

// A pair a step needs now: queue it if it is unresolved (the planner then exits for a host-side K3
// pass, or — coop mode — waits for the concurrent workers). Needed pairs are at most 2n per exit and
// the speculative ones stay below qcap/2, so the queue (qcap = 4n + 4096) cannot overflow; if it
// ever did, the pair is not marked and the host, seeing qcount > qcap, fails the call. In coop mode
// a pair already queued speculatively is promoted: queued again on the needed queue, which the
// workers serve first (the duplicate resolves to the same code).
// s_q[0]: needed pairs queued since the launch began, s_q[1]: speculative ones (coop mode).
__device__ __forceinline__ void enqueue_pair(const PlanArgs& P, uint32_t v, uint32_t g, int32_t tab, uint32_t* s_q) {
  uint8_t* p = P.nh + (uint64_t)tab * P.nstride + v;
  const uint8_t c = *p;
  if (c != NH_UNKNOWN && !(P.coop && c == NH_PENDING_S)) return;  // queued (PENDING) or resolved
  const uint32_t qi = atomicAdd(&s_q[0], 1u);
  if (qi < P.qcap) put_query(P, p, qi, v, g, tab);
}

// A pair wanted soon but not by this step (walk-ahead within urgent_hops, a pickup arrival within
// urgent_hops + 1): the needed queue while it has room to spare, else a speculative prefetch. In coop
// mode the needed queue is linear over the launch (qcap entries) and a needed pair it cannot hold stays
// UNKNOWN, so urgent pairs stop at half of it and the other half stays for the pairs a step waits on
// (ADVICE r5).
__device__ __forceinline__ void urgent_pair(const PlanArgs& P, uint32_t v, uint32_t g, int32_t tab, uint32_t* s_q,
                                            uint8_t code) {
  if (*(volatile const uint32_t*)&s_q[0] < P.qcap / 2u) enqueue_pair(P, v, g, tab, s_q);
  else if (code == NH_UNKNOWN) prefetch_pair(P, v, g, tab, s_q);
}

// speculative queue full (no more prefetches this launch)
__device__ __forceinline__ bool spec_full(const PlanArgs& P, const uint32_t* s_q) {
  return P.coop ? *(volatile const uint32_t*)&s_q[1] >= P.qscap : *(volatile const uint32_t*)&s_q[0] >= P.qcap / 2u;
}

// A speculative prefetch. Exit mode: the slot is reserved by CAS only while the queue holds fewer
// than qcap/2 pairs, so prefetches never take the room the needed pairs of an exit rely on. Coop
// mode: its own queue (QS), resolved by the workers after every needed pair.
__device__ __forceinline__ void prefetch_pair(const PlanArgs& P, uint32_t v, uint32_t g, int32_t tab, uint32_t* s_q) {
  uint8_t* p = P.nh + (uint64_t)tab * P.nstride + v;
  if (*p != NH_UNKNOWN) return;
  if (P.coop) {
    const uint32_t qi = atomicAdd(&s_q[1], 1u);
    if (qi >= P.qscap) return;
    *p = NH_PENDING_S;
    AstarQuery q;
    q.v = v;
    q.goal = g;
    q.tab = tab;
    q.out = s_q[5];  // enqueue timestep: the workers drop entries older than stale_steps
    P.QS[qi] = q;
    return;
  }
  const uint32_t lim = P.qcap / 2u;
  uint32_t cur = *(volatile uint32_t*)s_q;
  for (;;) {
    if (cur >= lim) return;
    const uint32_t prev = atomicCAS(s_q, cur, cur + 1u);
    if (prev == cur) break;
    cur = prev;
  }
  put_query(P, p, cur, v, g, tab);
}

// parallel: refresh next-hop codes of agents whose code is dirty; unresolved pairs are
// appended to the launch's K3 queue (s_q counts every pair queued since the launch began,
// speculative prefetches included). Returns how many dirty agents still lack a code
// (block-uniform): the planner must exit for K3 iff that is nonzero.
__device__ uint32_t refresh_codes(const PlanArgs& P, const Arrays& S, uint32_t* s_q, uint32_t* s_need,
                                  uint32_t sec) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  if (tid == 0) *s_need = 0;
  PBAR();
  for (uint32_t k = tid; k < P.n; k += bd) {
    if (S.NHC[k] <= NH_STAY) continue;
    const uint32_t v = S.V[k], g = S.G[k];
    if (v == g) continue;
    const int32_t tab = S.GT[k];
    if (tab < 0) {
      atomicOr(&P.ctl->err, ERR_NO_TABLE);
      continue;
    }
    const uint8_t code = nh_code(P, tab, v);
    if (code <= NH_STAY) {
      S.NHC[k] = code;
    } else {
      if (PLAN_DBG && P.coop && (code == NH_UNKNOWN || code == NH_PENDING_S)) {
        const uint32_t grp = sec == SEC_PRE1 ? 0u : sec == SEC_RULES ? 1u : 2u;
        atomicAdd(&P.cc->dbg_need[2u * grp + (code == NH_PENDING_S ? 1u : 0u)], 1u);
        // PRE1, never queued: assigned a task / picked up in this step's ASSIGN (DEC tag, diagnostics)
        if (sec == SEC_PRE1 && code == NH_UNKNOWN && (S.DEC[k] & 0x40u))
          atomicAdd(&P.cc->dbg_need[(S.DEC[k] & 1u) ? 7u : 6u], 1u);
      }
      enqueue_pair(P, v, g, tab, s_q);  // no-op if already queued (PENDING)
      atomicAdd(s_need, 1u);
    }
  }
  PBAR();
  return *s_need;
}

// ---- coop mode (concurrent K3 workers) ------------------------------------------------------
// Memory: the planner's queue entries and PENDING marks are plain stores published by one release
// store of the queue heads (agent scope: written back past this XCD's L2); workers read entries with
// agent-scope loads and write each code with an agent-scope store, which the planner polls with
// agent-scope loads. A code, once written, never changes, so a stale plain read of the table can
// only see an older state (UNKNOWN / PENDING) — a conservative "unresolved", never a wrong hop.
// (Write-through entries and PENDING marks with relaxed head stores instead were measured slower:
// every write-through drops the line from this XCD's L2, and the planner's next plain loads of
// those table lines missed — movement passes 3x slower.)
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host watchdog (coop and exit mode): the planner polls this in every loop that can run long
__device__ __forceinline__ bool plan_abort(const PlanArgs& P) {
  return P.hflags && __hip_atomic_load(&P.hflags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

// thread 0: make every entry queued so far visible to the workers (caller: after a barrier). A publish
// whose heads equal the last published ones is skipped: no entry and no PENDING mark was written since
// (marks are only written with an entry), and the agent-scope release it would cost writes back this
// XCD's L2. s_q[3] / s_q[4] hold the last published heads (0 = the launch's zeroed CoopCtl).
__device__ __forceinline__ void coop_publish(const PlanArgs& P, uint32_t* s_q) {
  const uint32_t hn = min(s_q[0], P.qcap), hs = min(s_q[1], P.qscap), hh = min(s_q[6], P.qhcap);
  const uint32_t hp = min(s_q[8], P.qpcap);
  if (hn == s_q[3] && hs == s_q[4] && hh == s_q[7] && hp == s_q[9]) return;
  s_q[3] = hn;
  s_q[4] = hs;
  s_q[7] = hh;
  s_q[9] = hp;
  if (P.QP) __hip_atomic_store(&P.cc->head_p, hp, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (P.QH) __hip_atomic_store(&P.cc->head_h, hh, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&P.cc->head_s, hs, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&P.cc->head_n, hn, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  // wake idle workers, which poll only this word (a plain agent-scope store of a new value)
  s_q[2] += 1u;
  __hip_atomic_store(&P.cc->pub, s_q[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0, while the other threads may be queueing speculative pairs: publish the needed queue's head
// only (no needed pair is queued concurrently; the speculative head waits for the next full publish,
// after a barrier, since a reserved speculative slot may not be written yet)
__device__ __forceinline__ void coop_publish_needed(const PlanArgs& P, uint32_t* s_q) {
  const uint32_t hn = min(s_q[0], P.qcap);
  if (hn == s_q[3]) return;
  s_q[3] = hn;
  __hip_atomic_store(&P.cc->head_n, hn, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  s_q[2] += 1u;
  __hip_atomic_store(&P.cc->pub, s_q[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned long long COOP_NO_WORKER_TICKS = 100000ull;    // 1 ms at 100 MHz after the launch: no worker running
constexpr unsigned long long COOP_RETRY_TICKS = 2000000ull;      // 20 ms pending: queue the pair again
constexpr unsigned long long COOP_GIVE_UP_TICKS = 500000000ull;  // 5 s: safety valve
enum : int { COOP_OK = 0, COOP_GIVE_UP = 1, COOP_RETRY = 2 };

// Parallel (block-uniform result): publish, then wait until every agent whose next-hop code is dirty
// has it or is no longer pending (UNKNOWN: not queued — the caller's refresh queues it). Codes read
// here go straight into the agent's NHC. COOP_GIVE_UP: no worker alive, a worker error, or the
// safety limit (the caller exits to the host). COOP_RETRY: a pair stayed pending for 20 ms — more
// than any A* on these grids; the caller queues the still-pending pairs again (a duplicate query
// resolves to the same code), so a lost update can cost a retry but never a stall.
__device__ int coop_wait(const PlanArgs& P, const Arrays& S, uint32_t* s_q, uint32_t* s_flag, uint32_t sec) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  if (tid == 0) {
    coop_publish(P, s_q);
    *s_flag = COOP_OK;
    if (PLAN_DBG) {
      const uint32_t hs = min(s_q[1], P.qscap), cs = ld_agent(&P.cc->claim_s);
      const uint32_t dep = hs > cs ? hs - cs : 0u;
      P.cc->dbg_depth += dep;
      P.cc->dbg_depth_max = max(P.cc->dbg_depth_max, dep);
    }
  }
  PBAR();
  const unsigned long long t0 = wall_clock64();
  int st = COOP_OK;
  for (uint32_t k = tid; k < P.n && st == COOP_OK; k += bd) {
    if (S.NHC[k] <= NH_STAY) continue;
    const uint32_t v = S.V[k];
    const int32_t tab = S.GT[k];
    if (v == S.G[k] || tab < 0) continue;
    const uint8_t* p = P.nh + (uint64_t)tab * P.nstride + v;
    const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3u);
    const uint32_t sh = 8u * (uint32_t)((uintptr_t)p & 3u);
    for (uint32_t spin = 0;; ++spin) {
      const uint8_t c = (uint8_t)(ld_agent(w) >> sh);
      if (c <= NH_STAY) {
        S.NHC[k] = c;
        break;
      }
      if (c == NH_UNKNOWN) break;
      const unsigned long long dt = wall_clock64() - t0;
      if (dt > COOP_GIVE_UP_TICKS || ld_agent(&P.cc->err) != 0u ||
          (ld_agent(&P.cc->alive) == 0u && wall_clock64() - S.t0 > COOP_NO_WORKER_TICKS) ||
          (P.hflags && __hip_atomic_load(&P.hflags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)) {
        st = COOP_GIVE_UP;
        break;
      }
      if (dt > COOP_RETRY_TICKS) {
        st = COOP_RETRY;
        break;
      }
      if (spin < 64) __builtin_amdgcn_s_sleep(1);
      else __builtin_amdgcn_s_sleep(8);
    }
  }
  if (st != COOP_OK) atomicMax(s_flag, (uint32_t)(st == COOP_GIVE_UP ? 3 : st));
  PBAR();
  const uint32_t f = *s_flag;
  if (tid == 0) {
    const unsigned long long dt = wall_clock64() - t0;
    // diagnostics: PRE1 waits classed by what the step's ASSIGN did (5: assigned a task, 6: only
    // pickup arrivals, 7: neither — walking agents)
    {
      const uint32_t kslot[6] = {0u, 0u, 3u, 5u, 6u, 7u};
      sec = (PLAN_DBG && (sec >> 8)) ? kslot[sec >> 8] : min(sec & 0xFFu, 7u);
    }
    P.cc->waits += 1u;
    P.cc->wait_ticks += dt;
    P.cc->waits_sec[sec] += 1u;
    P.cc->wait_sec[sec] += dt;
  }
  PBAR();
  return f == 3u ? COOP_GIVE_UP : (int)f;
}

// COOP_RETRY: every dirty agent whose pair still reads pending is queued again on the needed queue
__device__ void coop_requeue(const PlanArgs& P, const Arrays& S, uint32_t* s_q) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  for (uint32_t k = tid; k < P.n; k += bd) {
    if (S.NHC[k] <= NH_STAY) continue;
    const uint32_t v = S.V[k];
    const int32_t tab = S.GT[k];
    if (v == S.G[k] || tab < 0) continue;
    uint8_t* p = P.nh + (uint64_t)tab * P.nstride + v;
    const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3u);
    const uint8_t c = (uint8_t)(ld_agent(w) >> (8u * (uint32_t)((uintptr_t)p & 3u)));
    if (c != NH_PENDING && c != NH_PENDING_S) continue;
    const uint32_t qi = atomicAdd(&s_q[0], 1u);
    if (qi < P.qcap) put_query(P, p, qi, v, S.G[k], tab);
  }
  PBAR();
}

// Next hops are missing (refresh_codes returned nonzero and queued them). Coop mode: wait for the
// workers and re-run the refresh until nothing is missing (true: continue in the kernel). Otherwise,
// or if the workers do not answer, false: the caller exits for a host-side K3 pass.
__device__ bool coop_resolve(const PlanArgs& P, const Arrays& S, uint32_t* s_q, uint32_t* s_need, uint32_t* s_flag,
                             uint32_t sec) {
  if (!P.coop) return false;
  for (int it = 0; it < 1024; ++it) {
    const int st = coop_wait(P, S, s_q, s_flag, sec);
    if (st == COOP_GIVE_UP) return false;
    if (st == COOP_RETRY) coop_requeue(P, S, s_q);
    if (refresh_codes(P, S, s_q, s_need, sec & 0xFFu) == 0u) return true;
  }
  return false;
}

// Parallel, after rules_init: the next hops a firing of this rules round (or the movement phase
// after it) could need. A rule-3
// swap hands succ(k) the goal of k (tswap.rs:199-202); a rule-4 rotation hands every cycle
// member the goal of its predecessor on the cycle (:241-249) — both are the pair
// (cell of succ(k), goal of k) for a firing candidate k. Every unresolved such pair is queued
// speculatively (no exit): the planner exits only when a firing actually needs a code, and
// that one K3 launch then resolves everything queued so far. Half the queue stays free for the
// pairs an exit needs.
__device__ void rules_prefetch(const PlanArgs& P, const Arrays& S, uint32_t* s_q) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  for (uint32_t k = tid; k < P.n; k += bd) {
    if (spec_full(P, s_q)) break;
    const int32_t tab = S.GT[k];
    if (tab < 0) continue;
    // k's own next hop from the cell it moves to: read by the movement phase when k moved
    // earlier in the same step (tswap.rs:263-273, later agents see earlier moves) and by the
    // next step's refresh
    const uint8_t c = S.NHC[k];
    if (c < NH_STAY && S.V[k] != S.G[k]) {
      const uint32_t u = step_cell(S.V[k], c, P.W);
      if (u != S.G[k] && P.nh[(uint64_t)tab * P.nstride + u] == NH_UNKNOWN) prefetch_pair(P, u, S.G[k], tab, s_q);
    }
    const uint32_t s = S.SUCC[k];
    if (s == SUCC_TERM || s == k) continue;
    if (!P.wide_prefetch && !(S.ONC[k] || S.V[s] == S.G[s])) continue;
    const uint32_t vs = S.V[s];
    if (P.nh[(uint64_t)tab * P.nstride + vs] == NH_UNKNOWN) prefetch_pair(P, vs, S.G[k], tab, s_q);
  }
  PBAR();
}

// rules_prefetch restricted to the agents a firing changed (rule 3: b and s, rule 4: the cycle):
// only their goals, hence their next hops and successors, moved, so only their pairs are new.
// After rules_init (SUCC valid).
__device__ uint32_t walk_prefetch(const PlanArgs& P, uint32_t* s_q, uint32_t u, uint32_t g, int32_t tab,
                                  uint32_t hops, uint32_t h0 = 0u, uint32_t* end = nullptr,
                                  uint32_t* endh = nullptr);
__device__ void dag_prefetch(const PlanArgs& P, uint32_t* s_q, uint32_t u, uint32_t g, int32_t tab);

// coop mode: agent k will be idle at `cell` (its delivery): a worker predicts its next task and walks that
// task's pickup -> delivery chain ahead of the assignment (s_q[8]: entries queued, PlanArgs::QP)
__device__ __forceinline__ void predict_push(const PlanArgs& P, uint32_t* s_q, uint32_t cell, uint32_t k) {
  const uint32_t qi = atomicAdd(&s_q[8], 1u);
  if (qi < P.qpcap) P.QP[qi] = make_uint2(cell, k);
}

__device__ __forceinline__ void prefetch_changed(const PlanArgs& P, const Arrays& S, uint32_t* s_q, uint32_t k) {
  // delivering: a rule handed the agent another delivery cell, so its next task changes with it
  if ((P.predict & 2u) && P.QP && P.st[k] == ST_TO_DELIVERY) predict_push(P, s_q, S.G[k], k);
  if (spec_full(P, s_q)) return;
  // heading to a pickup: its new goal is where the state machine switches it to the delivery
  // (tswap.rs:113-118) — the (goal cell, delivery) pair, a step before nextnext_prefetch would queue it
  if (P.mode != MODE_STEP && P.m > 0 && P.st[k] == ST_TO_PICKUP) {
    const int32_t tk = P.task[k];
    if (tk >= 0 && (uint32_t)tk < P.m) {
      const uint32_t pc = S.G[k], dc = P.dlv[tk];
      const int32_t dt = dc == CELL_BAD ? -1 : P.goal_tab[dc];
      if (dt >= 0 && pc != dc && P.nh[(uint64_t)dt * P.nstride + pc] == NH_UNKNOWN) prefetch_pair(P, pc, dc, dt, s_q);
    }
  }
  const int32_t tab = S.GT[k];
  if (tab < 0) return;
  const uint8_t c = S.NHC[k];
  if (S.V[k] != S.G[k] && (P.prefetch_ext & 4u)) {
    // the agent's new path: walked ahead (and the DAG past its first unresolved cell) now, a step
    // before the next step's walk-ahead would queue it
    if (c < NH_STAY) walk_prefetch(P, s_q, step_cell(S.V[k], c, P.W), S.G[k], tab, P.wide_prefetch ? P.wide_prefetch : 1u);
    else if (c > NH_STAY && P.dag_prefetch) dag_prefetch(P, s_q, S.V[k], S.G[k], tab);
  } else if (c < NH_STAY && S.V[k] != S.G[k]) {
    const uint32_t u = step_cell(S.V[k], c, P.W);
    if (u != S.G[k] && P.nh[(uint64_t)tab * P.nstride + u] == NH_UNKNOWN) prefetch_pair(P, u, S.G[k], tab, s_q);
  }
  const uint32_t s = S.SUCC[k];
  if (s == SUCC_TERM || s == k) return;
  const uint32_t vs = S.V[s];
  if (P.nh[(uint64_t)tab * P.nstride + vs] == NH_UNKNOWN) prefetch_pair(P, vs, S.G[k], tab, s_q);
}

__device__ void rules_prefetch_list(const PlanArgs& P, const Arrays& S, uint32_t* s_q, const uint32_t* lst,
                                    uint32_t cnt) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  for (uint32_t i = tid; i < cnt; i += bd) prefetch_changed(P, S, s_q, lst[i]);
  PBAR();
}

// The shortest-path DAG toward goal g past cell u (u's own pair is queued by the caller): whichever
// neighbour u's code picks lies one step closer to the goal (every get_path is a shortest path), so
// the DAG ahead of u is where the agent goes next. Its cells are queued level by level (frontier
// capped at DAG_WIDTH; a resolved cell contributes only the cell its code points at), so a path
// resolves several cells per A* latency instead of one.
__device__ void dag_prefetch(const PlanArgs& P, uint32_t* s_q, uint32_t u, uint32_t g, int32_t tab) {
  constexpr uint32_t DAG_WIDTH = 16;  // array bound; P.dag_width caps the frontier (default 4)
  const uint32_t dwid = P.dag_width ? min(P.dag_width, DAG_WIDTH) : 4u;
  const uint8_t* dtb = P.dt + (uint64_t)tab * P.nstride;
  const uint8_t* ht = P.nh + (uint64_t)tab * P.nstride;
  const uint32_t gy = g / P.W, gx = g - gy * P.W;
  // K1 distance from the detour byte: |c - g|_1 + 2 * detour, ~0 when unknown (blocked / unreachable /
  // saturated: the speculative walk stops there)
  auto dist_of = [&](uint32_t c) -> uint32_t {
    const uint32_t b = dtb[c];
    if (b == DT_NONE) return 0xFFFFFFFFu;
    const uint32_t y = c / P.W, x = c - y * P.W;
    return (x > gx ? x - gx : gx - x) + (y > gy ? y - gy : gy - y) + 2u * b;
  };
  uint32_t fr[DAG_WIDTH], nf = 1;
  fr[0] = u;
  for (uint32_t lv = 0; lv < P.dag_prefetch && nf > 0u; ++lv) {
    uint32_t nx[DAG_WIDTH], nn = 0;
    auto add = [&](uint32_t w) {
      for (uint32_t i = 0; i < nn; ++i)
        if (nx[i] == w) return;
      if (nn < dwid) nx[nn++] = w;
    };
    for (uint32_t i = 0; i < nf; ++i) {
      const uint32_t x = fr[i];
      const uint8_t cx = ht[x];
      if (cx < NH_STAY) {  // resolved: the agent's path continues at one cell
        const uint32_t w = step_cell(x, cx, P.W);
        if (w != g) add(w);
        continue;
      }
      if (cx == NH_STAY) continue;
      const uint32_t dx = dist_of(x);
      if (dx == 0xFFFFFFFFu) continue;
      const uint8_t nb = P.nbmask[x];
#pragma unroll
      for (uint32_t d = 0; d < 4u; ++d) {
        if (!((nb >> d) & 1u)) continue;
        const uint32_t w = step_cell(x, d, P.W);
        if (w == g || dist_of(w) + 1u != dx) continue;
        if (ht[w] == NH_UNKNOWN) prefetch_pair(P, w, g, tab, s_q);
        add(w);
      }
    }
    for (uint32_t i = 0; i < nn; ++i) fr[i] = nx[i];
    nf = nn;
  }
}

// Walk the resolved codes toward g from cell u, which lies h0 resolved hops past the agent's next cell,
// until hop `hops`; queue the first unresolved pair (and the DAG past it). Returns the hops left when the
// walk reached g, else 0. *end / *endh (if given): the cell the walk stopped at and its hop index.
__device__ uint32_t walk_prefetch(const PlanArgs& P, uint32_t* s_q, uint32_t u, uint32_t g, int32_t tab,
                                  uint32_t hops, uint32_t h0, uint32_t* end, uint32_t* endh) {
  uint32_t h = h0;
  uint32_t left = 0;
  for (; h < hops; ++h) {
    if (u == g) {
      left = hops - h;
      break;
    }
    const uint8_t cu = P.nh[(uint64_t)tab * P.nstride + u];
    if (cu == NH_UNKNOWN || cu == NH_PENDING || cu == NH_PENDING_S) {
      // a pair the agent reads within urgent_hops steps goes to the needed queue (served before the
      // speculative backlog, which on wh10k holds ~500 pairs when a wait starts); farther ones are speculative
      if (P.coop && h < P.urgent_hops) urgent_pair(P, u, g, tab, s_q, cu);
      else if (cu == NH_UNKNOWN) prefetch_pair(P, u, g, tab, s_q);
      if (P.dag_prefetch) dag_prefetch(P, s_q, u, g, tab);
      break;
    }
    if (cu >= NH_STAY) break;  // a stay code
    u = step_cell(u, cu, P.W);
  }
  if (end) {
    *end = u;
    *endh = h;
  }
  return left;
}

// Parallel: the next hop of every agent from the cell its resolved code points at (the pair the
// movement phase or the next step reads after the agent moves, tswap.rs:263-273), walked `hops`
// resolved cells ahead; speculative, bounded by half the queue like rules_prefetch.
//  * an agent whose own code is still unresolved (just assigned, goal swapped) gets the DAG past its
//    cell queued now, beside its needed pair, instead of one cell per step after each wait
//    (prefetch_ext bit 0);
//  * an agent heading to a pickup whose walk reaches it continues along the delivery leg: the
//    state machine switches its goal there (tswap.rs:113-118) (prefetch_ext bit 1).
__device__ void nextnext_prefetch(const PlanArgs& P, const Arrays& S, uint32_t* s_q, uint32_t hops) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  for (uint32_t k = tid; k < P.n; k += bd) {
    if (spec_full(P, s_q)) break;
    // heading to a pickup: the pair the state machine needs on arrival (goal := delivery,
    // tswap.rs:113-118) is known since the assignment — (arrival cell, delivery goal). The arrival
    // cell is the agent's current goal: rule-3/4 swaps may have traded the task's pickup cell away.
    uint32_t pc = 0, dc = 0;
    int32_t dtab = -1;
    if (P.mode != MODE_STEP && P.m > 0 && P.st[k] == ST_TO_PICKUP) {
      const int32_t tk = P.task[k];
      if (tk >= 0 && (uint32_t)tk < P.m) {
        pc = S.G[k];
        dc = P.dlv[tk];
        const int32_t dt = dc == CELL_BAD ? -1 : P.goal_tab[dc];
        if (dt >= 0 && pc != dc) {
          dtab = dt;
          const uint8_t cp = P.nh[(uint64_t)dt * P.nstride + pc];
          const uint32_t vk = S.V[k], W = P.W;
          const uint32_t vx = vk % W, vy = vk / W, px = pc % W, py = pc / W;
          const uint32_t man = (vx > px ? vx - px : px - vx) + (vy > py ? vy - py : py - vy);
          // arriving within urgent_hops + 1 steps (Manhattan bounds the path from below): needed queue
          if (P.coop && man <= P.urgent_hops + 1u && (cp == NH_UNKNOWN || cp == NH_PENDING_S)) urgent_pair(P, pc, dc, dt, s_q, cp);
          else if (cp == NH_UNKNOWN) prefetch_pair(P, pc, dc, dt, s_q);
        }
      }
    }
    const int32_t tab = S.GT[k];
    const uint8_t c = S.NHC[k];
    if (tab < 0 || S.V[k] == S.G[k] || c == NH_STAY) continue;
    if (c > NH_STAY) {  // own pair unresolved (queued as needed by the refresh)
      if ((P.prefetch_ext & 1u) && P.dag_prefetch) dag_prefetch(P, s_q, S.V[k], S.G[k], tab);
      continue;
    }
    // Resolved codes never change, so the path from the agent's next cell is fixed while its goal is: the
    // walk resumes at last step's stopping cell (P.wf: cell at that walk, goal, stopping cell, its hop
    // index). An agent that moved since went one hop along that path, so the index drops by one.
    uint32_t u0 = step_cell(S.V[k], c, P.W), h0 = 0;
    const uint32_t vk = S.V[k], gk = S.G[k];
    if (P.wf) {
      const uint4 f = P.wf[k];
      // moved: exactly one hop along the cached path (goals can change and change back in between)
      bool on = f.y == gk && f.x == vk;
      if (f.y == gk && f.x != vk && f.x < P.ncell) {
        const uint8_t cf = P.nh[(uint64_t)tab * P.nstride + f.x];
        on = cf < NH_STAY && step_cell(f.x, cf, P.W) == vk;
      }
      if (on) {
        const uint32_t hp = f.x == vk ? f.w : (f.w > 0u ? f.w - 1u : 0u);
        if (hp > 0u) {
          u0 = f.z;
          h0 = hp;
        }
      }
    }
    uint32_t ue = u0, he = h0;
    const uint32_t left = h0 >= hops ? 0u : walk_prefetch(P, s_q, u0, gk, tab, hops, h0, &ue, &he);
    if (P.wf) P.wf[k] = make_uint4(vk, gk, ue, he);
    if (left > 0u && dtab >= 0 && (P.prefetch_ext & 2u)) walk_prefetch(P, s_q, pc, dc, dtab, left);
  }
  PBAR();
}

// Serial movement phase (tswap.rs:257-285) — used when cells are shared by several agents
// (duplicate start cells); false on an unresolved next hop.
__device__ bool walk_move(const PlanArgs& P, const Arrays& S, PlanCtl& ctl) {
  const uint32_t n = P.n, W = P.W;
  uint32_t i = ctl.i;
  for (; i < n; ++i) {
    const uint32_t vi = S.V[i], gi = S.G[i];
    if (vi == gi) continue;
    const int code = lookup_code(P, S, i);
    if (code < 0) {
      ctl.miss = code == -2 ? 2u : 1u;
      ctl.i = i;
      return false;
    }
    const uint32_t u = step_cell(vi, (uint32_t)code, W);
    const uint32_t o = S.OCC[u];
    if (o == OCC_NONE) {  // rule 2: move
      S.V[i] = u;
      S.NHC[i] = NHC_DIRTY;
      S.OCC[u] = i;
      if (S.OCC[vi] & OCC_FLAG) occ_rescan(P, S, vi);
      else S.OCC[vi] = OCC_NONE;
    } else if ((o & OCC_IDX) != i) {
      const uint32_t j = o & OCC_IDX;
      const uint32_t vj = S.V[j], gj = S.G[j];
      if (vj != gj) {
        const int cj = lookup_code(P, S, j);
        if (cj < 0) {
          ctl.miss = cj == -2 ? 2u : 1u;
          ctl.i = i;
          return false;
        }
        if (step_cell(vj, (uint32_t)cj, W) == vi) {  // mutual swap (:273-278)
          S.V[i] = vj;
          S.V[j] = vi;
          S.NHC[i] = NHC_DIRTY;
          S.NHC[j] = NHC_DIRTY;
          if (S.OCC[vi] & OCC_FLAG) occ_rescan(P, S, vi);
          else S.OCC[vi] = j;
          if (o & OCC_FLAG) occ_rescan(P, S, vj);
          else S.OCC[vj] = i;
        }
      }
    }
  }
  ctl.i = n;
  return true;
}

}  // namespace

// diagnostics: wall-clock ticks of sub-phases (P.sec_ticks[8..15], printed by TSW_PLAN_DEBUG)
#define DTAG(k, bits)                                        \
  do {                                                       \
    if (PLAN_DBG && P.dtag) atomicOr(&P.dtag[(k)], (uint32_t)(bits)); \
  } while (0)

#define PLAN_TICK(slot)                              \
  do {                                               \
    if (PLAN_DBG && tid == 0) {                         \
      const unsigned long long nw_ = wall_clock64(); \
      s_tick[slot] += nw_ - s_tp;                    \
      s_tp = nw_;                                    \
    }                                                \
  } while (0)

// AG: every agent array in LDS. OC: the occupancy grid OCC in LDS; MUL: the movement rounds' MU
// words too (OC alone fits grids whose MU does not, e.g. C3's 170x84 beside the agent arrays).
// AG: every agent array in LDS. PG (!AG): the fixed subset PART_PG (SUCC, V, G, ONC, NHC, CANDC) in
// LDS — carved unconditionally, so its accesses compile to ds_* instead of flat instructions (a flat
// access waits for every outstanding global load as well). Otherwise part_lds picks arrays at run time.
template <bool AG, bool OC, bool MUL, bool PG>
// PlanArgs lives in device memory (written by launch_plan before the dispatch) and is read through a
// const restrict pointer, so the out-of-line helpers get a reference to it instead of to a private copy
// (a by-value kernel argument whose address reaches a non-inlined call is copied to scratch, and every
// field access then became a scratch load; round 6). Its field loads are vector loads the compiler
// repeats after stores (each one a memory round trip and a wait): the fields read inside the rules and
// movement rounds — the instrumentation switch above all, tested at every sub-step — are read once here.
#undef PLAN_DBG
#define PLAN_DBG (kdbg)
__global__ void __launch_bounds__(PLAN_BLOCK_MAX) k_plan(const PlanArgs* __restrict__ Pg, WorkerArgs Wk) {
  const PlanArgs& P = *Pg;
  const bool kdbg = __builtin_amdgcn_readfirstlane(P.dbg) != 0u;
  const uint32_t kab = __builtin_amdgcn_readfirstlane(P.ab_flags);
  const uint32_t kwcap = __builtin_amdgcn_readfirstlane(P.walk_cap);
  const uint8_t* const knh = P.nh;  // next-hop tables, read by the rules rounds' swaps and rotations
  const uint64_t kns = P.nstride;
  const bool kcoop = P.coop != 0u;
  auto nh_code_k = [&](int32_t tab, uint32_t v) { return nh_code_at(knh, kns, kcoop, tab, v); };
  extern __shared__ __align__(16) uint8_t smem[];
  if (blockIdx.x != 0) {  // coop mode: a K3 worker workgroup (tsw_worker.h), Wk.wpb single-wave workers
    const uint32_t w = threadIdx.x >> 6;
    if (w < Wk.wpb) {
      const uint32_t wid = (blockIdx.x - 1u) * Wk.wpb + w;
      if (wid < Wk.nworkers) coop_worker(Wk, reinterpret_cast<uint64_t*>(smem + (size_t)w * Wk.lds_per_wave), wid);
    }
    return;
  }
  __shared__ PlanCtl s_ctl;
  __shared__ uint32_t s_q[10], s_need, s_cnt, s_doit, s_px, s_py, s_exit, s_best, s_miss, s_flag, s_abort, s_cabort, s_hops,
      s_badat;
  __shared__ uint32_t s_ap[128];  // rules: members of a rule-4 cycle rotated by the wave (<= 64), links
  __shared__ uint32_t s_wcount[16];
  __shared__ uint64_t s_red[16];
  __shared__ uint64_t s_bestk[ABATCH];  // K4: per batch agent, block minimum of (distance, task) (LDS atomic min)
  __shared__ uint32_t s_apos[ABATCH], s_acct[ABATCH], s_cnt2, s_ub[ABATCH];
  __shared__ unsigned long long s_tick[48], s_tlast, s_tp;
  __shared__ uint32_t s_tsec;
  __shared__ uint32_t s_bad;               // ASSIGN looked up an off-grid/blocked task cell
  __shared__ uint32_t s_nassign, s_npick;  // diagnostics: this step's assignments / pickup arrivals
  const uint32_t tid = threadIdx.x, bd = blockDim.x, lane = tid & 63u, wid = tid >> 6, nwaves = bd >> 6;
  const uint32_t n = P.n, W = P.W;

  // ---- carve LDS (order must match plan_lds_bytes) ---------------------------
  // coop mode: the XCD this block runs on, first thing — workers placed on it leave (their g-score
  // traffic would share the planner's L2; TSW_WORKER_AVOID_XCD)
  if (P.coop && threadIdx.x == 0)
    __hip_atomic_store(&P.cc->planner_xcc, 1u + hw_xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Arrays S;
  S.t0 = wall_clock64();
  uint8_t* p = smem;
  auto carve = [&](size_t bytes) {
    uint8_t* r = p;
    p += (bytes + 15u) & ~(size_t)15u;
    return r;
  };
  uint32_t* list = reinterpret_cast<uint32_t*>(carve(1024 * 4));
  if constexpr (AG) {
    S.V = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.G = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.GT = reinterpret_cast<int32_t*>(carve((size_t)n * 4));
    S.SUCC = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.F1 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
    S.F2 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
    S.MK = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
    S.NHC = carve(n);
    S.DEC = carve(n);
    S.ONC = carve(n);
    S.CANDC = carve(n);
  } else if constexpr (PG) {
    S.SUCC = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.V = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.G = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.GT = P.gt;
    S.ONC = carve(n);
    S.NHC = carve(n);
    S.CANDC = carve(n);
    if (P.f_lds) {
      S.F1 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
      S.F2 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
    } else {
      S.F1 = P.f1;
      S.F2 = P.f2;
    }
    S.DEC = P.dec;
    S.MK = P.mk;
  } else {
    // arrays the host admitted to LDS (part_lds; carve order = part_lds_bytes' order), else global
    auto pick32 = [&](uint32_t bit, uint32_t* g) {
      return (P.part_lds & bit) ? reinterpret_cast<uint32_t*>(carve((size_t)n * 4)) : g;
    };
    auto pick8 = [&](uint32_t bit, uint8_t* g) { return (P.part_lds & bit) ? carve(n) : g; };
    S.SUCC = pick32(PART_SUCC, P.succ);
    S.V = pick32(PART_V, P.v);
    S.G = pick32(PART_G, P.g);
    S.GT = reinterpret_cast<int32_t*>(pick32(PART_GT, reinterpret_cast<uint32_t*>(P.gt)));
    S.ONC = pick8(PART_ONC, P.onc);
    S.NHC = pick8(PART_NHC, P.nhc);
    S.CANDC = pick8(PART_CANDC, P.candc);
    if (P.f_lds) {  // pointer doubling (rules_init) on LDS instead of global memory
      S.F1 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
      S.F2 = reinterpret_cast<uint32_t*>(carve((size_t)(n + 1) * 4));
    } else {
      S.F1 = P.f1;
      S.F2 = P.f2;
    }
    S.DEC = P.dec;
    S.MK = P.mk;  // (batched firing runs only with the agent arrays in LDS; this copy stays unused)
  }
  if constexpr (OC) {
    S.OCC = reinterpret_cast<uint32_t*>(carve((size_t)P.ncell * 4));
    if constexpr (MUL) {
      S.MU32 = reinterpret_cast<uint32_t*>(carve((size_t)P.ncell * 4));
      S.MU = nullptr;
    } else {
      S.MU = P.mu;
    }
  } else {
    S.OCC = P.occ;
    S.MU = P.mu;
  }
  S.LIVE = P.live;
  for (uint32_t k = tid; k <= n; k += bd) S.MK[k] = 0xFFFFFFFFu;
  for (uint32_t k = tid; k < n; k += bd) {
    const uint32_t g = P.g[k];
    if constexpr (AG) {
      S.V[k] = P.v[k];
      S.G[k] = g;
      S.DEC[k] = P.dec[k];
    } else {
      if (P.part_lds & PART_V) S.V[k] = P.v[k];
      if (P.part_lds & PART_G) S.G[k] = g;
    }
    S.GT[k] = P.goal_tab[g];
    S.NHC[k] = NHC_DIRTY;
  }
  if constexpr (OC)
    for (uint32_t c = tid; c < P.ncell; c += bd) S.OCC[c] = P.occ[c];
  // round tags start at 1 (move_rounds is incremented before use), so zeroed MU is stale
  for (uint32_t c = tid; c < P.ncell; c += bd) {
    if constexpr (MUL) S.MU32[c] = 0u;
    else S.MU[c] = 0ull;
  }
  if (tid == 0) {
    s_ctl = *P.ctl;
    s_ctl.status = PLAN_RUNNING;
    s_exit = 0;
    s_abort = 0;
    s_cabort = 0;
    s_q[0] = 0;  // K3 queue of this launch (reported as qcount at every exit, DONE included)
    s_q[1] = 0;  // speculative queue (coop mode)
    s_q[2] = 0;  // publishes (coop mode)
    s_q[3] = 0;  // last published needed / speculative heads (coop mode)
    s_q[4] = 0;
    s_q[5] = s_ctl.t;  // the timestep speculative entries are queued in (coop mode)
    s_q[6] = 0;  // hot task chains queued this launch (coop mode)
    s_q[7] = 0;  // ... last published head
    s_q[8] = 0;  // predicted task chains queued this launch (coop mode)
    s_q[9] = 0;  // ... last published head
    if (P.coop) __hip_atomic_store(&P.cc->t_now, s_ctl.t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < 48; ++k) s_tick[k] = 0;
    bar_ids()[16] = 0u;
    s_tlast = wall_clock64();
    s_tsec = 7;  // entry / copy-in
    // the host's watchdog: the planner block is resident
    if (P.hflags) {
      __hip_atomic_store(&P.hflags[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  PBAR();
  if (s_ctl.section == SEC_RULES || s_ctl.section == SEC_MOVE) {
    // resuming after K3 resolved the missing next hops: every code starts dirty here
    const uint32_t q = refresh_codes(P, S, s_q, &s_need, s_ctl.section);
    if (q > 0 && !coop_resolve(P, S, s_q, &s_need, &s_flag, s_ctl.section)) {
      if (tid == 0) {
        s_ctl.qcount = s_q[0];
        s_ctl.status = PLAN_NEED_QUERIES;
        s_exit = 1;
      }
    }
    PBAR();
  }

  for (;;) {
    if (s_exit) break;
    if (s_cabort) {
      // coop mode, watchdog seen at a section boundary: the position is a clean resume point, so exit
      // as a coop give-up does and let the host finish the call in exit mode (the 1 ms watchdog test
      // used to need the flag to land inside a wait; a section boundary is as safe)
      if (tid == 0) {
        s_ctl.qcount = s_q[0];
        s_ctl.status = PLAN_NEED_QUERIES;
        s_exit = 1;
      }
      PBAR();
      break;
    }
    if (s_abort) {  // watchdog: exit with the position recorded in ctl (section, cursor, rounds)
      if (tid == 0) {
        s_ctl.status = PLAN_ERROR;
        P.ctl->err |= ERR_ABORT;
        s_exit = 1;
      }
      PBAR();
      break;
    }
    const uint32_t sec = s_ctl.section;
    if (tid == 0) {
      if (plan_abort(P)) {
        if (P.coop) s_cabort = 1;
        else s_abort = 1;
      }
      const unsigned long long now = wall_clock64();
      s_tick[s_tsec] += now - s_tlast;
      s_tlast = now;
      s_tsec = sec < 7 ? sec : 6;
    }
    if (sec == SEC_ASSIGN) {
      // ---- K4: state machine + task assignment (tswap.rs:106-139) -------------
      // The reference walks agents in index order: an agent at its goal advances its state (ToPickup ->
      // ToDelivery with g := delivery, :107-118; ToDelivery -> Idle, :119-121), then an Idle agent takes
      // the nearest unused pickup (:123-138). Transitions touch only their own agent, so they run in
      // parallel. The assignments depend on each other (a task taken by an earlier agent is gone): the
      // idle agents are taken in index order in adaptive batches of up to ABATCH. One block-wide pass
      // computes every batch agent's first minimum of (Manhattan distance, task index) over the Morton
      // index, reading only chunks whose box lower bound is within the agent's current bound; thread 0
      // then accepts the minima in agent order up to the first agent whose task an earlier batch agent
      // took (it and the rest re-run in the next batch). An accepted minimum was taken over a superset of
      // the tasks unused at its sequential turn and is still unused, so it is min_by_key's lowest-index
      // first minimum (tswap.rs:125-130). The first
      // agent whose delivery cell is bad (pos2id panics, :112) ends the step there: assignments of
      // agents below it still happen (and may panic first, :136), none above it.
      if (tid == 0) {
        s_nassign = s_npick = s_bad = 0;
        if (PLAN_DBG) {
          s_tp = wall_clock64();
          s_tick[39] += 1;  // diagnostics: ASSIGN sections (sub-phase ticks in [32..38])
        }
      }
      PBAR();
      for (uint32_t base = 0; base < n && !s_bad; base += bd) {
        const uint32_t i = base + tid;
        bool idle = false;
        if (tid == 0) s_badat = NO_AGENT;  // lowest agent of this chunk with a bad delivery cell
        PBAR();
        if (i < n) {
          uint8_t st = P.st[i];
          if (S.V[i] == S.G[i] && st != ST_IDLE) {
            if (st == ST_TO_PICKUP) {
              st = ST_TO_DELIVERY;
              atomicAdd(&s_npick, 1u);
              if (PLAN_DBG) S.DEC[i] = 0x41;  // diagnostics tag (MOVE re-initialises DEC)
              DTAG(i, 32u);
              const int32_t tk = P.task[i];
              if (tk >= 0) {
                const uint32_t ng = P.dlv[tk];
                if (ng == CELL_BAD) {  // pos2id[&task.delivery] panics (tswap.rs:112)
                  atomicMin(&s_badat, i);
                } else {
                  S.G[i] = ng;
                  S.GT[i] = P.goal_tab[ng];
                  S.NHC[i] = NHC_DIRTY;
                  if ((P.predict & 1u) && P.QP) predict_push(P, s_q, ng, i);
                }
              }
            } else {  // ST_TO_DELIVERY
              st = ST_IDLE;
              P.task[i] = -1;
            }
            P.st[i] = st;
          }
          idle = st == ST_IDLE;
        }
        const uint64_t bal = __ballot(idle);
        if (lane == 0) s_wcount[wid] = (uint32_t)__popcll(bal);
        PBAR();
        PLAN_TICK(32);
        if (idle) {
          uint32_t off = 0;
          for (uint32_t w = 0; w < wid; ++w) off += s_wcount[w];
          off += (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
          list[off] = i;
        }
        if (tid == 0) {
          uint32_t c = 0;
          for (uint32_t w = 0; w < nwaves; ++w) c += s_wcount[w];
          s_cnt = c;
        }
        PBAR();
        PLAN_TICK(33);
        const uint32_t cnt = s_cnt, bad_at = s_badat;
        // Assignments in batches of up to ABATCH agents (index order): one block-wide pass computes every
        // batch agent's first minimum over the unused tasks at once, then thread 0 accepts them in agent
        // order up to the first agent whose task an earlier agent of the batch took (that agent and the
        // rest re-run in the next batch, against the updated LIVE array). An accepted agent's minimum was
        // taken over a superset of what was unused at its sequential turn and its task is still unused,
        // so it IS the sequential first minimum (min_by_key, tswap.rs:125-130).
        // batch size adapts: it doubles after a batch without a conflict and drops to the accepted count
        // after one (the t = 0 burst of a dense instance conflicts often; a busy step's handful rarely)
        uint32_t bcur = (kab & 4u) ? 1u : ABATCH;
        for (uint32_t kk = 0; kk < cnt && !s_bad;) {
          const uint32_t B = min(bcur, cnt - kk);
          if (tid < B) {
            const uint32_t v = S.V[list[kk + tid]];
            s_apos[tid] = (v % W) | ((v / W) << 16);
            s_bestk[tid] = ~0ull;
            s_ub[tid] = 0xFFFFFFFFu;
          }
          PBAR();
          // Spatially pruned scan. The host orders the tasks along a Morton curve of their pickup points and
          // cuts that order into chunks of KCH entries with a bounding box each (static) and a count of
          // untaken entries (KCNT). Phase A: a chunk with an untaken entry holds one within
          // lb + diam of an agent (lb: distance to its box), so U_b = min over such chunks of lb + diam
          // bounds agent b's minimum from above. Phase B: only chunks with lb <= U_b can hold a task at
          // the minimum distance (ties included); their entries are compared as (distance, task index).
          uint32_t apos[ABATCH], ub[ABATCH];
#pragma unroll
          for (uint32_t b = 0; b < ABATCH; ++b) {
            apos[b] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b < B ? s_apos[b] : 0u));
            ub[b] = 0xFFFFFFFFu;
          }
          auto box_lb = [](uint32_t pa, uint32_t lo, uint32_t hi) -> uint32_t {  // distance from pa to a box
            const uint32_t px = pa & 0xFFFFu, py = pa >> 16;
            const uint32_t x0 = lo & 0xFFFFu, y0 = lo >> 16, x1 = hi & 0xFFFFu, y1 = hi >> 16;
            const uint32_t dx = px < x0 ? x0 - px : (px > x1 ? px - x1 : 0u);
            const uint32_t dy = py < y0 ? y0 - py : (py > y1 ? py - y1 : 0u);
            return dx + dy;
          };
          // a thread's first KPT chunks (every chunk while kchunks <= KPT * block) are loaded once, all
          // loads in flight together, and kept in registers for phase B; any further chunks are re-read
          const uint32_t nch = P.kchunks;
          uint32_t kc[KPT];
          uint2 kb[KPT];
#pragma unroll
          for (uint32_t s = 0; s < KPT; ++s) {
            const uint32_t c = tid + s * bd;
            kc[s] = c < nch ? P.kcnt[c] : 0u;
            kb[s] = c < nch ? P.kbox[c] : make_uint2(0u, 0u);
          }
          auto ub_chunk = [&](uint32_t cnt, uint2 bx) {
            if (cnt == 0u) return;
            const uint32_t diam = ((bx.y & 0xFFFFu) - (bx.x & 0xFFFFu)) + ((bx.y >> 16) - (bx.x >> 16));
#pragma unroll
            for (uint32_t b = 0; b < ABATCH; ++b) {
              if (b >= B) break;  // block-uniform
              ub[b] = min(ub[b], box_lb(apos[b], bx.x, bx.y) + diam);
            }
          };
#pragma unroll
          for (uint32_t s = 0; s < KPT; ++s) ub_chunk(kc[s], kb[s]);
          for (uint32_t c = tid + KPT * bd; c < nch; c += bd) ub_chunk(P.kcnt[c], P.kbox[c]);
#pragma unroll
          for (uint32_t b = 0; b < ABATCH; ++b) {
            if (b >= B) break;
            const uint32_t wm = __ockl_wfred_min_u32(ub[b]);
            if (lane == 0) atomicMin(&s_ub[b], wm);
          }
          PBAR();
          uint32_t bdst[ABATCH], btsk[ABATCH];
#pragma unroll
          for (uint32_t b = 0; b < ABATCH; ++b) {
            ub[b] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b < B ? s_ub[b] : 0u));
            bdst[b] = 0xFFFFFFFFu;
            btsk[b] = 0xFFFFFFFFu;
          }
          auto scan_chunk = [&](uint32_t c, uint32_t cnt, uint2 bx) {
            if (cnt == 0u) return;
            uint32_t mask = 0;
#pragma unroll
            for (uint32_t b = 0; b < ABATCH; ++b)
              if (b < B && box_lb(apos[b], bx.x, bx.y) <= ub[b]) mask |= 1u << b;
            if (mask == 0u) return;
            const uint4* L4 = reinterpret_cast<const uint4*>(P.live + (size_t)c * KCH);
            const uint4* T4 = reinterpret_cast<const uint4*>(P.klt + (size_t)c * KCH);
#pragma unroll 1
            for (uint32_t h = 0; h < KCH / 16u; ++h) {  // 16 entries (4 vectors of each array) at a time
              uint4 xa[4], ta[4];
#pragma unroll
              for (uint32_t u = 0; u < 4u; ++u) {
                xa[u] = L4[4u * h + u];
                ta[u] = T4[4u * h + u];
              }
#pragma unroll
              for (uint32_t u = 0; u < 4u; ++u) {
                const uint32_t xs[4] = {xa[u].x, xa[u].y, xa[u].z, xa[u].w};
                const uint32_t ts[4] = {ta[u].x, ta[u].y, ta[u].z, ta[u].w};
#pragma unroll
                for (uint32_t e = 0; e < 4u; ++e) {
                  const uint32_t xy = xs[e], t = ts[e];
                  if (xy == TASK_TAKEN) continue;
                  const uint32_t tx = xy & 0xFFFFu, ty = xy >> 16;
#pragma unroll
                  for (uint32_t b = 0; b < ABATCH; ++b) {
                    if (b >= B) break;  // block-uniform
                    if (!((mask >> b) & 1u)) continue;
                    const uint32_t d = __usad(apos[b] & 0xFFFFu, tx, __usad(apos[b] >> 16, ty, 0u));
                    const bool lt = d < bdst[b] || (d == bdst[b] && t < btsk[b]);
                    bdst[b] = lt ? d : bdst[b];
                    btsk[b] = lt ? t : btsk[b];
                  }
                }
              }
            }
          };
#pragma unroll
          for (uint32_t s = 0; s < KPT; ++s) scan_chunk(tid + s * bd, kc[s], kb[s]);
          for (uint32_t c = tid + KPT * bd; c < nch; c += bd) scan_chunk(c, P.kcnt[c], P.kbox[c]);
#pragma unroll
          for (uint32_t b = 0; b < ABATCH; ++b) {
            if (b >= B) break;  // block-uniform
            const uint32_t dm = __ockl_wfred_min_u32(bdst[b]);
            const uint32_t tm = __ockl_wfred_min_u32(bdst[b] == dm ? btsk[b] : 0xFFFFFFFFu);
            if (lane == 0 && dm != 0xFFFFFFFFu)
              atomicMin(reinterpret_cast<unsigned long long*>(&s_bestk[b]), ((unsigned long long)dm << 32) | tm);
          }
          PBAR();
          PLAN_TICK(34);
          if (tid == 0) {
            uint32_t acc = 0, stop = 0;
            for (uint32_t b = 0; b < B; ++b) {
              if (list[kk + b] > bad_at || s_ctl.unused == 0u || s_bestk[b] == ~0ull) {
                stop = 1;  // past the first bad delivery / out of tasks: this step assigns no more
                break;
              }
              const uint32_t t = (uint32_t)(s_bestk[b] & 0xFFFFFFFFu);
              bool taken = false;
              for (uint32_t e = 0; e < acc; ++e) taken |= s_acct[e] == t;
              if (taken) break;  // conflict: this agent re-runs in the next batch
              s_acct[acc++] = t;
              s_ctl.unused -= 1u;
            }
            s_cnt2 = acc;
            s_doit = stop;
            s_nassign += acc;
            if (PLAN_DBG) {
              s_tick[37] += 1;    // batches
              s_tick[38] += acc;  // agents accepted
            }
          }
          PBAR();
          PLAN_TICK(35);
          const uint32_t acc = s_cnt2;
          if (tid < acc) {  // the accepted agents' updates in parallel (tswap.rs:132-136)
            const uint32_t ai = list[kk + tid], t = s_acct[tid];
            const uint32_t pos = P.kpos[t];  // the task's entry in the Morton order
            P.live[pos] = TASK_TAKEN;
            atomicSub(&P.kcnt[pos / KCH], 1u);
            P.task[ai] = (int32_t)t;
            P.st[ai] = ST_TO_PICKUP;
            if (P.pred) {  // diagnostics: was this the task last predicted for the agent?
              atomicAdd(&P.cc->pred_asg, 1u);
              const uint32_t pt = ld_agent(&P.pred[ai]);
              if (pt == t) atomicAdd(&P.cc->pred_hit, 1u);
              else if (pt == 0xFFFFFFFFu) atomicAdd(&P.cc->pred_none, 1u);
              __hip_atomic_store(&P.pred[ai], 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (PLAN_DBG) S.DEC[ai] = 0x40;
            DTAG(ai, 16u);
            const uint32_t ng = P.pick[t];
            if (ng == CELL_BAD) {  // pos2id[&task.pickup] panics (tswap.rs:136)
              atomicOr(&P.ctl->err, ERR_BAD_PICKUP);
              s_bad = 1;
            } else {
              S.G[ai] = ng;
              S.GT[ai] = P.goal_tab[ng];
              S.NHC[ai] = NHC_DIRTY;
              // the task's pickup -> delivery path goes to the workers now (hot chain), ahead of the
              // index-ordered walk of every task's chain: this one is about to be carried
              const uint32_t dc = P.dlv[t];
              if (P.QH && dc != CELL_BAD && dc != ng) {
                const int32_t dtab = P.goal_tab[dc];
                const uint32_t qi = atomicAdd(&s_q[6], 1u);
                if (dtab >= 0 && qi < P.qhcap) {
                  AstarQuery q;
                  q.v = ng;
                  q.goal = dc;
                  q.tab = dtab;
                  q.out = 0u;
                  P.QH[qi] = q;
                } else if (dtab < 0 && qi < P.qhcap) {
                  AstarQuery q;  // keep the slot well-formed: a chain without a table is skipped
                  q.v = ng;
                  q.goal = dc;
                  q.tab = -1;
                  q.out = 0u;
                  P.QH[qi] = q;
                }
              }
            }
          }
          PBAR();
          PLAN_TICK(36);
          if (s_doit) break;  // block-uniform
          kk += acc;
          bcur = (kab & 4u) ? 1u : acc == B ? min(ABATCH, 2u * bcur) : max(acc, 1u);
        }
        if (bad_at != NO_AGENT && !s_bad) {  // block-uniform
          if (tid == 0) {
            atomicOr(&P.ctl->err, ERR_BAD_DELIVERY);
            s_bad = 1;
          }
          PBAR();
        }
      }
      if (P.t0_delay_ticks && s_ctl.t == 0u && tid == 0) {  // diagnostic A/B: workers get a head start
        const unsigned long long w0 = wall_clock64();
        while (wall_clock64() - w0 < P.t0_delay_ticks) __builtin_amdgcn_s_sleep(64);
      }
      if (s_bad) {  // block-uniform: stop with the error bit set, no record for this timestep
        if (tid == 0) {
          s_ctl.status = PLAN_ERROR;
          s_exit = 1;
        }
        PBAR();
        break;
      }
      if (tid == 0) {
        s_ctl.section = SEC_PRE1;
        s_ctl.i = 0;
      }
      PBAR();
    } else if (sec == SEC_PRE1 || sec == SEC_PRE2) {
      if (sec == SEC_PRE1 && tid == 0) {
        // walk-ahead depth (coop): wide_hi (32) hops on grids up to 2^18 cells while the workers keep up
        // with the speculative queue (wide_prefetch, 8, when it backs up), wide_lo (8) on larger grids,
        // where every hop is a miss into a 1 MB-stride code store. Round 4 set 16 / 4 on the frozen
        // instances; round 5 re-measured on the busy ones (profiles/r5/retune_busy_ab.txt, the walk now
        // resumes at its cached frontier): C3 0.98 -> 0.95 s, wh10k 11.66 -> 11.1-11.3 s at 32 hops
        // (48: C3 slower), C5 7.74 -> 7.42 s at 8 hops (12 and 16 slower)
        uint32_t h = P.wide_prefetch ? P.wide_prefetch : 1u;
        if (P.coop && P.wide_prefetch && P.spec_hi) {
          if (P.ncell > (1u << 18)) {
            h = P.wide_lo;
          } else {
            const uint32_t hs = min(s_q[1], P.qscap), cs = ld_agent(&P.cc->claim_s);
            h = (hs > cs ? hs - cs : 0u) <= P.spec_hi ? P.wide_hi : h;
          }
        }
        s_hops = h;
      }
      const uint32_t q = refresh_codes(P, S, s_q, &s_need, s_ctl.section);
      if (PLAN_DBG && P.dtag && P.coop && sec == SEC_PRE1) {  // diagnostics: unresolved PRE1 pairs by agent tag
        for (uint32_t k = tid; k < n; k += bd) {
          const uint32_t tg = P.dtag[k] & 63u;
          P.dtag[k] = 0u;
          if (S.NHC[k] <= NH_STAY || S.V[k] == S.G[k] || S.GT[k] < 0) continue;
          const uint8_t c = nh_code_k(S.GT[k], S.V[k]);
          if (c == NH_UNKNOWN || c == NH_PENDING) atomicAdd(&P.cc->dbg_tag[0][tg], 1u);
          else if (c == NH_PENDING_S) atomicAdd(&P.cc->dbg_tag[1][tg], 1u);
        }
      }
      // the pairs this step waits for go to the workers before the walk-ahead prefetch below: it
      // reads up to 8 codes per agent in dependent global loads, and publishing only after it held
      // every needed pair back ~40-60 us (round 4: the workers' enqueue -> claim delay)
      if (P.coop && q > 0 && sec == SEC_PRE1 && P.prefetch && tid == 0) coop_publish_needed(P, s_q);
      // step start: queue every agent's next hop from the cell it is about to enter now, so
      // the assignment exit's K3 batch (if any) already carries what the movement phase reads
      if (sec == SEC_PRE1 && P.prefetch) nextnext_prefetch(P, S, s_q, s_hops);
      if (P.coop && tid == 0) {  // speculative pairs start resolving now
        const unsigned long long t0 = PLAN_DBG ? wall_clock64() : 0ull;
        coop_publish(P, s_q);
        if (PLAN_DBG) {
          s_tick[24] += wall_clock64() - t0;
          s_tick[25] += 1;
        }
      }
      // diagnostics: PRE1 waits by timestep bucket (t < 50, < 150, < 400, < 1000, later)
      const uint32_t tt = s_ctl.t;
      const uint32_t wkind = sec == SEC_PRE1 ? (tt < 50 ? 1u : tt < 150 ? 2u : tt < 400 ? 3u : tt < 1000 ? 4u : 5u) : 0u;
      if (q > 0 && !coop_resolve(P, S, s_q, &s_need, &s_flag, s_ctl.section | (wkind << 8))) {
        if (tid == 0) {
          s_ctl.qcount = s_q[0];
          s_ctl.status = PLAN_NEED_QUERIES;
          s_exit = 1;
        }
        PBAR();
        break;
      }
      if (tid == 0) {
        s_ctl.section = sec == SEC_PRE1 ? SEC_RULES : SEC_MOVE;
        s_ctl.i = 0;
      }
      PBAR();
    } else if (sec == SEC_RULES) {
      // ---- rules phase as "first firing agent" rounds (see header) ------------
      // Cycle labels ONC (k lies on a cycle of succ) come from pointer doubling once per
      // phase and after rotations; a rule-3 swap (b, s) is folded in incrementally: b's
      // new goal is the adjacent cell it already targets (same next hop, same succ), and
      // s — terminal until now — gains one out-edge, so the only new cycle possible is
      // one through s. CANDC[k] prefetches s's next hop toward k's goal for every rule-3
      // candidate k, so a swap needs no global round trip on the serial path.
      if (PLAN_DBG && tid == 0) s_tp = wall_clock64();
      const bool fuse_pf = P.prefetch && P.wide_prefetch;  // rules_prefetch inside the first pass
      rules_init(P, S, fuse_pf ? s_q : nullptr);
      if (tid == 0) s_ctl.relabel_full += 1;
      if (PLAN_DBG && tid == 0) {
        const unsigned long long nw = wall_clock64();
        s_tick[26] += nw - s_tp;
        s_tp = nw;
      }
      if (P.prefetch && !fuse_pf) rules_prefetch(P, S, s_q);
      if (PLAN_DBG && tid == 0) {
        const unsigned long long nw = wall_clock64();
        s_tick[27] += nw - s_tp;
        s_tp = nw;
      }
      if (P.coop && tid == 0) {
        coop_publish(P, s_q);
        if (PLAN_DBG) {
          s_tick[28] += wall_clock64() - s_tp;
          s_tick[29] += 1;
        }
      }
      if (tid == 0) s_cnt = 0;
      PLAN_TICK(15);
      // One firing agent per round (tswap.rs:180-252 in agent order): fire(b) applies b's rule 3
      // swap or rule 4 rotation (tid 0 only) and sets s_miss when next hops must be refreshed.
      // agents whose goals changed since the last prefetch, in `list` (s_cnt; NO_AGENT = overflow,
      // the next relabel prefetches for everyone)
      auto note_changed = [&](uint32_t a) {
        if (s_cnt < LIST_CAP) list[s_cnt++] = a;
        else s_cnt = NO_AGENT;
      };
      // fire(b) returns what the wave-0 rounds need to update their per-lane firing flags
      // without re-reading LDS: FO_MISS (codes must be refreshed), FO_RESCAN (a new cycle or a
      // shared-start goal changed labels: rescan from the cursor), else a rule-3 swap (b, s)
      // whose only effects on the firing predicate of other agents are s's new successor `ns`
      // (firing flag `fs`) and the new at-goal status of b (`b_at`) and s (`s_at`).
      struct FireOut {
        uint32_t s, ns, flags;
        bool fs, b_at, s_at;
      };
      // FO_ROT: a rule-4 rotation of o.ns members (listed in S.F2) whose next hops are dirty
      // FO_WAVE (with FO_ROT): the wave rotated the cycle itself, members in s_ap
      constexpr uint32_t FO_MISS = 1u, FO_RESCAN = 2u, FO_ROT = 4u, FO_WAVE = 8u;
      auto fire = [&](uint32_t b) -> FireOut {
        FireOut o;
        o.flags = 0;
        o.fs = o.b_at = o.s_at = false;
        o.ns = SUCC_TERM;
        const uint32_t s = S.SUCC[b];
        o.s = s;
        // every load of the swap up front (independent LDS reads, one round trip)
        const uint32_t vs = S.V[s], gs = S.G[s], vb = S.V[b], gb = S.G[b];
        const int32_t tb = S.GT[b], ts = S.GT[s];
        const uint32_t candc = S.CANDC[b];
        if (vs == gs) {  // rule 3: goal swap (tswap.rs:198-202)
          DTAG(b, 1u);
          DTAG(s, 2u);
          uint32_t code = candc;
          if (code > NH_STAY && tb >= 0) code = nh_code_k(tb, vs);  // s's new goal is gb
          S.G[b] = gs;
          S.GT[b] = ts;
          S.G[s] = gb;
          S.GT[s] = tb;
          S.CANDC[s] = NHC_DIRTY;
          S.CANDC[b] = NHC_DIRTY;  // b's goal changed (a later rotation through b must not use it)
          o.b_at = vb == gs;
          o.s_at = vs == gb;
          if (o.b_at) {  // shared start cell: b now at its goal
            S.SUCC[b] = SUCC_TERM;
            o.flags |= FO_RESCAN;
          }
          if (code <= NH_STAY) {
            S.NHC[s] = (uint8_t)code;
            // succ_of(s) with the values already in registers
            uint32_t ns = SUCC_TERM;
            if (vs != gb) {
              const uint32_t oc = S.OCC[step_cell(vs, code, P.W)];
              ns = oc == OCC_NONE ? SUCC_TERM : (oc & OCC_IDX);
            }
            S.SUCC[s] = ns;
            o.ns = ns;
            if (ns != SUCC_TERM && ns != s) {
              // new cycle through s?
              uint32_t x = ns;
              uint32_t it = 0;
              // a labelled agent lies on a standing cycle, which cannot contain s (terminal until
              // now), and a self-loop is a chain end: neither leads back to s
              for (; it < n && x != SUCC_TERM && x != s; ++it) {
                const uint32_t nx = S.SUCC[x];
                if (S.ONC[x] || nx == x) {
                  x = SUCC_TERM;
                  break;
                }
                x = nx;
              }
              if (PLAN_DBG) s_tick[9] += it;  // diagnostics: rule-3 cycle-walk hops
              if (x == s) {
                uint32_t y = s;
                do {
                  S.ONC[y] = 1;
                  y = S.SUCC[y];
                } while (y != s);
                o.flags |= FO_RESCAN;
              } else {
                o.fs = S.V[ns] == S.G[ns];  // s fires rule 3 next (ONC[s] is 0: s was terminal)
              }
            }
          } else {
            S.NHC[s] = NHC_DIRTY;  // unresolved: refresh + full relabel below
            s_miss = 1;
            o.flags |= FO_MISS;
          }
          note_changed(b);  // goals of b and s changed (targeted prefetch after the next relabel)
          note_changed(s);
        } else {  // rule 4: rotate targets along the cycle b -> s -> ... -> last -> b
          uint32_t L = 0;
          // cycle members in S.F2 (free until the rules_init this rotation triggers; LDS when
          // the agent arrays are): the walk below re-reads them serially
          uint32_t* ap = S.F2;
          for (uint32_t a = b; L == 0 || a != b; a = S.SUCC[a]) ap[L++] = a;
          const uint32_t last = ap[L - 1];
          const uint32_t last_goal = S.G[last];
          const int32_t last_tab = S.GT[last];
          for (uint32_t kk = L - 1; kk >= 1; --kk) {
            const uint32_t a = ap[kk], pa = ap[kk - 1];
            S.G[a] = S.G[pa];
            S.GT[a] = S.GT[pa];
            S.NHC[a] = NHC_DIRTY;
          }
          S.G[b] = last_goal;
          S.GT[b] = last_tab;
          S.NHC[b] = NHC_DIRTY;
          // members' next hops changed: the wave rounds settle them in place (rot_settle), the
          // block rounds refresh + relabel below
          o.flags |= FO_ROT;
          o.ns = L;
          for (uint32_t kk = 0; kk < L; ++kk) {
            note_changed(ap[kk]);
            DTAG(ap[kk], 4u);
          }
          if (PLAN_DBG) s_tick[11] += 1;  // diagnostics: rule-4 rotations
        }
        s_ctl.i = b + 1;
        s_ctl.rule_rounds += 1;
        return o;
      };
      // n <= 512: wave 0 alone runs scan + fire rounds back to back — the scan is a ballot over
      // 64 agents from the cursor, the fire is lane 0 of the same wave, so a round needs no
      // workgroup barrier and no cross-wave reduction; the block joins only when a firing
      // changed next hops (refresh + relabel) or the phase ends.
      // Wave 0, after a rotation of L members (S.F2): every member's next hop for its new goal
      // (lanes in parallel, from CANDC of its predecessor when current), then an incremental
      // relabel from the members (lane 0; the labels were exact before the rotation and only the
      // members' successors changed). False (block path: refresh, wait, relabel) if a code is
      // unresolved or a walk runs long.
      auto rot_settle = [&](uint32_t L, const uint32_t* ap) -> bool {
        bool bad = false;
        for (uint32_t i = lane; i < L; i += 64u) {
          const uint32_t a = ap[i];
          if (S.V[a] == S.G[a]) continue;
          // a took the goal of its predecessor pa on the cycle and sits at succ(pa)'s cell: the code
          // is CANDC[pa] when that is still current, else a table read
          const uint32_t pa = ap[i == 0u ? L - 1u : i - 1u];
          uint8_t code = S.CANDC[pa];
          if (code > NH_STAY) {
            const int32_t tab = S.GT[a];
            code = tab >= 0 ? nh_code_k(tab, S.V[a]) : NH_UNKNOWN;
          }
          if (code <= NH_STAY) S.NHC[a] = code;
          else bad = true;
        }
        if (__ballot(bad)) return false;
        uint32_t ok = 0;
        if constexpr (AG || PG) {
          if (L <= 64u) {
            // Agent arrays in LDS, L <= 64: the relabel walks of all members run at once, one lane each.
            // Only the members' successors changed, so a new cycle passes through a member, no member
            // lies on a standing (labelled) cycle (they formed the rotated one), and a walk from a member
            // ends at TERM / a self-loop / a labelled node (no cycle) or at a member (marked ONC = 2 + its
            // index): the members' "next member" links then form a graph of <= 64 nodes whose cycles are
            // exactly the new cycles; their members label them. Same labels as relabel_walks.
            wave_order();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the code stores above are visible
            const unsigned long long rt0 = PLAN_DBG ? clock64() : 0ull;
            uint8_t cc = NHC_DIRTY;
            uint32_t a = 0;
            const bool mem = lane < L;
            if (mem) {
              a = ap[lane];
              const uint32_t sa = succ_of(P, S, a);
              S.SUCC[a] = sa;
              S.ONC[a] = (uint8_t)(2u + lane);
              const int32_t ta = S.GT[a];
              if (sa != SUCC_TERM && sa != a && ta >= 0) cc = knh[(uint64_t)ta * kns + S.V[sa]];
            }
            wave_order();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            const unsigned long long rt1 = PLAN_DBG ? clock64() : 0ull;
            uint32_t nm = 64u;  // next member's index (64: the walk ended without one)
            bool fail = false;
            if (mem) {
              uint32_t x = S.SUCC[a];
              for (uint32_t steps = 0; x != SUCC_TERM; ++steps) {
                const uint32_t o = S.ONC[x], nx = S.SUCC[x];
                if (o >= 2u) {
                  nm = o - 2u;
                  break;
                }
                if (o != 0u || nx == x) break;  // labelled standing cycle / chain end
                if (steps >= 4096u) {
                  fail = true;
                  break;
                }
                x = nx;
              }
            }
            if (mem) s_ap[64u + lane] = nm;  // (s_ap holds 128 entries: members, then next-member links)
            wave_order();
            __builtin_amdgcn_s_waitcnt(0xC07F);
            bool on = false;
            if (mem) {
              uint32_t y = nm;
              for (uint32_t t = 0; t < L && y < 64u && !on; ++t) {
                on = y == lane;
                y = s_ap[64u + y];
              }
            }
            wave_order();
            if (mem && !on) S.ONC[a] = 0;
            wave_order();
            if (on) {  // label the cycle through a (members and the non-members between them)
              uint32_t y = a;
              do {
                S.ONC[y] = 1;
                y = S.SUCC[y];
              } while (y != a);
            }
            if (mem) S.CANDC[a] = cc;
            wave_order();
            ok = __ballot(fail) ? 0u : 1u;
            if (PLAN_DBG && lane == 0) {  // diagnostics: rotation settle split (successors | walks)
              const unsigned long long rt2 = clock64();
              s_tick[30] += rt1 - rt0;
              s_tick[31] += rt2 - rt1;
            }
          }
        }
        if (!(AG || PG) || L > 64u) {
          __threadfence_block();
          for (uint32_t i = lane; i < L; i += 64u) relabel_reset(P, S, ap[i]);  // lanes in parallel
          __threadfence_block();
          if (lane == 0) ok = relabel_walks(P, S, ap, L, 4096u) ? 1u : 0u;
        }
        if (!__builtin_amdgcn_readfirstlane(ok)) return false;
        if (lane == 0) s_ctl.relabel_inc += 1;
        __threadfence_block();
        // (no prefetch here: the members' next hops are set, and the next step's walk-ahead
        // prefetch covers their paths; a publish costs an L2 write-back)
        return true;
      };
      const bool wave_scan = n <= P.wave_rules_max;
      for (;;) {
        if (wave_scan) {
          if (wid == 0) {
            // Per-lane state of the chunk [base, base+64): successor sk, ONC bit, firing flag f.
            // A rule-3 swap (b, s) changes the firing predicate of other agents only through
            // s's successor and the at-goal status of b and s: the flags are updated in place
            // and the next firing agent is the next set bit of the ballot — no LDS re-scan and
            // no cursor round trip per round.
            // Each candidate lane also precomputes its own swap (s's cell / goal / slot, the code of
            // s's new next hop, s's new successor ns and whether ns sits at its goal), all lanes at
            // once, so the common firing — a rule-3 swap whose code is resolved — is a handful of
            // stores by the firing lane with nothing to wait for. A firing invalidates the
            // precomputation of every lane it touches (k, its successor or its ns among b, s);
            // stale lanes redo it when one of them is next. Anything else (rule 4, a missing code,
            // a shared start cell) takes fire().
            __threadfence_block();
            uint32_t base = *(volatile uint32_t*)&s_ctl.i;
            uint32_t nc = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&s_cnt);  // changed-list length
            uint32_t rr = 0;                                                          // fast firings
            bool loaded = false;
            uint32_t sk = SUCC_TERM;
            bool f = false, onck = false;
            uint64_t m = 0;
            bool pv = false;  // precomputed swap valid
            uint32_t p_vs = 0, p_gs = 0, p_gk = 0, p_ns = SUCC_TERM, p_nk = SUCC_TERM;
            int32_t p_ts = -1, p_tk = -1;
            // bits 0-7: s's new next-hop code; rule-4 2-cycle: bits 8-15 k's new code, bit 16 set
            uint32_t p_code = NH_UNKNOWN;
            bool p_fsv = false, p_walk = false;
            auto precompute = [&](bool want) {
              if (!want) return;
              const uint32_t k = base + lane;
              p_vs = S.V[sk];
              p_gs = S.G[sk];
              p_ts = S.GT[sk];
              p_gk = S.G[k];
              p_tk = S.GT[k];
              const uint32_t vk = S.V[k];
              uint32_t code = S.CANDC[k];
              const bool r3 = p_vs == p_gs;
              // rule 4 on a 2-cycle k <-> s (two agents meeting head on, the common firing in 1-wide aisles):
              // the rotation (tswap.rs:241-249) is the exchange of their goals, and each one's new next hop is
              // the other's CANDC — the code of (the cell it sits on, the goal it takes)
              const bool r2 = !r3 && onck && !(kab & 1u) && S.SUCC[sk] == k;
              bool ok = (r3 && vk != p_gs) || r2;  // rule 3 without a shared start cell, or the 2-cycle
              if (ok && code > NH_STAY) code = p_tk >= 0 ? nh_code_k(p_tk, p_vs) : NH_UNKNOWN;
              ok = ok && code <= NH_STAY;
              uint32_t code2 = 0, nk = SUCC_TERM;
              if (ok && r2) {
                code2 = S.CANDC[sk];
                if (code2 > NH_STAY) code2 = p_ts >= 0 ? nh_code_k(p_ts, vk) : NH_UNKNOWN;
                ok = code2 <= NH_STAY;
                if (ok && vk != p_gs) {  // k's new successor (k takes s's goal; at it when vk == p_gs)
                  const uint32_t oc = S.OCC[step_cell(vk, code2, W)];
                  nk = oc == OCC_NONE ? SUCC_TERM : (oc & OCC_IDX);
                }
              }
              p_code = code | (code2 << 8) | (r2 ? 0x10000u : 0u);
              p_nk = nk;
              uint32_t ns = SUCC_TERM;
              if (ok && p_vs != p_gk) {
                const uint32_t oc = S.OCC[step_cell(p_vs, code, W)];
                ns = oc == OCC_NONE ? SUCC_TERM : (oc & OCC_IDX);
              }
              p_ns = ns;
              p_fsv = ok && ns != SUCC_TERM && ns != sk && S.V[ns] == S.G[ns];
              // s's new successor moves: cycle check; a 2-cycle rotation always walks (never batched)
              p_walk = ok && (r2 || (ns != SUCC_TERM && ns != sk && !p_fsv));
              pv = ok;
            };
            // diagnostics (TSW_PLAN_DEBUG): shader cycles per part of the loop -> s_tick[16..23]
            unsigned long long pt = PLAN_DBG ? clock64() : 0ull;
            auto prof = [&](int slot) {
              if (PLAN_DBG) {
                const unsigned long long nw = clock64();
                if (lane == 0) s_tick[slot] += nw - pt;
                pt = nw;
              }
            };
            for (uint32_t spin = 1;; ++spin) {
              if ((spin & 1023u) == 0u &&
                  (uint32_t)__builtin_amdgcn_readfirstlane(lane == 0 ? (plan_abort(P) ? 1u : 0u) : 0u)) {
                if (lane == 0) {
                  s_abort = 1;
                  s_best = NO_AGENT;
                }
                break;
              }
              if (!loaded) {
                if (base >= n) {
                  if (lane == 0) {
                    s_best = NO_AGENT;
                    s_ctl.i = n;
                  }
                  break;
                }
                const uint32_t k = base + lane;
                f = false;
                onck = false;
                sk = SUCC_TERM;
                pv = false;
                if (k < n) {
                  sk = S.SUCC[k];
                  onck = S.ONC[k] != 0;
                  f = sk != SUCC_TERM && sk != k && (S.V[sk] == S.G[sk] || onck);
                }
                m = __ballot(f);
                precompute(f);
                loaded = true;
                if (PLAN_DBG && lane == 0) s_tick[22] += 1;
                prof(16);
              }
              if (!m) {
                base += 64u;
                loaded = false;
                continue;
              }
              const uint32_t l = (uint32_t)__builtin_ctzll(m);
              const uint32_t b = base + l;
              // the next firing lane's precomputation is stale: redo it for every stale candidate
              if (!__builtin_amdgcn_readlane((int)(pv ? 1u : 0u), (int)l)) precompute(f && !pv);
              prof(17);
              const bool walk_batch = !(kab & 8u);  // A/B (diagnostic build): walking firings one at a time
              if (AG && __builtin_amdgcn_readlane((int)(pv && (walk_batch || !p_walk) ? 1u : 0u), (int)l)) {
                // ---- batch (agent arrays in LDS): the longest run of firing lanes from l whose firings cannot see
                // each other — rule-3 swaps and 2-cycle rotations (97 % of busy C3's firings) with their
                // precomputation current. Firing lanes mark the agents they write (b = k, s = sk) with their
                // lane (LDS min). A lane whose own agent, successor or precomputed ns carries an earlier
                // lane's mark reads state that earlier firing changes; the batch ends before the first
                // such lane (firing or not: a non-firing s may start firing) and before the first firing
                // lane that is not a plain precomputed one. A firing that moves a successor (s's, and b's
                // in a rotation) must not close a new cycle (its labels would change other agents'
                // firing): every such lane walks its new successor chains at once, on the state before
                // the batch plus its own change, as the serial path below does after its firing; a walk
                // that closes a cycle, runs past P.walk_cap hops or passes an agent an earlier lane marked
                // ends the batch at that lane. The firings of the batch then touch disjoint agents and
                // read nothing another one writes, so applying them at once equals applying them in
                // agent order (tswap.rs:180-252). Lanes past the batch that it touched reload.
                const uint32_t k = base + lane;
                const bool fire_l = ((m >> lane) & 1ull) != 0ull;  // m holds lanes >= l only
                const bool cand = fire_l && pv && (walk_batch || !p_walk);
                const bool r2 = cand && (p_code >> 16) != 0u;
                if (cand) {
                  atomicMin(&S.MK[k], lane);
                  atomicMin(&S.MK[sk], lane);
                }
                __threadfence_block();
                uint32_t c = 0xFFFFFFFFu;
                if (k < n) {
                  c = S.MK[k];
                  if (sk != SUCC_TERM) c = min(c, S.MK[sk]);
                  if (pv && p_ns != SUCC_TERM) c = min(c, S.MK[p_ns]);
                }
                prof(40);
                bool simple = cand;
                uint32_t cw = c;  // with the marks met on the walks
                uint32_t hops = 0;  // diagnostics
                if (cand && p_walk) {
                  // walk from st along the successors after this lane's firing (o = the other agent whose
                  // successor it changes, a rotation's b; its ONC label is cleared with the 2-cycle): 0 no
                  // new cycle (TERM, a self-loop or a labelled agent ends the chain), 1 a cycle or too long
                  auto walk = [&](uint32_t st, uint32_t first, uint32_t o, uint32_t o_next) -> uint32_t {
                    if (first == SUCC_TERM || first == st) return 0u;
                    uint32_t x = first;
                    for (uint32_t it = 0; it < kwcap; ++it) {
                      if (x == SUCC_TERM) return 0u;
                      if (x == st) return 1u;
                      cw = min(cw, S.MK[x]);
                      ++hops;
                      uint32_t nx;
                      bool lab;
                      if (x == o) {
                        nx = o_next;
                        lab = false;
                      } else {
                        nx = S.SUCC[x];
                        lab = S.ONC[x] != 0;
                      }
                      if (lab || nx == x) return 0u;
                      x = nx;
                    }
                    return 1u;
                  };
                  // rule 3: s was at its goal (terminal, unlabelled) and b keeps its successor s
                  uint32_t bad = walk(sk, p_ns, r2 ? k : SUCC_TERM, p_nk);
                  if (!bad && r2) bad = walk(k, p_nk, sk, p_ns);
                  simple = !bad;
                }
                if (PLAN_DBG) {  // diagnostics: batches, longest walk of each
                  const uint32_t mh = ~wave_min_u32(~hops);
                  if (lane == 0) {
                    s_tick[43] += 1;
                    s_tick[44] += mh;
                  }
                }
                prof(41);
                const uint64_t bm = __ballot(lane >= l && (cw < lane || (fire_l && !simple)));
                const uint32_t cut = bm ? (uint32_t)__builtin_ctzll(bm) : 64u;
                const uint64_t batch = cut >= 64u ? m : (m & ((1ull << cut) - 1ull));
                const bool inb = ((batch >> lane) & 1ull) != 0ull;
                if (inb) {  // rule 3 (tswap.rs:198-202): b <-> s goals, s's new code and successor
                  DTAG(k, r2 ? 4u : 1u);
                  DTAG(sk, r2 ? 4u : 2u);
                  S.G[k] = p_gs;
                  S.GT[k] = p_ts;
                  S.G[sk] = p_gk;
                  S.GT[sk] = p_tk;
                  S.CANDC[sk] = NHC_DIRTY;
                  S.CANDC[k] = NHC_DIRTY;
                  S.NHC[sk] = (uint8_t)p_code;
                  S.SUCC[sk] = p_ns;
                  if (r2) {  // rule 4 on the 2-cycle (:241-249): the same exchange, b's new code and successor
                    S.NHC[k] = (uint8_t)(p_code >> 8);
                    S.SUCC[k] = p_nk;
                    S.ONC[k] = 0;
                    S.ONC[sk] = 0;
                  }
                }
                const bool touched = lane >= cut && c < cut;
                __threadfence_block();
                if (cand) {
                  S.MK[k] = 0xFFFFFFFFu;
                  S.MK[sk] = 0xFFFFFFFFu;
                }
                __threadfence_block();
                prof(42);
                // an empty batch (lane l's own walk closed a cycle or ran long): lane l fires on the serial path
                if (batch != 0ull) {
                  if (PLAN_DBG && lane == 0) s_tick[11] += (uint32_t)__popcll(__ballot(inb && r2));  // rule-4 rotations
                  if (touched && k < n) {  // exact state after the batch, from LDS
                    sk = S.SUCC[k];
                    onck = S.ONC[k] != 0;
                    f = sk != SUCC_TERM && sk != k && (S.V[sk] == S.G[sk] || onck);
                    pv = false;
                  }
                  // b and s of every swap join the changed list (targeted prefetch at the next relabel)
                  const uint32_t nb = (uint32_t)__popcll(batch);
                  if (nc != NO_AGENT && nc + 2u * nb <= LIST_CAP) {
                    if (inb) {
                      const uint32_t r = lane_rank(batch);
                      list[nc + 2u * r] = k;
                      list[nc + 2u * r + 1u] = sk;
                    }
                    nc += 2u * nb;
                  } else {
                    nc = NO_AGENT;
                  }
                  rr += nb;
                  const uint32_t last = 63u - (uint32_t)__builtin_clzll(batch);
                  if (lane == last) {
                    s_best = k;
                    s_miss = 0;
                    s_ctl.i = k + 1u;
                  }
                  m = last == 63u ? 0ull : (__ballot(f) & ~((2ull << last) - 1ull));
                  if (PLAN_DBG && lane == 0) s_tick[23] += nb;
                  prof(18);
                  continue;
                }
              }
              uint32_t r_fl = 0, r_s = 0, r_ns = 0, r_bits = 0;
              const bool fast = __builtin_amdgcn_readlane((int)(pv ? 1u : 0u), (int)l) != 0;
              if (fast) {
                // rule 3 (tswap.rs:198-202) from registers: b <-> s goals, s's new code and successor;
                // a rule-4 rotation of the 2-cycle b <-> s (:241-249) is the same exchange plus b's new
                // code and successor, and both leave the broken cycle
                if (lane == l) {
                  const uint32_t s = sk;
                  const bool r2 = (p_code >> 16) != 0u;
                  S.G[b] = p_gs;
                  S.GT[b] = p_ts;
                  S.G[s] = p_gk;
                  S.GT[s] = p_tk;
                  S.CANDC[s] = NHC_DIRTY;
                  S.CANDC[b] = NHC_DIRTY;
                  S.NHC[s] = (uint8_t)p_code;
                  S.SUCC[s] = p_ns;
                  DTAG(b, r2 ? 4u : 1u);
                  DTAG(s, r2 ? 4u : 2u);
                  if (r2) {
                    S.NHC[b] = (uint8_t)(p_code >> 8);
                    S.SUCC[b] = p_nk;
                    S.ONC[b] = 0;
                    S.ONC[s] = 0;
                    if (PLAN_DBG) s_tick[11] += 1;  // diagnostics: rule-4 rotations
                  }
                  s_best = b;
                  s_miss = 0;
                  s_ctl.i = b + 1;
                  bool fs = p_fsv;
                  // new cycles pass through an agent whose successor changed: s (both firings) and b
                  // (rotation). A labelled agent lies on a standing cycle that contains neither, and a
                  // self-loop is a chain end: neither leads back.
                  const uint32_t starts[2] = {s, b};
                  for (uint32_t w = 0; w < (r2 ? 2u : 1u); ++w) {
                    const uint32_t st = starts[w];
                    const uint32_t first = S.SUCC[st];
                    if (S.ONC[st] || first == SUCC_TERM || first == st || (w == 0u && !r2 && p_fsv)) continue;
                    uint32_t x = first;
                    uint32_t it = 0;
                    for (; it < n && x != SUCC_TERM && x != st; ++it) {
                      const uint32_t nx = S.SUCC[x];
                      if (S.ONC[x] || nx == x) {
                        x = SUCC_TERM;
                        break;
                      }
                      x = nx;
                    }
                    if (PLAN_DBG) s_tick[9] += it;
                    if (x == st) {
                      uint32_t y = st;
                      do {
                        S.ONC[y] = 1;
                        y = S.SUCC[y];
                      } while (y != st);
                      r_fl = FO_RESCAN;
                    }
                  }
                  if (r_fl) fs = false;
                  r_s = s;
                  r_ns = p_ns;
                  r_bits = (fs ? 1u : 0u) | (r2 && S.V[b] == p_gs ? 2u : 0u) | (p_vs == p_gk ? 4u : 0u);
                }
                // b and s joined the changed list (targeted prefetch at the phase end / next relabel)
                const uint32_t fsx = (uint32_t)__builtin_amdgcn_readlane((int)r_s, (int)l);
                if (nc != NO_AGENT && nc + 2u <= LIST_CAP) {
                  if (lane == 0) {
                    list[nc] = b;
                    list[nc + 1u] = fsx;
                  }
                  nc += 2u;
                } else {
                  nc = NO_AGENT;
                }
                ++rr;
                prof(18);
              } else {
                // rule 4 (tswap.rs:205-249) with the agent arrays in LDS: lane 0 lists the cycle's
                // members (<= 64), then every member's lane rotates its goal at once — the serial
                // rotation of fire() reads and writes the members one after another, and with the goal
                // slots GT in global memory that was one memory latency per member
                bool wave_rot = false;
                if constexpr (AG || PG) {
                  const uint32_t s4 = (uint32_t)__builtin_amdgcn_readlane((int)sk, (int)l);
                  if (S.V[s4] != S.G[s4]) {
                    uint32_t L = 0;
                    if (lane == 0) {
                      uint32_t a = b;
                      do {
                        if (L < 64u) s_ap[L] = a;
                        ++L;
                        a = S.SUCC[a];
                      } while (a != b && L <= 64u);
                    }
                    L = (uint32_t)__builtin_amdgcn_readfirstlane((int)L);
                    wave_order();
                    if (L <= 64u) {
                      wave_rot = true;
                      uint32_t a = 0, ng = 0;
                      int32_t nt = 0;
                      if (lane < L) {  // a takes the goal of its predecessor on the cycle (last -> b)
                        a = s_ap[lane];
                        const uint32_t pa = s_ap[lane == 0u ? L - 1u : lane - 1u];
                        ng = S.G[pa];
                        nt = S.GT[pa];
                      }
                      wave_order();
                      __threadfence_block();
                      if (lane < L) {
                        S.G[a] = ng;
                        S.GT[a] = nt;
                        S.NHC[a] = NHC_DIRTY;
                        DTAG(a, 4u);
                      }
                      if (nc != NO_AGENT && nc + L <= LIST_CAP) {
                        if (lane < L) list[nc + lane] = a;
                        nc += L;
                      } else {
                        nc = NO_AGENT;
                      }
                      if (lane == 0) {
                        s_best = b;
                        s_miss = 0;
                        s_ctl.i = b + 1;
                        s_ctl.rule_rounds += 1;
                        if (PLAN_DBG) s_tick[11] += 1;  // diagnostics: rule-4 rotations
                      }
                      r_fl = FO_ROT | FO_WAVE;
                      r_ns = L;
                      __threadfence_block();
                    }
                  }
                }
                if (!wave_rot) {
                  if (lane == 0) s_cnt = nc;
                  __threadfence_block();
                  if (lane == l) {
                    s_best = b;
                    s_miss = 0;
                    const FireOut r = fire(b);
                    r_fl = r.flags;
                    r_s = r.s;
                    r_ns = r.ns;
                    r_bits = (r.fs ? 1u : 0u) | (r.b_at ? 2u : 0u) | (r.s_at ? 4u : 0u);
                  }
                  __threadfence_block();
                  nc = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&s_cnt);
                }
                prof(20);
              }
              __threadfence_block();
              const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)r_fl, (int)l);
              if (fl & FO_MISS) break;
              if (fl & FO_ROT) {
                // settle the rotation inside the wave when every member's new next hop is already
                // resolved (the rules prefetch queued them): rescan from b + 1 without a block join
                const bool settled = rot_settle((uint32_t)__builtin_amdgcn_readlane((int)r_ns, (int)l),
                                                 (fl & FO_WAVE) ? s_ap : S.F2);
                prof(21);
                if (settled) {
                  base = b + 1u;
                  loaded = false;
                  continue;
                }
                if (lane == 0) s_miss = 1;
                break;
              }
              if (fl & FO_RESCAN) {
                base = b + 1u;
                loaded = false;
                continue;
              }
              const uint32_t fs_ = (uint32_t)__builtin_amdgcn_readlane((int)r_s, (int)l);
              const uint32_t fns = (uint32_t)__builtin_amdgcn_readlane((int)r_ns, (int)l);
              const uint32_t fbits = (uint32_t)__builtin_amdgcn_readlane((int)r_bits, (int)l);
              const uint32_t k = base + lane;
              // precomputations that read b or s (own goal, successor's cell/goal, ns's goal) are stale
              if (k == b || k == fs_ || sk == b || sk == fs_ || p_ns == b || p_ns == fs_) pv = false;
              if (k == fs_) {
                sk = fns;
                f = (fbits & 1u) != 0;
                onck = false;  // s is on no cycle now (a new one rescans)
              } else if (sk != SUCC_TERM && sk != k) {
                if (sk == fs_) f = (fbits & 4u) != 0 || onck;
                else if (sk == b) f = (fbits & 2u) != 0 || onck;
              }
              m = __ballot(f) & ~((2ull << l) - 1ull);  // l == 63: shift wraps to 0, mask 0
              prof(19);
            }
            if (lane == 0) {
              s_cnt = nc;
              s_ctl.rule_rounds += rr;
            }
          }
        } else {
          const uint32_t cursor = s_ctl.i;
          uint32_t best = NO_AGENT;
          for (uint32_t k = cursor + tid; k < n; k += bd) {
            const uint32_t s = S.SUCC[k];
            if (s == SUCC_TERM || s == k) continue;
            if (S.V[s] == S.G[s] || S.ONC[k]) {
              best = k;  // later k of this thread are larger
              break;
            }
          }
          best = wave_min_u32(best);
          if (lane == 0) s_wcount[wid] = best;
          PBAR();
          PLAN_TICK(13);
          if (tid == 0) {
            uint32_t b = NO_AGENT;
            for (uint32_t w = 0; w < nwaves; ++w) b = s_wcount[w] < b ? s_wcount[w] : b;
            s_best = b;
            s_miss = 0;
            if (b != NO_AGENT) {
              if (fire(b).flags & FO_ROT) s_miss = 1;
            } else {
              s_ctl.i = n;
            }
          }
        }
        PBAR();
        PLAN_TICK(14);
        if (s_best == NO_AGENT) break;
        if (tid == 0 && (s_ctl.rule_rounds & 1023u) == 1023u && plan_abort(P)) s_abort = 1;
        if (s_miss) {
          // goals of the fired agents changed: their next hops (hence succ) must be looked up
          const uint32_t q = refresh_codes(P, S, s_q, &s_need, s_ctl.section);
          if (q > 0 && !coop_resolve(P, S, s_q, &s_need, &s_flag, s_ctl.section)) {
            if (tid == 0) {
              s_ctl.qcount = s_q[0];
              s_ctl.status = PLAN_NEED_QUERIES;
              s_exit = 1;
            }
            PBAR();
            break;
          }
          // only the agents in `list` changed since the last labelling: relabel incrementally when
          // they are few (a rotation's members), else by pointer doubling over every agent
          if (s_cnt != NO_AGENT && s_cnt <= 64u) {
            if (tid == 0) {
              const bool ok = rules_relabel_changed(P, S, list, s_cnt, 4096u);
              s_flag = ok ? 1u : 0u;
              if (ok) s_ctl.relabel_inc += 1;
            }
            PBAR();
            if (!s_flag) {
              rules_init(P, S);
              if (tid == 0) s_ctl.relabel_full += 1;
            }
          } else {
            rules_init(P, S);
            if (tid == 0) s_ctl.relabel_full += 1;
          }
          PBAR();
          if (P.prefetch) {
            if (P.wide_prefetch && s_cnt != NO_AGENT) rules_prefetch_list(P, S, s_q, list, s_cnt);
            else rules_prefetch(P, S, s_q);
            if (P.coop && tid == 0) coop_publish(P, s_q);
          }
          if (tid == 0) s_cnt = 0;
          PLAN_TICK(15);
        }
      }
      if (s_abort) continue;  // watchdog: exit at the top of the section loop, position kept
      if (s_exit) break;
      // agents the phase changed since the last relabel (fast rule-3 swaps and 2-cycle rotations never
      // take the relabel path): their new paths walked ahead and their rules candidates queued now, as
      // the relabel path does — the movement phase and the next step read them
      if (P.prefetch && s_cnt != 0u && !(kab & 2u)) {
        if (P.wide_prefetch && s_cnt != NO_AGENT) rules_prefetch_list(P, S, s_q, list, s_cnt);
        else rules_prefetch(P, S, s_q);
        if (P.coop && tid == 0) coop_publish(P, s_q);
        PBAR();
      }
      if (tid == 0) {
        s_ctl.section = SEC_PRE2;
        s_ctl.i = 0;
        s_cnt = 0;
      }
      PBAR();
    } else if (sec == SEC_MOVE && P.has_dups) {
      if (tid == 0) {
        s_ctl.miss = 0;
        if (walk_move(P, S, s_ctl)) {
          s_ctl.section = SEC_RECORD;
          s_ctl.i = 0;
        }
        if (s_ctl.miss == 2) atomicOr(&P.ctl->err, ERR_NO_TABLE);
      }
      PBAR();
      if (s_ctl.miss) {
        const uint32_t q = refresh_codes(P, S, s_q, &s_need, s_ctl.section);
        if (s_ctl.miss == 1 && q > 0 && coop_resolve(P, S, s_q, &s_need, &s_flag, s_ctl.section)) {
          if (tid == 0) s_ctl.miss = 0;
          PBAR();
          continue;  // resume the serial scan at ctl.i
        }
        if (tid == 0) {
          s_ctl.qcount = s_q[0];
          s_ctl.status = (q > 0 && s_q[0] > 0 && s_ctl.miss == 1) ? PLAN_NEED_QUERIES : PLAN_ERROR;
          s_exit = 1;
        }
        PBAR();
        break;
      }
    } else if (sec == SEC_MOVE) {
      // ---- movement phase as decidability rounds (see header) -----------------
      if (s_ctl.i == 0) {
        for (uint32_t k = tid; k < n; k += bd) S.DEC[k] = (S.V[k] == S.G[k]) ? DEC_DONE : DEC_OPEN;
        PBAR();
        if (tid == 0) s_ctl.i = 1;  // DEC initialised for this step (survives relaunches)
      }
      // Round passes as per-agent bodies, run either block-wide (k = tid, tid + bd, ...) or, in
      // the tail, by wave 0 alone over a compact list of the still-open agents.
      uint64_t tag = 0;
      uint32_t tag16 = 0;  // MUL: the round's 16-bit tag (1..65535; MU32 is cleared when it wraps to 1)
      auto set_tag = [&](uint32_t r) {
        tag = (uint64_t)r << 32;
        tag16 = (r - 1u) % 65535u + 1u;
      };
      // pass 1: target cell of an open agent; MU[c] = lowest open agent targeting c, as a
      // round-tagged max of ~k (no reset pass: entries of older rounds are stale)
      auto pass1 = [&](uint32_t k) -> bool {
        if (S.DEC[k] != DEC_OPEN) return false;
        const int code = lookup_code(P, S, k);
        if (code < 0) {
          if (code == -2) atomicOr(&P.ctl->err, ERR_NO_TABLE);
          else enqueue_pair(P, S.V[k], S.G[k], S.GT[k], s_q);
          s_miss = 1;
          S.SUCC[k] = NO_CELL;
          return true;
        }
        const uint32_t u = step_cell(S.V[k], (uint32_t)code, W);
        S.SUCC[k] = u;
        if constexpr (MUL) atomicMax(&S.MU32[u], (tag16 << 16) | (0xFFFFu - k));
        else atomicMax(reinterpret_cast<unsigned long long*>(&S.MU[u]), (unsigned long long)(tag | (uint32_t)~k));
        return true;
      };
      auto mu_of = [&](uint32_t c) -> uint32_t {  // lowest open agent targeting c this round
        if constexpr (MUL) {
          const uint32_t x = S.MU32[c];
          return (x >> 16) == tag16 ? 0xFFFFu - (x & 0xFFFFu) : NO_AGENT;
        } else {
          const uint64_t x = S.MU[c];
          return (x >> 32) == (tag >> 32) ? ~(uint32_t)x : NO_AGENT;
        }
      };
      // pass 2: tentatively decide an open agent whose turn can be replayed from the round-start
      // state. What k reads at its turn is OCC[u] (u = its target), the occupant j's cell, goal
      // and next hop, and its own cell; an undecided agent a < k changes one of them only by
      // targeting u (MU[u] != k), by being the occupant (j < k still open) or by targeting k's
      // cell (MU[v] < k). That alone is not enough: an open agent k whose open occupant b < k is
      // its mutual-swap partner is carried to b's cell before its turn and then targets a cell
      // nobody can name yet, so no agent above the lowest such k (s_best) may commit this
      // round. The same pass finds it.
      auto pass2 = [&](uint32_t k) {
        if (S.DEC[k] != DEC_OPEN) return;
        const uint32_t u = S.SUCC[k], v = S.V[k];
        const uint32_t o = S.OCC[u];
        if (o != OCC_NONE) {
          const uint32_t b = o & OCC_IDX;
          if (b < k && S.DEC[b] != DEC_DONE && S.SUCC[b] == v) {
            atomicMin(&s_best, k);
            return;
          }
        }
        if (mu_of(u) != k) return;
        if (mu_of(v) < k) return;
        uint8_t act;
        if (o == OCC_NONE) {
          act = DEC_MOVE;  // rule 2
        } else {
          const uint32_t j = o & OCC_IDX;
          if (j == k) {
            act = DEC_STAY;
          } else {
            if (j < k && S.DEC[j] != DEC_DONE) return;  // occupant still open below k
            if (S.V[j] == S.G[j]) {
              act = DEC_STAY;
            } else {
              const int cj = lookup_code(P, S, j);
              if (cj < 0) {
                if (cj == -2) atomicOr(&P.ctl->err, ERR_NO_TABLE);
                else enqueue_pair(P, S.V[j], S.G[j], S.GT[j], s_q);
                s_miss = 1;
                return;
              }
              act = step_cell(S.V[j], (uint32_t)cj, W) == v ? DEC_SWAP : DEC_STAY;  // :273
            }
          }
        }
        S.DEC[k] = act;
      };
      // pass 3: commit below s_best (disjoint cells by construction); undo the rest
      auto pass3 = [&](uint32_t k, uint32_t spmin) {
        const uint8_t d = S.DEC[k];
        if (d < DEC_STAY) return;
        if (k >= spmin) {
          S.DEC[k] = DEC_OPEN;
          return;
        }
        S.DEC[k] = DEC_DONE;
        if (d == DEC_STAY) return;
        const uint32_t u = S.SUCC[k], v = S.V[k];
        DTAG(k, 8u);
        if (d == DEC_MOVE) {
          S.V[k] = u;
          S.OCC[u] = k;
          S.OCC[v] = OCC_NONE;
          S.NHC[k] = NHC_DIRTY;
        } else {
          const uint32_t j = S.OCC[u] & OCC_IDX;
          DTAG(j, 8u);
          S.V[k] = u;
          S.V[j] = v;
          S.OCC[u] = k;
          S.OCC[v] = j;
          S.NHC[k] = NHC_DIRTY;
          S.NHC[j] = NHC_DIRTY;
        }
      };
      // Within a round DEC only goes OPEN -> {STAY, MOVE, SWAP} (own entry, pass 2) and the
      // commit pass turns those into DONE (or back to OPEN), so "open at round start" reads
      // as DEC != DEC_DONE for every other agent throughout the round.
      bool tail = false;  // block-uniform: the remaining rounds run in wave 0
      for (;;) {
        if (tid == 0) {
          s_miss = 0;
          s_best = NO_AGENT;
          s_ctl.move_rounds += 1;
          if (PLAN_DBG) s_tp = wall_clock64();
          if ((s_ctl.move_rounds & 1023u) == 0u && plan_abort(P)) s_abort = 1;
        }
        PBAR();
        if (s_abort) break;
        set_tag(s_ctl.move_rounds);
        if (MUL && tag16 == 1u && s_ctl.move_rounds > 1u) {  // the 16-bit tag wrapped: old entries would match
          for (uint32_t c = tid; c < P.ncell; c += bd) S.MU32[c] = 0u;
          PBAR();
        }
        int open = 0;
        for (uint32_t k = tid; k < n; k += bd) open |= pass1(k) ? 1 : 0;
        // one agent per thread: the count is exact and decides the switch to the wave tail
        const int nopen = n <= bd ? __syncthreads_count(open) : __syncthreads_or(open);
        PLAN_TICK(8);
        if (!nopen) break;
        if (s_miss) break;  // exit to K3 below
        if (n <= bd && nopen <= 64) {
          // compact the open agents (index order) into `list` for the wave tail
          const uint64_t bal = __ballot(open != 0);
          if (lane == 0) s_wcount[wid] = (uint32_t)__popcll(bal);
          PBAR();
          if (open) {
            uint32_t off = 0;
            for (uint32_t w = 0; w < wid; ++w) off += s_wcount[w];
            list[off + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = tid;
          }
          PBAR();
          tail = true;
          break;
        }
        for (uint32_t k = tid; k < n; k += bd) pass2(k);
        PBAR();
        PLAN_TICK(10);
        const uint32_t spmin = s_best;
        for (uint32_t k = tid; k < n; k += bd) pass3(k, spmin);
        PBAR();
        PLAN_TICK(12);
        if (s_miss) break;
      }
      if (tail) {
        // Wave tail: <= 64 open agents, one per lane of wave 0. The round that switched has
        // run pass 1; every pass boundary is a wave-level fence (LDS is in order per wave).
        if (wid == 0) {
          uint32_t nl = 0;
          for (uint32_t w = 0; w < nwaves; ++w) nl += s_wcount[w];
          const uint32_t k = lane < nl ? list[lane] : NO_AGENT;
          uint32_t kk = k;
          for (bool first = true;; first = false) {
            if (!first) {
              if (lane == 0) {
                s_miss = 0;
                s_best = NO_AGENT;
                s_ctl.move_rounds += 1;
                if ((s_ctl.move_rounds & 1023u) == 0u && plan_abort(P)) s_abort = 1;
              }
              __threadfence_block();
              if (*(volatile uint32_t*)&s_abort) break;
              __threadfence_block();
              set_tag(*(volatile uint32_t*)&s_ctl.move_rounds);
              if (MUL && tag16 == 1u) {  // wrapped (wave 0 alone here)
                for (uint32_t c = lane; c < P.ncell; c += 64u) S.MU32[c] = 0u;
                __threadfence_block();
              }
              const bool op = kk != NO_AGENT && pass1(kk);
              __threadfence_block();
              if (__ballot(op) == 0ull) break;
              if (*(volatile uint32_t*)&s_miss) break;
            }
            if (kk != NO_AGENT) pass2(kk);
            __threadfence_block();
            const uint32_t spmin = *(volatile uint32_t*)&s_best;
            if (kk != NO_AGENT) pass3(kk, spmin);
            __threadfence_block();
            if (*(volatile uint32_t*)&s_miss) break;
            if (kk != NO_AGENT && S.DEC[kk] != DEC_OPEN) kk = NO_AGENT;  // committed: leaves the tail
          }
        }
        PBAR();
      }
      if (s_abort) continue;  // watchdog: exit at the top of the section loop, position kept
      if (s_miss) {
        // the missing codes are queued (pass 1 / pass 2) and their agents' codes are dirty
        if (s_q[0] > 0 && coop_resolve(P, S, s_q, &s_need, &s_flag, s_ctl.section)) continue;  // replay the open rounds
        if (tid == 0) {
          s_ctl.qcount = s_q[0];
          s_ctl.status = s_q[0] > 0 ? PLAN_NEED_QUERIES : PLAN_ERROR;
          s_exit = 1;
        }
        PBAR();
        break;
      }
      if (tid == 0) {
        s_ctl.section = SEC_RECORD;
        s_ctl.i = 0;
      }
      PBAR();
    } else if (sec == SEC_RECORD) {
      if (P.mode == MODE_STEP) {
        if (tid == 0) {
          s_ctl.status = PLAN_DONE;
          s_ctl.section = SEC_DONE;
          s_ctl.qcount = s_q[0];  // speculative prefetches still queued: the host resolves them
          s_exit = 1;
        }
        PBAR();
        break;
      }
      // ---- record (tswap.rs:144-158) + termination (tswap.rs:163-169) --------
      const uint32_t t = s_ctl.t;
      uint64_t* rec = P.rec + (uint64_t)t * n;
      uint32_t* grec = P.grec ? P.grec + (uint64_t)t * n : nullptr;
      int busy = 0;
      for (uint32_t i = tid; i < n; i += bd) {
        const uint32_t v = S.V[i], g = S.G[i];
        const uint8_t st = P.st[i];
        uint64_t s;
        if (st == ST_IDLE) s = 3;
        else if (st == ST_TO_PICKUP) s = 0;
        else s = (v == g) ? 2 : 1;
        busy |= (st != ST_IDLE);
        rec[i] = (uint64_t)(v % W) | ((uint64_t)(v / W) << 16) | (s << 32);
        if (grec) grec[i] = g;
      }
      busy = __syncthreads_or(busy);
      if (tid == 0) {
        s_ctl.t = t + 1;
        s_ctl.steps_run += 1;
        // speculative entries carry their enqueue timestep (s_q[5]); the workers drop the stale ones
        s_q[5] = t + 1;
        if (P.coop) __hip_atomic_store(&P.cc->t_now, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (P.hflags) __hip_atomic_store(&P.hflags[2], s_ctl.steps_run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((s_ctl.unused == 0u && !busy) || s_ctl.t > s_ctl.max_t) {
          s_ctl.status = PLAN_DONE;
          s_ctl.section = SEC_DONE;
          s_ctl.qcount = s_q[0];  // speculative prefetches still queued: the host resolves them
          s_exit = 1;
        } else {
          s_ctl.section = SEC_ASSIGN;
        }
      }
      PBAR();
    } else {
      break;  // SEC_DONE
    }
  }

  // ---- write back ------------------------------------------------------------
  PBAR();
  if constexpr (AG)
    for (uint32_t k = tid; k < n; k += bd) {
      P.v[k] = S.V[k];
      P.g[k] = S.G[k];
      P.dec[k] = S.DEC[k];
    }
  else if (P.part_lds & (PART_V | PART_G))
    for (uint32_t k = tid; k < n; k += bd) {
      if (P.part_lds & PART_V) P.v[k] = S.V[k];
      if (P.part_lds & PART_G) P.g[k] = S.G[k];
    }
  if constexpr (OC)
    for (uint32_t c = tid; c < P.ncell; c += bd) P.occ[c] = S.OCC[c];
  if (tid == 0) {
    if (P.coop) {  // last publish, then release the workers (they drain the needed queue and exit)
      coop_publish(P, s_q);
      __hip_atomic_store(&P.cc->stop, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&P.cc->pub, s_q[2] + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t err = P.ctl->err;
    *P.ctl = s_ctl;
    P.ctl->err |= err;
    s_tick[s_tsec] += wall_clock64() - s_tlast;
    if (P.sec_ticks)
      for (int k = 0; k < 48; ++k) P.sec_ticks[k] += s_tick[k];
  }
}
#undef PLAN_DBG
#define PLAN_DBG (P.dbg != 0u)


template <bool AG, bool OC, bool MUL, bool PG = false>
hipError_t launch_plan_t(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                                hipStream_t s) {
  hipError_t e = hipFuncSetAttribute((const void*)k_plan<AG, OC, MUL, PG>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_plan<AG, OC, MUL, PG>), dim3(grid), dim3(block), lds, s, P, W);
  return hipGetLastError();
}

}  // namespace tsw
