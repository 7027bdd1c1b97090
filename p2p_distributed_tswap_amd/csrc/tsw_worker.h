// tsw_worker.h — coop-mode K3 workers: the exact A* (tsw_astar.h) run by the non-planner
// workgroups of the plan dispatch (k_plan, tsw_plan.hip) CONCURRENTLY with the planner block.
//
// One dispatch holds the planner (workgroup 0) and one worker workgroup per other CU; a worker
// workgroup runs `wpb` independent single-wave workers (the rest of its waves leave at once), each
// with its own slice of the workgroup's LDS (heap, g-scores, free-cell bitmap). Being one dispatch,
// the planner and its workers are resident together whatever serialises dispatches (a profiler's
// counter passes, another queue): nothing waits on a kernel that has not started. Workers never
// execute s_barrier (their waves run unrelated queries); LDS ordering within a wave is
// wave_order() — LDS instructions of one wave complete in issue order.
//
// Protocol (CoopCtl, tsw_internal.h): the planner appends (cell, goal) pairs to two queues —
// needed pairs (a step is waiting on them) and speculative prefetches — and publishes the heads;
// each worker claims one pair at a time (needed first, CAS on the claim counter), runs the A*
// (same BinaryHeap order and hand-off chain as k_astar_wave: LDS heap + LDS g-scores -> LDS heap +
// global u32 g-scores -> global heap) and stores the code into the next-hop table with an
// agent-scope store the planner polls. Task chains (every task's pickup -> delivery path, walked
// hop by hop) are the lowest-priority job. `alive` counts running workers (incremented at start,
// decremented at every exit), so the planner stops waiting within a millisecond when there are
// none. Termination: the planner sets `stop` when it leaves (also for a host round trip); workers
// then drain the needed queue and exit; an idle worker also exits after 5 s, and on the host
// watchdog's abort word.
#pragma once
#include <hip/hip_runtime.h>

#include "tsw_astar.h"
#include "tsw_internal.h"
#include "tsw_plan.h"

namespace tsw {

__device__ __forceinline__ uint32_t w_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool w_cas(uint32_t* p, uint32_t expect, uint32_t want) {
  return __hip_atomic_compare_exchange_strong(p, &expect, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}
// a worker is one wave of a multi-wave workgroup: order its own memory accesses without s_barrier
__device__ __forceinline__ void wave_sync() {
  __threadfence_block();
  wave_order();
}
__device__ __forceinline__ uint32_t hw_xcc_id() {
  return (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
}

// lane 0: claim the next pair (0: needed queue, 1: speculative queue, 2: task chain, 3: hot task chain,
// 4: predicted task chain, -1: exit).
// Task chains (long, lowest priority) only go to workers with take_t: the others stay free for the
// pairs the planner needs or will need soon.
__device__ __forceinline__ int worker_claim(CoopCtl* cc, uint32_t* idx, bool take_t, const uint32_t* hflags,
                                            unsigned long long idle_ticks, uint32_t wid, uint32_t gate,
                                            uint32_t slow_mask, uint32_t slow_mult) {
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
        // hot chains first: tasks the planner has just assigned
        const uint32_t hh = w_ld(&cc->head_h), ch = w_ld(&cc->claim_h);
        if (ch < hh) {
          if (w_cas(&cc->claim_h, ch, ch + 1u)) {
            *idx = ch;
            return 3;
          }
          continue;
        }
        // then predicted chains: tasks agents are about to be assigned
        const uint32_t hp = w_ld(&cc->head_p), cp = w_ld(&cc->claim_p);
        if (cp < hp) {
          if (w_cas(&cc->claim_p, cp, cp + 1u)) {
            *idx = cp;
            return 4;
          }
          continue;
        }
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
  // Who polls and who answers a publish (round 4): every idle wave polling `pub` every ~0.5 us (agent
  // scope, served past the L2) made that word a hot spot, and every publish woke all of them (C3: ~950
  // of 1,020 idle) into one herd of loads and CASes on the claim words — ~70 us from enqueue to claim
  // in the queue-delay diagnostics, and a slower planner. Now only the fast pollers (wid & slow_mask)
  // == 0 poll at full rate, and of those only the rotating subset with ((wid >> fbits) ^ pub) & gate
  // == 0 rescans at once; a slow poller (slow_mult times the interval) rescans whenever it sees a
  // change — a trickle, not a herd — and everybody rescans every 64 polls as a safety net.
  const bool fast = (wid & slow_mask) == 0u;
  const uint32_t fbits = (uint32_t)__builtin_popcount(slow_mask);
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
      if (wall_clock64() - t0 > idle_ticks) return -1;  // idle this long (5 s): safety exit
      if (k < 8) {
        __builtin_amdgcn_s_sleep(2);
      } else {
        // slow pollers (wid & slow_mask != 0) sleep slow_mult times longer: every idle wave polling the
        // one `pub` word (agent scope, served past the L2) every ~0.5 us makes it a hot spot
        const uint32_t m = fast ? 1u : slow_mult;
        for (uint32_t r = 0; r < m; ++r) __builtin_amdgcn_s_sleep(16);
      }
      const uint32_t p = w_ld(&cc->pub);
      if ((p != seen && (!fast || (((wid >> fbits) ^ p) & gate) == 0u)) || (k & 63u) == 63u) {
        seen = p;
        break;
      }
    }
  }
}

// lane 0, non-blocking: claim one pair of the needed or the speculative queue (0 / 1), else -1.
// A worker walking a task chain calls this between hops, so chains (lowest priority, up to ~100
// A* each) never hold a worker while pairs the planner needs or will need soon are queued. Once the
// planner has stopped only needed pairs are taken (as in worker_claim): the chain workers' preempt
// loop used to drain the whole speculative backlog after the plan ended (C5, 1 timestep: 4.2 s of
// dispatch for 0.2 s of planning, 113k speculative A* nobody would read).
__device__ __forceinline__ int worker_try_claim(CoopCtl* cc, uint32_t* idx) {
  for (;;) {
    const uint32_t hn = w_ld(&cc->head_n), cn = w_ld(&cc->claim_n);
    if (cn < hn) {
      if (w_cas(&cc->claim_n, cn, cn + 1u)) {
        *idx = cn;
        return 0;
      }
      continue;
    }
    if (w_ld(&cc->stop)) return -1;
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
  if (ep % 1023u == 0u && ep > 0u)
    for (uint32_t c = lane; c < ncell; c += 64u) GS[c] = 0u;
  wave_sync();
  const uint32_t tag = ep % 1023u + 1u;
  ++ep;
  return tag;
}

// One coop worker = one wave. wid: worker index (its global g-score slot / heap / epoch);
// wsm: this wave's LDS slice (A.lds_per_wave bytes: heap, then g-scores, then the free bitmap).
__device__ __forceinline__ void coop_worker(const WorkerArgs& A, uint64_t* wsm, uint32_t wid) {
  const DevGrid G = A.G;
  uint64_t* Hp = wsm;
  const uint32_t lane = threadIdx.x & 63u, ncell = G.ncell, hcap = A.hcap, gs_lds = A.gs_lds;
  // a worker on the planner's XCD leaves at once: the planner's agent arrays, occupancy and table
  // lines then share that XCD's 4 MB L2 with nobody's g-score slots. The planner publishes its XCD
  // first thing; a worker that does not see it within ~20 us stays.
  if (A.avoid_xcc) {
    uint32_t px = 0;
    for (int k = 0; k < 64 && px == 0u; ++k) {
      px = w_ld(&A.cc->planner_xcc);
      if (px == 0u) __builtin_amdgcn_s_sleep(8);
    }
    if (px != 0u && px - 1u == hw_xcc_id()) return;  // wave-uniform, before `alive`
  }
  uint32_t* GSl = reinterpret_cast<uint32_t*>(wsm + hcap);  // gs_lds == 1
  uint8_t* GB = reinterpret_cast<uint8_t*>(wsm + hcap);      // gs_lds == 2
  const uint32_t gsb = gs_lds == 1u ? ncell * 4u : gs_lds == 2u ? (ncell + 15u) / 16u * 16u : 0u;
  // the free-cell bitmap: staged in LDS (A.stage_fb; worker_config stages it whenever the g-scores
  // are in LDS) or read from global memory. The two are separate pointers passed to separate calls,
  // never one pointer selected at run time: a selected pointer is generic, and its loads become flat
  // loads (no ds_read), which sit on the A* pop's dependent chain.
  uint32_t* const FBl = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(wsm + hcap) + gsb);
  const uint32_t* const FBg = G.freebits;
  const uint32_t nfw = G.H * G.Ww;
  if (A.stage_fb)
    for (uint32_t t = lane; t < nfw; t += 64u) FBl[t] = G.freebits[t];
  // DAG early exit (A.dag == 1): the detour bytes of the goal last staged (dt_goal) over the box
  // dt_box = x0 | x1 << 16 (dt_bx), y0 | y1 << 16 (dt_by), after the bitmap
  uint8_t* DT = reinterpret_cast<uint8_t*>(wsm + hcap) + gsb + (A.stage_fb ? (nfw * 4u + 15u) / 16u * 16u : 0u);
  uint32_t dt_goal = 0xFFFFFFFFu, dt_bx = 0u, dt_by = 0u;
  if (gs_lds == 1u)
    for (uint32_t c = lane; c < ncell; c += 64u) GSl[c] = 0u;
  uint32_t* GSg = A.gs_all + (uint64_t)wid * ncell;
  uint64_t* Hg = A.heaps + (uint64_t)wid * A.ghcap;
  uint32_t ep = A.epochs[wid], epl = 0;
  wave_sync();
  if (lane == 0) __hip_atomic_fetch_add(&A.cc->alive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // exact A* for (v, goal): tier 1 LDS heap + LDS (or global) g-scores, tier 2 global u32
  // g-scores, tier 3 global heap (the k_astar_wave -> k_astar hand-off chain, in one wave)
  uint32_t last_pops = 0;      // heap pops of the last query (tiers 1-2; diagnostics)
  unsigned long long tiers = 0;  // queries handed to tier 2 (low half) / tier 3 (high half)
  // tab: the goal's table slot (< 0: no table, no early exit)
  auto resolve_exact = [&](uint32_t v, uint32_t goal, int32_t tab) -> uint8_t {
    int32_t L = 0;
    uint8_t code = NH_UNKNOWN;
    uint32_t np = 0, npt = 0;  // heap pops (diagnostics)
    uint32_t dag = tab >= 0 ? A.dag : 0u;
    const uint8_t* DGt = dag ? A.dt + (uint64_t)tab * A.nstride : nullptr;
    if (dag == 1u) {
      // the query's ellipse box: d* = |v - goal| + 2 * detour(v), margin detour(v) around the start/goal box
      const uint32_t W = G.W, vy = v / W, vx = v - vy * W, gy = goal / W, gx = goal - gy * W;
      const uint32_t dv = __builtin_amdgcn_readfirstlane((uint32_t)DGt[v]);
      if (dv == DT_NONE) {
        dag = 0u;  // unreachable or detour past the byte range: the full search
      } else {
        const uint32_t e = dv;
        const uint32_t x0 = min(vx, gx) > e ? min(vx, gx) - e : 0u, x1 = min(max(vx, gx) + e, W - 1u);
        const uint32_t y0 = min(vy, gy) > e ? min(vy, gy) - e : 0u, y1 = min(max(vy, gy) + e, G.H - 1u);
        const bool inside = dt_goal == goal && x0 >= (dt_bx & 0xFFFFu) && x1 <= (dt_bx >> 16) &&
                            y0 >= (dt_by & 0xFFFFu) && y1 <= (dt_by >> 16);
        if (!inside) {
          const unsigned long long ts0 = wall_clock64();
          stage_detour(DT, DGt, W, x0, x1, y0, y1, lane);
          dt_goal = goal;
          dt_bx = x0 | (x1 << 16);
          dt_by = y0 | (y1 << 16);
          if (lane == 0) {  // diagnostics: staging time / count
            __hip_atomic_fetch_add(&A.cc->wbusy[3], wall_clock64() - ts0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&A.cc->wcount[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    if (gs_lds == 2u) {
      uint4* g4 = reinterpret_cast<uint4*>(GB);
      for (uint32_t c = lane; c < (ncell + 15u) / 16u; c += 64u) g4[c] = make_uint4(0u, 0u, 0u, 0u);
      wave_sync();
      code = dag == 1u ? astar_wave_par<2, false, 1>(G, v, goal, 0u, Hp, hcap, nullptr, GB, FBl, &L, nullptr, DT, nullptr, &np, A.dag_mask, A.reg_heap)
                       : astar_wave_par<2, false>(G, v, goal, 0u, Hp, hcap, nullptr, GB, FBl, &L, nullptr, nullptr, nullptr, &np, 15u, A.reg_heap);
    } else if (gs_lds == 1u) {
      if (epl % 1023u == 0u && epl > 0u) {
        for (uint32_t c = lane; c < ncell; c += 64u) GSl[c] = 0u;
      }
      wave_sync();
      const uint32_t tag = epl % 1023u + 1u;
      ++epl;
      code = dag == 1u ? astar_wave_par<1, false, 1>(G, v, goal, tag, Hp, hcap, GSl, nullptr, FBl, &L, nullptr, DT, nullptr, &np, A.dag_mask, A.reg_heap)
                       : astar_wave_par<1, false>(G, v, goal, tag, Hp, hcap, GSl, nullptr, FBl, &L, nullptr, nullptr, nullptr, &np, 15u, A.reg_heap);
    } else {
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      if (A.stage_fb)
        code = dag == 2u
                   ? astar_wave_par<1, false, 2, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBl, &L, nullptr, nullptr, DGt, &np, A.dag_mask, A.reg_heap)
                   : astar_wave_par<1, false, 0, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBl, &L, nullptr, nullptr, nullptr, &np, 15u, A.reg_heap);
      else
        code = dag == 2u
                   ? astar_wave_par<1, false, 2, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBg, &L, nullptr, nullptr, DGt, &np, A.dag_mask, A.reg_heap)
                   : astar_wave_par<1, false, 0, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBg, &L, nullptr, nullptr, nullptr, &np, 15u, A.reg_heap);
    }
    npt = np;
    if (L == -2 && gs_lds != 0u) {  // tier 2: global u32 g-scores (the staged detour bytes still apply)
      tiers += 1ull;
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      code = dag == 1u ? astar_wave_par<1, false, 1>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBl, &L, nullptr, DT, nullptr, &np, A.dag_mask, A.reg_heap)
                       : astar_wave_par<1, false>(G, v, goal, tag, Hp, hcap, GSg, nullptr, FBl, &L, nullptr, nullptr, nullptr, &np, 15u, A.reg_heap);
      npt += np;
    }
    if (L == -2) {
      tiers += 1ull << 32;
      const uint32_t tag = slot_tag(GSg, ncell, ep, lane);
      if (lane == 0) code = astar_one(G, v, goal, tag, Hg, A.ghcap, GSg, &L, &A.cc->err);
      code = (uint8_t)__builtin_amdgcn_readfirstlane(code);
    }
    last_pops = npt;
    return code;
  };
  uint32_t cur_q = 0;  // queue of the query being resolved (0 needed, 1 spec, 2 chain)
  auto resolve = [&](uint32_t v, uint32_t goal, int32_t tab) -> uint8_t {
    const unsigned long long tr0 = wall_clock64();
    const uint8_t code = resolve_exact(v, goal, tab);
    if (lane == 0) {
      __hip_atomic_fetch_add(&A.cc->wbusy[cur_q], wall_clock64() - tr0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&A.cc->wcount[cur_q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&A.cc->wpops[cur_q], (unsigned long long)last_pops, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
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
  // a speculative entry older than the planner's stale threshold is dropped unresolved: its code goes
  // back PENDING_S -> UNKNOWN (CAS on the word, agent scope, so a code published meanwhile or a
  // promotion to PENDING by the planner is never overwritten), and the planner queues the pair again
  // if a step still needs it — results-neutral, only the workers' time is saved
  auto drop_stale = [&](const uint32_t* e, uint32_t v, int32_t tab) -> bool {
    if (tab < 0) return false;
    bool drop = false;
    if (lane == 0 && A.stale_steps != 0u) {
      if (w_ld(&A.cc->t_now) - w_ld(e + 3) > A.stale_steps) {
        uint32_t* wp = reinterpret_cast<uint32_t*>((uintptr_t)(A.nh + (uint64_t)tab * A.nstride + v) & ~(uintptr_t)3u);
        const uint32_t sh = 8u * (uint32_t)((uintptr_t)(A.nh + (uint64_t)tab * A.nstride + v) & 3u);
        bool reset = false;
        for (;;) {
          const uint32_t w = w_ld(wp);
          if (((w >> sh) & 0xFFu) != NH_PENDING_S) break;  // resolved, promoted or reset already
          if (w_cas(wp, w, w | (0xFFu << sh))) {           // NH_UNKNOWN = 0xFF
            reset = true;
            break;
          }
        }
        // only a reset is a drop; a code resolved meanwhile needs no work and a promoted one
        // sits on the needed queue, so the entry is skipped either way and counted as such
        if (reset) __hip_atomic_fetch_add(&A.cc->spec_dropped, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(&A.cc->qskip[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        drop = true;
      }
    }
    return __builtin_amdgcn_readfirstlane(drop ? 1 : 0) != 0;
  };
  const bool take_t = (wid & A.tmask) == A.tmask;
  // the task an agent idle at cell D will be assigned if nothing changes before: the untaken task whose
  // pickup is nearest to D, first by task index on ties (tswap.rs:123-130 as K4 computes it) — read from
  // K4's spatial index while the planner updates it, with plain loads (this XCD's L2 copy may be stale: a
  // prediction only picks a chain, and agent-scope loads of the whole chunk-count array for every
  // prediction moved ~128 KB each past the L2)
  auto predict_task = [&](uint32_t D) -> uint32_t {
    const uint32_t dy = D / G.W, dx = D - dy * G.W, nch = A.kchunks;
    auto box_lb = [&](uint2 bx) -> uint32_t {
      const uint32_t x0 = bx.x & 0xFFFFu, y0 = bx.x >> 16, x1 = bx.y & 0xFFFFu, y1 = bx.y >> 16;
      return (dx < x0 ? x0 - dx : dx > x1 ? dx - x1 : 0u) + (dy < y0 ? y0 - dy : dy > y1 ? dy - y1 : 0u);
    };
    uint32_t ub = 0xFFFFFFFFu;
    for (uint32_t c = lane; c < nch; c += 64u) {
      if (A.kcnt[c] == 0u) continue;
      const uint2 bx = A.kbox[c];
      ub = min(ub, box_lb(bx) + ((bx.y & 0xFFFFu) - (bx.x & 0xFFFFu)) + ((bx.y >> 16) - (bx.x >> 16)));
    }
    ub = __ockl_wfred_min_u32(ub);
    uint32_t bdst = 0xFFFFFFFFu, btsk = 0xFFFFFFFFu;
    for (uint32_t c = lane; c < nch; c += 64u) {
      if (A.kcnt[c] == 0u || box_lb(A.kbox[c]) > ub) continue;
      for (uint32_t e = 0; e < 32u; ++e) {
        const uint32_t xy = A.klive[c * 32u + e];
        if (xy == 0xFFFFFFFFu) continue;
        const uint32_t tx = xy & 0xFFFFu, ty = xy >> 16;
        const uint32_t d = (tx > dx ? tx - dx : dx - tx) + (ty > dy ? ty - dy : dy - ty), t = A.klt[c * 32u + e];
        if (d < bdst || (d == bdst && t < btsk)) {
          bdst = d;
          btsk = t;
        }
      }
    }
    const uint32_t dm = __ockl_wfred_min_u32(bdst);
    return __ockl_wfred_min_u32(bdst == dm ? btsk : 0xFFFFFFFFu);
  };
  auto walk_chain = [&](uint32_t c, uint32_t goal, int32_t tab) {
    const uint32_t max_hops = A.chain_hops ? A.chain_hops : ncell;
    for (uint32_t hop = 0; hop < max_hops && c != goal; ++hop) {
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
        if (w2 == 1 && drop_stale(e2, v2, t2)) continue;
        cur_q = (uint32_t)w2;
        publish_code(v2, t2, resolve(v2, g2, t2), false);
        cur_q = 2u;
      }
      uint8_t code = (uint8_t)__builtin_amdgcn_readfirstlane(lane == 0 ? code_at(c, tab) : 0u);
      if (code == NH_UNKNOWN) {
        code = resolve(c, goal, tab);
        publish_code(c, tab, code, true);
      }
      if (code >= NH_STAY) break;  // stay (unreachable goal), pending elsewhere, or overflow
      c = step_cell(c, code, G.W);
    }
  };
  for (;;) {
    int which = -1;
    uint32_t idx = 0;
    if (lane == 0) which = worker_claim(A.cc, &idx, take_t, A.hflags, A.idle_ticks, wid, A.wake_gate, A.slow_mask, A.slow_mult);
    which = __builtin_amdgcn_readfirstlane(which);
    if (which < 0) break;
    idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
    // the entry was published by the planner's release of the head (or by the host before the
    // launch): read it past stale caches
    const uint32_t* e =
        which == 4 ? reinterpret_cast<const uint32_t*>(A.QP + idx)
                   : reinterpret_cast<const uint32_t*>((which == 0 ? A.QN : which == 1 ? A.QS : which == 3 ? A.QH : A.QT) + idx);
    uint32_t v = w_ld(e), goal = w_ld(e + 1);
    int32_t tab = which == 4 ? -1 : (int32_t)w_ld(e + 2);  // a QP entry is two words
    if (which == 4) {  // predicted chain: entry = (delivery cell, agent)
      const uint32_t t = predict_task(v);
      if (lane == 0) {
        __hip_atomic_fetch_add(&A.cc->pred_jobs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (A.pred) __hip_atomic_store(&A.pred[goal], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (t == 0xFFFFFFFFu) continue;
      v = A.pick[t];
      goal = A.dlv[t];
      if (v == CELL_BAD || goal == CELL_BAD || v == goal) continue;
      tab = A.goal_tab[goal];
    }
    if (which >= 3) which = 2;  // hot and predicted chains are walked as any task chain
    cur_q = (uint32_t)which;
    if (which < 2) {
      // a pair resolved meanwhile (a promoted speculative pair whose first copy finished, or a chain
      // hop) is not searched again
      if (tab >= 0 && (uint32_t)__builtin_amdgcn_readfirstlane(lane == 0 ? code_at(v, tab) : 0u) <= NH_STAY) {
        if (lane == 0) __hip_atomic_fetch_add(&A.cc->qskip[which], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      if (which == 1 && drop_stale(e, v, tab)) continue;
      if (lane == 0) {  // diagnostics: queue delay (needed: enqueue wall time, speculative: timestep)
        const uint32_t dt = (which == 0 ? (uint32_t)wall_clock64() : w_ld(&A.cc->t_now)) - w_ld(e + 3);
        __hip_atomic_fetch_add(&A.cc->qdelay[which], (unsigned long long)dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dt > (which == 0 ? 100000u : 1u))
          __hip_atomic_fetch_add(&A.cc->qlate[which], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      publish_code(v, tab, resolve(v, goal, tab), false);
      continue;
    }
    // task chain: the path an agent carrying this task walks from its pickup to the delivery
    // (every hop is get_path(cell, delivery)[1], tswap.rs:263-266): follow resolved codes and
    // resolve each unresolved hop in turn; stop at a pair someone else has queued, at a stay code,
    // or at the goal. Pairs are not marked pending, so an abandoned chain leaves nothing behind.
    if (tab < 0) continue;
    walk_chain(v, goal, tab);
  }
  if (lane == 0) {
    A.epochs[wid] = ep;
    if (tiers) __hip_atomic_fetch_add(&A.cc->wpops[3], tiers, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every exit path after the increment: the planner's "no worker left" test reads this
    __hip_atomic_fetch_sub(&A.cc->alive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace tsw
