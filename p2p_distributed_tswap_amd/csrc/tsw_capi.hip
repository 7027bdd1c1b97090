// tsw_capi.hip — host runtime of the TSWAP planning core behind the C ABI
// declared in include/tswap.h. Owns device memory, the goal-table store
// (BFS distances + next-hop codes), the A* scratch slots and the per-step
// orchestration: K1 tables -> k_plan (persistent K4 assign + K2 step + record),
// relaunched after each batched K3 (A*) pass over the next hops it could not resolve.
//
// Reference call structure being replaced (RenKoya1/p2p_distributed_tswap):
//   tswap_mapd            src/algorithm/tswap.rs:39-172      -> tsw_plan_mapd
//   tswap_step            src/algorithm/tswap.rs:174-286     -> tsw_step
//   get_path              src/algorithm/tswap.rs:288-390     -> tsw_get_path_next
//   plan_all_paths' step  src/bin/centralized/manager.rs:101-144 -> tsw_step
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "tsw_internal.h"
#include "tsw_launch.h"
#include "tsw_plan.h"
#include "tswap.h"

using namespace tsw;

namespace {

thread_local std::string g_create_err;

struct DevStatus {
  uint32_t err;
  uint32_t done;
  uint32_t qcount;
  uint32_t novf;  // LDS A*: queries handed to the global-heap kernel
  uint32_t novf2;  // second tier (LDS heap, global g_scores): queries handed on to k_astar
  uint32_t work;  // k_bfs_wave goal dequeue counter
  uint32_t qnext;  // k_astar_lds / k_astar_wave dynamic query dequeue counter
  uint32_t qnext2;  // k_astar_wave second tier
};

enum { CAT_BFS = 0, CAT_ASTAR = 1, CAT_WALK = 2, CAT_ASSIGN = 3, NCAT = 4 };

// Diagnostic / A-B knobs. The production library (libtswap_hip.so) never reads the environment:
// these are its fixed defaults, and the only caller-visible options are tsw_opts (include/tswap.h).
// The diagnostic build (libtswap_hip_diag.so, -DTSW_DIAG, __graft_entry__.build) reads the TSW_*
// variables below ONCE when a context is created — kernel A/B variants, instrumentation, and
// TSW_BFS_DBG, which drops work and writes WRONG tables (measurement only).
struct Tunables {
  uint32_t bfs_mode = 0;          // TSW_BFS_KERNEL: 0 auto, 1 wave (row words), 2 block, 3 blk (8x8), 4 big, 5 mg
  uint32_t bfs_cap = 512;         // TSW_BFS_LISTCAP: k_bfs_wave LDS list entries
  uint32_t blk_cap = 576;         // TSW_BFS_BLKCAP: k_bfs_blk LDS list entries
  uint32_t bfs_waves = 16;        // TSW_BFS_WAVES: waves per K1 workgroup cap
  bool bfs_order = true;          // TSW_BFS_ORDER=0: keep the caller's goal order (no LPT)
  bool bfs_prof = false;          // TSW_BFS_PROF: print K1 cycle split per launch
  bool bfs_nostage = false;       // TSW_BFS_NOSTAGE: k_bfs_blk writes rows lane-strided (no LDS staging)
  uint32_t bfs_dbg = 0;           // TSW_BFS_DBG: k_bfs_blk diagnostics (BlkBfsArgs::dbg)
  uint32_t bfs_wls = 0;           // TSW_BFS_WLS: k_bfs_blk west-step blocks in LDS
  uint32_t bfs_pair = 0;          // TSW_BFS_PAIR: k_bfs_blk two goals per wave (one per 32-lane half)
  uint32_t wave_hcap = 0;         // TSW_ASTAR_WAVE_HCAP: k_astar_wave LDS heap entries (0 = default)
  int astar_global_gs = -1;       // TSW_ASTAR_GLOBAL_GS: -1 auto, 0 LDS g-scores, 1 global slots
  bool astar_tier2 = true;        // TSW_ASTAR_NO_TIER2: skip the LDS-heap/global-g second tier
  uint32_t astar_diag = 0;        // TSW_ASTAR_SERIAL / TSW_ASTAR_PROF (ASTAR_DIAG_*)
  bool prefetch = true;           // TSW_NO_PREFETCH: no speculative next-hop prefetch
  uint32_t wave_rules_max = 0xFFFFFFFFu;  // TSW_WAVE_RULES_MAX: wave-0 rules rounds when n <= this
  uint32_t walk_cap = 16;  // TSW_WALK_CAP: successor-walk hops of a batched rules firing (longer ones fire alone)
  uint32_t wide_prefetch = 8;     // TSW_WIDE_PREFETCH: resolved hops walked ahead (0 = candidates only)
  uint32_t wide_hi = 32, wide_lo = 8;  // TSW_WIDE_HI / TSW_WIDE_LO: coop step-start walk-ahead hops (grids <= 2^18 cells with a small backlog / grids > 2^18 cells); round 5, busy instances: 16 -> 32 and 4 -> 8 (profiles/r5/retune_busy_ab.txt)
  bool hot_chains = true;         // TSW_HOT_CHAINS=0: no planner-fed chains of just-assigned tasks (A/B)
  uint32_t chain_hops = 0;        // TSW_CHAIN_HOPS: hops resolved per task chain (0: the whole path)
  uint32_t move_round0 = 0;       // TSW_MOVE_ROUND0 (test knob): movement-round counter at the plan start (forces the MU32 tag wrap)
  bool walk_cache = true;         // TSW_WALK_CACHE=0: the step-start walk-ahead re-reads every code from the agent's next cell
  uint32_t predict = 1;           // TSW_PREDICT: predicted task chains, bit 0 at pickups, bit 1 at delivery-goal changes (0: off)
  uint32_t urgent_hops = 1;       // TSW_URGENT_HOPS: walk-ahead pairs this close are queued as needed (0: off)
  uint32_t dag_width = 4;         // TSW_DAG_WIDTH: cells per DAG prefetch level (<= 16)
  uint32_t dag_prefetch = 3;      // TSW_DAG_PREFETCH: DAG levels queued past the walk-ahead's first unresolved cell (round 2, frozen C3: 2 -> 6 levels, 465 -> 450 ms; round 5, busy instances with 32 / 8-hop walks: 3 best, profiles/r5/retune_busy_ab.txt)
  uint32_t prefetch_ext = 7;      // TSW_PREFETCH_EXT: bit 0 DAG from an agent's own unresolved cell, bit 1 walk past the pickup, bit 2 walk-ahead for agents a firing changed (C3 476 -> 409 ms with bits 0-1)
  bool flinks_lds = true;         // TSW_NO_FLINKS_LDS: pointer-doubling buffers stay global
  uint32_t part_lds = 0x7F;       // TSW_PART_LDS: PART_* agent arrays allowed in LDS one by one (tsw_plan.h)
  bool occ_split = true;          // TSW_OCC_SPLIT=0: the occupancy grid goes to LDS only together with MU
  uint32_t plan_block = 0;        // TSW_PLAN_BLOCK: k_plan workgroup size (0 = auto)
  bool plan_debug = false;        // TSW_PLAN_DEBUG: k_plan sub-phase ticks printed per plan
  bool coop = true;               // TSW_COOP=0: K3 as host-launched passes at planner exits (round-1 mode)
  bool task_chains = true;        // TSW_TASK_CHAINS=0: no task-chain jobs for the coop workers
  bool avoid_xcc = true;          // TSW_WORKER_AVOID_XCD=0: coop workers also run on the planner's XCD
  bool chain_preempt = true;      // TSW_CHAIN_PREEMPT=0: chain workers finish a chain before serving queued pairs
  int worker_gs = -1;             // TSW_WORKER_GS: coop workers' g-score placement (0 global, 1 LDS u32, 2 LDS bytes)
  int worker_fb = -1;             // TSW_WORKER_FB=0 / 1: global-g-score workers without / with the staged free bitmap (-1: by waves per CU)
  bool dag_exit = true;           // TSW_DAG_EXIT=0: coop workers' A* runs to the goal's pop (no DAG early exit)
  uint32_t dag_mask = 0;          // TSW_DAG_MASK: the DAG early-exit test runs every (mask + 1) pops (0: auto)
  uint32_t ab_flags = 0;          // TSW_AB_FLAGS (A/B): 1 no 2-cycle fast path, 2 no end-of-rules prefetch, 4 one agent per K4 batch, 8 no batched rules walks
  uint32_t t0_delay_us = 0;       // TSW_T0_DELAY_US (A/B): the planner idles this long after step 0's assignment
  uint32_t stale_steps = 16;      // TSW_SPEC_STALE: coop workers drop speculative pairs older than this many steps (0: never)
  uint32_t reg_heap = 63;         // TSW_ASTAR_REGHEAP: worker A* heaps up to this many entries in registers (0: LDS only)
  // idle-worker polling (tsw_worker.h worker_claim; profiles/r4/poll_ab.txt: C3 371-383 -> 355 ms)
  int chain_mask = -1;            // TSW_CHAIN_MASK: workers with (wid & mask) == mask walk task chains (-1: all)
  uint32_t wake_gate = 2;         // TSW_WAKE_GATE: log2 of the fast-poller subsets a publish rotates over (0: all)
  uint32_t slow_poll = 4;         // TSW_SLOW_POLL: log2 of 1 / (fraction of idle workers polling at full rate) (0: all)
  uint32_t slow_mult = 256;       // TSW_SLOW_MULT: the others' poll interval multiplier
  uint64_t worker_idle_us = 5000000;  // TSW_WORKER_IDLE_US: an idle coop worker exits after this long (test knob)

  static Tunables from_env() {
    Tunables t;
#ifdef TSW_DIAG
    auto num = [](const char* k, long lo, long hi, long def) -> long {
      const char* v = getenv(k);
      if (!v) return def;
      return std::max(lo, std::min(hi, atol(v)));
    };
    if (const char* m = getenv("TSW_BFS_KERNEL"))
      t.bfs_mode = !strcmp(m, "wave") ? 1u : !strcmp(m, "block") ? 2u : !strcmp(m, "blk") ? 3u : !strcmp(m, "big") ? 4u : !strcmp(m, "mg") ? 5u : 0u;
    t.bfs_cap = (uint32_t)num("TSW_BFS_LISTCAP", 1, 32768, t.bfs_cap);
    t.blk_cap = (uint32_t)num("TSW_BFS_BLKCAP", 1, 32768, t.blk_cap);
    t.bfs_waves = (uint32_t)num("TSW_BFS_WAVES", 1, 16, t.bfs_waves);
    t.bfs_order = num("TSW_BFS_ORDER", 0, 1, 1) != 0;
    t.bfs_prof = getenv("TSW_BFS_PROF") != nullptr;
    t.bfs_nostage = getenv("TSW_BFS_NOSTAGE") != nullptr;
    t.bfs_dbg = (uint32_t)num("TSW_BFS_DBG", 0, 7, 0);
    t.bfs_wls = (uint32_t)num("TSW_BFS_WLS", 0, 1, t.bfs_wls);
    t.bfs_pair = (uint32_t)num("TSW_BFS_PAIR", 0, 1, t.bfs_pair);
    t.wave_hcap = (uint32_t)num("TSW_ASTAR_WAVE_HCAP", 4, 1 << 20, 0);
    t.astar_global_gs = (int)num("TSW_ASTAR_GLOBAL_GS", 0, 1, -1);
    t.astar_tier2 = getenv("TSW_ASTAR_NO_TIER2") == nullptr;
    t.astar_diag = (getenv("TSW_ASTAR_SERIAL") ? ASTAR_DIAG_SERIAL : 0u) | (getenv("TSW_ASTAR_PROF") ? ASTAR_DIAG_PROF : 0u);
    t.prefetch = getenv("TSW_NO_PREFETCH") == nullptr;
    t.wave_rules_max = (uint32_t)num("TSW_WAVE_RULES_MAX", 0, 0xFFFFFFFFl, t.wave_rules_max);
    t.walk_cap = (uint32_t)num("TSW_WALK_CAP", 0, 4096, t.walk_cap);
    t.wide_prefetch = (uint32_t)num("TSW_WIDE_PREFETCH", 0, 1 << 16, t.wide_prefetch);
    t.wide_hi = (uint32_t)num("TSW_WIDE_HI", 0, 1 << 16, t.wide_hi);
    t.wide_lo = (uint32_t)num("TSW_WIDE_LO", 1, 1 << 16, t.wide_lo);
    t.dag_prefetch = (uint32_t)num("TSW_DAG_PREFETCH", 0, 16, t.dag_prefetch);
    t.dag_width = (uint32_t)num("TSW_DAG_WIDTH", 1, 16, t.dag_width);
    t.urgent_hops = (uint32_t)num("TSW_URGENT_HOPS", 0, 16, t.urgent_hops);
    t.chain_hops = (uint32_t)num("TSW_CHAIN_HOPS", 0, 1000000, t.chain_hops);
    t.hot_chains = num("TSW_HOT_CHAINS", 0, 1, t.hot_chains ? 1 : 0) != 0;
    t.predict = (uint32_t)num("TSW_PREDICT", 0, 3, t.predict);
    t.walk_cache = num("TSW_WALK_CACHE", 0, 1, 1) != 0;
    t.move_round0 = (uint32_t)num("TSW_MOVE_ROUND0", 0, 0x7FFFFFFF, 0);
    t.ab_flags = (uint32_t)num("TSW_AB_FLAGS", 0, 255, t.ab_flags);
    t.t0_delay_us = (uint32_t)num("TSW_T0_DELAY_US", 0, 10000000, t.t0_delay_us);
    t.prefetch_ext = (uint32_t)num("TSW_PREFETCH_EXT", 0, 7, t.prefetch_ext);
    t.flinks_lds = getenv("TSW_NO_FLINKS_LDS") == nullptr;
    t.part_lds = (uint32_t)num("TSW_PART_LDS", 0, 0x7F, t.part_lds);
    t.occ_split = num("TSW_OCC_SPLIT", 0, 1, 1) != 0;
    t.plan_block = (uint32_t)num("TSW_PLAN_BLOCK", 0, PLAN_BLOCK_MAX, 0) / 64u * 64u;
    t.plan_debug = getenv("TSW_PLAN_DEBUG") != nullptr;
    t.coop = num("TSW_COOP", 0, 1, 1) != 0;
    t.task_chains = num("TSW_TASK_CHAINS", 0, 1, 1) != 0;
    t.chain_preempt = num("TSW_CHAIN_PREEMPT", 0, 1, 1) != 0;
    t.avoid_xcc = num("TSW_WORKER_AVOID_XCD", 0, 1, 1) != 0;
    t.worker_gs = (int)num("TSW_WORKER_GS", -1, 2, -1);
    t.worker_fb = (int)num("TSW_WORKER_FB", -1, 1, -1);
    t.dag_exit = num("TSW_DAG_EXIT", 0, 1, 1) != 0;
    t.dag_mask = (uint32_t)num("TSW_DAG_MASK", 0, 0x7FFFFFFF, t.dag_mask);
    t.stale_steps = (uint32_t)num("TSW_SPEC_STALE", 0, 1 << 20, t.stale_steps);
    t.reg_heap = (uint32_t)num("TSW_ASTAR_REGHEAP", 0, 63, t.reg_heap);
    t.wake_gate = (uint32_t)num("TSW_WAKE_GATE", 0, 8, t.wake_gate);
    t.chain_mask = (int)num("TSW_CHAIN_MASK", -1, 15, -1);
    t.slow_poll = (uint32_t)num("TSW_SLOW_POLL", 0, 8, t.slow_poll);
    t.slow_mult = (uint32_t)num("TSW_SLOW_MULT", 1, 1024, t.slow_mult);
    t.worker_idle_us = (uint64_t)num("TSW_WORKER_IDLE_US", 1, 5000000, (long)t.worker_idle_us);
#endif
    return t;
  }
};

}  // namespace

struct tsw_ctx {
  int device = 0;
  hipStream_t s = nullptr;
  std::string err;
  uint32_t flags = 0;
  Tunables tun;
  DevGrid G{};
  std::vector<uint8_t> h_nbmask;
  uint8_t* d_nbmask = nullptr;
  uint32_t* d_freebits = nullptr;
  int max_lds = 65536, num_cu = 256;
  // K1 v2 (k_bfs_wave) padded grid + per-wave scratch
  uint32_t Wp = 0, npw = 0;
  uint32_t* d_frp = nullptr;
  // K1 v3 (k_bfs_blk) 8x8-block grid
  uint32_t BW = 0, BH = 0, Bp = 0, nbp = 0;
  uint64_t* d_frb = nullptr;
  uint32_t* d_abase = nullptr;  // k_bfs_blk run-start numbering
  uint32_t nrs = 0;
  uint32_t nfree = 0;                   // free cells (k_bfs_mg: u16 levels need <= 65535)
  // K1 v5 (k_bfs_mg): goal groups of the current launch order (bfs_order), per-workgroup scratch
  std::vector<uint32_t> h_mg_grp;
  uint32_t* d_mg_grp = nullptr;
  size_t mg_grp_cap = 0;
  uint32_t* d_mg_wl = nullptr;
  uint16_t* d_mg_anch = nullptr;
  uint32_t mg_wgs = 0;
  unsigned long long* d_wlg = nullptr;  // k_bfs_blk per-wave WL scratch
  uint64_t wlg_waves = 0;
  uint16_t* d_anch = nullptr;
  uint16_t* d_lovf = nullptr;
  uint64_t wave_scratch = 0;
  size_t scratch_words = 0, scratch_lwords = 0;
  unsigned long long* d_bprof = nullptr;  // TSW_BFS_PROF=1: k_bfs_wave cycle split, printed per launch

  // goal-table store: slots 0 .. tab_count-1 have been handed out at least once; a slot is live
  // iff h_tab_goal[slot] != NO_GOAL. Slots of evicted tables sit on tab_free for reuse.
  uint64_t tstride = 0;
  uint32_t tab_cap = 0, tab_count = 0, tab_live = 0;
  uint8_t* d_dt = nullptr;       // detour bytes per (slot, cell) (tsw_internal.h), 1 B / cell / goal
  uint8_t* d_nh = nullptr;       // next-hop codes per (slot, cell), 1 B / cell / goal
  uint16_t* d_ktmp = nullptr;    // K1 output of one build batch (u16 tables, tstride each), classified into the store
  size_t ktmp_tabs = 0;
  int32_t* d_goal_tab = nullptr;
  std::vector<int32_t> h_goal_tab;
  std::vector<uint32_t> h_tab_goal;
  std::vector<uint64_t> h_tab_stamp;  // call counter of the slot's last use (LRU eviction)
  // 1: the slot's goal is farther than u16 distances reach from some cell (K1 overflow): it is kept
  // WITHOUT a distance table (all TSW_DIST_INF) and every next hop toward it comes from the exact
  // A* (K3, 20-bit g) — get_path's usize g-scores (tswap.rs:288-390) have no such limit
  std::vector<uint8_t> h_tab_tableless;
  uint8_t* d_govf = nullptr;  // K1 per-goal overflow flags
  size_t govf_cap = 0;
  std::vector<uint32_t> tab_free;
  uint64_t call_stamp = 0;
  uint64_t table_budget = 0;
  uint64_t evictions = 0;

  // A* scratch
  uint32_t nslots = 0, hcap = 0;
  uint64_t* d_heaps = nullptr;
  uint32_t* d_gs = nullptr;
  uint32_t* d_epochs = nullptr;
  uint32_t nslots16 = 0;  // LDS-heap A* (small grids)
  uint16_t* d_gs16 = nullptr;
  uint32_t* d_ep16 = nullptr;
  AstarQuery* d_ovf = nullptr;
  AstarQuery* d_ovf2 = nullptr;  // second-tier overflow list (same capacity as d_ovf)
  std::vector<uint32_t> h_lpt_goals, h_lpt_slots;  // K1 launch-order staging (bfs_lpt_order)
  size_t ovf_cap = 0;

  // query queue
  AstarQuery* d_Q = nullptr;
  size_t qcap = 0;
  uint8_t* d_res = nullptr;
  int32_t* d_lens = nullptr;
  size_t rescap = 0;

  // coop mode: K3 workers in the plan dispatch beside the planner (control block, queues)
  CoopCtl* d_cc = nullptr;
  CoopCtl* h_cc = nullptr;       // pinned
  AstarQuery* d_QS = nullptr;
  size_t qscap = 0;
  AstarQuery* d_QT = nullptr;    // task chains of the current plan (host-filled)
  AstarQuery* d_QH = nullptr;    // hot task chains (planner-filled at assignment), one slot per task
  size_t qhcap = 0;
  uint2* d_QP = nullptr;         // predicted task chains (planner-filled at pickups), PlanArgs::QP
  size_t qpcap = 0;
  uint32_t* d_pred = nullptr;    // TSW_PLAN_DEBUG: per-agent last predicted task
  uint4* d_wf = nullptr;         // per-agent walk-ahead frontier (PlanArgs::wf)
  size_t wfcap = 0;
  size_t predcap = 0;
  size_t qtcap = 0;
  uint32_t qt_count = 0;
  uint32_t* h_flags = nullptr;   // pinned, coherent: [0] planner resident, [1] abort, [2] heartbeat, [8..23] PBAR
  uint32_t* d_flags = nullptr;
  uint64_t coop_aborts = 0;
  uint32_t watchdog_ms = 10000;  // tsw_opts.watchdog_ms
  // tsw_plan_mapd_resolved: the caller resolves the exit batches (exit mode, lazy next hops)
  tsw_resolve_fn resolver = nullptr;
  void* resolver_user = nullptr;

  DevStatus* d_stat = nullptr;
  DevStatus* h_stat = nullptr;   // pinned, D2H
  PlanCtl* d_ctl = nullptr;
  PlanCtl* h_ctl = nullptr;      // pinned
  PlanArgs* d_pargs = nullptr;  // k_plan reads its arguments from here
  unsigned long long* d_ticks = nullptr;
  uint32_t* d_dtag = nullptr;  // TSW_PLAN_DEBUG: per-agent change tags (PlanArgs::dtag)
  uint32_t dtag_cap = 0;
  int wall_khz = 100000;
  uint32_t chase_id = 0;

  // agents
  size_t acap = 0;
  uint32_t *d_v = nullptr, *d_g = nullptr, *d_cnt = nullptr, *d_succ = nullptr, *d_ap = nullptr;
  int32_t* d_gt = nullptr;
  uint8_t* d_dec = nullptr;
  uint8_t* d_onc = nullptr;
  uint8_t* d_candc = nullptr;
  uint32_t* d_f1 = nullptr;
  uint32_t* d_f2 = nullptr;
  uint64_t* d_mu = nullptr;
  uint32_t* d_dups = nullptr;
  uint32_t* h_dups = nullptr;  // pinned
  uint8_t* d_st = nullptr;
  int32_t* d_task = nullptr;
  uint32_t* d_occ = nullptr;
  uint8_t* d_nhc = nullptr;
  // tasks
  size_t tcap = 0;
  uint32_t *d_live = nullptr, *d_pick = nullptr, *d_dlv = nullptr, *d_unused = nullptr;
  // K4 spatial index (PlanArgs::klt / kpos / kbox / kcnt), rebuilt by every plan call
  uint32_t *d_klt = nullptr, *d_kpos = nullptr, *d_kcnt = nullptr;
  uint2* d_kbox = nullptr;
  size_t kcap = 0, kchcap = 0;
  uint32_t kchunks = 0;
  // records
  uint64_t* d_rec = nullptr;
  size_t rec_cap = 0;
  uint32_t* d_grec = nullptr;
  size_t grec_cap = 0;
  // temporaries
  uint32_t *d_tmp_a = nullptr, *d_tmp_b = nullptr, *d_tmp_c = nullptr;
  size_t tmp_cap = 0;

  // stats / timing
  tsw_stats st{};
  bool timing = true;
  struct Ev {
    int cat;
    hipEvent_t a, b;
  };
  std::vector<Ev> pending;
  std::vector<hipEvent_t> pool;
};

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      c->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);             \
      return TSW_EHIP;                                                                \
    }                                                                                 \
  } while (0)

#define RET(code, msg)   \
  do {                   \
    c->err = (msg);      \
    return (code);       \
  } while (0)

// a tsw_plan_mapd_resolved resolver must not call back into the planning context (its
// queue, result buffers and table store are in use by the suspended plan): every entry point that
// touches the context refuses such a call.
#define NOT_FROM_RESOLVER(c)                                                                         \
  do {                                                                                               \
    if ((c)->resolver) RET(TSW_EINVAL, "re-entrant call on a context inside its own next-hop resolver"); \
  } while (0)

// build provenance (tsw_build_id): first 16 hex digits of the sha1 of the sources, set by the build
#ifndef TSW_SRC_HASH
#define TSW_SRC_HASH 0ull
#endif

#define TRY(expr)            \
  do {                       \
    int r_ = (expr);         \
    if (r_ != TSW_OK) return r_; \
  } while (0)

namespace {

template <class T>
hipError_t dgrow(T*& p, size_t& cap, size_t need) {
  if (need <= cap && p) return hipSuccess;
  if (p) {
    hipError_t e = hipFree(p);
    if (e != hipSuccess) return e;
  }
  p = nullptr;
  size_t nc = std::max<size_t>(need, std::max<size_t>(cap + cap / 2, 16));
  hipError_t e = hipMalloc(&p, nc * sizeof(T));
  if (e != hipSuccess) {
    cap = 0;
    p = nullptr;
    return e;
  }
  cap = nc;
  return hipSuccess;
}

hipEvent_t ev_get(tsw_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

struct Timer {
  tsw_ctx* c;
  int cat;
  hipEvent_t a = nullptr, b = nullptr;
  Timer(tsw_ctx* c_, int cat_) : c(c_), cat(cat_) {
    if (c->timing) {
      a = ev_get(c);
      b = ev_get(c);
      hipEventRecord(a, c->s);
    }
  }
  ~Timer() {
    if (a) {
      hipEventRecord(b, c->s);
      c->pending.push_back({cat, a, b});
    }
  }
};

void resolve_timing(tsw_ctx* c) {
  if (c->pending.empty()) return;
  hipEventSynchronize(c->pending.back().b);
  for (auto& e : c->pending) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, e.a, e.b);
    switch (e.cat) {
      case CAT_BFS: c->st.bfs_ms += ms; break;
      case CAT_ASTAR: c->st.astar_ms += ms; break;
      case CAT_WALK: c->st.walker_ms += ms; break;
      case CAT_ASSIGN: c->st.assign_ms += ms; break;
    }
    c->pool.push_back(e.a);
    c->pool.push_back(e.b);
  }
  c->pending.clear();
}

int set_device(tsw_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return TSW_OK;
}

bool cell_ok(const tsw_ctx* c, uint32_t x, uint32_t y, uint32_t* cell) {
  if (x >= c->G.W || y >= c->G.H) return false;
  const uint32_t cc = y * c->G.W + x;
  if (!(c->h_nbmask[cc] & NB_FREE)) return false;
  *cell = cc;
  return true;
}

bool cell_id_ok(const tsw_ctx* c, uint32_t cell) {
  return cell < c->G.ncell && (c->h_nbmask[cell] & NB_FREE);
}

int ensure_tmp(tsw_ctx* c, size_t k) {
  if (k <= c->tmp_cap && c->d_tmp_a) return TSW_OK;
  size_t ca = c->tmp_cap, cb = c->tmp_cap;
  HIPCHK(hipStreamSynchronize(c->s));
  size_t cc = c->tmp_cap;
  HIPCHK(dgrow(c->d_tmp_a, ca, k));
  HIPCHK(dgrow(c->d_tmp_b, cb, k));
  HIPCHK(dgrow(c->d_tmp_c, cc, k));
  c->tmp_cap = std::min(ca, std::min(cb, cc));
  return TSW_OK;
}

// K1 output buffer of a table-build batch: u16 tables of KTMP_BYTES at most (C5's 2 MiB tables: 1,024
// goals per batch), at least one table. Returns the batch size in tables.
constexpr size_t KTMP_BYTES = (size_t)2 << 30;
int ensure_ktmp(tsw_ctx* c, size_t want, size_t* batch) {
  const size_t per = (size_t)c->tstride * 2u;
  const size_t b = std::max<size_t>(1, std::min(want, KTMP_BYTES / per));
  if (c->ktmp_tabs < b || !c->d_ktmp) {
    HIPCHK(hipStreamSynchronize(c->s));
    if (c->d_ktmp) HIPCHK(hipFree(c->d_ktmp));
    c->d_ktmp = nullptr;
    c->ktmp_tabs = 0;
    HIPCHK(hipMalloc(&c->d_ktmp, b * per));
    c->ktmp_tabs = b;
  }
  *batch = b;
  return TSW_OK;
}

// K1 launch order: longest BFS first. A goal's level count is its eccentricity; the distance
// to the farthest grid corner bounds it and ranks goals well enough that the work queue's last
// wave of goals is the short ones (LPT scheduling) instead of a few long ones running on an
// otherwise idle chip. Output positions are carried in `slots`. TSW_BFS_ORDER=0 keeps the
// caller's order (A/B).
// k_bfs_mg serves this launch: selected explicitly (TSW_BFS_KERNEL=mg, diagnostic build — measured
// 5.5 ms vs k_bfs_blk's 2.7 ms on den520d's 10k goals), its LDS layout fits and the
// levels fit u16 (<= 65535 free cells)
bool mg_selected(const tsw_ctx* c, size_t k) {
  (void)k;
  if (c->tun.bfs_mode != 5u) return false;
  if (c->nfree > 0xFFFFu || c->nbp > 0xFFFFu || c->max_lds <= 0) return false;
  return bfs_mg_lds_bytes(c->G.W, c->G.H, c->nbp) <= (size_t)c->max_lds;
}

uint32_t morton2(uint32_t x, uint32_t y) {
  uint32_t z = 0;
  for (uint32_t b = 0; b < 16u; ++b) z |= ((x >> b) & 1u) << (2u * b) | ((y >> b) & 1u) << (2u * b + 1u);
  return z;
}

// k_bfs_mg launch order: goals grouped by (cell parity, Morton order) into groups of <= 16 (one
// parity per group: the kernel advances all of a group's fronts on one checkerboard colour per
// level), groups ordered longest-first by the eccentricity bound of their first goal (LPT, as
// bfs_lpt_order). Fills c->h_mg_grp with the group offsets.
void bfs_mg_order(tsw_ctx* c, std::vector<uint32_t>& goals, std::vector<uint32_t>& slots) {
  const uint32_t W = c->G.W, H = c->G.H;
  const size_t k = goals.size();
  std::vector<std::pair<uint64_t, uint32_t>> key(k);
  for (size_t i = 0; i < k; ++i) {
    const uint32_t y = goals[i] / W, x = goals[i] - y * W;
    key[i] = {((uint64_t)((x + y) & 1u) << 40) | morton2(x, y), (uint32_t)i};
  }
  std::sort(key.begin(), key.end());
  std::vector<std::pair<uint32_t, uint32_t>> grp;  // (start, end) in key order
  for (size_t i = 0; i < k;) {
    size_t j = i + 1;
    while (j < k && j - i < 16u && (key[j].first >> 40) == (key[i].first >> 40)) ++j;
    grp.push_back({(uint32_t)i, (uint32_t)j});
    i = j;
  }
  auto ecc = [&](uint32_t g) {
    const uint32_t y = g / W, x = g - y * W;
    return std::max(x, W - 1 - x) + std::max(y, H - 1 - y);
  };
  std::stable_sort(grp.begin(), grp.end(), [&](const auto& a, const auto& b) {
    return ecc(goals[key[a.first].second]) > ecc(goals[key[b.first].second]);
  });
  std::vector<uint32_t> g2, s2;
  g2.reserve(k);
  s2.reserve(k);
  c->h_mg_grp.assign(1, 0u);
  for (const auto& gr : grp) {
    for (uint32_t i = gr.first; i < gr.second; ++i) {
      g2.push_back(goals[key[i].second]);
      s2.push_back(slots[key[i].second]);
    }
    c->h_mg_grp.push_back((uint32_t)g2.size());
  }
  goals.swap(g2);
  slots.swap(s2);
}

void bfs_lpt_order(tsw_ctx* c, std::vector<uint32_t>& goals, std::vector<uint32_t>& slots) {
  c->h_mg_grp.clear();
  if (mg_selected(c, goals.size())) {
    bfs_mg_order(c, goals, slots);
    return;
  }
  if (!c->tun.bfs_order || goals.size() < 2) return;
  const uint32_t W = c->G.W, H = c->G.H, maxe = W + H;
  // counting sort by eccentricity bound, descending, stable: O(k + W + H) on the host
  std::vector<uint32_t> cnt(maxe + 1u, 0u), ecc(goals.size());
  for (size_t i = 0; i < goals.size(); ++i) {
    const uint32_t y = goals[i] / W, x = goals[i] - y * W;
    ecc[i] = maxe - (std::max(x, W - 1 - x) + std::max(y, H - 1 - y));
    ++cnt[ecc[i]];
  }
  uint32_t acc = 0;
  for (uint32_t e = 0; e <= maxe; ++e) {
    const uint32_t t = cnt[e];
    cnt[e] = acc;
    acc += t;
  }
  std::vector<uint32_t> g2(goals.size()), s2(goals.size());
  for (size_t i = 0; i < goals.size(); ++i) {
    const uint32_t j = cnt[ecc[i]]++;
    g2[j] = goals[i];
    s2[j] = slots[i];
  }
  goals.swap(g2);
  slots.swap(s2);
}

// A* scratch slots (global g-scores + overflow heap, one per K3 wave), allocated for the waves that run:
// `need` slots (0: what a host-launched K3 pass uses, astar_wave_slots), grown on demand, at least 64 and
// at most 4,096 / a 32 GB cap. A coop dispatch asks for exactly its worker waves (C5's
// 2,295 workers x 4.5 MB = 10.3 GB instead of a fixed 20 GB budget).
int ensure_astar_scratch(tsw_ctx* c, uint32_t need = 0) {
  const uint64_t ncell = c->G.ncell;
  const uint32_t hcap = (uint32_t)std::min<uint64_t>(4ull * ncell + 8ull, 1ull << 16);
  const uint64_t per_slot = (uint64_t)hcap * 8ull + ncell * 4ull;
  if (need == 0)
    need = std::max(astar_wave_slots(c->G, c->num_cu, true), astar_wave_slots(c->G, c->num_cu, false));
  const uint64_t cap = std::max<uint64_t>(64, std::min<uint64_t>((32ull << 30) / per_slot, 4096));
  const uint32_t ns = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(need, 64), cap);
  if (c->d_heaps && ns <= c->nslots) return TSW_OK;
  HIPCHK(hipStreamSynchronize(c->s));
  if (c->d_heaps) HIPCHK(hipFree(c->d_heaps));
  if (c->d_gs) HIPCHK(hipFree(c->d_gs));
  if (c->d_epochs) HIPCHK(hipFree(c->d_epochs));
  c->d_heaps = nullptr;
  c->d_gs = nullptr;
  c->d_epochs = nullptr;
  c->nslots = 0;
  c->hcap = hcap;
  HIPCHK(hipMalloc(&c->d_heaps, (size_t)ns * c->hcap * 8ull));
  HIPCHK(hipMalloc(&c->d_gs, (size_t)ns * ncell * 4ull));
  // every initialisation goes on the context's (non-blocking) stream: a legacy
  // hipMemset is not ordered before kernels on c->s and recycled memory leaks through
  HIPCHK(hipMemsetAsync(c->d_gs, 0, (size_t)ns * ncell * 4ull, c->s));
  HIPCHK(hipMalloc(&c->d_epochs, (size_t)ns * 4ull));
  HIPCHK(hipMemsetAsync(c->d_epochs, 0, (size_t)ns * 4ull, c->s));
  c->nslots = ns;
  return TSW_OK;
}

int ensure_queue(tsw_ctx* c, size_t need) {
  if (need <= c->qcap && c->d_Q) return TSW_OK;
  HIPCHK(hipStreamSynchronize(c->s));
  HIPCHK(dgrow(c->d_Q, c->qcap, need));
  return TSW_OK;
}

int ensure_res(tsw_ctx* c, size_t need) {
  if (need <= c->rescap && c->d_res) return TSW_OK;
  HIPCHK(hipStreamSynchronize(c->s));
  size_t a = c->rescap, b = c->rescap;
  HIPCHK(dgrow(c->d_res, a, need));
  HIPCHK(dgrow(c->d_lens, b, need));
  c->rescap = std::min(a, b);
  return TSW_OK;
}

int check_err(tsw_ctx* c) {
  uint32_t e = 0;
  HIPCHK(hipMemcpyAsync(&c->h_stat->err, &c->d_stat->err, 4, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  e = c->h_stat->err;
  if (e) {
    char buf[160];
    snprintf(buf, sizeof buf, "device error bits 0x%x (1 heap overflow, 2 dist overflow, 4 g overflow, 8 no table)",
             e);
    c->err = buf;
    HIPCHK(hipMemsetAsync(&c->d_stat->err, 0, 4, c->s));
    return (e & (ERR_HEAP_OVERFLOW | ERR_DIST_OVERFLOW | ERR_G_OVERFLOW)) ? TSW_EOVERFLOW : TSW_EINVAL;
  }
  return TSW_OK;
}

// Run K3 over the queued queries until none are left (eager next hops).
// K3 over nq queued queries (device array Q): LDS-heap kernel on small grids, with the
// global-heap kernel for the few whose heap outgrows LDS; global-heap kernel otherwise.
// res / lens (per-query answers, indexed by AstarQuery::out) only for queues the host filled itself
// (tsw_get_path_next): queues written by k_plan reuse `out` for a diagnostic enqueue timestamp in
// coop mode and are always run with res == lens == nullptr, writing codes into the tables.
int run_astar(tsw_ctx* c, const AstarQuery* Q, uint32_t nq, bool to_tables, uint8_t* res, int32_t* lens) {
  if (nq == 0) return TSW_OK;
  if ((res || lens) && to_tables) RET(TSW_EINVAL, "internal: per-query answers are not table writes");
  TRY(ensure_astar_scratch(c));
  Timer t(c, CAT_ASTAR);
  uint8_t* nh = to_tables ? c->d_nh : nullptr;
  if (astar_lds_ok(c->G)) {
    if (!c->d_gs16) {
      c->nslots16 = 65536;
      HIPCHK(hipMalloc(&c->d_gs16, (size_t)c->nslots16 * c->G.ncell * 2));
      HIPCHK(hipMemsetAsync(c->d_gs16, 0, (size_t)c->nslots16 * c->G.ncell * 2, c->s));
      HIPCHK(hipMalloc(&c->d_ep16, (size_t)c->nslots16 * 4));
      HIPCHK(hipMemsetAsync(c->d_ep16, 0, (size_t)c->nslots16 * 4, c->s));
    }
    if (nq > c->ovf_cap) {
      HIPCHK(hipStreamSynchronize(c->s));
      HIPCHK(dgrow(c->d_ovf, c->ovf_cap, nq));
    }
    HIPCHK(hipMemsetAsync(&c->d_stat->novf, 0, 4, c->s));
    HIPCHK(hipMemsetAsync(&c->d_stat->qnext, 0, 4, c->s));
    HIPCHK(launch_astar_lds(c->G, Q, nq, nh, c->tstride, res, lens, c->d_gs16, c->d_ep16, c->nslots16, c->d_ovf,
                            &c->d_stat->novf, &c->d_stat->qnext, c->s));
    HIPCHK(hipMemcpyAsync(&c->h_stat->novf, &c->d_stat->novf, 4, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    const uint32_t novf = c->h_stat->novf;
    if (novf)
      HIPCHK(launch_astar(c->G, c->d_ovf, nullptr, novf, novf, nh, c->tstride, res, lens, c->d_heaps, c->hcap,
                          c->d_gs, c->d_epochs, c->nslots, &c->d_stat->err, c->s));
  } else {
    // one query per wave, LDS heap; the g_score slots are shared with k_astar (same tag scheme)
    if (nq > c->ovf_cap || !c->d_ovf2) {
      HIPCHK(hipStreamSynchronize(c->s));
      size_t cap2 = c->ovf_cap;
      HIPCHK(dgrow(c->d_ovf, c->ovf_cap, nq));
      HIPCHK(dgrow(c->d_ovf2, cap2, c->ovf_cap));
    }
    HIPCHK(hipMemsetAsync(&c->d_stat->novf, 0, 8, c->s));   // novf, novf2
    HIPCHK(hipMemsetAsync(&c->d_stat->qnext, 0, 8, c->s));  // qnext, qnext2
    // g_scores in LDS cap residency (the byte words of a 510x220 grid are 112 KB: one wave per
    // CU). When the batch has more queries than LDS-resident waves, throughput wins: keep only
    // the heap in LDS and the g_scores in the global slots (3-4 waves per CU; wh10k prefix
    // 3.32 -> 2.68 s); a smaller batch is bound by its slowest query, where LDS g_scores are
    // faster per pop. TSW_ASTAR_GLOBAL_GS=0/1 forces either (A/B).
    const int ge = c->tun.astar_global_gs;
    const bool ggs = ge >= 0 ? ge != 0
                             : astar_wave_lds_gs(c->G) && nq > std::min(astar_wave_slots(c->G, c->num_cu), c->nslots);
    const uint32_t slots = std::min(astar_wave_slots(c->G, c->num_cu, ggs), c->nslots);
    HIPCHK(launch_astar_wave(c->G, Q, nq, nh, c->tstride, res, lens, c->d_gs, c->d_epochs, slots, c->d_ovf,
                             &c->d_stat->novf, c->tun.wave_hcap, ggs, c->s, &c->d_stat->qnext, c->tun.astar_diag));
    HIPCHK(hipMemcpyAsync(&c->h_stat->novf, &c->d_stat->novf, 4, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    uint32_t novf = c->h_stat->novf;
    AstarQuery* rest = c->d_ovf;
    if (novf && astar_wave_lds_gs(c->G) && c->tun.astar_tier2) {
      // second tier: g_scores that outgrew the LDS encoding (byte words: detours > 62) move to
      // the global u32 slots while the heap stays in LDS; only heap overflows reach k_astar
      const uint32_t slots2 = std::min(astar_wave_slots(c->G, c->num_cu, true), c->nslots);
      HIPCHK(launch_astar_wave(c->G, c->d_ovf, novf, nh, c->tstride, res, lens, c->d_gs, c->d_epochs, slots2,
                               c->d_ovf2, &c->d_stat->novf2, c->tun.wave_hcap, true, c->s, &c->d_stat->qnext2,
                               c->tun.astar_diag));
      HIPCHK(hipMemcpyAsync(&c->h_stat->novf2, &c->d_stat->novf2, 4, hipMemcpyDeviceToHost, c->s));
      HIPCHK(hipStreamSynchronize(c->s));
      novf = c->h_stat->novf2;
      rest = c->d_ovf2;
    }
    if (novf)
      HIPCHK(launch_astar(c->G, rest, nullptr, novf, novf, nh, c->tstride, res, lens, c->d_heaps, c->hcap,
                          c->d_gs, c->d_epochs, c->nslots, &c->d_stat->err, c->s));
  }
  c->st.astar_queries += nq;
  c->st.astar_launches++;
  return TSW_OK;
}

// Error path after pairs were marked NH_PENDING (queued for a K3 pass that did not complete):
// put every pending code of the store back to NH_UNKNOWN so later calls re-queue them instead of
// waiting on a pass that will never run. Returns rc (the original failure).
int reset_pending_after(tsw_ctx* c, int rc) {
  if (rc == TSW_OK || !c->d_nh || c->tab_count == 0) return rc;
  (void)hipStreamSynchronize(c->s);
  if (launch_reset_pending(c->d_nh, (uint64_t)c->tab_count * c->tstride, c->s) == hipSuccess)
    (void)hipStreamSynchronize(c->s);
  return rc;
}

int resolve_all_unknown_impl(tsw_ctx* c, const std::vector<uint32_t>& goals, const std::vector<uint32_t>& slots) {
  if (goals.empty()) return TSW_OK;
  TRY(ensure_astar_scratch(c));
  TRY(ensure_tmp(c, goals.size()));
  HIPCHK(hipMemcpyAsync(c->d_tmp_a, goals.data(), goals.size() * 4, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_tmp_b, slots.data(), slots.size() * 4, hipMemcpyHostToDevice, c->s));
  // one queue for every pair of the batch (eager_policy bounds it to 8M): a single K3 launch
  // gives each lane several queries, so the launch is not the longest query times the number
  // of 64k-query batches
  const size_t bound = std::min<size_t>((size_t)goals.size() * c->G.ncell, (size_t)1 << 23);
  TRY(ensure_queue(c, std::max<size_t>({c->qcap, (size_t)1 << 16, bound})));
  for (int iter = 0; iter < 1000000; ++iter) {
    HIPCHK(hipMemsetAsync(&c->d_stat->qcount, 0, 4, c->s));
    HIPCHK(launch_enqueue_unknown(c->G, c->d_tmp_a, c->d_tmp_b, (uint32_t)goals.size(), c->d_nh, c->tstride,
                                  c->d_Q, &c->d_stat->qcount, (uint32_t)c->qcap, c->s));
    HIPCHK(hipMemcpyAsync(&c->h_stat->qcount, &c->d_stat->qcount, 4, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    const uint32_t cnt = c->h_stat->qcount;
    if (cnt == 0) break;
    const uint32_t run = (uint32_t)std::min<size_t>(cnt, c->qcap);
    TRY(run_astar(c, c->d_Q, run, true, nullptr, nullptr));
    TRY(check_err(c));
    if (cnt <= c->qcap) break;
  }
  return TSW_OK;
}

int resolve_all_unknown(tsw_ctx* c, const std::vector<uint32_t>& goals, const std::vector<uint32_t>& slots) {
  return reset_pending_after(c, resolve_all_unknown_impl(c, goals, slots));
}

bool eager_policy(const tsw_ctx* c, size_t new_tables) {
  if ((c->flags & TSW_F_LAZY_NEXTHOP) || c->resolver) return false;
  if (c->flags & TSW_F_EAGER_NEXTHOP) return true;
  return c->G.ncell <= 4096 && (uint64_t)new_tables * c->G.ncell <= (8ull << 20);
}

// K1 over k goals (device arrays; slots may be null = goal index): the wave-per-goal kernel
// when its LDS fits, else the workgroup-per-goal kernel. Next-hop codes (nh != null) come
// fused from k_bfs, or from k_classify over the finished tables after k_bfs_wave.
// per-wave scratch of the wave-per-goal kernels: `words` u16 anchors + `lwords` u16 list overflow
int ensure_wave_scratch(tsw_ctx* c, uint64_t want, size_t words, size_t lwords) {
  if (want <= c->wave_scratch && words <= c->scratch_words && lwords <= c->scratch_lwords) return TSW_OK;
  want = std::max(want, c->wave_scratch);
  words = std::max(words, c->scratch_words);
  lwords = std::max(lwords, c->scratch_lwords);
  HIPCHK(hipStreamSynchronize(c->s));
  if (c->d_anch) HIPCHK(hipFree(c->d_anch));
  if (c->d_lovf) HIPCHK(hipFree(c->d_lovf));
  c->d_anch = nullptr;
  c->d_lovf = nullptr;
  c->wave_scratch = 0;
  HIPCHK(hipMalloc(&c->d_anch, (size_t)want * words * 2u));
  HIPCHK(hipMalloc(&c->d_lovf, (size_t)want * lwords * 2u));
  c->wave_scratch = want;
  c->scratch_words = words;
  c->scratch_lwords = lwords;
  return TSW_OK;
}

unsigned long long* bfs_prof_buf(tsw_ctx* c) {
  if (!c->tun.bfs_prof) return nullptr;
  if (!c->d_bprof && hipMalloc(&c->d_bprof, 8 * sizeof(unsigned long long)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(c->d_bprof, 0, 8 * sizeof(unsigned long long), c->s) != hipSuccess) return nullptr;
  return c->d_bprof;
}

int bfs_prof_print(tsw_ctx* c, const char* name, uint32_t k) {
  unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(h, c->d_bprof, sizeof h, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  fprintf(stderr, "[%s] goals %u  bfs %.0f cyc/goal  decode %.0f cyc/goal  levels %.1f/goal  chunks %.1f/goal"
          "  (mg: wave-cycles list+barrier %.0f, tasks %.0f per goal)\n",
          name, k, (double)h[0] / k, (double)h[1] / k, (double)h[2] / k, (double)h[3] / k, (double)h[4] / k,
          (double)h[5] / k);
  return TSW_OK;
}

// K1 over k goals (device arrays; slots may be null = goal index): the 8x8-block wave-per-goal
// kernel when its LDS fits, else the row-word wave-per-goal kernel, else the workgroup-per-goal
// kernel. Next-hop codes (nh != null) come fused from k_bfs, or from k_classify over the
// finished tables after the wave kernels.
int run_bfs(tsw_ctx* c, const uint32_t* goals, const uint32_t* slots, uint32_t k, uint16_t* dist, uint64_t dstride,
            uint8_t* nh, uint8_t* govf = nullptr) {
  if (k == 0) return TSW_OK;
  const bool vec16 = c->G.W % 8u == 0u && dstride % 8u == 0u && ((uintptr_t)dist & 15u) == 0u;
  const uint32_t max_waves = c->tun.bfs_waves;
  const uint32_t bfs_mode = c->tun.bfs_mode;
  if (mg_selected(c, k) && !c->h_mg_grp.empty() && c->h_mg_grp.back() == k) {
    // goal-bit-parallel groups (the launch order came from bfs_mg_order)
    Timer t(c, CAT_BFS);
    const uint32_t ngroups = (uint32_t)c->h_mg_grp.size() - 1u;
    const uint32_t wlw = (c->G.ncell + 1u) / 2u;
    const uint32_t wgs = (uint32_t)std::max(c->num_cu, 1);
    if (c->mg_wgs < wgs || !c->d_mg_wl) {
      HIPCHK(hipStreamSynchronize(c->s));
      if (c->d_mg_wl) HIPCHK(hipFree(c->d_mg_wl));
      if (c->d_mg_anch) HIPCHK(hipFree(c->d_mg_anch));
      c->d_mg_wl = nullptr;
      c->d_mg_anch = nullptr;
      c->mg_wgs = 0;
      HIPCHK(hipMalloc(&c->d_mg_wl, (size_t)wgs * wlw * 4u));
      HIPCHK(hipMalloc(&c->d_mg_anch, (size_t)wgs * std::max<uint32_t>(c->nrs, 1u) * 16u * 2u));
      c->mg_wgs = wgs;
    }
    if (c->h_mg_grp.size() > c->mg_grp_cap || !c->d_mg_grp) {
      HIPCHK(hipStreamSynchronize(c->s));
      HIPCHK(dgrow(c->d_mg_grp, c->mg_grp_cap, c->h_mg_grp.size()));
    }
    HIPCHK(hipMemcpyAsync(c->d_mg_grp, c->h_mg_grp.data(), c->h_mg_grp.size() * 4u, hipMemcpyHostToDevice, c->s));
    MgBfsArgs A{};
    A.W = c->G.W;
    A.H = c->G.H;
    A.Bp = c->Bp;
    A.nbp = c->nbp;
    A.bp_magic = (uint32_t)((0xFFFFFFFFull + c->Bp) / c->Bp);
    A.frb = c->d_frb;
    A.abase = c->d_abase;
    A.nrs = std::max<uint32_t>(c->nrs, 1u);
    A.goals = goals;
    A.slots = slots;
    A.grp = c->d_mg_grp;
    A.ngroups = ngroups;
    A.dist = dist;
    A.dstride = dstride;
    A.wl = c->d_mg_wl;
    A.wlw = wlw;
    A.anch = c->d_mg_anch;
    A.work = &c->d_stat->work;
    A.err = &c->d_stat->err;
    A.scratch_wgs = c->mg_wgs;
    A.prof = (uint64_t*)bfs_prof_buf(c);
    HIPCHK(hipMemsetAsync(&c->d_stat->work, 0, 4, c->s));
    HIPCHK(launch_bfs_mg(A, c->max_lds, c->num_cu, c->s));
    // the host copy of the group offsets must outlive the async upload
    HIPCHK(hipStreamSynchronize(c->s));
    if (A.prof) TRY(bfs_prof_print(c, "k_bfs_mg", k));
    if (nh) HIPCHK(launch_classify(c->G, goals, slots, k, dist, dstride, nh, c->s));
    return TSW_OK;
  }
  if (bfs_mode == 5) RET(TSW_EINVAL, "k_bfs_mg does not fit this grid (forced kernel mg)");
  uint32_t nbw = 0;
  // two goals per wave only where two goal slots per wave fit LDS, else one
  bool pair = c->tun.bfs_pair != 0u;
  if ((bfs_mode == 0 || bfs_mode == 3) && c->nbp <= 0x10000u) {
    nbw = std::min(max_waves, bfs_blk_waves_per_block(c->nbp, c->tun.blk_cap, c->max_lds, c->tun.bfs_wls != 0u, pair));
    if (nbw == 0 && pair) {
      pair = false;
      nbw = std::min(max_waves, bfs_blk_waves_per_block(c->nbp, c->tun.blk_cap, c->max_lds, c->tun.bfs_wls != 0u, false));
    }
  }
  if (nbw == 0 && bfs_mode == 3) RET(TSW_EINVAL, "k_bfs_blk does not fit this grid (forced kernel blk)");
  if (nbw > 0) {
    Timer t(c, CAT_BFS);
    // scratch per goal slot: one per wave, two with TSW_BFS_PAIR
    TRY(ensure_wave_scratch(c, (uint64_t)c->num_cu * nbw * (pair ? 2u : 1u), std::max<size_t>(c->nrs, 1),
                            (size_t)c->nbp * 2u));
    if (c->wlg_waves < c->wave_scratch) {
      HIPCHK(hipStreamSynchronize(c->s));
      if (c->d_wlg) HIPCHK(hipFree(c->d_wlg));
      c->d_wlg = nullptr;
      c->wlg_waves = 0;
      HIPCHK(hipMalloc(&c->d_wlg, (size_t)c->wave_scratch * c->nbp * 8u));
      c->wlg_waves = c->wave_scratch;
    }
    BlkBfsArgs A{};
    A.W = c->G.W;
    A.H = c->G.H;
    A.BW = c->BW;
    A.BH = c->BH;
    A.Bp = c->Bp;
    A.nbp = c->nbp;
    A.cap = c->tun.blk_cap;
    A.frb = c->d_frb;
    A.abase = c->d_abase;
    A.nrs = c->nrs;
    A.goals = goals;
    A.slots = slots;
    A.k = k;
    A.dist = dist;
    A.dstride = dstride;
    A.anch = c->d_anch;
    A.lovf = c->d_lovf;
    A.wlg = c->d_wlg;
    A.work = &c->d_stat->work;
    A.err = &c->d_stat->err;
    A.govf = govf;
    A.vec16 = vec16 ? 1u : 0u;
    A.stage = (dstride % 8u == 0u && ((uintptr_t)dist & 15u) == 0u && !c->tun.bfs_nostage) ? 1u : 0u;
    A.dbg = c->tun.bfs_dbg;
    A.wls = c->tun.bfs_wls;
    A.pair = pair ? 1u : 0u;
    A.max_waves = nbw;
    A.scratch_waves = std::min(c->wave_scratch, c->wlg_waves);
    A.prof = (uint64_t*)bfs_prof_buf(c);
    HIPCHK(hipMemsetAsync(&c->d_stat->work, 0, 4, c->s));
    HIPCHK(launch_bfs_blk(A, c->max_lds, c->num_cu, c->s));
    if (A.prof) TRY(bfs_prof_print(c, "k_bfs_blk", k));
    if (nh) HIPCHK(launch_classify(c->G, goals, slots, k, dist, dstride, nh, c->s));
    return TSW_OK;
  }
  uint32_t nwv = 0;
  if ((bfs_mode == 0 || bfs_mode == 1) && c->npw <= 0x8000u)
    nwv = bfs_wave_waves_per_block(c->npw, c->tun.bfs_cap, c->max_lds);
  if (nwv == 0 && bfs_mode == 1) RET(TSW_EINVAL, "k_bfs_wave does not fit this grid (forced kernel wave)");
  uint32_t big_cap = 0;
  if (nwv == 0 && (bfs_mode == 0 || bfs_mode == 4) && bfs_big_fits(c->nbp, c->max_lds, &big_cap)) {
    // large grids (e.g. 1024x1024): one workgroup per goal, shared visited bitmap in LDS
    Timer t(c, CAT_BFS);
    const uint32_t nwg = bfs_big_workgroups(c->nbp, big_cap, c->num_cu);
    TRY(ensure_wave_scratch(c, nwg, std::max<size_t>(c->nrs, 1), (size_t)c->nbp * 2u));
    if (c->wlg_waves < c->wave_scratch) {
      HIPCHK(hipStreamSynchronize(c->s));
      if (c->d_wlg) HIPCHK(hipFree(c->d_wlg));
      c->d_wlg = nullptr;
      c->wlg_waves = 0;
      HIPCHK(hipMalloc(&c->d_wlg, (size_t)c->wave_scratch * c->nbp * 8u));
      c->wlg_waves = c->wave_scratch;
    }
    BigBfsArgs A{};
    A.W = c->G.W;
    A.H = c->G.H;
    A.BW = c->BW;
    A.BH = c->BH;
    A.Bp = c->Bp;
    A.nbp = c->nbp;
    A.cap = big_cap;
    A.frb = c->d_frb;
    A.abase = c->d_abase;
    A.goals = goals;
    A.slots = slots;
    A.k = k;
    A.dist = dist;
    A.dstride = dstride;
    A.nrs = std::max<uint32_t>(c->nrs, 1u);
    A.anch = c->d_anch;
    A.lovf = c->d_lovf;
    A.wlg = reinterpret_cast<uint64_t*>(c->d_wlg);
    A.work = &c->d_stat->work;
    A.err = &c->d_stat->err;
    A.govf = govf;
    A.vec16 = vec16 ? 1u : 0u;
    A.scratch_wgs = (uint32_t)std::min<uint64_t>(c->wave_scratch, c->wlg_waves);
    HIPCHK(hipMemsetAsync(&c->d_stat->work, 0, 4, c->s));
    HIPCHK(launch_bfs_big(A, c->max_lds, c->num_cu, c->s));
    if (nh) HIPCHK(launch_classify(c->G, goals, slots, k, dist, dstride, nh, c->s));
    return TSW_OK;
  }
  if (bfs_mode == 4) RET(TSW_EINVAL, "k_bfs_big does not fit this grid (forced kernel big)");
  Timer t(c, CAT_BFS);
  if (nwv == 0) {
    HIPCHK(launch_bfs(c->G, goals, slots, k, dist, dstride, nh, dstride, &c->d_stat->err, c->max_lds, c->num_cu,
                      c->s, govf));
    return TSW_OK;
  }
  TRY(ensure_wave_scratch(c, (uint64_t)c->num_cu * nwv, (size_t)c->npw * 32u, (size_t)c->npw * 2u));
  WaveBfsArgs A{};
  A.W = c->G.W;
  A.H = c->G.H;
  A.Ww = c->G.Ww;
  A.Wp = c->Wp;
  A.npw = c->npw;
  A.cap = c->tun.bfs_cap;
  A.frp = c->d_frp;
  A.goals = goals;
  A.slots = slots;
  A.k = k;
  A.dist = dist;
  A.dstride = dstride;
  A.anch = c->d_anch;
  A.lovf = c->d_lovf;
  A.work = &c->d_stat->work;
  A.err = &c->d_stat->err;
  A.govf = govf;
  A.vec16 = vec16 ? 1u : 0u;
  A.max_waves = max_waves;
  A.scratch_waves = c->wave_scratch;
  A.prof = (uint64_t*)bfs_prof_buf(c);
  HIPCHK(hipMemsetAsync(&c->d_stat->work, 0, 4, c->s));
  HIPCHK(launch_bfs_wave(A, c->max_lds, c->num_cu, c->s));
  if (A.prof) TRY(bfs_prof_print(c, "k_bfs_wave", k));
  if (nh) HIPCHK(launch_classify(c->G, goals, slots, k, dist, dstride, nh, c->s));
  return TSW_OK;
}

constexpr uint32_t NO_GOAL = 0xFFFFFFFFu;

// Grow the device store to at least `need` slots (never past the budget; callers check).
int grow_store(tsw_ctx* c, size_t need) {
  if (need <= c->tab_cap) return TSW_OK;
  const uint64_t max_tabs = c->table_budget / (c->tstride * 2ull);
  size_t nc = std::max<size_t>(need, std::max<size_t>((size_t)c->tab_cap * 2, 64));
  nc = std::max<size_t>(need, std::min<size_t>(nc, (size_t)max_tabs));
  HIPCHK(hipStreamSynchronize(c->s));
  uint8_t* nd = nullptr;
  uint8_t* nn = nullptr;
  HIPCHK(hipMalloc(&nd, nc * c->tstride));
  if (hipError_t e = hipMalloc(&nn, nc * c->tstride); e != hipSuccess) {
    (void)hipFree(nd);
    RET(TSW_ENOMEM, std::string("table store growth: ") + hipGetErrorString(e));
  }
  if (c->tab_count) {
    HIPCHK(hipMemcpyAsync(nd, c->d_dt, (size_t)c->tab_count * c->tstride, hipMemcpyDeviceToDevice, c->s));
    HIPCHK(hipMemcpyAsync(nn, c->d_nh, (size_t)c->tab_count * c->tstride, hipMemcpyDeviceToDevice, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
  }
  if (c->d_dt) HIPCHK(hipFree(c->d_dt));
  if (c->d_nh) HIPCHK(hipFree(c->d_nh));
  c->d_dt = nd;
  c->d_nh = nn;
  c->tab_cap = (uint32_t)nc;
  c->h_tab_goal.resize(nc, NO_GOAL);
  c->h_tab_stamp.resize(nc, 0);
  c->h_tab_tableless.resize(nc, 0);
  return TSW_OK;
}

// Stamp the tables of `goals` as used by the current call and collect the goals that have none
// (deduplicated, marked -2 in h_goal_tab until committed or rolled back).
void stamp_and_collect(tsw_ctx* c, const uint32_t* goals, size_t k, std::vector<uint32_t>& newg,
                       std::vector<uint32_t>* src = nullptr) {
  ++c->call_stamp;
  for (size_t i = 0; i < k; ++i) {
    const uint32_t g = goals[i];
    const int32_t t = c->h_goal_tab[g];
    if (t >= 0) {
      c->h_tab_stamp[t] = c->call_stamp;
    } else if (t == -1) {
      c->h_goal_tab[g] = -2;
      newg.push_back(g);
      if (src) src->push_back((uint32_t)i);
    }
  }
}

// Slots for k new tables: free slots first, then growth up to the budget, then the least-recently
// used live tables that the current call does not use (LRU eviction — a long-running per-tick
// manager streams goals through a bounded store instead of failing, SURVEY §7 hard part 4).
// Evicted goals lose their table (goal_tab -1); later calls rebuild them on demand.
int reserve_slots(tsw_ctx* c, size_t k, std::vector<uint32_t>& slots) {
  slots.clear();
  const uint64_t max_tabs = c->table_budget / (c->tstride * 2ull);
  while (slots.size() < k && !c->tab_free.empty()) {
    slots.push_back(c->tab_free.back());
    c->tab_free.pop_back();
  }
  size_t want = k - slots.size();
  const size_t fresh = std::min<size_t>(want, max_tabs > c->tab_count ? (size_t)(max_tabs - c->tab_count) : 0u);
  if (fresh) {
    if (int r = grow_store(c, (size_t)c->tab_count + fresh); r != TSW_OK) {
      c->tab_free.insert(c->tab_free.end(), slots.begin(), slots.end());
      slots.clear();
      return r;
    }
    for (size_t j = 0; j < fresh; ++j) slots.push_back(c->tab_count++);
    want -= fresh;
  }
  if (want) {
    std::vector<uint32_t> cand;
    for (uint32_t s = 0; s < c->tab_count; ++s)
      if (c->h_tab_goal[s] != NO_GOAL && c->h_tab_stamp[s] < c->call_stamp) cand.push_back(s);
    if (cand.size() < want) {
      c->tab_free.insert(c->tab_free.end(), slots.begin(), slots.end());
      slots.clear();
      RET(TSW_ENOMEM, "goal-table budget exceeded by the goals of one call (raise tsw_opts.table_budget_bytes)");
    }
    std::partial_sort(cand.begin(), cand.begin() + want, cand.end(),
                      [&](uint32_t a, uint32_t b) { return c->h_tab_stamp[a] < c->h_tab_stamp[b]; });
    for (size_t j = 0; j < want; ++j) {
      const uint32_t s = cand[j];
      c->h_goal_tab[c->h_tab_goal[s]] = -1;
      c->h_tab_goal[s] = NO_GOAL;
      --c->tab_live;
      ++c->evictions;
      slots.push_back(s);
    }
  }
  return TSW_OK;
}

// Commit (rc == OK) or roll back the new goals and their reserved slots, then publish goal_tab.
int finish_tables(tsw_ctx* c, int rc, const std::vector<uint32_t>& newg, const std::vector<uint32_t>& slots) {
  for (size_t j = 0; j < newg.size(); ++j) {
    if (rc == TSW_OK && j < slots.size()) {
      c->h_goal_tab[newg[j]] = (int32_t)slots[j];
      c->h_tab_goal[slots[j]] = newg[j];
      c->h_tab_stamp[slots[j]] = c->call_stamp;
    } else {
      c->h_goal_tab[newg[j]] = -1;
    }
  }
  if (rc == TSW_OK) c->tab_live += (uint32_t)newg.size();
  else c->tab_free.insert(c->tab_free.end(), slots.begin(), slots.end());
  c->st.tables = c->tab_live;
  const std::string keep = c->err;
  if (hipMemcpyAsync(c->d_goal_tab, c->h_goal_tab.data(), (size_t)c->G.ncell * 4, hipMemcpyHostToDevice, c->s) !=
          hipSuccess ||
      hipStreamSynchronize(c->s) != hipSuccess) {
    if (rc == TSW_OK) RET(TSW_EHIP, "goal_tab upload failed");
  }
  c->err = keep;
  return rc;
}

// tableless_ok: a goal whose distances overflow u16 is registered WITHOUT a table (next hops by K3)
// instead of failing the call — planning entry points; the table-returning ones pass false.
int build_new_tables(tsw_ctx* c, const std::vector<uint32_t>& newg, const std::vector<uint32_t>& slots,
                     bool tableless_ok) {
  std::vector<uint32_t>& lg = c->h_lpt_goals;
  std::vector<uint32_t>& ls = c->h_lpt_slots;
  lg.resize(newg.size());
  ls.resize(newg.size());
  TRY(ensure_tmp(c, newg.size()));
  if (tableless_ok) {
    if (newg.size() > c->govf_cap || !c->d_govf) {
      HIPCHK(hipStreamSynchronize(c->s));
      HIPCHK(dgrow(c->d_govf, c->govf_cap, newg.size()));
    }
    HIPCHK(hipMemsetAsync(c->d_govf, 0, newg.size(), c->s));
  }
  // K1 in batches into the u16 buffer, each batch classified into the store (codes + detour bytes):
  // the u16 tables never live in the store (round 6: 3 -> 2 B per cell per goal; C5 79.5 -> ~57 GiB)
  // (launch order per batch: longest BFS first, bfs_lpt_order; lg / ls hold the ordered goals / store slots)
  size_t batch = 0;
  TRY(ensure_ktmp(c, newg.size(), &batch));
  for (size_t i0 = 0; i0 < newg.size(); i0 += batch) {
    const uint32_t nb = (uint32_t)std::min(batch, newg.size() - i0);
    std::vector<uint32_t> bg(newg.begin() + i0, newg.begin() + i0 + nb), bs(slots.begin() + i0, slots.begin() + i0 + nb);
    bfs_lpt_order(c, bg, bs);
    std::copy(bg.begin(), bg.end(), lg.begin() + i0);
    std::copy(bs.begin(), bs.end(), ls.begin() + i0);
    HIPCHK(hipMemcpyAsync(c->d_tmp_a + i0, lg.data() + i0, (size_t)nb * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_b + i0, ls.data() + i0, (size_t)nb * 4, hipMemcpyHostToDevice, c->s));
    TRY(run_bfs(c, c->d_tmp_a + i0, nullptr, nb, c->d_ktmp, c->tstride, nullptr,
                tableless_ok ? c->d_govf + i0 : nullptr));
    HIPCHK(launch_classify_dt(c->G, c->d_tmp_a + i0, nullptr, c->d_tmp_b + i0, nb, c->d_ktmp, c->tstride, c->d_nh,
                              c->d_dt, c->tstride, c->s));
    HIPCHK(hipStreamSynchronize(c->s));  // the host copies bg / bs and the mg group offsets are reused next batch
  }
  c->st.bfs_goals += newg.size();
  c->st.bfs_launches++;
  for (uint32_t s : slots) c->h_tab_tableless[s] = 0;
  HIPCHK(hipMemcpyAsync(&c->h_stat->err, &c->d_stat->err, 4, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  if (tableless_ok && c->h_stat->err == ERR_DIST_OVERFLOW) {
    std::vector<uint8_t> f(newg.size());
    HIPCHK(hipMemcpy(f.data(), c->d_govf, f.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < f.size(); ++i) {
      if (!f[i]) continue;
      const uint32_t slot = ls[i];
      c->h_tab_tableless[slot] = 1;
      ++c->st.tableless_goals;
      // no distance (DAG prefetch reads DT_NONE: nothing to follow) and every code unresolved (K3)
      HIPCHK(hipMemsetAsync(c->d_dt + (size_t)slot * c->tstride, 0xFF, c->tstride, c->s));
      HIPCHK(hipMemsetAsync(c->d_nh + (size_t)slot * c->tstride, 0xFF, c->tstride, c->s));
    }
    HIPCHK(hipMemsetAsync(&c->d_stat->err, 0, 4, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
  }
  return check_err(c);
}

// K1 of `goals` (host array) into u16 tables for an API that returns them: batches through the K1
// buffer, each batch handed to `take(device tables, first goal index, count)` (the store holds detour
// bytes only, tsw_internal.h).
template <class Take>
int build_u16(tsw_ctx* c, const uint32_t* goals, uint32_t k, Take&& take) {
  size_t batch = 0;
  TRY(ensure_ktmp(c, k, &batch));
  TRY(ensure_tmp(c, std::min<size_t>(k, batch)));
  for (uint32_t i0 = 0; i0 < k; i0 += (uint32_t)batch) {
    const uint32_t nb = (uint32_t)std::min<size_t>(batch, k - i0);
    // launch order longest-first (bfs_lpt_order); the slots carry each table's position in the batch
    std::vector<uint32_t> bg(goals + i0, goals + i0 + nb), bs(nb);
    for (uint32_t j = 0; j < nb; ++j) bs[j] = j;
    bfs_lpt_order(c, bg, bs);
    HIPCHK(hipMemcpyAsync(c->d_tmp_a, bg.data(), (size_t)nb * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_b, bs.data(), (size_t)nb * 4, hipMemcpyHostToDevice, c->s));
    TRY(run_bfs(c, c->d_tmp_a, c->d_tmp_b, nb, c->d_ktmp, c->tstride, nullptr));
    TRY(take(c->d_ktmp, i0, nb));
    HIPCHK(hipStreamSynchronize(c->s));  // the next batch reuses the buffer and the goal upload
  }
  return check_err(c);
}

// Make sure every goal in `goals` (valid free cells) has a table. A failed K1 build (HIP error,
// distance overflow when !tableless_ok) leaves no goal registered against a partial table.
int ensure_tables(tsw_ctx* c, const std::vector<uint32_t>& goals_in, bool tableless_ok = false) {
  std::vector<uint32_t> newg, slots;
  newg.reserve(goals_in.size());
  stamp_and_collect(c, goals_in.data(), goals_in.size(), newg);
  if (newg.empty()) return TSW_OK;
  int rc = reserve_slots(c, newg.size(), slots);
  if (rc == TSW_OK) rc = build_new_tables(c, newg, slots, tableless_ok);
  TRY(finish_tables(c, rc, newg, slots));
  if (eager_policy(c, newg.size())) {
    // eager resolution over real tables only (a tableless goal stays lazy: one A* per cell would be
    // a whole-grid search per cell)
    std::vector<uint32_t> eg, es;
    for (size_t j = 0; j < newg.size(); ++j)
      if (!c->h_tab_tableless[slots[j]]) {
        eg.push_back(newg[j]);
        es.push_back(slots[j]);
      }
    TRY(resolve_all_unknown(c, eg, es));
  }
  return TSW_OK;
}

// TSW_EOVERFLOW if any of `goals` (with tables) is held without one (its distances overflow u16).
int require_real_tables(tsw_ctx* c, const std::vector<uint32_t>& goals) {
  for (uint32_t g : goals) {
    const int32_t t = c->h_goal_tab[g];
    if (t >= 0 && c->h_tab_tableless[t])
      RET(TSW_EOVERFLOW, "goal farther than 65534 steps from some cell: no u16 distance table (plans use K3)");
  }
  return TSW_OK;
}

int ensure_agents(tsw_ctx* c, size_t n) {
  if (n <= c->acap && c->d_v) return TSW_OK;
  HIPCHK(hipStreamSynchronize(c->s));
  size_t cap = std::max<size_t>(n, 64);
  auto fre = [](void* p) {
    if (p) (void)hipFree(p);
  };
  fre(c->d_v); fre(c->d_g); fre(c->d_succ); fre(c->d_ap); fre(c->d_st); fre(c->d_task); fre(c->d_nhc);
  fre(c->d_gt); fre(c->d_dec); fre(c->d_onc); fre(c->d_candc); fre(c->d_f1); fre(c->d_f2);
  HIPCHK(hipMalloc(&c->d_onc, cap));
  HIPCHK(hipMalloc(&c->d_candc, cap));
  HIPCHK(hipMalloc(&c->d_f1, (cap + 1) * 4));
  HIPCHK(hipMalloc(&c->d_f2, (cap + 1) * 4));
  HIPCHK(hipMalloc(&c->d_v, cap * 4));
  HIPCHK(hipMalloc(&c->d_g, cap * 4));
  HIPCHK(hipMalloc(&c->d_succ, cap * 4));
  HIPCHK(hipMalloc(&c->d_gt, cap * 4));
  HIPCHK(hipMalloc(&c->d_ap, (cap + 1) * 4));
  HIPCHK(hipMalloc(&c->d_st, cap));
  HIPCHK(hipMalloc(&c->d_nhc, cap));
  HIPCHK(hipMalloc(&c->d_dec, cap));
  HIPCHK(hipMalloc(&c->d_task, cap * 4));
  if (!c->d_occ) {
    HIPCHK(hipMalloc(&c->d_occ, (size_t)c->G.ncell * 4));
    HIPCHK(hipMalloc(&c->d_cnt, (size_t)c->G.ncell * 4));
    HIPCHK(hipMalloc(&c->d_mu, (size_t)c->G.ncell * 8));
    HIPCHK(hipMalloc(&c->d_dups, 4));
    HIPCHK(hipHostMalloc(&c->h_dups, 4, hipHostMallocDefault));
  }
  c->acap = cap;
  c->chase_id = 0;
  return TSW_OK;
}

// Coop-mode buffers: control block, speculative queue, the needed queue sized for a whole launch,
// the second stream and the host-visible "planner resident" flag.
int ensure_coop(tsw_ctx* c, uint32_t n, uint32_t max_t = 0) {
  TRY(ensure_astar_scratch(c));
  // the needed queue is linear over a coop launch too (urgent walk-ahead pairs join it): sized by the plan
  TRY(ensure_queue(c, std::max<size_t>(std::max<size_t>(4 * (size_t)n + 4096, (size_t)1 << 18),
                                       std::min<size_t>((size_t)n * (max_t + 1u) / 8u, (size_t)1 << 25))));
  if (!c->d_cc) {
    HIPCHK(hipMalloc(&c->d_cc, sizeof(CoopCtl)));
    HIPCHK(hipHostMalloc(&c->h_cc, sizeof(CoopCtl), hipHostMallocDefault));
  }
  // The speculative queue is linear over a plan launch (the planner appends, the workers claim in
  // order): once it is full the planner stops speculating for the rest of the launch. C5 (10,000 agents,
  // 2,001 steps) queues ~1M pairs, exactly the old fixed 2^20 entries: the queue filled up mid-plan and
  // every later step waited on unprefetched pairs (43 s instead of 8 s). Sized by the plan: half an entry
  // per agent-step, 2^20 .. 2^26 entries (16 MB .. 1 GB of HBM).
  const size_t want_qs = std::min<size_t>(std::max<size_t>((size_t)n * (max_t + 1u) / 2u, (size_t)1 << 20),
                                          (size_t)1 << 26);
  if (!c->d_QS || c->qscap < want_qs) {
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(dgrow(c->d_QS, c->qscap, want_qs));
  }
  return TSW_OK;
}

PlanArgs plan_args(tsw_ctx* c, uint32_t n, uint32_t m, uint32_t mode, bool want_goals) {
  PlanArgs P{};
  P.n = n;
  P.m = m;
  P.W = c->G.W;
  P.ncell = c->G.ncell;
  P.mode = mode;
  P.v = c->d_v;
  P.g = c->d_g;
  P.st = c->d_st;
  P.task = c->d_task;
  P.gt = c->d_gt;
  P.succ = c->d_succ;
  P.nhc = c->d_nhc;
  P.dec = c->d_dec;
  P.onc = c->d_onc;
  P.candc = c->d_candc;
  P.f1 = c->d_f1;
  P.f2 = c->d_f2;
  P.mk = c->d_ap;
  P.occ = c->d_occ;
  P.mu = c->d_mu;
  P.has_dups = *c->h_dups;
  // speculative next-hop prefetch only pays in lazy mode (eager tables have nothing unresolved)
  P.prefetch = (!c->tun.prefetch || eager_policy(c, 0)) ? 0u : 1u;
  // wide prefetch (default 8 hops; 4 -> 8: wh10k prefix 2.53 -> 2.28 s, 16 gave 2.32 s): every
  // agent's (succ cell, goal) pair, and its path walked this many hops ahead; TSW_WIDE_PREFETCH=0 restores candidates-only / one hop (A/B)
  // wave-0 rules rounds (scan 64 agents per ballot from the cursor, fire in lane 0): firing
  // agents are dense, so a scan rarely needs more than a chunk or two even for 10k agents;
  // TSW_WAVE_RULES_MAX caps n for A/B
  P.wave_rules_max = c->tun.wave_rules_max;
  P.walk_cap = c->tun.walk_cap;
  P.wide_prefetch = c->tun.wide_prefetch;
  P.wide_hi = c->tun.wide_hi ? c->tun.wide_hi : c->tun.wide_prefetch;
  P.wide_lo = c->tun.wide_lo;
  P.spec_hi = 0;  // set per launch from the worker count (run_plan_impl)
  P.dag_prefetch = c->tun.dag_prefetch;
  P.dag_width = c->tun.dag_width;
  P.urgent_hops = c->tun.urgent_hops;
  P.ab_flags = c->tun.ab_flags;
  P.t0_delay_ticks = c->tun.t0_delay_us * 100u;
  P.prefetch_ext = c->tun.prefetch_ext;
  P.dt = c->d_dt;
  P.nbmask = c->d_nbmask;
  P.live = c->d_live;
  P.klt = c->d_klt;
  P.kpos = c->d_kpos;
  P.kbox = c->d_kbox;
  P.kcnt = c->d_kcnt;
  P.kchunks = c->kchunks;
  P.pick = c->d_pick;
  P.dlv = c->d_dlv;
  P.goal_tab = c->d_goal_tab;
  P.nh = c->d_nh;
  P.nstride = c->tstride;
  P.Q = c->d_Q;
  P.qcap = (uint32_t)c->qcap;
  P.rec = c->d_rec;
  P.grec = want_goals ? c->d_grec : nullptr;
  P.ctl = c->d_ctl;
  P.sec_ticks = c->d_ticks;
  P.dbg = c->tun.plan_debug ? 1u : 0u;
  P.dtag = nullptr;
  if (P.dbg && n) {  // diagnostics only: per-agent change tags
    if (c->dtag_cap < n) {
      if (c->d_dtag) (void)hipFree(c->d_dtag);
      c->d_dtag = nullptr;
      c->dtag_cap = 0;
      if (hipMalloc(&c->d_dtag, (size_t)n * 4) == hipSuccess) c->dtag_cap = n;
    }
    if (c->d_dtag && hipMemsetAsync(c->d_dtag, 0, (size_t)n * 4, c->s) == hipSuccess) P.dtag = c->d_dtag;
  }
  P.wf = nullptr;
  if (c->tun.walk_cache && n) {  // re-armed per plan / step call (a goal never matches 0xFFFFFFFF)
    if (c->wfcap < n) {
      if (c->d_wf) (void)hipFree(c->d_wf);
      c->d_wf = nullptr;
      c->wfcap = 0;
      if (hipMalloc(&c->d_wf, (size_t)n * sizeof(uint4)) == hipSuccess) c->wfcap = n;
    }
    if (c->d_wf && hipMemsetAsync(c->d_wf, 0xFF, (size_t)n * sizeof(uint4), c->s) == hipSuccess) P.wf = c->d_wf;
  }
  P.pred = nullptr;
  if (P.dbg && n && mode == MODE_MAPD) {  // diagnostics only: prediction hits
    if (c->predcap < n) {
      if (c->d_pred) (void)hipFree(c->d_pred);
      c->d_pred = nullptr;
      c->predcap = 0;
      if (hipMalloc(&c->d_pred, (size_t)n * 4) == hipSuccess) c->predcap = n;
    }
    if (c->d_pred && hipMemsetAsync(c->d_pred, 0xFF, (size_t)n * 4, c->s) == hipSuccess) P.pred = c->d_pred;
  }
  // LDS residency, in priority order: agents, occupancy grid, task table
  const size_t budget = (size_t)std::max(c->max_lds - 2048, 0);
  bool ag = plan_lds_bytes(n, P.ncell, m, true, false, false) <= budget;
  // without the whole set, single agent arrays in priority order (PART_*: the rules phase's serial
  // successor walks and firing scans read SUCC / ONC / V / G; wh10k rules 3.9 -> ? s), then the rules
  // relabel's pointer-doubling buffers
  uint32_t part = 0;
  if (!ag)
    for (uint32_t bit : {PART_SUCC, PART_ONC, PART_V, PART_G, PART_NHC, PART_CANDC, PART_GT})
      if ((c->tun.part_lds & bit) && plan_lds_bytes(n, P.ncell, m, false, false, false, false, true, part | bit) <= budget)
        part |= bit;
  bool fl = !ag && c->tun.flinks_lds && plan_lds_bytes(n, P.ncell, m, false, false, false, true, true, part) <= budget;
  // the occupancy grid with the movement rounds' MU words, else OCC alone (every rules round reads
  // OCC: C3's 170x84 fits OCC but not MU beside the agent arrays)
  bool mu = n < 65535u && plan_lds_bytes(n, P.ncell, m, ag, true, false, fl, true, part) <= budget;  // MU32: 16-bit agent ids
  bool oc = mu || (c->tun.occ_split && plan_lds_bytes(n, P.ncell, m, ag, true, false, fl, false, part) <= budget);
  const bool tk = false;  // K4 reads its spatial index from global memory (the chunks it needs only)
  P.part_lds = part;
  P.f_lds = fl;
  P.mu_lds = mu;
  P.agents_lds = ag;
  P.occ_lds = oc;
  P.tasks_lds = tk;
  // coop mode: lazy next hops only (eager tables have nothing left to resolve)
  P.coop = (c->tun.coop && !c->resolver && P.prefetch && c->d_cc && c->d_QS) ? 1u : 0u;
  P.hflags = c->d_flags;  // watchdog words, both modes
  if (P.coop) {
    P.QS = c->d_QS;
    P.qscap = (uint32_t)c->qscap;
    P.cc = c->d_cc;
    P.QH = (mode == MODE_MAPD && c->tun.task_chains && c->tun.hot_chains && c->d_QH && m) ? c->d_QH : nullptr;
    P.qhcap = P.QH ? (uint32_t)std::min<size_t>(c->qhcap, m) : 0u;
    P.QP = (P.QH && c->tun.predict && c->d_QP) ? c->d_QP : nullptr;
    P.qpcap = P.QP ? (uint32_t)std::min<size_t>(c->qpcap, 0xFFFFFFFFu) : 0u;
    P.predict = P.QP ? c->tun.predict : 0u;
  }
  if (!P.QP) P.pred = nullptr;
  return P;
}

// Occupancy grid in k_plan encoding + whether any cell holds several agents.
int build_occ(tsw_ctx* c, uint32_t n) {
  HIPCHK(hipMemsetAsync(c->d_dups, 0, 4, c->s));
  HIPCHK(launch_occ(c->d_v, n, c->d_occ, c->d_cnt, c->G.ncell, c->d_dups, c->s));
  HIPCHK(hipMemcpyAsync(c->h_dups, c->d_dups, 4, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  return TSW_OK;
}

// The K3 pass of an exit-mode planner exit: the exact A* over the queue into the tables, or — with a
// caller resolver (tsw_plan_mapd_resolved) — the queue's pairs handed to the caller and its codes
// written into the tables.
int resolve_queue(tsw_ctx* c, const AstarQuery* Q, uint32_t nq) {
  if (!c->resolver) {
    TRY(run_astar(c, Q, nq, true, nullptr, nullptr));
    return check_err(c);
  }
  if (nq == 0) return TSW_OK;
  std::vector<AstarQuery> q(nq);
  HIPCHK(hipMemcpyAsync(q.data(), Q, (size_t)nq * sizeof(AstarQuery), hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  std::vector<uint32_t> st(nq), gl(nq);
  for (uint32_t i = 0; i < nq; ++i) {
    st[i] = q[i].v;
    gl[i] = q[i].goal;
  }
  std::vector<uint8_t> codes(nq, NH_UNKNOWN);
  if (c->resolver(c->resolver_user, nq, st.data(), gl.data(), codes.data()) != 0)
    RET(TSW_EINVAL, "the caller's next-hop resolver failed");
  for (uint32_t i = 0; i < nq; ++i)
    if (codes[i] > NH_STAY) RET(TSW_EINVAL, "the caller's next-hop resolver returned a code > 4");
  TRY(ensure_res(c, nq));
  HIPCHK(hipMemcpyAsync(c->d_res, codes.data(), nq, hipMemcpyHostToDevice, c->s));
  HIPCHK(launch_put_codes(Q, nq, c->d_res, c->d_nh, c->tstride, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  c->st.astar_queries += nq;
  return TSW_OK;
}

// Drive k_plan until it reports done; each NEED_QUERIES exit runs K3 on the queued pairs.
int run_plan_impl(tsw_ctx* c, PlanArgs& P, const PlanCtl& init) {
  *c->h_ctl = init;
  HIPCHK(hipMemcpyAsync(c->d_ctl, c->h_ctl, sizeof(PlanCtl), hipMemcpyHostToDevice, c->s));
  size_t lds = plan_lds_bytes(P.n, P.ncell, P.m, P.agents_lds, P.occ_lds, P.tasks_lds, P.f_lds, P.mu_lds, P.part_lds);
  // coop mode: the planner block reserves its CU's whole LDS so no worker wave is placed beside it
  // (they would compete for its SIMDs and LDS bandwidth on the critical path)
  if (P.coop) lds = std::max<size_t>(lds, (size_t)std::max(c->max_lds - 2048, 0));
  // one lane per agent in the parallel passes when possible; >= 4 waves for the task argmin
  uint32_t block = std::min<uint32_t>(PLAN_BLOCK_MAX, std::max<uint32_t>(256, (P.n + 63) / 64 * 64));
  if (c->tun.plan_block) block = std::max<uint32_t>(64u, c->tun.plan_block);
  WorkerArgs W{};
  uint32_t wblocks = 0;
  if (P.coop) {
    W.G = c->G;
    W.cc = c->d_cc;
    W.QN = c->d_Q;
    W.QS = c->d_QS;
    W.QT = c->d_QT;
    W.QH = c->d_QH;
    W.QP = P.QP;
    W.klive = c->d_live;
    W.klt = c->d_klt;
    W.kbox = c->d_kbox;
    W.kcnt = c->d_kcnt;
    W.kchunks = c->kchunks;
    W.pick = c->d_pick;
    W.dlv = c->d_dlv;
    W.goal_tab = c->d_goal_tab;
    W.pred = P.pred;
    W.nh = c->d_nh;
    W.nstride = c->tstride;
    // every worker may walk task chains: a chain worker serves queued needed / speculative pairs
    // between hops (W.preempt), so chains only use otherwise idle time. Round 4 A/B (chain share 1/4
    // -> all, profiles/r4/chain_share_ab.txt): wh10k 11.58 -> 10.25 s, C5 3.33 -> 2.76 s, C3 unchanged
    // (it was a quarter with many agents, a half otherwise)
    W.tmask = c->tun.chain_mask >= 0 ? (uint32_t)c->tun.chain_mask : 0u;
    W.preempt = c->tun.chain_preempt ? 1u : 0u;
    W.chain_hops = c->tun.chain_hops;
    W.avoid_xcc = c->tun.avoid_xcc ? 1u : 0u;
    W.hflags = c->d_flags;
    const WorkerCfg wcfg =
        worker_config(c->G, c->num_cu, P.n, c->tun.wave_hcap, c->tun.worker_gs, c->tun.dag_exit, lds, c->tun.worker_fb);
    W.dag = wcfg.dag;
    // the test's heap scan gathers D from LDS (detour bytes) or from the u16 table in global memory:
    // every 16 / 64 pops (C3 worker busy -20 %, wh10k 400 steps 5.77 -> 5.42 s; profiles/r3/dag_exit_ab.txt)
    W.dag_mask = c->tun.dag_mask ? c->tun.dag_mask : (W.dag == 1u ? 15u : 63u);
    W.stale_steps = c->tun.stale_steps;
    W.reg_heap = c->tun.reg_heap;
    W.wake_gate = (1u << c->tun.wake_gate) - 1u;
    W.slow_mask = (1u << c->tun.slow_poll) - 1u;
    W.slow_mult = c->tun.slow_mult;
    W.idle_ticks = c->tun.worker_idle_us * 100ull;  // wall clock: 100 MHz
    W.dt = c->d_dt;
    W.gs_lds = wcfg.gs_lds;
    W.stage_fb = wcfg.stage_fb;
    W.hcap = wcfg.hcap;
    // one dispatch: the planner (workgroup 0) and one worker workgroup on every other CU, each holding
    // as many single-wave workers as its dynamic LDS (the planner's, whole-CU size) carves
    W.lds_per_wave = (uint32_t)((wcfg.lds + 15u) & ~(size_t)15u);
    W.wpb = W.lds_per_wave ? (uint32_t)std::min<size_t>(block / 64u, lds / W.lds_per_wave) : 0u;
    const uint32_t want = W.wpb * (uint32_t)std::max(c->num_cu - 1, 0);
    TRY(ensure_astar_scratch(c, want));  // one g-score / heap slot per worker wave
    W.gs_all = c->d_gs;
    W.epochs = c->d_epochs;
    W.heaps = c->d_heaps;
    W.ghcap = c->hcap;
    W.nworkers = std::min(want, c->nslots);
    P.spec_hi = 2u * W.nworkers;  // a backlog of two pairs per worker counts as keeping up
    wblocks = W.wpb ? (W.nworkers + W.wpb - 1u) / W.wpb : 0u;
    if (c->tun.plan_debug)
      fprintf(stderr, "[k_plan] workers: %u waves (%u per workgroup), g-scores %u, heap %u entries, DAG exit %u, %u B LDS each\n",
              W.nworkers, W.wpb, wcfg.gs_lds, wcfg.hcap, wcfg.dag, W.lds_per_wave);
    if (W.nworkers == 0 || wcfg.hcap < 4u) P.coop = 0;  // nothing fits beside the planner: exit mode
  }
  if (c->tun.plan_debug)
    fprintf(stderr, "[k_plan] planner LDS: agents %u part 0x%x flinks %u occ %u mu %u tasks %u (%zu B)\n", P.agents_lds,
            P.part_lds, P.f_lds, P.occ_lds, P.mu_lds, P.tasks_lds,
            plan_lds_bytes(P.n, P.ncell, P.m, P.agents_lds, P.occ_lds, P.tasks_lds, P.f_lds, P.mu_lds, P.part_lds));
  const bool coop = P.coop != 0;
  // every return below happens after the dispatch has drained (workers included): nothing of this
  // call keeps running into the next one
  for (uint64_t round = 0;; ++round) {
    if (round > 16ull * P.n + 4096ull * (init.max_t + 1)) RET(TSW_EINVAL, "plan kernel made no progress");
    if (coop) {
      HIPCHK(hipMemsetAsync(c->d_cc, 0, sizeof(CoopCtl), c->s));
      const uint32_t nt = P.mode == MODE_MAPD ? c->qt_count : 0u;
      if (nt) HIPCHK(hipMemcpyAsync(&c->d_cc->head_t, &c->qt_count, 4, hipMemcpyHostToDevice, c->s));
    }
    {
      volatile uint32_t* hf = c->h_flags;
      hf[0] = 0u;
      hf[1] = 0u;
      hf[2] = 0u;
      for (int w = 4; w < 40; ++w) hf[w] = 0u;  // barrier breadcrumbs (TSW_PLAN_DEBUG)
    }
    {
      Timer t(c, CAT_WALK);
      HIPCHK(launch_plan(P, c->d_pargs, coop ? &W : nullptr, wblocks, lds, block, c->s));
      c->st.plan_block = block;
    }
    c->st.walker_launches++;
    if (coop) c->st.astar_launches++;
    HIPCHK(hipMemcpyAsync(c->h_ctl, c->d_ctl, sizeof(PlanCtl), hipMemcpyDeviceToHost, c->s));
    {
      // watchdog: the planner publishes its timestep count; if it stops moving for 10 s while the
      // planner still runs, raise `abort`. In coop mode its waits give up (it exits to the host),
      // the workers leave and the rest of the call runs in exit mode; a planner stuck anywhere else
      // sees the flag in its round loops and exits with ERR_ABORT and its position. A fault can
      // then cost time or fail the call, but never hang it.
      volatile uint32_t* hf = c->h_flags;
      uint32_t last = hf[2];
      auto seen = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipStreamQuery(c->s);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIPCHK(q);
        const uint32_t hb = hf[2];
        const auto now = std::chrono::steady_clock::now();
        if (hb != last) {
          last = hb;
          seen = now;
        } else if (!hf[1] && now - seen > std::chrono::milliseconds(c->watchdog_ms)) {
          hf[1] = 1u;
          ++c->coop_aborts;
          ++c->st.watchdog_fires;
          if (c->watchdog_ms >= 1000u)
            fprintf(stderr, "[tswap] watchdog: planner made no step for %u ms; finishing the call in exit mode\n",
                    c->watchdog_ms);
          if (c->tun.plan_debug && hf[24]) {  // per-wave barrier breadcrumbs (-DTSW_PBAR): line | 0x10000 once passed
            fprintf(stderr, "[tswap] planner waves at barriers:");
            for (int w = 0; w < 16; ++w) fprintf(stderr, " %u%s", hf[8 + w] & 0xFFFFu, (hf[8 + w] >> 16) ? "+" : "");
            fprintf(stderr, "\n[tswap] barriers passed per wave:");
            for (int w = 0; w < 16; ++w) fprintf(stderr, " %u", hf[24 + w]);
            fprintf(stderr, "\n[tswap] first mismatch: wave 0 at %u, another at %u\n", hf[4] >> 16, hf[4] & 0xFFFFu);
          }
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    }
    HIPCHK(hipStreamSynchronize(c->s));
    if (coop) {
      HIPCHK(hipMemcpy(c->h_cc, c->d_cc, sizeof(CoopCtl), hipMemcpyDeviceToHost));
      const CoopCtl& cc = *c->h_cc;
      c->st.coop_waits += cc.waits;
      c->st.coop_wait_ms += (double)cc.wait_ticks / (double)c->wall_khz;
      for (int k = 0; k < 8; ++k) {
        c->st.coop_wait_sec_ms[k] += (double)cc.wait_sec[k] / (double)c->wall_khz;
        c->st.coop_waits_sec[k] += cc.waits_sec[k];
      }
      c->st.astar_queries += cc.worker_queries;
      c->st.coop_workers = W.nworkers;
      for (int k = 0; k < 3; ++k) {
        c->st.coop_worker_busy_ms[k] += (double)cc.wbusy[k] / (double)c->wall_khz;
        c->st.coop_worker_queries[k] += cc.wcount[k];
        c->st.coop_worker_pops[k] += cc.wpops[k];
      }
      if (cc.err) RET(TSW_EOVERFLOW, "K3 worker: A* heap overflow");
      // speculative pairs nobody claimed stay PENDING_S: back to UNKNOWN for later calls — only the
      // unclaimed queue entries (every claimed one was resolved, or reset by the worker that dropped
      // it as stale): a whole-store sweep cost C5 ~4 s per call (18 GB of codes)
      if (cc.head_s > cc.claim_s) {
        HIPCHK(launch_reset_queue(c->d_QS, cc.claim_s, std::min<uint32_t>(cc.head_s, (uint32_t)c->qscap), c->d_nh,
                                  c->tstride, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
      }
    }
    const PlanCtl& k = *c->h_ctl;
    if (k.err & ERR_ABORT) {
      if (c->tun.plan_debug) {  // diagnostics: where the stopped planner spent its time (section / sub-phase ticks)
        unsigned long long tk[48];
        if (hipMemcpy(tk, c->d_ticks, sizeof tk, hipMemcpyDeviceToHost) == hipSuccess) {
          std::string line = "[k_plan] watchdog stop, ticks:";
          for (int q = 0; q < 40; ++q) line += " " + std::to_string(q) + ":" + std::to_string(tk[q]);
          fprintf(stderr, "%s\n", line.c_str());
        }
      }
      char buf[256];
      snprintf(buf, sizeof buf,
               "planner stopped by the watchdog (no timestep for %u ms): t %u section %u cursor %u, %u rule rounds, "
               "%u move rounds", c->watchdog_ms, k.t, k.section, k.i, k.rule_rounds, k.move_rounds);
      RET(TSW_EINVAL, buf);
    }
    if (k.err & ERR_BAD_PICKUP)
      RET(TSW_EINVAL, "assigned task's pickup is off-grid or blocked (reference panics at tswap.rs:136)");
    if (k.err & ERR_BAD_DELIVERY)
      RET(TSW_EINVAL, "reached pickup's task delivery is off-grid or blocked (reference panics at tswap.rs:112)");
    if (k.err) {
      char buf[128];
      snprintf(buf, sizeof buf, "plan kernel error bits 0x%x", k.err);
      RET((k.err & ERR_NO_TABLE) ? TSW_EINVAL : TSW_EOVERFLOW, buf);
    }
    c->st.relabels_full += k.relabel_full;
    c->st.relabels_inc += k.relabel_inc;
    if (k.status == PLAN_DONE) {
      c->chase_id = k.chase_id;
      c->st.rule_rounds += k.rule_rounds;
      c->st.move_rounds += k.move_rounds;
      if (c->tun.plan_debug) {
        unsigned long long tk[48];
        HIPCHK(hipMemcpy(tk, c->d_ticks, sizeof tk, hipMemcpyDeviceToHost));
        fprintf(stderr, "[k_plan] assign us: transitions %.0f compaction %.0f scan %.0f accept %.0f update %.0f | sections %llu batches %llu accepted %llu\n",
                tk[32] / 100.0, tk[33] / 100.0, tk[34] / 100.0, tk[35] / 100.0, tk[36] / 100.0, tk[39], tk[37], tk[38]);
        fprintf(stderr, "[k_plan] PRE1 publish us %.0f (%llu) | rules init us %.0f prefetch us %.0f publish us %.0f (%llu)\n",
                tk[24] / 100.0, tk[25], tk[26] / 100.0, tk[27] / 100.0, tk[28] / 100.0, tk[29]);
        fprintf(stderr, "[k_plan] wave rules kcycles: load %.0f stale %.0f fast %.0f update %.0f slow %.0f rot %.0f | "
                "loads %llu fast firings %llu | rotations %llu, settle kcycles: successors %.0f walk %.0f\n",
                tk[16] / 1e3, tk[17] / 1e3, tk[18] / 1e3, tk[19] / 1e3, tk[20] / 1e3, tk[21] / 1e3, tk[22], tk[23],
                tk[11], tk[30] / 1e3, tk[31] / 1e3);
        fprintf(stderr, "[k_plan] wave rules batches %llu (longest walks %llu hops) kcycles: marks %.0f walks %.0f apply %.0f\n",
                tk[43], tk[44], tk[40] / 1e3, tk[41] / 1e3, tk[42] / 1e3);
        fprintf(stderr, "[k_plan] steps %u rule rounds %u move rounds %u launches %llu | move A-E us %.0f %.0f %.0f %.0f %.0f"
                " | rules scan %.0f fire %.0f relabel %.0f\n", k.steps_run, k.rule_rounds, k.move_rounds,
                (unsigned long long)round + 1ull, tk[8] / 100.0, tk[9] / 100.0, tk[10] / 100.0, tk[11] / 100.0,
                tk[12] / 100.0, tk[13] / 100.0, tk[14] / 100.0, tk[15] / 100.0);
        if (coop) {
          const CoopCtl& cc = *c->h_cc;
          fprintf(stderr, "[k_plan] needed pairs unresolved (never queued / queued speculatively): PRE1 %u/%u RULES %u/%u "
                  "MOVE %u/%u | PRE1 never queued: assigned %u, picked up %u | chain queries %llu of %llu\n", cc.dbg_need[0], cc.dbg_need[1], cc.dbg_need[2],
                  cc.dbg_need[3], cc.dbg_need[4], cc.dbg_need[5], cc.dbg_need[6], cc.dbg_need[7],
                  (unsigned long long)cc.chain_queries, (unsigned long long)cc.worker_queries);
          {
            static const char* nm[6] = {"r3b", "r3s", "rot", "mv", "asg", "pick"};
            std::string line = "[k_plan] PRE1 unresolved by agent change (unknown/pending):";
            for (int tg = 0; tg < 64; ++tg) {
              if (!cc.dbg_tag[0][tg] && !cc.dbg_tag[1][tg]) continue;
              std::string name;
              for (int b = 0; b < 6; ++b)
                if (tg & (1 << b)) name += (name.empty() ? "" : "+") + std::string(nm[b]);
              char buf[96];
              snprintf(buf, sizeof buf, " %s %u/%u", name.empty() ? "none" : name.c_str(), cc.dbg_tag[0][tg], cc.dbg_tag[1][tg]);
              line += buf;
            }
            fprintf(stderr, "%s\n", line.c_str());
          }
          fprintf(stderr, "[k_plan] speculative pairs dropped as stale: %u (older than %u timesteps)\n",
                  cc.spec_dropped, c->tun.stale_steps);
          fprintf(stderr, "[k_plan] predicted chains: %u jobs | assignments %u: predicted task %u, no prediction %u\n",
                  cc.pred_jobs, cc.pred_asg, cc.pred_hit, cc.pred_none);
          fprintf(stderr, "[k_plan] spec backlog at wait start: avg %.1f max %u | queue delay enqueue -> claim: needed "
                  "avg %.1f us (%u > 1 ms, %u already resolved), speculative avg %.1f timesteps (%u > 1, %u already resolved)\n",
                  cc.waits ? (double)cc.dbg_depth / cc.waits : 0.0, cc.dbg_depth_max,
                  cc.wcount[0] ? cc.qdelay[0] / 100.0 / cc.wcount[0] : 0.0, cc.qlate[0], cc.qskip[0],
                  cc.wcount[1] ? (double)cc.qdelay[1] / cc.wcount[1] : 0.0, cc.qlate[1], cc.qskip[1]);
          fprintf(stderr, "[k_plan] worker A* ms (queries, pops): needed %.1f (%u, %llu) spec %.1f (%u, %llu) task chains "
                  "%.1f (%u, %llu) | tier-2 hand-offs %llu tier-3 %llu | detour staging %.1f ms (%u)\n",
                  cc.wbusy[0] / (double)c->wall_khz, cc.wcount[0], cc.wpops[0], cc.wbusy[1] / (double)c->wall_khz,
                  cc.wcount[1], cc.wpops[1], cc.wbusy[2] / (double)c->wall_khz, cc.wcount[2], cc.wpops[2],
                  cc.wpops[3] & 0xFFFFFFFFull, cc.wpops[3] >> 32, cc.wbusy[3] / (double)c->wall_khz, cc.wcount[3]);
        }
      }
      // exit mode: pairs the prefetch queued but no firing needed — resolve them so no table entry
      // is left PENDING for later calls (coop mode: the workers drained the needed queue)
      if (!coop && k.qcount > 0) {
        if (k.qcount > P.qcap) RET(TSW_EINVAL, "plan kernel queue overflow");
        TRY(resolve_queue(c, c->d_Q, k.qcount));
      }
      return TSW_OK;
    }
    c->st.plan_exits[std::min<uint32_t>(k.section, 7u)]++;
    if (coop) {
      if (k.status != PLAN_NEED_QUERIES) RET(TSW_EINVAL, "plan kernel stopped without resolvable next hops");
      if (c->h_flags[1]) {
        // watchdog fired: finish this call in exit mode (host-side K3 passes at planner exits);
        // pairs the aborted workers left queued are unqueued first
        HIPCHK(launch_reset_pending(c->d_nh, (uint64_t)c->tab_count * c->tstride, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
        P.coop = 0;
        PlanCtl resume = k;
        resume.status = PLAN_RUNNING;
        resume.qcount = 0;
        return run_plan_impl(c, P, resume);
      }
      // the planner gave up waiting (no worker left — they exit after an idle spell — or a pair stayed
      // pending): resolve its needed queue on the host side before relaunching, so every relaunch makes
      // progress whatever the workers of the next dispatch do (exact codes; resolved ones rewrite the same)
      if (k.qcount > 0) {
        if (k.qcount > P.qcap) RET(TSW_EINVAL, "plan kernel queue overflow");
        TRY(run_astar(c, c->d_Q, k.qcount, true, nullptr, nullptr));
        TRY(check_err(c));
      }
      continue;
    }
    if (k.status != PLAN_NEED_QUERIES || k.qcount == 0 || k.qcount > P.qcap)
      RET(TSW_EINVAL, "plan kernel stopped without resolvable next hops");
    TRY(resolve_queue(c, c->d_Q, k.qcount));
  }
}

// Any failure after k_plan queued pairs leaves their codes PENDING: reset them.
int run_plan(tsw_ctx* c, PlanArgs& P, const PlanCtl& init) {
  return reset_pending_after(c, run_plan_impl(c, P, init));
}

int plan_impl(tsw_ctx* c, const tsw_point* starts, uint32_t n, const tsw_task* tasks, uint32_t m,
              uint32_t max_t, tsw_rec* out, uint32_t* goal_out, uint32_t* out_T) {
  auto t0 = std::chrono::steady_clock::now();
  if (!out_T || (n && (!starts || !out)) || (m && !tasks)) RET(TSW_EINVAL, "null argument");
  if (max_t > (1u << 20)) RET(TSW_EINVAL, "max_t too large");
  TRY(set_device(c));
  // K4 spatial index: tasks in Morton order of their (clamped) pickup points, cut into chunks of KCH = 32
  // entries with static bounding boxes (tsw_plan.h PlanArgs::kbox)
  constexpr uint32_t KCHH = 32;
  const uint32_t nch = std::max<uint32_t>((m + KCHH - 1u) / KCHH, 1u);
  std::vector<uint32_t> vcell(n), pick(m), dlv(m), pxy(m), live((size_t)nch * KCHH, TASK_TAKEN),
      klt((size_t)nch * KCHH, 0xFFFFFFFFu), kpos(std::max<uint32_t>(m, 1u)), kcnt(nch, 0u);
  std::vector<uint2> kbox(nch, make_uint2(0u, 0u));
  std::vector<uint32_t> goalset;
  goalset.reserve(n + 2 * (size_t)m);
  for (uint32_t i = 0; i < n; ++i) {
    if (!cell_ok(c, starts[i].x, starts[i].y, &vcell[i]))
      RET(TSW_EINVAL, "start position off-grid or blocked (reference panics at tswap.rs:94)");
    goalset.push_back(vcell[i]);
  }
  // Task cells are looked up only when the planner needs them — the pickup when the task is
  // assigned (pos2id[&task.pickup], tswap.rs:136), the delivery when its agent reaches the pickup
  // (:112) — so an off-grid or blocked one fails the call only then (k_plan ERR_BAD_*), exactly
  // where the reference panics. The assignment's Manhattan distance still uses the raw point
  // (:125-130); coordinates are clamped to 0xFFFE (0xFFFFFFFF marks a taken task), which cannot
  // change which task wins: any point past 0xFFFE is farther than every on-grid pickup (sides <=
  // 2048), and assigning it fails anyway.
  for (uint32_t k = 0; k < m; ++k) {
    if (!cell_ok(c, tasks[k].pickup.x, tasks[k].pickup.y, &pick[k])) pick[k] = CELL_BAD;
    if (!cell_ok(c, tasks[k].delivery.x, tasks[k].delivery.y, &dlv[k])) dlv[k] = CELL_BAD;
    pxy[k] = std::min<uint32_t>(tasks[k].pickup.x, 0xFFFEu) | (std::min<uint32_t>(tasks[k].pickup.y, 0xFFFEu) << 16);
    if (pick[k] != CELL_BAD) goalset.push_back(pick[k]);
    if (dlv[k] != CELL_BAD) goalset.push_back(dlv[k]);
  }
  {
    auto morton = [](uint32_t xy) {
      uint64_t z = 0;
      for (uint32_t bt = 0; bt < 16u; ++bt)
        z |= (uint64_t)((xy >> bt) & 1u) << (2u * bt) | (uint64_t)((xy >> (16u + bt)) & 1u) << (2u * bt + 1u);
      return z;
    };
    std::vector<std::pair<uint64_t, uint32_t>> ord(m);
    for (uint32_t k = 0; k < m; ++k) ord[k] = {morton(pxy[k]), k};
    std::sort(ord.begin(), ord.end());
    for (uint32_t pos = 0; pos < m; ++pos) {
      const uint32_t k = ord[pos].second, xy = pxy[k], ch = pos / KCHH;
      live[pos] = xy;
      klt[pos] = k;
      kpos[k] = pos;
      const uint32_t x = xy & 0xFFFFu, y = xy >> 16;
      uint2& bx = kbox[ch];
      if (kcnt[ch] == 0u) {
        bx = make_uint2(xy, xy);
      } else {
        bx.x = std::min(bx.x & 0xFFFFu, x) | (std::min(bx.x >> 16, y) << 16);
        bx.y = std::max(bx.y & 0xFFFFu, x) | (std::max(bx.y >> 16, y) << 16);
      }
      ++kcnt[ch];
    }
  }
  TRY(ensure_agents(c, std::max<uint32_t>(n, 1)));
  if (live.size() > c->tcap || !c->d_live) {
    HIPCHK(hipStreamSynchronize(c->s));
    size_t a = c->tcap, b = c->tcap, d = c->tcap;
    HIPCHK(dgrow(c->d_live, a, live.size()));
    HIPCHK(dgrow(c->d_pick, b, live.size()));
    HIPCHK(dgrow(c->d_dlv, d, live.size()));
    c->tcap = std::min(std::min(a, b), d);
    if (!c->d_unused) HIPCHK(hipMalloc(&c->d_unused, 4));
  }
  if (live.size() > c->kcap || !c->d_klt) {
    HIPCHK(hipStreamSynchronize(c->s));
    size_t a = c->kcap, b = c->kcap;
    HIPCHK(dgrow(c->d_klt, a, live.size()));
    HIPCHK(dgrow(c->d_kpos, b, live.size()));
    c->kcap = std::min(a, b);
  }
  if (nch > c->kchcap || !c->d_kbox) {
    HIPCHK(hipStreamSynchronize(c->s));
    size_t a = c->kchcap, b = c->kchcap;
    HIPCHK(dgrow(c->d_kbox, a, (size_t)nch));
    HIPCHK(dgrow(c->d_kcnt, b, (size_t)nch));
    c->kchcap = std::min(a, b);
  }
  c->kchunks = nch;
  const size_t stride_t = (size_t)max_t + 1;
  const size_t recs = stride_t * std::max<uint32_t>(n, 1);
  if (recs > c->rec_cap || !c->d_rec) {
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(dgrow(c->d_rec, c->rec_cap, recs));
  }
  if (goal_out && (recs > c->grec_cap || !c->d_grec)) {
    HIPCHK(hipStreamSynchronize(c->s));
    HIPCHK(dgrow(c->d_grec, c->grec_cap, recs));
  }
  // agent + task state
  if (n) {
    HIPCHK(hipMemcpyAsync(c->d_v, vcell.data(), n * 4ull, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_g, vcell.data(), n * 4ull, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemsetAsync(c->d_st, 0, n, c->s));
    HIPCHK(hipMemsetAsync(c->d_task, 0xFF, n * 4ull, c->s));
  }
  HIPCHK(hipMemcpyAsync(c->d_live, live.data(), live.size() * 4ull, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_klt, klt.data(), klt.size() * 4ull, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_kpos, kpos.data(), kpos.size() * 4ull, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_kbox, kbox.data(), kbox.size() * sizeof(uint2), hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_kcnt, kcnt.data(), kcnt.size() * 4ull, hipMemcpyHostToDevice, c->s));
  if (m) {
    HIPCHK(hipMemcpyAsync(c->d_pick, pick.data(), m * 4ull, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_dlv, dlv.data(), m * 4ull, hipMemcpyHostToDevice, c->s));
  }
  HIPCHK(hipMemcpyAsync(c->d_unused, &m, 4, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipStreamSynchronize(c->s));  // host vectors above go out of scope only at return, but keep it simple
  auto tphase = [&](const char* what) {  // diagnostics (TSW_PLAN_DEBUG): host-side phases of the call
    if (c->tun.plan_debug)
      fprintf(stderr, "[plan] %s at %.1f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  };
  tphase("inputs uploaded");
  TRY(build_occ(c, n));
  TRY(ensure_tables(c, goalset, true));
  HIPCHK(hipStreamSynchronize(c->s));
  tphase("tables built");
  TRY(ensure_queue(c, 4 * (size_t)n + 4096));  // needed pairs (<= 2n per exit) + speculative prefetch (qcap/2)
  c->qt_count = 0;
  if (c->tun.coop && !c->resolver && !eager_policy(c, 0)) {
    TRY(ensure_coop(c, n, max_t));
    if (c->tun.task_chains && m) {
      // every task's pickup -> delivery path, resolved hop by hop by the workers in the background
      // (lowest priority): an agent that picks the task up finds its next hops already there
      std::vector<AstarQuery> qt;
      qt.reserve(m);
      for (uint32_t k = 0; k < m; ++k)
        if (pick[k] != dlv[k] && pick[k] != CELL_BAD && dlv[k] != CELL_BAD) qt.push_back(AstarQuery{pick[k], dlv[k], c->h_goal_tab[dlv[k]], 0u});
      if (qt.size() > c->qtcap) {
        HIPCHK(hipStreamSynchronize(c->s));
        HIPCHK(dgrow(c->d_QT, c->qtcap, qt.size()));
      }
      if (!qt.empty()) {
        HIPCHK(hipMemcpyAsync(c->d_QT, qt.data(), qt.size() * sizeof(AstarQuery), hipMemcpyHostToDevice, c->s));
        HIPCHK(hipStreamSynchronize(c->s));
      }
      c->qt_count = (uint32_t)qt.size();
      if (c->tun.hot_chains && (m > c->qhcap || !c->d_QH)) {
        HIPCHK(hipStreamSynchronize(c->s));
        HIPCHK(dgrow(c->d_QH, c->qhcap, (size_t)m));
      }
      // predictions: one per pickup (<= m) plus, with bit 1, one per goal change of a delivering agent;
      // a full queue only stops predicting
      const size_t qp = (size_t)m + 16u * (size_t)n * (c->tun.predict & 2u ? 8u : 0u);
      if (c->tun.hot_chains && c->tun.predict && (qp > c->qpcap || !c->d_QP)) {
        HIPCHK(hipStreamSynchronize(c->s));
        HIPCHK(dgrow(c->d_QP, c->qpcap, qp));
      }
    }
  }
  PlanArgs P = plan_args(c, n, m, MODE_MAPD, goal_out != nullptr);
  PlanCtl init{};
  init.section = SEC_ASSIGN;
  init.unused = m;
  init.max_t = max_t;
  init.chase_id = c->chase_id;
  init.move_rounds = c->tun.move_round0;
  tphase("plan dispatch starts");
  TRY(run_plan(c, P, init));
  tphase("plan dispatch done");
  const uint32_t t = c->h_ctl->t;
  c->st.steps += t;
  *out_T = t;
  if (n) {
    std::vector<uint64_t> rec((size_t)t * n);
    HIPCHK(hipMemcpyAsync(rec.data(), c->d_rec, rec.size() * 8, hipMemcpyDeviceToHost, c->s));
    std::vector<uint32_t> grec;
    if (goal_out) {
      grec.resize((size_t)t * n);
      HIPCHK(hipMemcpyAsync(grec.data(), c->d_grec, grec.size() * 4, hipMemcpyDeviceToHost, c->s));
    }
    HIPCHK(hipStreamSynchronize(c->s));
    for (uint32_t tt = 0; tt < t; ++tt)
      for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = rec[(size_t)tt * n + i];
        tsw_rec& o = out[(size_t)i * stride_t + tt];
        o.x = (uint16_t)(r & 0xFFFF);
        o.y = (uint16_t)((r >> 16) & 0xFFFF);
        o.state = (uint8_t)((r >> 32) & 0xFF);
        o.pad[0] = o.pad[1] = o.pad[2] = 0;
        if (goal_out) goal_out[(size_t)i * stride_t + tt] = grec[(size_t)tt * n + i];
      }
  }
  resolve_timing(c);
  c->st.plan_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return TSW_OK;
}

}  // namespace

extern "C" {

tsw_ctx* tsw_create(const uint8_t* cells, uint32_t w, uint32_t h, const tsw_opts* opts) {
  if (!cells || w == 0 || h == 0) {
    g_create_err = "tsw_create: empty grid";
    return nullptr;
  }
  if (w > MAX_WH || h > MAX_WH || (uint64_t)w * h > MAX_CELLS) {
    g_create_err = "tsw_create: grid exceeds 2048 per side or 2^20 cells";
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    g_create_err = "tsw_create: no HIP device visible (the HIP path has no CPU fallback)";
    return nullptr;
  }
  tsw_ctx* c = new tsw_ctx();
  c->tun = Tunables::from_env();  // diagnostic build only: the only place the environment is read
  c->device = opts ? opts->device : 0;
  c->flags = opts ? opts->flags : 0;
  if (c->flags & TSW_F_EXIT_MODE) c->tun.coop = false;
  if (opts && opts->watchdog_ms) c->watchdog_ms = opts->watchdog_ms;
  if (c->device < 0 || c->device >= ndev) {
    g_create_err = "tsw_create: bad device ordinal";
    delete c;
    return nullptr;
  }
  auto fail = [&](const char* what, hipError_t e) {
    g_create_err = std::string("tsw_create: ") + what + ": " + hipGetErrorString(e);
    tsw_destroy(c);
    return (tsw_ctx*)nullptr;
  };
  hipError_t e;
  if ((e = hipSetDevice(c->device)) != hipSuccess) return fail("hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
  hipDeviceGetAttribute(&c->max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, c->device);
  hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, c->device);
  if (c->max_lds <= 0) c->max_lds = 65536;
  if (c->num_cu <= 0) c->num_cu = 256;

  const uint32_t ncell = w * h, ncp = (ncell + 7u) & ~7u, Ww = (w + 31u) / 32u;
  c->G.W = w;
  c->G.H = h;
  c->G.ncell = ncell;
  c->G.Ww = Ww;
  c->tstride = ncp;
  // graph build (tswap.rs:44-77): '@' blocked, neighbours S,E,N,W
  c->h_nbmask.assign(ncp, 0);
  std::vector<uint32_t> fb((size_t)h * Ww, 0u);
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x)
      if (cells[(size_t)y * w + x] != '@') {
        c->h_nbmask[(size_t)y * w + x] = NB_FREE;
        fb[(size_t)y * Ww + (x >> 5)] |= 1u << (x & 31u);
      }
  auto is_free = [&](long x, long y) {
    return x >= 0 && y >= 0 && x < (long)w && y < (long)h && cells[(size_t)y * w + x] != '@';
  };
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      uint8_t& m = c->h_nbmask[(size_t)y * w + x];
      if (!(m & NB_FREE)) continue;
      if (is_free(x, (long)y + 1)) m |= 1;
      if (is_free((long)x + 1, y)) m |= 2;
      if (is_free(x, (long)y - 1)) m |= 4;
      if (is_free((long)x - 1, y)) m |= 8;
    }
  if ((e = hipMalloc(&c->d_nbmask, ncp)) != hipSuccess) return fail("malloc nbmask", e);
  if ((e = hipMemcpy(c->d_nbmask, c->h_nbmask.data(), ncp, hipMemcpyHostToDevice)) != hipSuccess)
    return fail("copy nbmask", e);
  if ((e = hipMalloc(&c->d_freebits, fb.size() * 4)) != hipSuccess) return fail("malloc freebits", e);
  if ((e = hipMemcpy(c->d_freebits, fb.data(), fb.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail("copy freebits", e);
  c->G.nbmask = c->d_nbmask;
  c->G.freebits = c->d_freebits;
  {
    // k_bfs_wave layout: word (r, cw) at (r + 1) * Wp + cw, zero guard column and rows
    c->Wp = Ww + 1u;
    c->npw = (h + 2u) * c->Wp;
    std::vector<uint32_t> frp(c->npw, 0u);
    for (uint32_t y = 0; y < h; ++y)
      for (uint32_t cw = 0; cw < Ww; ++cw) frp[(size_t)(y + 1u) * c->Wp + cw] = fb[(size_t)y * Ww + cw];
    if ((e = hipMalloc(&c->d_frp, (size_t)c->npw * 4)) != hipSuccess) return fail("malloc frp", e);
    if ((e = hipMemcpy(c->d_frp, frp.data(), (size_t)c->npw * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return fail("copy frp", e);
    // k_bfs_blk layout: block (bx, by) at (by + 1) * Bp + bx, zero guard block column and rows
    c->BW = (w + 7u) / 8u;
    c->BH = (h + 7u) / 8u;
    c->Bp = c->BW + 1u;
    c->nbp = (c->BH + 2u) * c->Bp;
    std::vector<uint64_t> frb(c->nbp, 0ull);
    for (uint32_t y = 0; y < h; ++y)
      for (uint32_t x = 0; x < w; ++x)
        if (c->h_nbmask[(size_t)y * w + x] & NB_FREE)
          frb[(size_t)((y >> 3) + 1u) * c->Bp + (x >> 3)] |= 1ull << (((y & 7u) << 3) | (x & 7u));
    // run starts (free cells whose west is blocked or x % 32 == 0) numbered in block order
    std::vector<uint32_t> abase(c->nbp, 0u);
    uint64_t nrs = 0;
    for (uint32_t p = 0; p < c->nbp; ++p) {
      const uint32_t bx = p % c->Bp;
      const uint64_t f = frb[p], fw = p ? frb[p - 1u] : 0ull;
      const uint64_t col0 = 0x0101010101010101ull;
      const uint64_t wf = ((f << 1) & ~col0) | ((bx & 3u) ? ((fw >> 7) & col0) : 0ull);
      abase[p] = (uint32_t)nrs;
      nrs += (uint64_t)__builtin_popcountll(f & ~wf);
    }
    c->nrs = (uint32_t)nrs;
    uint64_t nf = 0;
    for (uint32_t p = 0; p < c->nbp; ++p) nf += (uint64_t)__builtin_popcountll(frb[p]);
    c->nfree = (uint32_t)std::min<uint64_t>(nf, 0xFFFFFFFFull);
    if ((e = hipMalloc(&c->d_abase, (size_t)c->nbp * 4)) != hipSuccess) return fail("malloc abase", e);
    if ((e = hipMemcpy(c->d_abase, abase.data(), (size_t)c->nbp * 4, hipMemcpyHostToDevice)) != hipSuccess)
      return fail("copy abase", e);
    if ((e = hipMalloc(&c->d_frb, (size_t)c->nbp * 8)) != hipSuccess) return fail("malloc frb", e);
    if ((e = hipMemcpy(c->d_frb, frb.data(), (size_t)c->nbp * 8, hipMemcpyHostToDevice)) != hipSuccess)
      return fail("copy frb", e);
  }
  c->h_goal_tab.assign(ncell, -1);
  if ((e = hipMalloc(&c->d_goal_tab, (size_t)ncell * 4)) != hipSuccess) return fail("malloc goal_tab", e);
  if ((e = hipMemcpy(c->d_goal_tab, c->h_goal_tab.data(), (size_t)ncell * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail("copy goal_tab", e);
  if ((e = hipMalloc(&c->d_stat, sizeof(DevStatus))) != hipSuccess) return fail("malloc status", e);
  if ((e = hipMemsetAsync(c->d_stat, 0, sizeof(DevStatus), c->s)) != hipSuccess) return fail("memset status", e);
  if ((e = hipHostMalloc(&c->h_stat, sizeof(DevStatus), hipHostMallocDefault)) != hipSuccess)
    return fail("pinned status", e);
  if ((e = hipMalloc(&c->d_ctl, sizeof(PlanCtl))) != hipSuccess) return fail("malloc ctl", e);
  if ((e = hipMalloc(&c->d_pargs, sizeof(PlanArgs))) != hipSuccess) return fail("malloc plan args", e);
  if ((e = hipMalloc(&c->d_ticks, 48 * sizeof(unsigned long long))) != hipSuccess) return fail("malloc ticks", e);
  if ((e = hipMemsetAsync(c->d_ticks, 0, 48 * sizeof(unsigned long long), c->s)) != hipSuccess)
    return fail("memset ticks", e);
  hipDeviceGetAttribute(&c->wall_khz, hipDeviceAttributeWallClockRate, c->device);
  if (c->wall_khz <= 0) c->wall_khz = 100000;
  if ((e = hipHostMalloc(&c->h_ctl, sizeof(PlanCtl), hipHostMallocDefault)) != hipSuccess)
    return fail("pinned ctl", e);
  if ((e = hipHostMalloc(&c->h_flags, 256, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
    return fail("pinned flags", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_flags, c->h_flags, 0)) != hipSuccess)
    return fail("flags device pointer", e);
  memset(c->h_stat, 0, sizeof(DevStatus));
  size_t freeb = 0, totalb = 0;
  hipMemGetInfo(&freeb, &totalb);
  c->table_budget = (opts && opts->table_budget_bytes) ? opts->table_budget_bytes : (uint64_t)(freeb / 2);
  if ((e = hipStreamSynchronize(c->s)) != hipSuccess) return fail("stream sync", e);
  return c;
}

void tsw_destroy(tsw_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->s) hipStreamSynchronize(c->s);
  auto fre = [](void* p) {
    if (p) (void)hipFree(p);
  };
  fre(c->d_nbmask); fre(c->d_freebits); fre(c->d_frp); fre(c->d_frb); fre(c->d_abase); fre(c->d_wlg); fre(c->d_anch); fre(c->d_lovf); fre(c->d_bprof); fre(c->d_dt); fre(c->d_ktmp); fre(c->d_tmp_c); fre(c->d_nh); fre(c->d_goal_tab);
  fre(c->d_heaps); fre(c->d_gs); fre(c->d_epochs); fre(c->d_Q); fre(c->d_res); fre(c->d_lens);
  fre(c->d_gs16); fre(c->d_ep16); fre(c->d_ovf); fre(c->d_ovf2);
  fre(c->d_stat); fre(c->d_v); fre(c->d_g); fre(c->d_cnt); fre(c->d_succ); fre(c->d_ap); fre(c->d_st);
  fre(c->d_gt); fre(c->d_dec); fre(c->d_mu); fre(c->d_dups); fre(c->d_onc); fre(c->d_candc); fre(c->d_f1); fre(c->d_f2);
  if (c->h_dups) (void)hipHostFree(c->h_dups);
  fre(c->d_task); fre(c->d_occ); fre(c->d_nhc); fre(c->d_ctl); fre(c->d_pargs); fre(c->d_ticks); fre(c->d_dtag); fre(c->d_live); fre(c->d_klt); fre(c->d_kpos); fre(c->d_kbox); fre(c->d_kcnt); fre(c->d_pick); fre(c->d_dlv); fre(c->d_unused);
  fre(c->d_rec); fre(c->d_grec); fre(c->d_tmp_a); fre(c->d_tmp_b);
  fre(c->d_cc); fre(c->d_QS); fre(c->d_QT); fre(c->d_QH); fre(c->d_QP); fre(c->d_pred); fre(c->d_wf); fre(c->d_govf); fre(c->d_mg_grp); fre(c->d_mg_wl); fre(c->d_mg_anch);
  if (c->h_cc) (void)hipHostFree(c->h_cc);
  if (c->h_flags) (void)hipHostFree(c->h_flags);
  if (c->h_stat) hipHostFree(c->h_stat);
  if (c->h_ctl) hipHostFree(c->h_ctl);
  for (auto& e : c->pending) {
    hipEventDestroy(e.a);
    hipEventDestroy(e.b);
  }
  for (auto e : c->pool) hipEventDestroy(e);
  if (c->s) hipStreamDestroy(c->s);
  delete c;
}

const char* tsw_last_error(const tsw_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int tsw_abi_version(void) { return TSW_ABI_VERSION; }

uint64_t tsw_build_id(void) { return (uint64_t)TSW_SRC_HASH; }

int tsw_plan_mapd(tsw_ctx* c, const tsw_point* starts, uint32_t n, const tsw_task* tasks, uint32_t m,
                  uint32_t max_t, tsw_rec* out, uint32_t* out_T) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  return plan_impl(c, starts, n, tasks, m, max_t, out, nullptr, out_T);
}

int tsw_plan_mapd_trace(tsw_ctx* c, const tsw_point* starts, uint32_t n, const tsw_task* tasks, uint32_t m,
                        uint32_t max_t, tsw_rec* out, uint32_t* goal_out, uint32_t* out_T) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  return plan_impl(c, starts, n, tasks, m, max_t, out, goal_out, out_T);
}

int tsw_plan_mapd_resolved(tsw_ctx* c, const tsw_point* starts, uint32_t n, const tsw_task* tasks, uint32_t m,
                           uint32_t max_t, tsw_rec* out, uint32_t* goal_out, uint32_t* out_T, tsw_resolve_fn resolve,
                           void* user) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (!resolve) RET(TSW_EINVAL, "null resolver");
  c->resolver = resolve;
  c->resolver_user = user;
  const int rc = plan_impl(c, starts, n, tasks, m, max_t, out, goal_out, out_T);
  c->resolver = nullptr;
  c->resolver_user = nullptr;
  return rc;
}

int next_hop_codes_impl(tsw_ctx* c, const uint32_t* start, const uint32_t* goal, uint32_t k, uint8_t* code) {
  for (uint32_t i = 0; i < k; ++i)
    if (!cell_id_ok(c, start[i]) || !cell_id_ok(c, goal[i])) RET(TSW_EINVAL, "query cell off-grid or blocked");
  std::vector<uint32_t> goals(goal, goal + k);
  std::sort(goals.begin(), goals.end());
  goals.erase(std::unique(goals.begin(), goals.end()), goals.end());
  TRY(ensure_tables(c, goals, true));
  std::vector<AstarQuery> q;
  q.reserve(k);
  for (uint32_t i = 0; i < k; ++i) {
    if (start[i] == goal[i]) {
      code[i] = NH_STAY;
      continue;
    }
    q.push_back(AstarQuery{start[i], goal[i], c->h_goal_tab[goal[i]], i});
  }
  if (q.empty()) return TSW_OK;
  const uint32_t nq = (uint32_t)q.size();
  TRY(ensure_queue(c, nq));
  TRY(ensure_res(c, nq));
  std::vector<uint8_t> res(nq);
  for (int pass = 0; pass < 2; ++pass) {
    HIPCHK(hipMemcpyAsync(c->d_Q, q.data(), (size_t)nq * sizeof(AstarQuery), hipMemcpyHostToDevice, c->s));
    HIPCHK(launch_gather_codes(c->d_Q, nq, c->d_nh, c->tstride, c->d_res, c->s));
    HIPCHK(hipMemcpyAsync(res.data(), c->d_res, nq, hipMemcpyDeviceToHost, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    std::vector<AstarQuery> miss;
    for (uint32_t i = 0; i < nq; ++i)
      if (res[i] > NH_STAY) miss.push_back(q[i]);
    if (miss.empty()) break;
    if (pass == 1) RET(TSW_EINVAL, "next hop left unresolved by K3");
    // the exact A* into the tables (the store keeps them for later calls)
    HIPCHK(hipMemcpyAsync(c->d_Q, miss.data(), miss.size() * sizeof(AstarQuery), hipMemcpyHostToDevice, c->s));
    TRY(run_astar(c, c->d_Q, (uint32_t)miss.size(), true, nullptr, nullptr));
    TRY(check_err(c));
  }
  for (uint32_t i = 0; i < nq; ++i) code[q[i].out] = res[i];
  return TSW_OK;
}

int tsw_next_hop_codes(tsw_ctx* c, const uint32_t* start, const uint32_t* goal, uint32_t k, uint8_t* code) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!start || !goal || !code) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  const int rc = reset_pending_after(c, next_hop_codes_impl(c, start, goal, k, code));
  resolve_timing(c);
  return rc;
}

int tsw_step(tsw_ctx* c, uint32_t* v, uint32_t* g, uint32_t n) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (n == 0) return TSW_OK;
  if (!v || !g) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  std::vector<uint32_t> goals;
  goals.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (!cell_id_ok(c, v[i]) || !cell_id_ok(c, g[i])) RET(TSW_EINVAL, "agent cell off-grid or blocked");
    goals.push_back(g[i]);
  }
  TRY(ensure_agents(c, n));
  HIPCHK(hipMemcpyAsync(c->d_v, v, n * 4ull, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_g, g, n * 4ull, hipMemcpyHostToDevice, c->s));
  TRY(build_occ(c, n));
  TRY(ensure_tables(c, goals, true));
  TRY(ensure_queue(c, 4 * (size_t)n + 4096));  // needed pairs (<= 2n per exit) + speculative prefetch (qcap/2)
  if (c->tun.coop && !eager_policy(c, 0)) TRY(ensure_coop(c, n));
  PlanArgs P = plan_args(c, n, 0, MODE_STEP, false);
  PlanCtl init{};
  init.section = SEC_PRE1;
  init.chase_id = c->chase_id;
  init.move_rounds = c->tun.move_round0;
  TRY(run_plan(c, P, init));
  HIPCHK(hipMemcpyAsync(v, c->d_v, n * 4ull, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipMemcpyAsync(g, c->d_g, n * 4ull, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  c->st.steps++;
  resolve_timing(c);
  return TSW_OK;
}

static int decide_impl(tsw_ctx* c, const uint32_t* my_v, const uint32_t* my_g, uint32_t n, const uint32_t* nb_off,
                       const uint32_t* nb_v, const uint32_t* nb_g, uint32_t* act, uint32_t* cell, uint32_t* partner,
                       uint32_t* npart, uint32_t* part) {
  if (!c) return TSW_EINVAL;
  if (n == 0) return TSW_OK;
  if (!my_v || !my_g || !nb_off || !act || !cell || !partner || !npart || !part) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  const uint32_t tot = nb_off[n];
  if (nb_off[0] != 0) RET(TSW_EINVAL, "nb_off[0] must be 0");
  for (uint32_t i = 0; i < n; ++i)
    if (nb_off[i + 1] < nb_off[i]) RET(TSW_EINVAL, "nb_off must be non-decreasing");
  if (tot && (!nb_v || !nb_g)) RET(TSW_EINVAL, "null nearby list");
  // goal tables for every goal a decision can route to: own goals and the nearby agents'
  // (those on free cells — a goal off the map stops the chase, agent.rs:389-393)
  std::vector<uint32_t> goals;
  goals.reserve(n + tot);
  for (uint32_t i = 0; i < n; ++i) {
    if (!cell_id_ok(c, my_v[i]) || !cell_id_ok(c, my_g[i]))
      RET(TSW_EINVAL, "agent cell or goal off-grid or blocked (reference panics at agent.rs:358)");
    goals.push_back(my_g[i]);
  }
  for (uint32_t k = 0; k < tot; ++k)
    if (cell_id_ok(c, nb_g[k]) && cell_id_ok(c, nb_v[k])) goals.push_back(nb_g[k]);
  TRY(ensure_tables(c, goals, true));
  // device copies: inputs, outputs, pending lists (ping-pong)
  const size_t nb = std::max<uint32_t>(tot, 1u);
  std::vector<uint32_t> idx(n);
  for (uint32_t i = 0; i < n; ++i) idx[i] = i;
  uint32_t* d = nullptr;
  const size_t words = 2 * (size_t)n + (n + 1) + 2 * nb + 4 * (size_t)n + (tot + n) + 2 * (size_t)n + 2;
  HIPCHK(hipMalloc(&d, words * 4));
  uint32_t *d_v = d, *d_g = d_v + n, *d_off = d_g + n, *d_nv = d_off + n + 1, *d_ng = d_nv + nb;
  uint32_t *d_act = d_ng + nb, *d_cell = d_act + n, *d_par = d_cell + n, *d_np = d_par + n;
  uint32_t *d_part = d_np + n, *d_q0 = d_part + tot + n, *d_q1 = d_q0 + n, *d_cnt = d_q1 + n;
  auto cleanup = [&]() { hipFree(d); };
  auto fail = [&](hipError_t e) {
    cleanup();
    c->err = std::string("HIP: ") + hipGetErrorString(e);
    return TSW_EHIP;
  };
  hipError_t e;
#define DCHK(x)                                 \
  do {                                          \
    if ((e = (x)) != hipSuccess) return fail(e); \
  } while (0)
  DCHK(hipMemcpyAsync(d_v, my_v, n * 4ull, hipMemcpyHostToDevice, c->s));
  DCHK(hipMemcpyAsync(d_g, my_g, n * 4ull, hipMemcpyHostToDevice, c->s));
  DCHK(hipMemcpyAsync(d_off, nb_off, (n + 1) * 4ull, hipMemcpyHostToDevice, c->s));
  if (tot) {
    DCHK(hipMemcpyAsync(d_nv, nb_v, tot * 4ull, hipMemcpyHostToDevice, c->s));
    DCHK(hipMemcpyAsync(d_ng, nb_g, tot * 4ull, hipMemcpyHostToDevice, c->s));
  }
  DCHK(hipMemcpyAsync(d_q0, idx.data(), n * 4ull, hipMemcpyHostToDevice, c->s));
  if (int r = ensure_queue(c, std::max<size_t>(2 * ((size_t)n + tot), 1024)); r != TSW_OK) {
    cleanup();
    return r;
  }
  DecideArgs A{};
  A.W = c->G.W;
  A.ncell = c->G.ncell;
  A.my_v = d_v;
  A.my_g = d_g;
  A.nb_off = d_off;
  A.nb_v = d_nv;
  A.nb_g = d_ng;
  A.nbmask = c->d_nbmask;
  A.goal_tab = c->d_goal_tab;
  A.nh = c->d_nh;
  A.nstride = c->tstride;
  A.act = d_act;
  A.cell = d_cell;
  A.partner = d_par;
  A.npart = d_np;
  A.part = d_part;
  A.Q = c->d_Q;
  A.qcap = (uint32_t)c->qcap;
  A.err = &c->d_stat->err;
  uint32_t nq = n;
  uint32_t* qin = d_q0;
  uint32_t* qout = d_q1;
  for (int round = 0; nq > 0; ++round) {
    if (round > 1 + 2 * (int)std::min<uint64_t>(tot + n, 1u << 20)) {
      cleanup();
      RET(TSW_EINVAL, "decision made no progress");
    }
    A.qidx = qin;
    A.nq = nq;
    A.pending_out = qout;
    A.qcount = d_cnt;
    A.npending = d_cnt + 1;
    DCHK(hipMemsetAsync(d_cnt, 0, 8, c->s));
    DCHK(launch_decide(A, c->s));
    uint32_t h[2] = {0, 0};
    DCHK(hipMemcpyAsync(h, d_cnt, 8, hipMemcpyDeviceToHost, c->s));
    DCHK(hipStreamSynchronize(c->s));
    if (int r = check_err(c); r != TSW_OK) {
      cleanup();
      return r;
    }
    if (h[1] == 0) break;
    if (h[0] == 0 || h[0] > c->qcap) {
      cleanup();
      RET(TSW_EINVAL, "decision stalled on an unresolvable next hop");
    }
    if (int r = run_astar(c, c->d_Q, h[0], true, nullptr, nullptr); r != TSW_OK) {
      cleanup();
      return r;
    }
    nq = h[1];
    std::swap(qin, qout);
  }
  DCHK(hipMemcpyAsync(act, d_act, n * 4ull, hipMemcpyDeviceToHost, c->s));
  DCHK(hipMemcpyAsync(cell, d_cell, n * 4ull, hipMemcpyDeviceToHost, c->s));
  DCHK(hipMemcpyAsync(partner, d_par, n * 4ull, hipMemcpyDeviceToHost, c->s));
  DCHK(hipMemcpyAsync(npart, d_np, n * 4ull, hipMemcpyDeviceToHost, c->s));
  DCHK(hipMemcpyAsync(part, d_part, ((size_t)tot + n) * 4ull, hipMemcpyDeviceToHost, c->s));
  DCHK(hipStreamSynchronize(c->s));
#undef DCHK
  cleanup();
  resolve_timing(c);
  return TSW_OK;
}

int tsw_decide(tsw_ctx* c, const uint32_t* my_v, const uint32_t* my_g, uint32_t n, const uint32_t* nb_off,
               const uint32_t* nb_v, const uint32_t* nb_g, uint32_t* act, uint32_t* cell, uint32_t* partner,
               uint32_t* npart, uint32_t* part) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  // a failed round may leave queued pairs PENDING: reset them before returning the error
  return reset_pending_after(c, decide_impl(c, my_v, my_g, n, nb_off, nb_v, nb_g, act, cell, partner, npart, part));
}

int tsw_get_path_next(tsw_ctx* c, const uint32_t* start, const uint32_t* goal, uint32_t k, uint32_t* next,
                      int32_t* len) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!start || !goal || !next || !len) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  std::vector<AstarQuery> q;
  q.reserve(k);
  for (uint32_t i = 0; i < k; ++i) {
    if (!cell_id_ok(c, start[i]) || !cell_id_ok(c, goal[i])) RET(TSW_EINVAL, "query cell off-grid or blocked");
    if (start[i] == goal[i]) {
      next[i] = start[i];
      len[i] = 1;
      continue;
    }
    AstarQuery a;
    a.v = start[i];
    a.goal = goal[i];
    a.tab = -1;
    a.out = i;
    q.push_back(a);
  }
  if (q.empty()) return TSW_OK;
  TRY(ensure_astar_scratch(c));
  TRY(ensure_queue(c, q.size()));
  TRY(ensure_res(c, k));
  HIPCHK(hipMemcpyAsync(c->d_Q, q.data(), q.size() * sizeof(AstarQuery), hipMemcpyHostToDevice, c->s));
  TRY(run_astar(c, c->d_Q, (uint32_t)q.size(), false, c->d_res, c->d_lens));
  std::vector<uint8_t> res(k);
  std::vector<int32_t> lens(k);
  HIPCHK(hipMemcpyAsync(res.data(), c->d_res, k, hipMemcpyDeviceToHost, c->s));
  HIPCHK(hipMemcpyAsync(lens.data(), c->d_lens, k * 4ull, hipMemcpyDeviceToHost, c->s));
  TRY(check_err(c));
  for (const auto& a : q) {
    const uint8_t code = res[a.out];
    uint32_t nx = a.v;
    switch (code) {
      case 0: nx = a.v + c->G.W; break;
      case 1: nx = a.v + 1; break;
      case 2: nx = a.v - c->G.W; break;
      case 3: nx = a.v - 1; break;
      default: nx = a.v; break;
    }
    next[a.out] = nx;
    len[a.out] = lens[a.out];
  }
  resolve_timing(c);
  return TSW_OK;
}

int tsw_dist_tables(tsw_ctx* c, const uint32_t* goals, uint32_t k, uint16_t* out) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !out) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  std::vector<uint32_t> gv(goals, goals + k);
  for (uint32_t g : gv)
    if (!cell_id_ok(c, g)) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  TRY(ensure_tables(c, gv));
  TRY(require_real_tables(c, gv));
  const size_t ncell = c->G.ncell;
  TRY(build_u16(c, gv.data(), k, [&](const uint16_t* d, uint32_t i0, uint32_t nb) -> int {
    for (uint32_t j = 0; j < nb; ++j)
      HIPCHK(hipMemcpyAsync(out + (size_t)(i0 + j) * ncell, d + (size_t)j * c->tstride, ncell * 2,
                            hipMemcpyDeviceToHost, c->s));
    return TSW_OK;
  }));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_dist_tables_device(tsw_ctx* c, const uint32_t* goals, uint32_t k, uint16_t* dev_out) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !dev_out) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  for (uint32_t i = 0; i < k; ++i)
    if (!cell_id_ok(c, goals[i])) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  // dev_out may have been allocated / zero-filled on another stream of the caller (e.g. torch's
  // current stream): order every outstanding device work before writing into it
  HIPCHK(hipDeviceSynchronize());
  TRY(ensure_tmp(c, k));
  // context-owned staging (like the caller's `goals`, read by the copy before it returns)
  std::vector<uint32_t>& lg = c->h_lpt_goals;
  std::vector<uint32_t>& ls = c->h_lpt_slots;
  lg.assign(goals, goals + k);
  ls.resize(k);
  for (uint32_t i = 0; i < k; ++i) ls[i] = i;
  bfs_lpt_order(c, lg, ls);
  HIPCHK(hipMemcpyAsync(c->d_tmp_a, lg.data(), (size_t)k * 4, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipMemcpyAsync(c->d_tmp_b, ls.data(), (size_t)k * 4, hipMemcpyHostToDevice, c->s));
  TRY(run_bfs(c, c->d_tmp_a, c->d_tmp_b, k, dev_out, c->G.ncell, nullptr));
  c->st.bfs_goals += k;
  c->st.bfs_launches++;
  TRY(check_err(c));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_import_tables_device(tsw_ctx* c, const uint32_t* goals, uint32_t k, const uint16_t* dev_tables) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !dev_tables) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  for (uint32_t i = 0; i < k; ++i)
    if (!cell_id_ok(c, goals[i])) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  // the tables were produced on the caller's streams (e.g. an RCCL all-gather): complete first
  HIPCHK(hipDeviceSynchronize());
  std::vector<uint32_t> newg, src, slots;
  stamp_and_collect(c, goals, k, newg, &src);
  if (newg.empty()) return TSW_OK;
  auto ingest = [&]() -> int {
    TRY(reserve_slots(c, newg.size(), slots));
    for (uint32_t sl : slots) c->h_tab_tableless[sl] = 0;  // imported: real u16 tables
    TRY(ensure_tmp(c, newg.size()));
    HIPCHK(hipMemcpyAsync(c->d_tmp_a, newg.data(), newg.size() * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_b, slots.data(), slots.size() * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_c, src.data(), src.size() * 4, hipMemcpyHostToDevice, c->s));
    // codes and detour bytes straight from the caller's u16 tables (the store keeps no u16 copy)
    HIPCHK(launch_classify_dt(c->G, c->d_tmp_a, c->d_tmp_c, c->d_tmp_b, (uint32_t)newg.size(), dev_tables,
                              c->G.ncell, c->d_nh, c->d_dt, c->tstride, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return TSW_OK;
  };
  TRY(finish_tables(c, ingest(), newg, slots));
  if (eager_policy(c, newg.size())) TRY(resolve_all_unknown(c, newg, slots));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_next_hop_tables(tsw_ctx* c, const uint32_t* goals, uint32_t k, uint8_t* out) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !out) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  std::vector<uint32_t> gv(goals, goals + k);
  for (uint32_t g : gv)
    if (!cell_id_ok(c, g)) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  TRY(ensure_tables(c, gv, true));
  const size_t ncell = c->G.ncell;
  for (uint32_t i = 0; i < k; ++i) {
    const int32_t slot = c->h_goal_tab[gv[i]];
    HIPCHK(hipMemcpyAsync(out + (size_t)i * ncell, c->d_nh + (size_t)slot * c->tstride, ncell,
                          hipMemcpyDeviceToHost, c->s));
  }
  HIPCHK(hipStreamSynchronize(c->s));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_next_hop_tables_device(tsw_ctx* c, const uint32_t* goals, uint32_t k, uint8_t* dev_out, uint16_t* dev_dist) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !dev_out) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  std::vector<uint32_t> gv(goals, goals + k);
  for (uint32_t g : gv)
    if (!cell_id_ok(c, g)) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  HIPCHK(hipDeviceSynchronize());  // dev_out may come from another stream of the caller
  TRY(ensure_tables(c, gv));
  TRY(require_real_tables(c, gv));
  // eager resolution of this shard's multi-candidate cells, whatever the context's policy
  std::vector<uint32_t> ug, us;
  std::vector<uint8_t> seen(c->tab_count, 0);
  for (uint32_t g : gv) {
    const int32_t slot = c->h_goal_tab[g];
    if (slot >= 0 && !seen[slot]) {
      seen[slot] = 1;
      ug.push_back(g);
      us.push_back((uint32_t)slot);
    }
  }
  TRY(resolve_all_unknown(c, ug, us));
  const size_t ncell = c->G.ncell;
  for (uint32_t i = 0; i < k; ++i) {
    const int32_t slot = c->h_goal_tab[gv[i]];
    HIPCHK(hipMemcpyAsync(dev_out + (size_t)i * ncell, c->d_nh + (size_t)slot * c->tstride, ncell,
                          hipMemcpyDeviceToDevice, c->s));
  }
  // the u16 K1 tables beside the codes (the store holds detour bytes only: K1 again, into the caller's buffer)
  if (dev_dist)
    TRY(build_u16(c, gv.data(), k, [&](const uint16_t* d, uint32_t i0, uint32_t nb) -> int {
      for (uint32_t j = 0; j < nb; ++j)
        HIPCHK(hipMemcpyAsync(dev_dist + (size_t)(i0 + j) * ncell, d + (size_t)j * c->tstride, ncell * 2,
                              hipMemcpyDeviceToDevice, c->s));
      return TSW_OK;
    }));
  HIPCHK(hipStreamSynchronize(c->s));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_import_next_hops_device(tsw_ctx* c, const uint32_t* goals, uint32_t k, const uint16_t* dev_dist,
                                const uint8_t* dev_nh) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (k == 0) return TSW_OK;
  if (!goals || !dev_dist || !dev_nh) RET(TSW_EINVAL, "null argument");
  TRY(set_device(c));
  for (uint32_t i = 0; i < k; ++i)
    if (!cell_id_ok(c, goals[i])) RET(TSW_EINVAL, "goal cell off-grid or blocked");
  HIPCHK(hipDeviceSynchronize());  // produced on the caller's streams (e.g. an RCCL all-gather)
  std::vector<uint32_t> newg, src, slots;
  stamp_and_collect(c, goals, k, newg, &src);
  if (newg.empty()) return TSW_OK;
  auto ingest = [&]() -> int {
    TRY(reserve_slots(c, newg.size(), slots));
    for (uint32_t sl : slots) c->h_tab_tableless[sl] = 0;  // imported: real u16 tables
    const size_t ncell = c->G.ncell;
    for (size_t j = 0; j < newg.size(); ++j)
      HIPCHK(hipMemcpyAsync(c->d_nh + (size_t)slots[j] * c->tstride, dev_nh + (size_t)src[j] * ncell, ncell,
                            hipMemcpyDeviceToDevice, c->s));
    // detour bytes from the u16 tables (the imported codes stay: nh = null)
    TRY(ensure_tmp(c, newg.size()));
    HIPCHK(hipMemcpyAsync(c->d_tmp_a, newg.data(), newg.size() * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_b, slots.data(), slots.size() * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(hipMemcpyAsync(c->d_tmp_c, src.data(), src.size() * 4, hipMemcpyHostToDevice, c->s));
    HIPCHK(launch_classify_dt(c->G, c->d_tmp_a, c->d_tmp_c, c->d_tmp_b, (uint32_t)newg.size(), dev_dist, ncell,
                              nullptr, c->d_dt, c->tstride, c->s));
    // a pending marker from the producing context means "not resolved": unknown here — swept over
    // the imported slots only (a whole-store sweep grows with every table the context holds)
    for (size_t j = 0; j < newg.size(); ++j)
      HIPCHK(launch_reset_pending(c->d_nh + (size_t)slots[j] * c->tstride, c->tstride, c->s));
    HIPCHK(hipStreamSynchronize(c->s));
    return TSW_OK;
  };
  TRY(finish_tables(c, ingest(), newg, slots));
  resolve_timing(c);
  return TSW_OK;
}

int tsw_clear_tables(tsw_ctx* c) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  TRY(set_device(c));
  HIPCHK(hipStreamSynchronize(c->s));
  std::fill(c->h_goal_tab.begin(), c->h_goal_tab.end(), -1);
  HIPCHK(hipMemcpyAsync(c->d_goal_tab, c->h_goal_tab.data(), (size_t)c->G.ncell * 4, hipMemcpyHostToDevice, c->s));
  HIPCHK(hipStreamSynchronize(c->s));
  c->tab_count = 0;
  c->tab_live = 0;
  c->tab_free.clear();
  std::fill(c->h_tab_goal.begin(), c->h_tab_goal.end(), NO_GOAL);
  c->st.tables = 0;
  return TSW_OK;
}

int tsw_get_stats(const tsw_ctx* c, tsw_stats* out) {
  if (!c || !out) return TSW_EINVAL;
  tsw_ctx* cc = const_cast<tsw_ctx*>(c);
  resolve_timing(cc);
  unsigned long long ticks[8] = {0};
  if (hipSetDevice(c->device) == hipSuccess && hipStreamSynchronize(c->s) == hipSuccess)
    (void)hipMemcpy(ticks, c->d_ticks, sizeof ticks, hipMemcpyDeviceToHost);
  *out = c->st;
  out->tables = c->tab_live;
  out->table_evictions = c->evictions;
  for (int k = 0; k < 8; ++k) out->plan_section_ms[k] = (double)ticks[k] / (double)c->wall_khz;
  return TSW_OK;
}

int tsw_reset_stats(tsw_ctx* c) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  resolve_timing(c);
  const uint64_t tabs = c->st.tables;
  c->st = tsw_stats{};
  c->st.tables = tabs;
  if (c->d_ticks) (void)hipMemsetAsync(c->d_ticks, 0, 48 * sizeof(unsigned long long), c->s);
  return TSW_OK;
}

int tsw_set_timing(tsw_ctx* c, int enabled) {
  if (!c) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  resolve_timing(c);
  c->timing = enabled != 0;
  return TSW_OK;
}

int tsw_probe_round_floors(tsw_ctx* c, uint32_t block, double* out) {
  if (!c || !out) return TSW_EINVAL;
  NOT_FROM_RESOLVER(c);
  if (block == 0) block = c->st.plan_block ? c->st.plan_block : PLAN_BLOCK_MAX;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->s));
  HIPCHK(probe_round_floors(block, std::max<uint32_t>(c->acap ? (uint32_t)c->acap : 1024u, 64u), c->s, &out[0],
                            &out[1]));
  return TSW_OK;
}

}  // extern "C"
