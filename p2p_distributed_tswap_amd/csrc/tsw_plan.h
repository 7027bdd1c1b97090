// tsw_plan.h — arguments and resumable control block of the persistent plan kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "tsw_internal.h"

namespace tsw {

enum : uint32_t {
  SEC_ASSIGN = 0,
  SEC_PRE1 = 1,
  SEC_RULES = 2,
  SEC_PRE2 = 3,
  SEC_MOVE = 4,
  SEC_RECORD = 5,
  SEC_DONE = 6,
};
enum : uint32_t { PLAN_RUNNING = 0, PLAN_NEED_QUERIES = 1, PLAN_DONE = 2, PLAN_ERROR = 3 };
enum : uint32_t { MODE_MAPD = 0, MODE_STEP = 1 };
// k_plan's workgroup size cap (its __launch_bounds__). The planner's live state peaks at ~195 VGPRs; at
// 1,024 threads (4 waves per SIMD) a wave gets 128, so ~60 VGPRs spill, but its latency-bound per-agent
// passes (K4 scan, walk-ahead, movement rounds) run one agent per thread on C3. Round 6 measured the
// spill-free 512-thread bound 3-6 % slower end to end (ASSIGN +25 ms, PRE1 +40 ms per busy C3 plan:
// two agents per thread, one after the other), profiles/r6/ab_r6_pg.txt.
constexpr uint32_t PLAN_BLOCK_MAX = 1024;
constexpr uint32_t TASK_TAKEN = 0xFFFFFFFFu;  // PlanArgs::live entry of an assigned task

// Persisted in device memory between launches (exact resume point).
struct PlanCtl {
  uint32_t t;         // timesteps recorded so far
  uint32_t section;   // SEC_*
  uint32_t i;         // rules: cursor (first agent not yet scanned); movement: DEC initialised
  uint32_t in_chase;  // (unused, kept for layout)
  uint32_t b;
  uint32_t ap_len;
  uint32_t chase_id;
  uint32_t status;    // PLAN_*
  uint32_t qcount;    // pairs enqueued for K3
  uint32_t err;       // ERR_* bits
  uint32_t unused;    // tasks not yet used
  uint32_t max_t;     // stop when t > max_t
  uint32_t miss;      // serial movement scan: 1 = unresolved next hop, 2 = goal without table
  uint32_t steps_run;
  uint32_t rule_rounds;  // first-firing rounds executed (rules phase)
  uint32_t move_rounds;  // decidability rounds executed (movement phase)
  uint32_t relabel_full;  // rules-phase relabels by block-wide pointer doubling
  uint32_t relabel_inc;   // ... and incremental ones (walks from the changed agents)
};

struct PlanArgs {
  uint32_t n, m, W, ncell;
  uint32_t mode, agents_lds, occ_lds, tasks_lds;
  uint32_t has_dups, prefetch;  // prefetch: enqueue rules-round next hops up front (rules_prefetch)
  uint32_t f_lds;               // F1/F2 carved in LDS although the agent arrays are global
  uint32_t mu_lds;              // occ_lds and the movement rounds' MU words in LDS too
  uint32_t part_lds;            // !agents_lds: PART_* agent arrays carved in LDS anyway (flat accesses)
  uint32_t wave_rules_max;      // rules rounds run in wave 0 alone when n <= this
  uint32_t walk_cap;            // wave rules batches: longest successor walk a batched firing may take
  uint32_t wide_prefetch;       // 0: off; else also (succ cell, goal) of every agent, path walked this many hops ahead
  uint32_t wide_hi, wide_lo;    // coop mode: step-start walk-ahead hops when the speculative backlog is small / large
  uint32_t spec_hi;             // coop mode: backlog (queued, unclaimed speculative pairs) counted as small up to this
  uint32_t dag_prefetch;        // walk-ahead also queues the shortest-path successors of the first unresolved cell
  uint32_t dag_width;           // ... at most this many cells per DAG level (0: 4)
  uint32_t urgent_hops;         // coop: walk-ahead pairs within this many hops (pickup pairs within + 1) go to the needed queue
  uint32_t ab_flags;            // diagnostic A/B switches (Tunables::ab_flags; 0 in the product build)
  uint32_t t0_delay_ticks;      // diagnostic: idle after step 0's assignment (100 MHz ticks)
  uint32_t prefetch_ext;        // bit 0: DAG from an agent's own unresolved cell; bit 1: walk on past the pickup
  const uint8_t* dt;            // detour bytes of the table store (nstride per slot; tsw_internal.h), for dag_prefetch
  const uint8_t* nbmask;        // per cell: bit d = neighbour in direction d is free
  uint32_t* v;
  uint32_t* g;
  uint8_t* st;
  int32_t* task;
  int32_t* gt;    // per agent goal-table slot (global copy, used when agents are not in LDS)
  uint32_t* succ; // per agent successor / target cell (global copy)
  uint8_t* nhc;   // per agent next-hop code (global copy)
  uint8_t* dec;   // per agent movement-round state (persisted across relaunches)
  uint8_t* onc;   // per agent rule-4 cycle label (global copy)
  uint8_t* candc; // per agent rule-3 next-hop prefetch (global copy)
  uint32_t* f1;   // pointer-doubling buffers, n + 1 entries each (global copy)
  uint32_t* f2;
  uint32_t* mk;   // per agent batch marks of the wave rules rounds (global copy, n + 1 entries)
  uint32_t* occ;  // per cell occupancy
  uint64_t* mu;   // per cell round-tagged lowest undecided targeting agent (global copy)
  // K4 spatial index (tsw_capi.hip plan_impl): the tasks in Morton order of their pickup points (coordinates
  // clamped to 0xFFFE). live[pos] = pickup point (x | y << 16) while unused, TASK_TAKEN once assigned; klt[pos] =
  // the task index; kpos[task] = its position; chunks of KCH positions have a static bounding box kbox
  // (x0 | y0 << 16, x1 | y1 << 16) and a count of untaken entries kcnt. Padding entries are TASK_TAKEN.
  uint32_t* live;
  const uint32_t* klt;
  const uint32_t* kpos;
  const uint2* kbox;
  uint32_t* kcnt;
  uint32_t kchunks;
  const uint32_t* pick;
  const uint32_t* dlv;
  const int32_t* goal_tab;
  uint8_t* nh;
  uint64_t nstride;
  AstarQuery* Q;
  uint32_t qcap;
  uint64_t* rec;
  uint32_t* grec;
  PlanCtl* ctl;
  unsigned long long* sec_ticks;  // [48] wall-clock ticks per section [0..7], sub-phase ticks and counters [8..47] (diagnostics)
  uint32_t dbg;                   // sub-phase ticks on (TSW_PLAN_DEBUG)
  uint32_t* dtag;                 // diagnostics (TSW_PLAN_DEBUG): per agent, what changed it since PRE1 (CoopCtl::dbg_tag)
  // coop mode: K3 runs concurrently in the dispatch's worker workgroups (tsw_worker.h); Q is the needed queue (qcap entries for the
  // whole launch), QS the speculative one; missing next hops are waited for instead of exiting
  uint32_t coop;
  AstarQuery* QS;
  uint32_t qscap;
  AstarQuery* QH;  // hot task chains: (pickup, delivery) of every task as it is assigned (qhcap = m entries)
  uint32_t qhcap;
  // predicted task chains: (delivery cell, agent) of an agent that picks up a task (and, with bit 1 of
  // predict, of a delivering agent whose goal a rule changed); a worker predicts the task the agent will
  // be assigned at that cell — the nearest untaken pickup now — and walks that task's chain (tsw_worker.h)
  uint2* QP;
  uint32_t qpcap;
  uint32_t predict;     // bit 0: at pickups, bit 1: at goal changes of delivering agents
  uint32_t* pred;       // diagnostics (TSW_PLAN_DEBUG): per agent, the task last predicted for it
  uint4* wf;            // per agent: step-start walk-ahead frontier (cell at the walk, goal, stopping cell, its hop); nullptr: off
  CoopCtl* cc;
  // host-visible (pinned, system-coherent) words: [0] set when the planner block is resident,
  // [1] abort (host watchdog: planner waits give up, workers exit), [2] planner heartbeat (timesteps)
  uint32_t* hflags;
};

// Agent arrays that go to LDS one by one when all of them do not fit (PlanArgs::part_lds), in the
// order the host admits them: the rules phase's successor chains and labels first (its relabel walks
// and firing scans are serial dependent loads), then cells and goals, then the code caches.
enum : uint32_t {
  PART_SUCC = 1u, PART_ONC = 2u, PART_V = 4u, PART_G = 8u, PART_NHC = 16u, PART_CANDC = 32u, PART_GT = 64u,
  PART_PG = 0x3Fu,  // the subset k_plan<false, *, *, true> carves unconditionally (LDS-typed accesses)
};
size_t part_lds_bytes(uint32_t n, uint32_t part);
// flinks: the pointer-doubling buffers F1/F2 alone in LDS (when the agent arrays are not)
size_t plan_lds_bytes(uint32_t n, uint32_t ncell, uint32_t m, bool agents, bool occ, bool tasks, bool flinks = false,
                      bool mu = true, uint32_t part = 0u);
hipError_t launch_occ(const uint32_t* v, uint32_t n, uint32_t* occ, uint32_t* cnt, uint32_t ncell, uint32_t* dups,
                      hipStream_t s);
// Coop-mode K3 workers (tsw_worker.h) run in the workgroups 1.. of the plan dispatch: claim queued
// pairs from cc's queues (needed first), resolve them with the exact A* and write the next-hop code;
// exit when the planner has stopped and the needed queue is drained (speculative leftovers are
// abandoned).
struct WorkerArgs {
  DevGrid G;
  CoopCtl* cc;
  const AstarQuery* QN;
  const AstarQuery* QS;
  const AstarQuery* QT;  // task chains: (pickup, delivery) of every task, walked hop by hop
  const AstarQuery* QH;  // hot task chains: the same walk for tasks the planner has just assigned (first)
  const uint2* QP;       // predicted task chains: (delivery cell, agent); the chain of the predicted task (PlanArgs::QP)
  const uint32_t* klive;  // K4 spatial index (PlanArgs::live / klt / kbox / kcnt), read for predictions
  const uint32_t* klt;
  const uint2* kbox;
  const uint32_t* kcnt;
  uint32_t kchunks;
  const uint32_t* pick;
  const uint32_t* dlv;
  const int32_t* goal_tab;
  uint32_t* pred;         // diagnostics: per agent, the task last predicted for it (nullptr: off)
  uint8_t* nh;
  uint64_t nstride;
  uint32_t hcap;      // LDS heap entries
  uint32_t gs_lds;    // 0: u32 g-scores in the global slots, 1: u32 in LDS, 2: bytes in LDS
  uint32_t stage_fb;  // free-cell bitmap staged in LDS (else read from global memory / L2)
  uint32_t tmask;     // workers with (blockIdx & tmask) == tmask also take task-chain jobs
  uint32_t preempt;   // chain workers serve queued needed / speculative pairs between hops
  uint32_t chain_hops;  // hops a chain worker resolves per task chain (0: the whole pickup -> delivery path)
  const uint32_t* hflags;  // host watchdog words (hflags[1] = abort)
  uint32_t* gs_all;   // per-wave global g-score slots (tier 2 / tier 3), ncell u32 each
  uint32_t* epochs;   // per-slot tag epochs
  uint64_t* heaps;    // per-wave global heaps (tier 3), ghcap entries each
  uint32_t ghcap;
  uint32_t avoid_xcc;  // workers placed on the planner's XCD exit at once (its L2 stays the planner's)
  uint32_t wpb;        // worker waves per workgroup (each owns lds_per_wave bytes of the dynamic LDS)
  uint32_t lds_per_wave;
  uint32_t nworkers;   // worker waves in the dispatch (<= the global g-score / heap slots)
  // exact DAG early exit of the A* (tsw_astar.h): 0 off, 1 the goal's detour bytes staged in this
  // wave's LDS (after the free bitmap), 2 the goal's detour bytes read from the table store
  uint32_t dag;
  const uint8_t* dt;     // detour bytes of the table store, nstride per goal slot
  uint32_t dag_mask;     // the DAG test runs when (pops & dag_mask) == 0
  uint32_t stale_steps;  // speculative entries queued more than this many timesteps ago are dropped (0: never)
  uint32_t reg_heap;     // A* heaps up to this many entries live in registers (0: LDS array only; <= 63)
  uint32_t wake_gate;    // idle workers with (wid & wake_gate) == (pub & wake_gate) rescan at once on a publish
  uint32_t slow_mask, slow_mult;  // idle workers with (wid & slow_mask) != 0 poll slow_mult times less often
  unsigned long long idle_ticks;  // a worker idle this long (100 MHz ticks) exits (5 s)
};
// Worker placement: per-wave LDS (heap, g-scores, free bitmap) sets the waves per CU. g-scores stay
// in LDS (fastest per pop) unless that leaves < 3 waves per CU while many agents can need queries at
// once (n > 2000): then they move to the global slots and more waves run.
struct WorkerCfg {
  uint32_t gs_lds, stage_fb, hcap, waves;
  uint32_t dag;  // WorkerArgs::dag
  size_t lds;
};
WorkerCfg worker_config(const DevGrid& G, int num_cu, uint32_t n_agents, uint32_t hcap_want, int force_gs = -1,
                        bool dag_exit = true, size_t lds_cap = 160u * 1024u, int force_fb = -1);

// The plan dispatch: workgroup 0 runs k_plan's planner (block threads, lds bytes of dynamic LDS);
// with W (coop mode) workgroups 1..worker_blocks run W->wpb K3 worker waves each.
hipError_t launch_plan(const PlanArgs& P, PlanArgs* d_args, const WorkerArgs* W, uint32_t worker_blocks, size_t lds,
                       uint32_t block, hipStream_t s);

}  // namespace tsw
