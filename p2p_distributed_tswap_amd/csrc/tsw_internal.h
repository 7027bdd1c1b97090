// tsw_internal.h — device-side data layout shared by the HIP kernels and the
// host context (tsw_capi.hip). gfx950 only.
//
// HBM layout (per context):
//   nbmask  [ncell]            u8   bit d (0..3) = neighbour in dir d exists
//                                   (S,E,N,W: tswap.rs:62), bit 7 = free cell
//   freebits[H*Ww]             u32  row-major bitmap of free cells, Ww = ceil(W/32)
//   dt      [cap][tstride]     u8   detour byte per (goal, cell): min((D - |c - goal|_1) / 2, 255),
//                                   D = the K1 BFS distance; 255 = blocked / unreachable / detour
//                                   >= 510 (round 6: the u16 table D is built per batch, classified
//                                   and dropped), tstride = round_up(ncell, 8)
//   nh      [cap][tstride]     u8   next-hop code per (goal, cell): 0..3 = move in
//                                   dir d, 4 = stay (fallback with no closer
//                                   neighbour), NH_UNKNOWN = needs exact A*
//   goal_tab[ncell]            i32  goal cell -> table slot (-1 = none)
//   tab_goal[cap]              u32  table slot -> goal cell
// Agent state (SoA, n agents): v, g (u32 cell ids), st (u8), task (i32); occupancy
// occ[ncell] (u32 lowest agent index at the cell | 0x80000000 if shared, ~0 if empty).
// Persistent plan kernel arguments / control block: tsw_plan.h.
#pragma once
#include <stdint.h>

// Diagnostic-build switches (-DTSW_DIAG, libtswap_hip_diag.so): in the production build every
// diagnostic bit reads as 0, so the code paths that drop work for measurement are compiled out.
#ifdef TSW_DIAG
#define TSW_DIAG_BITS(x) (x)
#else
#define TSW_DIAG_BITS(x) 0u
#endif

namespace tsw {

constexpr uint8_t NH_STAY = 4;
constexpr uint8_t NH_PENDING_S = 0xFD;  // queued speculatively for the concurrent K3 workers (coop mode)
constexpr uint8_t NH_PENDING = 0xFE;    // queued for a K3 pass (needed)
constexpr uint8_t NH_UNKNOWN = 0xFF;
constexpr uint16_t DIST_INF = 0xFFFF;
constexpr uint8_t DT_NONE = 0xFF;  // detour byte: blocked / unreachable / saturated
constexpr uint8_t NB_FREE = 0x80;

// internal agent states (tswap.rs:84-88)
constexpr uint8_t ST_IDLE = 0, ST_TO_PICKUP = 1, ST_TO_DELIVERY = 2;

// A* heap entry: f:21 | g:21 | x:11 | y:11. Rust Ord (tswap.rs:314-321)
// "a > b <=> a.f < b.f || (a.f == b.f && a.g < b.g)" == "key(a) < key(b)"
// with key = entry >> 22.
constexpr int KEY_SHIFT = 22;
constexpr uint32_t MAX_WH = 2048;             // x, y fit 11 bits
constexpr uint32_t MAX_CELLS = 1u << 20;      // g fits 20 bits in the g_score word
constexpr uint32_t GS_G_MASK = (1u << 20) - 1;

struct DevGrid {
  uint32_t W, H, ncell, Ww;
  const uint8_t* nbmask;
  const uint32_t* freebits;
};

struct Tables {
  uint8_t* dt;
  uint8_t* nh;
  int32_t* goal_tab;
  uint32_t* tab_goal;
  uint64_t tstride;  // elements per table (dist and nh)
};

// Concurrent K3 (coop mode): the planner publishes queued pairs, persistent A* worker waves on the
// other CUs — workgroups 1.. of the same k_plan dispatch — claim and resolve them while the planner keeps
// running (tsw_worker.h).
// Counters live on separate 128-B lines (claimed by CAS from many CUs, polled by the planner).
struct CoopCtl {
  uint32_t head_n, pad0[31];   // needed queue: entries published by the planner
  uint32_t claim_n, pad1[31];  // needed queue: entries claimed by workers
  uint32_t head_s, pad2[31];   // speculative queue: published
  uint32_t claim_s, pad3[31];  // speculative queue: claimed
  uint32_t head_t, pad5[31];   // task-chain queue (filled by the host before the launch)
  uint32_t claim_t, pad6[31];  // task-chain queue: claimed
  uint32_t head_h, pad9[31];   // hot task chains: tasks the planner has assigned (published like head_s)
  uint32_t claim_h, pad10[31]; // hot task chains: claimed
  uint32_t head_p, pad11[31];   // predicted task chains: delivery cells whose next task a worker predicts
  uint32_t claim_p, pad12[31];  // predicted task chains: claimed
  uint32_t pub, pad7[31];      // planner publish count: idle workers poll this one word
  uint32_t planner_xcc, pad8[31];  // 1 + XCD of the planner block (0: unknown), written before it signals residency
  uint32_t stop, alive, err, waits;  // planner finished / workers started / worker error bits / planner waits
  unsigned long long wait_ticks;     // planner time spent waiting on workers (100 MHz ticks)
  unsigned long long worker_queries; // queries resolved by workers
  unsigned long long chain_queries;  // ... of which on task chains
  unsigned long long wait_sec[8];    // wait ticks by planner section (SEC_*)
  uint32_t waits_sec[8];             // waits by planner section
  // diagnostics (TSW_PLAN_DEBUG): pairs a step needed that were unresolved, per section group
  // (PRE1, RULES, MOVE, other) x (never queued, queued speculatively but not resolved yet)
  uint32_t dbg_need[8];
  // diagnostics: worker wall-clock ticks inside A* and queries, by queue (needed, spec, chain)
  unsigned long long wbusy[4];
  uint32_t wcount[4];
  unsigned long long wpops[4];  // ... and heap pops (all tiers)
  unsigned long long qdelay[2];  // diagnostics: enqueue -> claim wall ticks, needed / speculative queue
  uint32_t qlate[2];             // ... claims later than 1 ms after the enqueue
  uint32_t qskip[2];             // claimed pairs already resolved when claimed (not searched again)
  // diagnostics: speculative-queue backlog (published - claimed) when a planner wait starts
  unsigned long long dbg_depth;
  uint32_t dbg_depth_max;
  // the planner's current timestep (agent-scope store at every step end): speculative entries carry
  // their enqueue timestep, and a worker drops one older than WorkerArgs::stale_steps unresolved
  // (its code goes back PENDING_S -> UNKNOWN)
  uint32_t t_now;
  uint32_t spec_dropped;  // ... entries dropped that way
  uint32_t pad4;
  // diagnostics (TSW_PLAN_DEBUG): PRE1 agents whose pair was unresolved after the step-start refresh, by
  // what changed them since the previous PRE1 (PlanArgs::dtag bits: 1 rule-3 b, 2 rule-3 s, 4 rotated,
  // 8 moved, 16 assigned, 32 picked up), [0] unknown / [1] pending-speculative per tag combination
  uint32_t dbg_tag[2][64];
  // predicted task chains: jobs run, and (TSW_PLAN_DEBUG) assignments whose task was the agent's last prediction
  uint32_t pred_jobs, pred_asg, pred_hit, pred_none;
};

struct AstarQuery {
  uint32_t v;     // start cell
  uint32_t goal;  // goal cell
  int32_t tab;    // table slot to write the code into (-1: none)
  uint32_t out;   // index into the result array
};

// error bits reported by kernels
constexpr uint32_t ERR_HEAP_OVERFLOW = 1u;
constexpr uint32_t ERR_DIST_OVERFLOW = 2u;
constexpr uint32_t ERR_G_OVERFLOW = 4u;
constexpr uint32_t ERR_NO_TABLE = 8u;
constexpr uint32_t ERR_WALK_OVERFLOW = 16u;
constexpr uint32_t ERR_BFS_LIST = 32u;     // k_bfs_wave: a queued word gained no cell (logic error)
constexpr uint32_t ERR_DECIDE_LIST = 64u;  // k_decide: a nearby list longer than DEC_MAX_LIST
constexpr uint32_t ERR_ABORT = 128u;       // k_plan: stopped by the host watchdog (no step for 10 s)
constexpr uint32_t ERR_BAD_PICKUP = 256u;  // k_plan: assigned a task whose pickup is off-grid/blocked (tswap.rs:136)
constexpr uint32_t ERR_BAD_DELIVERY = 512u;  // k_plan: reached a pickup whose delivery is off-grid/blocked (:112)
// task cell that is off-grid or blocked: the reference panics only when the planner looks it up
constexpr uint32_t CELL_BAD = 0xFFFFFFFFu;

}  // namespace tsw
