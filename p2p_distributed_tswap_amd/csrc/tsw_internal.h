// tsw_internal.h — device-side data layout shared by the HIP kernels and the
// host context (tsw_capi.hip). gfx950 only.
//
// HBM layout (per context):
//   nbmask  [ncell]            u8   bit d (0..3) = neighbour in dir d exists
//                                   (S,E,N,W: tswap.rs:62), bit 7 = free cell
//   freebits[H*Ww]             u32  row-major bitmap of free cells, Ww = ceil(W/32)
//   dist    [cap][tstride]     u16  K1 BFS table per goal (TSW_DIST_INF = blocked /
//                                   unreachable), tstride = round_up(ncell, 8)
//   nh      [cap][tstride]     u8   next-hop code per (goal, cell): 0..3 = move in
//                                   dir d, 4 = stay (fallback with no closer
//                                   neighbour), NH_UNKNOWN = needs exact A*
//   goal_tab[ncell]            i32  goal cell -> table slot (-1 = none)
//   tab_goal[cap]              u32  table slot -> goal cell
// Agent state (SoA, n agents): v, g (u32 cell ids), st (u8), task (i32),
// occ[ncell] (i32 lowest agent index at cell, -1 none), cnt[ncell] (u32).
#pragma once
#include <stdint.h>

namespace tsw {

constexpr uint8_t NH_STAY = 4;
constexpr uint8_t NH_PENDING = 0xFE;
constexpr uint8_t NH_UNKNOWN = 0xFF;
constexpr uint16_t DIST_INF = 0xFFFF;
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
  uint16_t* dist;
  uint8_t* nh;
  int32_t* goal_tab;
  uint32_t* tab_goal;
  uint64_t tstride;  // elements per table (dist and nh)
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

// serial-commit (walker) resumable state, tswap.rs:180-285
struct WalkState {
  uint32_t phase;     // 0 rules, 1 movement, 2 done
  uint32_t i;         // current agent
  uint32_t in_chase;  // rule-4 chase in progress
  uint32_t b;         // current_b_idx
  uint32_t ap_len;    // len(a_p)
  uint32_t chase_id;  // membership stamp for a_p.contains()
  uint32_t status;    // 0 = phase finished, 1 = stopped on an unresolved next hop
  uint32_t miss_agent;
};

struct AgentsDev {
  uint32_t n;
  uint32_t* v;
  uint32_t* g;
  uint8_t* st;
  int32_t* task;
  int32_t* occ;
  uint32_t* cnt;
  uint32_t* stamp;
  uint32_t* ap;
};

struct TasksDev {
  uint32_t m;
  const uint32_t* pick_xy;  // x | y << 16
  const uint32_t* pick;     // cell
  const uint32_t* dlv;      // cell
  uint8_t* used;
  uint32_t* unused;         // single counter
};

}  // namespace tsw
