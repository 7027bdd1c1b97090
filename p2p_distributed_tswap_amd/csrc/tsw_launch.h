// tsw_launch.h — host-callable launch wrappers for the kernels in tsw_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>

#include "tsw_internal.h"

namespace tsw {

size_t bfs_lds_bytes(const DevGrid& G, bool lds_table);

hipError_t launch_bfs(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                      uint16_t* dist_base, uint64_t dstride, uint8_t* nh_base, uint64_t nstride,
                      uint32_t* err, int max_lds, int num_cu, hipStream_t s, uint8_t* govf = nullptr);

// K1 v2 (tsw_bfs.hip): one wavefront per goal. Padded layout: word (r, c) of the W x H grid
// sits at p = (r + 1) * Wp + c, Wp = Ww + 1 (zero guard word per row, zero guard rows).
struct WaveBfsArgs {
  uint32_t W, H, Ww, Wp, npw, cap, klog;
  const uint32_t* frp;    // [npw] padded free-cell bitmap
  const uint32_t* goals;
  const uint32_t* slots;  // table slot per goal (nullptr: slot = goal index)
  uint32_t k;
  uint16_t* dist;
  uint64_t dstride;
  uint16_t* anch;         // per-wave anchor scratch, npw * 32 u16 each (cell-indexed)
  uint16_t* lovf;         // per-wave list overflow, 2 * npw u16 each
  uint32_t* work;         // goal dequeue counter (zeroed before the launch)
  uint32_t* err;
  uint8_t* govf;          // optional: govf[goal index] = 1 when its distances overflow u16
  uint32_t vec16;         // 16-B stores allowed (W % 8 == 0, 16-B aligned tables)
  uint32_t max_waves;     // waves per workgroup cap
  uint64_t scratch_waves; // waves the scratch buffers are sized for
  uint64_t* prof;         // optional: [bfs cycles, decode cycles, levels, chunks] summed over waves
};
// waves per workgroup that fit max_lds (0: the kernel does not fit this grid)
uint32_t bfs_wave_waves_per_block(uint32_t npw, uint32_t cap, int max_lds);
hipError_t launch_bfs_wave(const WaveBfsArgs& A, int max_lds, int num_cu, hipStream_t s);

// K1 v3 (tsw_bfs_blk.hip): one wavefront per goal over 8x8 cell blocks. Block (bx, by) sits at
// p = (by + 1) * Bp + bx, Bp = BW + 1 (zero guard block per block row, zero guard block rows).
struct BlkBfsArgs {
  uint32_t W, H, BW, BH, Bp, nbp, cap, klog, bp_magic;
  const uint64_t* frb;    // [nbp] padded free-cell blocks (bit r*8+c = cell (8bx+c, 8by+r))
  const uint32_t* goals;
  const uint32_t* slots;  // table slot per goal (nullptr: slot = goal index)
  uint32_t k;
  uint16_t* dist;
  uint64_t dstride;
  const uint32_t* abase;  // [nbp] index of the first run start of block p (run starts in block order)
  uint32_t nrs;           // run starts in the grid
  uint16_t* anch;         // per-wave compact anchor scratch, nrs u16 each
  uint16_t* lovf;         // per-wave list overflow, 2 * nbp u16 each
  unsigned long long* wlg;  // per-wave west-step blocks, nbp u64 each
  uint32_t* work;         // goal dequeue counter (zeroed before the launch)
  uint32_t* err;
  uint8_t* govf;          // optional: govf[goal index] = 1 when its distances overflow u16
  uint32_t vec16;         // 16-B stores allowed (W % 8 == 0, 16-B aligned tables)
  uint32_t stage;         // tables 16-B aligned (dist, dstride % 8 == 0): decoded rows leave through an
                          // LDS staging pass as coalesced 16-B stores (any W)
  uint32_t max_waves;
  uint64_t scratch_waves;  // goal slots (waves, or 2 per wave with pair) the scratch is sized for
  uint64_t* prof;         // optional: [bfs cycles, decode cycles, levels, chunks] summed over waves
  uint32_t dbg;           // TSW_BFS_DBG (diagnostics): 1 nontemporal table stores, 2 no WL atomics, 4 no anchors
  uint32_t wls;           // west-step blocks in LDS (k_bfs_blk<true, *>) instead of global scratch
  uint32_t pair;          // two goals per wave, one per 32-lane half (k_bfs_blk<*, true>)
};
// waves per workgroup that fit LDS (pair: two goal slots per wave)
uint32_t bfs_blk_waves_per_block(uint32_t nbp, uint32_t cap, int max_lds, bool wls, bool pair);
hipError_t launch_bfs_blk(const BlkBfsArgs& A, int max_lds, int num_cu, hipStream_t s);

// K1 v4 (tsw_bfs_big.hip): one WORKGROUP per goal over 8x8 cell blocks, free blocks and run
// numbering read from global memory (L2-resident), for grids too large for k_bfs_blk's per-wave LDS.
struct BigBfsArgs {
  uint32_t W, H, BW, BH, Bp, nbp, cap, klog, bp_magic;
  const uint64_t* frb;    // [nbp] padded free-cell blocks (global)
  const uint32_t* abase;  // [nbp] first run-start index of block p (global)
  const uint32_t* goals;
  const uint32_t* slots;  // table slot per goal (nullptr: slot = goal index)
  uint32_t k;
  uint16_t* dist;
  uint64_t dstride;
  uint32_t nrs;
  uint16_t* anch;         // per-workgroup compact anchor scratch, nrs u16 each
  uint16_t* lovf;         // per-workgroup list overflow, 2 * nbp u16 each
  uint64_t* wlg;          // per-workgroup west-step blocks, nbp u64 each
  uint32_t* work;         // goal dequeue counter (zeroed before the launch)
  uint32_t* err;
  uint8_t* govf;          // optional: govf[goal index] = 1 when its distances overflow u16
  uint32_t vec16;
  uint32_t scratch_wgs;   // workgroups the scratch buffers are sized for
};
bool bfs_big_fits(uint32_t nbp, int max_lds, uint32_t* cap_out);
uint32_t bfs_big_workgroups(uint32_t nbp, uint32_t cap, int num_cu);
hipError_t launch_bfs_big(const BigBfsArgs& A, int max_lds, int num_cu, hipStream_t s);

// K1 v5 (tsw_bfs_mg.hip): one WORKGROUP per group of <= 16 same-parity goals, a u16 goal mask per
// cell in LDS; blocks numbered as k_bfs_blk (frb, abase shared with it).
struct MgBfsArgs {
  uint32_t W, H, Bp, nbp, bp_magic;  // bp_magic = ceil(2^32 / Bp): exact p / Bp for the block indices
  const uint64_t* frb;    // [nbp] padded free-cell blocks
  const uint32_t* abase;  // [nbp] first run-start index of block p
  uint32_t nrs;           // run starts in the grid
  const uint32_t* goals;  // grouped: group j = goals[grp[j] .. grp[j+1]), one cell parity, <= 16
  const uint32_t* slots;  // table slot per goal (nullptr: slot = goal index)
  const uint32_t* grp;    // [ngroups + 1] group offsets
  uint32_t ngroups;
  uint16_t* dist;
  uint64_t dstride;
  uint32_t* wl;           // per-workgroup west-step masks, wlw u32 (two cells' u16 each)
  uint32_t wlw;
  uint16_t* anch;         // per-workgroup run-start levels, nrs * 16 u16 each
  uint32_t* work;         // group dequeue counter (zeroed before the launch)
  uint32_t* err;
  uint32_t scratch_wgs;   // workgroups the scratch buffers are sized for
  uint64_t* prof;         // optional: [bfs cycles, decode cycles, levels] summed over groups
};
size_t bfs_mg_lds_bytes(uint32_t W, uint32_t H, uint32_t nbp);
hipError_t launch_bfs_mg(const MgBfsArgs& A, int max_lds, int num_cu, hipStream_t s);

hipError_t launch_classify(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                           const uint16_t* dist_base, uint64_t stride, uint8_t* nh_base, hipStream_t s);
// store slots[i] <- codes (nh_base != null) + detour bytes of the u16 table src[i] (or i) of `dist`
hipError_t launch_classify_dt(const DevGrid& G, const uint32_t* goals, const uint32_t* src, const uint32_t* slots,
                              uint32_t k, const uint16_t* dist, uint64_t dstride, uint8_t* nh_base, uint8_t* dt_base,
                              uint64_t tstride, hipStream_t s);

hipError_t launch_astar(const DevGrid& G, const AstarQuery* Q, const uint32_t* nq_dev, uint32_t nq_host,
                        uint32_t launch_threads, uint8_t* nh_base, uint64_t nstride, uint8_t* res,
                        int32_t* lens, uint64_t* heaps, uint32_t hcap, uint32_t* gs_all, uint32_t* epochs,
                        uint32_t nslots, uint32_t* err, hipStream_t s);

// LDS-heap A* for grids of <= 1024 cells; queries whose heap outgrows LDS land in ovf.
bool astar_lds_ok(const DevGrid& G);
hipError_t launch_astar_lds(const DevGrid& G, const AstarQuery* Q, uint32_t nq, uint8_t* nh_base, uint64_t nstride,
                            uint8_t* res, int32_t* lens, uint16_t* gs16, uint32_t* epochs, uint32_t nslots,
                            AstarQuery* ovf, uint32_t* novf, uint32_t* qnext, hipStream_t s);

// One query per wave, LDS heap (grids of > 1024 cells); gs_all/epochs: nslots u32 g_score
// arrays of ncell words (used only when the grid's g_scores do not fit LDS).
// global_gs: keep the g_scores in the global slots even when the grid's fit LDS (second tier
// for queries whose byte-encoded g_scores overflowed).
uint32_t astar_wave_slots(const DevGrid& G, int num_cu, bool global_gs = false);
bool astar_wave_lds_gs(const DevGrid& G);  // k_astar_wave keeps this grid's g_scores in LDS
// diagnostics of k_astar_wave (read once per context from the environment, tsw_capi.hip Tunables)
constexpr uint32_t ASTAR_DIAG_SERIAL = 1u;  // lone-lane heap core instead of the wave-cooperative one
constexpr uint32_t ASTAR_DIAG_PROF = 2u;    // per-query pop / clock profile printed to stderr
hipError_t launch_astar_wave(const DevGrid& G, const AstarQuery* Q, uint32_t nq, uint8_t* nh_base, uint64_t nstride,
                             uint8_t* res, int32_t* lens, uint32_t* gs_all, uint32_t* epochs, uint32_t nslots,
                             AstarQuery* ovf, uint32_t* novf, uint32_t hcap /*0: default*/, bool global_gs,
                             hipStream_t s, uint32_t* qnext = nullptr, uint32_t diag = 0);

// codes of queued (start, goal) pairs out of / into the next-hop store (caller-resolved K3)
hipError_t launch_gather_codes(const AstarQuery* Q, uint32_t nq, const uint8_t* nh, uint64_t nstride, uint8_t* out,
                               hipStream_t s);
hipError_t launch_put_codes(const AstarQuery* Q, uint32_t nq, const uint8_t* codes, uint8_t* nh, uint64_t nstride,
                            hipStream_t s);

// NH_PENDING(_S) -> NH_UNKNOWN for the pairs of queue entries [from, to)
hipError_t launch_reset_queue(const AstarQuery* Q, uint32_t from, uint32_t to, uint8_t* nh, uint64_t nstride,
                              hipStream_t s);

// NH_PENDING -> NH_UNKNOWN over nbytes of next-hop codes (error recovery)
hipError_t launch_reset_pending(uint8_t* nh, uint64_t nbytes, hipStream_t s);

// Batched decentralized decision (tsw_decide.hip, agent.rs:329-462).
constexpr uint32_t DEC_ACT_MOVE = 0, DEC_ACT_GOAL_SWAP = 1, DEC_ACT_ROTATION = 2, DEC_ACT_WAIT = 3;
struct DecideArgs {
  uint32_t W, ncell;
  const uint32_t* my_v;    // [n] agent cells
  const uint32_t* my_g;    // [n] goal cells
  const uint32_t* nb_off;  // [n + 1] nearby-list offsets
  const uint32_t* nb_v;    // nearby agents' cells (any value >= ncell: off the map)
  const uint32_t* nb_g;    // nearby agents' goal cells
  const uint8_t* nbmask;
  const int32_t* goal_tab;
  uint8_t* nh;
  uint64_t nstride;
  const uint32_t* qidx;    // agents to decide in this launch
  uint32_t nq;
  uint32_t *act, *cell, *partner, *npart;
  uint32_t* part;          // per agent i: nb_off[i] + i .. + nn_i + 1 (participant list indices)
  AstarQuery* Q;
  uint32_t* qcount;
  uint32_t qcap;
  uint32_t* pending_out;   // agents parked on an unresolved next hop
  uint32_t* npending;
  uint32_t* err;
};
hipError_t launch_decide(const DecideArgs& A, hipStream_t s);

hipError_t launch_enqueue_unknown(const DevGrid& G, const uint32_t* goals, const uint32_t* slots, uint32_t k,
                                  uint8_t* nh, uint64_t nstride, AstarQuery* Q, uint32_t* qcount,
                                  uint32_t qcap, hipStream_t s);

// Latency floors of k_plan's round shapes (tsw_probe.hip): us per wave-0 rules firing chain and per
// block-wide pass (LDS exchange + barrier) on a `block`-thread workgroup.
hipError_t probe_round_floors(uint32_t block, uint32_t n, hipStream_t s, double* us_wave_round, double* us_block_pass);

}  // namespace tsw
