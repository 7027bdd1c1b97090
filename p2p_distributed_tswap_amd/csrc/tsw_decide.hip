// tsw_decide.hip — batched decentralized TSWAP decision.
//
// compute_next_move_with_tswap (src/bin/decentralized/agent.rs:329-462) for many agents at
// once: one lane per agent, each with its own local view (the nearby list of
// NearbyAgents::get_nearby, agent.rs:108-153 — every other agent within Manhattan radius 15,
// self excluded, in the caller's order; `find` takes the FIRST entry at a position).
//   Rule 1  at goal                                  -> Move(my_pos)           (:355-356)
//   Rule 2  next hop free in the view                -> Move(next)             (:454-456)
//   Rule 3  blocker sits at its goal                 -> WaitForGoalSwap(b)     (:371-377)
//   Rule 4  chase blockers by their next hops; a chase that meets a POSITION already in
//           a_p either completes a cycle (it is my position) or clears a_p (:403-411)
//           -> WaitForRotation(participants) when |a_p| > 1 and > 1 participant (:430-447)
//   Rule 5  otherwise                                -> Wait                   (:449-451)
// Every get_path(...)[1] is a next-hop code from the goal tables (K1 + K3, exact A*
// tie-break). A lane that meets an unresolved (cell, goal) pair queues it for K3 and parks
// its agent on the pending list; the host resolves the queue and relaunches the pending
// agents (each decision is a pure function of its inputs, so re-running it is exact).
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

namespace {

__device__ __forceinline__ uint32_t dec_step(uint32_t c, uint32_t code, uint32_t W) {
  switch (code) {
    case 0: return c + W;
    case 1: return c + 1;
    case 2: return c - W;
    case 3: return c - 1;
    default: return c;
  }
}

__device__ __forceinline__ int64_t dec_first_at(const uint32_t* nv, uint32_t nn, uint32_t pos) {
  for (uint32_t k = 0; k < nn; ++k)
    if (nv[k] == pos) return k;
  return -1;
}

}  // namespace

constexpr uint32_t DEC_MAX_LIST = 1024;  // nearby entries per agent (radius 15: <= 480 free cells)

__global__ void k_decide(DecideArgs A) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.nq) return;
  const uint32_t i = A.qidx[t];
  const uint32_t W = A.W, ncell = A.ncell;
  const uint32_t my_v = A.my_v[i], my_g = A.my_g[i];
  const uint32_t o0 = A.nb_off[i], nn = A.nb_off[i + 1] - o0;
  const uint32_t* nv = A.nb_v + o0;
  const uint32_t* ng = A.nb_g + o0;
  uint32_t* part = A.part + o0 + i;  // nn + 1 entries: a_p positions, then participant indices
  auto is_free = [&](uint32_t c) { return c < ncell && (A.nbmask[c] & NB_FREE); };
  // get_path(v, g)[1] (v != g, both free): true with *out = next cell, or false after queueing
  // the unresolved pair for K3
  bool pending = false;
  auto next_hop = [&](uint32_t v, uint32_t g, uint32_t* out) -> bool {
    const int32_t tab = A.goal_tab[g];
    if (tab < 0) {
      atomicOr(A.err, ERR_NO_TABLE);
      pending = true;
      return false;
    }
    uint8_t* p = A.nh + (uint64_t)tab * A.nstride + v;
    const uint8_t code = *p;
    if (code <= NH_STAY) {
      *out = dec_step(v, code, W);
      return true;
    }
    if (code == NH_UNKNOWN) {
      // queue the pair (two lanes racing on it may both queue it: K3 then resolves a
      // duplicate to the same code, which is harmless)
      // reserve the queue slot first: a pair is marked PENDING only when it is really queued
      // (past the capacity the host sees qcount > qcap and fails the call)
      const uint32_t qi = atomicAdd(A.qcount, 1u);
      if (qi < A.qcap) {
        *p = NH_PENDING;
        AstarQuery q;
        q.v = v;
        q.goal = g;
        q.tab = tab;
        q.out = qi;
        A.Q[qi] = q;
      }
    }
    pending = true;
    return false;
  };

  uint32_t act = DEC_ACT_WAIT, cell = my_v, partner = 0xFFFFFFFFu, npart = 0;
  do {
    if (my_v == my_g) {  // Rule 1
      act = DEC_ACT_MOVE;
      break;
    }
    uint32_t next;
    if (!next_hop(my_v, my_g, &next)) break;
    const int64_t b = dec_first_at(nv, nn, next);
    if (b < 0) {  // Rule 2
      act = DEC_ACT_MOVE;
      cell = next;
      break;
    }
    if (nv[b] == ng[b]) {  // Rule 3
      act = DEC_ACT_GOAL_SWAP;
      partner = (uint32_t)b;
      break;
    }
    // Rule 4 (agent.rs:379-427). a_p holds POSITIONS: my cell, then the cell of every chased
    // agent. Every chased agent is the FIRST list entry at its cell (b and nx come from `find`),
    // so "the cell of entry nx is in a_p" is "nx is my cell's first entry, or nx was chased":
    // a bitmask over list indices in private memory answers it — the participant list in
    // global memory is written, never read back.
    if (nn > DEC_MAX_LIST) {
      atomicOr(A.err, ERR_DECIDE_LIST);
      break;
    }
    uint64_t chased[DEC_MAX_LIST / 64u];
#pragma unroll
    for (uint32_t w = 0; w < DEC_MAX_LIST / 64u; ++w) chased[w] = 0ull;
    uint32_t ap_len = 1;  // a_p = [my_v]
    uint32_t cur = (uint32_t)b;
    bool found = false;
    for (uint32_t guard = 0; guard <= nn + 1u; ++guard) {
      if (nv[cur] == ng[cur]) break;
      const uint32_t cv = nv[cur], cg = ng[cur];
      if (!is_free(cv) || !is_free(cg)) break;  // not in pos2id (:389-393)
      uint32_t nd;
      if (!next_hop(cv, cg, &nd)) break;
      const int64_t nx = dec_first_at(nv, nn, nd);
      if (nx < 0) break;
      if (nv[nx] == my_v) {  // in a_p: my own cell closes the cycle (:403-408)
        found = true;
        break;
      }
      if ((chased[(uint32_t)nx >> 6] >> ((uint32_t)nx & 63u)) & 1ull) {  // in a_p elsewhere: clear (:409-411)
        ap_len = 0;
        break;
      }
      part[ap_len++] = cur;  // participant k >= 1 = the k-th chased entry (:413, :433-437)
      chased[cur >> 6] |= 1ull << (cur & 63u);
      cur = (uint32_t)nx;
    }
    if (pending) break;
    act = DEC_ACT_WAIT;
    if (found && ap_len > 1) {
      part[0] = (uint32_t)dec_first_at(nv, nn, my_v);  // exists: the entry that closed the cycle
      act = DEC_ACT_ROTATION;
      npart = ap_len;
    }
  } while (false);

  if (pending) {
    A.pending_out[atomicAdd(A.npending, 1u)] = i;
    return;
  }
  A.act[i] = act;
  A.cell[i] = cell;
  A.partner[i] = partner;
  A.npart[i] = npart;
}

hipError_t launch_decide(const DecideArgs& A, hipStream_t s) {
  if (A.nq == 0) return hipSuccess;
  hipLaunchKernelGGL(k_decide, dim3((A.nq + 255u) / 256u), dim3(256), 0, s, A);
  return hipGetLastError();
}

}  // namespace tsw
