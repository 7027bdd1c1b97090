// tsw_plan.hip — k_plan: the persistent MAPD planning kernel (K2 step + K4 assignment).
//
// One workgroup (16 waves) runs whole timesteps of tswap_mapd (tswap.rs:104-170) on the
// device without returning to the host:
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
//           Agents that do not fire change nothing, so this equals the sequential scan.
//   PRE2    parallel lookup for agents whose goal changed
//   MOVE    serial movement phase (tswap.rs:257-285) on LDS-resident state
//   RECORD  parallel (Point, AgentState) record (tswap.rs:144-158) + termination (:163-169)
// When a next hop is unresolved (lazy next-hop mode) the kernel enqueues every such
// (cell, goal) pair, saves its exact resume point and exits; the host runs K3 (k_astar)
// and relaunches.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_plan.h"

namespace tsw {

namespace {

constexpr uint8_t NHC_DIRTY = 0xFE;  // per-agent next-hop code must be re-looked-up
constexpr uint32_t OCC_NONE = 0xFFFFFFFFu;
constexpr uint32_t OCC_FLAG = 0x80000000u;  // cell holds more than one agent (duplicate starts)
constexpr uint32_t OCC_IDX = 0x7FFFFFFFu;
constexpr uint32_t SUCC_TERM = 0xFFFFFFFFu;
constexpr uint32_t NO_AGENT = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t step_cell(uint32_t c, uint32_t code, uint32_t W) {
  switch (code) {
    case 0: return c + W;
    case 1: return c + 1;
    case 2: return c - W;
    case 3: return c - 1;
    default: return c;
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t y = __shfl_xor(x, off, 64);
    x = y < x ? y : x;
  }
  return x;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t y = __shfl_xor(x, off, 64);
    x = y < x ? y : x;
  }
  return x;
}

// Agent/occupancy arrays; AG / OC select LDS (compile time) so loads are ds_read, not flat.
struct Arrays {
  uint32_t* V;
  uint32_t* G;
  uint32_t* SUCC;
  uint8_t* NHC;
  uint32_t* OCC;
  const uint32_t* PXY;
  uint8_t* USED;
};

// next-hop code of agent k for its current (v, g); -1 unresolved, -2 goal has no table
__device__ __forceinline__ int lookup_code(const PlanArgs& P, const Arrays& S, uint32_t k) {
  const uint8_t c = S.NHC[k];
  if (c <= NH_STAY) return c;
  const int32_t tab = P.goal_tab[S.G[k]];
  if (tab < 0) return -2;
  const uint8_t code = P.nh[(uint64_t)tab * P.nstride + S.V[k]];
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

// Rule 4 test for agent k with succ(k) = s (s != k, s not at goal): does the chase of
// tswap.rs:205-238 return to k? == k lies on a cycle of succ. Floyd walk from k.
__device__ __forceinline__ bool on_cycle(const Arrays& S, uint32_t k, uint32_t n) {
  uint32_t tort = k, hare = k;
  for (uint32_t it = 0; it <= n; ++it) {
    hare = S.SUCC[hare];
    if (hare == SUCC_TERM) return false;
    if (hare == k) return true;
    hare = S.SUCC[hare];
    if (hare == SUCC_TERM) return false;
    if (hare == k) return true;
    tort = S.SUCC[tort];
    if (hare == tort) return false;  // entered a cycle that does not contain k
  }
  return false;
}

// parallel: refresh next-hop codes of agents whose code is dirty; unresolved pairs are
// enqueued for K3. Returns the number of enqueued pairs (block-uniform).
__device__ uint32_t refresh_codes(const PlanArgs& P, const Arrays& S, uint32_t* s_q) {
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  if (tid == 0) *s_q = 0;
  __syncthreads();
  for (uint32_t k = tid; k < P.n; k += bd) {
    if (S.NHC[k] <= NH_STAY) continue;
    const uint32_t v = S.V[k], g = S.G[k];
    if (v == g) continue;
    const int32_t tab = P.goal_tab[g];
    if (tab < 0) {
      atomicOr(&P.ctl->err, ERR_NO_TABLE);
      continue;
    }
    uint8_t* p = P.nh + (uint64_t)tab * P.nstride + v;
    const uint8_t code = *p;
    if (code <= NH_STAY) {
      S.NHC[k] = code;
      continue;
    }
    if (code == NH_UNKNOWN) {
      *p = NH_PENDING;
      const uint32_t qi = atomicAdd(s_q, 1u);
      if (qi < P.qcap) {
        AstarQuery q;
        q.v = v;
        q.goal = g;
        q.tab = tab;
        q.out = qi;
        P.Q[qi] = q;
      }
    }
    // NH_PENDING: the agent that flipped it to PENDING in this pass enqueued it.
  }
  __syncthreads();
  return *s_q;
}

// Serial movement phase (tswap.rs:257-285); false on an unresolved next hop.
template <bool AG, bool OC>
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

template <bool AG, bool OC>
__global__ void __launch_bounds__(1024) k_plan(PlanArgs P) {
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ PlanCtl s_ctl;
  __shared__ uint32_t s_q, s_cnt, s_doit, s_px, s_py, s_exit, s_best;
  __shared__ uint32_t s_wcount[16];
  __shared__ uint64_t s_red[16];
  const uint32_t tid = threadIdx.x, bd = blockDim.x, lane = tid & 63u, wid = tid >> 6, nwaves = bd >> 6;
  const uint32_t n = P.n;

  // ---- carve LDS (order must match plan_lds_bytes) ---------------------------
  Arrays S;
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
    S.SUCC = reinterpret_cast<uint32_t*>(carve((size_t)n * 4));
    S.NHC = carve(n);
  } else {
    S.V = P.v;
    S.G = P.g;
    S.SUCC = P.stamp;
    S.NHC = P.nhc;
  }
  if constexpr (OC) S.OCC = reinterpret_cast<uint32_t*>(carve((size_t)P.ncell * 4));
  else S.OCC = P.occ;
  if (P.tasks_lds) {
    uint32_t* pxy = reinterpret_cast<uint32_t*>(carve((size_t)P.m * 4));
    S.USED = carve(P.m);
    S.PXY = pxy;
    for (uint32_t k = tid; k < P.m; k += bd) {
      pxy[k] = P.pick_xy[k];
      S.USED[k] = P.used[k];
    }
  } else {
    S.PXY = P.pick_xy;
    S.USED = P.used;
  }
  for (uint32_t k = tid; k < n; k += bd) {
    if constexpr (AG) {
      S.V[k] = P.v[k];
      S.G[k] = P.g[k];
    }
    S.NHC[k] = NHC_DIRTY;
  }
  if constexpr (OC)
    for (uint32_t c = tid; c < P.ncell; c += bd) S.OCC[c] = P.occ[c];
  if (tid == 0) {
    s_ctl = *P.ctl;
    s_ctl.status = PLAN_RUNNING;
    s_exit = 0;
  }
  __syncthreads();
  if (s_ctl.section == SEC_RULES || s_ctl.section == SEC_MOVE) {
    // resuming after K3 resolved the missing next hops: every code starts dirty here
    const uint32_t q = refresh_codes(P, S, &s_q);
    if (q > 0 && tid == 0) {
      s_ctl.qcount = q;
      s_ctl.status = PLAN_NEED_QUERIES;
      s_exit = 1;
    }
    __syncthreads();
  }

  for (;;) {
    if (s_exit) break;
    const uint32_t sec = s_ctl.section;
    if (sec == SEC_ASSIGN) {
      // ---- K4: state machine + task assignment (tswap.rs:106-139) -------------
      for (uint32_t base = 0; base < n; base += bd) {
        const uint32_t i = base + tid;
        bool needy = false;
        if (i < n) {
          const uint8_t st = P.st[i];
          needy = (S.V[i] == S.G[i] && st != ST_IDLE) || (st == ST_IDLE && s_ctl.unused > 0u);
        }
        const uint64_t bal = __ballot(needy);
        if (lane == 0) s_wcount[wid] = (uint32_t)__popcll(bal);
        __syncthreads();
        if (needy) {
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
        __syncthreads();
        const uint32_t cnt = s_cnt;
        for (uint32_t kk = 0; kk < cnt; ++kk) {
          const uint32_t ai = list[kk];
          if (tid == 0) {
            const uint32_t v = S.V[ai];
            uint8_t st = P.st[ai];
            if (v == S.G[ai]) {
              if (st == ST_TO_PICKUP) {
                st = ST_TO_DELIVERY;
                const int32_t tk = P.task[ai];
                if (tk >= 0) {
                  S.G[ai] = P.dlv[tk];
                  S.NHC[ai] = NHC_DIRTY;
                }
              } else if (st == ST_TO_DELIVERY) {
                st = ST_IDLE;
                P.task[ai] = -1;
              }
              P.st[ai] = st;
            }
            s_doit = (st == ST_IDLE && s_ctl.unused > 0u) ? 1u : 0u;
            s_px = v % P.W;
            s_py = v / P.W;
          }
          __syncthreads();
          if (s_doit) {
            const uint32_t px = s_px, py = s_py;
            uint64_t best = ~0ull;
            for (uint32_t t = tid; t < P.m; t += bd) {
              if (!S.USED[t]) {
                const uint32_t xy = S.PXY[t];
                const uint32_t tx = xy & 0xFFFFu, ty = xy >> 16;
                const uint32_t d = (px > tx ? px - tx : tx - px) + (py > ty ? py - ty : ty - py);
                const uint64_t key = ((uint64_t)d << 32) | t;
                best = key < best ? key : best;
              }
            }
            best = wave_min_u64(best);
            if (lane == 0) s_red[wid] = best;
            __syncthreads();
            if (tid == 0) {
              uint64_t b = ~0ull;
              for (uint32_t w = 0; w < nwaves; ++w) b = s_red[w] < b ? s_red[w] : b;
              if (b != ~0ull) {  // first minimum (min_by_key, tswap.rs:130)
                const uint32_t t = (uint32_t)(b & 0xFFFFFFFFu);
                S.USED[t] = 1;
                if (P.tasks_lds) P.used[t] = 1;
                s_ctl.unused -= 1u;
                P.task[ai] = (int32_t)t;
                P.st[ai] = ST_TO_PICKUP;
                S.G[ai] = P.pick[t];
                S.NHC[ai] = NHC_DIRTY;
              }
            }
          }
          __syncthreads();
        }
      }
      if (tid == 0) {
        s_ctl.section = SEC_PRE1;
        s_ctl.i = 0;
      }
      __syncthreads();
    } else if (sec == SEC_PRE1 || sec == SEC_PRE2) {
      const uint32_t q = refresh_codes(P, S, &s_q);
      if (q > 0) {
        if (tid == 0) {
          s_ctl.qcount = q;
          s_ctl.status = PLAN_NEED_QUERIES;
          s_exit = 1;
        }
        __syncthreads();
        break;
      }
      if (tid == 0) s_ctl.section = sec == SEC_PRE1 ? SEC_RULES : SEC_MOVE;
      __syncthreads();
    } else if (sec == SEC_RULES) {
      // ---- rules phase as "first firing agent" rounds (see header) ------------
      for (uint32_t k = tid; k < n; k += bd) S.SUCC[k] = succ_of(P, S, k);
      __syncthreads();
      for (;;) {
        const uint32_t cursor = s_ctl.i;
        uint32_t best = NO_AGENT;
        for (uint32_t k = cursor + tid; k < n; k += bd) {
          const uint32_t s = S.SUCC[k];
          if (s == SUCC_TERM || s == k) continue;
          if (S.V[s] == S.G[s] || on_cycle(S, k, n)) {
            best = k;  // later k of this thread are larger
            break;
          }
        }
        best = wave_min_u32(best);
        if (lane == 0) s_wcount[wid] = best;
        __syncthreads();
        if (tid == 0) {
          uint32_t b = NO_AGENT;
          for (uint32_t w = 0; w < nwaves; ++w) b = s_wcount[w] < b ? s_wcount[w] : b;
          s_best = b;
          if (b != NO_AGENT) {
            const uint32_t s = S.SUCC[b];
            if (S.V[s] == S.G[s]) {  // rule 3: goal swap (tswap.rs:198-202)
              const uint32_t gb = S.G[b];
              S.G[b] = S.G[s];
              S.G[s] = gb;
              S.NHC[b] = NHC_DIRTY;
              S.NHC[s] = NHC_DIRTY;
            } else {  // rule 4: rotate targets along the cycle b -> s -> ... -> last -> b
              uint32_t L = 0;
              for (uint32_t a = b; L == 0 || a != b; a = S.SUCC[a]) P.ap[L++] = a;
              const uint32_t last_goal = S.G[P.ap[L - 1]];
              for (uint32_t kk = L - 1; kk >= 1; --kk) {
                const uint32_t a = P.ap[kk];
                S.G[a] = S.G[P.ap[kk - 1]];
                S.NHC[a] = NHC_DIRTY;
              }
              S.G[b] = last_goal;
              S.NHC[b] = NHC_DIRTY;
            }
            s_ctl.i = b + 1;
          } else {
            s_ctl.i = n;
          }
        }
        __syncthreads();
        if (s_best == NO_AGENT) break;
        // goals of the fired agents changed: their next hops (hence succ) must be looked up
        const uint32_t q = refresh_codes(P, S, &s_q);
        if (q > 0) {
          if (tid == 0) {
            s_ctl.qcount = q;
            s_ctl.status = PLAN_NEED_QUERIES;
            s_exit = 1;
          }
          __syncthreads();
          break;
        }
        for (uint32_t k = tid; k < n; k += bd) S.SUCC[k] = succ_of(P, S, k);
        __syncthreads();
      }
      if (s_exit) break;
      if (tid == 0) {
        s_ctl.section = SEC_PRE2;
        s_ctl.i = 0;
      }
      __syncthreads();
    } else if (sec == SEC_MOVE) {
      if (tid == 0) {
        s_ctl.miss = 0;
        if (walk_move<AG, OC>(P, S, s_ctl)) {
          s_ctl.section = SEC_RECORD;
          s_ctl.i = 0;
        }
        if (s_ctl.miss == 2) atomicOr(&P.ctl->err, ERR_NO_TABLE);
      }
      __syncthreads();
      if (s_ctl.miss) {
        // enqueue every dirty agent's unresolved pair, then return to the host
        const uint32_t q = refresh_codes(P, S, &s_q);
        if (tid == 0) {
          s_ctl.qcount = q;
          s_ctl.status = (q > 0 && s_ctl.miss == 1) ? PLAN_NEED_QUERIES : PLAN_ERROR;
          s_exit = 1;
        }
        __syncthreads();
        break;
      }
    } else if (sec == SEC_RECORD) {
      if (P.mode == MODE_STEP) {
        if (tid == 0) {
          s_ctl.status = PLAN_DONE;
          s_ctl.section = SEC_DONE;
          s_exit = 1;
        }
        __syncthreads();
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
        rec[i] = (uint64_t)(v % P.W) | ((uint64_t)(v / P.W) << 16) | (s << 32);
        if (grec) grec[i] = g;
      }
      busy = __syncthreads_or(busy);
      if (tid == 0) {
        s_ctl.t = t + 1;
        s_ctl.steps_run += 1;
        if ((s_ctl.unused == 0u && !busy) || s_ctl.t > s_ctl.max_t) {
          s_ctl.status = PLAN_DONE;
          s_ctl.section = SEC_DONE;
          s_exit = 1;
        } else {
          s_ctl.section = SEC_ASSIGN;
        }
      }
      __syncthreads();
    } else {
      break;  // SEC_DONE
    }
  }

  // ---- write back ------------------------------------------------------------
  __syncthreads();
  if constexpr (AG)
    for (uint32_t k = tid; k < n; k += bd) {
      P.v[k] = S.V[k];
      P.g[k] = S.G[k];
    }
  if constexpr (OC)
    for (uint32_t c = tid; c < P.ncell; c += bd) P.occ[c] = S.OCC[c];
  if (tid == 0) {
    const uint32_t err = P.ctl->err;
    *P.ctl = s_ctl;
    P.ctl->err |= err;
  }
}

// occupancy in the k_plan encoding: lowest agent index | OCC_FLAG if shared, OCC_NONE if empty
__global__ void k_occ_init(uint32_t* occ, uint32_t* cnt, uint32_t ncell) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncell) {
    occ[c] = OCC_NONE;
    cnt[c] = 0u;
  }
}
__global__ void k_occ_add(const uint32_t* v, uint32_t n, uint32_t* occ, uint32_t* cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    atomicAdd(&cnt[v[i]], 1u);
    atomicMin(&occ[v[i]], i);
  }
}
__global__ void k_occ_flag(uint32_t* occ, const uint32_t* cnt, uint32_t ncell) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncell && cnt[c] > 1u) occ[c] |= OCC_FLAG;
}

size_t plan_lds_bytes(uint32_t n, uint32_t ncell, uint32_t m, bool agents, bool occ, bool tasks) {
  auto r16 = [](size_t b) { return (b + 15u) & ~(size_t)15u; };
  size_t b = r16(1024 * 4);
  if (agents) b += 3 * r16((size_t)n * 4) + r16(n);
  if (occ) b += r16((size_t)ncell * 4);
  if (tasks) b += r16((size_t)m * 4) + r16(m);
  return b;
}

hipError_t launch_occ(const uint32_t* v, uint32_t n, uint32_t* occ, uint32_t* cnt, uint32_t ncell, hipStream_t s) {
  hipLaunchKernelGGL(k_occ_init, dim3((ncell + 255) / 256), dim3(256), 0, s, occ, cnt, ncell);
  if (n) hipLaunchKernelGGL(k_occ_add, dim3((n + 255) / 256), dim3(256), 0, s, v, n, occ, cnt);
  hipLaunchKernelGGL(k_occ_flag, dim3((ncell + 255) / 256), dim3(256), 0, s, occ, cnt, ncell);
  return hipGetLastError();
}

template <bool AG, bool OC>
static hipError_t launch_plan_t(const PlanArgs& P, size_t lds, hipStream_t s) {
  hipError_t e = hipFuncSetAttribute((const void*)k_plan<AG, OC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_plan<AG, OC>), dim3(1), dim3(1024), lds, s, P);
  return hipGetLastError();
}

hipError_t launch_plan(const PlanArgs& P, size_t lds, hipStream_t s) {
  if (P.agents_lds && P.occ_lds) return launch_plan_t<true, true>(P, lds, s);
  if (P.agents_lds) return launch_plan_t<true, false>(P, lds, s);
  if (P.occ_lds) return launch_plan_t<false, true>(P, lds, s);
  return launch_plan_t<false, false>(P, lds, s);
}

}  // namespace tsw
