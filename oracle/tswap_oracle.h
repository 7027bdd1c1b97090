/*
 * tswap_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference TSWAP planning path
 * (RenKoya1/p2p_distributed_tswap @ 2025-11-21, src/algorithm/tswap.rs:39-394).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline. The product path
 * (p2p_distributed_tswap_amd, libtswap_hip.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned". The reference is Rust and no Rust toolchain
 * exists in this image; the reference's own tests pin no planning result
 * (SURVEY.md §4, §8c). This restatement is cross-checked against a second,
 * independently written pure-Python restatement (oracle/py_restatement.py) on
 * small seeded cases; golden fixtures under tests/golden/ carry the tag
 * "std-heap-model v1" (Rust std BinaryHeap sift semantics restated by hand).
 *
 * Cell ids: the reference numbers free cells row-major (tswap.rs:51-59); ids
 * only key HashMaps and equality tests, so this restatement uses the dense
 * cell index c = y*W + x instead — an order-preserving relabelling that does
 * not change any result.
 */
#ifndef TSWAP_ORACLE_H
#define TSWAP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_graph orc_graph;

/* Build the node graph from raw grid bytes (H rows of W bytes, '@' blocked),
 * tswap.rs:44-77. Returns NULL on bad arguments. */
orc_graph *orc_graph_create(const uint8_t *cells, uint32_t w, uint32_t h);
void orc_graph_destroy(orc_graph *gr);

/* get_path (tswap.rs:288-390): writes path[1] to *next (start if len==1) and
 * returns len(path) (1 if start==goal; 2 for the unreachable fallback;
 * D+1 for an A* path of D moves). pops_out (optional) = heap pops done. */
int32_t orc_get_path_next(orc_graph *gr, uint32_t start, uint32_t goal,
                          uint32_t *next, uint64_t *pops_out);

/* BFS distances from goal over the same graph; 0xFFFF = blocked/unreachable.
 * (Not in the reference — the reference never builds tables; this is the
 * oracle for the K1 kernel: d_g(v) == len(get_path(v,g)) - 1.) */
int orc_bfs_u16(orc_graph *gr, uint32_t goal, uint16_t *out);

/* get_path(c, goal)[1] for every cell as a direction code (0..3 S,E,N,W, 4 = stay,
 * 0xFF blocked) — checker for the device next-hop tables. */
int orc_next_codes(orc_graph *gr, uint32_t goal, uint8_t *out);

/* One tswap_step (tswap.rs:174-286) over agents with cell ids v[i], g[i]
 * (in/out). Order = array order, exactly as the reference. */
int orc_tswap_step(orc_graph *gr, uint32_t *v, uint32_t *g, uint32_t n);

/* tswap_mapd (tswap.rs:39-172). starts: n (x,y) pairs; tasks: m rows of
 * (pickup_x, pickup_y, delivery_x, delivery_y). rec_out: caller buffer of
 * n*(max_t+1) records, agent-major: rec[i*(max_t+1)+t] = x | y<<16 | state<<32
 * (AgentState: PICKING=0 CARRYING=1 DELIVERED=2 IDLE=3, map/agent.rs:9-15).
 * goal_out (optional, same shape, u32 cell id of g after the step) is a debug
 * trace for localising divergences. The reference's step cap is
 * `timestep > 2000` (tswap.rs:167); max_t generalises the 2000.
 * Returns number of recorded timesteps T, or <0 on invalid input where the
 * reference panics: an off-grid/blocked start (tswap.rs:94, checked up front), a
 * task whose off-grid/blocked pickup is assigned (:136) or whose off-grid/blocked
 * delivery is looked up on reaching the pickup (:112). A bad task cell that is
 * never looked up does not fail the call, as in the reference. */
int32_t orc_tswap_mapd(orc_graph *gr, const uint32_t *starts_xy, uint32_t n,
                       const uint32_t *tasks_xyxy, uint32_t m, uint32_t max_t,
                       uint64_t *rec_out, uint32_t *goal_out);

/* Decentralized per-agent decision, compute_next_move_with_tswap
 * (src/bin/decentralized/agent.rs:329-462). nb_v/nb_g: the nearby agents' current/goal cells
 * in the caller's list order (self excluded, agent.rs:134). Outputs: act (ORC_ACT_*), cell
 * (Move destination), partner (list index, GOAL_SWAP), npart + part[0..npart) (list indices
 * of the rotation participants, ROTATION; part must hold nn + 1 entries).
 * Returns -1 if my_v or my_g is not a free cell (the reference panics, agent.rs:358). */
#define ORC_ACT_MOVE 0u
#define ORC_ACT_GOAL_SWAP 1u
#define ORC_ACT_ROTATION 2u
#define ORC_ACT_WAIT 3u
int orc_decide(orc_graph *gr, uint32_t my_v, uint32_t my_g, const uint32_t *nb_v, const uint32_t *nb_g,
               uint32_t nn, uint32_t *act, uint32_t *cell, uint32_t *partner, uint32_t *npart, uint32_t *part);

/* Counter of get_path calls / heap pops since the graph was created. */
uint64_t orc_stat_calls(orc_graph *gr);
uint64_t orc_stat_pops(orc_graph *gr);

#ifdef __cplusplus
}
#endif
#endif
