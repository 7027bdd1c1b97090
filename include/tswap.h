/*
 * tswap.h — C ABI of the MI355X-native TSWAP planning core (libtswap_hip.so).
 *
 * Drop-in boundary for the reference's src/algorithm path
 * (RenKoya1/p2p_distributed_tswap @ 2025-11-21). Plain pointers and sizes,
 * no torch types. Every call is synchronous for the caller (like the
 * reference); device work runs on the context's own HIP stream.
 *
 * Coordinates: Point = (x, y) with x = column, y = row, grid[y][x]
 * (src/map/map.rs:4, tswap.rs:53). Cell id = y*w + x. A cell is blocked iff
 * its byte is '@' (tswap.rs:53); every other byte is passable.
 *
 * Errors: 0 on success, negative errno-style code otherwise; the reference
 * panics where these return TSW_EINVAL (tswap.rs:94,112,136).
 * tsw_last_error(ctx) gives the message of the last failure. A failed call
 * leaves the context consistent: no goal stays registered against a partial
 * table and no next hop stays queued for a K3 pass that did not run.
 * One context is single-threaded; separate contexts may live on separate
 * threads or devices.
 *
 * Hard limits where the reference (usize arithmetic, unbounded Vec/HashMap)
 * would keep going — each returns an error code, never a wrong answer:
 *   - grid: at most 2048 cells per side and 2^20 cells      (tsw_create -> NULL)
 *   - BFS distances are u16: a goal whose farthest reachable cell is more than
 *     65534 steps away (only possible on grids of more than 65535 free cells,
 *     e.g. a serpentine maze) has no distance table. Planning entry points
 *     (tsw_plan_mapd, tsw_step, tsw_decide, tsw_next_hop_tables) keep such a goal
 *     WITHOUT a table and resolve every next hop toward it with the exact A*
 *     (K3, 20-bit g): same results, slower. The table-returning entry points
 *     (tsw_dist_tables*, tsw_next_hop_tables_device) return TSW_EOVERFLOW for it.
 *   - exact A*: the LDS-heap kernels hand queries with g >= 2^15, f >= 2^17 or
 *     a heap past their LDS capacity to the global-heap kernel (20-bit g, enough
 *     for any path on a 2^20-cell grid); its heap holds min(4*cells+8, 65536)
 *     entries, past that TSW_EOVERFLOW
 *   - tsw_decide: at most 1024 entries in one agent's nearby list (TSW_EOVERFLOW;
 *     get_nearby, decentralized/agent.rs:108-153, has no bound)
 *   - goal tables: table_budget_bytes (2 B per cell per goal). Tables not used by
 *     the current call are evicted least-recently-used first; TSW_ENOMEM only
 *     when the goals of ONE call do not fit.
 *
 * Device-memory arguments (*_device entry points) may be produced on any stream
 * of the caller: the library synchronises the device before reading or writing
 * them, and the call has completed its device work when it returns.
 */
#ifndef TSWAP_H
#define TSWAP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSW_OK 0
#define TSW_EINVAL (-22)
#define TSW_ENOMEM (-12)
#define TSW_EHIP (-5)
#define TSW_EOVERFLOW (-75)
#define TSW_ENODEV (-19)

/* Revision of this ABI: bumped whenever a struct or a signature changes, so a caller
 * built against an older header can refuse to run. 3: tsw_opts grew to 24 bytes (watchdog_ms),
 * tsw_next_hop_tables_device gained dev_dist; 4: tsw_abi_version, lazy task-cell checks,
 * tsw_plan_mapd_resolved / tsw_next_hop_codes; 5: tsw_build_id, entry points refuse re-entry from a
 * tsw_plan_mapd_resolved resolver (TSW_EINVAL). */
#define TSW_ABI_VERSION 6

/* AgentState discriminants in declaration order (src/map/agent.rs:9-15) */
#define TSW_PICKING 0
#define TSW_CARRYING 1
#define TSW_DELIVERED 2
#define TSW_IDLE 3

/* Sentinel distance in tables: blocked or unreachable cell. */
#define TSW_DIST_INF 0xFFFFu

typedef struct tsw_ctx tsw_ctx;

/* src/map/map.rs:4 `pub type Point = (usize, usize)` */
typedef struct {
    uint32_t x, y;
} tsw_point;

/* src/map/task_generator.rs:6-12 `Task{pickup, delivery, peer_id, task_id}`;
 * peer_id/task_id are never read by the planner and are not carried. */
typedef struct {
    tsw_point pickup, delivery;
} tsw_task;

/* One element of tswap_mapd's Vec<Vec<(Point, AgentState)>> (tswap.rs:43). */
typedef struct {
    uint16_t x, y;
    uint8_t state; /* TSW_PICKING .. TSW_IDLE */
    uint8_t pad[3];
} tsw_rec;

/* Context options. Every option is results-neutral: plans, tables and next hops are bit-identical
 * whatever is set here; only time and memory change. The production library reads nothing from the
 * environment — these fields are its whole configuration surface. */
typedef struct {
    int32_t device;              /* HIP device ordinal (default 0)                                  */
    uint32_t flags;              /* TSW_F_* below                                                   */
    uint64_t table_budget_bytes; /* cap for detour-byte+next-hop tables, 2 B per cell per goal
                                    (0 = half of the device's free memory at tsw_create)            */
    uint32_t watchdog_ms;        /* plan calls: if the planner records no timestep for this long,
                                    the call finishes in exit mode (0 = 10000)                      */
    uint32_t reserved;
} tsw_opts;

/* Resolve every multi-candidate next hop of every table eagerly (one big
 * batched A* pass right after the BFS tables) instead of lazily per step.
 * (default: eager when the grid has <= 4096 cells and the new tables hold <= 8M cells) */
#define TSW_F_EAGER_NEXTHOP 1u
/* Never eager (lazy only), even when the auto policy would pick eager. */
#define TSW_F_LAZY_NEXTHOP 2u
/* Lazy next hops without concurrent K3 workers: the plan kernel exits to the host whenever a step
 * needs unresolved next hops and is relaunched after a batched A* pass ("exit mode"). Default
 * (coop mode): the plan dispatch also runs exact-A* worker waves on the other CUs, which the planner
 * feeds through device queues and waits on only when a step needs a code. */
#define TSW_F_EXIT_MODE 4u

/* Replaces the graph build of tswap_mapd (tswap.rs:44-77) and of the
 * centralized manager (bin/centralized/manager.rs:503-535): uploads the grid
 * and builds the device neighbour masks. cells: h rows of w bytes.
 * opts may be NULL. Returns NULL on failure (see tsw_last_error(NULL)). */
tsw_ctx *tsw_create(const uint8_t *cells, uint32_t w, uint32_t h, const tsw_opts *opts);
void tsw_destroy(tsw_ctx *ctx);
/* Message of the last failure on ctx (ctx may be NULL: last create failure). */
const char *tsw_last_error(const tsw_ctx *ctx);
/* TSW_ABI_VERSION the library was built with; compare it with the header's before tsw_create. */
int tsw_abi_version(void);
/* Provenance of the build: the first 8 bytes of the sha1 of the library's sources (kernels, host
 * runtime, this header) as computed by the build, 0 if the build did not set it. Measurement tools
 * record it beside a profile and refuse to pair a profile with a different build. */
uint64_t tsw_build_id(void);

/* Replaces `tswap_mapd(grid, initial_positions, tasks)` (tswap.rs:39-172).
 * out: caller-allocated n*(max_t+1) records, agent-major:
 *   out[i*(max_t+1) + t] == paths[i][t]  for t < *out_T.
 * max_t = 2000 reproduces the reference's `timestep > 2000` stop (:167).
 * Returns TSW_EINVAL where the reference panics: a start off-grid or blocked
 * (checked up front, :94), a task whose off-grid/blocked pickup gets assigned
 * (:136), or whose off-grid/blocked delivery is looked up when its agent reaches
 * the pickup (:112). A bad task cell that is never looked up does not fail the
 * call. The nearest-pickup choice uses the raw pickup point (:125-130), its
 * coordinates clamped to 0xFFFE (cannot change the winner: see tsw_capi.hip). */
int tsw_plan_mapd(tsw_ctx *ctx, const tsw_point *starts, uint32_t n, const tsw_task *tasks,
                  uint32_t m, uint32_t max_t, tsw_rec *out, uint32_t *out_T);

/* As tsw_plan_mapd, additionally writing the goal cell id of every agent after
 * each step (same layout as out) — a debug trace for parity localisation.
 * goal_out may be NULL. */
int tsw_plan_mapd_trace(tsw_ctx *ctx, const tsw_point *starts, uint32_t n, const tsw_task *tasks,
                        uint32_t m, uint32_t max_t, tsw_rec *out, uint32_t *goal_out,
                        uint32_t *out_T);

/* Caller-resolved K3 (the per-step query batch sharded by goal owner, the
 * answers gathered). tsw_plan_mapd_resolved plans like tsw_plan_mapd_trace, in exit mode (no K3
 * workers in the plan dispatch), and hands every batch of (start, goal) cell pairs a step needs
 * — plus the speculative pairs queued with it — to `resolve` instead of running the exact A*
 * itself. resolve must fill code[i] with the next-hop code of get_path(start[i], goal[i]) (0..3
 * = S,E,N,W neighbour, tswap.rs:62 order; 4 = stay), e.g. by sending each pair to the rank that
 * owns its goal (tsw_next_hop_codes there) and gathering the codes, and return 0; anything else,
 * or a code > 4, fails the call with TSW_EINVAL. The plan is bit-identical to tsw_plan_mapd's.
 * The resolver must not call back into `ctx` (the suspended plan owns its queues and table store):
 * every entry point returns TSW_EINVAL on a context whose resolver is running. Answer the pairs
 * from another context (e.g. the goal owner's, tsw_next_hop_codes there). */
typedef int (*tsw_resolve_fn)(void *user, uint32_t k, const uint32_t *start, const uint32_t *goal, uint8_t *code);
int tsw_plan_mapd_resolved(tsw_ctx *ctx, const tsw_point *starts, uint32_t n, const tsw_task *tasks,
                           uint32_t m, uint32_t max_t, tsw_rec *out, uint32_t *goal_out, uint32_t *out_T,
                           tsw_resolve_fn resolve, void *user);

/* Next-hop codes of get_path(start[i], goal[i]) (tswap.rs:288-390) as tsw_plan_mapd_resolved's
 * resolver returns them (0..3 S,E,N,W, 4 = stay), served from this context's table store: new
 * goals get their K1 table, unresolved cells the exact A*, and both persist for later calls (a
 * goal owner's shard of the next-hop cache). */
int tsw_next_hop_codes(tsw_ctx *ctx, const uint32_t *start, const uint32_t *goal, uint32_t k, uint8_t *code);

/* Replaces one `tswap_step(&mut agents, &nodes)` call (tswap.rs:174-286;
 * per-tick copy in bin/centralized/manager.rs:147-259 via plan_all_paths
 * :101-144). v[i], g[i]: cell ids in/out, agent order = array order. */
int tsw_step(tsw_ctx *ctx, uint32_t *v, uint32_t *g, uint32_t n);

/* Batched `get_path(start, goal)` (tswap.rs:288-390), reduced to what every
 * caller consumes: next[q] = path[1] (start if len==1) and len[q] = len(path)
 * (1: start==goal, 2: unreachable fallback or adjacent goal, D+1 otherwise). */
int tsw_get_path_next(tsw_ctx *ctx, const uint32_t *start, const uint32_t *goal, uint32_t k,
                      uint32_t *next, int32_t *len);

/* Batched decentralized decision: compute_next_move_with_tswap
 * (src/bin/decentralized/agent.rs:329-462) for n agents, each with its own local view.
 * Agent i: cell my_v[i], goal my_g[i] (free cells, else TSW_EINVAL — the reference panics at
 * pos2id[&my_pos], :358); its nearby list is entries nb_off[i] .. nb_off[i+1]-1 of nb_v/nb_g
 * (the other agents' cell / goal cell ids in NearbyAgents::get_nearby order, self excluded,
 * :108-153; an id >= w*h or a blocked cell means "not on the map", :389-393).
 * Outputs per agent: act[i] = TSW_ACT_* (TswapAction, :321-326); cell[i] = Move destination
 * (the agent's own cell for Rule 1); partner[i] = list index of the goal-swap partner
 * (0xFFFFFFFF otherwise); npart[i] = number of rotation participants, whose list indices are
 * part[nb_off[i] + i .. + npart[i]) (part holds nb_off[n] + n entries). */
#define TSW_ACT_MOVE 0u
#define TSW_ACT_GOAL_SWAP 1u
#define TSW_ACT_ROTATION 2u
#define TSW_ACT_WAIT 3u
int tsw_decide(tsw_ctx *ctx, const uint32_t *my_v, const uint32_t *my_g, uint32_t n, const uint32_t *nb_off,
               const uint32_t *nb_v, const uint32_t *nb_g, uint32_t *act, uint32_t *cell, uint32_t *partner,
               uint32_t *npart, uint32_t *part);

/* K1: BFS distance tables for k goal cells, u16 per cell, row-major
 * (TSW_DIST_INF for blocked/unreachable). out: host buffer k*w*h. */
int tsw_dist_tables(tsw_ctx *ctx, const uint32_t *goals, uint32_t k, uint16_t *out);

/* K1 into caller-owned DEVICE memory (e.g. a torch tensor's data_ptr on the
 * context's device): dev_out receives k*w*h u16. Used for goal-sharded
 * construction + RCCL all-gather. */
int tsw_dist_tables_device(tsw_ctx *ctx, const uint32_t *goals, uint32_t k, uint16_t *dev_out);

/* Ingest k tables (k*w*h u16, DEVICE memory, e.g. the all-gather result)
 * into the context's table store so steps use them without recomputing. */
int tsw_import_tables_device(tsw_ctx *ctx, const uint32_t *goals, uint32_t k,
                             const uint16_t *dev_tables);

/* Next-hop codes of k goal tables (building them if needed), one byte per cell,
 * row-major: 0..3 = path[1] is the S,E,N,W neighbour (tswap.rs:62 order), 4 = stay
 * (unreachable goal, no closer neighbour), 0xFF = not resolved yet (lazy mode:
 * needs the exact A*). out: host buffer k*w*h. A goal held without a distance table
 * (u16 overflow, see the limits above) always comes back all 0xFF here, also with
 * TSW_F_EAGER_NEXTHOP: its next hops are resolved per query (tsw_get_path_next, plans),
 * never as a whole table; tsw_next_hop_tables_device returns TSW_EOVERFLOW for it. */
int tsw_next_hop_tables(tsw_ctx *ctx, const uint32_t *goals, uint32_t k, uint8_t *out);

/* Goal-sharded K3: the fully resolved next-hop codes of k goals into
 * caller-owned DEVICE memory (k*w*h bytes, row-major, codes as tsw_next_hop_tables). Builds the
 * goals' tables if needed and resolves every multi-candidate cell with the exact A* (eager,
 * whatever the context's next-hop policy): one rank's share of an all-gathered code table.
 * dev_dist (may be NULL): also receives the goals' K1 distance tables (k*w*h u16), so one K1 build
 * serves both all-gathers. */
int tsw_next_hop_tables_device(tsw_ctx *ctx, const uint32_t *goals, uint32_t k, uint8_t *dev_out,
                               uint16_t *dev_dist);

/* Ingest k tables AND their next-hop codes (DEVICE memory: k*w*h u16 + k*w*h u8, e.g. the
 * all-gather of tsw_dist_tables_device / tsw_next_hop_tables_device shards): steps then need
 * neither K1 nor K3 for those goals. Code 0xFF (or a pending marker) = not resolved here. */
int tsw_import_next_hops_device(tsw_ctx *ctx, const uint32_t *goals, uint32_t k, const uint16_t *dev_dist,
                                const uint8_t *dev_nh);

/* Drop every goal table and next-hop code held by the context (device memory
 * is kept for reuse). Later calls rebuild what they need. */
int tsw_clear_tables(tsw_ctx *ctx);

/* Per-context counters and kernel timings (HIP events on the context stream). */
typedef struct {
    uint64_t bfs_goals, bfs_launches;
    double bfs_ms;              /* summed K1 kernel time                     */
    uint64_t astar_queries, astar_launches;
    double astar_ms;            /* summed K3 kernel time                     */
    uint64_t walker_launches;   /* K2 serial-commit launches                 */
    double walker_ms;
    uint64_t assign_launches;
    double assign_ms;
    uint64_t steps;             /* timesteps planned                         */
    uint64_t tables;            /* goal tables resident                      */
    double plan_ms;             /* wall time of the last plan call           */
    /* inside the persistent plan kernel: device wall time per section, ms:
     * [0] assign [1] next-hop refresh [2] rules [3] refresh [4] movement
     * [5] record [6] done/other [7] launch copy-in/out */
    double plan_section_ms[8];
    uint64_t rule_rounds;       /* first-firing rounds run by the rules phase */
    /* plan-kernel exits for K3 next-hop resolution, by the section that needed the codes
     * (same indices as plan_section_ms; [7] = relaunch entry) */
    uint64_t plan_exits[8];
    uint64_t table_evictions;   /* goal tables dropped by the LRU (table_budget_bytes reached) */
    /* coop mode (K3 workers running concurrently with the planner): times the planner waited for
     * a worker, and its total waiting time (inside walker_ms) */
    uint64_t coop_waits;
    double coop_wait_ms;
    double coop_wait_sec_ms[8]; /* ... by planner section (plan_section_ms indices) */
    uint64_t coop_waits_sec[8];
    /* rules-phase cycle relabels: block-wide pointer doubling / incremental walks */
    uint64_t relabels_full, relabels_inc;
    uint64_t move_rounds;       /* decidability rounds run by the movement phase */
    uint32_t plan_block;        /* workgroup size of the last plan kernel launch */
    uint32_t coop_workers;      /* K3 worker waves in the last coop plan dispatch */
    /* coop mode: wall time the workers spent inside A*, summed over worker waves (wave-ms), by queue:
     * [0] needed pairs, [1] speculative prefetches, [2] task chains */
    double coop_worker_busy_ms[3];
    uint64_t watchdog_fires;    /* plan calls the host watchdog moved to exit mode */
    uint64_t tableless_goals;   /* goals held without a distance table (u16 overflow; next hops by K3) */
    /* coop mode (ABI 6): A* queries the workers ran and the heap pops they took, by queue (as
     * coop_worker_busy_ms): busy / pops = the in-dispatch time per pop */
    uint64_t coop_worker_queries[3];
    uint64_t coop_worker_pops[3];
} tsw_stats;
int tsw_get_stats(const tsw_ctx *ctx, tsw_stats *out);
int tsw_reset_stats(tsw_ctx *ctx);
/* Enable/disable HIP-event timing around kernels (default on). */
int tsw_set_timing(tsw_ctx *ctx, int enabled);
/* Measurement probe (not part of the reference interface): latency floors of the plan kernel's
 * round shapes on a `block`-thread workgroup (0 = the last plan's), HIP-event timed on the context
 * stream. out[0] = us per wave-0 rules firing chain (LDS load of 64 candidates, ballot, first lane,
 * readlane, that lane's store), out[1] = us per block-wide pass (LDS exchange + barrier; a movement
 * round is three). bench.py reports k_plan against rule_rounds * out[0] + 3 * move_rounds * out[1]. */
int tsw_probe_round_floors(tsw_ctx *ctx, uint32_t block, double *out);

#ifdef __cplusplus
}
#endif
#endif
