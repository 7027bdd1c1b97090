//! `tswap-amd-sys` — the reference's Rust side of the drop-in boundary.
//!
//! Raw declarations mirror `include/tswap.h` one to one (every entry point, struct and constant;
//! `tests/test_host.py::test_rust_crate_mirrors_header` checks it), plus a safe owner `Planner`
//! whose methods take and return the reference's own shapes:
//!
//! * `tswap_mapd` (free function) — the reference's exact signature and return type
//!   (src/algorithm/tswap.rs:39-43) over the caller's own `Task` / `AgentState` through the
//!   `TaskLike` / `FromAgentState` traits; panics where the reference panics.
//! * `Planner::tswap_mapd`  — the same plan on a long-lived context, returning `Err` where the
//!   reference panics (tswap.rs:94,112,136).
//! * `Planner::step`        — the private `tswap_step(&mut agents, &nodes)` copy the centralized
//!   manager calls from `plan_all_paths` (src/bin/centralized/manager.rs:101-144, :147-259).
//! * `Planner::get_path_next` — `get_path(start, goal, nodes)` reduced to what its callers read:
//!   `path[1]` and `path.len()` (tswap.rs:288-390).
//! * `Planner::decide`      — `compute_next_move_with_tswap` (src/bin/decentralized/agent.rs:329-462),
//!   batched over many agents.
//!
//! One `Planner` owns one device context; keep it alive across ticks so goal tables and resolved
//! next hops persist (a per-tick manager streams goals through an LRU bounded by
//! `table_budget_bytes`).

use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};

// ---------------------------------------------------------------------------------------------
// raw C ABI (include/tswap.h)
// ---------------------------------------------------------------------------------------------
pub const TSW_OK: c_int = 0;
pub const TSW_EINVAL: c_int = -22;
pub const TSW_ENOMEM: c_int = -12;
pub const TSW_EHIP: c_int = -5;
pub const TSW_EOVERFLOW: c_int = -75;
pub const TSW_ENODEV: c_int = -19;

/// ABI revision of include/tswap.h this crate mirrors; `Planner::new` refuses a library built
/// against another one.
pub const TSW_ABI_VERSION: c_int = 6;

pub const TSW_PICKING: u8 = 0;
pub const TSW_CARRYING: u8 = 1;
pub const TSW_DELIVERED: u8 = 2;
pub const TSW_IDLE: u8 = 3;

pub const TSW_DIST_INF: u16 = 0xFFFF;

pub const TSW_F_EAGER_NEXTHOP: u32 = 1;
pub const TSW_F_LAZY_NEXTHOP: u32 = 2;
pub const TSW_F_EXIT_MODE: u32 = 4;

pub const TSW_ACT_MOVE: u32 = 0;
pub const TSW_ACT_GOAL_SWAP: u32 = 1;
pub const TSW_ACT_ROTATION: u32 = 2;
pub const TSW_ACT_WAIT: u32 = 3;

/// `tsw_resolve_fn`: the caller's K3 for `tsw_plan_mapd_resolved` — fill `code[i]` (0..3 S,E,N,W,
/// 4 stay) for get_path(start[i], goal[i]) and return 0 (e.g. send each pair to its goal's owner).
pub type TswResolveFn =
    Option<unsafe extern "C" fn(user: *mut c_void, k: u32, start: *const u32, goal: *const u32, code: *mut u8) -> c_int>;

#[repr(C)]
pub struct TswCtx {
    _opaque: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct TswPoint {
    pub x: u32,
    pub y: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct TswTask {
    pub pickup: TswPoint,
    pub delivery: TswPoint,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct TswRec {
    pub x: u16,
    pub y: u16,
    pub state: u8,
    pub pad: [u8; 3],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct TswOpts {
    pub device: i32,
    pub flags: u32,
    pub table_budget_bytes: u64,
    pub watchdog_ms: u32,
    pub reserved: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct TswStats {
    pub bfs_goals: u64,
    pub bfs_launches: u64,
    pub bfs_ms: f64,
    pub astar_queries: u64,
    pub astar_launches: u64,
    pub astar_ms: f64,
    pub walker_launches: u64,
    pub walker_ms: f64,
    pub assign_launches: u64,
    pub assign_ms: f64,
    pub steps: u64,
    pub tables: u64,
    pub plan_ms: f64,
    pub plan_section_ms: [f64; 8],
    pub rule_rounds: u64,
    pub plan_exits: [u64; 8],
    pub table_evictions: u64,
    pub coop_waits: u64,
    pub coop_wait_ms: f64,
    pub coop_wait_sec_ms: [f64; 8],
    pub coop_waits_sec: [u64; 8],
    pub relabels_full: u64,
    pub relabels_inc: u64,
    pub move_rounds: u64,
    pub plan_block: u32,
    pub coop_workers: u32,
    pub coop_worker_busy_ms: [f64; 3],
    pub watchdog_fires: u64,
    pub tableless_goals: u64,
    pub coop_worker_queries: [u64; 3],
    pub coop_worker_pops: [u64; 3],
}

extern "C" {
    pub fn tsw_create(cells: *const u8, w: u32, h: u32, opts: *const TswOpts) -> *mut TswCtx;
    pub fn tsw_destroy(ctx: *mut TswCtx);
    pub fn tsw_last_error(ctx: *const TswCtx) -> *const c_char;
    pub fn tsw_plan_mapd_resolved(ctx: *mut TswCtx, starts: *const TswPoint, n: u32, tasks: *const TswTask, m: u32,
                                  max_t: u32, out: *mut TswRec, goal_out: *mut u32, out_t: *mut u32,
                                  resolve: TswResolveFn, user: *mut c_void) -> c_int;
    pub fn tsw_next_hop_codes(ctx: *mut TswCtx, start: *const u32, goal: *const u32, k: u32, code: *mut u8) -> c_int;
    pub fn tsw_abi_version() -> c_int;
    pub fn tsw_build_id() -> u64;
    pub fn tsw_plan_mapd(ctx: *mut TswCtx, starts: *const TswPoint, n: u32, tasks: *const TswTask, m: u32,
                         max_t: u32, out: *mut TswRec, out_t: *mut u32) -> c_int;
    pub fn tsw_plan_mapd_trace(ctx: *mut TswCtx, starts: *const TswPoint, n: u32, tasks: *const TswTask, m: u32,
                               max_t: u32, out: *mut TswRec, goal_out: *mut u32, out_t: *mut u32) -> c_int;
    pub fn tsw_step(ctx: *mut TswCtx, v: *mut u32, g: *mut u32, n: u32) -> c_int;
    pub fn tsw_get_path_next(ctx: *mut TswCtx, start: *const u32, goal: *const u32, k: u32, next: *mut u32,
                             len: *mut i32) -> c_int;
    pub fn tsw_decide(ctx: *mut TswCtx, my_v: *const u32, my_g: *const u32, n: u32, nb_off: *const u32,
                      nb_v: *const u32, nb_g: *const u32, act: *mut u32, cell: *mut u32, partner: *mut u32,
                      npart: *mut u32, part: *mut u32) -> c_int;
    pub fn tsw_dist_tables(ctx: *mut TswCtx, goals: *const u32, k: u32, out: *mut u16) -> c_int;
    pub fn tsw_dist_tables_device(ctx: *mut TswCtx, goals: *const u32, k: u32, dev_out: *mut u16) -> c_int;
    pub fn tsw_import_tables_device(ctx: *mut TswCtx, goals: *const u32, k: u32, dev_tables: *const u16) -> c_int;
    pub fn tsw_next_hop_tables(ctx: *mut TswCtx, goals: *const u32, k: u32, out: *mut u8) -> c_int;
    pub fn tsw_next_hop_tables_device(ctx: *mut TswCtx, goals: *const u32, k: u32, dev_out: *mut u8,
                                      dev_dist: *mut u16) -> c_int;
    pub fn tsw_import_next_hops_device(ctx: *mut TswCtx, goals: *const u32, k: u32, dev_dist: *const u16,
                                       dev_nh: *const u8) -> c_int;
    pub fn tsw_clear_tables(ctx: *mut TswCtx) -> c_int;
    pub fn tsw_get_stats(ctx: *const TswCtx, out: *mut TswStats) -> c_int;
    pub fn tsw_reset_stats(ctx: *mut TswCtx) -> c_int;
    pub fn tsw_set_timing(ctx: *mut TswCtx, enabled: c_int) -> c_int;
    pub fn tsw_probe_round_floors(ctx: *mut TswCtx, block: u32, out: *mut f64) -> c_int;
}

// ---------------------------------------------------------------------------------------------
// safe layer in the reference's shapes
// ---------------------------------------------------------------------------------------------

/// `pub type Point = (usize, usize)` (src/map/map.rs:4): x = column, y = row, `grid[y][x]`.
pub type Point = (usize, usize);

/// `AgentState` (src/map/agent.rs:9-15), same declaration order and discriminants.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum AgentState {
    PICKING = 0,
    CARRYING = 1,
    DELIVERED = 2,
    IDLE = 3,
}

impl AgentState {
    fn from_u8(s: u8) -> AgentState {
        match s {
            TSW_PICKING => AgentState::PICKING,
            TSW_CARRYING => AgentState::CARRYING,
            TSW_DELIVERED => AgentState::DELIVERED,
            _ => AgentState::IDLE,
        }
    }
}

/// What the planner reads of the reference's `Task` (src/map/task_generator.rs:6-12): its two
/// points (peer_id / task_id are never read, tswap.rs:106-139). The caller's crate adds
/// `impl TaskLike for map::task_generator::Task` (two one-line methods) and passes `&[Task]`
/// unchanged.
pub trait TaskLike {
    fn pickup(&self) -> Point;
    fn delivery(&self) -> Point;
}

impl TaskLike for (Point, Point) {
    fn pickup(&self) -> Point {
        self.0
    }
    fn delivery(&self) -> Point {
        self.1
    }
}

/// Builds the caller's own `AgentState` (src/map/agent.rs:9-15) from this crate's, so the return
/// type is exactly the reference's `Vec<Vec<(Point, AgentState)>>`. The caller's crate adds
/// `impl FromAgentState for map::agent::AgentState` (a four-arm match).
pub trait FromAgentState {
    fn from_agent_state(s: AgentState) -> Self;
}

impl FromAgentState for AgentState {
    fn from_agent_state(s: AgentState) -> Self {
        s
    }
}

/// Drop-in with the reference's exact signature, `pub fn tswap_mapd(grid: &[Vec<char>],
/// initial_positions: Vec<Point>, tasks: &[Task]) -> Vec<Vec<(Point, AgentState)>>`
/// (src/algorithm/tswap.rs:39-43): swap `use crate::algorithm::tswap::tswap_mapd` for
/// `use tswap_amd_sys::tswap_mapd` and the call sites stay as they are. Like the reference it
/// panics where the plan is invalid (an off-grid or blocked start, or a task cell looked up when
/// assigned / reached, tswap.rs:94,112,136) and stops after timestep 2000 (:167). It builds a
/// context per call, as the reference rebuilds its graph per call; keep a `Planner` instead to
/// reuse tables across calls.
pub fn tswap_mapd<T: TaskLike, S: FromAgentState>(grid: &[Vec<char>], initial_positions: Vec<Point>,
                                                  tasks: &[T]) -> Vec<Vec<(Point, S)>> {
    let mut planner = Planner::new(grid).unwrap_or_else(|e| panic!("{}", e));
    planner
        .tswap_mapd_tasks(initial_positions, tasks, 2000)
        .unwrap_or_else(|e| panic!("{}", e))
        .into_iter()
        .map(|path| path.into_iter().map(|(p, s)| (p, S::from_agent_state(s))).collect())
        .collect()
}

/// A failed call: the C error code and `tsw_last_error`'s message.
#[derive(Clone, Debug)]
pub struct TswapError {
    pub code: c_int,
    pub message: String,
}

impl std::fmt::Display for TswapError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "tswap error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for TswapError {}

fn last_error(ctx: *const TswCtx) -> String {
    unsafe {
        let p = tsw_last_error(ctx);
        if p.is_null() {
            String::new()
        } else {
            CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    }
}

/// Options of one context (all results-neutral; see `TswOpts` in include/tswap.h).
#[derive(Clone, Copy, Debug, Default)]
pub struct Options {
    pub device: i32,
    pub flags: u32,
    pub table_budget_bytes: u64,
    pub watchdog_ms: u32,
}

/// One device context bound to a grid (`tswap_mapd`'s graph build, tswap.rs:44-77).
pub struct Planner {
    ctx: *mut TswCtx,
    w: usize,
    h: usize,
}

// A context is single-threaded (like the reference) but may move between threads.
unsafe impl Send for Planner {}

impl Planner {
    /// `grid[y][x]`, '@' blocked (tswap.rs:53); every row must have `grid[0].len()` cells.
    pub fn new(grid: &[Vec<char>]) -> Result<Self, TswapError> {
        Self::with_options(grid, Options::default())
    }

    pub fn with_options(grid: &[Vec<char>], opts: Options) -> Result<Self, TswapError> {
        let h = grid.len();
        let w = if h > 0 { grid[0].len() } else { 0 };
        if grid.iter().any(|r| r.len() != w) {
            return Err(TswapError { code: TSW_EINVAL, message: "ragged grid rows".into() });
        }
        let abi = unsafe { tsw_abi_version() };
        if abi != TSW_ABI_VERSION {
            return Err(TswapError {
                code: TSW_EINVAL,
                message: format!("libtswap_hip ABI {} but this crate mirrors ABI {}", abi, TSW_ABI_VERSION),
            });
        }
        let cells: Vec<u8> = grid.iter().flat_map(|r| r.iter().map(|&c| if c == '@' { b'@' } else { b'.' })).collect();
        let o = TswOpts {
            device: opts.device,
            flags: opts.flags,
            table_budget_bytes: opts.table_budget_bytes,
            watchdog_ms: opts.watchdog_ms,
            reserved: 0,
        };
        let ctx = unsafe { tsw_create(cells.as_ptr(), w as u32, h as u32, &o) };
        if ctx.is_null() {
            return Err(TswapError { code: TSW_EHIP, message: last_error(std::ptr::null()) });
        }
        Ok(Planner { ctx, w, h })
    }

    fn check(&self, rc: c_int) -> Result<(), TswapError> {
        if rc == TSW_OK {
            Ok(())
        } else {
            Err(TswapError { code: rc, message: last_error(self.ctx) })
        }
    }

    /// Cell id of a point (y * w + x), the id space of `step`, `get_path_next` and `decide`.
    pub fn cell(&self, p: Point) -> u32 {
        (p.1 * self.w + p.0) as u32
    }

    pub fn point(&self, cell: u32) -> Point {
        (cell as usize % self.w, cell as usize / self.w)
    }

    pub fn width(&self) -> usize {
        self.w
    }

    pub fn height(&self) -> usize {
        self.h
    }

    /// Drop-in for `tswap_mapd(grid, initial_positions, tasks)` (tswap.rs:39-172): tasks as
    /// (pickup, delivery) pairs (`Task{pickup, delivery, ..}`, src/map/task_generator.rs:6-12;
    /// peer_id / task_id are never read by the planner). `max_t = 2000` is the reference's
    /// `timestep > 2000` stop.
    pub fn tswap_mapd(&mut self, initial_positions: Vec<Point>, tasks: &[(Point, Point)], max_t: u32)
                      -> Result<Vec<Vec<(Point, AgentState)>>, TswapError> {
        self.tswap_mapd_tasks(initial_positions, tasks, max_t)
    }

    /// As `tswap_mapd`, over any task type exposing the reference `Task`'s two points.
    /// Coordinates past u32 saturate (such a point is off-grid either way).
    pub fn tswap_mapd_tasks<T: TaskLike>(&mut self, initial_positions: Vec<Point>, tasks: &[T], max_t: u32)
                                         -> Result<Vec<Vec<(Point, AgentState)>>, TswapError> {
        let c32 = |v: usize| v.min(u32::MAX as usize) as u32;
        let starts: Vec<TswPoint> =
            initial_positions.iter().map(|&(x, y)| TswPoint { x: c32(x), y: c32(y) }).collect();
        let ts: Vec<TswTask> = tasks
            .iter()
            .map(|t| {
                let (p, d) = (t.pickup(), t.delivery());
                TswTask {
                    pickup: TswPoint { x: c32(p.0), y: c32(p.1) },
                    delivery: TswPoint { x: c32(d.0), y: c32(d.1) },
                }
            })
            .collect();
        let n = starts.len();
        let stride = max_t as usize + 1;
        let mut out = vec![TswRec::default(); n.max(1) * stride];
        let mut t = 0u32;
        self.check(unsafe {
            tsw_plan_mapd(self.ctx, starts.as_ptr(), n as u32, ts.as_ptr(), ts.len() as u32, max_t, out.as_mut_ptr(),
                          &mut t)
        })?;
        Ok((0..n)
            .map(|i| {
                (0..t as usize)
                    .map(|k| {
                        let r = out[i * stride + k];
                        ((r.x as usize, r.y as usize), AgentState::from_u8(r.state))
                    })
                    .collect()
            })
            .collect())
    }

    /// One `tswap_step` (tswap.rs:174-286) over cell ids, in place, agent order = slice order.
    pub fn step(&mut self, v: &mut [u32], g: &mut [u32]) -> Result<(), TswapError> {
        if v.len() != g.len() {
            return Err(TswapError { code: TSW_EINVAL, message: "v and g lengths differ".into() });
        }
        self.check(unsafe { tsw_step(self.ctx, v.as_mut_ptr(), g.as_mut_ptr(), v.len() as u32) })
    }

    /// `get_path(start, goal)` for many pairs: (path[1], path.len()) — path[1] is `start` when
    /// len == 1 (start == goal) (tswap.rs:288-390).
    pub fn get_path_next(&mut self, start: &[u32], goal: &[u32]) -> Result<Vec<(u32, i32)>, TswapError> {
        let k = start.len().min(goal.len());
        let (mut next, mut len) = (vec![0u32; k], vec![0i32; k]);
        self.check(unsafe {
            tsw_get_path_next(self.ctx, start.as_ptr(), goal.as_ptr(), k as u32, next.as_mut_ptr(), len.as_mut_ptr())
        })?;
        Ok(next.into_iter().zip(len).collect())
    }

    /// Batched `compute_next_move_with_tswap` (src/bin/decentralized/agent.rs:329-462): per agent
    /// (my cell, my goal cell) and its nearby list of (cell, goal cell) in `get_nearby` order.
    /// Returns (act TSW_ACT_*, cell, partner list index or u32::MAX, rotation participants).
    pub fn decide(&mut self, mine: &[(u32, u32)], nearby: &[Vec<(u32, u32)>])
                  -> Result<Vec<(u32, u32, u32, Vec<u32>)>, TswapError> {
        let n = mine.len();
        if nearby.len() != n {
            return Err(TswapError { code: TSW_EINVAL, message: "one nearby list per agent".into() });
        }
        let mut off = vec![0u32; n + 1];
        for i in 0..n {
            off[i + 1] = off[i] + nearby[i].len() as u32;
        }
        let nv: Vec<u32> = nearby.iter().flatten().map(|a| a.0).collect();
        let ng: Vec<u32> = nearby.iter().flatten().map(|a| a.1).collect();
        let mv: Vec<u32> = mine.iter().map(|a| a.0).collect();
        let mg: Vec<u32> = mine.iter().map(|a| a.1).collect();
        let (mut act, mut cell, mut partner, mut npart) = (vec![0u32; n], vec![0u32; n], vec![0u32; n], vec![0u32; n]);
        let mut part = vec![0u32; off[n] as usize + n];
        self.check(unsafe {
            tsw_decide(self.ctx, mv.as_ptr(), mg.as_ptr(), n as u32, off.as_ptr(), nv.as_ptr(), ng.as_ptr(),
                       act.as_mut_ptr(), cell.as_mut_ptr(), partner.as_mut_ptr(), npart.as_mut_ptr(),
                       part.as_mut_ptr())
        })?;
        Ok((0..n)
            .map(|i| {
                let b = off[i] as usize + i;
                (act[i], cell[i], partner[i], part[b..b + npart[i] as usize].to_vec())
            })
            .collect())
    }

    /// K1 distance tables (u16 per cell, TSW_DIST_INF blocked / unreachable), goal-major.
    pub fn dist_tables(&mut self, goals: &[u32]) -> Result<Vec<u16>, TswapError> {
        let mut out = vec![0u16; goals.len() * self.w * self.h];
        self.check(unsafe { tsw_dist_tables(self.ctx, goals.as_ptr(), goals.len() as u32, out.as_mut_ptr()) })?;
        Ok(out)
    }

    /// Next-hop codes per (goal, cell): 0..3 = S,E,N,W (tswap.rs:62), 4 = stay, 0xFF = unresolved.
    pub fn next_hop_tables(&mut self, goals: &[u32]) -> Result<Vec<u8>, TswapError> {
        let mut out = vec![0u8; goals.len() * self.w * self.h];
        self.check(unsafe { tsw_next_hop_tables(self.ctx, goals.as_ptr(), goals.len() as u32, out.as_mut_ptr()) })?;
        Ok(out)
    }

    /// Goal-sharded construction (one rank's share of an all-gather): K1 tables of `goals` into
    /// DEVICE memory the caller owns (e.g. an RCCL buffer). Unsafe: `dev_out` must hold
    /// goals.len() * w * h u16 on this context's device.
    pub unsafe fn dist_tables_device(&mut self, goals: &[u32], dev_out: *mut u16) -> Result<(), TswapError> {
        self.check(tsw_dist_tables_device(self.ctx, goals.as_ptr(), goals.len() as u32, dev_out))
    }

    /// Ingest gathered tables (DEVICE memory, goals.len() * w * h u16). Unsafe: raw device pointer.
    pub unsafe fn import_tables_device(&mut self, goals: &[u32], dev_tables: *const u16) -> Result<(), TswapError> {
        self.check(tsw_import_tables_device(self.ctx, goals.as_ptr(), goals.len() as u32, dev_tables))
    }

    /// Fully resolved next-hop codes (and, if `dev_dist` is non-null, the K1 tables) of `goals` into
    /// DEVICE memory. Unsafe: raw device pointers sized goals.len() * w * h (u8 / u16).
    pub unsafe fn next_hop_tables_device(&mut self, goals: &[u32], dev_out: *mut u8, dev_dist: *mut u16)
                                         -> Result<(), TswapError> {
        self.check(tsw_next_hop_tables_device(self.ctx, goals.as_ptr(), goals.len() as u32, dev_out, dev_dist))
    }

    /// Ingest gathered tables + next-hop codes (DEVICE memory). Unsafe: raw device pointers.
    pub unsafe fn import_next_hops_device(&mut self, goals: &[u32], dev_dist: *const u16, dev_nh: *const u8)
                                          -> Result<(), TswapError> {
        self.check(tsw_import_next_hops_device(self.ctx, goals.as_ptr(), goals.len() as u32, dev_dist, dev_nh))
    }

    pub fn clear_tables(&mut self) -> Result<(), TswapError> {
        self.check(unsafe { tsw_clear_tables(self.ctx) })
    }

    pub fn stats(&self) -> Result<TswStats, TswapError> {
        let mut s = TswStats::default();
        self.check(unsafe { tsw_get_stats(self.ctx, &mut s) })?;
        Ok(s)
    }

    pub fn reset_stats(&mut self) -> Result<(), TswapError> {
        self.check(unsafe { tsw_reset_stats(self.ctx) })
    }

    pub fn set_timing(&mut self, enabled: bool) -> Result<(), TswapError> {
        self.check(unsafe { tsw_set_timing(self.ctx, if enabled { 1 } else { 0 }) })
    }

    /// Measurement probe: (us per wave-0 rules firing chain, us per block-wide pass).
    pub fn probe_round_floors(&mut self, block: u32) -> Result<(f64, f64), TswapError> {
        let mut out = [0f64; 2];
        self.check(unsafe { tsw_probe_round_floors(self.ctx, block, out.as_mut_ptr()) })?;
        Ok((out[0], out[1]))
    }
}

impl Drop for Planner {
    fn drop(&mut self) {
        unsafe { tsw_destroy(self.ctx) }
    }
}
