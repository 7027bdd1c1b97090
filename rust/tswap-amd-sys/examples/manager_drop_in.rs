//! The centralized manager's planning tick on the MI355X planner — what replaces
//! `plan_all_paths` (src/bin/centralized/manager.rs:101-144) and its private `tswap_step` copy
//! (:147-259). Self-contained: the manager's per-agent record is mirrored by `ManagedAgent`
//! (the fields `plan_all_paths` reads and writes); in the reference binary the same body works on
//! its `AgentState` values and `pos2id` map.
//!
//! Differences from the reference body, none of which changes a result:
//! * the graph build (`pos2id`, `nodes`, :503-535) is the planner's own (`Planner::new` once, kept
//!   for the manager's lifetime so goal tables and resolved next hops persist across ticks);
//! * node ids become cell ids (y * w + x); `pos2id.get(..).unwrap_or(0)` (:119) maps an unknown
//!   position to node 0, the first free cell in row-major order — `first_free` below.

use tswap_amd_sys::{Planner, Point};

/// The fields of the manager's per-agent state that `plan_all_paths` touches.
#[derive(Clone, Debug)]
pub struct ManagedAgent {
    pub peer_id: String,
    pub current_pos: Point,
    pub goal_pos: Option<Point>,
}

/// `MoveInstruction { peer_id, next_pos, timestamp }` (manager.rs:136-140).
#[derive(Clone, Debug)]
pub struct MoveInstruction {
    pub peer_id: String,
    pub next_pos: Point,
    pub timestamp: u64,
}

fn is_free(grid: &[Vec<char>], p: Point) -> bool {
    p.1 < grid.len() && p.0 < grid[p.1].len() && grid[p.1][p.0] != '@'
}

/// Row-major first free cell: node 0 of the reference's graph build (tswap.rs:51-59).
fn first_free(grid: &[Vec<char>]) -> Point {
    for (y, row) in grid.iter().enumerate() {
        for (x, &c) in row.iter().enumerate() {
            if c != '@' {
                return (x, y);
            }
        }
    }
    (0, 0)
}

/// Drop-in body of `plan_all_paths`: agents in the caller's order (the reference takes them from a
/// HashMap, so parity is per call for a given slice), one `tswap_step`, positions written back
/// (goal swaps are not written back, as in the reference :132-141).
pub fn plan_all_paths(planner: &mut Planner, grid: &[Vec<char>], agents: &mut [ManagedAgent])
                      -> Result<Vec<MoveInstruction>, tswap_amd_sys::TswapError> {
    let timestamp = std::time::SystemTime::now()
        .duration_since(std::time::UNIX_EPOCH)
        .unwrap()
        .as_secs();
    let node0 = first_free(grid);
    let mut v: Vec<u32> = Vec::with_capacity(agents.len());
    let mut g: Vec<u32> = Vec::with_capacity(agents.len());
    for a in agents.iter() {
        let cur = if is_free(grid, a.current_pos) { a.current_pos } else { node0 };  // :119
        let goal = a.goal_pos.filter(|&p| is_free(grid, p)).unwrap_or(cur);           // :120-123
        v.push(planner.cell(cur));
        g.push(planner.cell(goal));
    }
    planner.step(&mut v, &mut g)?;  // :129
    Ok(agents
        .iter_mut()
        .zip(v.iter())
        .map(|(a, &cell)| {
            let next_pos = planner.point(cell);  // :133-134
            a.current_pos = next_pos;
            MoveInstruction { peer_id: a.peer_id.clone(), next_pos, timestamp }
        })
        .collect())
}

fn main() -> Result<(), Box<dyn std::error::Error>> {
    // the bundled 100x100 open map (src/map/map.rs:5-106) and three agents
    let grid: Vec<Vec<char>> = vec![vec!['.'; 100]; 100];
    let mut planner = Planner::new(&grid)?;
    let mut agents = vec![
        ManagedAgent { peer_id: "a".into(), current_pos: (0, 0), goal_pos: Some((5, 3)) },
        ManagedAgent { peer_id: "b".into(), current_pos: (5, 3), goal_pos: Some((0, 0)) },
        ManagedAgent { peer_id: "c".into(), current_pos: (9, 9), goal_pos: None },
    ];
    for tick in 0..8 {
        let moves = plan_all_paths(&mut planner, &grid, &mut agents)?;
        println!("tick {tick}: {:?}", moves.iter().map(|m| (m.peer_id.as_str(), m.next_pos)).collect::<Vec<_>>());
    }
    Ok(())
}
