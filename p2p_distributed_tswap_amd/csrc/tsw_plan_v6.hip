// tsw_plan_v6.hip — one instantiation of k_plan (tsw_plan_kernel.h): AG=false, OC=false, MUL=false, PG=false.
#include "tsw_plan_kernel.h"

namespace tsw {
hipError_t launch_plan_v6(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s) {
  return launch_plan_t<false, false, false, false>(P, W, grid, lds, block, s);
}
}  // namespace tsw
