// tsw_plan.hip — host side of the persistent plan kernel k_plan (tsw_plan_kernel.h): LDS sizing, the
// occupancy build and the launch, which picks one of the k_plan instantiations compiled in tsw_plan_v*.hip.
#include "tsw_plan_kernel.h"

namespace tsw {

hipError_t launch_plan_v0(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v1(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v2(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v3(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v4(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v5(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);
hipError_t launch_plan_v6(const PlanArgs* P, const WorkerArgs& W, uint32_t grid, size_t lds, uint32_t block,
                          hipStream_t s);

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
__global__ void k_occ_flag(uint32_t* occ, const uint32_t* cnt, uint32_t ncell, uint32_t* dups) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncell && cnt[c] > 1u) {
    occ[c] |= OCC_FLAG;
    *dups = 1u;
  }
}

size_t part_lds_bytes(uint32_t n, uint32_t part) {
  auto r16 = [](size_t b) { return (b + 15u) & ~(size_t)15u; };
  size_t b = 0;
  for (uint32_t bit : {PART_SUCC, PART_V, PART_G, PART_GT})
    if (part & bit) b += r16((size_t)n * 4);
  for (uint32_t bit : {PART_ONC, PART_NHC, PART_CANDC})
    if (part & bit) b += r16(n);
  return b;
}

size_t plan_lds_bytes(uint32_t n, uint32_t ncell, uint32_t m, bool agents, bool occ, bool tasks, bool flinks,
                      bool mu, uint32_t part) {
  auto r16 = [](size_t b) { return (b + 15u) & ~(size_t)15u; };
  size_t b = r16(1024 * 4);
  if (agents) b += 4 * r16((size_t)n * 4) + 3 * r16((size_t)(n + 1) * 4) + 4 * r16(n);
  else {
    b += part_lds_bytes(n, part);
    if (flinks) b += 2 * r16((size_t)(n + 1) * 4);
  }
  if (occ) b += r16((size_t)ncell * 4) + (mu ? r16((size_t)ncell * 4) : 0u);  // MU in LDS: u32 words (MU32)
  if (tasks) b += r16((size_t)((m + 3u) & ~3u) * 4);
  return b;
}

hipError_t launch_occ(const uint32_t* v, uint32_t n, uint32_t* occ, uint32_t* cnt, uint32_t ncell, uint32_t* dups,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_occ_init, dim3((ncell + 255) / 256), dim3(256), 0, s, occ, cnt, ncell);
  if (n) hipLaunchKernelGGL(k_occ_add, dim3((n + 255) / 256), dim3(256), 0, s, v, n, occ, cnt);
  hipLaunchKernelGGL(k_occ_flag, dim3((ncell + 255) / 256), dim3(256), 0, s, occ, cnt, ncell, dups);
  return hipGetLastError();
}

hipError_t launch_plan(const PlanArgs& P, PlanArgs* d_args, const WorkerArgs* W, uint32_t worker_blocks, size_t lds,
                       uint32_t block, hipStream_t s) {
  WorkerArgs none{};
  const WorkerArgs& A = (W && P.coop) ? *W : none;
  const uint32_t grid = 1u + ((W && P.coop) ? worker_blocks : 0u);
  if (grid > 1u && ((size_t)A.wpb * A.lds_per_wave > lds || A.wpb * 64u > block)) return hipErrorInvalidValue;
  const bool mu = P.occ_lds && P.mu_lds;
  // the kernel reads its arguments from d_args (stream order: after the previous dispatch has finished)
  if (hipError_t e = hipMemcpyAsync(d_args, &P, sizeof(PlanArgs), hipMemcpyHostToDevice, s); e != hipSuccess) return e;
  if (P.agents_lds && mu) return launch_plan_v0(d_args, A, grid, lds, block, s);
  if (P.agents_lds && P.occ_lds) return launch_plan_v1(d_args, A, grid, lds, block, s);
  if (P.agents_lds) return launch_plan_v2(d_args, A, grid, lds, block, s);
  if (P.part_lds == PART_PG && !P.occ_lds) return launch_plan_v3(d_args, A, grid, lds, block, s);
  if (mu) return launch_plan_v4(d_args, A, grid, lds, block, s);
  if (P.occ_lds) return launch_plan_v5(d_args, A, grid, lds, block, s);
  return launch_plan_v6(d_args, A, grid, lds, block, s);
}

}  // namespace tsw
