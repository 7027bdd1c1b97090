// tsw_probe.hip — latency floors of the persistent planner's rounds (k_plan), measured on the device.
//
// k_plan (tsw_plan.hip) is bound by dependent round latency, not by bytes: one workgroup runs
// tswap_step's sequential rules scan (tswap.rs:180-252) as first-firing rounds and its movement scan
// (:257-285) as decidability rounds. These kernels time the irreducible skeleton of each round
// shape, so bench.py can report the planner against its own floor (a latency roofline):
//   k_probe_wave_round  the wave-0 rules firing: the next firing reads state that the previous one
//                       wrote — LDS load of 64 candidate flags at the cursor, ballot, first set lane,
//                       readlane of its successor, that lane's LDS store, cursor moves past it.
//   k_probe_block_pass  one block-wide pass of a movement round: every thread loads an LDS word
//                       another thread wrote in the previous pass, stores a word another thread
//                       reads in the next one, barrier (one barrier per pass orders both).
//                       A movement round is three such passes (targets + MU, decide, commit).
// Both run `iters` rounds in one launch on the planner's workgroup size; the host divides the
// HIP-event time of the launch by the round count.
#include <hip/hip_runtime.h>

#include "tsw_internal.h"
#include "tsw_launch.h"

namespace tsw {

__global__ void __launch_bounds__(1024) k_probe_wave_round(uint32_t iters, uint32_t n, uint32_t* sink) {
  extern __shared__ uint32_t sm[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  for (uint32_t i = tid; i < n; i += blockDim.x) sm[i] = ((i * 2654435761u) >> 29) != 0u ? 1u : 0u;
  __syncthreads();
  if (tid >= 64u) return;
  uint32_t cur = 0, acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t k = cur + lane;
    if (k >= n) k -= n;
    const uint32_t f = sm[k];
    const uint64_t m = __ballot(f != 0u);
    const uint32_t l = m ? (uint32_t)__builtin_ctzll(m) : 63u;
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)k, (int)l);
    if (lane == l) sm[b] = f ^ 1u;  // the firing's state change
    acc += b;
    cur = b + 1u >= n ? 0u : b + 1u;  // (one wave's LDS accesses complete in order: no wait needed)
  }
  if (lane == 0) sink[0] = acc;
}

__global__ void __launch_bounds__(1024) k_probe_block_pass(uint32_t iters, uint32_t* sink) {
  extern __shared__ uint32_t sm[];
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  sm[tid] = tid;  // two buffers of bd words: pass `it` reads buffer it & 1 and writes the other
  sm[bd + tid] = tid;
  __syncthreads();
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t* rd = sm + (it & 1u) * bd;
    uint32_t* wr = sm + ((it + 1u) & 1u) * bd;
    const uint32_t v = rd[(tid + 1u + (it & 63u)) % bd];  // written by another thread last pass
    acc += v;
    wr[tid] = v * 2654435761u + it;  // read by another thread next pass
    __syncthreads();
  }
  if (tid == 0) sink[0] = acc;
}

hipError_t probe_round_floors(uint32_t block, uint32_t n, hipStream_t s, double* us_wave_round,
                              double* us_block_pass) {
  if (block < 64u || block > 1024u || block % 64u) return hipErrorInvalidValue;
  n = std::max<uint32_t>(64u, std::min<uint32_t>(n, 16384u));
  uint32_t* sink = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipMalloc(&sink, 16);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  const uint32_t wave_iters = 200000u, pass_iters = 50000u;
  float ms_w = 0.f, ms_b = 0.f;
  for (int rep = 0; rep < 2 && e == hipSuccess; ++rep) {  // first repetition warms up
    if ((e = hipEventRecord(e0, s)) != hipSuccess) break;
    hipLaunchKernelGGL(k_probe_wave_round, dim3(1), dim3(block), n * 4u, s, wave_iters, n, sink);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipEventRecord(e1, s)) != hipSuccess) break;
    if ((e = hipEventSynchronize(e1)) != hipSuccess) break;
    if ((e = hipEventElapsedTime(&ms_w, e0, e1)) != hipSuccess) break;
    if ((e = hipEventRecord(e0, s)) != hipSuccess) break;
    hipLaunchKernelGGL(k_probe_block_pass, dim3(1), dim3(block), block * 8u, s, pass_iters, sink);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipEventRecord(e1, s)) != hipSuccess) break;
    if ((e = hipEventSynchronize(e1)) != hipSuccess) break;
    e = hipEventElapsedTime(&ms_b, e0, e1);
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (sink) (void)hipFree(sink);
  if (e != hipSuccess) return e;
  *us_wave_round = (double)ms_w * 1e3 / wave_iters;
  *us_block_pass = (double)ms_b * 1e3 / pass_iters;
  return hipSuccess;
}

}  // namespace tsw
