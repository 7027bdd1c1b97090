// Write-pattern calibration for WRITE_SIZE (gfx950): the same bytes stored three ways.
//   strided : lane l writes 64 B at 64*l with four 16-B stores (K1's decode pattern)
//   coal    : four 16-B stores, each instruction covering 1 KB contiguous (lane l at 16*l)
//   u16     : lane l writes its 32 cells as 32 separate u16 stores (the W % 8 != 0 path)
// Run: rocprofv3 --pmc WRITE_SIZE -- scripts/bin/calib_write ; each kernel writes 256 MiB once.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_strided(uint4* out, size_t nwords) {  // one 64-B word per lane
  const size_t w = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  uint4* q = out + 4 * w;
  const uint32_t v = (uint32_t)w;
  q[0] = make_uint4(v, v, v, v);
  q[1] = make_uint4(v, v, v, v);
  q[2] = make_uint4(v, v, v, v);
  q[3] = make_uint4(v, v, v, v);
}

__global__ void k_coal(uint4* out, size_t nwords) {
  const size_t w = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  const size_t base = 4 * (w & ~(size_t)63), l = w & 63;
  const uint32_t v = (uint32_t)w;
  out[base + l] = make_uint4(v, v, v, v);
  out[base + 64 + l] = make_uint4(v, v, v, v);
  out[base + 128 + l] = make_uint4(v, v, v, v);
  out[base + 192 + l] = make_uint4(v, v, v, v);
}

__global__ void k_u16(uint16_t* out, size_t nwords) {
  const size_t w = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  uint16_t* d = out + 32 * w;
#pragma unroll
  for (int b = 0; b < 32; ++b) d[b] = (uint16_t)(w + b);
}

int main() {
  const size_t bytes = 256ull << 20, nwords = bytes / 64;
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return 1;
  const dim3 blk(256), grd((unsigned)((nwords + 255) / 256));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int kind = 0; kind < 3; ++kind) {
    hipMemset(p, 0, bytes);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    if (kind == 0) hipLaunchKernelGGL(k_strided, grd, blk, 0, 0, (uint4*)p, nwords);
    if (kind == 1) hipLaunchKernelGGL(k_coal, grd, blk, 0, 0, (uint4*)p, nwords);
    if (kind == 2) hipLaunchKernelGGL(k_u16, grd, blk, 0, 0, (uint16_t*)p, nwords);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%s %.3f ms %.1f GB/s\n", kind == 0 ? "strided" : kind == 1 ? "coal" : "u16", ms, bytes / (ms * 1e6));
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
