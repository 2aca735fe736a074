// ggd_diag.hip -- calibration micro-kernels behind ggd_diag(what = 5): the cost model the
// fused kernels are designed against (launch floor, dependent-load latency, clock, bulk load).
#include "ggd_common.h"

namespace ggd {

__global__ void mb_empty_kernel(int* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && sink[0] == 12345) sink[1] = 1;
}

// one lane chases `steps` dependent loads through `next` (indices), returns the sum
__global__ void mb_chase_kernel(const int* next, int steps, int* out) {
  if (threadIdx.x != 0) return;
  int p = 0;
  for (int i = 0; i < steps; ++i) p = next[p];
  out[0] = p;
}

// one wave spins a dependent VALU chain; stamps shader cycles and the 100 MHz real-time clock
__global__ void mb_clock_kernel(unsigned long long* out, int iters) {
  if (threadIdx.x >= 64) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float v = (float)threadIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = (unsigned long long)(v > 1e30f);
  }
}

// every block loads `bytes` (multiple of 4096) with 16-byte lane loads, all issued before use
template <int PER>
__global__ void __launch_bounds__(256) mb_bulk_kernel(const uint4* src, size_t blk_stride, uint4* out) {
  const uint4* p = src + blockIdx.x * blk_stride;
  uint4 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = p[threadIdx.x + i * 256];
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < PER; ++i) { acc.x ^= v[i].x; acc.y ^= v[i].y; acc.z ^= v[i].z; acc.w ^= v[i].w; }
  if (acc.x == 0x12345678u) out[blockIdx.x] = acc;
}

hipError_t launch_mb(int mode, void* buf, size_t buf_bytes, int arg, int blocks, hipStream_t s) {
  switch (mode) {
    case 0: hipLaunchKernelGGL(mb_empty_kernel, dim3(blocks), dim3(256), 0, s, (int*)buf); break;
    case 1: hipLaunchKernelGGL(mb_chase_kernel, dim3(1), dim3(64), 0, s, (const int*)buf, arg, (int*)buf + (buf_bytes / 4 - 1)); break;
    case 2: hipLaunchKernelGGL(mb_clock_kernel, dim3(1), dim3(64), 0, s, (unsigned long long*)buf, arg); break;
    case 3: hipLaunchKernelGGL(mb_bulk_kernel<16>, dim3(blocks), dim3(256), 0, s, (const uint4*)buf,
                               (size_t)16 * 256, (uint4*)buf); break;  // 64 KiB per block
    case 4: hipLaunchKernelGGL(mb_bulk_kernel<4>, dim3(blocks), dim3(256), 0, s, (const uint4*)buf,
                               (size_t)4 * 256, (uint4*)buf); break;   // 16 KiB per block
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ggd
