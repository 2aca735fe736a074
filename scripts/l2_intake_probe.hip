// l2_intake_probe.hip -- diagnostic (not product code): how many bytes per second ONE CU takes in
// from L2 when every CU of the chip streams 16-byte-per-lane loads, as a function of the loads each
// wave keeps in flight (D).  The clip-group loop (ggd_mega.hip) streams ~2.3 MB of weights and
// hand-off rows per CU per denoise step and its phases wait on that stream; this
// measures the ceiling it runs against.
//
// One workgroup of 512 threads (8 waves) per CU, as mk_kernel.  Mode "shared": every workgroup
// reads the same 128 KiB (the out-projection weights every workgroup of a clip group reads; L2
// hits after the first touch).  Mode "own": workgroup w reads its own 128 KiB.  Each wave issues D
// independent 1 KiB loads (64 lanes x 16 B), waits for all of them, and repeats.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/l2_intake_probe.hip -o scripts/build/l2probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int NT = 512;
constexpr size_t REGION = 128 * 1024;                  // bytes per workgroup stream
constexpr int REGION_U4 = (int)(REGION / 16);           // 16-byte pieces

template <int D>
__global__ void __launch_bounds__(NT) probe(const uint4* src, int iters, int own, unsigned* sink) {
  const uint4* base = src + (own ? (size_t)blockIdx.x * REGION_U4 : 0);
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  unsigned acc = 0;
  int piece = wave * 64 + lane;  // wave w starts at its own 1 KiB; the 8 waves cover 8 KiB per step
  for (int it = 0; it < iters; ++it) {
    uint4 v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = base[(piece + d * NT) % REGION_U4];
    }
    // every component is consumed: with only .x / .w used the compiler narrows each 16-byte load
    // into two global_load_dword (the round-3 figures of this probe measured THAT, not dwordx4)
#pragma unroll
    for (int d = 0; d < D; ++d) acc ^= (v[d].x ^ v[d].y) ^ (v[d].z ^ v[d].w);
    piece = (piece + D * NT) % REGION_U4;
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;  // keeps the loads alive
}

// the same stream through LDS-DMA (global_load_lds_dwordx4: 16 B per lane straight into LDS, no
// result registers); D loads per wave in flight, then s_waitcnt vmcnt(0)
typedef __attribute__((address_space(3))) void lds_void;
template <int D>
__global__ void __launch_bounds__(NT) probe_lds(const uint4* src, int iters, int own, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) unsigned char buf[8 * 16 * 1024];  // 16 KiB per wave
  const uint4* base = src + (own ? (size_t)blockIdx.x * REGION_U4 : 0);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int piece = wave * 64;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      __builtin_amdgcn_global_load_lds((const void*)(base + ((piece + d * NT) % REGION_U4) + lane),
                                       (lds_void*)(buf + wave * 16384 + (d & 15) * 1024), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    piece = (piece + D * NT) % REGION_U4;
  }
  __syncthreads();
  if (buf[tid] == 0x5a) sink[blockIdx.x] = buf[tid + 1];
}

template <int D>
static void run_lds(const uint4* src, unsigned* sink, int nwg) {
  const int iters = (int)((16u << 20) / ((size_t)NT * 16 * D));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe_lds<D>, dim3(nwg), dim3(NT), 0, 0, src, 8, 1, sink);
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(probe_lds<D>, dim3(nwg), dim3(NT), 0, 0, src, iters, 1, sink);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)nwg * NT * 16.0 * D * iters;
  printf("%3d WG lds-dma D=%2d  loads in flight per CU %3d KiB  per-CU %6.1f GB/s  chip %6.2f TB/s  (%.2f ms)\n",
         nwg, D, 8 * D, bytes / nwg / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e12, ms);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

template <int D>
static void run(const uint4* src, unsigned* sink, int nwg, int own) {
  // ~64 MiB per workgroup in total
  const int iters = (int)((16u << 20) / ((size_t)NT * 16 * D));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe<D>, dim3(nwg), dim3(NT), 0, 0, src, 8, own, sink);  // warm
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(probe<D>, dim3(nwg), dim3(NT), 0, 0, src, iters, own, sink);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)nwg * NT * 16.0 * D * iters;
  printf("%3d WG %-6s D=%2d  loads in flight per CU %3d KiB  per-CU %6.1f GB/s  chip %6.2f TB/s  (%.2f ms)\n",
         nwg, own ? "own" : "shared", D, 8 * D, bytes / nwg / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 1e12, ms);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int nwg = cus;  // one 512-thread workgroup per CU (the occupancy mk_kernel runs at)
  uint4* src = nullptr;
  unsigned* sink = nullptr;
  CHECK(hipMalloc(&src, REGION * nwg));
  CHECK(hipMalloc(&sink, sizeof(unsigned) * nwg));
  CHECK(hipMemset(src, 1, REGION * nwg));
  printf("%d CUs, one workgroup of %d threads each, 1 KiB per wave load instruction\n", cus, NT);
  for (int own = 0; own < 2; ++own) {
    run<1>(src, sink, nwg, own);
    run<2>(src, sink, nwg, own);
    run<4>(src, sink, nwg, own);
    run<8>(src, sink, nwg, own);
    run<12>(src, sink, nwg, own);
    run<16>(src, sink, nwg, own);
  }
  // few CUs streaming (no contention for the XCD's L2 bandwidth): 8 workgroups, one per XCD
  // under the usual round-robin dispatch, and 32 (4 per XCD)
  run<4>(src, sink, 8, 1);
  run<8>(src, sink, 8, 1);
  run<12>(src, sink, 8, 1);
  run<8>(src, sink, 32, 1);
  run<8>(src, sink, 64, 1);
  run<8>(src, sink, 128, 1);
  run_lds<4>(src, sink, nwg);
  run_lds<8>(src, sink, nwg);
  run_lds<16>(src, sink, nwg);
  run_lds<8>(src, sink, 8);
  CHECK(hipFree(src));
  CHECK(hipFree(sink));
  return 0;
}
