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

// Clip-group hand-off cost: groups of 8 workgroups; each round every workgroup writes `kb`
// KiB with sc1 (write-through) 16-byte stores, arrives on its group's counter (agent atomic,
// after every wave's vmcnt(0) + a workgroup barrier), polls it with sc1 loads, then reads the
// next member's slice with sc1 loads -- the protocol a persistent multi-workgroup-per-clip
// kernel would use between decoder phases.  buf layout: [counters 4 KiB][slices].
__global__ void __launch_bounds__(256) mb_groupsync_kernel(unsigned char* buf, int rounds, int kb) {
  unsigned* ctr = (unsigned*)buf;
  const int g = blockIdx.x >> 3, m = blockIdx.x & 7;
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf + 4096, (short)0, 0x7fffffff, 0x00020000);
  const int slice = kb * 1024, per = slice / (256 * 16);
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int r = 0; r < rounds; ++r) {
    for (int i = 0; i < per; ++i) {
      const u32x4 v = {(unsigned)r, (unsigned)i, (unsigned)m, acc.x};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, (threadIdx.x + i * 256) * 16, blockIdx.x * slice, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr + g * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = 8u * (unsigned)(r + 1);
      for (int spin = 0; spin < (1 << 24); ++spin) {
        if (__hip_atomic_load(ctr + g * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    const int src = (g << 3) | ((m + 1) & 7);
    for (int i = 0; i < per; ++i) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + i * 256) * 16, src * slice, 16);
      acc += v;
    }
  }
  if (acc.x == 0x12345678u) ctr[4095 / 4] = acc.y;
}

// Clip-group hand-off inside one launch (the seam a persistent 8-workgroups-per-clip decoder
// would pay instead of a kernel boundary).  Placement: a workgroup reads its XCC id, takes a
// ticket on that XCD's counter and joins group (xcc * 4 + ticket / 8), so the 8 members of a
// group share one L2 (SPREAD: group = blockIdx / 8, members on 8 different XCDs).  Each round
// every member publishes KB KiB (16-byte stores, cache policy AS), drains, arrives on the group
// counter; once all 8 arrived it gathers ALL 8 slices (8 x KB KiB -- whole clip rows, what a
// decoder phase reads) with every load issued before any is used (cache policy AL: 0 plain,
// 1 sc0, 16 sc1, 17 both).  Slices are double-buffered by round parity; every value is checked.
// Control words [0, 4 KiB): XCD tickets (stride 64 B) | group counters (from word 128) |
// stats {errors, misplaced, timeouts} at word 1000.
template <int KB, int AL, int AS, bool SPREAD>
__global__ void __launch_bounds__(512) mb_xcdsync_kernel(unsigned char* buf, int rounds) {
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  constexpr int PER = KB * 1024 / (512 * 16), SLICE = KB * 1024;
  static_assert(PER >= 1, "at least one 16-byte piece per thread and slice");
  unsigned* ctl = (unsigned*)buf;
  __shared__ int role;
  if (threadIdx.x == 0) {
    if (SPREAD) {
      role = blockIdx.x;
    } else {
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      xcc &= 7;
      const unsigned t = __hip_atomic_fetch_add(ctl + xcc * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      role = t < 32 ? (int)(xcc * 32 + t) : -1;
      if (t >= 32) __hip_atomic_fetch_add(ctl + 1001, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  const int me = role;
  if (me < 0) return;
  const int g = me >> 3, m = me & 7;
  unsigned* gctr = ctl + 128 + g * 16;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(buf + 4096, (short)0, 0x7fffffff, 0x00020000);
  unsigned errs = 0;
  for (int r = 0; r < rounds; ++r) {
    const int base = ((r & 1) * 256) * SLICE;  // parity half: 256 slices each
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const u32x4 v = {(unsigned)r, (unsigned)i, (unsigned)m, (unsigned)g};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, (threadIdx.x + i * 512) * 16, base + me * SLICE, AS);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = 8u * (unsigned)(r + 1);
      int spin = 0;
      for (; spin < (1 << 20); ++spin) {
        if (__hip_atomic_load(gctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (spin == (1 << 20)) {
        __hip_atomic_fetch_add(ctl + 1002, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        role = -2;
      }
    }
    __syncthreads();
    if (role == -2) break;
    u32x4 v[8][PER];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int i = 0; i < PER; ++i)
        v[q][i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + i * 512) * 16, base + ((g << 3) | q) * SLICE, AL);
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int i = 0; i < PER; ++i)
        errs += (v[q][i].x != (unsigned)r) | (v[q][i].y != (unsigned)i) | (v[q][i].z != (unsigned)q) |
                (v[q][i].w != (unsigned)g);
  }
  if (errs) __hip_atomic_fetch_add(ctl + 1000, errs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    case 5: {  // arg = rounds (low 16 bits) | KiB per workgroup << 16; counters must be zero
      (void)hipMemsetAsync(buf, 0, 4096, s);
      hipLaunchKernelGGL(mb_groupsync_kernel, dim3(blocks), dim3(256), 0, s, (unsigned char*)buf, arg & 0xffff,
                         arg >> 16);
      break;
    }
    case 6: {  // arg = rounds (bits 0-11) | variant << 20
      (void)hipMemsetAsync(buf, 0, 4000, s);  // tickets + counters; stats accumulate (word 1000+)
      const int rounds = arg & 0xfff, var = arg >> 20;
      unsigned char* b = (unsigned char*)buf;
#define XS(KB, AL, AS, SP) hipLaunchKernelGGL((mb_xcdsync_kernel<KB, AL, AS, SP>), dim3(blocks), dim3(512), 0, s, b, rounds)
      switch (var) {
        case 0: XS(8, 0, 0, false); break;      // plain loads (stale L1 expected)
        case 1: XS(8, 1, 0, false); break;      // sc0 loads
        case 2: XS(8, 16, 0, false); break;     // sc1 loads
        case 3: XS(8, 16, 16, false); break;    // sc1 loads, sc1 stores
        case 4: XS(8, 16, 16, true); break;     // spread: sc1 loads, sc1 stores
        case 5: XS(8, 1, 0, true); break;       // spread: sc0 loads (not coherent across XCDs)
        case 6: XS(16, 1, 0, false); break;     // 128 KiB gather
        case 7: XS(16, 16, 16, false); break;
        case 8: XS(16, 16, 16, true); break;
        default: return hipErrorInvalidValue;
      }
#undef XS
      break;
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ggd
