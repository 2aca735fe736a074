// ggd_fused.hip -- one launch per decoder phase (ggd_phases.h): the kernels, their launchers.
#include "ggd_phases.h"

namespace ggd {

template <typename T, int RT>
__global__ void __launch_bounds__(FT) ka_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (a.bump_counter && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(a.step_counter, 1);
  KAPre<T, RT> pre = ka_pre<T, RT>(a, blockIdx.x, ltid() >> 6);
  pre.load(ltid() & 63);
  ka_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, smem, pre);
}

template <typename T, int RT>
__global__ void __launch_bounds__(FT) kb_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  KBPre<T, RT> pre(a, ltid() >> 6);
  pre.load(ltid() & 63);
  kb_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, a.t_clip ? 0 : *a.step_counter, smem, pre);
}

template <typename T, int RT>
__global__ void __launch_bounds__(FT) kc_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  KCPre<T, RT> pre(a, blockIdx.x, ltid() >> 6);
  pre.load(ltid() & 63);
  kc_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, smem, pre);
}

template <typename T, int RT>
__global__ void __launch_bounds__(FT) kd_kernel(FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  KDPre<T, RT> pre(a, blockIdx.x, ltid() >> 6);
  pre.load(ltid() & 63);
  kd_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, smem, pre);
}

template <typename T, int RT>
__global__ void __launch_bounds__(FT) ke_kernel(FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  KEPre<T, RT> pre = ke_pre<T, RT>(a, blockIdx.x);
  pre.load(ltid() & 63);
  ke_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, a.do_update ? *a.step_counter : 0, smem, pre);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <typename K>
static void set_lds_attr(K kernel) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <typename T, int RT>
static void set_attrs_rt() {
  set_lds_attr(ka_kernel<T, RT>);
  set_lds_attr(kb_kernel<T, RT>);
  set_lds_attr(kc_kernel<T, RT>);
  set_lds_attr(kd_kernel<T, RT>);
  set_lds_attr(ke_kernel<T, RT>);
}

static bool fused_attrs_done = false;
static void fused_attrs() {
  if (fused_attrs_done) return;
  set_attrs_rt<float, 3>();
  set_attrs_rt<float, 4>();
  set_attrs_rt<bf16_t, 3>();
  set_attrs_rt<bf16_t, 4>();
  fused_attrs_done = true;
}

bool fused_supported(int dtype, int d_model, int heads, int L, int Ts, int C) {
  (void)dtype;
  return d_model == FD && heads == FD / FDK && L >= 1 && L <= FR && Ts >= 1 && 1 + Ts <= FLK && C >= 1 && C <= 128;
}

template <int RT>
static hipError_t launch_fused_rt(int which, int dtype, const FusedArgs& a, int n, hipStream_t s) {
  const dim3 blk(FT), grid(8, n);
  const bool f = dtype == 0;
  switch (which) {
    case 0:
      if (f) hipLaunchKernelGGL((ka_kernel<float, RT>), grid, blk, Plan<float>::KA, s, a);
      else hipLaunchKernelGGL((ka_kernel<bf16_t, RT>), grid, blk, Plan<bf16_t>::KA, s, a);
      break;
    case 1:
      if (f) hipLaunchKernelGGL((kb_kernel<float, RT>), grid, blk, Plan<float>::KB, s, a);
      else hipLaunchKernelGGL((kb_kernel<bf16_t, RT>), grid, blk, Plan<bf16_t>::KB, s, a);
      break;
    case 2:
      if (f) hipLaunchKernelGGL((kc_kernel<float, RT>), grid, blk, Plan<float>::KC, s, a);
      else hipLaunchKernelGGL((kc_kernel<bf16_t, RT>), grid, blk, Plan<bf16_t>::KC, s, a);
      break;
    case 3:
      if (f) hipLaunchKernelGGL((kd_kernel<float, RT>), grid, blk, Plan<float>::KD, s, a);
      else hipLaunchKernelGGL((kd_kernel<bf16_t, RT>), grid, blk, Plan<bf16_t>::KD, s, a);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// row tiles: 48 padded rows for clips of <= 48 frames (the C2 shape, L = 40), else 64
static inline bool rt3(int L) { return L <= 48; }

hipError_t launch_fused(int which, int dtype, const FusedArgs& a, int n, hipStream_t s) {
  fused_attrs();
  return rt3(a.L) ? launch_fused_rt<3>(which, dtype, a, n, s) : launch_fused_rt<4>(which, dtype, a, n, s);
}

hipError_t launch_final(int dtype, const FinalArgs& a, hipStream_t s) {
  fused_attrs();
  const dim3 blk(FT), grid(8, a.n);
  if (rt3(a.L)) {
    if (dtype == 0) hipLaunchKernelGGL((ke_kernel<float, 3>), grid, blk, Plan<float>::KE, s, a);
    else hipLaunchKernelGGL((ke_kernel<bf16_t, 3>), grid, blk, Plan<bf16_t>::KE, s, a);
  } else {
    if (dtype == 0) hipLaunchKernelGGL((ke_kernel<float, 4>), grid, blk, Plan<float>::KE, s, a);
    else hipLaunchKernelGGL((ke_kernel<bf16_t, 4>), grid, blk, Plan<bf16_t>::KE, s, a);
  }
  return hipGetLastError();
}

}  // namespace ggd
