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
  KEPre<T, RT> pre = ke_pre<T, RT>(a, blockIdx.x, ltid() >> 6);
  pre.load(ltid() & 63);
  ke_phase<T, RT, CP_KERNEL>(a, blockIdx.x, blockIdx.y, a.do_update ? *a.step_counter : 0, smem, pre);
}

// Step-invariant cross-attention K / V of every (clip, head) of one layer, convolved and in the
// attention-image order (KVC_ELEMS, ggd_fusedlib.h): the 3-tap conv of transformer.py:28-44 over
// the memory rows of nn.py:223 reaches the step token (memory row 0) only from rows 0 and 1, so
// rows 2 .. Ts are the same in every denoise step; they are convolved here once per clip batch
// (ggd_set_memory), with conv3's operation order, and rows 0 / 1 are left to the step kernels.
template <typename T>
__global__ void __launch_bounds__(256) ca_kv_conv_kernel(const float* kv_mem, const float* kw, const float* kb,
                                                         const float* vw, const float* vb, int Ts, T* out) {
  const int h = blockIdx.x, b = blockIdx.y, Lk = 1 + Ts;
  T* K = out + ((size_t)b * (FD / FDK) + h) * KVC_ELEMS;
  T* Vt = K + FLK * FDK;
  const int c = threadIdx.x & 31;  // channel fastest: the memory rows are read coalesced
  const ConvW wk = conv_w(kw, kb, c), wv = conv_w(vw, vb, c);
  const float* base = kv_mem + (size_t)b * Ts * 2 * FD + h * FDK + c;  // speech row j at j 2 FD (K), + FD (V)
  for (int i = threadIdx.x >> 5; i < FLK; i += 256 / 32) {
    float k = 0.f, v = 0.f;
    if (i >= 2 && i < Lk) {
      const float* p0 = base + (size_t)(i - 2) * 2 * FD;
      const float* p1 = p0 + 2 * FD;
      const bool nx = i + 1 < Lk;
      k = conv3(wk, p0[0], p1[0], nx ? p1[2 * FD] : 0.f);
      v = conv3(wv, p0[FD], p1[FD], nx ? p1[3 * FD] : 0.f);
    }
    K[i * FDK + c] = from_f32<T>(k);
    Vt[c * FLK + i] = from_f32<T>(v);
  }
}

hipError_t launch_ca_kv_conv(int dtype, const float* kv_mem, const float* kw, const float* kb, const float* vw,
                             const float* vb, int n, int Ts, void* out, hipStream_t s) {
  if (n < 1 || Ts < 1 || 1 + Ts > FLK) return hipErrorInvalidValue;
  const dim3 grid(FD / FDK, n), blk(256);
  if (dtype == 0) hipLaunchKernelGGL(ca_kv_conv_kernel<float>, grid, blk, 0, s, kv_mem, kw, kb, vw, vb, Ts, (float*)out);
  else hipLaunchKernelGGL(ca_kv_conv_kernel<bf16_t>, grid, blk, 0, s, kv_mem, kw, kb, vw, vb, Ts, (bf16_t*)out);
  return hipGetLastError();
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
