// ggd_mega.hip -- the reverse loop as ONE persistent launch: the head / chunk clip-group loop, f32
// (the parity mode) only since round 6 -- bf16 contexts run the row-block decomposition of the same
// loop (ggd_rows.hip: 69.2 vs 75.1 ms per C2 pass on one box, profiles/r06d_c2_rows_ab.txt).
//
// The per-phase launches of ggd_fused.hip pay a kernel boundary (grid fill / drain, and loads
// that start cold behind the boundary's cache maintenance) 17 times per denoise step.  Here
// the same phase bodies (ggd_phases.h, instantiated with CP_COH) run back to back inside one
// launch of 8 workgroups per clip; consecutive phases of a clip meet at a barrier of the
// clip's 8 workgroups only (no grid-wide barrier).
//
// Placement: dispatch order and the workgroup -> XCD map are not guaranteed, so a workgroup
// reads its XCC id and takes a ticket on that XCD's counter; clip group g lives on XCD g % 8
// and is filled from that XCD's tickets, so its 8 members share one L2 (measured on MI355X,
// scripts/handoff_bench.py: a 64 KiB clip-row gather + barrier costs 2.0 us per round
// XCD-local against 4.3 us across XCDs).  Workgroups that land on an over-full XCD fill the
// remaining slots elsewhere.  Correctness does not depend on placement: every byte handed
// between workgroups is stored write-through (sc1) and drained before the arrival, and read
// with sc1 loads after the barrier.
//
// Residency: every workgroup must be resident at once (one per CU: 132 KiB LDS); the host
// sizes the grid from the occupancy query, and all waits are bounded -- a barrier that times
// out sets `status` and its workgroups leave, so a wrong assumption ends the launch instead
// of hanging the GPU.
//
// GEMM k-step fences (ggd_phases.h GGD_MK_FENCE_*): kept everywhere except in KA's QKV tile, where
// letting the scheduler move the next k step's LDS reads gives 73.5-73.7 ms per C2 launch against
// 73.9-74.0 (one box, three alternations: profiles/r05w10_c2_fence_qkv_ab.txt); dropping it at the
// cross-attention query costs 1 ms, at the out-projections / FFN 0.1-0.3 ms (r05w9_c2_fence_sites_ab.txt)
#define GGD_MK_FENCE_QKV 0
#include "ggd_megasync.h"

namespace ggd {

template <typename T, int RT, int CPV>
__global__ void __launch_bounds__(FT) mk_kernel(MegaArgs m, int G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_role, s_ok;
  if (m.gate && ggd::G(m.gate)[0] != 3) return;  // gated re-run: the XCD-local launch placed (or failed otherwise)
  if (m.sim_unresident == 1) {  // test hook: as if the workgroups were never all resident
    if (threadIdx.x == 0) atomicMax(m.status, 2);
    return;
  }
  if (threadIdx.x == 0) s_role = CPV == CP_XL ? mk_role_xl(m, gridDim.x, G) : mk_role(m, gridDim.x);
  __syncthreads();
  const int role = s_role;
  if (role < 0) return;
  if (m.sim_unresident == 2 && (role & 1)) {  // test hook: odd parts report 2, the rest wait in a barrier
    if (threadIdx.x == 0) atomicMax(m.status, 2);
    return;
  }
  const int grp = role >> 3, b = m.clip0 + grp, part = role & 7, lane = ltid() & 63, wave = ltid() >> 6;
  unsigned* ctr = m.ctl + MK_GROUP + grp * 16;
  unsigned* flags = m.ctl + MK_FLAGS + grp * 32;
  unsigned epoch = 0;
  if (m.stamps && role == 0 && threadIdx.x == 0) m.stamps[2 * 17 * MEGA_STAMP_STEPS] = __builtin_amdgcn_s_memtime();
  // per-phase arguments as constant-address-space objects: field reads are scalar loads
  typedef const __attribute__((address_space(4))) FusedArgs* cfa_t;
  typedef const __attribute__((address_space(4))) FinalArgs* cfe_t;
  const int NL = m.n_layers;
  cfa_t fa0 = (cfa_t)m.fa;
  cfe_t fe = (cfe_t)m.fe;
  // prologue: the first step's layer-0 residual rows from the initial x (every later step's come
  // from the KE rows phase of the step before)
  emb_prologue<T, CPV>(*fe, part, b, smem);
  // weights of the next phase, issued at the barrier in front of it; KA's and KE's tiles share one
  // register set (Pre1)
  Pre1<T, RT> pn = ka_pre<T, RT>(fa0[0], part, wave);
  if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, nullptr, [&] { pn.load(lane); })) return;
  for (int k = 0; k < m.n_steps; ++k) {
    const int it = m.k0 + k;
    unsigned long long* st = (m.stamps && role == 0 && k < MEGA_STAMP_STEPS) ? m.stamps : nullptr;
    unsigned long long* ar = (m.stamps && grp == 0 && k < MEGA_STAMP_STEPS) ? m.stamps + 2 * 17 * MEGA_STAMP_STEPS + 1 : nullptr;
    for (int li = 0; li < NL; ++li) {
      cfa_t f = fa0 + 4 * li;
      asm volatile("" : "+s"(f));  // per-layer arguments are re-read, not held across the loop
      // the out-projection fragments of KB / KC are issued by the hook behind the attention in front
      KBPre<T, RT> pb(f[1], wave);
      ka_phase<T, RT, CPV, false>(f[0], part, b, smem, pn, [&] { pb.load_tile(1, lane); }, [&] { pb.load_tile(0, lane); });
      if (!mk_sync<CPV, KBPre<T, RT>::TILE_LOADS>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [] {}, ar)) return;
      KCPre<T, RT> pc(f[2], part, wave);
      kb_phase<T, RT, CPV>(f[1], part, b, it, smem, pb, [&] { pc.load_tile(1, lane); }, [&] { pc.load_tile(0, lane); });
      if (!mk_sync<CPV, KCPre<T, RT>::TILE_LOADS>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [] {}, ar)) return;
      kc_phase<T, RT, CPV>(f[2], part, b, smem, pc);
      if (li + 1 < NL) {
        KDPre<T, RT> pd(f[3], part, wave);
        if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pd.load(lane); }, ar)) return;
        kd_phase<T, RT, CPV>(f[3], part, b, smem, pd);
        pn = li + 1 < NL ? ka_pre<T, RT>(f[4], part, wave) : ker_pre<T, RT>(*fe, wave);
      } else {  // the last layer's KD runs inside the KE rows phase, for each block's rows
        pn = ker_pre<T, RT>(*fe, wave);
      }
      if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pn.load(lane); }, ar)) return;
    }
    ker_phase<T, RT, CPV>(*fe, part, b, it, smem, pn);
    pn = ka_pre<T, RT>(fa0[0], part, wave);
    if (!mk_sync<CPV>(ctr, flags, part, ++epoch, m.status, &s_ok, st, [&] { pn.load(lane); }, ar)) return;
  }
}

// LDS: the phases' private regions sit behind the resident residual rows (Res<T>); the kernel's
// static words (role, barrier verdict) need room beside the dynamic allocation
constexpr size_t MK_LDS_STATIC = 256;
constexpr size_t MK_LDS = 160 * 1024 - MK_LDS_STATIC;

// clips one launch of either clip-group loop holds (this one, f32; ggd_rows.hip, bf16): one
// 512-thread workgroup per CU (160 KiB LDS; 186+ VGPRs allow only one too), 8 per clip
int mega_capacity(int dtype, int L) {
  (void)dtype;
  (void)L;
  static int cap = -1;
  if (cap < 0) {
    int dev = 0, cus = 0, lds_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    (void)hipGetLastError();  // nothing above may leave a sticky error for the next launch
    const int per = lds_cu >= (int)MK_LDS ? 1 : 0;
    cap = std::min(32, per * cus / 8);  // control words hold 32 groups
  }
  return cap;
}

template <int RT>
static hipError_t launch_mega_t(const MegaArgs& a, int n, bool xl, hipStream_t s) {
  const int G = n, nwg = xl ? 64 * ((G + 7) / 8) : 8 * G;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mk_kernel<float, RT, CP_XL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)mk_kernel<float, RT, CP_COH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  if (xl)
    hipLaunchKernelGGL((mk_kernel<float, RT, CP_XL>), dim3(nwg), dim3(FT), MK_LDS, s, a, G);
  else
    hipLaunchKernelGGL((mk_kernel<float, RT, CP_COH>), dim3(nwg), dim3(FT), MK_LDS, s, a, G);
  return hipGetLastError();
}

// f32 only: bf16 contexts run the row-block loop (launch_rows)
hipError_t launch_mega(int dtype, int L, const MegaArgs& a, int n, bool xl, hipStream_t s) {
  if (dtype != 0 || L > 64 || n < 1 || n > mega_capacity(dtype, L)) return hipErrorInvalidValue;
  if (xl && (a.placement != 0 || 64 * ((n + 7) / 8) > 8 * mega_capacity(dtype, L))) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.ctl, 0, sizeof(unsigned) * MEGA_CTL_WORDS, s);
  if (e != hipSuccess) return e;
  return L <= 48 ? launch_mega_t<3>(a, n, xl, s) : launch_mega_t<4>(a, n, xl, s);
}

}  // namespace ggd
