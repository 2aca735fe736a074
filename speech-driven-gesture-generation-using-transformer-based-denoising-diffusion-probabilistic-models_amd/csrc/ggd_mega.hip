// ggd_mega.hip -- the reverse loop as ONE persistent launch.
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
#include "ggd_phases.h"

namespace ggd {

constexpr int MK_SPIN_LIMIT = 1 << 21;   // ~ seconds: only a broken launch ever gets there
constexpr int MK_ARRIVE = 128, MK_OVF = 144, MK_GROUP = 256, MK_FLAGS = 256 + 32 * 16;

__device__ __forceinline__ unsigned mk_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned mk_add(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// slots of XCD x.  placement 0: clip group g lives on XCD g % 8 (8 x the number of groups g < G
// with g % 8 == x); placement 1: part p of every clip lives on XCD p (G slots on every XCD)
__device__ __forceinline__ int mk_slots(int x, int G, int place) {
  if (place == 1) return G;
  return x < G ? 8 * ((G - 1 - x) / 8 + 1) : 0;
}

// thread 0: (clip << 3 | part), or -1 (status set)
__device__ int mk_role(const MegaArgs& m, int nwg) {
  unsigned* ctl = m.ctl;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)mk_add(ctl + xcc * 16, 1u);
  mk_add(ctl + MK_ARRIVE, 1u);
  for (int spin = 0; mk_load(ctl + MK_ARRIVE) < (unsigned)nwg; ++spin) {  // every workgroup is resident
    if (spin > MK_SPIN_LIMIT) {
      atomicMax(m.status, 2);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  const int G = nwg / 8, place = m.placement;
  int x = (int)xcc, s = t;
  if (t >= mk_slots(x, G, place)) {  // over-full XCD: take the o-th unfilled slot, in XCD order
    int o = (int)mk_add(ctl + MK_OVF, 1u);
    for (x = 0; x < 8; ++x) {
      const int have = min((int)mk_load(ctl + x * 16), mk_slots(x, G, place)), holes = mk_slots(x, G, place) - have;
      if (o < holes) {
        s = have + o;
        break;
      }
      o -= holes;
    }
    if (x == 8) {
      atomicMax(m.status, 2);
      return -1;
    }
  }
  if (place == 1) return (s << 3) | x;
  return ((x + 8 * (s >> 3)) << 3) | (s & 7);
}

// XCD-local placement (CP_XL): the grid is padded to 8 workgroups per XCD per 8 clip groups, so
// that XCD x can host every group g with g % 8 == x.  After all workgroups have arrived, every
// XCD must hold at least its groups' slots; otherwise the whole launch leaves before any work
// with status 3 and the host runs it again on the write-through path.  Surplus workgroups idle.
// thread 0: (clip << 3 | part), -2 (idle surplus), or -1 (status set)
__device__ int mk_role_xl(const MegaArgs& m, int nwg, int G) {
  unsigned* ctl = m.ctl;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)mk_add(ctl + xcc * 16, 1u);
  __hip_atomic_fetch_add(ctl + MK_ARRIVE, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  for (int spin = 0; __hip_atomic_load(ctl + MK_ARRIVE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nwg;
       ++spin) {
    if (spin > MK_SPIN_LIMIT) {
      atomicMax(m.status, 2);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  for (int x = 0; x < 8; ++x)  // every workgroup reads the same final counts: a launch-wide verdict
    if ((int)mk_load(ctl + x * 16) < mk_slots(x, G, 0)) {
      atomicMax(m.status, 3);
      return -1;
    }
  if (t >= mk_slots((int)xcc, G, 0)) return -2;
  return (((int)xcc + 8 * (t >> 3)) << 3) | (t & 7);
}

// barrier of the clip's 8 workgroups; epoch counts the barriers passed so far (+1).  After the
// arrival the waves issue `prefetch` (the next phase's weight fragments; the polling wave after its
// poll); the exit barrier does not wait for vector memory, so that stream stays in flight.
// Write-through path (CP_COH): one agent-scope counter per group.  XCD-local path (CP_XL): the
// group's 8 workgroups share one L2, so each publishes its epoch with a plain store into its own
// word of the group's flag line (after its waves' stores have reached that L2) and wave 0 polls
// the 8 words with sc1 loads -- L2 round trips instead of memory-side atomics.
// VMC: vector loads the wave issued after its last hand-off store (the next phase's weights, issued
// by the phase's hook): vmcnt completes in issue order, so waiting down to VMC outstanding drains
// every store without waiting for those loads
// (stamps are indexed by epoch - 2: the prologue's barrier is epoch 1 and is not stamped)
template <int CPV, int VMC = 0, typename F>
__device__ __forceinline__ bool mk_sync(unsigned* ctr, unsigned* flags, int part, unsigned epoch, int* status,
                                        int* s_ok, unsigned long long* st, F&& prefetch,
                                        unsigned long long* arr = nullptr) {
  static_assert(VMC >= 0 && VMC < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");  // this wave's hand-off stores landed
  __syncthreads();
  if (st && threadIdx.x == 0) st[2 * (epoch - 2)] = __builtin_amdgcn_s_memtime();
  // diag: arrival and exit of every workgroup of clip group 0, on the chip-wide 100 MHz clock
  if (arr && threadIdx.x == 0) arr[2 * (8 * (epoch - 2) + part)] = __builtin_amdgcn_s_memrealtime();
  if constexpr (CPV == CP_XL) {
    if (threadIdx.x == 0) {
      const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 32u);
      __builtin_amdgcn_raw_buffer_store_b32(epoch, r, part * 4, 0, 0);
    }
  } else {
    if (threadIdx.x == 0) mk_add(ctr, 1u);
  }
  const bool poller = threadIdx.x < 64;
  if (!poller) prefetch();
  if constexpr (CPV == CP_XL) {  // vector poll (a poll load retires behind the wave's earlier loads:
    if (threadIdx.x < 64) {      // the poller issues its prefetch after it)
      const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 32u);
      const int off = (threadIdx.x & 7) * 4;
      int ok = 1;
      for (int spin = 0;; ++spin) {
        const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, CP_COH);
        if (__ballot(v < epoch) == 0) break;
        if ((spin & 255) == 255 && (spin > MK_SPIN_LIMIT || __hip_atomic_load(status, __ATOMIC_RELAXED,
                                                                               __HIP_MEMORY_SCOPE_AGENT))) {
          if (threadIdx.x == 0) atomicMax(status, 1);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (threadIdx.x == 0) *s_ok = ok;
    }
  } else {
    if (threadIdx.x == 0) {
      const unsigned target = 8u * epoch;
      int ok = 1;
      for (int spin = 0; mk_load(ctr) < target; ++spin) {
        if ((spin & 255) == 255 && (spin > MK_SPIN_LIMIT || __hip_atomic_load(status, __ATOMIC_RELAXED,
                                                                               __HIP_MEMORY_SCOPE_AGENT))) {
          atomicMax(status, 1);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      *s_ok = ok;
    }
  }
  if (poller) prefetch();
  bar_lds();
  if (st && threadIdx.x == 0) st[2 * (epoch - 2) + 1] = __builtin_amdgcn_s_memtime();
  if (arr && threadIdx.x == 0) arr[2 * (8 * (epoch - 2) + part) + 1] = __builtin_amdgcn_s_memrealtime();
  return *s_ok != 0;
}

template <typename T, int RT, int CPV>
__global__ void __launch_bounds__(FT) mk_kernel(MegaArgs m, int G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_role, s_ok;
  if (m.gate && ggd::G(m.gate)[0] != 3) return;  // gated re-run: the XCD-local launch placed (or failed otherwise)
  if (m.sim_unresident) {  // test hook: as if the workgroups were never all resident
    if (threadIdx.x == 0) atomicMax(m.status, 2);
    return;
  }
  if (threadIdx.x == 0) s_role = CPV == CP_XL ? mk_role_xl(m, gridDim.x, G) : mk_role(m, gridDim.x);
  __syncthreads();
  const int role = s_role;
  if (role < 0) return;
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
      if (li + 1 < NL || !GGD_MK_FUSE_KD) {
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
template <typename T, int RT>
static size_t mk_lds() {
  return 160 * 1024 - MK_LDS_STATIC;
}

template <typename T, int RT>
static int mk_capacity_t() {
  static int cap = -1;
  if (cap < 0) {
    (void)hipFuncSetAttribute((const void*)mk_kernel<T, RT, CP_COH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    // residency from the LDS budget (the occupancy query rejects > 64 KiB of dynamic LDS):
    // one 512-thread workgroup per CU
    int dev = 0, cus = 0, lds_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    (void)hipGetLastError();  // nothing above may leave a sticky error for the next launch
    const int per = lds_cu >= (int)mk_lds<T, RT>() ? 1 : 0;  // registers: 186+ VGPRs also allow only one
    cap = std::min(32, per * cus / 8);  // control words hold 32 groups
  }
  return cap;
}

static inline bool mk_rt3(int L) { return L <= 48; }

int mega_capacity(int dtype, int L) {
  if (dtype == 0) return mk_rt3(L) ? mk_capacity_t<float, 3>() : mk_capacity_t<float, 4>();
  return mk_rt3(L) ? mk_capacity_t<bf16_t, 3>() : mk_capacity_t<bf16_t, 4>();
}

template <typename T, int RT>
static hipError_t launch_mega_t(const MegaArgs& a, int n, bool xl, hipStream_t s) {
  const int G = n, nwg = xl ? 64 * ((G + 7) / 8) : 8 * G;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)mk_kernel<T, RT, CP_XL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)mk_kernel<T, RT, CP_COH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  if (xl)
    hipLaunchKernelGGL((mk_kernel<T, RT, CP_XL>), dim3(nwg), dim3(FT), (mk_lds<T, RT>()), s, a, G);
  else
    hipLaunchKernelGGL((mk_kernel<T, RT, CP_COH>), dim3(nwg), dim3(FT), (mk_lds<T, RT>()), s, a, G);
  return hipGetLastError();
}

hipError_t launch_mega(int dtype, int L, const MegaArgs& a, int n, bool xl, hipStream_t s) {
  if (n < 1 || n > mega_capacity(dtype, L)) return hipErrorInvalidValue;
  if (xl && (a.placement != 0 || 64 * ((n + 7) / 8) > 8 * mega_capacity(dtype, L))) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.ctl, 0, sizeof(unsigned) * MEGA_CTL_WORDS, s);
  if (e != hipSuccess) return e;
  if (dtype == 0) return mk_rt3(L) ? launch_mega_t<float, 3>(a, n, xl, s) : launch_mega_t<float, 4>(a, n, xl, s);
  return mk_rt3(L) ? launch_mega_t<bf16_t, 3>(a, n, xl, s) : launch_mega_t<bf16_t, 4>(a, n, xl, s);
}

}  // namespace ggd
