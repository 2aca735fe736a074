// ggd_megasync.h -- placement and clip-group barriers of the persistent clip-group loops
// (ggd_mega.hip: heads / FFN chunks per workgroup; ggd_rows.hip: row blocks where the work is
// row-local).  See ggd_mega.hip's header comment for the placement and residency rules.
#pragma once
#include "ggd_phases.h"


namespace ggd {

// every wait is bounded by elapsed time (wait_expired, ggd_common.h)
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
static __device__ int mk_role(const MegaArgs& m, int nwg) {
  unsigned* ctl = m.ctl;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)mk_add(ctl + xcc * 16, 1u);
  mk_add(ctl + MK_ARRIVE, 1u);
  const unsigned t0 = wait_t0();
  while (mk_load(ctl + MK_ARRIVE) < (unsigned)nwg) {  // every workgroup is resident
    if (wait_expired(t0)) {
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
static __device__ int mk_role_xl(const MegaArgs& m, int nwg, int G) {
  unsigned* ctl = m.ctl;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)mk_add(ctl + xcc * 16, 1u);
  __hip_atomic_fetch_add(ctl + MK_ARRIVE, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned t0 = wait_t0();
  while (__hip_atomic_load(ctl + MK_ARRIVE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nwg) {
    if (wait_expired(t0)) {
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
  if (!poller) prefetch();  // (the poller issues its share before the exit barrier, not after: round 6
                            // measured 69.7 vs 67.6 ms per C2 launch; two polls in flight: 68.0,
                            // profiles/r06q_c2_barrier_poll_ab.txt)
  if constexpr (CPV == CP_XL) {  // vector poll (a poll load retires behind the wave's earlier loads:
    if (threadIdx.x < 64) {      // the poller issues its prefetch after it)
      const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 32u);
      const int off = (threadIdx.x & 7) * 4;
      int ok = 1;
      const unsigned t0 = wait_t0();
      for (int spin = 0;; ++spin) {
        const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, CP_COH);
        if (__ballot(v < epoch) == 0) break;
        if ((spin & 255) == 255) {
          const bool expired = wait_expired(t0);
          if (expired || __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            if (threadIdx.x == 0) status_leave(status, expired);
            ok = 0;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (threadIdx.x == 0) *s_ok = ok;
    }
  } else {
    if (threadIdx.x == 0) {
      const unsigned target = 8u * epoch;
      int ok = 1;
      const unsigned t0 = wait_t0();
      for (int spin = 0; mk_load(ctr) < target; ++spin) {
        if ((spin & 255) == 255) {
          const bool expired = wait_expired(t0);
          if (expired || __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            status_leave(status, expired);
            ok = 0;
            break;
          }
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

}  // namespace ggd
