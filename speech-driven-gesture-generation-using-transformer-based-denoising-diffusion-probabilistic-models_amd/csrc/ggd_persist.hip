// ggd_persist.hip -- the persistent per-clip sampler: ONE workgroup owns ONE clip for the whole
// reverse loop (gaussian_diffusion.py:331-412 / 414-529 around nn.py:216-228), bf16 MFMA.
//
// Why: a denoise step of a 40-frame clip is ~0.3 GFLOP, far too little to fill the chip with
// one launch per decoder phase; split over 8 workgroups per clip, every phase pays a launch
// (or an in-kernel hand-off) of ~2-4 us plus a cold round trip for the activations.  Here the
// clip's residual stream, LayerNorm images, attention operands, FFN chunk and pose state stay
// in LDS / registers across all T' steps; nothing crosses workgroups, so there is no barrier
// between clips, no counter and no hipGraph -- one launch runs the whole sampling call.
// The only global traffic per step is the bf16 weights (7.5 MB, fragment-packed, L2 / MALL
// resident, streamed with 1 KiB coalesced wave loads one GEMM ahead of their use) and the
// clip's cached cross-attention memory rows.
//
// Per step (clip b, L <= 16 RT rows, d 256, 8 heads, Lk = 1 + Ts <= 64, C <= 128):
//   emb:    Xb = bf16(x) ; Hs = Xb W_emb^T + b + PE                       (transformer.py:176-180)
//   layer:  Xn = LN1(Hs); per head pair: Y = Xn Wqkv^T + b, per head conv Q/K/V + attention -> O
//           Hs += O Wo^T + b ; Xn = LN2(Hs); per head: Q = conv(Xn Wq^T + b), K/V = conv(memory
//           rows [step token(t); speech]) , attention -> O ; Hs += O Wo^T + b ; Xn = LN3(Hs);
//           per 128-wide chunk: H = relu(Xn W1^T + b)^2, acc += H W2^T ; Hs += acc + b2
//   out:    E = LN_out(Hs) W_out^T + b ; x = posterior update (Philox noise)  (nn.py:211-228)
// No scheduling fence between a GEMM's k steps in this unit (ggd_fusedlib.h GGD_SCHED_FENCE; the
// clip-group loop keeps it): the per-clip loops sit at 256 VGPRs, and letting the scheduler move the
// next step's LDS reads across the MFMAs measured 7.15-7.17 ms per C5 launch against 7.46-7.60 with
// the fence (profiles/r05w3_c5_fence_ab.txt; the clip-group loop is 1.6 % slower without it,
// r05w3_c2_fence_ab.txt).  Same instructions, same results.
#ifndef GGD_SCHED_FENCE
#define GGD_SCHED_FENCE 0
#endif
#include "ggd_fusedlib.h"

namespace ggd {

template <int RT> struct PPlan {
  static constexpr int R = RT * 16;                  // padded rows
  static constexpr int SX = FD + 8;                  // bf16 operand image stride
  static constexpr int SY = 192 + 4;                 // f32 QKV of a head pair
  static constexpr int SYQ = FDK + 4;                // f32 cross-attn Q of a head
  static constexpr int SHD = 128 + 8;                // bf16 FFN chunk / emb operand
  static constexpr int SE = 128 + 4;                 // f32 eps
  static constexpr size_t HS = al16(sizeof(float) * R * SH);
  static constexpr size_t IMG = al16(sizeof(bf16_t) * R * SX);
  static constexpr size_t ST = al16(sizeof(float2) * R);
  static constexpr size_t Y = al16(sizeof(float) * R * SY);
  static constexpr size_t ATT = al16(FAtt<bf16_t, R>::BYTES);
  static constexpr size_t YQ = al16(sizeof(float) * R * SYQ);
  static constexpr size_t RAW = al16(sizeof(float) * 2 * (FLK + 2) * FDK);
  static constexpr size_t HID = al16(sizeof(bf16_t) * R * SHD);
  static constexpr size_t E = al16(sizeof(float) * R * SE);
  // attention of a head PAIR at once: two attention images, the second overlaying the first's
  // 4th P tile (query row tile 3 is always past L <= 48, its wave never touches it)
  static constexpr int SYB = 192 + 8;                // bf16 pre-conv QKV of a head pair
  static constexpr size_t YB = al16(sizeof(bf16_t) * R * SYB);
  static constexpr size_t ATT_B = FAtt<bf16_t, R>::BYTES - sizeof(bf16_t) * 16 * FAtt<bf16_t, R>::SP;
  static constexpr size_t ATT2 = ATT_B + ATT;
  static constexpr size_t RAWB = sizeof(bf16_t) * 2 * 2 * FLK * FDK;  // bf16 memory K|V of a head pair
  static constexpr size_t SCR = std::max(std::max(YB + ATT2, RAWB + ATT2), std::max(HID, E + HID));
  static constexpr size_t OFF_XN = HS, OFF_O = HS + IMG, OFF_ST = HS + 2 * IMG, OFF_S = OFF_ST + ST;
  static constexpr size_t TOTAL = OFF_S + SCR;
};
static_assert(PPlan<3>::TOTAL <= 160 * 1024, "persistent plan must fit 160 KiB of LDS");

// fragments of NJ tiles x KS k steps (tile t, step k0 + s) -> f[j * KS + s]
template <int NJ, int KS, int N, int NTL>
__device__ __forceinline__ void pload(uint4 (&f)[N], const void* W, int kt_total, const int (&tiles)[NTL], int k0,
                                      int lane) {
  static_assert(NJ * KS <= N && NJ <= NTL, "fragment buffer / tile list too small");
  // buffer loads: the SGPR resource + scalar byte offset carry the (tile, step) address, so all
  // fragment loads of a wave share ONE vector register (lane * 16) instead of a 64-bit address each
  const __amdgpu_buffer_rsrc_t rs = uni_rsrc(W, 0x7fffffffu);
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
          rs, lane * 16, __builtin_amdgcn_readfirstlane((tiles[j] * kt_total + k0 + s) * 1024), 0);
      f[j * KS + s] = make_uint4(v.x, v.y, v.z, v.w);
    }
}

// acc[rt][j] += A[rows of tile rt][k steps kc0 .. kc0 + KS) x f[j * KS + s] for j < nj (wave-
// uniform).  The A fragments of step s + 1 are read from LDS before the MFMAs of step s issue,
// so the LDS latency runs under the matrix work instead of between every MFMA.
// TR: computed transposed (the weight fragments as the MFMA A operand), so lane (c16, g4) of tile
// (rt, j) holds row 16 rt + c16, columns 16 j' + 4 g4 .. + 3 (four consecutive channels of one token)
template <int RT, int NJ, int KS, int N, bool TR = false, int FENCE = -1>  // FENCE -1: the unit's SCHED_FENCE
__device__ __forceinline__ void pmma_n(f32x4 (&acc)[RT][NJ], const bf16_t* A, int SA, int kc0, const uint4 (&f)[N],
                                       int nj, int lane) {
  constexpr bool FEN = FENCE < 0 ? SCHED_FENCE : FENCE != 0;
  const int r16 = lane & 15, g = lane >> 4;
  const bf16_t* a0 = A + r16 * SA + kc0 * 32 + g * 8;
  bf16x8 cur[RT], nxt[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) cur[rt] = *(const bf16x8*)(a0 + rt * 16 * SA);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + 1 < KS) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) nxt[rt] = *(const bf16x8*)(a0 + rt * 16 * SA + (s + 1) * 32);
    }
    if constexpr (FEN) __builtin_amdgcn_sched_barrier(0);  // reads of s + 1 stay ahead (WGemm::run)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (j < nj) {
          if constexpr (TR)
            acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f[j * KS + s]), cur[rt],
                                                                 acc[rt][j], 0, 0, 0);
          else
            acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[rt], __builtin_bit_cast(bf16x8, f[j * KS + s]),
                                                                 acc[rt][j], 0, 0, 0);
        }
    if constexpr (FEN) __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < KS) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) cur[rt] = nxt[rt];
    }
  }
}

template <int RT, int NJ, int KS, int N, bool TR = false, int FENCE = -1>
__device__ __forceinline__ void pmma(f32x4 (&acc)[RT][NJ], const bf16_t* A, int SA, int kc0, const uint4 (&f)[N],
                                     int lane) {
  pmma_n<RT, NJ, KS, N, TR, FENCE>(acc, A, SA, kc0, f, NJ, lane);
}

// residual epilogue of a transposed (TR) tile pair: lane (c16, g4) of tile (rt, j) holds row
// 16 rt + c16, columns 16 (2 w + j) + 4 g4 .. + 3 -> one float4 read-modify-write of Hs per tile
// (instead of four scalar ones); b: the bias of those 4 columns per j
template <int RT>
__device__ __forceinline__ void p_resid_tr(float* Hs, const f32x4 (&acc)[RT][2], const float4 (&b)[2], int wave,
                                           int c16, int g4) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (2 * wave + j) * 16 + 4 * g4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float4* p = (float4*)(Hs + (rt * 16 + c16) * SH + col);
      const float4 h = *p;
      *p = make_float4(h.x + (acc[rt][j][0] + b[j].x), h.y + (acc[rt][j][1] + b[j].y), h.z + (acc[rt][j][2] + b[j].z),
                       h.w + (acc[rt][j][3] + b[j].w));
    }
  }
}

template <int RT, int NJ>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[RT][NJ]) {
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int QR>
__device__ __forceinline__ void fattn_lds(unsigned char* att, int Lq, int Lk, float scale, bf16_t* out, int ldo,
                                          int tid, const bf16_t* qext = nullptr, int sqe = 0) {
  if (Lk <= 32)
    fattn<bf16_t, 2, QR, true>(att, Lq, Lk, scale, out, ldo, tid, qext, sqe);
  else
    fattn<bf16_t, 4, QR, true>(att, Lq, Lk, scale, out, ldo, tid, qext, sqe);
}

// Per-loop-body thread ids.  threadIdx.x is laundered through an empty asm so that every
// value derived from it is recomputed inside the loop body: LICM would otherwise hoist dozens
// of lane-dependent offsets out of the step loop, keep them live for all T' steps and spill
// them -- and each spill reload is a vmcnt wait that also drains the weight prefetches.
#define LANE_IDS()                                                      \
  int tid = threadIdx.x;                                                \
  asm volatile("" : "+v"(tid));                                         \
  const int lane = tid & 63, c16 = lane & 15, g4 = lane >> 4;           \
  const int c4 = lane * 4;                                              \
  (void)c16; (void)g4; (void)c4

#define PSTAMP(i)                                                                               \
  do {                                                                                          \
    if (a.stamps && k == 0 && blockIdx.x == 0 && threadIdx.x == 0) a.stamps[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// stamps inside the last layer (scripts/pair_stamps.py: slots 6 .. 15)
#define LSTAMP(i)                                                                               \
  do {                                                                                          \
    if (li + 1 == a.n_layers) PSTAMP(i);                                                        \
  } while (0)
#define FSTAMP(i)                                                                               \
  do {                                                                                          \
    if (a.stamps && k == 0 && li == 0 && hd == 1 && blockIdx.x == 0 && threadIdx.x == 0)         \
      a.stamps[i] = __builtin_amdgcn_s_memtime();                                               \
  } while (0)

// Per-GEMM k-step fences of the transposed pair / clip route (pmma FENCE; -1: the unit's
// GGD_SCHED_FENCE): only the output projection keeps the fence -- 7.14 vs 7.20 ms per C5 launch, mean
// of five alternations on two boxes (profiles/r05w14_c5_fence_sites_ab.txt, r05w15_c5_fence_out_ab.txt)
constexpr int PSK_FENCE_OUT = 1;

constexpr int PK_THREADS = 512;  // 8 waves: two per SIMD, so one wave's LDS / L2 waits overlap the other's MFMAs

// ------------------------------------------------------------------------------------------
// Clip pairs.  With fewer clips than CUs (C5: 128 clips per GPU on 256 CUs) one workgroup per
// clip leaves half the chip idle, so a clip can be split over TWO workgroups: part p runs the
// attention of heads 4p .. 4p + 3 and FFN chunks 4p .. 4p + 3 (1024 / 128 = 8 chunks).  The
// partners meet three times per layer: after the self- and the cross-attention each runs the
// out-projection on its OWN four heads' columns (K = 128 of 256) and after the FFN its FFN-down on its
// own four chunks; each hands that partial sum (L x 256, rounded to bf16) to the other and both add
// part 0's + part 1's (round 5: half the out-projection MFMAs and weight stream; swapping the heads'
// attention outputs and running the whole out-projection in both was 7.53 vs 7.43 ms per C5 launch).
// Every other step-loop value (embedding, LayerNorms, output projection, posterior update with its
// counter noise) is computed identically by both, so both hold the same pose state and part 0 alone
// writes it.
//
// Placement: a workgroup takes a ticket on its XCD; when every XCD holds its pairs' slots, the
// partners share an L2 and hand-offs are plain stores + sc1 loads (as ggd_mega.hip's CP_XL);
// otherwise every workgroup takes pair blockIdx.x / 2 and hand-off stores write through (sc1).
// All waits are bounded: a timed-out barrier sets `status` and its workgroups leave.
// ------------------------------------------------------------------------------------------
constexpr int PP_ARRIVE = 128, PP_FLAGS = 256;

__device__ __forceinline__ int pp_slots(int x, int P) { return x < P ? 2 * ((P - 1 - x) / 8 + 1) : 0; }

// thread 0: (pair << 2) | (xl << 1) | part, -2 (idle surplus) or -1 (status set)
__device__ int pp_role(const PersistArgs& a, int nwg, int P) {
  unsigned* ctl = a.ctl;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  const int t = (int)__hip_atomic_fetch_add(ctl + xcc * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(ctl + PP_ARRIVE, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned t_res = wait_t0();
  while (__hip_atomic_load(ctl + PP_ARRIVE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nwg) {
    if (wait_expired(t_res)) {
      atomicMax(a.status, 2);
      return -1;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  bool xl = !a.force_coh;  // every workgroup reads the same final counts: one verdict per launch
  for (int x = 0; x < 8; ++x)
    if ((int)__hip_atomic_load(ctl + x * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < pp_slots(x, P)) xl = false;
  if (xl) {
    if (t >= pp_slots((int)xcc, P)) return -2;
    return (((int)xcc + 8 * (t >> 1)) << 2) | 2 | (t & 1);
  }
  const int pair = (int)blockIdx.x >> 1;
  return pair < P ? (pair << 2) | ((int)blockIdx.x & 1) : -2;
}

// barrier of a clip's two workgroups: every wave's hand-off stores have landed (vmcnt(0)), then
// thread 0 publishes `epoch` in its word of the pair's flag line and wave 0 polls the partner's
__device__ __forceinline__ bool pp_sync(unsigned* flags, int part, unsigned epoch, bool xl, int* status, int* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = uni_rsrc(flags, 8u);
  if (threadIdx.x == 0) {
    if (xl)
      __builtin_amdgcn_raw_buffer_store_b32(epoch, r, part * 4, 0, 0);
    else
      __hip_atomic_store(flags + part, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x < 64) {
    int ok = 1;
    const unsigned t0 = wait_t0();
    for (int spin = 0;; ++spin) {
      const unsigned v = xl ? __builtin_amdgcn_raw_buffer_load_b32(r, (part ^ 1) * 4, 0, CP_COH)
                            : __hip_atomic_load(flags + (part ^ 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= epoch) break;
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
  bar_lds();
  return *s_ok != 0;
}

typedef __attribute__((ext_vector_type(4))) unsigned int pp_u32x4;
__device__ __forceinline__ void pp_put16(const __amdgpu_buffer_rsrc_t& r, int off, pp_u32x4 v, bool xl) {
  if (xl)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, CP_COH);
}

// partial sums of the two halves of a K split (FFN-down and the attention out-projections): wave w's accumulators of column tiles 2w, 2w + 1, rounded to bf16 and handed
// over in lane order; both parts add part 0's + part 1's -- each rounds its OWN partial too, so both
// add the same two bf16 values and hold the same bits
template <int RT>
__device__ __forceinline__ bool pp_sum_partials(f32x4 (&acc)[RT][2], int part, unsigned char* xb, unsigned& ep,
                                                unsigned* flags, bool xl, int* status, int* s_ok, int wave, int lane) {
  ++ep;
  const size_t sl = (size_t)(ep & 1) * PAIR_SLOT_BYTES;
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  u32x2 mine[RT][2];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4 v = acc[rt][j];
      mine[rt][j] = u32x2{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])};
    }
  {
    const __amdgpu_buffer_rsrc_t r = uni_rsrc(xb + (size_t)part * 2 * PAIR_SLOT_BYTES + sl, (uint32_t)PAIR_SLOT_BYTES);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int off = (((wave * RT + rt) * 2 + j) * 64 + lane) * 8;
        if (xl) __builtin_amdgcn_raw_buffer_store_b64(mine[rt][j], r, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(mine[rt][j], r, off, 0, CP_COH);
      }
  }
  if (!pp_sync(flags, part, ep, xl, status, s_ok)) return false;
  const __amdgpu_buffer_rsrc_t r = uni_rsrc(xb + (size_t)(part ^ 1) * 2 * PAIR_SLOT_BYTES + sl, (uint32_t)PAIR_SLOT_BYTES);
  u32x2 o[RT][2];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      o[rt][j] = __builtin_amdgcn_raw_buffer_load_b64(r, (((wave * RT + rt) * 2 + j) * 64 + lane) * 8, 0, CP_COH);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u32x2 m = mine[rt][j], q = o[rt][j];
      acc[rt][j] = f32x4{__uint_as_float(m.x << 16) + __uint_as_float(q.x << 16),              // commutative:
                         __uint_as_float(m.x & 0xffff0000u) + __uint_as_float(q.x & 0xffff0000u),  // same bits
                         __uint_as_float(m.y << 16) + __uint_as_float(q.y << 16),              // in both parts
                         __uint_as_float(m.y & 0xffff0000u) + __uint_as_float(q.y & 0xffff0000u)};
    }
  return true;
}

template <int RT, bool PAIR>
__global__ void __launch_bounds__(PK_THREADS) psk_kernel(PersistArgs a, int P) {
  // the split out-projections: pairs on the transposed route
  constexpr bool SPLITO = PAIR;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_role, s_ok;
  if (a.gate && !gate_open(a.gate, a.gate_xl)) return;  // the loop this launch stands in for ran
  using PL = PPlan<RT>;
  using T = bf16_t;
  using AT = FAtt<T, PL::R>;
  constexpr int NT = PK_THREADS;
  constexpr int R = PL::R, SX = PL::SX, SY = PL::SY, SYQ = PL::SYQ, SHD = PL::SHD, SE = PL::SE;
  constexpr int NQ = (R * 128 / 4 + NT - 1) / NT;  // state quads per thread
  float* Hs = (float*)smem;
  T* Xn = (T*)(smem + PL::OFF_XN);
  T* Ob = (T*)(smem + PL::OFF_O);
  float2* st = (float2*)(smem + PL::OFF_ST);
  unsigned char* scr = smem + PL::OFF_S;
  T* Yb = (T*)scr;                              // self-attention: bf16 QKV (pre-conv) of a head pair
  unsigned char* att_sa = scr + PL::YB;         // two attention images (head pair)
  unsigned char* att_ca = scr + PL::RAWB;
  T* Hd = (T*)scr;                              // FFN chunk
  float* E = (float*)scr;                       // eps (out projection)
  T* Xb = (T*)(scr + PL::E);                    // emb operand

  // clip b; PAIR: this workgroup's part (heads 4 part .., FFN chunks 4 part ..), its pair's flag
  // line and hand-off slots [part][epoch & 1]
  int b = a.clip0 + (int)blockIdx.x, part = 0;
  bool xl = false;
  unsigned* flags = nullptr;
  unsigned char* xb = nullptr;
  unsigned ep = 0;
  if constexpr (PAIR) {
    if (a.sim_unresident == 1) {  // test hook: as if the pairs were never all resident
      if (threadIdx.x == 0) atomicMax(a.status, 2);
      return;
    }
    if (threadIdx.x == 0) s_role = pp_role(a, gridDim.x, P);
    __syncthreads();
    const int role = __builtin_amdgcn_readfirstlane(s_role);
    if (role < 0) return;
    b = a.clip0 + (role >> 2);
    part = role & 1;
    xl = (role & 2) != 0;
    flags = a.ctl + PP_FLAGS + (role >> 2) * 32;
    xb = a.xbuf + (size_t)(role >> 2) * 4 * PAIR_SLOT_BYTES;
    if (a.sim_unresident == 2 && part == 1) {  // test hook: part 1 reports 2, part 0 waits in its first hand-off
      if (threadIdx.x == 0) atomicMax(a.status, 2);
      return;
    }
  }
  constexpr int HP = PAIR ? 2 : 4, NC = PAIR ? 4 : 8;  // head pairs, FFN chunks of this workgroup
  const int hp0 = PAIR ? 2 * part : 0, c0f = PAIR ? 4 * part : 0, qoff = 12 * hp0;
  const int tid = threadIdx.x, lane = tid & 63, c16 = lane & 15, g4 = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile indices live in SGPRs
  const int Lk = 1 + a.Ts;
  const size_t row0 = (size_t)b * a.L;
  const int c4 = (tid & 63) * 4;
  // QKV head pair: waves 0-3 own local tiles 2w, 2w+1; waves 4-7 own tile 8 + (w - 4)
  const int nq = wave < 4 ? 2 : 1;
  const int tq0 = wave < 4 ? 2 * wave : 8 + (wave - 4), tq1 = wave < 4 ? 2 * wave + 1 : tq0;

  // pose state of the clip in registers: quad q = tid + NT j holds elements e = 4q + u of the
  // reference (C, L) order (c = e / L, l = e % L); read from the internal (L, C) layout
  float xr[NQ][4];
  {
    const int L = a.L, C = a.C, LC = L * C;
#pragma unroll
    for (int j = 0; j < NQ; ++j)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = min(4 * (tid + NT * j) + u, LC - 1), cc = e / L, l = e - cc * L;
        xr[j][u] = a.x[(row0 + l) * C + cc];
      }
  }

  // fa: 2 tiles x 8 k steps (QKV pair, out-projections, CA query, FFN-up, output projection)
  // fb: 2 tiles x 4 k steps (FFN-down chunk, emb).  Each is refilled right after its last use
  // with the next GEMM that uses it, so its loads run under the phases in between.
  uint4 fa[16], fb[8];
  {
    const int te[2] = {2 * wave, 2 * wave + 1};
    pload<2, 4>(fb, a.w_emb, 4, te, 0, lane);
    const int tq[2] = {qoff + tq0, qoff + tq1};
    if (nq == 2) pload<2, 8>(fa, a.layers[0].qkv, 8, tq, 0, lane);
    else pload<1, 8>(fa, a.layers[0].qkv, 8, tq, 0, lane);
  }

  for (int k = 0; k < a.n_steps; ++k) {
    LANE_IDS();
    const StepRec rec = a.steps[a.k0 + k];
    const int t = rec.t_orig;
    // Laundered per-iteration copies of the shape scalars: index / address arithmetic derived
    // from them is recomputed every step instead of being hoisted out of the step loop, where
    // loop-invariant addresses would sit in registers for all T' steps and spill.
    int L = a.L, C = a.C;
    asm volatile("" : "+s"(L), "+s"(C));
    const int LC = L * C;
    PSTAMP(0);
    // ---------------- emb_x + PE of the current state -> Hs (transformer.py:176-180) ----------------
    {
      float pe[2][RT][4], be[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = (2 * wave + j) * 16 + c16;
        be[j] = a.b_emb[col];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) pe[j][rt][r] = a.pe[(size_t)min(rt * 16 + 4 * g4 + r, L - 1) * FD + col];
      }
      for (int i = tid; i < R * SHD / 8; i += NT) ((uint4*)Xb)[i] = make_uint4(0, 0, 0, 0);
      bar_lds();
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const int q = tid + NT * j;
        int cc = (4 * q) / L, l = 4 * q - cc * L;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (4 * q + u < LC) Xb[l * SHD + cc] = from_f32<T>(xr[j][u]);
          if (++l == L) { l = 0; ++cc; }
        }
      }
      bar_lds();
      f32x4 acc[RT][2];
      zero_acc(acc);
      pmma<RT, 2, 4, 8, false, -1>(acc, Xb, SHD, 0, fb, lane);
      {  // fb <- layer 0's first FFN-down chunk
        const int td[2] = {2 * wave, 2 * wave + 1};
        pload<2, 4>(fb, a.layers[0].ff2, 32, td, 4 * c0f, lane);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = (2 * wave + j) * 16 + c16;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) Hs[(rt * 16 + 4 * g4 + r) * SH + col] = acc[rt][j][r] + be[j] + pe[j][rt][r];
      }
      bar_lds();
    }
    PSTAMP(1);

    for (int li = 0; li < a.n_layers; ++li) {
      LANE_IDS();
      const FusedLayer& w = a.layers[li];
      // ---------------- self-attention block (nn.py:160-162) ----------------
      {
        ln_rows<T, NT, R, SX>(Hs, L, Xn, tid);  // LN1 affine folded into the next Linear
        bar_lds();
      }
      LSTAMP(6);
      for (int hi = 0; hi < HP; ++hi) {
        LANE_IDS();
        const int hp = hp0 + hi;
        // the head pair's QKV computed transposed, the 3-tap conv over tokens in registers (DPP
        // lane rotations, conv_tokens: the clip-group loop's KA epilogue) and the convolved rows
        // written straight into the two attention images -- no pre-conv image, no conv pass, one
        // LDS barrier fewer per head pair.  Local tile t (0 .. 11) = head t / 6, kind (Q, K, V)
        // (t % 6) / 2, channels 16 (t % 2) .. of the head
        {
          f32x4 acc[RT][2];
          zero_acc(acc);
          pmma_n<RT, 2, 8, 16, true, -1>(acc, Xn, SX, 0, fa, nq, lane);
          if (hi < HP - 1) {  // refill: the next head pair, or the SA out-projection
            const int tq[2] = {12 * (hp + 1) + tq0, 12 * (hp + 1) + tq1};
            if (nq == 2) pload<2, 8>(fa, w.qkv, 8, tq, 0, lane);
            else pload<1, 8>(fa, w.qkv, 8, tq, 0, lane);
          } else {
            const int to[2] = {2 * wave, 2 * wave + 1};
            if constexpr (SPLITO) pload<2, 4>(fa, w.o_sa, 8, to, 4 * part, lane);  // K rows of its own heads
            else pload<2, 8>(fa, w.o_sa, 8, to, 0, lane);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (j >= nq) break;
            const int t = j == 0 ? tq0 : tq1, hh = t / 6, kind = (t % 6) >> 1, c0 = (t & 1) * 16 + 4 * g4;
            const float4 bq = ld_f4(w.qkv_b + hp * 192 + t * 16 + 4 * g4);
            ConvW cw[4];
            conv_w4(cw, kind == 0 ? w.sa_qw : kind == 1 ? w.sa_kw : w.sa_vw,
                    kind == 0 ? w.sa_qb : kind == 1 ? w.sa_kb : w.sa_vb, c0);
            f32x4 v[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
              v[rt] = f32x4{acc[rt][j][0] + bq.x, acc[rt][j][1] + bq.y, acc[rt][j][2] + bq.z, acc[rt][j][3] + bq.w};
            conv_tokens<RT>(v, cw, L, c16);
            unsigned char* at = att_sa + hh * PL::ATT_B;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
              if (kind == 0) put_tok4<T, false>((T*)(at + AT::OQ), AT::SQ, rt * 16 + c16, c0, v[rt]);
              else if (kind == 1) put_tok4<T, false>((T*)(at + AT::OK), AT::SQ, rt * 16 + c16, c0, v[rt]);
              else put_tok4<T, true>((T*)(at + AT::OV), AT::SV, rt * 16 + c16, c0, v[rt]);
            }
          }
          if constexpr (R < FLK) {  // keys past the row tiles: K rows finite, V^T columns zero
            for (int e = tid; e < 2 * FDK * (FLK - R); e += NT) {
              const int hh = e / (FDK * (FLK - R)), q = e % (FDK * (FLK - R)), c = q / (FLK - R), key = R + q % (FLK - R);
              unsigned char* at = att_sa + hh * PL::ATT_B;
              ((T*)(at + AT::OV))[c * AT::SV + key] = from_f32<T>(0.f);
              ((T*)(at + AT::OK))[key * AT::SQ + c] = from_f32<T>(0.f);
            }
          }
        }
        bar_lds();
        {  // both heads of the pair at once: threads 0-255 head 2hp, 256-511 head 2hp + 1
          LANE_IDS();
          const int hh = tid >> 8, t2 = tid & 255;
          fattn_lds<R>(att_sa + hh * PL::ATT_B, L, L, a.scale, Ob + (2 * hp + hh) * FDK, SX, t2);
          bar_lds();
        }
      }
      PSTAMP(2);
      // SA out-projection + residual
      {
        const float4 bo4[2] = {ld_f4(w.o_sa_b + (2 * wave) * 16 + 4 * g4), ld_f4(w.o_sa_b + (2 * wave + 1) * 16 + 4 * g4)};
        f32x4 acc[RT][2];
        zero_acc(acc);
        if constexpr (SPLITO) pmma<RT, 2, 4, 16, true, -1>(acc, Ob, SX, 4 * part, fa, lane);  // its own heads' columns
        else pmma<RT, 2, 8, 16, true>(acc, Ob, SX, 0, fa, lane);
        if constexpr (PAIR) {  // fa <- cross-attn Q of this part's heads: wave w owns column tile 8 part + w
          const int tq[1] = {8 * part + wave};
          pload<1, 8>(fa, w.q_ca, 8, tq, 0, lane);
        } else {  // fa <- cross-attn Q of every head: wave w owns head w's two column tiles
          const int tq[2] = {2 * wave, 2 * wave + 1};
          pload<2, 8>(fa, w.q_ca, 8, tq, 0, lane);
        }
        LSTAMP(7);
        if constexpr (SPLITO)
          if (!pp_sum_partials<RT>(acc, part, xb, ep, flags, xl, a.status, &s_ok, wave, lane)) return;
        LSTAMP(8);
        p_resid_tr<RT>(Hs, acc, bo4, wave, c16, g4);
        bar_lds();
      }
      // ---------------- cross-attention block (nn.py:163-167) ----------------
      {
        ln_rows<T, NT, R, SX>(Hs, L, Xn, tid);  // LN2 affine folded into the next Linear
        bar_lds();
      }
      LSTAMP(9);
      // memory K / V of a head pair: the step-invariant rows come convolved and in image order
      // from the kvc block (set_memory); rows 0 / 1 (the step token's conv reach) are computed by
      // the last wave of each half.  Threads 0-255 stage head 2hp, 256-511 head 2hp + 1.
      const T* kvc_b = (const T*)w.kvc + (size_t)b * (FD / FDK) * KVC_ELEMS;
      const float* kvs_t = w.kv_step + (size_t)t * 2 * FD;
      const float* kvm_b = w.kv_mem + (size_t)b * a.Ts * 2 * FD;
      const bool fixer = (wave & 3) == 3;
      KvcStage<T, NT / 2, R> kvs;
      KvFix fx;
      kvs.load(kvc_b + (size_t)(2 * hp0 + (tid >> 8)) * KVC_ELEMS, tid & 255);
      if (fixer) fx.load(kvs_t, kvm_b, a.Ts, 2 * hp0 + (tid >> 8), lane);
      // the cross-attention queries of all 8 heads in one GEMM (wave w: head w's 32 columns), kept
      // pre-conv in bf16 in the Xn image once every wave is done reading Xn
      T* Yqb = Xn;
      {
        // PAIR: the part's 4 heads, wave w one column tile (8 part + w)
        constexpr int NQJ = PAIR ? 1 : 2;
        const int qt0 = PAIR ? 8 * part + wave : 2 * wave;
        // transposed, the 3-tap conv over tokens in registers: Yqb holds the CONVOLVED queries,
        // which the attention reads in place (no conv pass per head pair)
        f32x4 acc[RT][NQJ];
        zero_acc(acc);
        pmma<RT, NQJ, 8, 16, true, -1>(acc, Xn, SX, 0, fa, lane);
        {  // fa <- the CA out-projection
          const int to[2] = {2 * wave, 2 * wave + 1};
          if constexpr (SPLITO) pload<2, 4>(fa, w.o_ca, 8, to, 4 * part, lane);
          else pload<2, 8>(fa, w.o_ca, 8, to, 0, lane);
        }
        bar_lds();
#pragma unroll
        for (int j = 0; j < NQJ; ++j) {
          const int c0 = ((qt0 + j) & 1) * 16 + 4 * g4;  // channel of the head
          const float4 bq = ld_f4(w.q_ca_b + (qt0 + j) * 16 + 4 * g4);
          ConvW cw[4];
          conv_w4(cw, w.ca_qw, w.ca_qb, c0);
          f32x4 v[RT];
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
            v[rt] = f32x4{acc[rt][j][0] + bq.x, acc[rt][j][1] + bq.y, acc[rt][j][2] + bq.z, acc[rt][j][3] + bq.w};
          conv_tokens<RT>(v, cw, L, c16);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) put_tok4<T, false>(Yqb, SX, rt * 16 + c16, (qt0 + j) * 16 + 4 * g4, v[rt]);
        }
      }
      LSTAMP(10);
      // head pairs: both heads' conv and attention at once (threads 0-255 head 2hp, 256-511 head
      // 2hp + 1); the next pair's memory K|V loads fly under this pair's work
      for (int hi = 0; hi < HP; ++hi) {
        LANE_IDS();
        const int hp = hp0 + hi;
        const ConvW dq = conv_w(w.ca_qw, w.ca_qb, tid & 31), dk = conv_w(w.ca_kw, w.ca_kb, tid & 31),
                    dv = conv_w(w.ca_vw, w.ca_vb, tid & 31);
        const int hh = tid >> 8, t2 = tid & 255, hd = 2 * hp + hh;
        unsigned char* at = att_ca + hh * PL::ATT_B;
        kvs.store(at, t2);
        if (hi < HP - 1) kvs.load(kvc_b + (size_t)(hd + 2) * KVC_ELEMS, t2);
        bar_lds();
        if (fixer) {
          fx.store<T, R>(at, dk, dv, Lk, lane);
          if (hi < HP - 1) fx.load(kvs_t, kvm_b, a.Ts, hd + 2, lane);
        }
        bar_lds();
        fattn_lds<R>(at, L, Lk, a.scale, Ob + hd * FDK, SX, t2, Yqb + hd * FDK, SX);
        bar_lds();
      }
      PSTAMP(3);
      // CA out-projection + residual
      {
        const float4 bo4[2] = {ld_f4(w.o_ca_b + (2 * wave) * 16 + 4 * g4), ld_f4(w.o_ca_b + (2 * wave + 1) * 16 + 4 * g4)};
        f32x4 acc[RT][2];
        zero_acc(acc);
        if constexpr (SPLITO) pmma<RT, 2, 4, 16, true, -1>(acc, Ob, SX, 4 * part, fa, lane);
        else pmma<RT, 2, 8, 16, true>(acc, Ob, SX, 0, fa, lane);
        {  // fa <- FFN-up chunk c0f (fb already holds FFN-down chunk c0f)
          const int tf[1] = {8 * c0f + wave};
          pload<1, 8>(fa, w.ff1, 8, tf, 0, lane);
        }
        LSTAMP(15);
        if constexpr (SPLITO)
          if (!pp_sum_partials<RT>(acc, part, xb, ep, flags, xl, a.status, &s_ok, wave, lane)) return;
        LSTAMP(16);
        p_resid_tr<RT>(Hs, acc, bo4, wave, c16, g4);
        bar_lds();
      }
      // ---------------- feed-forward block (nn.py:170-172) ----------------
      LSTAMP(11);
      {
        ln_rows<T, NT, R, SX>(Hs, L, Xn, tid);  // LN3 affine folded into the next Linear
        bar_lds();
      }
      LSTAMP(12);
      {
        const bool last = li + 1 == a.n_layers;
        const FusedLayer& wn = a.layers[last ? li : li + 1];
        f32x4 accd[RT][2];
        zero_acc(accd);
        for (int ci = 0; ci < NC; ++ci) {
          LANE_IDS();
          const int c = c0f + ci;
          const float4 bf4 = ld_f4(w.ff1_b + (8 * c + wave) * 16 + 4 * g4);
          f32x4 acc[RT][1];
          zero_acc(acc);
          pmma<RT, 1, 8, 16, true, -1>(acc, Xn, SX, 0, fa, lane);
          if (ci < NC - 1) {
            const int tf[1] = {8 * (c + 1) + wave};
            pload<1, 8>(fa, w.ff1, 8, tf, 0, lane);
          } else if (!last) {  // fa <- the next layer's first QKV pair
            const int tq[2] = {qoff + tq0, qoff + tq1};
            if (nq == 2) pload<2, 8>(fa, wn.qkv, 8, tq, 0, lane);
            else pload<1, 8>(fa, wn.qkv, 8, tq, 0, lane);
          } else {             // fa <- the output projection
            const int to[1] = {wave};
            pload<1, 8>(fa, a.w_out, 8, to, 0, lane);
          }
          // the chunk image is double-buffered: chunk c + 1 writes the other buffer, so no barrier
          // is needed behind the FFN-down MFMAs (the next chunk's barrier orders the reuse)
          T* Hc = Hd + (c & 1) * (PL::HID / sizeof(T));
          {  // row 16 rt + c16, chunk columns 16 w + 4 g4 .. + 3: one 8-byte store per row tile
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
              const float v0 = fmaxf(acc[rt][0][0] + bf4.x, 0.f), v1 = fmaxf(acc[rt][0][1] + bf4.y, 0.f);
              const float v2 = fmaxf(acc[rt][0][2] + bf4.z, 0.f), v3 = fmaxf(acc[rt][0][3] + bf4.w, 0.f);
              put_tok4<T, false>(Hc, SHD, rt * 16 + c16, wave * 16 + 4 * g4, f32x4{v0 * v0, v1 * v1, v2 * v2, v3 * v3});
            }
          }
          bar_lds();
          pmma<RT, 2, 4, 8, true, -1>(accd, Hc, SHD, 0, fb, lane);
          {
            const int td[2] = {2 * wave, 2 * wave + 1};
            if (ci < NC - 1)
              pload<2, 4>(fb, w.ff2, 32, td, 4 * (c + 1), lane);
            else if (!last)  // fb <- the next layer's first FFN-down chunk
              pload<2, 4>(fb, wn.ff2, 32, td, 4 * c0f, lane);
            else             // fb <- the next step's emb fragments
              pload<2, 4>(fb, a.w_emb, 4, td, 0, lane);
          }
        }
        static_assert(2 * PL::HID <= PL::SCR, "double-buffered FFN chunk image");
        LSTAMP(13);
        if constexpr (PAIR)  // FFN-down partials of the two halves of K
          if (!pp_sum_partials<RT>(accd, part, xb, ep, flags, xl, a.status, &s_ok, wave, lane)) return;
        LSTAMP(14);
        const float4 b24[2] = {ld_f4(w.ff2_b + (2 * wave) * 16 + 4 * g4), ld_f4(w.ff2_b + (2 * wave + 1) * 16 + 4 * g4)};
        p_resid_tr<RT>(Hs, accd, b24, wave, c16, g4);
        bar_lds();
      }
    }
    PSTAMP(4);
    // ---------------- out_layers + posterior update (nn.py:211-214,228; gaussian_diffusion.py) -------
    {
      ln_rows<T, NT, R, SX>(Hs, L, Xn, tid);  // out_layers.0 affine folded into out_layers.1
      bar_lds();
    }
    {
      const float bo = a.b_out[wave * 16 + c16];
      f32x4 acc[RT][1];
      zero_acc(acc);
      pmma<RT, 1, 8, 16, false, PSK_FENCE_OUT>(acc, Xn, SX, 0, fa, lane);
      {  // fa <- layer 0's first QKV pair (next step)
        const int tq[2] = {qoff + tq0, qoff + tq1};
        if (nq == 2) pload<2, 8>(fa, a.layers[0].qkv, 8, tq, 0, lane);
        else pload<1, 8>(fa, a.layers[0].qkv, 8, tq, 0, lane);
      }
      const int col = wave * 16 + c16;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int r = 0; r < 4; ++r) E[(rt * 16 + 4 * g4 + r) * SE + col] = acc[rt][0][r] + bo;
    }
    bar_lds();
    {
      const size_t plane = (size_t)a.n * LC;
      const float* nz = a.noise ? a.noise + (size_t)(a.k0 + k) * plane + (size_t)b * LC : nullptr;
      const bool inp = a.inp_mask != nullptr;
      const bool ex = a.extras != nullptr && k + 1 == a.n_steps && part == 0;
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const int q = tid + NT * j;
        if (4 * q >= LC) continue;
        float z[4];
        if (nz) {
#pragma unroll
          for (int u = 0; u < 4; ++u) z[u] = nz[min(4 * q + u, LC - 1)];
        } else {
          philox_normal4(a.seed, (uint32_t)(a.clip_offset + b), (uint32_t)rec.i, TAG_STEP, (uint32_t)q, z);
        }
        int cc = (4 * q) / L, l = 4 * q - cc * L;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = 4 * q + u;
          if (e < LC) {
            const float ev = E[l * SE + cc];
            const size_t gi = (row0 + l) * C + cc;
            const UpdOut o = upd_math(rec, a.alg, xr[j][u], ev, false, 0.f, inp, inp ? a.inp_mask[row0 + l] : 0.f,
                                      inp ? a.inp_pose[gi] : 0.f, inp ? a.trans[l] : 0.f, z[u]);
            xr[j][u] = o.xn;
            if (ex) {
              const size_t ncl = (size_t)b * LC + e;
              a.extras[0 * plane + ncl] = o.mean;
              a.extras[1 * plane + ncl] = rec.var;
              a.extras[2 * plane + ncl] = rec.logvar;
              a.extras[3 * plane + ncl] = ev;
              a.extras[4 * plane + ncl] = o.x0;
              a.extras[5 * plane + ncl] = o.raw;
            }
          }
          if (++l == L) { l = 0; ++cc; }
        }
      }
    }
    bar_lds();  // E is dead before the next step's Xb zero fill (same scratch)
    PSTAMP(5);
  }
  // final state -> the internal (L, C) layout (PAIR: both parts hold it; part 0 writes)
  if (part != 0) return;
  const int L = a.L, C = a.C, LC = L * C;
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int q = tid + NT * j;
    int cc = (4 * q) / L, l = 4 * q - cc * L;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (4 * q + u < LC) a.x[(row0 + l) * C + cc] = xr[j][u];
      if (++l == L) { l = 0; ++cc; }
    }
  }
}

static bool persist_attrs_done = false;

bool persist_supported(int dtype, int d_model, int heads, int L, int Ts, int C) {
  return dtype == 1 && d_model == FD && heads == FD / FDK && L >= 1 && L <= 48 && Ts >= 1 && 1 + Ts <= FLK &&
         C >= 1 && C <= 128;
}

static void persist_attrs() {
  if (persist_attrs_done) return;
#define GGD_PSK_ATTR(rt, pr) \
  (void)hipFuncSetAttribute((const void*)psk_kernel<rt, pr>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)
  GGD_PSK_ATTR(1, false); GGD_PSK_ATTR(2, false); GGD_PSK_ATTR(3, false);
  GGD_PSK_ATTR(1, true); GGD_PSK_ATTR(2, true); GGD_PSK_ATTR(3, true);
#undef GGD_PSK_ATTR
  (void)hipGetLastError();
  persist_attrs_done = true;
}

template <bool PAIR>
static hipError_t launch_psk(const PersistArgs& a, int P, dim3 grid, hipStream_t s) {
  const int rt = (a.L + 15) / 16;
  const dim3 blk(PK_THREADS);
  if (rt == 1) hipLaunchKernelGGL((psk_kernel<1, PAIR>), grid, blk, PPlan<1>::TOTAL, s, a, P);
  else if (rt == 2) hipLaunchKernelGGL((psk_kernel<2, PAIR>), grid, blk, PPlan<2>::TOTAL, s, a, P);
  else if (rt == 3) hipLaunchKernelGGL((psk_kernel<3, PAIR>), grid, blk, PPlan<3>::TOTAL, s, a, P);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_persist(const PersistArgs& a, hipStream_t s) {
  persist_attrs();
  PersistArgs b = a;
  b.clip0 = 0;
  return launch_psk<false>(b, b.n, dim3(b.n), s);
}

hipError_t launch_persist_range(const PersistArgs& a, int clips, hipStream_t s) {
  if (clips < 1 || a.clip0 < 0 || a.clip0 + clips > a.n) return hipErrorInvalidValue;
  persist_attrs();
  return launch_psk<false>(a, clips, dim3(clips), s);
}

// pairs per launch: the grid (16 workgroups per 8 pairs, one per CU) must be co-resident
int persist_pair_capacity() {
  static int cap = -1;
  if (cap < 0) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipGetLastError();
    cap = std::min(PAIR_MAX, 8 * (cus / 16));
  }
  return cap;
}

hipError_t launch_persist_pair(const PersistArgs& a, int pairs, hipStream_t s) {
  if (pairs < 1 || pairs > persist_pair_capacity() || !a.ctl || !a.status || !a.xbuf) return hipErrorInvalidValue;
  persist_attrs();
  hipError_t e = hipMemsetAsync(a.ctl, 0, sizeof(unsigned) * PAIR_CTL_WORDS, s);
  if (e != hipSuccess) return e;
  return launch_psk<true>(a, pairs, dim3(16 * ((pairs + 7) / 8)), s);
}

}  // namespace ggd
