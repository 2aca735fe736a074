// ggd_api.hip -- host side of libggd: the C ABI declared in include/ggd.h.
//
// Owns: weights in the compute dtype (uploaded once), the step-token tables for every
// original t, the per-clip cross-attention K/V cache, activation workspaces sized for
// desc.max_batch, the schedule's per-iteration coefficient records, and the captured
// per-step hipGraph.  One denoise step is the launch chain of launch_step():
//   emb_x(+PE) | n_layers x [LN1+QKV | attn(self) | out+res | LN2+Qca | attn(cross) | out+res |
//   LN3+FFN1+ReLU^2 | FFN2+res] | LNout+out | diffusion update
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ggd.h"
#include "ggd_kernels.h"

using namespace ggd;

namespace {

struct Lin {            // packed Linear: T [npad][kpad] (or e4m3 bytes + scale), f32 bias [npad]
  void* w = nullptr;
  float* b = nullptr;
  float* scale = nullptr;  // GGD_FP8W per-step Linears: per-output-channel dequantization scale
  void* wf = nullptr;      // row-block chain route: fragment-packed copy of w (ggd_chain.hip)
  void* wmx = nullptr;     // GGD_FP8W long loop: e4m3 copy in the block-scaled fp8 MFMA's B order
  int n = 0, k = 0, npad = 0, kpad = 0;
};

struct Conv3 {          // depthwise 3-tap: f32 [dk][3] + [dk]
  float* w = nullptr;
  float* b = nullptr;
};

struct FLin {           // MFMA B-fragment packed Linear: T [tiles][k steps][64 lanes][16 B], f32 bias
  void* w = nullptr;
  float* b = nullptr;
};

struct Layer {
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b, *ln3_g, *ln3_b;
  Lin qkv, o_sa, q_ca, kv_ca, o_ca, ff1, ff2;
  Conv3 sa_q, sa_k, sa_v, ca_q, ca_k, ca_v;
  FLin f_qkv, f_o_sa, f_q_ca, f_o_ca, f_ff1, f_ff2;  // fused-path copies
};

// two-way decoder layer (CrossAttentionLayer, models/nn.py:55-125)
struct Layer2 {
  float *ln_sa_g, *ln_sa_b, *ln_sam_g, *ln_sam_b, *ln_ca_g, *ln_ca_b, *ln_ff_g, *ln_ff_b;
  float *ln_ffm_g = nullptr, *ln_ffm_b = nullptr;
  Lin qkv_sa, o_sa, qkv_sam, o_sam, qkv_ca, o_ca, ff1, ff2, ffm1, ffm2;
  Conv3 sa_q, sa_k, sa_v, sam_q, sam_k, sam_v, ca_q, ca_k, ca_v;
  bool has_ffm = false;  // every layer but the last feed-forwards the memory (nn.py:408-418)
};

struct ProfEvents {
  std::vector<hipEvent_t> ev;  // timing events; eager marks consume ev[next++]
  size_t next = 0;
};

}  // namespace

struct ggd_ctx {
  int device = 0;
  ggd_desc desc{};
  std::string err;
  hipStream_t stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  size_t tsize = 4;  // bytes per compute-dtype element

  std::map<std::string, std::vector<float>> staged;
  bool finalized = false;
  std::vector<void*> allocs;

  // weights
  Lin emb_x, emb_mem, out_lin, step0, step2, blend;
  Lin inp0, inp2, inp4;      // Speech2GestureModelInpaint.proj (model.py:135-142)
  float *inp_in = nullptr, *inp_h1 = nullptr, *inp_h2 = nullptr, *inp_delta = nullptr;
  bool inp_on = false;       // ggd_set_inpaint installed a projection
  FLin f_emb, f_out;
  bool fused = false;        // per-clip fused kernels (L <= 64, d_model 256, 8 heads)
  bool persist = false;      // persistent per-clip sampler (bf16, L <= 48): ggd_sample runs it
  FusedLayer* d_layers = nullptr;  // device copy of every layer's FusedLayer (persistent kernel)
  void* arena = nullptr;     // current device arena (dalloc) and its fill level
  size_t arena_off = 0;
  int persist_mode = 0;      // ggd_diag what=7: 0 auto, 1 never, 2 always the one-workgroup-per-clip loop.
                             // Auto: when the clip-group loop would need >= 3 chunks (measured on MI355X,
                             // scripts/route_compare.py: 314 us/step for any n <= 256 vs 113 us per
                             // 32-clip chunk)
  unsigned long long* stamps = nullptr;  // ggd_diag what=8: phase stamps of the persistent kernel
  int pair_mode = 0;         // ggd_diag what=14: 0 auto, 1 never, 2 always two workgroups per clip
  unsigned* pair_ctl = nullptr;           // clip-pair loop: control words, status, hand-off slots
  int* pair_status = nullptr;
  unsigned char* pair_xbuf = nullptr;
  int pair_launches = 0;                  // last ggd_sample: clip-pair launches (0: one workgroup per clip)
  int pair_force_coh = 0;                 // ggd_diag what=14 p[1]: write-through hand-offs on any placement
  float *out_ln_g = nullptr, *out_ln_b = nullptr;
  std::vector<Layer> layers;
  float* pe = nullptr;       // [pe_len][d]
  int pe_len = 0;
  float* kv_step = nullptr;  // [layers][T_orig][2d]
  float* zero_row = nullptr; // 1 KiB of zeros: the attention conv's padding rows

  // row-block chains (ggd_chain.hip): the one-way generic route's GEMMs, 4 launches per layer
  bool chain = false;        // fragment-packed weights built (one-way, not fused, bf16 / fp8, d 256, FFN 1024)
  int gemm_launches = 0;     // GGD_ROUTE_GEMM_LAUNCHES: 1 = one launch per GEMM instead
  int attn_qsplit = 0;       // GGD_ROUTE_ATTN_QSPLIT: 1 = long clips on the query-split attention
  long clip_attn_launches = 0;  // GGD_INFO_CLIP_ATTN_LAUNCHES: whole-clip attention launches (running count)
  // long-clip persistent loop (ggd_long.hip): every step of clips of >= 96 frames in one launch
  bool long_ok = false;      // the shape and dtype have a long-loop instance (needs the chain weights)
  int long_off = 0;          // GGD_ROUTE_LONG_LOOP: 1 = never
  int fp8_mfma_off = 0;      // GGD_ROUTE_FP8_MFMA: 1 = the long loop's fp8 weights widened into bf16 MFMAs
  ChainStage* long_stages_mx = nullptr;  // the stage table with the F1 / F2 / P / P2 weights' MX copies
  LongLayer* long_layers = nullptr;
  bf16_t* long_kvc = nullptr;  // [layers][max_batch] convolved memory K / V^T (ggd_set_memory)
  ChainStage* long_stages = nullptr;
  unsigned* long_ctl = nullptr;
  int* long_status = nullptr;
  int long_launches = 0, long_fallbacks = 0;  // last ggd_sample
  unsigned long long* long_stamps = nullptr;  // ggd_diag what = 16

  // two-way decoder (generic kernels, joint layout [n][J = L + 1 + Ts][d])
  bool twoway = false;
  int J = 0;
  std::vector<Layer2> layers2;
  float *hj = nullptr, *mem_base = nullptr, *step_tab = nullptr;
  void *qkvj = nullptr, *attj = nullptr, *zbuf = nullptr, *ffnj = nullptr;

  // schedule
  std::vector<double> betas;
  std::vector<int> tmap;
  StepRec* d_steps = nullptr;
  int steps_cap = 0;
  int n_steps_T = 0;

  // memory
  float* kv_mem = nullptr;   // [layers][maxB*Ts][2d]
  void* kvc = nullptr;       // fused paths: [layers][maxB][heads][KVC_ELEMS] T, convolved step-invariant K | V^T
  float* ffp = nullptr;      // fused paths: FFN-down partial sums per hidden chunk [maxB][8][L][d]
  float* mem_tmp = nullptr;  // [maxB*Ts][d]
  float* tok_tmp = nullptr;  // [maxB*Ts][d]
  int mem_n = -1;

  // workspaces
  float *x = nullptr, *h = nullptr, *h2 = nullptr, *eps = nullptr;
  void *qkv = nullptr, *att = nullptr, *q = nullptr, *ffn = nullptr;
  int* d_counter = nullptr;  // iteration counter k
  int* d_t = nullptr;        // per-clip t (denoise path)
  int cpad = 0;

  // graph
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  std::string graph_key;

  // profiling
  bool profiling = false;
  ProfEvents prof;
  double prof_avg_us = 0;
  int64_t prof_launches = 0;
  unsigned long long* span = nullptr;  // fused path: KB stamps [T * n_layers][2][workgroups] (realtime ticks)
  size_t span_cap = 0;                 // allocated stamps
  size_t span_pending = 0, span_wg = 0;  // stamps written by the last profiled ggd_sample
  int prof_kind = 0;                   // what the last profiled ggd_sample timed: 0 kb_kernel, 1 mk_kernel,
                                       // 2 the generic path's FFN-up GEMM (LN prologue, ReLU^2 epilogue)

  // persistent reverse loop (ggd_mega.hip)
  bool no_mega = false;                // ggd_diag what = 9: route sampling through per-phase launches
  int mega_place = 0;                  // ggd_diag what = 12: 0 XCD-local, 1 part per XCD, 2 group per XCD
  bool mega_rows_last = false;         // the last clip-group loop issued was the row-block loop (bf16)
  FusedArgs* mega_fa = nullptr;        // device [n_layers][4]
  unsigned long long* mega_phase_stamps = nullptr;  // ggd_diag what = 11: layer 1's phases + KE
  FinalArgs* mega_fe = nullptr;
  unsigned* mega_ctl = nullptr;
  int* mega_status = nullptr;
  unsigned long long* mega_stamps = nullptr;  // ggd_diag what = 10
  std::vector<FusedArgs> mega_fa_host;
  FinalArgs mega_fe_host{};
  int mega_status_host = 0;
  int mega_xl_launches = 0, mega_fallbacks = 0;  // last ggd_sample: XCD-local launches, chunks re-run elsewhere
  int64_t barrier_timeouts = 0;        // running count of loop chunks / batches whose status word carried a timeout
  double wall_mhz = 100.0;             // realtime counter rate (hipDeviceAttributeWallClockRate)

  // Deferred status checks of the persistent loops: a ggd_sample that does not ask for `sync`
  // returns once its launches are issued; the loop's status words are copied to pinned host memory
  // behind it and an event marks their arrival.  Later calls (and ggd_sync) read them; a failure
  // becomes a sticky error returned by the next call.
  struct Pending {
    hipEvent_t ev = nullptr;
    int* host = nullptr;     // pinned: [2 * MEGA_MAX_CHUNKS] status words
    int kind = 0;            // 1 clip-group loop (XCD-local words, then the gated write-through re-runs), 4 clip pairs
    int chunks = 0;
    bool xl = false;
    bool fb = false;         // a device-gated fallback launch stands behind the loop (status 2 is then no error)
  };
  std::vector<Pending> pend;           // ring
  size_t pend_head = 0, pend_count = 0;
  int sticky = 0;                      // 0, or the ggd_status of a failed earlier loop
  std::string sticky_msg;
  bool mega_none_ran = false;          // settled clip-group check: every chunk reported 2 (nothing ran)
  int gated_ran = 0;                   // settled check: chunks the device-gated fallback loop ran instead
  int sim_unresident = 0;              // GGD_ROUTE_SIMULATE_UNRESIDENT

  // Per-call uploads (step records, the loop's argument blocks): from pageable memory a small
  // hipMemcpyAsync is staged by the runtime in pieces (several blit kernels and host waits per
  // call); here they go through pinned slots, one DMA each, and are skipped when the device copy
  // already holds the same bytes.
  struct Upload {
    void* dev = nullptr;               // destination (the last bytes uploaded there are `last`)
    std::vector<unsigned char> last;
    unsigned char* slot[2] = {nullptr, nullptr};  // pinned staging, alternating
    hipEvent_t ev[2] = {nullptr, nullptr};        // the copy out of each slot has completed
    size_t cap = 0;
    int next = 0;
  };
  std::map<const void*, Upload> uploads;
  bool prof_lazy = false;              // profiled loop: elapsed time read by ggd_kernel_time
  int prof_lazy_div = 1;
};

namespace {

// clip-pair step time / one-workgroup-per-clip step time (ggd_persist.hip), measured on MI355X
constexpr double PAIR_STEP_RATIO = 0.68;  // 172 / 253 us per DDIM step at 128 clips (r02b)

int fail(ggd_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_TRY(ctx, expr)                                                                  \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return fail(ctx, GGD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));     \
  } while (0)

constexpr size_t PEND_RING = 8;

// Read the status words of a finished deferred check (see ggd_ctx::Pending).
void settle(ggd_ctx* c, const ggd_ctx::Pending& p) {
  c->gated_ran = 0;
  if (p.kind == 1) {
    int worst = 0, unrun = 0;
    c->mega_xl_launches = 0;
    c->mega_fallbacks = 0;
    for (int ci = 0; ci < p.chunks; ++ci) {
      int st = p.host[ci];
      bool fell_back = false;  // a chunk counts once in mega_fallbacks, however many re-runs it took
      if (p.xl && st == 3) {   // the gated write-through launch ran instead
        fell_back = true;
        st = p.host[MEGA_MAX_CHUNKS + ci];
      } else if (p.xl) {
        ++c->mega_xl_launches;
      }
      if (st == 2 && p.fb) {  // never all resident: the gated one-workgroup-per-clip loop ran the chunk
        fell_back = true;
        ++c->gated_ran;
        st = 0;
      }
      if (st & STATUS_TIMEOUT) ++c->barrier_timeouts;
      c->mega_fallbacks += fell_back ? 1 : 0;
      worst = std::max(worst, st);
      unrun += st == 2 ? 1 : 0;
    }
    c->mega_none_ran = unrun == p.chunks;
    c->mega_status_host = worst;
    if (worst && !c->sticky) {
      c->sticky = GGD_ERR_HIP;
      c->sticky_msg = worst == 2 ? "persistent loop (earlier ggd_sample): workgroups were not all resident"
                      : (worst & STATUS_TIMEOUT) || worst == 1 ? "persistent loop (earlier ggd_sample): a clip-group barrier timed out"
                                                               : "persistent loop (earlier ggd_sample): failed (status " +
                                                                     std::to_string(worst) + ")";
    }
  } else if (p.kind == 4) {
    if (p.host[0] & STATUS_TIMEOUT) ++c->barrier_timeouts;
    if (p.host[0] == 2 && p.fb) {
      c->gated_ran = 1;
      c->pair_launches = 0;   // the pair launches ran nothing: the gated fallback ran the batch
    }
    if (p.host[0] && !(p.host[0] == 2 && p.fb) && !c->sticky) {
      c->sticky = GGD_ERR_HIP;
      c->sticky_msg = p.host[0] == 2 ? "clip-pair loop (earlier ggd_sample): workgroups were not all resident"
                                     : "clip-pair loop (earlier ggd_sample): a pair barrier timed out";
    }
  }
}

// Settle every deferred check whose copy has landed (wait = true: all of them, blocking).
int poll_pending(ggd_ctx* c, bool wait) {
  while (c->pend_count) {
    ggd_ctx::Pending& p = c->pend[c->pend_head];
    if (wait) {
      HIP_TRY(c, hipEventSynchronize(p.ev));
    } else {
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) return fail(c, GGD_ERR_HIP, std::string("status event: ") + hipGetErrorString(q));
    }
    settle(c, p);
    c->pend_head = (c->pend_head + 1) % PEND_RING;
    --c->pend_count;
  }
  return GGD_OK;
}

// Settle every deferred check except the newest (blocking): the checks of earlier calls.
int poll_pending_before_last(ggd_ctx* c) {
  while (c->pend_count > 1) {
    ggd_ctx::Pending& p = c->pend[c->pend_head];
    HIP_TRY(c, hipEventSynchronize(p.ev));
    settle(c, p);
    c->pend_head = (c->pend_head + 1) % PEND_RING;
    --c->pend_count;
  }
  return GGD_OK;
}

// Queue a deferred check of `nwords` device status words (stream-ordered behind the loop).
int defer_check(ggd_ctx* c, const int* dev_words, int nwords, int kind, int chunks, bool xl, bool fb, hipStream_t s) {
  if (c->pend.empty()) {
    c->pend.resize(PEND_RING);
    for (auto& p : c->pend) {
      HIP_TRY(c, hipEventCreateWithFlags(&p.ev, hipEventDisableTiming));
      HIP_TRY(c, hipHostMalloc((void**)&p.host, sizeof(int) * 2 * MEGA_MAX_CHUNKS, hipHostMallocDefault));
    }
  }
  if (c->pend_count == PEND_RING) {  // ring full: the oldest check must settle first
    ggd_ctx::Pending& o = c->pend[c->pend_head];
    HIP_TRY(c, hipEventSynchronize(o.ev));
    settle(c, o);
    c->pend_head = (c->pend_head + 1) % PEND_RING;
    --c->pend_count;
  }
  ggd_ctx::Pending& p = c->pend[(c->pend_head + c->pend_count) % PEND_RING];
  p.kind = kind;
  p.chunks = chunks;
  p.xl = xl;
  p.fb = fb;
  HIP_TRY(c, hipMemcpyAsync(p.host, dev_words, sizeof(int) * nwords, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipEventRecord(p.ev, s));
  ++c->pend_count;
  return GGD_OK;
}

// hipMemcpyAsync(dev, host, bytes) through a pinned slot, skipped when `dev` already holds these
// bytes from an earlier upload_cached (stream-ordered: a change is copied behind the kernels that
// read the old contents).
int upload_cached(ggd_ctx* c, void* dev, const void* host, size_t bytes, hipStream_t s) {
  ggd_ctx::Upload& u = c->uploads[dev];
  if (u.last.size() == bytes && std::memcmp(u.last.data(), host, bytes) == 0) return GGD_OK;
  if (u.cap < bytes) {
    for (int i = 0; i < 2; ++i) {
      if (u.ev[i]) HIP_TRY(c, hipEventSynchronize(u.ev[i]));
      if (u.slot[i]) HIP_TRY(c, hipHostFree(u.slot[i]));
      HIP_TRY(c, hipHostMalloc((void**)&u.slot[i], bytes, hipHostMallocDefault));
      if (!u.ev[i]) HIP_TRY(c, hipEventCreateWithFlags(&u.ev[i], hipEventDisableTiming));
    }
    u.cap = bytes;
  }
  const int i = u.next;
  u.next ^= 1;
  HIP_TRY(c, hipEventSynchronize(u.ev[i]));   // the copy out of this slot (two calls ago) is done
  std::memcpy(u.slot[i], host, bytes);
  HIP_TRY(c, hipMemcpyAsync(dev, u.slot[i], bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(c, hipEventRecord(u.ev[i], s));
  u.dev = dev;
  u.last.assign((const unsigned char*)host, (const unsigned char*)host + bytes);
  return GGD_OK;
}

// A device buffer written by other means than upload_cached: forget what it held.
void upload_forget(ggd_ctx* c, const void* dev) {
  auto it = c->uploads.find(dev);
  if (it != c->uploads.end()) it->second.last.clear();
}

// The sticky error of an earlier deferred check, reported once.
int take_sticky(ggd_ctx* c) {
  if (!c->sticky) return GGD_OK;
  const int r = fail(c, c->sticky, c->sticky_msg);
  c->sticky = 0;
  c->sticky_msg.clear();
  return r;
}

// Device memory of a context: sub-allocated (256-B aligned) from a few 64 MiB arenas, so the
// weights, tables and workspaces that every step streams sit in a handful of large, physically
// contiguous mappings instead of dozens of small ones (fewer translation misses per weight stream).
template <typename P>
hipError_t dalloc(ggd_ctx* c, P** p, size_t bytes) {
  constexpr size_t ARENA = 64ull << 20, ALIGN = 256;
  bytes = bytes < 16 ? 16 : bytes;
  void* v = nullptr;
  if (bytes > ARENA / 4) {
    hipError_t e = hipMalloc(&v, bytes);
    if (e != hipSuccess) return e;
    c->allocs.push_back(v);
  } else {
    if (!c->arena || c->arena_off + bytes > ARENA) {
      hipError_t e = hipMalloc(&c->arena, ARENA);
      if (e != hipSuccess) return e;
      c->allocs.push_back(c->arena);
      c->arena_off = 0;
    }
    v = (char*)c->arena + c->arena_off;
    c->arena_off = (c->arena_off + bytes + ALIGN - 1) & ~(ALIGN - 1);
  }
  hipError_t e = hipMemset(v, 0, bytes);
  *p = (P*)v;
  return e;
}

uint16_t f2bf_host(float f) {  // round to nearest even, NaN preserved
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

// float -> OCP fp8 e4m3fn (bias 7, max 448, no infinities), round to nearest even, saturating.
// Restated in oracle/fp8.py (the parity tests quantize the oracle's weights with it).
uint8_t f2e4m3_host(float f) {
  if (std::isnan(f)) return 0x7f;
  const uint8_t sign = std::signbit(f) ? 0x80 : 0;
  float a = std::fabs(f);
  if (a >= 448.f) return sign | 0x7e;
  if (a < std::ldexp(1.f, -6)) {                       // subnormal: steps of 2^-9
    const int m = (int)std::nearbyint(std::ldexp(a, 9));  // 0 .. 8 (8 = smallest normal)
    return sign | (uint8_t)m;
  }
  int e;
  const float fr = std::frexp(a, &e);                   // a = fr * 2^e, fr in [0.5, 1)
  int m = (int)std::nearbyint((fr * 2.f - 1.f) * 8.f);  // 3 mantissa bits of 1.m * 2^(e-1)
  int ex = e - 1;
  if (m == 8) { m = 0; ++ex; }
  if (ex > 8 || (ex == 8 && m > 6)) return sign | 0x7e;
  return sign | (uint8_t)(((ex + 7) << 3) | m);
}


const std::vector<float>* get(ggd_ctx* c, const std::string& name, size_t numel) {
  auto it = c->staged.find(name);
  if (it == c->staged.end()) {
    c->err = "missing weight: " + name;
    return nullptr;
  }
  if (numel && it->second.size() != numel) {
    c->err = "weight " + name + " has " + std::to_string(it->second.size()) + " elements, expected " +
             std::to_string(numel);
    return nullptr;
  }
  return &it->second;
}

// Pack one or more torch Linear weights (rows stacked) into T [npad][kpad].  `step`: the Linear
// runs inside every denoise step, so a GGD_FP8W context stores it as e4m3 rows with one scale
// per output channel (amax / 448; all-zero rows scale 1).
int pack_lin(ggd_ctx* c, Lin& L, const std::vector<std::string>& prefixes, int n_each, int k, bool step = false) {
  const int n = n_each * (int)prefixes.size();
  L.n = n;
  L.k = k;
  L.npad = round_up(n, 64);
  L.kpad = round_up(k, 256);
  std::vector<float> w((size_t)L.npad * L.kpad, 0.f), b(L.npad, 0.f);
  for (size_t p = 0; p < prefixes.size(); ++p) {
    const auto* W = get(c, prefixes[p] + ".weight", (size_t)n_each * k);
    const auto* B = get(c, prefixes[p] + ".bias", (size_t)n_each);
    if (!W || !B) return GGD_ERR_NAME;
    for (int r = 0; r < n_each; ++r) {
      std::memcpy(&w[(size_t)(p * n_each + r) * L.kpad], &(*W)[(size_t)r * k], sizeof(float) * k);
      b[p * n_each + r] = (*B)[r];
    }
  }
  HIP_TRY(c, dalloc(c, &L.b, sizeof(float) * L.npad));
  HIP_TRY(c, hipMemcpy(L.b, b.data(), sizeof(float) * L.npad, hipMemcpyHostToDevice));
  if (step && c->desc.dtype == GGD_FP8W) {
    std::vector<uint8_t> q(w.size());
    std::vector<float> sc(L.npad, 1.f);
    for (int r = 0; r < L.npad; ++r) {
      const float* row = &w[(size_t)r * L.kpad];
      float amax = 0.f;
      for (int j = 0; j < L.kpad; ++j) amax = std::max(amax, std::fabs(row[j]));
      if (amax > 0.f) sc[r] = amax / 448.f;
      for (int j = 0; j < L.kpad; ++j) q[(size_t)r * L.kpad + j] = f2e4m3_host(row[j] / sc[r]);
    }
    HIP_TRY(c, dalloc(c, &L.scale, sizeof(float) * L.npad));
    HIP_TRY(c, hipMemcpy(L.scale, sc.data(), sizeof(float) * L.npad, hipMemcpyHostToDevice));
    HIP_TRY(c, dalloc(c, &L.w, q.size()));
    HIP_TRY(c, hipMemcpy(L.w, q.data(), q.size(), hipMemcpyHostToDevice));
    return GGD_OK;
  }
  HIP_TRY(c, dalloc(c, &L.w, c->tsize * w.size()));
  if (c->desc.dtype == GGD_F32) {
    HIP_TRY(c, hipMemcpy(L.w, w.data(), sizeof(float) * w.size(), hipMemcpyHostToDevice));
  } else {
    std::vector<uint16_t> wb(w.size());
    for (size_t i = 0; i < w.size(); ++i) wb[i] = f2bf_host(w[i]);
    HIP_TRY(c, hipMemcpy(L.w, wb.data(), 2 * wb.size(), hipMemcpyHostToDevice));
  }
  return GGD_OK;
}

int upload_vec(ggd_ctx* c, float** dst, const std::string& name, size_t numel) {
  const auto* v = get(c, name, numel);
  if (!v) return GGD_ERR_NAME;
  HIP_TRY(c, dalloc(c, dst, sizeof(float) * numel));
  HIP_TRY(c, hipMemcpy(*dst, v->data(), sizeof(float) * numel, hipMemcpyHostToDevice));
  return GGD_OK;
}

int pack_conv(ggd_ctx* c, Conv3& cv, const std::string& prefix, int dk) {
  int r = upload_vec(c, &cv.w, prefix + ".conv.weight", (size_t)dk * 3);
  if (r) return r;
  return upload_vec(c, &cv.b, prefix + ".conv.bias", (size_t)dk);
}

// Pack the rows `perm` of a row-major f32 matrix W (k columns) into MFMA B fragments:
// fragment (tile nt, k step kf), lane l, element e holds W[perm[nt*16 + (l & 15)]][kf*KF + (l >> 4)*EPL + e]
// with KF = 64 / sizeof(T) and EPL = 16 / sizeof(T); out-of-range rows / columns are zero.
int pack_frag(ggd_ctx* c, FLin& F, const std::vector<const float*>& rows_w, const std::vector<float>& bias, int k) {
  const int n = (int)rows_w.size();
  const int tsz = (int)c->tsize, KF = 64 / tsz, EPL = 16 / tsz;
  const int ntiles = (n + 15) / 16, kpad = round_up(k, KF), KT = kpad / KF;
  std::vector<float> buf((size_t)ntiles * KT * 64 * EPL, 0.f), b((size_t)ntiles * 16, 0.f);
  for (int nt = 0; nt < ntiles; ++nt)
    for (int kf = 0; kf < KT; ++kf)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < EPL; ++e) {
          const int row = nt * 16 + (l & 15), kk = kf * KF + (l >> 4) * EPL + e;
          if (row < n && kk < k)
            buf[(((size_t)nt * KT + kf) * 64 + l) * EPL + e] = rows_w[row][kk];
        }
  for (int r = 0; r < n; ++r) b[r] = bias[r];
  HIP_TRY(c, dalloc(c, &F.b, sizeof(float) * b.size()));
  HIP_TRY(c, hipMemcpy(F.b, b.data(), sizeof(float) * b.size(), hipMemcpyHostToDevice));
  HIP_TRY(c, dalloc(c, &F.w, c->tsize * buf.size()));
  if (c->desc.dtype == GGD_F32) {
    HIP_TRY(c, hipMemcpy(F.w, buf.data(), sizeof(float) * buf.size(), hipMemcpyHostToDevice));
  } else {
    std::vector<uint16_t> wb(buf.size());
    for (size_t i = 0; i < buf.size(); ++i) wb[i] = f2bf_host(buf[i]);
    HIP_TRY(c, hipMemcpy(F.w, wb.data(), 2 * wb.size(), hipMemcpyHostToDevice));
  }
  return GGD_OK;
}

// rows of the named Linear(s) in the given order; `order` indexes the concatenated rows.
// ln: the LayerNorm in front of this Linear (nn.LayerNorm([d]) of models/nn.py:141-147,212),
// folded in: LN(x) W^T + b = xhat (W diag(gamma))^T + (b + W beta), xhat = (x - mu) / sigma,
// so the fused kernels write the bare normalised rows (no per-column affine).  Folded in f64.
int frag_from(ggd_ctx* c, FLin& F, const std::vector<std::string>& prefixes, int n_each, int k,
              const std::vector<int>& order, const std::string& ln = "") {
  std::vector<const float*> rw;
  std::vector<float> bias;
  std::vector<const std::vector<float>*> W, B;
  for (const auto& p : prefixes) {
    const auto* w = get(c, p + ".weight", (size_t)n_each * k);
    const auto* b = get(c, p + ".bias", (size_t)n_each);
    if (!w || !b) return GGD_ERR_NAME;
    W.push_back(w);
    B.push_back(b);
  }
  const std::vector<float>* g = nullptr;
  const std::vector<float>* be = nullptr;
  if (!ln.empty()) {
    g = get(c, ln + ".weight", (size_t)k);
    be = get(c, ln + ".bias", (size_t)k);
    if (!g || !be) return GGD_ERR_NAME;
  }
  std::vector<std::vector<float>> folded(g ? order.size() : 0);
  for (size_t oi = 0; oi < order.size(); ++oi) {
    const int r = order[oi], p = r / n_each, i = r % n_each;
    const float* row = W[p]->data() + (size_t)i * k;
    float bv = (*B[p])[i];
    if (g) {
      std::vector<float>& fr = folded[oi];
      fr.resize(k);
      double acc = (double)bv;
      for (int kk = 0; kk < k; ++kk) {
        fr[kk] = row[kk] * (*g)[kk];
        acc += (double)row[kk] * (double)(*be)[kk];
      }
      row = fr.data();
      bv = (float)acc;
    }
    rw.push_back(row);
    bias.push_back(bv);
  }
  return pack_frag(c, F, rw, bias, k);
}

std::vector<int> iota_n(int n) {
  std::vector<int> v(n);
  for (int i = 0; i < n; ++i) v[i] = i;
  return v;
}

GemmArgs gemm_args(const Lin& L, int M, const void* A, int lda, void* out, int ldo) {
  GemmArgs g{};
  g.M = M;
  g.N = L.npad;
  g.K = L.kpad;
  g.k_valid = L.k;
  g.A = A;
  g.lda = lda;
  g.W = L.w;
  g.bias = L.b;
  g.out = out;
  g.ldo = ldo;
  g.n_valid = L.n;
  g.wscale = L.scale;
  return g;
}

#define GEMM(ctx, pro, epi, args, s)                                                          \
  do {                                                                                        \
    hipError_t _e = launch_gemm((ctx)->desc.dtype, pro, epi, args, s);                        \
    if (_e != hipSuccess) return fail(ctx, GGD_ERR_HIP, std::string("gemm launch: ") + hipGetErrorString(_e)); \
  } while (0)

// Positional-encoding table (transformer.py:157-166), f32 like the reference.
void build_pe(std::vector<float>& pe, int len, int d) {
  pe.assign((size_t)len * d, 0.f);
  const float lg = (float)(-(std::log(10000.0) / d));
  for (int p = 0; p < len; ++p)
    for (int i = 0; i < d; i += 2) {
      const float div = std::exp((float)i * lg);
      const float arg = (float)p * div;
      pe[(size_t)p * d + i] = std::sin(arg);
      if (i + 1 < d) pe[(size_t)p * d + i + 1] = std::cos(arg);
    }
}

// Step-token tables: for every original t, memory row 0 (step MLP -> emb_mem + PE[0]) and its
// cross-attention K|V pre-conv projection per layer.  nn.py:38-52, nn.py:223, nn.py:166.
int build_step_tables(ggd_ctx* c) {
  const int T = c->desc.diffusion_steps, d = c->desc.d_model;
  hipStream_t s = c->stream;
  float *emb, *hid, *tok, *mem0;
  HIP_TRY(c, hipMalloc(&emb, sizeof(float) * T * d));
  HIP_TRY(c, hipMalloc(&hid, sizeof(float) * T * d));
  HIP_TRY(c, hipMalloc(&tok, sizeof(float) * T * d));
  HIP_TRY(c, hipMalloc(&mem0, sizeof(float) * T * d));
  HIP_TRY(c, launch_step_embed(emb, T, d, s));
  GemmArgs g = gemm_args(c->step0, T, emb, d, hid, d);
  GEMM(c, PRO_F32, EPI_SILU, g, s);
  g = gemm_args(c->step2, T, hid, d, tok, d);
  GEMM(c, PRO_F32, EPI_F32, g, s);
  // memory row 0 sits at position 0 of the memory stream (one-way, nn.py:223) or at position
  // L of the joint sequence (two-way, nn.py:438-442)
  g = gemm_args(c->emb_mem, T, tok, d, c->twoway ? c->step_tab : mem0, d);
  g.pe = c->pe;
  g.pe_period = 1;
  g.pe_offset = c->twoway ? c->desc.seq_len : 0;
  GEMM(c, PRO_F32, EPI_PE, g, s);
  for (int l = 0; l < (c->twoway ? 0 : c->desc.n_layers); ++l) {
    g = gemm_args(c->layers[l].kv_ca, T, mem0, d, c->kv_step + (size_t)l * T * 2 * d, 2 * d);
    GEMM(c, PRO_F32, EPI_F32, g, s);
  }
  HIP_TRY(c, hipStreamSynchronize(s));
  hipFree(emb);
  hipFree(hid);
  hipFree(tok);
  hipFree(mem0);
  return GGD_OK;
}

// Timing mark around the dominant kernel (profiling mode runs the loop eagerly; marks pair up
// as start / end of consecutive launches of that kernel).
int prof_mark(ggd_ctx* c, hipStream_t s) {
  while (c->prof.ev.size() <= c->prof.next) {
    hipEvent_t n;
    HIP_TRY(c, hipEventCreate(&n));
    c->prof.ev.push_back(n);
  }
  HIP_TRY(c, hipEventRecord(c->prof.ev[c->prof.next++], s));
  return GGD_OK;
}

FinalArgs final_args(ggd_ctx* c, int n) {
  FinalArgs f{};
  f.n = n;
  f.L = c->desc.seq_len;
  f.C = c->desc.d_pose;
  f.h = c->h;
  f.ln_g = c->out_ln_g;
  f.ln_b = c->out_ln_b;
  f.w_out = c->f_out.w;
  f.b_out = c->f_out.b;
  f.w_emb = c->f_emb.w;
  f.b_emb = c->f_emb.b;
  f.pe = c->pe;
  f.x = c->x;
  f.steps = c->d_steps;
  f.step_counter = c->d_counter;
  f.extras_k = -1;
  return f;
}

// Fused decoder layers (ggd_fused.hip) on h (= emb_x(x) + PE, already in c->h): per layer
// KA, KB, KC and the FFN-down GEMM.  Residual rows ping-pong h -> h2 -> h so that no
// workgroup overwrites rows a sibling workgroup of the same clip still reads.
// The fused kernels' view of layer li: fragment-packed weights, LN / conv parameters and the
// step-invariant memory K/V tables.
FusedLayer fused_layer(ggd_ctx* c, int li) {
  const ggd_desc& D = c->desc;
  const int d = D.d_model;
  const Layer& Ly = c->layers[li];
  FusedLayer w{};
  w.qkv = Ly.f_qkv.w; w.qkv_b = Ly.f_qkv.b;
  w.o_sa = Ly.f_o_sa.w; w.o_sa_b = Ly.f_o_sa.b;
  w.q_ca = Ly.f_q_ca.w; w.q_ca_b = Ly.f_q_ca.b;
  w.o_ca = Ly.f_o_ca.w; w.o_ca_b = Ly.f_o_ca.b;
  w.ff1 = Ly.f_ff1.w; w.ff1_b = Ly.f_ff1.b;
  w.ff2 = Ly.f_ff2.w; w.ff2_b = Ly.f_ff2.b;
  w.ln1_g = Ly.ln1_g; w.ln1_b = Ly.ln1_b; w.ln2_g = Ly.ln2_g; w.ln2_b = Ly.ln2_b;
  w.ln3_g = Ly.ln3_g; w.ln3_b = Ly.ln3_b;
  w.sa_qw = Ly.sa_q.w; w.sa_qb = Ly.sa_q.b; w.sa_kw = Ly.sa_k.w; w.sa_kb = Ly.sa_k.b;
  w.sa_vw = Ly.sa_v.w; w.sa_vb = Ly.sa_v.b;
  w.ca_qw = Ly.ca_q.w; w.ca_qb = Ly.ca_q.b; w.ca_kw = Ly.ca_k.w; w.ca_kb = Ly.ca_k.b;
  w.ca_vw = Ly.ca_v.w; w.ca_vb = Ly.ca_v.b;
  w.kv_mem = c->kv_mem + (size_t)li * D.max_batch * D.speech_len * 2 * d;
  w.kv_step = c->kv_step + (size_t)li * D.diffusion_steps * 2 * d;
  w.kvc = c->kvc ? (const char*)c->kvc + c->tsize * (size_t)li * D.max_batch * D.heads * KVC_ELEMS : nullptr;
  return w;
}

// every attention launch of the generic routes: counts the whole-clip kernel's launches
hipError_t run_attention(ggd_ctx* c, int dtype, const AttnArgs& at, int n, hipStream_t s) {
  if (attention_clip_supported(dtype, at)) ++c->clip_attn_launches;
  return launch_attention(dtype, at, n, s);
}

// KA / KB arguments of layer li (KC runs on h2 -> h, KD on h in place)
FusedArgs fused_args(ggd_ctx* c, int li, const int* t_clip) {
  const ggd_desc& D = c->desc;
  FusedArgs f{};
  f.w = fused_layer(c, li);
  f.L = D.seq_len;
  f.Ts = D.speech_len;
  f.o_sa = c->att;
  f.o_ca = c->q;
  f.hid = c->ffn;
  f.ffp = c->ffp;
  f.t_clip = t_clip;
  f.steps = c->d_steps;
  f.step_counter = c->d_counter;
  f.scale = 1.0f / std::sqrt((float)(D.d_model / D.heads));
  f.h = c->h;
  f.h_out = c->h2;
  if (li == 0) {  // layer 0's KA also computes h = emb_x(x) + PE from the state x
    f.x_emb = c->x;
    f.w_emb = c->f_emb.w;
    f.b_emb = c->f_emb.b;
    f.pe = c->pe;
    f.C = D.d_pose;
  }
  return f;
}

int launch_fused_layers(ggd_ctx* c, int n, bool sampling, const int* t_clip) {
  const ggd_desc& D = c->desc;
  const int L = D.seq_len, d = D.d_model, M = n * L;
  hipStream_t s = c->stream;
  for (int li = 0; li < D.n_layers; ++li) {
    FusedArgs f = fused_args(c, li, t_clip);
    f.bump_counter = sampling && li == 0;
    HIP_TRY(c, launch_fused(0, D.dtype, f, n, s));     // KA: [emb +] LN1 + QKV + conv + self-attention
    f.x_emb = nullptr;
    f.bump_counter = 0;
    if (c->profiling && sampling && c->span) {         // KB is the dominant kernel of the step
      f.span = c->span;
      f.span_stride = D.n_layers;
      f.span_layer = li;
    }
    HIP_TRY(c, launch_fused(1, D.dtype, f, n, s));     // KB: out-proj + LN2 + Q + cross-attention
    f.span = nullptr;
    f.h = c->h2;
    f.h_out = c->h;
    HIP_TRY(c, launch_fused(2, D.dtype, f, n, s));     // KC: out-proj + LN3 + FFN-up + ReLU^2
    f.h = c->h;
    HIP_TRY(c, launch_fused(3, D.dtype, f, n, s));     // KD: FFN-down + residual (in place on h)
  }
  return GGD_OK;
}

// The decoder forward on the internal x state (M = n*L rows) ending in eps [M][cpad].
// In sampling mode (`sampling`), the first GEMM advances the iteration counter and the
// cross-attention reads t from the step records.
// CrossAttention.forward (nn.py:428-447) with CrossAttentionLayer (nn.py:90-125) on the generic
// kernels.  Joint layout: clip b's rows b*J .. b*J+J-1 hold [x (L rows); memory (1 + Ts rows)];
// the x-only / memory-only sub-layers address their segment through GEMM row maps and the
// attention's row offset, so [x; memory] is never concatenated or split by a copy.
int launch_decoder_twoway(ggd_ctx* c, int n, bool sampling, const int* t_clip) {
  const ggd_desc& D = c->desc;
  const int L = D.seq_len, d = D.d_model, J = c->J, Tm = J - L, dk = d / D.heads, dt = D.dtype;
  hipStream_t s = c->stream;
  // x rows: emb_x + PE[0 .. L) (the first launch of a step bumps the iteration counter)
  GemmArgs g = gemm_args(c->emb_x, n * L, c->x, D.d_pose, c->hj, d);
  g.a_add = c->inp_on ? c->inp_delta : nullptr;
  g.pe = c->pe;
  g.pe_period = L;
  g.pe_offset = 0;
  g.o_len = L;
  g.o_stride = J;
  g.step_counter = sampling ? c->d_counter : nullptr;
  GEMM(c, PRO_F32, EPI_PE, g, s);
  // memory rows: step token of t + the installed speech rows (both already carry their PE)
  HIP_TRY(c, launch_mem_assemble(c->hj, c->mem_base, c->step_tab, t_clip, c->d_steps, c->d_counter, n, L,
                                 D.speech_len, d, s));

  struct Seg { int len, off, rows; };  // rows per clip of a segment and its first row
  const Seg SX{L, 0, L}, SM{Tm, L, Tm}, SJ{J, 0, J};
  auto ln = [&](const Seg& sg, const float* gm, const float* bt) -> hipError_t {
    return launch_layernorm(dt, c->hj, sg.len == J ? 0 : sg.len, J, sg.off, gm, bt, c->zbuf, n * sg.rows, d, s);
  };
  // x_seg += MDHA(LN(x_seg)) over the segment's own sequence (nn.py:96-104, 106-113)
  auto attn_block = [&](const Seg& sg, const float* gm, const float* bt, const Lin& qkv, const Lin& o,
                        const Conv3& cq, const Conv3& ck, const Conv3& cv) -> int {
    const int M = n * sg.rows, map = sg.len == J ? 0 : sg.len;
    HIP_TRY(c, ln(sg, gm, bt));
    GemmArgs q = gemm_args(qkv, M, c->zbuf, d, c->qkvj, 3 * d);
    q.o_len = map;
    q.o_stride = J;
    q.o_off = sg.off;
    GEMM(c, PRO_T, EPI_T, q, s);
    AttnArgs at{};
    at.zero = c->zero_row;
    at.no_clip = c->attn_qsplit;
  at.no_clip = c->attn_qsplit;
    at.cross = 0;
    at.q = c->qkvj;
    at.ldq = 3 * d;
    at.k = (const char*)c->qkvj + c->tsize * d;
    at.v = (const char*)c->qkvj + c->tsize * 2 * d;
    at.ldkv = 3 * d;
    at.cw_q = cq.w; at.cb_q = cq.b;
    at.cw_k = ck.w; at.cb_k = ck.b;
    at.cw_v = cv.w; at.cb_v = cv.b;
    at.out = c->attj;
    at.ldo = d;
    at.Lq = at.Lk = sg.rows;
    at.dk = dk;
    at.heads = D.heads;
    at.d = d;
    at.scale = 1.0f / std::sqrt((float)dk);
    at.seq_stride = J;
    at.seq_off = sg.off;
    HIP_TRY(c, run_attention(c, dt, at, n, s));
    GemmArgs op = gemm_args(o, M, c->attj, d, c->hj, d);
    op.a_len = op.o_len = map;
    op.a_stride = op.o_stride = J;
    op.a_off = op.o_off = sg.off;
    GEMM(c, PRO_T, EPI_RESID, op, s);
    return GGD_OK;
  };
  // seg += FFN(LN(seg)) (nn.py:116-124)
  auto ffn_block = [&](const Seg& sg, const float* gm, const float* bt, const Lin& f1, const Lin& f2) -> int {
    const int M = n * sg.rows;
    HIP_TRY(c, ln(sg, gm, bt));
    GemmArgs a1 = gemm_args(f1, M, c->zbuf, d, c->ffnj, 4 * d);
    GEMM(c, PRO_T, EPI_RELU2, a1, s);
    GemmArgs a2 = gemm_args(f2, M, c->ffnj, 4 * d, c->hj, d);
    a2.o_len = sg.len;
    a2.o_stride = J;
    a2.o_off = sg.off;
    GEMM(c, PRO_T, EPI_RESID, a2, s);
    return GGD_OK;
  };
  int r;
  for (int li = 0; li < D.n_layers; ++li) {
    const Layer2& Y = c->layers2[li];
    if ((r = attn_block(SX, Y.ln_sa_g, Y.ln_sa_b, Y.qkv_sa, Y.o_sa, Y.sa_q, Y.sa_k, Y.sa_v))) return r;
    if ((r = attn_block(SM, Y.ln_sam_g, Y.ln_sam_b, Y.qkv_sam, Y.o_sam, Y.sam_q, Y.sam_k, Y.sam_v))) return r;
    if ((r = attn_block(SJ, Y.ln_ca_g, Y.ln_ca_b, Y.qkv_ca, Y.o_ca, Y.ca_q, Y.ca_k, Y.ca_v))) return r;
    if ((r = ffn_block(SX, Y.ln_ff_g, Y.ln_ff_b, Y.ff1, Y.ff2))) return r;
    if (Y.has_ffm && (r = ffn_block(SM, Y.ln_ffm_g, Y.ln_ffm_b, Y.ffm1, Y.ffm2))) return r;
  }
  // out_layers on the x rows (nn.py:434-436, 447)
  HIP_TRY(c, ln(SX, c->out_ln_g, c->out_ln_b));
  g = gemm_args(c->out_lin, n * L, c->zbuf, d, c->eps, c->cpad);
  GEMM(c, PRO_T, EPI_F32, g, s);
  return GGD_OK;
}

ChainLin chain_lin(const Lin& L) {
  ChainLin r{};
  r.w = L.wf;
  r.b = L.b;
  r.scale = L.scale;
  r.npad = L.npad;
  r.kpad = L.kpad;
  return r;
}

AttnArgs self_attn_args(ggd_ctx* c, const Layer& Ly) {
  const ggd_desc& D = c->desc;
  const int d = D.d_model, dk = d / D.heads;
  AttnArgs at{};
  at.zero = c->zero_row;
  at.no_clip = c->attn_qsplit;
  at.cross = 0;
  at.q = c->qkv;
  at.ldq = 3 * d;
  at.k = (const char*)c->qkv + c->tsize * d;
  at.v = (const char*)c->qkv + c->tsize * 2 * d;
  at.ldkv = 3 * d;
  at.cw_q = Ly.sa_q.w; at.cb_q = Ly.sa_q.b;
  at.cw_k = Ly.sa_k.w; at.cb_k = Ly.sa_k.b;
  at.cw_v = Ly.sa_v.w; at.cb_v = Ly.sa_v.b;
  at.out = c->att;
  at.ldo = d;
  at.Lq = D.seq_len;
  at.Lk = D.seq_len;
  at.dk = dk;
  at.heads = D.heads;
  at.d = d;
  at.scale = 1.0f / std::sqrt((float)dk);
  return at;
}

void cross_attn_args(ggd_ctx* c, const Layer& Ly, int li, const int* t_clip, AttnArgs& at) {
  const ggd_desc& D = c->desc;
  const int d = D.d_model;
  at.cross = 1;
  at.q = c->q;
  at.ldq = d;
  at.kv_mem = c->kv_mem + (size_t)li * D.max_batch * D.speech_len * 2 * d;
  at.kv_step = c->kv_step + (size_t)li * D.diffusion_steps * 2 * d;
  at.t_clip = t_clip;
  at.steps = c->d_steps;
  at.step_counter = c->d_counter;
  at.cw_q = Ly.ca_q.w; at.cb_q = Ly.ca_q.b;
  at.cw_k = Ly.ca_k.w; at.cb_k = Ly.ca_k.b;
  at.cw_v = Ly.ca_v.w; at.cb_v = Ly.ca_v.b;
  at.Lk = 1 + D.speech_len;
}

// The one-way decoder as row-block chains (ggd_chain.hip): emb_x + PE, then per layer
// [self-attention, chain R(o_sa) + P(LN2, q_ca), cross-attention, chain R(o_ca) + F + P(next
// layer's LN1 + QKV, or out_layers)].  Same arithmetic as the per-GEMM route, bit for bit.
int launch_decoder_chain(ggd_ctx* c, int n, bool sampling, const int* t_clip) {
  const ggd_desc& D = c->desc;
  const int L = D.seq_len, d = D.d_model, M = n * L, w8 = D.dtype == GGD_FP8W;
  hipStream_t s = c->stream;
  GemmArgs g = gemm_args(c->emb_x, M, c->x, D.d_pose, c->h, d);
  g.a_add = c->inp_on ? c->inp_delta : nullptr;
  g.pe = c->pe;
  g.pe_period = L;
  g.pe_offset = 0;
  g.step_counter = sampling ? c->d_counter : nullptr;
  GEMM(c, PRO_F32, EPI_PE, g, s);
  auto chain = [&](const ChainArgs& ca) -> int {
    HIP_TRY(c, launch_chain(w8, ca, s));
    return GGD_OK;
  };
  auto qkv_proj = [&](ChainArgs& ca, const Layer& Ly) {  // P: LN1 + the self-attention QKV
    ca.p_g = Ly.ln1_g;
    ca.p_b = Ly.ln1_b;
    ca.p = chain_lin(Ly.qkv);
    ca.out = c->qkv;
    ca.ldo = 3 * d;
  };
  int r;
  ChainArgs c0{};
  c0.M = M;
  c0.h = c->h;
  qkv_proj(c0, c->layers[0]);
  if ((r = chain(c0))) return r;
  for (int li = 0; li < D.n_layers; ++li) {
    const Layer& Ly = c->layers[li];
    AttnArgs at = self_attn_args(c, Ly);
    if (c->profiling && sampling && (r = prof_mark(c, s))) return r;
    HIP_TRY(c, run_attention(c, D.dtype, at, n, s));
    if (c->profiling && sampling && (r = prof_mark(c, s))) return r;
    ChainArgs ca{};
    ca.M = M;
    ca.h = c->h;
    ca.a_in = (const bf16_t*)c->att;
    ca.r = chain_lin(Ly.o_sa);
    ca.p_g = Ly.ln2_g;
    ca.p_b = Ly.ln2_b;
    ca.p = chain_lin(Ly.q_ca);
    ca.out = c->q;
    ca.ldo = d;
    if ((r = chain(ca))) return r;
    cross_attn_args(c, Ly, li, t_clip, at);
    if (c->profiling && sampling && (r = prof_mark(c, s))) return r;
    HIP_TRY(c, run_attention(c, D.dtype, at, n, s));
    if (c->profiling && sampling && (r = prof_mark(c, s))) return r;
    ChainArgs cb{};
    cb.M = M;
    cb.h = c->h;
    cb.a_in = (const bf16_t*)c->att;
    cb.r = chain_lin(Ly.o_ca);
    cb.f_g = Ly.ln3_g;
    cb.f_b = Ly.ln3_b;
    cb.f1 = chain_lin(Ly.ff1);
    cb.f2 = chain_lin(Ly.ff2);
    if (li + 1 < D.n_layers) {
      qkv_proj(cb, c->layers[li + 1]);
    } else {  // out_layers: LayerNorm + Linear(d -> d_pose) (nn.py:211-214,228)
      cb.p_g = c->out_ln_g;
      cb.p_b = c->out_ln_b;
      cb.p = chain_lin(c->out_lin);
      cb.out = c->eps;
      cb.ldo = c->cpad;
      cb.out_f32 = 1;
      cb.n_valid = c->out_lin.n;
    }
    if ((r = chain(cb))) return r;
  }
  return GGD_OK;
}

int launch_decoder(ggd_ctx* c, int n, bool sampling, const int* t_clip) {
  const ggd_desc& D = c->desc;
  if (c->twoway) return launch_decoder_twoway(c, n, sampling, t_clip);
  if (c->fused) return launch_fused_layers(c, n, sampling, t_clip);
  if (c->chain && !c->gemm_launches) return launch_decoder_chain(c, n, sampling, t_clip);
  const int L = D.seq_len, d = D.d_model, M = n * L, dk = d / D.heads;
  hipStream_t s = c->stream;

  GemmArgs g = gemm_args(c->emb_x, M, c->x, D.d_pose, c->h, d);
  g.a_add = c->inp_on ? c->inp_delta : nullptr;
  g.pe = c->pe;
  g.pe_period = L;
  g.pe_offset = 0;
  g.step_counter = sampling ? c->d_counter : nullptr;
  GEMM(c, PRO_F32, EPI_PE, g, s);

  for (int li = 0; li < D.n_layers; ++li) {
    const Layer& Ly = c->layers[li];
    // self-attention block (nn.py:160-162)
    g = gemm_args(Ly.qkv, M, c->h, d, c->qkv, 3 * d);
    g.ln_g = Ly.ln1_g;
    g.ln_b = Ly.ln1_b;
    GEMM(c, PRO_LN, EPI_T, g, s);

    AttnArgs at{};
    at.zero = c->zero_row;
    at.no_clip = c->attn_qsplit;
  at.no_clip = c->attn_qsplit;
    at.cross = 0;
    at.q = c->qkv;
    at.ldq = 3 * d;
    at.k = (const char*)c->qkv + c->tsize * d;
    at.v = (const char*)c->qkv + c->tsize * 2 * d;
    at.ldkv = 3 * d;
    at.cw_q = Ly.sa_q.w; at.cb_q = Ly.sa_q.b;
    at.cw_k = Ly.sa_k.w; at.cb_k = Ly.sa_k.b;
    at.cw_v = Ly.sa_v.w; at.cb_v = Ly.sa_v.b;
    at.out = c->att;
    at.ldo = d;
    at.Lq = L;
    at.Lk = L;
    at.dk = dk;
    at.heads = D.heads;
    at.d = d;
    at.scale = 1.0f / std::sqrt((float)dk);
    if (c->profiling && sampling) { int r = prof_mark(c, s); if (r) return r; }
    HIP_TRY(c, run_attention(c, D.dtype, at, n, s));
    if (c->profiling && sampling) { int r = prof_mark(c, s); if (r) return r; }

    g = gemm_args(Ly.o_sa, M, c->att, d, c->h, d);
    GEMM(c, PRO_T, EPI_RESID, g, s);

    // cross-attention block (nn.py:165-167)
    g = gemm_args(Ly.q_ca, M, c->h, d, c->q, d);
    g.ln_g = Ly.ln2_g;
    g.ln_b = Ly.ln2_b;
    GEMM(c, PRO_LN, EPI_T, g, s);

    at.cross = 1;
    at.q = c->q;
    at.ldq = d;
    at.kv_mem = c->kv_mem + (size_t)li * D.max_batch * D.speech_len * 2 * d;
    at.kv_step = c->kv_step + (size_t)li * D.diffusion_steps * 2 * d;
    at.t_clip = t_clip;
    at.steps = c->d_steps;
    at.step_counter = c->d_counter;
    at.cw_q = Ly.ca_q.w; at.cb_q = Ly.ca_q.b;
    at.cw_k = Ly.ca_k.w; at.cb_k = Ly.ca_k.b;
    at.cw_v = Ly.ca_v.w; at.cb_v = Ly.ca_v.b;
    at.Lk = 1 + D.speech_len;
    if (c->profiling && sampling) { int r = prof_mark(c, s); if (r) return r; }
    HIP_TRY(c, run_attention(c, D.dtype, at, n, s));
    if (c->profiling && sampling) { int r = prof_mark(c, s); if (r) return r; }

    g = gemm_args(Ly.o_ca, M, c->att, d, c->h, d);
    GEMM(c, PRO_T, EPI_RESID, g, s);

    // feed-forward block (nn.py:170-172)
    g = gemm_args(Ly.ff1, M, c->h, d, c->ffn, 4 * d);
    g.ln_g = Ly.ln3_g;
    g.ln_b = Ly.ln3_b;
    GEMM(c, PRO_LN, EPI_RELU2, g, s);

    g = gemm_args(Ly.ff2, M, c->ffn, 4 * d, c->h, d);
    GEMM(c, PRO_T, EPI_RESID, g, s);
  }
  // out_layers: LayerNorm + Linear(d -> d_pose) (nn.py:211-214,228)
  g = gemm_args(c->out_lin, M, c->h, d, c->eps, c->cpad);
  g.ln_g = c->out_ln_g;
  g.ln_b = c->out_ln_b;
  GEMM(c, PRO_LN, EPI_F32, g, s);
  return GGD_OK;
}

int launch_step(ggd_ctx* c, const ggd_sample_args& a, float* extras, int fixed_k) {
  int r = launch_decoder(c, a.n, true, nullptr);
  if (r) return r;
  if (c->fused) {  // KE: LN_out + out-proj + update (the next step's emb is in its first KA)
    FinalArgs f = final_args(c, a.n);
    f.alg = a.alg;
    f.noise = a.noise;
    f.seed = a.seed;
    f.clip_offset = a.clip_offset;
    f.inp_pose = a.inpaint_masks ? a.inpaint_poses : nullptr;
    f.inp_mask = a.inpaint_masks;
    f.trans = a.trans;
    f.extras = extras;
    f.do_out = 1;
    f.do_update = 1;
    HIP_TRY(c, launch_final(c->desc.dtype, f, c->stream));
    return GGD_OK;
  }
  UpdArgs u{};
  u.n = a.n;
  u.C = c->desc.d_pose;
  u.L = c->desc.seq_len;
  u.ld_eps = c->cpad;
  u.alg = a.alg;
  u.eps = c->eps;
  u.x = c->x;
  u.steps = c->d_steps;
  u.step_counter = c->d_counter;
  u.fixed_k = fixed_k;
  u.noise = a.noise;
  u.seed = a.seed;
  u.clip_offset = a.clip_offset;
  u.inp_pose = a.inpaint_masks ? a.inpaint_poses : nullptr;
  u.inp_mask = a.inpaint_masks;
  u.trans = a.trans;
  u.extras = extras;
  HIP_TRY(c, launch_update(u, c->stream));
  return GGD_OK;
}

// Host f32 step records in the reference's op order (all f32 IEEE, like torch CPU):
//   DDPM sigma = exp(0.5 * logvar_f32)                        gaussian_diffusion.py:328
//   DDIM sigma = eta * sqrt((1-abp)/(1-ab)) * sqrt(1 - ab/abp) :468-472
//        c_eps = sqrt(1 - abp - sigma^2)                       :477
void make_records(ggd_ctx* c, int alg, float eta, std::vector<StepRec>& recs, uint64_t seed = 0,
                  int64_t clip_offset = 0) {
#pragma clang fp contract(off)
  const int T = (int)c->betas.size();
  std::vector<double> ac(T), acp(T);
  double run = 1.0;
  for (int i = 0; i < T; ++i) {
    acp[i] = run;
    run *= (1.0 - c->betas[i]);
    ac[i] = run;
  }
  // numpy: alphas_cumprod = cumprod(1 - betas); recompute exactly like np.cumprod (sequential)
  recs.resize(T);
  for (int k = 0; k < T; ++k) {
    const int i = T - 1 - k;
    const double beta = c->betas[i];
    const double a_i = 1.0 - beta;
    StepRec& r = recs[k];
    r.sra = (float)std::sqrt(1.0 / ac[i]);
    r.srm1 = (float)std::sqrt(1.0 / ac[i] - 1.0);
    const double pv_i = beta * (1.0 - acp[i]) / (1.0 - ac[i]);
    double pv_clip = pv_i;
    if (i == 0 && T > 1) {
      const double a1 = ac[1], ap1 = acp[1];
      pv_clip = c->betas[1] * (1.0 - ap1) / (1.0 - a1);
    }
    r.var = (float)pv_i;
    r.logvar = (float)std::log(pv_clip);
    r.c1 = (float)(beta * std::sqrt(acp[i]) / (1.0 - ac[i]));
    r.c2 = (float)((1.0 - acp[i]) * std::sqrt(a_i) / (1.0 - ac[i]));
    const float ab = (float)ac[i], abp = (float)acp[i];
    r.sqrt_abp = std::sqrt(abp);
    if (alg == GGD_DDPM) {
      r.sigma = std::exp(0.5f * r.logvar);
      r.c_eps = 0.f;
    } else {
      volatile float t1 = (1.0f - abp) / (1.0f - ab);
      volatile float t2 = 1.0f - ab / abp;
      volatile float sg = eta * std::sqrt((float)t1);
      sg = sg * std::sqrt((float)t2);
      r.sigma = sg;
      volatile float sq = sg * sg;
      volatile float inner = (1.0f - abp) - sq;
      r.c_eps = std::sqrt((float)inner);
    }
    r.i = i;
    r.t_orig = c->tmap[i];
    r.seed_lo = (uint32_t)seed;
    r.seed_hi = (uint32_t)(seed >> 32);
    r.clip_offset = (uint32_t)clip_offset;
  }
}

}  // namespace

extern "C" {

const char* ggd_version(void) { return "ggd 0.1 (gfx950)"; }

const char* ggd_last_error(const ggd_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ggd_create(int device, const ggd_desc* desc, ggd_ctx** out) {
  if (!desc || !out) return GGD_ERR_ARG;
  *out = nullptr;
  ggd_ctx* c = new ggd_ctx();
  c->device = device;
  c->desc = *desc;
  const ggd_desc& D = *desc;
  if (D.d_model <= 0 || D.heads <= 0 || D.d_model % D.heads || D.n_layers <= 0 || D.d_pose <= 0 ||
      D.seq_len <= 0 || D.speech_len <= 0 || D.max_batch <= 0 || D.diffusion_steps <= 0) {
    c->err = "invalid descriptor";
    *out = c;
    return GGD_ERR_ARG;
  }
  const int dk = D.d_model / D.heads;
  if (D.decoder_type == GGD_DEC_TWOWAY) {
    // CrossAttention (nn.py:381-447) on the generic kernels: joint sequence [x; memory]
    if ((dk != 32 && dk != 64) || D.d_model % 256 || D.d_model > 1024 || D.seq_len + 1 + D.speech_len > 192) {
      c->err = "unsupported two-way shape (need d_model % 256 == 0, d_k in {32,64}, L + 1 + Ts <= 192)";
      *out = c;
      return GGD_ERR_UNSUPPORTED;
    }
  } else if (D.decoder_type != GGD_DEC_ONEWAY) {
    c->err = "unknown decoder type";
    *out = c;
    return GGD_ERR_UNSUPPORTED;
  } else if ((dk != 32 && dk != 64) || D.d_model != 256 || D.seq_len > 192 || D.speech_len + 1 > 192) {
    c->err = "unsupported shape (need d_model == 256, d_k in {32,64}, L <= 192, memory <= 192)";
    *out = c;
    return GGD_ERR_UNSUPPORTED;
  }
  if (D.dtype != GGD_F32 && D.dtype != GGD_BF16 && D.dtype != GGD_FP8W) {
    c->err = "unsupported dtype";
    *out = c;
    return GGD_ERR_UNSUPPORTED;
  }
  c->tsize = D.dtype == GGD_F32 ? 4 : 2;
  *out = c;
  HIP_TRY(c, hipSetDevice(device));
  {  // the sampler's stream takes the highest priority: a prefetched speech encoder on another
     // stream (Speech2GestureModel.prefetch_speech) must not hold up the next loop's set-up GEMMs
    int least = 0, greatest = 0;
    HIP_TRY(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(c, hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
  }
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) == hipSuccess && khz > 0)
      c->wall_mhz = khz / 1000.0;
  }
  HIP_TRY(c, hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
  HIP_TRY(c, hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming));

  const int d = D.d_model, L = D.seq_len, B = D.max_batch, M = B * L, Ts = D.speech_len;
  c->cpad = round_up(D.d_pose, 64);
  HIP_TRY(c, dalloc(c, &c->x, sizeof(float) * M * D.d_pose));
  HIP_TRY(c, dalloc(c, &c->h, sizeof(float) * M * d));
  HIP_TRY(c, dalloc(c, &c->h2, sizeof(float) * M * d));
  HIP_TRY(c, dalloc(c, &c->eps, sizeof(float) * M * c->cpad));
  HIP_TRY(c, dalloc(c, &c->qkv, c->tsize * M * 3 * d));
  HIP_TRY(c, dalloc(c, &c->att, c->tsize * M * d));
  HIP_TRY(c, dalloc(c, &c->q, c->tsize * M * d));
  HIP_TRY(c, dalloc(c, &c->ffn, c->tsize * M * 4 * d));
  HIP_TRY(c, dalloc(c, &c->d_counter, sizeof(int)));
  HIP_TRY(c, dalloc(c, &c->zero_row, 1024));
  if (D.model_type == GGD_MODEL_INPAINT) {
    HIP_TRY(c, dalloc(c, &c->inp_in, sizeof(float) * M * (D.d_pose + 1)));
    HIP_TRY(c, dalloc(c, &c->inp_h1, sizeof(float) * M * d));
    HIP_TRY(c, dalloc(c, &c->inp_h2, sizeof(float) * M * d));
    HIP_TRY(c, dalloc(c, &c->inp_delta, sizeof(float) * M * D.d_pose));
  }
  HIP_TRY(c, dalloc(c, &c->d_t, sizeof(int) * B));
  HIP_TRY(c, dalloc(c, &c->mem_tmp, sizeof(float) * (size_t)B * Ts * d));
  HIP_TRY(c, dalloc(c, &c->tok_tmp, sizeof(float) * (size_t)B * Ts * d));
  if (D.decoder_type == GGD_DEC_TWOWAY) {
    c->twoway = true;
    c->J = L + 1 + Ts;
    const size_t MJ = (size_t)B * c->J;
    HIP_TRY(c, dalloc(c, &c->hj, sizeof(float) * MJ * d));
    HIP_TRY(c, dalloc(c, &c->qkvj, c->tsize * MJ * 3 * d));
    HIP_TRY(c, dalloc(c, &c->attj, c->tsize * MJ * d));
    HIP_TRY(c, dalloc(c, &c->zbuf, c->tsize * MJ * d));
    HIP_TRY(c, dalloc(c, &c->ffnj, c->tsize * (size_t)B * std::max(L, 1 + Ts) * 4 * d));
    HIP_TRY(c, dalloc(c, &c->mem_base, sizeof(float) * (size_t)B * Ts * d));
    HIP_TRY(c, dalloc(c, &c->step_tab, sizeof(float) * (size_t)D.diffusion_steps * d));
    c->pe_len = c->J + 1;
  } else {
    HIP_TRY(c, dalloc(c, &c->kv_mem, sizeof(float) * D.n_layers * (size_t)B * Ts * 2 * d));
    HIP_TRY(c, dalloc(c, &c->kv_step, sizeof(float) * D.n_layers * (size_t)D.diffusion_steps * 2 * d));
    c->pe_len = std::max(L, Ts + 1) + 1;
  }
  std::vector<float> pe;
  build_pe(pe, c->pe_len, d);
  HIP_TRY(c, dalloc(c, &c->pe, sizeof(float) * pe.size()));
  HIP_TRY(c, hipMemcpy(c->pe, pe.data(), sizeof(float) * pe.size(), hipMemcpyHostToDevice));

  return GGD_OK;
}

int ggd_destroy(ggd_ctx* c) {
  if (!c) return GGD_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (auto& p : c->pend) {
    if (p.ev) hipEventDestroy(p.ev);
    if (p.host) hipHostFree(p.host);
  }
  c->pend.clear();
  for (auto& kv : c->uploads)
    for (int i = 0; i < 2; ++i) {
      if (kv.second.ev[i]) hipEventDestroy(kv.second.ev[i]);
      if (kv.second.slot[i]) hipHostFree(kv.second.slot[i]);
    }
  c->uploads.clear();
  if (c->gexec) hipGraphExecDestroy(c->gexec);
  if (c->graph) hipGraphDestroy(c->graph);
  for (void* p : c->allocs) hipFree(p);
  for (auto& e : c->prof.ev) hipEventDestroy(e);
  if (c->ev_in) hipEventDestroy(c->ev_in);
  if (c->ev_out) hipEventDestroy(c->ev_out);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return GGD_OK;
}

int ggd_load_weight(ggd_ctx* c, const char* name, const float* host_data, int64_t numel) {
  if (!c || !name || (!host_data && numel > 0) || numel < 0) return fail(c, GGD_ERR_ARG, "bad argument");
  const std::string n(name);
  if (n.rfind("speech_encoder.", 0) == 0) return GGD_IGNORED;
  const bool known = n.rfind("pose_decoder.", 0) == 0 || n.rfind("diffusion_step_encoder.", 0) == 0 ||
                     n.rfind("blend_layer.", 0) == 0 ||
                     (c->desc.model_type == GGD_MODEL_INPAINT && n.rfind("proj.", 0) == 0);
  if (!known) return fail(c, GGD_ERR_NAME, "unknown weight name: " + n);
  c->staged[n].assign(host_data, host_data + numel);
  c->finalized = false;
  return GGD_OK;
}

int ggd_finalize_weights(ggd_ctx* c) {
  if (!c) return GGD_ERR_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  const ggd_desc& D = c->desc;
  const int d = D.d_model, C = D.d_pose, dk = d / D.heads;
  const std::string P = "pose_decoder.";
  int r;
#define TRY(x) do { r = (x); if (r) return r; } while (0)
  TRY(pack_lin(c, c->emb_x, {P + "emb_x"}, d, C, true));
  TRY(pack_lin(c, c->emb_mem, {P + "emb_mem"}, d, d));
  TRY(pack_lin(c, c->out_lin, {P + "out_layers.1"}, C, d, true));
  TRY(upload_vec(c, &c->out_ln_g, P + "out_layers.0.weight", d));
  TRY(upload_vec(c, &c->out_ln_b, P + "out_layers.0.bias", d));
  TRY(pack_lin(c, c->step0, {"diffusion_step_encoder.proj.0"}, d, d));
  TRY(pack_lin(c, c->step2, {"diffusion_step_encoder.proj.2"}, d, d));
  if (D.model_type == GGD_MODEL_S2G_V2) TRY(pack_lin(c, c->blend, {"blend_layer"}, d, 3 * d));
  if (D.model_type == GGD_MODEL_INPAINT) {  // step-invariant: evaluated once per ggd_set_inpaint
    TRY(pack_lin(c, c->inp0, {"proj.0"}, d, C + 1));
    TRY(pack_lin(c, c->inp2, {"proj.2"}, d, d));
    TRY(pack_lin(c, c->inp4, {"proj.4"}, C, d));
  }
  if (c->twoway) {
    c->layers2.assign(D.n_layers, Layer2{});
    for (int l = 0; l < D.n_layers; ++l) {
      Layer2& Ly = c->layers2[l];
      const std::string q = P + "layers." + std::to_string(l) + ".";
      auto ln = [&](float** g, float** b, const std::string& name) {
        int rr = upload_vec(c, g, q + name + ".weight", d);
        return rr ? rr : upload_vec(c, b, q + name + ".bias", d);
      };
      auto mdha = [&](Lin& qkv, Lin& o, Conv3& cq, Conv3& ck, Conv3& cv, const std::string& name) {
        const std::string a = q + name + ".";
        int rr = pack_lin(c, qkv, {a + "query.0.linear", a + "key.0.linear", a + "value.0.linear"}, d, d, true);
        if (!rr) rr = pack_lin(c, o, {a + "output"}, d, d, true);
        if (!rr) rr = pack_conv(c, cq, a + "query.1", dk);
        if (!rr) rr = pack_conv(c, ck, a + "key.1", dk);
        if (!rr) rr = pack_conv(c, cv, a + "value.1", dk);
        return rr;
      };
      TRY(ln(&Ly.ln_sa_g, &Ly.ln_sa_b, "norm_self_attn"));
      TRY(mdha(Ly.qkv_sa, Ly.o_sa, Ly.sa_q, Ly.sa_k, Ly.sa_v, "self_attn"));
      TRY(ln(&Ly.ln_sam_g, &Ly.ln_sam_b, "norm_self_attn_mem"));
      TRY(mdha(Ly.qkv_sam, Ly.o_sam, Ly.sam_q, Ly.sam_k, Ly.sam_v, "self_attn_mem"));
      TRY(ln(&Ly.ln_ca_g, &Ly.ln_ca_b, "norm_cross_attn"));
      TRY(mdha(Ly.qkv_ca, Ly.o_ca, Ly.ca_q, Ly.ca_k, Ly.ca_v, "cross_attn"));
      TRY(ln(&Ly.ln_ff_g, &Ly.ln_ff_b, "norm_ff"));
      TRY(pack_lin(c, Ly.ff1, {q + "feed_forward.layer1"}, 4 * d, d, true));
      TRY(pack_lin(c, Ly.ff2, {q + "feed_forward.layer2"}, d, 4 * d, true));
      Ly.has_ffm = c->staged.count(q + "feed_forward_mem.layer1.weight") != 0;
      if (Ly.has_ffm) {
        TRY(ln(&Ly.ln_ffm_g, &Ly.ln_ffm_b, "norm_ff_mem"));
        TRY(pack_lin(c, Ly.ffm1, {q + "feed_forward_mem.layer1"}, 4 * d, d, true));
        TRY(pack_lin(c, Ly.ffm2, {q + "feed_forward_mem.layer2"}, d, 4 * d, true));
      } else if (l + 1 < D.n_layers) {
        return fail(c, GGD_ERR_NAME, "missing weight: " + q + "feed_forward_mem.layer1.weight");
      }
    }
    TRY(build_step_tables(c));
    c->fused = c->persist = false;
    c->staged.clear();
    c->finalized = true;
    return GGD_OK;
  }
  c->layers.assign(D.n_layers, Layer{});
  for (int l = 0; l < D.n_layers; ++l) {
    Layer& Ly = c->layers[l];
    const std::string q = P + "layers." + std::to_string(l) + ".";
    TRY(upload_vec(c, &Ly.ln1_g, q + "norm_self_attn.weight", d));
    TRY(upload_vec(c, &Ly.ln1_b, q + "norm_self_attn.bias", d));
    TRY(upload_vec(c, &Ly.ln2_g, q + "norm_cross_attn.weight", d));
    TRY(upload_vec(c, &Ly.ln2_b, q + "norm_cross_attn.bias", d));
    TRY(upload_vec(c, &Ly.ln3_g, q + "norm_ff.weight", d));
    TRY(upload_vec(c, &Ly.ln3_b, q + "norm_ff.bias", d));
    const std::string sa = q + "self_attn.", ca = q + "cross_attn.";
    TRY(pack_lin(c, Ly.qkv, {sa + "query.0.linear", sa + "key.0.linear", sa + "value.0.linear"}, d, d, true));
    TRY(pack_lin(c, Ly.o_sa, {sa + "output"}, d, d, true));
    TRY(pack_lin(c, Ly.q_ca, {ca + "query.0.linear"}, d, d, true));
    TRY(pack_lin(c, Ly.kv_ca, {ca + "key.0.linear", ca + "value.0.linear"}, d, d));
    TRY(pack_lin(c, Ly.o_ca, {ca + "output"}, d, d, true));
    TRY(pack_conv(c, Ly.sa_q, sa + "query.1", dk));
    TRY(pack_conv(c, Ly.sa_k, sa + "key.1", dk));
    TRY(pack_conv(c, Ly.sa_v, sa + "value.1", dk));
    TRY(pack_conv(c, Ly.ca_q, ca + "query.1", dk));
    TRY(pack_conv(c, Ly.ca_k, ca + "key.1", dk));
    TRY(pack_conv(c, Ly.ca_v, ca + "value.1", dk));
    TRY(pack_lin(c, Ly.ff1, {q + "feed_forward.layer1"}, 4 * d, d, true));
    TRY(pack_lin(c, Ly.ff2, {q + "feed_forward.layer2"}, d, 4 * d, true));
  }
  c->fused = D.decoder_type == GGD_DEC_ONEWAY && D.dtype != GGD_FP8W && D.model_type != GGD_MODEL_INPAINT &&
             fused_supported(D.dtype, D.d_model, D.heads, D.seq_len, D.speech_len, D.d_pose);
  if (c->fused) {
    TRY(frag_from(c, c->f_emb, {P + "emb_x"}, d, C, iota_n(d)));
    TRY(frag_from(c, c->f_out, {P + "out_layers.1"}, C, d, iota_n(C), P + "out_layers.0"));
    std::vector<int> head_major;  // per head h: q rows h*32.., k rows 256 + h*32.., v rows 512 + h*32..
    for (int h = 0; h < D.heads; ++h)
      for (int part = 0; part < 3; ++part)
        for (int i = 0; i < dk; ++i) head_major.push_back(part * d + h * dk + i);
    for (int l = 0; l < D.n_layers; ++l) {
      Layer& Ly = c->layers[l];
      const std::string q = P + "layers." + std::to_string(l) + ".";
      const std::string sa = q + "self_attn.", ca = q + "cross_attn.";
      TRY(frag_from(c, Ly.f_qkv, {sa + "query.0.linear", sa + "key.0.linear", sa + "value.0.linear"}, d, d,
                    head_major, q + "norm_self_attn"));
      TRY(frag_from(c, Ly.f_o_sa, {sa + "output"}, d, d, iota_n(d)));
      TRY(frag_from(c, Ly.f_q_ca, {ca + "query.0.linear"}, d, d, iota_n(d), q + "norm_cross_attn"));
      TRY(frag_from(c, Ly.f_o_ca, {ca + "output"}, d, d, iota_n(d)));
      TRY(frag_from(c, Ly.f_ff1, {q + "feed_forward.layer1"}, 4 * d, d, iota_n(4 * d), q + "norm_ff"));
      TRY(frag_from(c, Ly.f_ff2, {q + "feed_forward.layer2"}, d, 4 * d, iota_n(d)));
    }
  }
  if (c->fused) {  // convolved step-invariant cross-attention K / V images, filled by ggd_set_memory
    HIP_TRY(c, dalloc(c, &c->kvc, c->tsize * (size_t)D.n_layers * D.max_batch * D.heads * KVC_ELEMS));
    HIP_TRY(c, dalloc(c, &c->ffp, sizeof(float) * (size_t)D.max_batch * 8 * D.seq_len * D.d_model));
  }
  // row-block chains for the one-way generic route (ggd_chain.hip)
  const int on = c->out_lin.npad;
  c->chain = !c->fused && D.dtype != GGD_F32 && d == 256 && c->out_lin.kpad == 256 &&
             chain_p_supported(on) && chain_p_supported(3 * d) && chain_p_supported(d);
  for (int l = 0; c->chain && l < D.n_layers; ++l) {
    const Layer& Ly = c->layers[l];
    c->chain = Ly.qkv.npad == 3 * d && Ly.o_sa.npad == d && Ly.q_ca.npad == d && Ly.o_ca.npad == d &&
               Ly.ff1.npad == 4 * d && Ly.ff1.kpad == d && Ly.ff2.npad == d && Ly.ff2.kpad == 4 * d;
  }
  if (c->chain) {
    auto pack = [&](Lin& L) -> int {
      const int w8 = L.scale != nullptr;
      HIP_TRY(c, dalloc(c, &L.wf, chain_pack_bytes(w8, L.npad, L.kpad)));
      HIP_TRY(c, launch_chain_pack(w8, L.w, L.wf, L.npad, L.kpad, c->stream));
      return GGD_OK;
    };
    for (Layer& Ly : c->layers)
      for (Lin* L : {&Ly.qkv, &Ly.o_sa, &Ly.q_ca, &Ly.o_ca, &Ly.ff1, &Ly.ff2}) TRY(pack(*L));
    TRY(pack(c->out_lin));
    c->long_ok = D.model_type != GGD_MODEL_INPAINT && c->emb_x.npad == d && c->emb_x.kpad == d &&
                 long_loop_supported(D.dtype, d, D.heads, D.seq_len, D.speech_len, C, c->out_lin.npad);
    if (c->long_ok) {
      TRY(pack(c->emb_x));
      if (D.dtype == GGD_FP8W)  // the FFN / LN-projection weights the block-scaled stages read
        for (Layer& Ly : c->layers)
          for (Lin* L : {&Ly.qkv, &Ly.q_ca, &Ly.ff1, &Ly.ff2}) {
            HIP_TRY(c, dalloc(c, &L->wmx, chain_pack_bytes(1, L->npad, L->kpad)));
            HIP_TRY(c, launch_chain_pack(2, L->w, L->wmx, L->npad, L->kpad, c->stream));
          }
      HIP_TRY(c, dalloc(c, &c->long_kvc, D.n_layers * long_kv_cache_bytes(D.max_batch, D.speech_len, D.heads)));
    }
  }
  TRY(build_step_tables(c));
  c->persist = c->fused && persist_supported(D.dtype, D.d_model, D.heads, D.seq_len, D.speech_len, D.d_pose);
  if (c->persist) {
    std::vector<FusedLayer> fl(D.n_layers);
    for (int l = 0; l < D.n_layers; ++l) fl[l] = fused_layer(c, l);
    HIP_TRY(c, dalloc(c, &c->d_layers, sizeof(FusedLayer) * fl.size()));
    HIP_TRY(c, hipMemcpy(c->d_layers, fl.data(), sizeof(FusedLayer) * fl.size(), hipMemcpyHostToDevice));
  }
#undef TRY
  c->staged.clear();
  c->finalized = true;
  return GGD_OK;
}

int ggd_set_schedule(ggd_ctx* c, const double* betas, int32_t T, const int64_t* timestep_map) {
  if (!c || !betas || !timestep_map || T <= 0) return fail(c, GGD_ERR_ARG, "bad schedule");
  for (int i = 0; i < T; ++i) {
    if (!(betas[i] > 0.0 && betas[i] <= 1.0)) return fail(c, GGD_ERR_ARG, "betas must lie in (0, 1]");
    if (timestep_map[i] < 0 || timestep_map[i] >= c->desc.diffusion_steps)
      return fail(c, GGD_ERR_ARG, "timestep_map entry out of range");
  }
  c->betas.assign(betas, betas + T);
  c->tmap.assign(timestep_map, timestep_map + T);
  HIP_TRY(c, hipSetDevice(c->device));
  if (T > c->steps_cap) {
    HIP_TRY(c, dalloc(c, &c->d_steps, sizeof(StepRec) * T));
    c->steps_cap = T;
  }
  c->n_steps_T = T;
  return GGD_OK;
}

int ggd_set_memory(ggd_ctx* c, const float* tok, int32_t n, int32_t ts, int32_t dz, void* stream) {
  if (!c) return GGD_ERR_ARG;
  if (!c->finalized) return fail(c, GGD_ERR_STATE, "weights not finalized");
  const ggd_desc& D = c->desc;
  const int d = D.d_model;
  if (n <= 0 || n > D.max_batch) return fail(c, GGD_ERR_ARG, "batch exceeds max_batch");
  if (ts != D.speech_len) return fail(c, GGD_ERR_ARG, "speech length mismatch with descriptor");
  const int want_dz = D.model_type == GGD_MODEL_S2G_V2 ? 3 * d : d;
  if (dz != want_dz) return fail(c, GGD_ERR_ARG, "speech feature width mismatch");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  HIP_TRY(c, hipEventRecord(c->ev_in, (hipStream_t)stream));
  HIP_TRY(c, hipStreamWaitEvent(s, c->ev_in, 0));
  const int M = n * ts;
  const float* src = tok;
  GemmArgs g;
  if (D.model_type == GGD_MODEL_S2G_V2) {  // blend_layer (model.py:104-106)
    g = gemm_args(c->blend, M, tok, dz, c->tok_tmp, d);
    GEMM(c, PRO_F32, EPI_F32, g, s);
    src = c->tok_tmp;
  }
  if (c->twoway) {  // emb_mem + PE at joint positions L+1 .. L+Ts (nn.py:433-442), assembled per step
    g = gemm_args(c->emb_mem, M, src, d, c->mem_base, d);
    g.pe = c->pe;
    g.pe_period = ts;
    g.pe_offset = D.seq_len + 1;
    GEMM(c, PRO_F32, EPI_PE, g, s);
    HIP_TRY(c, hipEventRecord(c->ev_out, s));
    HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
    c->mem_n = n;
    return GGD_OK;
  }
  // emb_mem + PE at positions 1..Ts (row 0 is the step token), nn.py:223
  g = gemm_args(c->emb_mem, M, src, d, c->mem_tmp, d);
  g.pe = c->pe;
  g.pe_period = ts;
  g.pe_offset = 1;
  GEMM(c, PRO_F32, EPI_PE, g, s);
  for (int l = 0; l < D.n_layers; ++l) {
    g = gemm_args(c->layers[l].kv_ca, M, c->mem_tmp, d,
                  c->kv_mem + (size_t)l * D.max_batch * D.speech_len * 2 * d, 2 * d);
    GEMM(c, PRO_F32, EPI_F32, g, s);
  }
  if (c->fused) {  // the fused paths read the step-invariant K / V rows convolved, in image order
    const size_t per_layer = c->tsize * (size_t)D.max_batch * D.heads * KVC_ELEMS;
    for (int l = 0; l < D.n_layers; ++l) {
      const Layer& Ly = c->layers[l];
      HIP_TRY(c, launch_ca_kv_conv(D.dtype == GGD_F32 ? 0 : 1, c->kv_mem + (size_t)l * D.max_batch * D.speech_len * 2 * d,
                                   Ly.ca_k.w, Ly.ca_k.b, Ly.ca_v.w, Ly.ca_v.b, n, ts, (char*)c->kvc + per_layer * l, s));
    }
  }
  if (c->long_ok) {  // the long loop's convolved memory keys (2 ..) per layer
    for (int l = 0; l < D.n_layers; ++l) {
      const Layer& Ly = c->layers[l];
      HIP_TRY(c, launch_long_kv_cache(c->kv_mem + (size_t)l * D.max_batch * D.speech_len * 2 * d, Ly.ca_k.w, Ly.ca_k.b,
                                      Ly.ca_v.w, Ly.ca_v.b, n, D.speech_len,  D.heads,
                                      (bf16_t*)((char*)c->long_kvc + l * long_kv_cache_bytes(D.max_batch, D.speech_len, D.heads)), s));
    }
  }
  HIP_TRY(c, hipEventRecord(c->ev_out, s));
  HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
  c->mem_n = n;
  return GGD_OK;
}

int ggd_set_inpaint(ggd_ctx* c, const float* poses, const float* masks, int32_t n, void* stream) {
  if (!c) return GGD_ERR_ARG;
  if (c->desc.model_type != GGD_MODEL_INPAINT) return fail(c, GGD_ERR_UNSUPPORTED, "not an inpaint model");
  if (!c->finalized) return fail(c, GGD_ERR_STATE, "weights not finalized");
  if (!poses) {
    c->inp_on = false;
    return GGD_OK;
  }
  if (!masks || n <= 0 || n > c->desc.max_batch) return fail(c, GGD_ERR_ARG, "bad inpaint arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const ggd_desc& D = c->desc;
  const int M = n * D.seq_len, d = D.d_model, C = D.d_pose;
  HIP_TRY(c, hipEventRecord(c->ev_in, (hipStream_t)stream));
  HIP_TRY(c, hipStreamWaitEvent(s, c->ev_in, 0));
  HIP_TRY(c, launch_inpaint_input(c->inp_in, poses, masks, M, C, s));
  GemmArgs g = gemm_args(c->inp0, M, c->inp_in, C + 1, c->inp_h1, d);
  GEMM(c, PRO_F32, EPI_SILU, g, s);
  g = gemm_args(c->inp2, M, c->inp_h1, d, c->inp_h2, d);
  GEMM(c, PRO_F32, EPI_SILU, g, s);
  g = gemm_args(c->inp4, M, c->inp_h2, d, c->inp_delta, C);
  GEMM(c, PRO_F32, EPI_F32, g, s);
  c->inp_on = true;
  HIP_TRY(c, hipEventRecord(c->ev_out, s));
  HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
  return GGD_OK;
}

int ggd_denoise(ggd_ctx* c, const float* x_t, const int32_t* t, float* eps, int32_t n, void* stream) {
  if (!c || !x_t || !t || !eps) return fail(c, GGD_ERR_ARG, "null pointer");
  if (!c->finalized) return fail(c, GGD_ERR_STATE, "weights not finalized");
  if (n != c->mem_n) return fail(c, GGD_ERR_STATE, "batch differs from the installed speech memory");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const ggd_desc& D = c->desc;
  HIP_TRY(c, hipEventRecord(c->ev_in, (hipStream_t)stream));
  HIP_TRY(c, hipStreamWaitEvent(s, c->ev_in, 0));
  HIP_TRY(c, launch_init_state(c->x, x_t, 0, 0, n, D.d_pose, D.seq_len, s));
  if (c->fused) {
    int r = launch_decoder(c, n, false, t);  // layer 0's KA embeds x_t
    if (r) return r;
    FinalArgs f = final_args(c, n);
    f.do_out = 1;  // LN_out + out-proj -> eps in (N, C, L)
    f.eps_out = eps;
    HIP_TRY(c, launch_final(D.dtype, f, s));
  } else {
    int r = launch_decoder(c, n, false, t);
    if (r) return r;
    HIP_TRY(c, launch_nlc_to_ncl(eps, c->eps, n, D.d_pose, D.seq_len, c->cpad, s));
  }
  HIP_TRY(c, hipEventRecord(c->ev_out, s));
  HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
  return GGD_OK;
}

int ggd_posterior_step(ggd_ctx* c, int32_t alg, float eta, int32_t i, const float* x, const float* eps,
                       const float* x0, const float* noise, float* x_out, float* x0_out, int32_t n,
                       void* stream) {
  if (!c || !x || !eps || !noise) return fail(c, GGD_ERR_ARG, "null pointer");
  if (c->betas.empty()) return fail(c, GGD_ERR_STATE, "no schedule installed");
  if (alg != GGD_DDPM && alg != GGD_DDIM) return fail(c, GGD_ERR_UNSUPPORTED, "unsupported sample algorithm");
  const int T = (int)c->betas.size();
  if (i < 0 || i >= T) return fail(c, GGD_ERR_ARG, "step index out of range");
  std::vector<StepRec> recs;
  make_records(c, alg, eta, recs);
  PostArgs p{};
  p.n = n;
  p.C = c->desc.d_pose;
  p.L = c->desc.seq_len;
  p.alg = alg;
  p.rec = recs[T - 1 - i];
  p.x = x;
  p.eps = eps;
  p.x0 = x0;
  p.noise = noise;
  p.x_out = x_out;
  p.x0_out = x0_out;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, launch_posterior(p, (hipStream_t)stream));
  return GGD_OK;
}

int ggd_set_profiling(ggd_ctx* c, int32_t on) {
  if (!c) return GGD_ERR_ARG;
  c->profiling = on != 0;
  return GGD_OK;
}

int ggd_profile_kind(ggd_ctx* c) { return c ? c->prof_kind : GGD_ERR_ARG; }

int ggd_kernel_time(ggd_ctx* c, int32_t which, double* avg_us, int64_t* launches) {
  if (!c || !avg_us || !launches || which != 0) return fail(c, GGD_ERR_ARG, "bad argument");
  if (c->prof_lazy) {  // a non-blocking loop's event pair: read once both have completed
    c->prof_lazy = false;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipEventSynchronize(c->prof.ev[1]));
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->prof.ev[0], c->prof.ev[1]));
    c->prof_avg_us = ms * 1000.0 / std::max(1, c->prof_lazy_div);
    int r = poll_pending(c, true);
    if (r) return r;
    if (c->gated_ran)  // the timed span holds a loop that never ran; its untimed fallback made the result
      return fail(c, GGD_ERR_STATE, "profiled loop did not run (workgroups not all resident): no kernel time");
  }
  if (c->span_pending) {  // launch span = latest workgroup end - earliest workgroup start
    const size_t n = c->span_pending, wg = c->span_wg;
    c->span_pending = 0;
    std::vector<unsigned long long> h(n);
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->span, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    double total = 0;
    int64_t cnt = 0;
    for (size_t slot = 0; slot < n / (2 * wg); ++slot) {
      const unsigned long long* b = h.data() + slot * 2 * wg;
      unsigned long long lo = ~0ull, hi = 0;
      bool full = true;
      for (size_t w = 0; w < wg; ++w) {
        full = full && b[w] && b[wg + w];
        lo = std::min(lo, b[w]);
        hi = std::max(hi, b[wg + w]);
      }
      if (full && hi >= lo) {
        total += (double)(hi - lo) / c->wall_mhz;
        ++cnt;
      }
    }
    c->prof_avg_us = cnt ? total / cnt : 0;
    c->prof_launches = cnt;
  }
  *avg_us = c->prof_avg_us;
  *launches = c->prof_launches;
  return GGD_OK;
}

// Clips one clip-group launch holds on this context's shape (0: no clip-group loop runs it): f32 (the
// parity mode) the head / chunk loop (ggd_mega.hip mk_kernel), bf16 the row-block loop (ggd_rows.hip
// mr_kernel; round 6: 69.2 vs 75.1 ms per C2 pass, so the bf16 head / chunk loop was removed) where
// its shape limits hold.  sampling: also honour the per-phase-launch switch (ggd_diag what = 9).
static int group_capacity(const ggd_ctx* c, bool sampling) {
  const ggd_desc& D = c->desc;
  if (!c->fused || (sampling && c->no_mega)) return 0;
  if (D.dtype != 0 && !(c->kvc && rows_supported(D.dtype, D.seq_len, D.speech_len))) return 0;
  return mega_capacity(D.dtype, D.seq_len);
}

int ggd_set_route(ggd_ctx* c, int32_t knob, int32_t value) {
  if (!c) return GGD_ERR_ARG;
  switch (knob) {
    case GGD_ROUTE_PER_CLIP:  // 0 auto, 1 never, 2 always the one-workgroup / clip-pair loops
      if (value < 0 || value > 2) break;
      c->persist_mode = value;
      return GGD_OK;
    case GGD_ROUTE_PAIR:      // 0 auto, 1 never, 2 always two workgroups per clip (per-clip loops)
      if (value < 0 || value > 2) break;
      c->pair_mode = value;
      return GGD_OK;
    case GGD_ROUTE_PAIR_WRITE_THROUGH:
      c->pair_force_coh = value != 0;
      return GGD_OK;
    case GGD_ROUTE_PHASE_LAUNCHES:  // 1: per-phase launches instead of the persistent clip-group loop
      c->no_mega = value != 0;
      return GGD_OK;
    case GGD_ROUTE_PLACEMENT:       // clip-group loop: 0 XCD-local, 1 part p on XCD p, 2 group per XCD
      if (value < 0 || value > 2) break;
      c->mega_place = value;
      return GGD_OK;
    case GGD_ROUTE_GEMM_LAUNCHES:   // 1: one launch per GEMM instead of the row-block chains
      c->gemm_launches = value != 0;
      return GGD_OK;
    case GGD_ROUTE_ATTN_QSPLIT:     // 1: long clips on the query-split attention kernel
      c->attn_qsplit = value != 0;
      return GGD_OK;
    case GGD_ROUTE_LONG_LOOP:       // 1: never the long-clip persistent loop
      c->long_off = value != 0;
      return GGD_OK;
    case GGD_ROUTE_FP8_MFMA:        // 1: the long loop's e4m3 weights widened into bf16 MFMAs
      c->fp8_mfma_off = value != 0;
      return GGD_OK;
    case GGD_ROUTE_SIMULATE_UNRESIDENT:  // test hook: 1 co-resident loops report status 2, run nothing;
      if (value < 0 || value > 2) break;  // 2 only odd parts do, the rest wait in a barrier
      c->sim_unresident = value;
      return GGD_OK;
    default:
      break;
  }
  return fail(c, GGD_ERR_ARG, "unknown route knob or value");
}

int ggd_route_info(ggd_ctx* c, int32_t what, double* out) {
  if (!c || !out) return GGD_ERR_ARG;
  if (what == GGD_INFO_XL_LAUNCHES || what == GGD_INFO_WT_RERUNS || what == GGD_INFO_GATED_FALLBACKS) {
    // counters of a deferred check
    HIP_TRY(c, hipSetDevice(c->device));
    int r = poll_pending(c, true);
    if (r) return r;
  }
  switch (what) {
    case GGD_INFO_PER_CLIP_AVAILABLE: *out = c->persist ? 1.0 : 0.0; return GGD_OK;
    case GGD_INFO_LOOP_CAPACITY: *out = (double)group_capacity(c, false); return GGD_OK;
    case GGD_INFO_PAIR_LAUNCHES: *out = c->pair_launches; return GGD_OK;
    case GGD_INFO_XL_LAUNCHES: *out = c->mega_xl_launches; return GGD_OK;
    case GGD_INFO_WT_RERUNS: *out = c->mega_fallbacks; return GGD_OK;
    case GGD_INFO_CHAIN_AVAILABLE: *out = c->chain ? 1.0 : 0.0; return GGD_OK;
    case GGD_INFO_LONG_LAUNCHES: *out = c->long_launches; return GGD_OK;
    case GGD_INFO_CLIP_ATTN_LAUNCHES: *out = (double)c->clip_attn_launches; return GGD_OK;
    case GGD_INFO_GATED_FALLBACKS: *out = (double)c->gated_ran; return GGD_OK;
    case GGD_INFO_ROWS_LOOP: *out = c->mega_rows_last ? 1.0 : 0.0; return GGD_OK;
    case GGD_INFO_BARRIER_TIMEOUTS: *out = (double)c->barrier_timeouts; return GGD_OK;
    default: return fail(c, GGD_ERR_ARG, "unknown route info");
  }
}

#ifdef GGD_DIAG
int ggd_diag(ggd_ctx* c, int32_t what, const int32_t* p, int32_t np, int32_t iters, double* avg_us) {
  if (!c || !p || !avg_us || iters <= 0) return fail(c, GGD_ERR_ARG, "bad argument");
  HIP_TRY(c, hipSetDevice(c->device));
  if (what == 10 && np >= 1) {  // persistent-loop barrier stamps: {1} arm, {2} read, {0} off
    // [0, B): workgroup 0's (done, passed) per barrier; [B]: its loop start; then raw 100 MHz
    // real-time stamps of the arrival and exit of each of clip group 0's 8 workgroups at every
    // barrier ([barrier][part][2], returned as ticks)
    const int B = 2 * 17 * MEGA_STAMP_STEPS, NS = B + 1 + 16 * 17 * MEGA_STAMP_STEPS;
    if (p[0] == 1) {
      if (!c->mega_stamps) HIP_TRY(c, dalloc(c, &c->mega_stamps, NS * sizeof(unsigned long long)));
      HIP_TRY(c, hipMemset(c->mega_stamps, 0, NS * sizeof(unsigned long long)));
    }
    if (p[0] == 2 && c->mega_stamps) {  // avg_us[j] = us from the loop start to stamp j (j != B)
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      std::vector<unsigned long long> h(NS);
      HIP_TRY(c, hipMemcpy(h.data(), c->mega_stamps, NS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      const int n_out = std::min(NS, np >= 2 ? p[1] : B);
      for (int j = 0; j < n_out; ++j)
        avg_us[j] = j > B ? (double)h[j] : j == B ? 0.0 : h[j] ? ((double)h[j] - (double)h[B]) / 2400.0 : -1.0;
    }
    if (p[0] == 0) c->mega_stamps = nullptr;  // stays owned by the ctx allocation list
    return GGD_OK;
  }
  if (what == 16 && np >= 1) {  // long-clip loop barrier stamps: {1} arm, {2} read, {0} off
    if (p[0] == 1) {
      if (!c->long_stamps) HIP_TRY(c, dalloc(c, &c->long_stamps, LONG_STAMPS * sizeof(unsigned long long)));
      HIP_TRY(c, hipMemset(c->long_stamps, 0, LONG_STAMPS * sizeof(unsigned long long)));
    }
    if (p[0] == 2 && c->long_stamps) {  // avg_us[j] = us from the loop start to barrier j (-1: not stamped)
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      std::vector<unsigned long long> h(LONG_STAMPS);
      HIP_TRY(c, hipMemcpy(h.data(), c->long_stamps, LONG_STAMPS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      for (int j = 0; j < LONG_STAMPS; ++j) avg_us[j] = h[j] && h[0] ? (double)(h[j] - h[0]) / c->wall_mhz : -1.0;
    }
    if (p[0] == 0) c->long_stamps = nullptr;
    return GGD_OK;
  }
  if (what == 11 && np >= 1) {  // persistent-loop phase stamps of layer 1 + KE: {1} arm, {2} read, {0} off
    if (p[0] == 1) {
      if (!c->mega_phase_stamps) HIP_TRY(c, dalloc(c, &c->mega_phase_stamps, 80 * sizeof(unsigned long long)));
      HIP_TRY(c, hipMemset(c->mega_phase_stamps, 0, 80 * sizeof(unsigned long long)));
    }
    if (p[0] == 2 && c->mega_phase_stamps) {  // avg_us[16 j + i] = us from phase j's stamp 0 to its stamp i
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      unsigned long long h[80];
      HIP_TRY(c, hipMemcpy(h, c->mega_phase_stamps, sizeof h, hipMemcpyDeviceToHost));
      for (int j = 0; j < 5; ++j)
        for (int i = 0; i < 16; ++i)
          avg_us[16 * j + i] = (h[16 * j] && h[16 * j + i] >= h[16 * j]) ? (double)(h[16 * j + i] - h[16 * j]) / 2400.0 : -1.0;
    }
    if (p[0] == 0) c->mega_phase_stamps = nullptr;
    return GGD_OK;
  }
  if (what == 12 && np >= 1) {  // persistent-loop placement: {0} XCD-local clip groups (CP_XL, default),
                                // {1} part p on XCD p (write-through), {2} clip group per XCD (write-through)
    c->mega_place = p[0] >= 0 && p[0] <= 2 ? p[0] : 0;
    *avg_us = c->mega_place;
    return GGD_OK;
  }
  if (what == 14 && np >= 1) {  // clip pairs: {0} auto, {1} never, {2} always (persistent per-clip route)
    c->pair_mode = p[0] >= 0 && p[0] <= 2 ? p[0] : 0;
    c->pair_force_coh = np >= 2 && p[1] != 0;
    *avg_us = c->pair_launches;
    return GGD_OK;
  }
  if (what == 15) {  // last ggd_sample: clip-pair launches
    *avg_us = c->pair_launches;
    return GGD_OK;
  }
  if (what == 13) {  // last ggd_sample: [XCD-local launches, write-through re-runs]
    avg_us[0] = c->mega_xl_launches;
    if (iters > 1) avg_us[1] = c->mega_fallbacks;
    return GGD_OK;
  }
  if (what == 9 && np >= 1) {  // p[0] != 0: sample through the per-phase launches, not the persistent loop
    c->no_mega = p[0] != 0;
    *avg_us = (double)group_capacity(c, false);
    return GGD_OK;
  }
  if (what == 7 && np >= 1) {  // p[0] != 0: route ggd_sample through the per-step launches
    c->persist_mode = p[0] == 0 ? 2 : p[0] == 1 ? 1 : 0;
    *avg_us = c->persist ? 1.0 : 0.0;
    return GGD_OK;
  }
  if (what == 8 && np >= 1) {  // persistent-kernel phase stamps: 1 arm, 2 read (8 deltas, us), 0 off
    if (p[0] == 1 && !c->stamps) HIP_TRY(c, dalloc(c, &c->stamps, 64 * sizeof(unsigned long long)));
    if (p[0] == 1) HIP_TRY(c, hipMemset(c->stamps, 0, 64 * sizeof(unsigned long long)));
    if (p[0] == 2 && c->stamps) {
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      unsigned long long h[17];
      HIP_TRY(c, hipMemcpy(h, c->stamps, sizeof h, hipMemcpyDeviceToHost));
      for (int i = 0; i < 16; ++i)
        avg_us[i] = (h[0] && h[i + 1] >= h[0]) ? (double)(h[i + 1] - h[0]) / 2400.0 : -1.0;
    }
    if (p[0] == 0) c->stamps = nullptr;  // the buffer stays owned by the ctx allocation list
    return GGD_OK;
  }
  hipStream_t s = c->stream;
  const ggd_desc& D = c->desc;
  const int d = D.d_model;
  hipEvent_t e0, e1;
  HIP_TRY(c, hipEventCreate(&e0));
  HIP_TRY(c, hipEventCreate(&e1));
  std::vector<void*> tmp;
  auto talloc = [&](size_t bytes) -> void* {
    void* v = nullptr;
    if (hipMalloc(&v, bytes) != hipSuccess) return nullptr;
    (void)hipMemset(v, 0x3c, bytes);  // small finite values in f32 and bf16
    (void)hipDeviceSynchronize();     // ordered before work on the (non-blocking) ctx stream
    tmp.push_back(v);
    return v;
  };
  int rc = GGD_OK;
  float ms = 0.f;
  if (what == 0 && np >= 7) {
    GemmArgs g{};
    const int pro = p[0], epi = p[1];
    g.M = p[2]; g.N = p[3]; g.K = p[4]; g.force_mt = p[5]; g.no_xcd_remap = p[6];
    g.k_valid = g.K;
    const size_t asz = (pro == PRO_T ? c->tsize : 4) * (size_t)g.M * g.K;
    g.A = talloc(asz);
    g.lda = g.K;
    g.W = talloc(c->tsize * (size_t)g.N * g.K);
    g.bias = (float*)talloc(4 * (size_t)g.N);
    g.ln_g = (float*)talloc(4 * (size_t)g.K);
    g.ln_b = (float*)talloc(4 * (size_t)g.K);
    g.out = talloc(4 * (size_t)g.M * g.N);
    g.ldo = g.N;
    g.n_valid = g.N;
    g.pe = c->pe;
    g.pe_period = 1;
    if (!g.A || !g.W || !g.out) rc = fail(c, GGD_ERR_HIP, "diag alloc");
    for (int it = 0; rc == GGD_OK && it < iters + 1; ++it) {
      if (it == 1) HIP_TRY(c, hipEventRecord(e0, s));
      GEMM(c, pro, epi, g, s);
    }
  } else if (what == 1 && np >= 2) {
    const int n = p[1];
    if (n > D.max_batch) rc = fail(c, GGD_ERR_ARG, "n > max_batch");
    AttnArgs at{};
    at.zero = c->zero_row;
    at.no_clip = c->attn_qsplit;
  at.no_clip = c->attn_qsplit;
    const Layer& Ly = c->layers[0];
    at.cross = p[0];
    at.q = c->qkv; at.ldq = 3 * d;
    at.k = (const char*)c->qkv + c->tsize * d;
    at.v = (const char*)c->qkv + c->tsize * 2 * d;
    at.ldkv = 3 * d;
    at.kv_mem = c->kv_mem;
    at.kv_step = c->kv_step;
    at.t_clip = c->d_t;
    at.cw_q = Ly.sa_q.w; at.cb_q = Ly.sa_q.b;
    at.cw_k = Ly.sa_k.w; at.cb_k = Ly.sa_k.b;
    at.cw_v = Ly.sa_v.w; at.cb_v = Ly.sa_v.b;
    at.out = c->att; at.ldo = d;
    at.Lq = D.seq_len;
    at.Lk = at.cross ? 1 + D.speech_len : D.seq_len;
    at.dk = d / D.heads; at.heads = D.heads; at.d = d;
    at.scale = 1.0f / std::sqrt((float)at.dk);
    at.no_qsplit = np >= 3 ? p[2] : 0;
    for (int it = 0; rc == GGD_OK && it < iters + 1; ++it) {
      if (it == 1) HIP_TRY(c, hipEventRecord(e0, s));
      HIP_TRY(c, run_attention(c, D.dtype, at, n, s));
    }
  } else if ((what == 2 || what == 3) && np >= 1) {
    const int n = p[0];
    if (n > D.max_batch || c->betas.empty()) rc = fail(c, GGD_ERR_STATE, "need schedule and n <= max_batch");
    ggd_sample_args sa{};
    sa.alg = GGD_DDPM;
    sa.n = n;
    std::vector<StepRec> recs;
    if (rc == GGD_OK) {
      make_records(c, GGD_DDPM, 0.f, recs);
      upload_forget(c, c->d_steps);
      HIP_TRY(c, hipMemcpyAsync(c->d_steps, recs.data(), sizeof(StepRec) * recs.size(), hipMemcpyHostToDevice, s));
      HIP_TRY(c, launch_init_state(c->x, nullptr, 1, 0, n, D.d_pose, D.seq_len, s));
    }
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    if (rc == GGD_OK && what == 3) {
      HIP_TRY(c, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      rc = launch_step(c, sa, nullptr, -1);
      hipError_t e = hipStreamEndCapture(s, &g);
      if (rc == GGD_OK && e != hipSuccess) rc = fail(c, GGD_ERR_HIP, "capture");
      if (rc == GGD_OK) HIP_TRY(c, hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    const int T = (int)recs.size();
    for (int it = 0; rc == GGD_OK && it < iters + 1; ++it) {
      if (it % T == 0) HIP_TRY(c, launch_set_int(c->d_counter, -1, s));
      if (it == 1) HIP_TRY(c, hipEventRecord(e0, s));
      if (what == 3)
        HIP_TRY(c, hipGraphLaunch(ge, s));
      else
        rc = launch_step(c, sa, nullptr, -1);
    }
    if (ge) (void)hipGraphExecDestroy(ge);
    if (g) (void)hipGraphDestroy(g);
  } else if ((what == 4 || what == 6) && np >= 2 && c->fused) {
    const int which = p[0], n = p[1];
    unsigned long long* st = what == 6 ? (unsigned long long*)talloc(64 * 8) : nullptr;
    if (what == 6) iters = 1;
    if (n > D.max_batch || c->betas.empty()) rc = fail(c, GGD_ERR_STATE, "need schedule and n <= max_batch");
    std::vector<StepRec> recs;
    if (rc == GGD_OK) {
      make_records(c, GGD_DDPM, 0.f, recs);
      upload_forget(c, c->d_steps);
      HIP_TRY(c, hipMemcpyAsync(c->d_steps, recs.data(), sizeof(StepRec) * recs.size(), hipMemcpyHostToDevice, s));
      HIP_TRY(c, launch_set_int(c->d_counter, 0, s));
    }
    for (int it = 0; rc == GGD_OK && it < iters + 1; ++it) {
      if (it == 1) HIP_TRY(c, hipEventRecord(e0, s));
      if (which < 4) {
        // the layer-0 arguments of launch_fused_layers
        FusedArgs f{};
        f.w = fused_layer(c, 0);
        f.L = D.seq_len; f.Ts = D.speech_len;
        f.o_sa = c->att; f.o_ca = c->q; f.hid = c->ffn; f.ffp = c->ffp;
        f.steps = c->d_steps; f.step_counter = c->d_counter;
        f.scale = 1.0f / std::sqrt((float)(d / D.heads));
        f.h = c->h; f.h_out = c->h2;
        f.stamps = it == iters ? st : nullptr;
        HIP_TRY(c, launch_fused(which, D.dtype, f, n, s));
      } else {
        FinalArgs f = final_args(c, n);
        f.do_out = 1; f.do_update = 1;
        f.stamps = it == iters ? st : nullptr;
        HIP_TRY(c, launch_final(D.dtype, f, s));
      }
    }
    if (rc == GGD_OK && what == 6) {  // avg_us -> 8 phase deltas in microseconds (2.4 GHz-independent: s_memtime ticks / 2400)
      (void)hipMemset(st, 0, 0);
      HIP_TRY(c, hipStreamSynchronize(s));
      unsigned long long h_st[16];
      HIP_TRY(c, hipMemcpy(h_st, st, sizeof h_st, hipMemcpyDeviceToHost));
      for (int i = 0; i < 8; ++i) avg_us[i] = (h_st[i + 1] > h_st[0] && h_st[i + 1] < h_st[0] + 100000000ull) ? (h_st[i + 1] - h_st[0]) / 2400.0 : -1.0;
      for (void* v : tmp) (void)hipFree(v);
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      return GGD_OK;
    }
  } else if (what == 5 && np >= 4) {
    // calibration micro-kernels: p = {mode, arg, blocks, buffer MiB}
    const int mode = p[0], arg = p[1], blocks = p[2];
    const size_t bytes = (size_t)p[3] << 20;
    void* buf = talloc(bytes);
    if (!buf) rc = fail(c, GGD_ERR_HIP, "diag alloc");
    if (rc == GGD_OK && mode == 1) {  // chase ring: jump ~1 MiB + 64 B per step through the buffer
      const size_t n = bytes / 4 - 16;
      std::vector<int> nx(n);
      const size_t stride = (size_t)(1 << 18) + 16;
      for (size_t i = 0; i < n; ++i) nx[i] = (int)((i + stride) % n);
      HIP_TRY(c, hipMemcpy(buf, nx.data(), 4 * n, hipMemcpyHostToDevice));
    }
    if (rc == GGD_OK && mode == 6) HIP_TRY(c, hipMemsetAsync((char*)buf + 4000, 0, 96, s));  // hand-off stats
    for (int it = 0; rc == GGD_OK && it < iters + 1; ++it) {
      if (it == 1) HIP_TRY(c, hipEventRecord(e0, s));
      HIP_TRY(c, launch_mb(mode, buf, bytes, arg, blocks, s));
    }
    if (rc == GGD_OK && mode == 2) {
      HIP_TRY(c, hipEventRecord(e1, s));
      HIP_TRY(c, hipEventSynchronize(e1));
      unsigned long long st[3];
      HIP_TRY(c, hipMemcpy(st, buf, sizeof st, hipMemcpyDeviceToHost));
      *avg_us = st[1] ? (double)st[0] / ((double)st[1] / 100.0) / 1000.0 : 0.0;  // GHz
      (void)hipStreamSynchronize(s);
      for (void* v : tmp) (void)hipFree(v);
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      return GGD_OK;
    }
  } else {
    rc = fail(c, GGD_ERR_ARG, "unknown diagnostic");
  }
  if (rc == GGD_OK) {
    HIP_TRY(c, hipEventRecord(e1, s));
    HIP_TRY(c, hipEventSynchronize(e1));
    HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
    *avg_us = ms * 1000.0 / iters;
    if (what == 5 && np >= 4 && p[0] == 6) {  // avg_us[1..3] = errors, misplaced, timeouts (all launches)
      unsigned st[3];
      HIP_TRY(c, hipMemcpy(st, (char*)tmp.back() + 4000, sizeof st, hipMemcpyDeviceToHost));
      for (int i = 0; i < 3; ++i) avg_us[1 + i] = st[i];
    }
  }
  (void)hipStreamSynchronize(s);
  for (void* v : tmp) (void)hipFree(v);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return rc;
}

#endif  // GGD_DIAG

}  // extern "C"

namespace {

// Tables of the long-clip loop (ggd_long.hip): per layer its chain-route weights, conv taps and
// memory K|V; the chain stages [loop start: emb_x, QKV] + per layer [A: o_sa, q_ca | B: o_ca,
// ff1, ff2, next QKV or out_layers, emb_x, layer 0's QKV].
int long_tables(ggd_ctx* c) {
  const ggd_desc& D = c->desc;
  const int NL = D.n_layers, d = D.d_model;
  if (c->long_layers) return GGD_OK;
  std::vector<LongLayer> ly(NL);
  std::vector<ChainStage> st(2 + LONG_STAGES_PER_LAYER * NL, ChainStage{});
  auto stage = [&](int i, const Lin& w, const float* g, const float* b, void* out, int ldo) {
    st[i].w = chain_lin(w);
    st[i].ln_g = g;
    st[i].ln_b = b;
    st[i].out = out;
    st[i].ldo = ldo;
  };
  stage(0, c->emb_x, nullptr, nullptr, nullptr, 0);
  stage(1, c->layers[0].qkv, c->layers[0].ln1_g, c->layers[0].ln1_b, c->qkv, 3 * d);
  for (int li = 0; li < NL; ++li) {
    const Layer& Y = c->layers[li];
    LongLayer& L = ly[li];
    L.qkv = chain_lin(Y.qkv); L.o_sa = chain_lin(Y.o_sa); L.q_ca = chain_lin(Y.q_ca);
    L.o_ca = chain_lin(Y.o_ca); L.ff1 = chain_lin(Y.ff1); L.ff2 = chain_lin(Y.ff2);
    L.ln1_g = Y.ln1_g; L.ln1_b = Y.ln1_b; L.ln2_g = Y.ln2_g; L.ln2_b = Y.ln2_b; L.ln3_g = Y.ln3_g; L.ln3_b = Y.ln3_b;
    L.sa_qw = Y.sa_q.w; L.sa_qb = Y.sa_q.b; L.sa_kw = Y.sa_k.w; L.sa_kb = Y.sa_k.b; L.sa_vw = Y.sa_v.w; L.sa_vb = Y.sa_v.b;
    L.ca_qw = Y.ca_q.w; L.ca_qb = Y.ca_q.b; L.ca_kw = Y.ca_k.w; L.ca_kb = Y.ca_k.b; L.ca_vw = Y.ca_v.w; L.ca_vb = Y.ca_v.b;
    L.kv_mem = c->kv_mem + (size_t)li * D.max_batch * D.speech_len * 2 * d;
    L.kv_step = c->kv_step + (size_t)li * D.diffusion_steps * 2 * d;
    L.kvc = (const bf16_t*)((const char*)c->long_kvc + li * long_kv_cache_bytes(D.max_batch, D.speech_len, D.heads));
    const int b0 = 2 + LONG_STAGES_PER_LAYER * li;
    stage(b0 + 0, Y.o_sa, nullptr, nullptr, nullptr, 0);
    stage(b0 + 1, Y.q_ca, Y.ln2_g, Y.ln2_b, c->q, d);
    stage(b0 + 2, Y.o_ca, nullptr, nullptr, nullptr, 0);
    stage(b0 + 3, Y.ff1, Y.ln3_g, Y.ln3_b, nullptr, 0);
    stage(b0 + 4, Y.ff2, nullptr, nullptr, nullptr, 0);
    if (li + 1 < NL) {
      stage(b0 + 5, c->layers[li + 1].qkv, c->layers[li + 1].ln1_g, c->layers[li + 1].ln1_b, c->qkv, 3 * d);
    } else {
      stage(b0 + 5, c->out_lin, c->out_ln_g, c->out_ln_b, nullptr, 0);
      stage(b0 + 6, c->emb_x, nullptr, nullptr, nullptr, 0);
      stage(b0 + 7, c->layers[0].qkv, c->layers[0].ln1_g, c->layers[0].ln1_b, c->qkv, 3 * d);
    }
  }
  if (D.dtype == GGD_FP8W) {  // the same table with the block-scaled stages' weights on their MX copies
    std::vector<ChainStage> mx = st;
    auto use = [&](int i, const Lin& w) { mx[i].w.w = w.wmx; };
    use(1, c->layers[0].qkv);
    for (int li = 0; li < NL; ++li) {
      const int b0 = 2 + LONG_STAGES_PER_LAYER * li;
      use(b0 + 1, c->layers[li].q_ca);
      use(b0 + 3, c->layers[li].ff1);
      use(b0 + 4, c->layers[li].ff2);
      if (li + 1 < NL) use(b0 + 5, c->layers[li + 1].qkv);
      else use(b0 + 7, c->layers[0].qkv);
    }
    for (const ChainStage& x : mx)
      if (x.w.scale && !x.w.w) return fail(c, GGD_ERR_STATE, "long-clip loop: missing block-scaled weight copy");
    HIP_TRY(c, dalloc(c, &c->long_stages_mx, sizeof(ChainStage) * mx.size()));
    HIP_TRY(c, hipMemcpy(c->long_stages_mx, mx.data(), sizeof(ChainStage) * mx.size(), hipMemcpyHostToDevice));
  }
  HIP_TRY(c, dalloc(c, &c->long_layers, sizeof(LongLayer) * NL));
  HIP_TRY(c, dalloc(c, &c->long_stages, sizeof(ChainStage) * st.size()));
  HIP_TRY(c, dalloc(c, &c->long_ctl, sizeof(unsigned) * LONG_CTL_WORDS));
  HIP_TRY(c, dalloc(c, &c->long_status, sizeof(int) * MEGA_MAX_CHUNKS));
  HIP_TRY(c, hipMemcpy(c->long_layers, ly.data(), sizeof(LongLayer) * NL, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMemcpy(c->long_stages, st.data(), sizeof(ChainStage) * st.size(), hipMemcpyHostToDevice));
  return GGD_OK;
}

// The first `nsteps` iterations of a long-clip batch in the persistent loop (ggd_long.hip), one
// launch per `long_loop_capacity()` clips.  The first step's emb_x + PE and LN1 + QKV run as
// launches in front (every later step's run inside the loop).  Returns 1 when the loop could not
// be placed (status 3: nothing ran; the caller takes the launch route), after a host sync.
int run_long(ggd_ctx* c, const ggd_sample_args& a, int nsteps) {
  const ggd_desc& D = c->desc;
  const int L = D.seq_len, d = D.d_model, M = a.n * L;
  hipStream_t s = c->stream;
  int r = long_tables(c);
  if (r) return r;
  const int cap = long_loop_capacity(), chunks = (a.n + cap - 1) / cap;
  if (chunks > MEGA_MAX_CHUNKS) return fail(c, GGD_ERR_ARG, "batch too large for the long-clip loop");
  GemmArgs g = gemm_args(c->emb_x, M, c->x, D.d_pose, c->h, d);
  g.pe = c->pe;
  g.pe_period = L;
  g.pe_offset = 0;
  GEMM(c, PRO_F32, EPI_PE, g, s);
  ChainArgs c0{};
  c0.M = M;
  c0.h = c->h;
  c0.p_g = c->layers[0].ln1_g;
  c0.p_b = c->layers[0].ln1_b;
  c0.p = chain_lin(c->layers[0].qkv);
  c0.out = c->qkv;
  c0.ldo = 3 * d;
  HIP_TRY(c, launch_chain(D.dtype == GGD_FP8W, c0, s));
  HIP_TRY(c, hipMemsetAsync(c->long_status, 0, sizeof(int) * MEGA_MAX_CHUNKS, s));
  if (c->profiling) {
    c->prof.next = 0;
    if ((r = prof_mark(c, s))) return r;
  }
  for (int c0i = 0, ci = 0; c0i < a.n; c0i += cap, ++ci) {
    LongArgs la{};
    la.layers = c->long_layers;
    const bool mx = D.dtype == GGD_FP8W && !c->fp8_mfma_off;
    la.stages = mx ? c->long_stages_mx : c->long_stages;
    la.n_layers = D.n_layers;
    la.n = a.n;
    la.L = L;
    la.Ts = D.speech_len;
    la.C = D.d_pose;
    la.alg = a.alg;
    la.k0 = 0;
    la.n_steps = nsteps;
    la.clip0 = c0i;
    la.emb = chain_lin(c->emb_x);
    la.out = chain_lin(c->out_lin);
    la.out_g = c->out_ln_g;
    la.out_b = c->out_ln_b;
    la.pe = c->pe;
    la.x = c->x;
    la.h = c->h;
    la.qkv = c->qkv;
    la.att = c->att;
    la.q = c->q;
    la.steps = c->d_steps;
    la.noise = a.noise;
    la.extras = a.extras;           // written by the loop's own last iteration
    la.scale = 1.0f / std::sqrt((float)(d / D.heads));
    la.ctl = c->long_ctl;
    la.status = c->long_status + ci;
    la.stamps = ci == 0 ? c->long_stamps : nullptr;
    HIP_TRY(c, launch_long_loop(mx ? 2 : D.dtype == GGD_FP8W ? 1 : 0, la, std::min(cap, a.n - c0i), s));
  }
  if (c->profiling && (r = prof_mark(c, s))) return r;
  int st[MEGA_MAX_CHUNKS];
  HIP_TRY(c, hipMemcpyAsync(st, c->long_status, sizeof(int) * MEGA_MAX_CHUNKS, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  int worst = 0;
  for (int ci = 0; ci < chunks; ++ci) worst = std::max(worst, st[ci]);
  if (worst & STATUS_TIMEOUT) ++c->barrier_timeouts;
  c->long_launches = chunks;
  if (worst == 3) {  // not placeable: nothing ran in the chunks that report 3; all chunks re-run on launches
    for (int ci = 0; ci < chunks; ++ci)
      if (st[ci] != 3) return fail(c, GGD_ERR_HIP, "long-clip loop: placement differed between chunks");
    c->long_launches = 0;
    ++c->long_fallbacks;
    return 1;
  }
  if (worst)
    return fail(c, GGD_ERR_HIP, worst == 2 ? "long-clip loop: workgroups were not all resident"
                                           : "long-clip loop: a clip-group barrier timed out");
  if (c->profiling) {
    float ms = 0;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->prof.ev[0], c->prof.ev[1]));
    c->prof_avg_us = ms * 1000.0 / chunks;
    c->prof_launches = chunks;
    c->prof_kind = 5;
    c->span_pending = 0;
  }
  return GGD_OK;
}

// Arguments of the one-workgroup-per-clip loop (ggd_persist.hip) for this sampling call.
PersistArgs persist_args(ggd_ctx* c, const ggd_sample_args& a, int nsteps) {
  const ggd_desc& D = c->desc;
  PersistArgs p{};
  p.layers = c->d_layers;
  p.n_layers = D.n_layers;
  p.n = a.n;
  p.L = D.seq_len;
  p.Ts = D.speech_len;
  p.C = D.d_pose;
  p.alg = a.alg;
  p.ln_g = c->out_ln_g;
  p.ln_b = c->out_ln_b;
  p.w_out = c->f_out.w;
  p.b_out = c->f_out.b;
  p.w_emb = c->f_emb.w;
  p.b_emb = c->f_emb.b;
  p.pe = c->pe;
  p.x = c->x;
  p.steps = c->d_steps;
  p.k0 = 0;
  p.n_steps = nsteps;
  p.noise = a.noise;
  p.seed = a.seed;
  p.clip_offset = a.clip_offset;
  p.inp_pose = a.inpaint_poses;
  p.inp_mask = a.inpaint_masks;
  p.trans = a.trans;
  p.extras = a.extras;
  p.scale = 1.0f / std::sqrt((float)(D.d_model / D.heads));
  return p;
}

// Behind a persistent loop that needs every workgroup resident at once: the same clips re-initialised
// and run on the one-workgroup-per-clip loop (no co-residency needed), both launches gated on the
// device by the loop's status word, so a non-blocking call never hands back an unrun x
int launch_gated_fallback(ggd_ctx* c, const ggd_sample_args& a, int nsteps, int clip0, int clips, const int* gate,
                          int gate_xl, hipStream_t s) {
  const ggd_desc& D = c->desc;
  PersistArgs p = persist_args(c, a, nsteps);
  p.clip0 = clip0;
  p.gate = gate;
  p.gate_xl = gate_xl;
  HIP_TRY(c, launch_init_state_gated(c->x, a.x_T, a.seed, a.clip_offset, clip0, clips, D.d_pose, D.seq_len, gate,
                                     gate_xl, s));
  HIP_TRY(c, launch_persist_range(p, clips, s));
  return GGD_OK;
}

// The first `nsteps` iterations as ONE persistent launch (ggd_mega.hip) per chunk of clips.
// The XCD-local variant runs first; a chunk it cannot place (status 3: nothing ran) is re-run on the
// write-through variant by a second launch that the device gates on that status word, so the host
// never waits.  sync = false: returns once issued, the status words are checked later
// (defer_check); sync = true: blocks, and returns 1 when the loop could not run at all (status 2:
// its workgroups were never all resident, nothing ran) so that the caller takes the launch route.
int run_mega(ggd_ctx* c, const ggd_sample_args& a, int nsteps, bool sync) {
  const ggd_desc& D = c->desc;
  const int NL = D.n_layers;
  hipStream_t s = c->stream;
  if (!c->mega_fa) {
    HIP_TRY(c, dalloc(c, &c->mega_fa, sizeof(FusedArgs) * 4 * NL));
    HIP_TRY(c, dalloc(c, &c->mega_fe, sizeof(FinalArgs)));
    HIP_TRY(c, dalloc(c, &c->mega_ctl, sizeof(unsigned) * MEGA_CTL_WORDS));
    HIP_TRY(c, dalloc(c, &c->mega_status, sizeof(int) * 2 * MEGA_MAX_CHUNKS));
  }
  c->mega_fa_host.assign(4 * NL, FusedArgs{});
  for (int li = 0; li < NL; ++li) {
    FusedArgs f = fused_args(c, li, nullptr);
    f.x_emb = nullptr;                // layer 0's h rows come from the loop's KE rows phase
    c->mega_fa_host[4 * li] = f;      // KA
    c->mega_fa_host[4 * li + 1] = f;  // KB: h -> h2
    f.h = c->h2;
    f.h_out = c->h;
    c->mega_fa_host[4 * li + 2] = f;  // KC: h2 -> h
    f.h = c->h;
    c->mega_fa_host[4 * li + 3] = f;  // KD: h in place
  }
  if (c->mega_phase_stamps && NL > 1)  // workgroup 0 stamps layer 1's phases (last step wins)
    for (int j = 0; j < 4; ++j) c->mega_fa_host[4 + j].stamps = c->mega_phase_stamps + 16 * j;
  FinalArgs& fe = c->mega_fe_host;
  fe = final_args(c, a.n);
  fe.alg = a.alg;
  fe.noise = a.noise;
  fe.inp_pose = a.inpaint_masks ? a.inpaint_poses : nullptr;
  fe.inp_mask = a.inpaint_masks;
  fe.trans = a.trans;
  fe.do_out = 1;
  fe.do_update = 1;
  fe.extras = a.extras;             // written by the loop's own last iteration
  fe.extras_k = nsteps - 1;
  fe.stamps = c->mega_phase_stamps ? c->mega_phase_stamps + 64 : nullptr;
  fe.ffp = c->ffp;                               // the last layer's KD runs in the KE rows phase
  fe.ff2_b = fused_layer(c, NL - 1).ff2_b;
  {
    int r = upload_cached(c, c->mega_fa, c->mega_fa_host.data(), sizeof(FusedArgs) * 4 * NL, s);
    if (!r) r = upload_cached(c, c->mega_fe, &fe, sizeof(FinalArgs), s);
    if (r) return r;
  }
  // batches above the loop's capacity run as consecutive launches of up to `cap` clips each
  const int cap = group_capacity(c, true);
  const int chunks = (a.n + cap - 1) / cap;
  if (chunks > MEGA_MAX_CHUNKS) return fail(c, GGD_ERR_ARG, "batch too large for the persistent loop");
  HIP_TRY(c, hipMemsetAsync(c->mega_status, 0, sizeof(int) * 2 * MEGA_MAX_CHUNKS, s));
  const bool xl = c->mega_place == 0;
  // Shapes the one-workgroup-per-clip loop can run (bf16, L <= 48: persist_supported) get a
  // device-gated fallback and the call returns once issued.  Every other shape is blocking: f32
  // (the parity mode) AND bf16 clips of 49..64 frames (the clip-group loops run them, the
  // one-workgroup loop does not) -- the call checks the status itself before returning and, when
  // nothing ran, re-initialises x and hands the call to the launch route (include/ggd.h ggd_sample)
  const bool fb = c->persist;
  if (!fb) sync = true;
  if (c->profiling) {
    c->prof.next = 0;
    int r = prof_mark(c, s);
    if (r) return r;
  }
  // bf16 on the row-block decomposition (ggd_rows.hip), f32 (the parity mode) on the head / chunk one
  const bool rows = D.dtype != 0;
  c->mega_rows_last = rows;
  auto launch = [&](const MegaArgs& m, int n, bool x) {
    return rows ? launch_rows(D.dtype, D.seq_len, D.speech_len, m, n, x, s) : launch_mega(D.dtype, D.seq_len, m, n, x, s);
  };
  for (int c0 = 0, ci = 0; c0 < a.n; c0 += cap, ++ci) {
    MegaArgs m{c->mega_fa, c->mega_fe, NL, 0, nsteps, c->mega_ctl, c->mega_status + ci,
               c0 == 0 ? c->mega_stamps : nullptr, c0, c->mega_place == 1 ? 1 : 0, nullptr, c->sim_unresident};
    HIP_TRY(c, launch(m, std::min(cap, a.n - c0), xl));
    if (xl) {  // the write-through re-run of this chunk, live only if the launch above reported 3
      MegaArgs g{c->mega_fa, c->mega_fe, NL, 0, nsteps, c->mega_ctl, c->mega_status + MEGA_MAX_CHUNKS + ci,
                 nullptr, c0, 0, c->mega_status + ci, c->sim_unresident};
      HIP_TRY(c, launch(g, std::min(cap, a.n - c0), false));
    }
  }
  if (c->profiling) {  // the loop's launches are the one timed span (read by ggd_kernel_time)
    int r = prof_mark(c, s);
    if (r) return r;
    c->prof_lazy = true;
    c->prof_lazy_div = chunks;
    c->prof_launches = chunks;
    c->prof_kind = 1;
    c->span_pending = 0;
  }
  // each chunk on the one-workgroup-per-clip loop, live only if it never ran (status 2); outside the
  // profiled span (the gated launches exit at once when the loop ran)
  for (int c0 = 0, ci = 0; fb && c0 < a.n; c0 += cap, ++ci) {
    int r = launch_gated_fallback(c, a, nsteps, c0, std::min(cap, a.n - c0), c->mega_status + ci, xl ? 1 : 0, s);
    if (r) return r;
  }
  int r = defer_check(c, c->mega_status, 2 * MEGA_MAX_CHUNKS, 1, chunks, xl, fb, s);
  if (r) return r;
  if (!sync) return GGD_OK;
  // earlier calls' checks first: an error they left is reported, not taken for this loop's
  if ((r = poll_pending_before_last(c))) return r;
  if ((r = take_sticky(c))) return r;
  if ((r = poll_pending(c, true))) return r;
  if (c->sticky && c->mega_none_ran && !fb) {  // nothing ran (status 2 everywhere): the launch route runs it
    c->sticky = 0;
    c->sticky_msg.clear();
    ++c->mega_fallbacks;
    HIP_TRY(c, launch_init_state(c->x, a.x_T, a.seed, a.clip_offset, a.n, D.d_pose, D.seq_len, s));
    return 1;
  }
  return take_sticky(c);
}

}  // namespace

extern "C" {

int ggd_sample(ggd_ctx* c, const ggd_sample_args* a, void* stream) {
  if (!c || !a || !a->out) return fail(c, GGD_ERR_ARG, "null argument");
  if (!c->finalized) return fail(c, GGD_ERR_STATE, "weights not finalized");
  if (c->betas.empty()) return fail(c, GGD_ERR_STATE, "no schedule installed");
  if (a->alg != GGD_DDPM && a->alg != GGD_DDIM) return fail(c, GGD_ERR_UNSUPPORTED, "unsupported sample algorithm");
  if (a->n != c->mem_n) return fail(c, GGD_ERR_STATE, "batch differs from the installed speech memory");
  if ((a->inpaint_masks == nullptr) != (a->inpaint_poses == nullptr))
    return fail(c, GGD_ERR_ARG, "inpaint poses and masks must be given together");
  if (a->inpaint_masks && !a->trans) return fail(c, GGD_ERR_ARG, "inpaint requires the trans ramp");
  HIP_TRY(c, hipSetDevice(c->device));
  {  // an earlier non-blocking loop that failed is reported here, once
    int r = poll_pending(c, false);
    if (r) return r;
    if ((r = take_sticky(c))) return r;
  }
  const ggd_desc& D = c->desc;
  const int T = (int)c->betas.size();
  int nsteps = a->n_steps > 0 && a->n_steps < T ? a->n_steps : T;
  hipStream_t s = c->stream;
  const bool sync = a->sync != 0;

  std::vector<StepRec> recs;
  make_records(c, a->alg, a->eta, recs, a->seed, a->clip_offset);
  HIP_TRY(c, hipEventRecord(c->ev_in, (hipStream_t)stream));
  HIP_TRY(c, hipStreamWaitEvent(s, c->ev_in, 0));
  {
    int r = upload_cached(c, c->d_steps, recs.data(), sizeof(StepRec) * T, s);
    if (r) return r;
  }
  HIP_TRY(c, launch_init_state(c->x, a->x_T, a->seed, a->clip_offset, a->n, D.d_pose, D.seq_len, s));
  bool use_persist = c->persist && c->persist_mode != 1;
  if (use_persist && c->persist_mode == 0) {
    const int cap = group_capacity(c, true);
    use_persist = cap <= 0 || (a->n + cap - 1) / cap >= 3;
  }
  if (use_persist) {
    // ONE launch: a workgroup per clip runs all nsteps iterations (ggd_persist.hip); in
    // profiling mode that launch is the timed kernel
    PersistArgs p = persist_args(c, *a, nsteps);
    p.stamps = c->stamps;
    // clip pairs (two workgroups per clip) when the one-workgroup loop would leave CUs idle:
    // chunks of <= pcap clips, each filling the chip, vs rounds of 2 pcap clips at one per CU
    // (a pair step measured PAIR_STEP_RATIO x the one-workgroup step)
    const int pcap = persist_pair_capacity();
    bool pair = c->pair_mode == 2 && pcap > 0;
    if (c->pair_mode == 0 && pcap > 0) {
      const int chunks = (a->n + pcap - 1) / pcap, rounds = (a->n + 2 * pcap - 1) / (2 * pcap);
      pair = chunks * PAIR_STEP_RATIO < rounds;
    }
    c->pair_launches = 0;
    if (pair) {
      if (!c->pair_ctl) {
        HIP_TRY(c, dalloc(c, &c->pair_ctl, sizeof(unsigned) * PAIR_CTL_WORDS));
        HIP_TRY(c, dalloc(c, &c->pair_status, sizeof(int)));
        HIP_TRY(c, dalloc(c, &c->pair_xbuf, (size_t)PAIR_MAX * 4 * PAIR_SLOT_BYTES));
      }
      p.ctl = c->pair_ctl;
      p.status = c->pair_status;
      p.xbuf = c->pair_xbuf;
      p.force_coh = c->pair_force_coh;
      p.sim_unresident = c->sim_unresident;
      HIP_TRY(c, hipMemsetAsync(c->pair_status, 0, sizeof(int), s));
    }
    if (c->profiling) {
      c->prof.next = 0;
      int r = prof_mark(c, s);
      if (r) return r;
    }
    if (pair) {
      for (int c0 = 0; c0 < a->n; c0 += pcap) {  // chunks share the control words: stream-ordered
        p.clip0 = c0;
        HIP_TRY(c, launch_persist_pair(p, std::min(pcap, a->n - c0), s));
        ++c->pair_launches;
      }
    } else {
      HIP_TRY(c, launch_persist(p, s));
    }
    if (c->profiling) {  // the loop's launches are the one timed span (read by ggd_kernel_time)
      int r = prof_mark(c, s);
      if (r) return r;
      c->prof_lazy = true;
      c->prof_lazy_div = 1;
      c->prof_launches = 1;
      c->prof_kind = pair ? 4 : 3;
      c->span_pending = 0;
    }
    if (pair) {  // status 2 (the pairs were never all resident): the whole batch re-runs on the
                 // one-workgroup-per-clip loop, which needs no co-residency, gated on the device; the
                 // status word is checked later (or now, with sync)
      int r = launch_gated_fallback(c, *a, nsteps, 0, a->n, c->pair_status, 0, s);
      if (r) return r;
      if ((r = defer_check(c, c->pair_status, 1, 4, 1, false, true, s))) return r;
      if (sync) {
        if ((r = poll_pending_before_last(c))) return r;
        if ((r = take_sticky(c))) return r;
        if ((r = poll_pending(c, true))) return r;
        if ((r = take_sticky(c))) return r;
      }
    }
    HIP_TRY(c, launch_nlc_to_ncl(a->out, c->x, a->n, D.d_pose, D.seq_len, D.d_pose, s));
    HIP_TRY(c, hipEventRecord(c->ev_out, s));
    HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
    return GGD_OK;
  }
  HIP_TRY(c, launch_set_int(c->d_counter, -1, s));

  // the persistent loops run every iteration, the last one writing the extras itself
  if (nsteps > 0 && group_capacity(c, true) > 0) {
    int r = run_mega(c, *a, nsteps, sync);
    if (r < 0) return r;
    if (r == 0) {
      HIP_TRY(c, launch_nlc_to_ncl(a->out, c->x, a->n, D.d_pose, D.seq_len, D.d_pose, s));
      HIP_TRY(c, hipEventRecord(c->ev_out, s));
      HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
      return GGD_OK;
    }
    // r == 1 (sync only): the loop's workgroups were never all resident -> the per-phase launches
  }
  c->long_launches = 0;
  if (c->long_ok && !c->long_off && !c->gemm_launches && !c->attn_qsplit && !a->inpaint_masks && nsteps > 0) {
    int r = run_long(c, *a, nsteps);
    if (r < 0) return r;
    if (r == 0) {
      HIP_TRY(c, launch_nlc_to_ncl(a->out, c->x, a->n, D.d_pose, D.seq_len, D.d_pose, s));
      HIP_TRY(c, hipEventRecord(c->ev_out, s));
      HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
      return GGD_OK;
    }
  }
  const int graph_steps = a->extras ? nsteps - 1 : nsteps;
  // pointer / shape key: a captured graph is reused only for identical arguments
  char keybuf[512];
  std::snprintf(keybuf, sizeof keybuf, "%d|%d|%p|%p|%p|%p|%d|%d", a->alg, a->n, (const void*)a->noise,
                (const void*)a->inpaint_poses, (const void*)a->inpaint_masks, (const void*)a->trans,
                (int)c->profiling, c->gemm_launches * 2 + c->attn_qsplit);
  const std::string key(keybuf);
  // fused path profiling: KB stamps its own launch span per (step, layer) on the device clock,
  // so the graph replays unchanged; the generic path brackets its launches with events (eager)
  const bool spans = c->profiling && c->fused;
  const size_t span_wg = (size_t)D.heads * a->n;  // KB grid: (heads, clips)
  const size_t span_n = (size_t)T * D.n_layers * 2 * span_wg;
  if (spans) {
    if (c->span_cap < span_n) {  // arena memory is never returned; grow only
      HIP_TRY(c, dalloc(c, &c->span, span_n * sizeof(unsigned long long)));
      c->span_cap = span_n;
    }
    HIP_TRY(c, hipMemsetAsync(c->span, 0, span_n * sizeof(unsigned long long), s));
  }
  if (graph_steps > 0) {
    if (a->use_graph && (!c->profiling || spans)) {
      // one captured step, replayed: the step's kernels read the iteration from the device
      // counter that the step's first kernel advances
      if (!c->gexec || c->graph_key != key) {
        if (c->gexec) {
          hipGraphExecDestroy(c->gexec);
          c->gexec = nullptr;
        }
        if (c->graph) {
          hipGraphDestroy(c->graph);
          c->graph = nullptr;
        }
        HIP_TRY(c, hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        int r = launch_step(c, *a, nullptr, -1);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(s, &g);
        if (r) return r;
        if (e != hipSuccess) return fail(c, GGD_ERR_HIP, std::string("capture: ") + hipGetErrorString(e));
        c->graph = g;
        HIP_TRY(c, hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0));
        c->graph_key = key;
      }
      for (int k = 0; k < graph_steps; ++k) HIP_TRY(c, hipGraphLaunch(c->gexec, s));
    } else {
      // eager launches; in profiling mode every launch of the dominant kernel is bracketed
      // by a pair of events on the context stream (ggd_kernel_time reads them back)
      c->prof.next = 0;
      for (int k = 0; k < graph_steps; ++k) {
        int r = launch_step(c, *a, nullptr, -1);
        if (r) return r;
      }
      if (c->profiling && !spans && c->prof.next >= 2) {
        HIP_TRY(c, hipStreamSynchronize(s));
        double total = 0;
        int64_t cnt = 0;
        for (size_t j = 0; j + 1 < c->prof.next; j += 2) {
          float ms = 0;
          HIP_TRY(c, hipEventElapsedTime(&ms, c->prof.ev[j], c->prof.ev[j + 1]));
          total += ms * 1000.0;
          ++cnt;
        }
        c->prof_avg_us = cnt ? total / cnt : 0;
        c->prof_launches = cnt;
        c->prof_kind = 2;
      }
    }
  }
  if (a->extras && nsteps > 0) {
    int r = launch_step(c, *a, a->extras, -1);
    if (r) return r;
  }
  if (spans) {  // reduced on the host by ggd_kernel_time, outside the caller's timed region
    c->span_pending = span_n;
    c->span_wg = span_wg;
    c->prof_kind = 0;
  }
  HIP_TRY(c, launch_nlc_to_ncl(a->out, c->x, a->n, D.d_pose, D.seq_len, D.d_pose, s));
  HIP_TRY(c, hipEventRecord(c->ev_out, s));
  HIP_TRY(c, hipStreamWaitEvent((hipStream_t)stream, c->ev_out, 0));
  return GGD_OK;
}

int ggd_sync(ggd_ctx* c) {
  if (!c) return GGD_ERR_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int r = poll_pending(c, true);
  if (r) return r;
  return take_sticky(c);
}

}  // extern "C"
