// MX fp8 MFMA lane-map probe (diagnostic, not product): v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3
// operands, exact small integers and power-of-two scales, against host products under several
// hypotheses -- the one with 0 mismatches is the hardware's map.
//   data maps (A: lane l byte j -> A[l & 15][k], B: -> B[k][l & 15], the same map for both):
//     H0  k = 32 (l >> 4) + j
//     H1  k = 16 (l >> 4) + j (j < 16), 64 + 16 (l >> 4) + j - 16 (j >= 16)
//   scale maps (lane l's e8m0 byte 0 scales):
//     S0  the block (row / column l & 15, k block l >> 4)
//     S1  exactly the lane's own 32 bytes
//   D: lane l reg r = D[4 (l >> 4) + r][l & 15]
// Three runs: uniform scales (data map), A scales varying (B uniform), B scales varying.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void mx_kernel(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x4* d) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = acc;
}
static uint8_t e4m3(int v) {  // exact small integers
  if (v == 0) return 0;
  const uint8_t s = v < 0 ? 0x80 : 0;
  const int m = v < 0 ? -v : v;
  int e = 0;
  while ((1 << (e + 1)) <= m) ++e;
  const int frac = ((m << 3) >> e) & 7;
  return s | (uint8_t)((e + 7) << 3) | (uint8_t)frac;
}
static int kmap(int h, int l, int j) {
  const int g = l >> 4;
  if (h == 0) return 32 * g + j;
  return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
}
int main() {
  static uint8_t A[64][32], B[64][32];
  static int va[64][32], vb[64][32];
  int sa[64], sb[64];
  unsigned seed = 12345;
  auto rnd = [&]() { seed = seed * 1103515245u + 12345u; return (int)((seed >> 16) % 9) - 4; };
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      va[l][j] = rnd();
      vb[l][j] = rnd();
      A[l][j] = e4m3(va[l][j]);
      B[l][j] = e4m3(vb[l][j]);
    }
  void *da, *db, *dsa, *dsb, *dd;
  (void)hipMalloc(&da, sizeof(A));
  (void)hipMalloc(&db, sizeof(B));
  (void)hipMalloc(&dsa, sizeof(sa));
  (void)hipMalloc(&dsb, sizeof(sb));
  (void)hipMalloc(&dd, 64 * 16);
  (void)hipMemcpy(da, A, sizeof(A), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, B, sizeof(B), hipMemcpyHostToDevice);
  int total_bad = 0;
  for (int run = 0; run < 3; ++run) {
    for (int l = 0; l < 64; ++l) {
      sa[l] = run == 1 ? 127 + (l % 3) + ((l >> 4) & 1) * 3 : 127;
      sb[l] = run == 2 ? 127 + ((l >> 2) % 2) + ((l >> 4) == 2 ? 4 : 0) : 127;
    }
    (void)hipMemcpy(dsa, sa, sizeof(sa), hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, sb, sizeof(sb), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mx_kernel, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, (const int*)dsa,
                       (const int*)dsb, (f32x4*)dd);
    float D[64][4];
    (void)hipMemcpy(D, dd, sizeof(D), hipMemcpyDeviceToHost);
    int best = 1 << 30;
    for (int h = 0; h < 2; ++h)
      for (int sm = 0; sm < 2; ++sm) {
        // dense operands with their scales applied, under (h, sm)
        static double Am[16][128], Bm[128][16];
        static int sAblk[16][4], sBblk[16][4];
        for (int l = 0; l < 64; ++l) {
          sAblk[l & 15][l >> 4] = sa[l];
          sBblk[l & 15][l >> 4] = sb[l];
        }
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 32; ++j) {
            const int k = kmap(h, l, j);
            const int ea = sm == 0 ? sAblk[l & 15][k / 32] : sa[l];
            const int eb = sm == 0 ? sBblk[l & 15][k / 32] : sb[l];
            Am[l & 15][k] = va[l][j] * std::ldexp(1.0, ea - 127);
            Bm[k][l & 15] = vb[l][j] * std::ldexp(1.0, eb - 127);
          }
        int bad = 0;
        for (int l = 0; l < 64; ++l)
          for (int r = 0; r < 4; ++r) {
            const int i = 4 * (l >> 4) + r, n = l & 15;
            double ref = 0;
            for (int k = 0; k < 128; ++k) ref += Am[i][k] * Bm[k][n];
            if (std::fabs(ref - D[l][r]) > 1e-3) ++bad;
          }
        printf("run %d (%s): data H%d scale S%d: %d of 1024 outputs differ\n", run,
               run == 0 ? "uniform scales" : run == 1 ? "A scales vary" : "B scales vary", h, sm, bad);
        best = bad < best ? bad : best;
      }
    total_bad += best != 0;
  }
  printf("mx probe: %s\n", total_bad ? "NO hypothesis explains every run" : "a hypothesis explains every run");
  return total_bad ? 1 : 0;
}
