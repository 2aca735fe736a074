// MX fp8 MFMA lane-map probe (diagnostic, not product): v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3
// operands against a host product under the hypothesis
//   A: lane l byte j = A[l & 15][32 (l >> 4) + j],  B: lane l byte j = B[32 (l >> 4) + j][l & 15],
//   scale_a of lane l (e8m0, byte 0) scales A's block (row l & 15, k 32 (l >> 4) ..), likewise B,
//   D: lane l reg r = D[4 (l >> 4) + r][l & 15]
// Exact small integers (e4m3 encodes -4..4 exactly), power-of-two scales: any mismatch is a map error.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
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
  int m = v < 0 ? -v : v;
  int e = 0;
  while ((1 << (e + 1)) <= m) ++e;
  const int frac = ((m << 3) >> e) & 7;
  return s | (uint8_t)((e + 7) << 3) | (uint8_t)frac;
}
int main() {
  uint8_t A[64][32], B[64][32];
  int sa[64], sb[64];
  float Am[16][128], Bm[128][16];
  unsigned seed = 12345;
  auto rnd = [&]() { seed = seed * 1103515245u + 12345u; return (int)((seed >> 16) % 9) - 4; };
  for (int l = 0; l < 64; ++l) {
    sa[l] = 127 + (l % 3);
    sb[l] = 127 + ((l >> 2) % 2);
    for (int j = 0; j < 32; ++j) {
      const int va = rnd(), vb = rnd();
      A[l][j] = e4m3(va);
      B[l][j] = e4m3(vb);
      Am[l & 15][32 * (l >> 4) + j] = va * std::ldexp(1.0f, sa[l] - 127);
      Bm[32 * (l >> 4) + j][l & 15] = vb * std::ldexp(1.0f, sb[l] - 127);
    }
  }
  void *da, *db, *dsa, *dsb, *dd;
  hipMalloc(&da, sizeof(A)); hipMalloc(&db, sizeof(B)); hipMalloc(&dsa, sizeof(sa)); hipMalloc(&dsb, sizeof(sb));
  hipMalloc(&dd, 64 * 16);
  hipMemcpy(da, A, sizeof(A), hipMemcpyHostToDevice);
  hipMemcpy(db, B, sizeof(B), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa, sizeof(sa), hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb, sizeof(sb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mx_kernel, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, (const int*)dsa, (const int*)dsb, (f32x4*)dd);
  float D[64][4];
  hipMemcpy(D, dd, sizeof(D), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * (l >> 4) + r, n = l & 15;
      double ref = 0;
      for (int k = 0; k < 128; ++k) ref += (double)Am[i][k] * Bm[k][n];
      if (std::fabs(ref - D[l][r]) > 1e-3) {
        if (bad < 8) printf("mismatch lane %d reg %d: gpu %g ref %g\n", l, r, D[l][r], ref);
        ++bad;
      }
    }
  printf("mx fp8 16x16x128 lane-map hypothesis: %s (%d of 1024 outputs differ)\n", bad ? "WRONG" : "holds", bad);
  return bad ? 1 : 0;
}
