// permlane_probe.hip -- checks the lane semantics of gfx950's v_permlane16_swap_b32 /
// v_permlane32_swap_b32 that ggd_fusedlib.h's lane-row reductions and broadcasts rely on.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/permlane_probe.hip -o scripts/build/permlane_probe
// Prints the four outputs for lanes 0, 16, 32, 48 (value = lane index) and PASS / FAIL.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(float* o) {
  const float x = (float)threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  o[4 * threadIdx.x + 0] = __uint_as_float(a[0]);
  o[4 * threadIdx.x + 1] = __uint_as_float(a[1]);
  o[4 * threadIdx.x + 2] = __uint_as_float(b[0]);
  o[4 * threadIdx.x + 3] = __uint_as_float(b[1]);
}

int main() {
  float* d = nullptr;
  float h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  bool ok = true;
  for (int l = 0; l < 64; ++l) {
    const int r = l >> 4, c = l & 15, half = l >> 5;
    // expected: permlane16_swap -> {row (r & ~1), row (r | 1)} of the lane's column;
    //           permlane32_swap -> {lower half, upper half} of the lane's position in its half
    const float e0 = (float)(((r & ~1) << 4) | c), e1 = (float)(((r | 1) << 4) | c);
    const float e2 = (float)(l & 31), e3 = (float)(32 | (l & 31));
    (void)half;
    ok = ok && h[4 * l] == e0 && h[4 * l + 1] == e1 && h[4 * l + 2] == e2 && h[4 * l + 3] == e3;
    if ((l & 15) == 0) printf("lane %2d: p16 {%g, %g} p32 {%g, %g}\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  }
  printf("%s\n", ok ? "PASS" : "FAIL");
  (void)hipFree(d);
  return ok ? 0 : 1;
}
