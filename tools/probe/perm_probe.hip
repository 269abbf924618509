// Probe: semantics of v_permlane32_swap_b32 (gfx950) via __builtin_amdgcn_permlane32_swap.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
  const unsigned l = threadIdx.x;
  const unsigned a = 1000 + l, b = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  o[l] = r[0];
  o[64 + l] = r[1];
}
int main() {
  unsigned *d, h[128];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  k<<<1, 64>>>(d);
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int i : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0=%u r1=%u\n", i, h[i], h[64 + i]);
  return hipFree(d) == hipSuccess ? 0 : 1;
}
