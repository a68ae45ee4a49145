// Probe: lane mapping of v_permlane16_swap / v_permlane32_swap on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  const int l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(100 + l, 200 + l, false, false);
  auto s = __builtin_amdgcn_permlane32_swap(100 + l, 200 + l, false, false);
  o[l] = r[0]; o[64 + l] = r[1]; o[128 + l] = s[0]; o[192 + l] = s[1];
}
int main() {
  int* d; hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  const char* nm[4] = {"p16.vdst", "p16.vsrc", "p32.vdst", "p32.vsrc"};
  for (int a = 0; a < 4; a++) {
    printf("%s:", nm[a]);
    for (int l = 0; l < 64; l += 8) printf(" [%d]=%d", l, h[a * 64 + l]);
    printf("\n");
  }
  return 0;
}
