// probe: what lane i reads with DPP row_shr:1 / row_shr:2 (diagnostic, tools/dev)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(float* o) {
  const int t = threadIdx.x;
  const float v = (float)t;
  o[t] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xF, 0xF, true));
  o[64 + t] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xF, 0xF, true));
}
int main() {
  float* d; hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  float h[128]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < 20; i++) printf("%d:%g/%g ", i, h[i], h[64 + i]);
  printf("\n");
  return 0;
}
