// dpp_probe.hip -- checks the DPP wave_shl:1 / wave_shr:1 lane mapping the register heap relies on
// (kvc.hip RegHeap::adjust: lane i reads lane i + 1 / i - 1).  Tool, GPU box only.
#include <hip/hip_runtime.h>
__global__ void k(int* o) {
  int v = threadIdx.x * 10;
  int a = __builtin_amdgcn_update_dpp(-1, v, 0x130, 0xF, 0xF, false);  // wave_shl:1
  int b = __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
  o[threadIdx.x] = a;
  o[64 + threadIdx.x] = b;
}
int main() {
  int* d; hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[128]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  printf("shl:"); for (int i = 0; i < 64; i += 15) printf(" %d->%d", i, h[i]); printf(" 63->%d\n", h[63]);
  printf("shr:"); for (int i = 0; i < 64; i += 15) printf(" %d->%d", i, h[64 + i]); printf(" 63->%d\n", h[127]);
  return 0;
}
