// Probe: largest by-value kernel argument the ROCm runtime accepts (the engine passes layer
// tables of up to 64 x 136 B = 8.7 KiB by value).  Build: hipcc --offload-arch=gfx950 -O2
// tools/kernarg_probe.hip -o tools/_kat ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int N> struct Big { int v[N]; };
template <int N>
__global__ void k(Big<N> b, int* out) { if (threadIdx.x == 0) out[0] = b.v[0] + b.v[N - 1]; }
template <int N> void run() {
  Big<N> b;
  for (int i = 0; i < N; ++i) b.v[i] = i;
  int* d = nullptr;
  (void)hipMalloc(&d, 4);
  (void)hipMemset(d, 0, 4);
  hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, 0, b, d);
  hipError_t e = hipGetLastError();
  int h = -1;
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("bytes=%d err=%s result=%d expect=%d\n", N * 4, hipGetErrorString(e), h, N - 1);
  (void)hipFree(d);
}
int main() { run<960>(); run<2048>(); run<4096>(); return 0; }
