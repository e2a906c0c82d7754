// launch_gap_probe.hip -- time per back-to-back dependent launch of a short kernel on one stream
// with a small (8 B) and a large (8 784 B, the engine's LayerChunk) kernel-argument block, and
// with 256 vs 32 768 workgroups.  Tool, GPU box only:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_gap_probe.hip -o tools/launch_gap_probe
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
  char b[8776];
};

__global__ void small_k(int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = (int)blockIdx.x;
}
__global__ void big_k(const Big a, int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = (int)a.b[blockIdx.x & 1023];
}

template <typename F>
static float per_launch(F f, int n) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int i = 0; i < n; ++i) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / n;
}

int main() {
  int* p;
  hipMalloc(&p, 64);
  hipMemset(p, 0, 64);
  Big big{};
  const int N = 200;
  for (int grid : {256, 32768}) {
    const float s = per_launch([&] { hipLaunchKernelGGL(small_k, dim3(grid), dim3(512), 0, 0, p); }, N);
    const float l = per_launch([&] { hipLaunchKernelGGL(big_k, dim3(grid), dim3(512), 0, 0, big, p); }, N);
    printf("{\"grid\": %d, \"us_per_launch_kernarg_8B\": %.2f, \"us_per_launch_kernarg_8784B\": %.2f}\n",
           grid, s, l);
  }
  return 0;
}
