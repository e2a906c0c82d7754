// read_probe.hip -- ceiling of a pure HBM read stream on this GPU (tuning aid, GPU box only).
// Reads a 4 GiB buffer (the headline's 32 layers of K) with 16-B loads, `U` loads in flight per
// thread, non-temporal or default policy, one xor-reduced dword written per workgroup; reports
// the best of 10 launches for several grid shapes.  Build:
//   hipcc --offload-arch=gfx950 -O3 tools/read_probe.hip -o tools/read_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const u32x4* __restrict__ src, size_t n_vec,
                                                   uint32_t* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  uint32_t acc = 0;
  for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n_vec; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = base + (size_t)u * 256;
      if (i < n_vec) {
        if (NT) v[u] = __builtin_nontemporal_load(src + i);
        else v[u] = src[i];
      } else {
        v[u] = u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  __shared__ uint32_t red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = 0;
    for (int i = 0; i < 256; ++i) r ^= red[i];
    out[blockIdx.x] = r;
  }
}

template <int U, bool NT>
static float run(const u32x4* src, size_t n_vec, uint32_t* out, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 12; ++r) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((read_kernel<U, NT>), dim3(grid), dim3(256), 0, 0, src, n_vec, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (r >= 2 && ms < best) best = ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best;
}

int main() {
  const size_t bytes = (size_t)4 << 30;
  const size_t n_vec = bytes / 16;
  u32x4* src;
  uint32_t* out;
  if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
  hipMemset(src, 1, bytes);
  hipDeviceSynchronize();
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("{\"cus\": %d, \"bytes\": %zu, \"runs\": [", cus, bytes);
  const int grids[] = {cus * 4, cus * 8, cus * 16, cus * 32, (int)(n_vec / 256 / 8)};
  bool first = true;
  for (int gi = 0; gi < 5; ++gi) {
    const int g = grids[gi];
    const float t[4] = {run<4, true>(src, n_vec, out, g), run<8, true>(src, n_vec, out, g),
                        run<8, false>(src, n_vec, out, g), run<16, true>(src, n_vec, out, g)};
    const char* nm[4] = {"U4nt", "U8nt", "U8", "U16nt"};
    for (int q = 0; q < 4; ++q) {
      printf("%s{\"grid\": %d, \"variant\": \"%s\", \"ms\": %.4f, \"TB_s\": %.3f}", first ? "" : ", ",
             g, nm[q], t[q], bytes / (t[q] * 1e-3) / 1e12);
      first = false;
    }
  }
  printf("]}\n");
  return 0;
}
