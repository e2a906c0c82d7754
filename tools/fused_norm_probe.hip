// fused_norm_probe.hip -- can a selection workgroup compute its own row's key norms at the
// SCORE kernel's HBM rate?  (GPU box only; tuning aid for a SCORE + SELECT_GATHER fusion.)
//
// Workload: K [1024 rows x 16384 tokens x 128] bf16 (4 GiB, the headline's 32 layers x 32 heads).
// Each variant streams every row once and computes every token's L2 norm with the engine's
// bf16 accumulation order (8 accumulators, element e of each 16-B chunk into accumulator e, chunks
// in order; csrc/kvc.hip accum_chunk), writing the rounded norm bits as u16 into LDS (as the
// selection's keys would be) and one checksum per row to global memory.  Workgroups of 1 024
// threads with 80 KiB of static LDS: two per CU, like select_gather_kernel.
//   lane   lane-per-token loads: thread t reads its own tokens' 16 chunks (8 in flight), no LDS
//          transpose (each load instruction touches 64 token rows 256 B apart)
//   slab   coalesced loads transposed through a per-wave LDS slab of 2 chunks per token (3 KiB
//          per wave, inside the 80 KiB), like score_tile with CP = 2
// Grids: 1 024 workgroups (one row each, two resident per CU) and 256 workgroups looping over
// 4 rows each (one per CU, the other slot empty: the rate a CU gets from ONE streaming row).
// stdout: one JSON object, best-of-7 ms and TB/s per variant / grid, and whether the two
// variants' checksums agree.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fused_norm_probe.hip -o tools/fused_norm_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

constexpr int ROWS = 1024, S = 16384, D = 128, NC = D * 2 / 16;  // 16 chunks per token
constexpr int NT = 1024, LDSB = 80 * 1024;

__device__ __forceinline__ float bits_to_f32(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t bf16_rne(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0u;
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ void accum(float (&acc)[8], uint4 x) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float e0 = bits_to_f32(w[q] << 16), e1 = bits_to_f32(w[q] & 0xFFFF0000u);
    acc[2 * q] = __builtin_fmaf(e0, e0, acc[2 * q]);
    acc[2 * q + 1] = __builtin_fmaf(e1, e1, acc[2 * q + 1]);
  }
}
__device__ __forceinline__ uint32_t finish(const float (&acc)[8]) {
  float s = acc[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) s = s + acc[j];
  return bf16_rne(__builtin_sqrtf(s));
}

template <int VAR>
__device__ void row_norms(const char* __restrict__ k, int row, char* lds, uint32_t* sum_out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint16_t* key = reinterpret_cast<uint16_t*>(lds);  // 32 KiB
  const char* base = k + (size_t)row * S * D * 2;
  if constexpr (VAR != 1) {  // lane per token: 0 / 3 eight chunks in flight, 2 / 4 sixteen;
                             // 3 / 4 non-temporal loads
    constexpr int F = (VAR == 2 || VAR == 4) ? 16 : 8;
    constexpr bool NTL = VAR >= 3;
    for (int t = tid; t < S; t += NT) {
      const char* src = base + (size_t)t * D * 2;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int h = 0; h < NC / F; ++h) {
        uint4 v[F];
#pragma unroll
        for (int c = 0; c < F; ++c) {
          if constexpr (NTL) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 w = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(src + (h * F + c) * 16));
            v[c] = make_uint4(w.x, w.y, w.z, w.w);
          } else {
            v[c] = *reinterpret_cast<const uint4*>(src + (h * F + c) * 16);
          }
        }
#pragma unroll
        for (int c = 0; c < F; ++c) accum(acc, v[c]);
      }
      key[t] = (uint16_t)finish(acc);
    }
  } else {  // coalesced, CP = 2 slab per wave (64 tokens x 48 B) after the key region
    char* slab = lds + 32768 + wid * 64 * 48;
    for (int t0 = wid * 64; t0 < S; t0 += NT) {  // one 64-token tile per wave
      const char* tb = base + (size_t)t0 * D * 2;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int ph = 0; ph < NC / 2; ++ph) {
        uint4 v[2];
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int q = it * 64 + lane, tok = q >> 1, c = q & 1;
          v[it] = *reinterpret_cast<const uint4*>(tb + (size_t)tok * D * 2 + (ph * 2 + c) * 16);
        }
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          const int q = it * 64 + lane, tok = q >> 1, c = q & 1;
          *reinterpret_cast<uint4*>(slab + tok * 48 + c * 16) = v[it];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < 2; ++c) accum(acc, *reinterpret_cast<const uint4*>(slab + lane * 48 + c * 16));
        __builtin_amdgcn_wave_barrier();
      }
      key[t0 + lane] = (uint16_t)finish(acc);
    }
  }
  __syncthreads();
  uint32_t s = 0;
  for (int t = tid; t < S; t += NT) s += (uint32_t)key[t] * (uint32_t)(t + 1);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ uint32_t part[16];
  if (lane == 0) part[wid] = s;
  __syncthreads();
  if (tid == 0) {
    uint32_t x = 0;
    for (int w = 0; w < 16; ++w) x += part[w];
    sum_out[row] = x;
  }
  __syncthreads();
}

template <int VAR>
__global__ void __launch_bounds__(NT) probe(const char* __restrict__ k, uint32_t* sums, int rows_per_wg) {
  __shared__ __attribute__((aligned(16))) char lds[LDSB];
  for (int i = 0; i < rows_per_wg; ++i) row_norms<VAR>(k, blockIdx.x * rows_per_wg + i, lds, sums);
}

__global__ void fill(uint16_t* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = (uint16_t)(0x3C00u + (h & 0x3FFu) - 0x200u + ((h >> 10) & 0x8000u));  // |x| ~ 2^-1..2^1
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t n = (size_t)ROWS * S * D;
  uint16_t* k;
  uint32_t *s0, *s1;
  CK(hipMalloc(&k, n * 2));
  CK(hipMalloc(&s0, ROWS * 4));
  CK(hipMalloc(&s1, ROWS * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, k, n);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](auto kern, int grid, int rpw, uint32_t* so) {
    float best = 1e30f;
    for (int r = 0; r < 7; ++r) {
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), 0, 0, (const char*)k, so, rpw);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = std::min(best, ms);
    }
    return best;
  };
  const double gb = (double)n * 2 / 1e9;
  float t[8];
  t[0] = timed(probe<0>, ROWS, 1, s0);
  t[1] = timed(probe<1>, ROWS, 1, s1);
  t[2] = timed(probe<0>, ROWS / 4, 4, s0);
  t[3] = timed(probe<2>, ROWS, 1, s0);
  t[4] = timed(probe<3>, ROWS, 1, s0);
  t[5] = timed(probe<4>, ROWS, 1, s0);
  t[6] = timed(probe<4>, ROWS / 4, 4, s0);
  t[7] = timed(probe<2>, ROWS / 4, 4, s0);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> h0(ROWS), h1(ROWS);
  CK(hipMemcpy(h0.data(), s0, ROWS * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h1.data(), s1, ROWS * 4, hipMemcpyDeviceToHost));
  const bool same = h0 == h1;
  const char* names[8] = {"lane8_2perCU", "slab_2perCU", "lane8_1perCU", "lane16_2perCU",
                          "lane8nt_2perCU", "lane16nt_2perCU", "lane16nt_1perCU", "lane16_1perCU"};
  printf("{\"bytes\": %.0f, \"checksums_agree\": %s", gb * 1e9, same ? "true" : "false");
  for (int i = 0; i < 8; ++i) printf(", \"%s\": {\"ms\": %.4f, \"TB_s\": %.3f}", names[i], t[i], gb / t[i]);
  printf("}\n");
  return 0;
}
