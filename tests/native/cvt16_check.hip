// cvt16_check.hip -- the hardware converts the snapkv scoring uses (f16_to_f32_hw /
// f32_to_f16_hw / f32x2_to_bf16x2_hw, csrc/kvc_common.h) against the c10-exact integer
// conversions (f16_to_f32 / f32_to_f16_rne / f32_to_bf16_rne), on the GPU, for every input: all
// 2^16 binary16 patterns and all 2^32 fp32 patterns (to fp16 and to bf16).  Equal bits for every
// non-NaN input; NaN out for every NaN in (payloads may differ).
// Test infrastructure (tests/test_native_abi.py::test_hw_fp16_converts_match_c10); built by
// __graft_entry__.build().  Prints "<n> mismatches" and exits 0 only when n == 0.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "kvc_common.h"

using namespace kvc;

constexpr int kThreads = 256;
constexpr int kPerThread = 256;

// per-thread mismatch counts, plain vector stores (summed on the host)
__global__ void __launch_bounds__(kThreads) to_f32_check(uint32_t* bad) {
  const uint32_t h = blockIdx.x * kThreads + threadIdx.x;  // 2^16 threads
  const float a = f16_to_f32(h), b = f16_to_f32_hw(h);
  const bool nan = a != a;
  const bool ok = nan ? (b != b) : (f32_to_bits(a) == f32_to_bits(b));
  bad[h] = ok ? 0u : 1u;
}

__global__ void __launch_bounds__(kThreads) to_f16_check(uint32_t base_hi, uint32_t* bad) {
  const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
  uint32_t n = 0;
  for (uint32_t j = 0; j < kPerThread; ++j) {
    const uint32_t u = (base_hi << 28) | (t * kPerThread + j);
    const float f = bits_to_f32(u);
    const uint32_t a = f32_to_f16_rne(f), b = f32_to_f16_hw(f);
    const bool nan = (a & 0x7FFFu) > 0x7C00u;
    n += nan ? ((b & 0x7FFFu) > 0x7C00u ? 0u : 1u) : (a == b ? 0u : 1u);
  }
  bad[t] = n;
}

__global__ void __launch_bounds__(kThreads) to_bf16_check(uint32_t base_hi, uint32_t* bad) {
  const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
  uint32_t n = 0;
  for (uint32_t j = 0; j < kPerThread; j += 2) {  // both halves of the packed convert
    const uint32_t u0 = (base_hi << 28) | (t * kPerThread + j), u1 = u0 + 1;
    const uint32_t hw = f32x2_to_bf16x2_hw(bits_to_f32(u0), bits_to_f32(u1));
    const uint32_t b[2] = {hw & 0xFFFFu, hw >> 16};
    const uint32_t u[2] = {u0, u1};
    for (int h = 0; h < 2; ++h) {
      const uint32_t a = f32_to_bf16_rne(bits_to_f32(u[h]));
      const bool nan = (u[h] & 0x7FFFFFFFu) > 0x7F800000u;
      n += nan ? ((b[h] & 0x7FFFu) > 0x7F80u ? 0u : 1u) : (a == b[h] ? 0u : 1u);
    }
  }
  bad[t] = n;
}

#define HIP_OK(x)                                                   \
  do {                                                              \
    if ((x) != hipSuccess) {                                        \
      fprintf(stderr, "cvt16_check: %s failed\n", #x);              \
      return 2;                                                     \
    }                                                               \
  } while (0)

int main() {
  const uint32_t slice = 1u << 28;  // fp32 patterns per launch (16 launches)
  const uint32_t nthreads = slice / kPerThread;
  uint32_t* d;
  HIP_OK(hipMalloc(&d, (size_t)nthreads * 4));
  uint32_t* h = (uint32_t*)malloc((size_t)nthreads * 4);
  if (!h) return 2;
  uint64_t bad16 = 0, bad32 = 0, badb = 0;
  to_f32_check<<<65536 / kThreads, kThreads>>>(d);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpy(h, d, 65536 * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < 65536; ++i) bad16 += h[i];
  for (uint32_t s = 0; s < 16; ++s) {
    to_f16_check<<<nthreads / kThreads, kThreads>>>(s, d);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(h, d, (size_t)nthreads * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nthreads; ++i) bad32 += h[i];
    to_bf16_check<<<nthreads / kThreads, kThreads>>>(s, d);
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpy(h, d, (size_t)nthreads * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nthreads; ++i) badb += h[i];
  }
  printf("f16->f32: %llu mismatches of 65536; f32->f16: %llu, f32->bf16: %llu mismatches of "
         "4294967296\n", (unsigned long long)bad16, (unsigned long long)bad32,
         (unsigned long long)badb);
  printf("%llu mismatches\n", (unsigned long long)(bad16 + bad32 + badb));
  (void)hipFree(d);
  free(h);
  return bad16 + bad32 + badb == 0 ? 0 : 1;
}
