// kvc_common.h -- numerics shared by the HIP kernels (and their host unit test).
//
// Everything here reproduces a PyTorch CPU behaviour the reference relies on:
//   * c10::BFloat16 round-to-nearest-even with NaN -> 0x7FC0 (c10/util/BFloat16.h)
//   * the total order PyTorch's sort/topk comparators induce on float keys
//     (aten SortingUtils.h KeyValueCompAsc / KeyValueCompDesc, TopKImpl.h), mapped to unsigned
//     integers so the selection kernels compare keys with a single integer '<'.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define KVC_HD __host__ __device__ __forceinline__

namespace kvc {

KVC_HD float bits_to_f32(uint32_t u) {
  union { uint32_t u; float f; } c;
  c.u = u;
  return c.f;
}
KVC_HD uint32_t f32_to_bits(float f) {
  union { uint32_t u; float f; } c;
  c.f = f;
  return c.u;
}
KVC_HD float bf16_to_f32(uint32_t b) { return bits_to_f32((b & 0xFFFFu) << 16); }

// c10::BFloat16 round_to_nearest_even
KVC_HD uint32_t f32_to_bf16_rne(float f) {
  uint32_t u = f32_to_bits(f);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return 0x7FC0u;
  u += ((u >> 16) & 1u) + 0x7FFFu;
  return u >> 16;
}

// Sort keys.  Ascending base order is PyTorch's asc comparator
//   (!isnan(a) && isnan(b)) || a < b
// i.e. numeric order with -0 == +0 and every NaN tied above +inf.  Descending order
//   (isnan(a) && !isnan(b)) || a > b
// is the exact reverse (NaN first), obtained by complementing the key.  Equal keys <=> the
// comparator considers the two elements equivalent, so tie dynamics are preserved exactly.
KVC_HD uint16_t key_bf16(uint32_t b, bool desc) {
  b &= 0xFFFFu;
  uint32_t k;
  if ((b & 0x7FFFu) > 0x7F80u) {
    k = 0xFFFFu;
  } else {
    if (b == 0x8000u) b = 0;
    k = (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
  }
  return (uint16_t)(desc ? (~k & 0xFFFFu) : k);
}

KVC_HD uint32_t key_f32(uint32_t b, bool desc) {
  uint32_t k;
  if ((b & 0x7FFFFFFFu) > 0x7F800000u) {
    k = 0xFFFFFFFFu;
  } else {
    if (b == 0x80000000u) b = 0;
    k = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  }
  return desc ? ~k : k;
}

// torch.gather on CPU rewrites every bf16 NaN to 0xFFFF (measured over all 65536 patterns);
// applied to the gathered segment of bf16 outputs only.
KVC_HD uint32_t canon_nan_bf16x2(uint32_t w) {
  uint32_t lo = w & 0xFFFFu, hi = w >> 16;
  if ((lo & 0x7FFFu) > 0x7F80u) lo = 0xFFFFu;
  if ((hi & 0x7FFFu) > 0x7F80u) hi = 0xFFFFu;
  return lo | (hi << 16);
}

}  // namespace kvc
