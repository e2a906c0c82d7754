// kvc_common.h -- numerics shared by the HIP kernels (and their host unit test).
//
// Everything here reproduces a PyTorch CPU behaviour the reference relies on:
//   * c10::BFloat16 round-to-nearest-even with NaN -> 0x7FC0 (c10/util/BFloat16.h)
//   * c10::Half conversions (IEEE binary16, round-to-nearest-even, NaN -> 0x7E00 | sign)
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

// IEEE binary16 -> fp32, exact (subnormals: man * 2^-24 is exact and normal in fp32)
KVC_HD float f16_to_f32(uint32_t h) {
  const uint32_t sign = (h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1Fu, man = h & 0x3FFu;
  if (e == 0x1Fu) return bits_to_f32(sign | 0x7F800000u | (man << 13));
  if (e == 0) {
    const float f = (float)man * 5.9604644775390625e-8f;  // 2^-24
    return sign ? -f : f;
  }
  return bits_to_f32(sign | ((e + 112u) << 23) | (man << 13));
}

// c10::Half(float) (fp16_ieee_from_fp32_value): round to nearest even, NaN -> 0x7E00 | sign;
// integer arithmetic only, so it does not depend on the FP mode or denormal flushing.
KVC_HD uint32_t f32_to_f16_rne(float f) {
  const uint32_t u = f32_to_bits(f);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const uint32_t a = u & 0x7FFFFFFFu;
  if (a > 0x7F800000u) return sign | 0x7E00u;
  if (a >= 0x477FF000u) return sign | 0x7C00u;  // >= 65520 rounds to inf
  if (a >= 0x38800000u)                         // normal binary16
    return sign | (((a + 0xFFFu + ((a >> 13) & 1u)) >> 13) - (112u << 10));
  // subnormal binary16: units of 2^-24, RNE on the shifted-out bits
  const uint32_t e = a >> 23;
  if (e < 102u) return sign;  // below 2^-25: rounds to zero (2^-25 itself ties to even 0)
  const uint32_t m = (a & 0x7FFFFFu) | 0x800000u;
  const uint32_t sh = 126u - e;  // 14..24
  uint32_t r = m >> sh;
  const uint32_t rem = m & ((1u << sh) - 1u), half = 1u << (sh - 1u);
  r += (rem > half || (rem == half && (r & 1u))) ? 1u : 0u;
  return sign | r;
}

// The same two conversions with the hardware converts (v_cvt_f32_f16 / v_cvt_f16_f32: IEEE
// round-to-nearest-even, fp16 denormals kept -- the gfx950 default mode).  Bit-identical to
// f16_to_f32 / f32_to_f16_rne on every non-NaN input and NaN for every NaN input; only NaN
// payloads may differ, so they serve where a NaN is only ever tested or mapped to a key (the
// snapkv scores).  tests/native/cvt16_check.hip checks all 2^16 and 2^32 inputs on the GPU.
__device__ __forceinline__ float f16_to_f32_hw(uint32_t h) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)h);
}
__device__ __forceinline__ uint32_t f32_to_f16_hw(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

// fp32 pair -> packed bf16 pair with the hardware convert (v_cvt_pk_bf16_f32: IEEE round to
// nearest even, fp32 denormals kept -- the gfx950 default mode).  Bit-identical to
// f32_to_bf16_rne on every non-NaN input and NaN for every NaN input (payload / sign may differ),
// so it serves where a NaN is only tested or mapped to a key (the snapkv scores);
// tests/native/cvt16_check.hip checks all 2^32 inputs on the GPU.
__device__ __forceinline__ uint32_t f32x2_to_bf16x2_hw(float lo, float hi) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{lo, hi}, b2));
}

// Sort keys of two packed bf16 values with packed 16-bit integer ops: k = 0x8000 + mag for
// positive, 0x8000 - mag for negative values (+-0 -> 0x8000), every NaN -> 0xFFFF; desc = ~k.
// Same order and the same ties as key_bf16 (PyTorch's comparators), not the same codes: use it
// for every key of a row or for none.
// key_h16x2: any 16-bit format whose NaNs are the magnitudes above inf_bits (bf16 0x7F80,
// fp16 0x7C00).
__device__ __forceinline__ uint32_t key_h16x2(uint32_t w, bool desc, uint32_t inf_bits) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 b = __builtin_bit_cast(u16x2, w);
  const u16x2 mag = b & (u16x2)0x7FFF;
  const u16x2 neg = (u16x2)0 - (b >> 15);                      // 0xFFFF where negative
  const u16x2 nan =                                            // 0xFFFF where mag > inf_bits
      (u16x2)0 - ((mag + (u16x2)(unsigned short)(0x7FFFu - inf_bits)) >> 15);
  u16x2 k = ((u16x2)0x8000 + ((mag ^ neg) - neg)) | nan;       // 0x8000 +- mag (mod 2^16)
  if (desc) k = ~k;
  return __builtin_bit_cast(uint32_t, k);
}
__device__ __forceinline__ uint32_t key_bf16x2(uint32_t w, bool desc) {
  return key_h16x2(w, desc, 0x7F80u);
}

// Sort keys.  Ascending base order is PyTorch's asc comparator
//   (!isnan(a) && isnan(b)) || a < b
// i.e. numeric order with -0 == +0 and every NaN tied above +inf.  Descending order
//   (isnan(a) && !isnan(b)) || a > b
// is the exact reverse (NaN first), obtained by complementing the key.  Equal keys <=> the
// comparator considers the two elements equivalent, so tie dynamics are preserved exactly.
// 16-bit storage formats differ only in where NaN starts: bf16 above 0x7F80, fp16 above 0x7C00.
KVC_HD uint16_t key_h16(uint32_t b, bool desc, uint32_t inf_bits) {
  b &= 0xFFFFu;
  uint32_t k;
  if ((b & 0x7FFFu) > inf_bits) {
    k = 0xFFFFu;
  } else {
    if (b == 0x8000u) b = 0;
    k = (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
  }
  return (uint16_t)(desc ? (~k & 0xFFFFu) : k);
}
KVC_HD uint16_t key_bf16(uint32_t b, bool desc) { return key_h16(b, desc, 0x7F80u); }
KVC_HD uint16_t key_f16(uint32_t b, bool desc) { return key_h16(b, desc, 0x7C00u); }

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

// torch.gather on CPU quiets every fp16 NaN (sets bit 9: 0x7C01 -> 0x7E01; measured over all
// 65536 patterns); applied to the gathered segment of fp16 outputs only.
KVC_HD uint32_t canon_nan_f16x2(uint32_t w) {
  uint32_t lo = w & 0xFFFFu, hi = w >> 16;
  if ((lo & 0x7FFFu) > 0x7C00u) lo |= 0x200u;
  if ((hi & 0x7FFFu) > 0x7C00u) hi |= 0x200u;
  return lo | (hi << 16);
}

}  // namespace kvc
