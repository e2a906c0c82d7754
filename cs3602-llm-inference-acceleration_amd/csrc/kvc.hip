// kvc.hip -- MI355X (gfx950) kernels and C ABI of the KV-cache compression engine.
// ABI documentation: include/kvc.h.  Design and rooflines: DESIGN.md.
//
// Kernels (one launch each, all layers of a compress_fn call batched into every launch):
//   score_kernel  : HBM-streaming key L2 norms.  One wave = one 64-token tile of one (b,h) row;
//                   tiles are read with coalesced 16-B loads, transposed through a padded LDS
//                   slab so each lane owns one token row, and reduced with torch.norm's exact
//                   8-accumulator FMA order (reference: torch.norm at fix_size_l2.py:106 etc.).
//   select_kernel : one 1024-thread workgroup per (layer, b, h) row, the row's keys resident in
//                   LDS.  Reproduces the first-k SET of libstdc++ std::sort (argsort, stable=False)
//                   or std::nth_element / std::partial_sort (torch.topk) by following only the
//                   chain of Hoare partitions that straddle position k; each partition is computed
//                   in parallel from ballot prefix ranks ("Selection").  Emits the
//                   kept zone-local indices in ascending order (= torch.sort(indices) of the
//                   reference, e.g. fix_size_l2.py:129).
//   gather_kernel : segment copy sink ++ zone[selected] ++ tail for K and V (torch.gather +
//                   torch.cat of the reference, e.g. fix_size_l2.py:137-147).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <tuple>
#include <type_traits>
#include <utility>

#include "kvc.h"
#include "kvc_common.h"
#include "kvc_serial.h"

namespace kvc {

constexpr int kTile = 64;  // tokens per score tile (one per lane)
constexpr int kSelThreads = 1024;
constexpr int kSelWaves = kSelThreads / 64;
// Zones of up to kSmallZone positions select with 512-thread workgroups and LDS sized by the
// call's longest zone, at most kSmallBudget bytes: four rows per CU (all 1 024 rows of a
// 32-layer call resident at once), a row's copy phase with 8 waves of loads in flight
// (256-thread rows: SELECT_GATHER 0.129 ms at S = 4 096, 0.104 ms at S = 513; 512: 0.115 /
// 0.096).  Up to 8 192 positions the budget holds the bf16 / fp16 rows with rank windows
// (profiles/r03_d_small_path_rows_per_cu_ab.jsonl, S = 8 192: 0.137 ms with 1 024-thread rows
// two per CU, 0.148 ms with 512-thread rows three per CU and full tables, 0.1265 ms four per CU
// with windows).  Longer zones keep 1 024 threads.
constexpr int kSelThreadsSmall = 512;
constexpr int kSmallZone = 8192;
// occupancy the select kernels ask the compiler for (waves per SIMD)
// (the heavy-hitter select kernels run one row per CU: no occupancy target to spill for)
constexpr int sel_waves_per_eu(int kc, int nt, bool hh = false) {
  return hh || (kc == KVC_F32 && nt == kSelThreads) ? 4 : 8;
}
constexpr long kSmallBudget = 40448;  // 4 x (this + scalars) <= 160 KiB of LDS per CU
constexpr long kBigBudget = 81408;    // 2 x (this + scalars) <= 160 KiB
constexpr int kZoneMax = 16384;        // longest zone whose selection runs from LDS
constexpr int kZoneMaxGlobal = 65536;  // longest zone of the u16-position global variant
constexpr int kZoneMaxLong = 1 << 24;   // longest zone at all (u32 positions; global scratch)
#ifndef KVC_WAVE_SEG
#define KVC_WAVE_SEG 256
#endif
constexpr int kWaveSeg = KVC_WAVE_SEG;  // segments this short are finished by one wave (64 / 128 / 512 / 1024 measured slower)
// the same for 512-thread rows (128 / 512 / 1 024 measured the same or slower at S = 4 096 and
// 8 192: profiles/r03_g_small_wave_threshold_ab.jsonl)
constexpr int kWaveSegSmall = 256;
constexpr int kGatherThreads = 256;
constexpr int kGatherTokens = 64;  // output tokens per gather block
constexpr int kBig = 0x7FFFFFFF;
// Layer tables travel to the score / select / gather kernels BY VALUE in the kernel arguments
// (chunks of kArgLayers, 8.7 KiB): no host->device table copy, whose completion would stand
// ~10 us between the copy and the first kernel of every call.
constexpr int kArgLayers = 64;
// SELECT_GATHER launches of at most this many rows (fewer than the 256 CUs: one row per CU)
// copy each row's sink / tail rows in a second workgroup beside the selecting one
#ifndef KVC_SPLIT_COPY_ROWS
#define KVC_SPLIT_COPY_ROWS 255
#endif
constexpr int kSplitCopyRows = KVC_SPLIT_COPY_ROWS;
// SELECT_GATHER's output stores: non-temporal (written once) unless built with KVC_SG_NTS=false
#ifndef KVC_SG_NTS
#define KVC_SG_NTS true
#endif
constexpr bool kSgNts = KVC_SG_NTS;
// the fused copy's row loads: default policy unless built with KVC_SG_NTL=true (non-temporal)
#ifndef KVC_SG_NTL
#define KVC_SG_NTL false
#endif
constexpr bool kSgNtl = KVC_SG_NTL;
// SCORE also derives each plain-norm row's level-0 pivot and writes per-tile ge / le counts
// (score_tile), which the selection's first partition level sums instead of re-reading the row
// (partition_level); 0: level 0 counts its keys itself (A/B)
#ifndef KVC_L0_TILE_COUNTS
#define KVC_L0_TILE_COUNTS 0
#endif
constexpr bool kL0TileCounts = KVC_L0_TILE_COUNTS;
// Level 0 of a 1 024-thread row with 16-bit keys keeps its rank tables in the idx region (the
// indices are still the identity there, rebuilt after the swaps): room for every rank a level
// can need, so no second rank window (partition_level); 0: the shared windows (A/B)
#ifndef KVC_L0_ITAB
#define KVC_L0_ITAB 1
#endif
constexpr bool kL0Itab = KVC_L0_ITAB;
// which rows' level 0 takes the idx-region tables: 0 plain-norm rows, 1 every row (A/B)
#ifndef KVC_L0_ITAB_ALL
#define KVC_L0_ITAB_ALL 1
#endif
constexpr bool kL0ItabAll = KVC_L0_ITAB_ALL;
#ifndef KVC_ITAB_COLD
#define KVC_ITAB_COLD 0
#endif
// Smallest positions-per-lane bound a level body is specialised on: levels with J <= this run in
// that body (1: one body per power of two up to 16).  2 folds the J = 1 levels into the J = 2
// body -- less code for the instruction cache; 1 / 2 / 4 / 8 measured within noise of each other
// (profiles/r06_f_itab_ab.jsonl)
#ifndef KVC_LEVEL_JM_MIN
#define KVC_LEVEL_JM_MIN 2
#endif
constexpr int kLevelJmMin = KVC_LEVEL_JM_MIN;
// SELECT_GATHER rows touch the rows they already know they keep while wave 0 finishes the chain
// (select_body; diagnostic A/B, off)
#ifndef KVC_SG_PREFETCH
#define KVC_SG_PREFETCH 0
#endif
constexpr bool kSgPrefetch = KVC_SG_PREFETCH;
// the wave chain's segments of <= 64 positions in registers (wave_tiny_chain); 0: LDS levels
#ifndef KVC_TINY_CHAIN
#define KVC_TINY_CHAIN 1
#endif
constexpr bool kTinyChain = KVC_TINY_CHAIN;
struct LayerChunk {
  kvc_layer_t l[kArgLayers];
};

template <int DT>
struct DTypeTraits;
template <>
struct DTypeTraits<KVC_BF16> {
  static constexpr int esz = 2;
  typedef uint16_t key_t;
};
template <>
struct DTypeTraits<KVC_F16> {
  static constexpr int esz = 2;
  typedef uint16_t key_t;
};
template <>
struct DTypeTraits<KVC_F32> {
  static constexpr int esz = 4;
  typedef uint32_t key_t;
};

template <int DT>
__device__ __forceinline__ float load_dt(const char* base, int i) {
  if constexpr (DT == KVC_BF16)
    return bf16_to_f32(reinterpret_cast<const uint16_t*>(base)[i]);
  else if constexpr (DT == KVC_F16)
    return f16_to_f32(reinterpret_cast<const uint16_t*>(base)[i]);
  else
    return reinterpret_cast<const float*>(base)[i];
}

// storage bits of an fp32 value rounded to a 16-bit dtype (c10 conversions)
template <int DT>
__device__ __forceinline__ uint32_t bits16_dt(float f) {
  if constexpr (DT == KVC_BF16)
    return f32_to_bf16_rne(f);
  else
    return f32_to_f16_rne(f);
}

template <int DT>
__device__ __forceinline__ float round_dt(float f) {
  if constexpr (DT == KVC_BF16)
    return bf16_to_f32(f32_to_bf16_rne(f));
  else if constexpr (DT == KVC_F16)
    return f16_to_f32(f32_to_f16_rne(f));
  else
    return f;
}

// sort key of a 16-bit storage pattern
template <int DT>
__device__ __forceinline__ uint16_t key16_dt(uint32_t bits, bool desc) {
  if constexpr (DT == KVC_BF16)
    return key_bf16(bits, desc);
  else
    return key_f16(bits, desc);
}

template <int DT>
__device__ __forceinline__ typename DTypeTraits<DT>::key_t key_of(float f, bool desc) {
  if constexpr (DT == KVC_F32)
    return key_f32(f32_to_bits(f), desc);
  else
    return key16_dt<DT>(bits16_dt<DT>(f), desc);
}

// Selection kernels are compiled per KEY CLASS (KC): KVC_BF16 stands for every 16-bit storage
// dtype (u16 keys), KVC_F32 for fp32 (u32 keys).  bf16 and fp16 rows run the same binary with the
// storage dtype as a runtime argument: the two differ only in the NaN threshold of the key map
// and in the float conversions of the snapkv scores.  (Two instantiations of identical source
// compiled ~2x apart in speed -- DESIGN.md "fp16 selection".)  f(integral_constant<int, DT>)
// runs with the row's storage dtype.
template <int KC, typename F>
__device__ __forceinline__ void with_dt(int dt, F&& f) {
  if constexpr (KC == KVC_F32)
    f(std::integral_constant<int, KVC_F32>());
  else if (dt == KVC_F16)
    f(std::integral_constant<int, KVC_F16>());
  else
    f(std::integral_constant<int, KVC_BF16>());
}
__device__ __forceinline__ uint32_t inf_bits16(int dt) { return dt == KVC_F16 ? 0x7C00u : 0x7F80u; }

// torch.gather's NaN rewrite on two 16-bit elements (kvc_common.h canon_nan_bf16x2 /
// canon_nan_f16x2) in five packed-u16 VALU ops instead of two compare/select chains:
// x = |w| per half; x + (0xFFFE - NANMIN) saturates to 0xFFFF exactly for x > NANMIN (a NaN);
// that - 0xFFFE (saturating) is 1 for a NaN half and 0 otherwise, scaled to the bits to set.
// Equal to the scalar forms on all 2^32 inputs (checked exhaustively when it was written).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
template <uint16_t NANMIN, uint16_t SET>
__device__ __forceinline__ uint32_t canon_nan_pk(uint32_t w) {
  const u16x2 x = __builtin_bit_cast(u16x2, w & 0x7FFF7FFFu);
  const u16x2 m = __builtin_elementwise_add_sat(
      x, (u16x2){(uint16_t)(0xFFFEu - NANMIN), (uint16_t)(0xFFFEu - NANMIN)});
  const u16x2 t = __builtin_elementwise_sub_sat(m, (u16x2){0xFFFE, 0xFFFE});
  return w | __builtin_bit_cast(uint32_t, t * (u16x2){SET, SET});
}
template <int DT>
__device__ __forceinline__ uint4 canon_nan_dt(uint4 a) {
  if constexpr (DT == KVC_BF16)  // NaN -> 0xFFFF
    return make_uint4(canon_nan_pk<0x7F80, 0xFFFF>(a.x), canon_nan_pk<0x7F80, 0xFFFF>(a.y),
                      canon_nan_pk<0x7F80, 0xFFFF>(a.z), canon_nan_pk<0x7F80, 0xFFFF>(a.w));
  else if constexpr (DT == KVC_F16)  // NaN |= 0x200 (quiet bit)
    return make_uint4(canon_nan_pk<0x7C00, 0x200>(a.x), canon_nan_pk<0x7C00, 0x200>(a.y),
                      canon_nan_pk<0x7C00, 0x200>(a.z), canon_nan_pk<0x7C00, 0x200>(a.w));
  else
    return a;
}

// Diagnostic build only (-DKVC_STAMPS): thread 0 of every select workgroup records s_memtime at
// phase boundaries into a per-row slot after the index region; the product build has no stamps.
#ifdef KVC_STAMPS
#define KVC_STAMP(i)                                                             \
  do {                                                                           \
    if (stamps && threadIdx.x == 0) stamps[blockIdx.x * 32 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define KVC_STAMP(i) \
  do {               \
  } while (0)
#endif

// Materialises x in a VGPR here: keeps the compiler from sinking the computation of a select
// operand into an exec-mask branch (s_and_saveexec / s_or_b64 exec: scalar instructions on the
// CU's one scalar unit, shared by all its waves) when only some lanes use it.
__device__ __forceinline__ int vreg(int x) {
  asm("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------------
// SCORE
// ---------------------------------------------------------------------------------------------
template <int DT, int NC>
__device__ __forceinline__ void accum_chunk(float (&acc)[8], const uint4 x, int gchunk) {
  if constexpr (DT == KVC_F16) {
    // NormTwoOps<Half, float> (binary_kernel_reduce): ONE accumulator in dim order; x*x is exact
    // in fp32 for an fp16 x, so the fma equals torch's acc + x*x.  (acc[1..7] stay 0: the final
    // lane sum adds +0 to a non-negative sum, which changes nothing.)
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[q] & 0xFFFFu));
      const float e1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[q] >> 16));
      acc[0] = __builtin_fmaf(e0, e0, acc[0]);
      acc[0] = __builtin_fmaf(e1, e1, acc[0]);
    }
  } else if constexpr (DT == KVC_BF16) {
    // chunk c holds elements 8c..8c+7: element e feeds accumulator e
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e0 = bits_to_f32(w[q] << 16);
      const float e1 = bits_to_f32(w[q] & 0xFFFF0000u);
      acc[2 * q] = __builtin_fmaf(e0, e0, acc[2 * q]);
      acc[2 * q + 1] = __builtin_fmaf(e1, e1, acc[2 * q + 1]);
    }
  } else {
    // chunk c holds elements 4c..4c+3: accumulators 4*(c&1) + e
    const int j0 = (gchunk & 1) * 4;
    const float e[4] = {bits_to_f32(x.x), bits_to_f32(x.y), bits_to_f32(x.z), bits_to_f32(x.w)};
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[j0 + q] = __builtin_fmaf(e[q], e[q], acc[j0 + q]);
  }
}

// 16-B chunks of a token row staged per phase: 4 (64-B rows), 8 (multiples of 128 B), 10 (160 B
// multiples); a row of NC chunks takes NC / CP phases.
__host__ __device__ constexpr int score_cp(int nc) { return nc == 4 ? 4 : (nc % 8 == 0 ? 8 : 10); }
// padded LDS row of CP chunks: an odd number of 16-B granules keeps every lane's ds_read_b128 of
// its own token row conflict-free
__host__ __device__ constexpr int score_rowb(int cp) { return (cp + (cp % 2 == 0 ? 1 : 2)) * 16; }
// waves (tiles) per workgroup: 8 for CP-8 rows (9.2 KB slab per wave: two 74 KB workgroups per
// CU, 2.5% faster than four 4-wave ones); 2 for CP-10 rows (11.3 KB per wave: seven 2-wave
// workgroups per CU, 14 waves -- D = 80 score 0.1049 -> 0.1011 ms against three 4-wave ones
// (12 waves); two 7-wave ones, also 14 waves, 0.1063; 8-wave ones 45% slower); 4 for 64-B
// rows.  A/B in profiles/r03_j_score_variants_ab.jsonl and r03_l_select_variants.json.
__host__ __device__ constexpr int score_waves(int nc) {
  return score_cp(nc) == 8 ? 8 : score_cp(nc) == 10 ? 2 : 4;
}

// One 64-token tile of one (layer, b, h) row: coalesced 16-B loads -> per-wave LDS slab ->
// one lane per token, torch.norm's 8-accumulator FMA order (fp16: its serial order).  `wl` is
// this wave's slab (kTile * ROWB bytes).
// snapkv_lite rows (KVC_SCORE_SNAPKV) also get each tile's maximum stored norm, as the bits of
// the stored value (u16 for 16-bit dtypes, u32 for fp32) in tmax[row * tmax_stride + tile]: a
// norm is never negative (nor -0: the accumulators start at +0 and add squares), so the bit
// order is the value order and every NaN's bits exceed +inf's.  The select kernel forms the
// row's `max(norms)` (snapkv_lite.py:99) from them without a block reduction.
template <int DT, int NC, bool NTL = false>
__device__ __forceinline__ void score_tile(const kvc_layer_t* ly, int row, int tt, int H,
                                           char* wl, char* norms, int64_t norm_stride,
                                           uint32_t* tmax, int64_t tmax_stride) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  constexpr int CP = score_cp(NC);  // 16-B chunks per token per phase
  constexpr int NPH = NC / CP;
  constexpr int ROWB = score_rowb(CP);  // padded LDS row: conflict-free ds_read_b128 per lane
  const int lane = threadIdx.x & 63;
  const int zlen = ly->zone_len;
  const int b = row / H, h = row - (row / H) * H;
  const int tok0 = tt * kTile;
  const int ntok = min(kTile, zlen - tok0);
  const int64_t sbytes = ly->k_stride[2] * ESZ;
  const char* base = static_cast<const char*>(ly->k) +
                     ((int64_t)b * ly->k_stride[0] + (int64_t)h * ly->k_stride[1] +
                      (int64_t)(ly->zone_start + tok0) * ly->k_stride[2]) * ESZ;
  // plain-norm rows: the three level-0 pivot token rows (see below), loaded before the tile so
  // that their latency passes under it -- lane u < 3 NC holds row u / NC's chunk u % NC
  const bool piv = kL0TileCounts && ly->score_mode == KVC_SCORE_NORM && tmax && zlen > 2;
  constexpr int PV = (3 * NC + 63) / 64;
  uint4 pvr[PV];
  if (piv) {
    const char* zb = static_cast<const char*>(ly->k) +
                     ((int64_t)b * ly->k_stride[0] + (int64_t)h * ly->k_stride[1] +
                      (int64_t)ly->zone_start * ly->k_stride[2]) * ESZ;
#pragma unroll
    for (int q = 0; q < PV; ++q) {
      const int u = lane + 64 * q, r = u / NC, c = u - r * NC;
      const int pt = r == 0 ? 1 : r == 1 ? zlen / 2 : zlen - 1;
      pvr[q] = u < 3 * NC ? *reinterpret_cast<const uint4*>(zb + pt * sbytes + c * 16)
                          : make_uint4(0, 0, 0, 0);
    }
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ph = 0; ph < NPH; ++ph) {
    uint4 v[CP];
#pragma unroll
    for (int it = 0; it < CP; ++it) {
      const int q = it * 64 + lane;
      const int tok = q / CP, c = q - (q / CP) * CP;
      const char* src = base + tok * sbytes + (ph * CP + c) * 16;
      if (tok < ntok) {
        if constexpr (NTL) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 w = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
          v[it] = make_uint4(w.x, w.y, w.z, w.w);
        } else {
          v[it] = *reinterpret_cast<const uint4*>(src);
        }
      } else {
        v[it] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < CP; ++it) {
      const int q = it * 64 + lane;
      const int tok = q / CP, c = q - (q / CP) * CP;
      *reinterpret_cast<uint4*>(wl + tok * ROWB + c * 16) = v[it];
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      const uint4 x = *reinterpret_cast<const uint4*>(wl + lane * ROWB + c * 16);
      accum_chunk<DT, NC>(acc, x, ph * CP + c);
    }
    wave_sync();
  }
  uint32_t bits = 0;  // the stored norm's bits (0 for lanes past the zone)
  if (lane < ntok) {
    float s = acc[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) s = s + acc[j];
    const float r = __builtin_sqrtf(s);
    char* nrow = norms + (int64_t)(ly->row0 + row) * norm_stride * ESZ;
    // non-temporal: the select phase reads the norms back from the Infinity Cache, not from
    // this XCD's L2, so keeping them in L2 only evicts key lines (2.5% faster score pass)
    if constexpr (DT != KVC_F32) {
      bits = bits16_dt<DT>(r);
      __builtin_nontemporal_store((uint16_t)bits, reinterpret_cast<uint16_t*>(nrow) + tok0 + lane);
    } else {
      bits = f32_to_bits(r);
      __builtin_nontemporal_store(r, reinterpret_cast<float*>(nrow) + tok0 + lane);
    }
  }
  if (ly->score_mode == KVC_SCORE_SNAPKV && tmax) {  // wave-uniform
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bits = max(bits, (uint32_t)__shfl_xor((int)bits, o, 64));
    if (lane == 0) tmax[(int64_t)(ly->row0 + row) * tmax_stride + tt] = bits;
  }
  // Plain-norm rows: level 0's P1 counts, per tile (round 6).  Each wave re-derives the row's
  // level-0 pivot -- the median of the keys at zone positions 1, n/2, n-1, as
  // std::__move_median_to_first picks it (partition_level) -- from those three token rows (L2
  // hits after their first wave) with their norms in torch.norm's order, then counts its tile's
  // keys >= / <= that pivot (ascending keys; a descending selection swaps the two) and stores
  // ge | le << 16.  bf16 / fp32: one lane per (row, accumulator) runs that accumulator's FMA
  // chain and the row's lane adds the eight in order (the tile's own lanes run all eight chains
  // each; a pivot norm on one lane would cost the wave as much VALU work as its whole tile);
  // fp16's single dim-order accumulator stays on one lane per row.
  if (piv) {
#pragma unroll
    for (int q = 0; q < PV; ++q) {
      const int u = lane + 64 * q, r = u / NC, c = u - r * NC;
      if (u < 3 * NC)
        *reinterpret_cast<uint4*>(wl + (r * NPH + c / CP) * ROWB + (c % CP) * 16) = pvr[q];
    }
    wave_sync();
    float ps;
    constexpr int plane = DT == KVC_F16 ? 1 : 8;  // lane holding row r's norm: plane * r
    if constexpr (DT == KVC_F16) {
      float pa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (lane < 3) {
#pragma unroll
        for (int c = 0; c < NC; ++c)
          accum_chunk<DT, NC>(pa, *reinterpret_cast<const uint4*>(wl + (lane * NPH + c / CP) * ROWB +
                                                                   (c % CP) * 16), c);
      }
      ps = pa[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) ps = ps + pa[j];
    } else {
      // lane 8 r + j: accumulator j of row r -- bf16: element j of every chunk; fp32: element
      // j & 3 of the chunks c with c & 1 = j >> 2 (accum_chunk's assignment), in chunk order
      const int r = min(lane >> 3, 2), j = lane & 7;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (DT == KVC_BF16) {
          const uint16_t e = *reinterpret_cast<const uint16_t*>(
              wl + (r * NPH + c / CP) * ROWB + (c % CP) * 16 + j * 2);
          const float x = bits_to_f32((uint32_t)e << 16);
          a = __builtin_fmaf(x, x, a);
        } else {
          if ((c & 1) != (j >> 2)) continue;
          const float x = *reinterpret_cast<const float*>(
              wl + (r * NPH + c / CP) * ROWB + (c % CP) * 16 + (j & 3) * 4);
          a = __builtin_fmaf(x, x, a);
        }
      }
      ps = a;  // lane 8 r: acc[0] + acc[1] + ... + acc[7], in that order
#pragma unroll
      for (int q = 1; q < 8; ++q) ps = ps + __shfl(a, (lane & ~7) + q, 64);
    }
    const float pr = __builtin_sqrtf(ps);
    uint32_t pk;
    if constexpr (DT != KVC_F32) pk = key16_dt<DT>(bits16_dt<DT>(pr), false);
    else pk = key_f32(f32_to_bits(pr), false);
    const uint32_t ka = (uint32_t)__builtin_amdgcn_readlane((int)pk, 0);
    const uint32_t kb = (uint32_t)__builtin_amdgcn_readlane((int)pk, plane);
    const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)pk, 2 * plane);
    const uint32_t p = ka < kb ? (kb < kc ? kb : (ka < kc ? kc : ka))
                               : (ka < kc ? ka : (kb < kc ? kc : kb));
    uint32_t mk;
    if constexpr (DT != KVC_F32) mk = key16_dt<DT>(bits, false);
    else mk = key_f32(bits, false);
    const bool in = lane < ntok;
    const int ge = __popcll(__builtin_amdgcn_ballot_w64(in && mk >= p));
    const int le = __popcll(__builtin_amdgcn_ballot_w64(in && mk <= p));
    if (lane == 0)
      tmax[(int64_t)(ly->row0 + row) * tmax_stride + tt] = (uint32_t)ge | ((uint32_t)le << 16);
    wave_sync();
  }
}

template <int DT, int NC, bool NTL>
__global__ void __launch_bounds__(score_waves(NC) * 64)
    score_kernel(const LayerChunk T, int nl, int H, int64_t tile_base, int64_t chunk_tiles,
                 char* __restrict__ norms, int64_t norm_stride, uint32_t* __restrict__ tmax,
                 int64_t tmax_stride) {
  constexpr int CP = score_cp(NC);
  constexpr int ROWB = score_rowb(CP);
  constexpr int kScoreWaves = score_waves(NC);
  __shared__ __attribute__((aligned(16))) char lds[kScoreWaves][kTile * ROWB];
  const kvc_layer_t* L = T.l;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // one tile per wave (default grid); a smaller grid makes the waves stride over the tiles
  const int64_t stride = (int64_t)gridDim.x * kScoreWaves;
  for (int64_t gl = (int64_t)blockIdx.x * kScoreWaves + wid; gl < chunk_tiles; gl += stride) {
    const int64_t g = tile_base + gl;  // global tile index (kvc_plan's tile0 numbering)
    int lo = 0, hi = nl - 1;  // largest layer with tile0 <= g
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (L[mid].tile0 <= g)
        lo = mid;
      else
        hi = mid - 1;
    }
    const kvc_layer_t* ly = L + lo;
    const int tpr = (ly->zone_len + kTile - 1) / kTile;
    const int local = (int)(g - ly->tile0);
    const int row = local / tpr;
    score_tile<DT, NC, NTL>(ly, row, local - row * tpr, H, lds[wid], norms, norm_stride, tmax,
                            tmax_stride);
  }
}

// ---------------------------------------------------------------------------------------------
// SELECT
// ---------------------------------------------------------------------------------------------
template <typename KeyT>
struct SelScalars {
  int wa[kSelWaves];  // per wave: ge count | le count << 16 (P1); snapkv scratch
  int wb[kSelWaves];  //           snapkv scratch
  int wm[kSelWaves];  //           swaps | first unswapped ge position << 16 (P2)
  float fmax[kSelWaves];
  int fnan[kSelWaves];
};

// Selection arrays for zones of up to n_cap positions:
//   key[n_cap] | idx[n_cap] (u16) | 64 sinks | spos[cap + 8] | 64 sinks | gpos[cap + 8]
// spos / gpos are the s / g rank -> position tables (1-based) of one window of `cap` swap ranks
// (m <= (n-1)/2 swapped pairs per level; a level with m > cap runs its swaps in windows); the 64
// entries before each are per-lane sinks for lanes with nothing to record (branch-free scatter).
// In LDS (dynamic, sized by the call's longest zone), or in a per-row global scratch for zones
// longer than kZoneMax.
__host__ __device__ constexpr size_t sel_bytes(int n_cap, int key_size, int cap) {
  return (size_t)n_cap * key_size + (size_t)n_cap * 2 + (size_t)(64 + cap + 8) * 2 * 2;
}
// Rank-window size for an n_cap-position LDS selection within `budget` bytes of arrays.  16-bit
// keys fit the budget when the tables hold fewer than the n_cap/2 ranks a level can need; levels
// with more swaps take further windows.  fp32 keys (whose snapkv scores use the tables as
// scratch) and short zones get full tables.
__host__ __device__ constexpr int sel_cap(int n_cap, int key_size, long budget) {
  const int full = n_cap / 2 + 1;
  const long tables = budget - (long)n_cap * (key_size + 2) - 4L * 72;  // bytes for the tables
  const int fit = tables > 0 ? (int)(tables / 4) : 0;
  return (key_size == 2 && fit < full && fit >= 1024) ? (fit & ~63) : full;
}
template <typename KeyT>
struct SelArrays {
  KeyT* key;
  uint16_t* idx;
  uint16_t* spos;
  uint16_t* gpos;
  __device__ SelArrays(char* base, int n_cap, int cap)
      : key(reinterpret_cast<KeyT*>(base)),
        idx(reinterpret_cast<uint16_t*>(base + (size_t)n_cap * sizeof(KeyT))),
        spos(idx + n_cap + 64),
        gpos(spos + cap + 8 + 64) {}
};

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }
__device__ __forceinline__ uint64_t lanemask_le(int lane) {
  return lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
}

// 16-bit score conversions of the snapkv keys: bf16 by the c10 bit arithmetic, fp16 by the
// hardware converts (kvc_common.h: c10-exact except NaN payloads, which the keys never see --
// every NaN maps to the one NaN key).
template <int DT>
__device__ __forceinline__ float in16(uint32_t u) {
  if constexpr (DT == KVC_BF16) return bf16_to_f32(u);
  else return f16_to_f32_hw(u);
}
template <int DT>
__device__ __forceinline__ uint32_t out16(float f) {
  if constexpr (DT == KVC_BF16) return f32_to_bf16_rne(f);
  else return f32_to_f16_hw(f);
}

// snapkv_lite importance scores (snapkv_lite.py:96-121) computed from the row's norms and
// written as sort keys:  m = dt(max(norms) + 1e-6);  s = dt(m - norm);
// pooled_i = dt(sum_{window} s / pool_size) (avg_pool1d, zero pad, count_include_pad).
template <int DT, typename KeyT, int NT>
__device__ void snapkv_keys(const char* nrow, int n, int pool_k, bool desc, KeyT* key,
                            char* tmp, SelScalars<KeyT>& sc) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float mx = -__builtin_huge_valf();
  int has_nan = 0;
  for (int i = tid; i < n; i += NT) {
    const float v = load_dt<DT>(nrow, i);
    if (v != v) has_nan = 1;
    else if (v > mx) mx = v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float y = __shfl_xor(mx, o, 64);
    mx = y > mx ? y : mx;
    has_nan |= __shfl_xor(has_nan, o, 64);
  }
  if (lane == 0) {
    sc.fmax[wid] = mx;
    sc.fnan[wid] = has_nan;
  }
  __syncthreads();
  mx = sc.fmax[0];
  has_nan = sc.fnan[0];
  for (int w = 1; w < NT / 64; ++w) {
    mx = sc.fmax[w] > mx ? sc.fmax[w] : mx;
    has_nan |= sc.fnan[w];
  }
  if (has_nan) mx = __builtin_nanf("");
  // `max + 1e-6` (snapkv_lite.py:99): the python scalar takes the tensor's dtype first
  const float m = round_dt<DT>(mx + round_dt<DT>(1e-6f));
  for (int i = tid; i < n; i += NT) {
    const float s = round_dt<DT>(m - load_dt<DT>(nrow, i));
    if constexpr (DT != KVC_F32)
      reinterpret_cast<uint16_t*>(tmp)[i] = (uint16_t)bits16_dt<DT>(s);
    else
      reinterpret_cast<float*>(tmp)[i] = s;
  }
  __syncthreads();
  const bool pool = pool_k > 1 && n >= pool_k;
  const int pad = pool_k / 2;
  for (int i = tid; i < n; i += NT) {
    float r;
    if (pool) {
      int hs = i - pad;
      int he = min(hs + pool_k, n + pad);
      const int psize = he - hs;
      hs = max(hs, 0);
      he = min(he, n);
      float sum = 0.f;
      for (int j = hs; j < he; ++j) sum = sum + load_dt<DT>(tmp, j);
      r = sum / (float)psize;
    } else {
      r = load_dt<DT>(tmp, i);
    }
    key[i] = key_of<DT>(r, desc);
  }
}

// x / 5 correctly rounded (= the IEEE division avg_pool1d performs), without the division
// sequence: q0 = x * RN(1/5), residual r = x - 5 q0 exact in one FMA, q1 = q0 + r * RN(1/5);
// q0 itself where r == 0 (keeps -0) or q0 is infinite.  Checked against x / 5.0f for all 2^32
// fp32 patterns (tests/native/div5_check.c; tests/test_native_abi.py runs a strided sample).
__device__ __forceinline__ float div5_rn(float x) {
  const float q0 = x * 0.2f;
  const float r = __builtin_fmaf(-q0, 5.0f, x);
  return (r == 0.0f || __builtin_isinf(q0)) ? q0 : __builtin_fmaf(r, 0.2f, q0);
}

// The pooled key vector of positions 8v .. 8v+7 (default pooling kernel 5, or none) from the
// 16-bit scores of positions 8v-8 .. 8v+15 as floats in sw[0..24) (only 8v-2 .. 8v+9 are read;
// terms outside [hs, he) are skipped): avg_pool1d's window sums in its order, / 5 by div5_rn,
// rounded to the dtype, mapped to sort keys; positions past n get 0.
// nonneg (bf16): every score of the row is finite and >= +0 -- the row max is finite, so m >=
// every norm, and a finite norm is at most sqrt(FLT_MAX) < 2e19, so no whole-window sum (<= 5 m)
// overflows.  div5_rn's guards then never fire but for r == 0, which only decides the sign of a
// zero quotient (the keys equate +0 and -0), the division runs as packed fp32 ops, and a value
// >= +0 maps to key 0x8000 | bits, key_bf16x2's code for it.
template <int DT>
__device__ __forceinline__ uint4 snapkv_pool_vec(const float (&sw)[24], int v, int n, bool pool,
                                                 bool desc, bool nonneg = false) {
  uint32_t o[4] = {0, 0, 0, 0};
  if constexpr (DT == KVC_BF16) {
    // bf16: pairs of positions with packed fp32 adds, one hardware convert and one packed key
    // map per pair (key_bf16x2 codes for every key of the row).  The window sums drop
    // avg_pool1d's leading 0 + s: it only turns a -0 into +0, and the keys equate the two.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const bool inner = pool && v >= 1 && v * 8 + 10 <= n;  // every window of the vector whole
    if (inner && nonneg) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        f2 acc = f2{sw[2 * p + 6], sw[2 * p + 7]};
#pragma unroll
        for (int t = 1; t < 5; ++t) acc = acc + f2{sw[2 * p + 6 + t], sw[2 * p + 7 + t]};
        const f2 q0 = acc * f2{0.2f, 0.2f};
        const f2 r = __builtin_elementwise_fma(-q0, f2{5.0f, 5.0f}, acc);
        const f2 q = __builtin_elementwise_fma(r, f2{0.2f, 0.2f}, q0);
        const uint32_t k = f32x2_to_bf16x2_hw(q.x, q.y) | 0x80008000u;
        o[p] = desc ? ~k : k;  // inner: all 8 positions < n
      }
      return make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      f2 r;
      if (inner) {
        f2 acc = f2{sw[2 * p + 6], sw[2 * p + 7]};
#pragma unroll
        for (int t = 1; t < 5; ++t) acc = acc + f2{sw[2 * p + 6 + t], sw[2 * p + 7 + t]};
        r = f2{div5_rn(acc.x), div5_rn(acc.y)};
      } else {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int e = 2 * p + b, i = v * 8 + e;
          float x = sw[8 + e];
          if (pool) {  // pool_k == 5, pad 2: window [i - 2, i + 3) clipped to [0, n), / 5
            int hs = i - 2;
            int he = min(hs + 5, n + 2);
            const int psize = he - hs;
            hs = max(hs, 0);
            he = min(he, n);
            float sum = 0.f;
#pragma unroll
            for (int t = 0; t < 5; ++t) {
              const int j = i - 2 + t;
              if (j >= hs && j < he) sum = sum + sw[8 + e - 2 + t];
            }
            x = psize == 5 ? div5_rn(sum) : sum / (float)psize;
          }
          r[b] = x;
        }
      }
      const int i0 = v * 8 + 2 * p;
      o[p] = key_bf16x2(f32x2_to_bf16x2_hw(r.x, r.y), desc) &
             (i0 + 1 < n ? 0xFFFFFFFFu : i0 < n ? 0x0000FFFFu : 0u);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int i = v * 8 + e;
      float r;
      if (pool) {  // pool_k == 5, pad 2: window [i - 2, i + 3) clipped to [0, n), / 5
        int hs = i - 2;
        int he = min(hs + 5, n + 2);
        const int psize = he - hs;
        hs = max(hs, 0);
        he = min(he, n);
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const int j = i - 2 + t;
          if (j >= hs && j < he) sum = sum + sw[8 + e - 2 + t];
        }
        r = psize == 5 ? div5_rn(sum) : sum / (float)psize;
      } else {
        r = sw[8 + e];
      }
      o[e >> 1] |= (i < n ? (uint32_t)key16_dt<DT>(out16<DT>(r), desc) : 0u) << (16 * (e & 1));
    }
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// 16-bit scores s = dt(m - norm) of the two positions of a norm dword (the positions' order in
// the dword kept): bf16 by one hardware convert per pair (NaN payloads unobserved), fp16 by the
// hardware converts.
template <int DT>
__device__ __forceinline__ uint32_t snapkv_score_pair(float m, uint32_t w) {
  if constexpr (DT == KVC_BF16)
    return f32x2_to_bf16x2_hw(m - bf16_to_f32(w), m - bits_to_f32(w & 0xFFFF0000u));
  else
    return out16<DT>(m - in16<DT>(w & 0xFFFFu)) | (out16<DT>(m - in16<DT>(w >> 16)) << 16);
}

// snapkv_keys for 16-bit scores on LDS rows (n <= MAXV * 8 * NT): the same arithmetic per
// position (snapkv_lite.py:96-121), each thread making the keys of 8 consecutive positions.
// `key`, `idx`, `tmp` and `nrow` are 16-B aligned; norm rows are padded to a multiple of 64
// elements (a vector or dword past n stays inside the row; its values are never used).
//  * With `trow` (SCORE's per-tile maxima of this row, score_tile) and the default pooling kernel
//    5 (or none): no block barrier and no scores round trip -- every wave reduces the tile
//    maxima to `max(norms)` itself, and each thread forms the scores of its 8 positions and the
//    two on either side (a 16-B load of its norms and two 4-B halo loads) in registers, pools
//    them and writes its keys AND its index vector (returns true: idx is initialised).
//  * Otherwise (rounds 2-5 form): the row's norms read once as 16-B vectors (kept in registers
//    for the max and the scores), a block max, scores stored to `tmp` as 16-B vectors, and each
//    thread pooling 8 positions from three 16-B reads of them (kernel 5; other kernels one
//    position at a time as snapkv_keys).  Returns false: the caller initialises idx (tmp
//    aliases it).
template <int DT, int NT, int MAXV>
__device__ __forceinline__ bool snapkv_keys16(const char* nrow, const uint32_t* trow, int n,
                                              int pool_k, bool desc, uint16_t* key, uint16_t* idx,
                                              uint16_t* tmp, SelScalars<uint16_t>& sc,
                                              uint64_t* stamps = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nvec = (n + 7) >> 3;
  constexpr uint32_t kInf = DT == KVC_BF16 ? 0x7F80u : 0x7C00u;
  const bool pool = pool_k > 1 && n >= pool_k;
  if (trow && (pool_k == 5 || !pool)) {
    // max(norms) from the tile maxima (bits of the stored norms, at most 256 tiles: <= 4 loads
    // per lane), one wave reduction; a NaN's bits exceed +inf's.  (Issuing every norm load
    // before this reduction measured the same: profiles/r06_b_snapkv_ab.jsonl, snap2.)
    uint32_t mb = 0;
    const int nt = (n + kTile - 1) / kTile;
    for (int t = lane; t < nt; t += 64) mb = max(mb, trow[t]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (uint32_t)__shfl_xor((int)mb, o, 64));
    const float mx = mb > kInf ? __builtin_nanf("") : in16<DT>(mb);
    // `max + 1e-6` (snapkv_lite.py:99): the python scalar takes the tensor's dtype first
    const float m = in16<DT>(out16<DT>(mx + in16<DT>(out16<DT>(1e-6f))));
    const bool nonneg = mb < kInf;  // finite max: every score m - norm is finite and >= +0
    KVC_STAMP(26);
    const uint32_t* nw = reinterpret_cast<const uint32_t*>(nrow);
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      const int v = tid + q * NT;
      if (v >= nvec) continue;
      const uint4 c = reinterpret_cast<const uint4*>(nrow)[v];
      const uint32_t wp = v > 0 ? nw[4 * v - 1] : 0u;          // positions 8v-2, 8v-1
      const uint32_t wn = v + 1 < nvec ? nw[4 * v + 4] : 0u;   // positions 8v+8, 8v+9
      const uint32_t sc6[6] = {snapkv_score_pair<DT>(m, wp), snapkv_score_pair<DT>(m, c.x),
                               snapkv_score_pair<DT>(m, c.y), snapkv_score_pair<DT>(m, c.z),
                               snapkv_score_pair<DT>(m, c.w), snapkv_score_pair<DT>(m, wn)};
      float sw[24];
#pragma unroll
      for (int e = 0; e < 24; ++e) sw[e] = 0.f;
#pragma unroll
      for (int d = 0; d < 6; ++d) {  // scores of positions 8v - 2 + 2d, +1 at sw[6 + 2d], +1
        sw[6 + 2 * d] = in16<DT>(sc6[d] & 0xFFFFu);
        sw[7 + 2 * d] = in16<DT>(sc6[d] >> 16);
      }
      reinterpret_cast<uint4*>(key)[v] = snapkv_pool_vec<DT>(sw, v, n, pool, desc, nonneg);
      const uint32_t b = (uint32_t)v * 8;
      reinterpret_cast<uint4*>(idx)[v] =
          make_uint4(b | (b + 1) << 16, (b + 2) | (b + 3) << 16, (b + 4) | (b + 5) << 16,
                     (b + 6) | (b + 7) << 16);
    }
    KVC_STAMP(29);
    return true;
  }
  uint4 raw[MAXV];
  float mx = -__builtin_huge_valf();
  // Branch-free local max: the NaN-ignoring float max (v_max_f32) of every element, NaN
  // detected apart as the packed-u16 max magnitude above inf.  Positions past n read as -inf.
  // (A signed zero max is harmless: m = dt(max + 1e-6) is the same for -0 and +0.)
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  u16x2 mag = (u16x2)0;
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int v = tid + q * NT;
    raw[q] = v < nvec ? reinterpret_cast<const uint4*>(nrow)[v] : make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int v = tid + q * NT;
    const uint32_t w[4] = {raw[q].x, raw[q].y, raw[q].z, raw[q].w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int i0 = v * 8 + 2 * h;
      const uint32_t ninf = 0x8000u | kInf;  // -inf
      const uint32_t x = i0 + 1 < n ? w[h] : i0 < n ? (w[h] & 0xFFFFu) | (ninf << 16)
                                                     : ninf | (ninf << 16);
      mx = __builtin_fmaxf(mx, __builtin_fmaxf(in16<DT>(x & 0xFFFFu), in16<DT>(x >> 16)));
      mag = __builtin_elementwise_max(mag, __builtin_bit_cast(u16x2, x & 0x7FFF7FFFu));
    }
  }
  int has_nan = (mag.x > kInf || mag.y > kInf) ? 1 : 0;
  KVC_STAMP(26);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float y = __shfl_xor(mx, o, 64);
    mx = __builtin_fmaxf(mx, y);
    has_nan |= __shfl_xor(has_nan, o, 64);
  }
  if (lane == 0) {
    sc.fmax[wid] = mx;
    sc.fnan[wid] = has_nan;
  }
  __syncthreads();
  mx = sc.fmax[0];
  has_nan = sc.fnan[0];
  for (int w = 1; w < NT / 64; ++w) {
    mx = __builtin_fmaxf(mx, sc.fmax[w]);
    has_nan |= sc.fnan[w];
  }
  if (has_nan) mx = __builtin_nanf("");
  // `max + 1e-6` (snapkv_lite.py:99): the python scalar takes the tensor's dtype first
  const float m = in16<DT>(out16<DT>(mx + in16<DT>(out16<DT>(1e-6f))));
  KVC_STAMP(27);
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int v = tid + q * NT;
    if (v >= nvec) continue;
    const uint32_t w[4] = {raw[q].x, raw[q].y, raw[q].z, raw[q].w};
    uint32_t o[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int i0 = v * 8 + 2 * h;
      o[h] = snapkv_score_pair<DT>(m, w[h]) &
             (i0 + 1 < n ? 0xFFFFFFFFu : i0 < n ? 0x0000FFFFu : 0u);
    }
    reinterpret_cast<uint4*>(tmp)[v] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();
  KVC_STAMP(28);
  if (pool && pool_k != 5) {  // other kernels: one position at a time (snapkv_keys)
    const int pad = pool_k / 2;
    for (int i = tid; i < n; i += NT) {
      int hs = i - pad;
      int he = min(hs + pool_k, n + pad);
      const int psize = he - hs;
      hs = max(hs, 0);
      he = min(he, n);
      float sum = 0.f;
      for (int j = hs; j < he; ++j) sum = sum + in16<DT>(tmp[j]);
      key[i] = key16_dt<DT>(out16<DT>(sum / (float)psize), desc);
    }
    return false;
  }
  const uint4* tv = reinterpret_cast<const uint4*>(tmp);
#pragma unroll
  for (int q = 0; q < MAXV; ++q) {
    const int v = tid + q * NT;
    if (v >= nvec) continue;
    // scores of positions 8v - 8 .. 8v + 15 (zero outside the row: never summed)
    float sw[24];
    const uint4 c3[3] = {v > 0 ? tv[v - 1] : make_uint4(0, 0, 0, 0), tv[v],
                         v + 1 < nvec ? tv[v + 1] : make_uint4(0, 0, 0, 0)};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint32_t w[4] = {c3[c].x, c3[c].y, c3[c].z, c3[c].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t u = (w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
        sw[c * 8 + e] = in16<DT>(u);
      }
    }
    reinterpret_cast<uint4*>(key)[v] = snapkv_pool_vec<DT>(sw, v, n, pool, desc);
  }
  KVC_STAMP(29);
  return false;
}

template <int NT>
__device__ __forceinline__ void group_sync() {
  if constexpr (NT == 64)
    wave_sync();
  else
    __syncthreads();
}

// The final insertion sort of a <= 64-element segment [lo, hi) (std::__insertion_sort /
// __unguarded_linear_insert: an element moves left only past strictly greater ones, i.e. a
// STABLE sort by key) computed by one wave in parallel: lane i holds element i and stores it at
// #{key_j < key_i} + #{j < i : key_j == key_i}.  Every lane reads its element before any lane
// of the wave stores (the ranks need all of them), so the in-place stores are race-free.
// Replaces a one-lane loop of dependent LDS accesses.  Call with all 64 lanes of one wave.
template <typename KeyT>
__device__ __forceinline__ void wave_stable_sort(KeyT* key, uint16_t* idx, int lo, int hi) {
  const int lane = threadIdx.x & 63;
  const int m = hi - lo;
  const bool own = lane < m;
  const uint32_t kk = own ? (uint32_t)key[lo + lane] : 0u;
  const uint16_t ii = own ? idx[lo + lane] : (uint16_t)0;
  int r = 0;
  for (int j = 0; j < m; ++j) {  // m is wave-uniform
    const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)kk, j);
    r += (kj < kk || (kj == kk && j < lane)) ? 1 : 0;
  }
  if (own) {
    key[lo + r] = (KeyT)kk;
    idx[lo + r] = ii;
  }
}

// std::__heap_select(first, first + middle, first + len) -- std::partial_sort's selection, which
// torch.topk uses when k * 64 <= n (aten TopKImpl.h) -- run by one wave: lane 0 builds the heap
// and performs every pop_heap exactly as libstdc++ does (kvc_serial.h), while the wave scans the
// candidates 64 at a time: element i enters iff key[i] < key[0] at its turn, and key[0] only
// decreases, so a ballot against the current top leaves exactly the elements the serial loop
// would pop, in index order (re-checked against the new top after each pop).  The scan of the
// n - middle elements no longer costs one dependent LDS round trip each.  For middle <= 64 (the
// h2o heavy hitters' 64) the heap itself lives in the wave's registers (RegHeap) and only its
// final slots are stored; otherwise lane 0 keeps it in LDS.  Call with all 64 lanes of one wave;
// the result is the first `middle` positions (positions >= middle are not part of it).
// The heap of a wave_heap_select with middle <= 64 held in registers: lane j owns heap slot j
// (key hk, index hi).  adjust() is std::__adjust_heap + std::__push_heap (kvc_serial.h
// adjust_heap) computed wave-parallel instead of level by level:
//   * the down phase moves the hole along the path of "chosen" children (the right child unless
//     it is strictly smaller than the left; a lone child at (len-2)/2 for even len) to a leaf,
//     every path node taking its chosen child's entry;
//   * the up phase moves the value back up while its parent is strictly smaller.  Path keys do
//     not increase with depth (heap order), so it stops at depth m = #{path nodes below `top`
//     with !(key < value)}, and its moves undo the down phase below m.
// Net effect: path depths 0..m-1 take their chosen child's entry, depth m takes the value, the
// rest of the heap is unchanged; m is one ballot.
// PACKED (16-bit keys and positions): slot j's entry is one word, key << 16 | index, so each
// pop permutes one register instead of two (the children's keys and indices travel together).
template <bool PACKED>
struct RegHeap {
  uint32_t hk;   // PACKED: key << 16 | index
  uint32_t hi;   // !PACKED: index
  uint64_t anc;  // this slot and its ancestors below the root, as lane bits (fixed per lane)
  int dep;       // this slot's depth
  __device__ __forceinline__ uint32_t key_of(uint32_t x) const { return PACKED ? x >> 16 : x; }
  __device__ __forceinline__ uint32_t k(int j) const {
    return key_of((uint32_t)__builtin_amdgcn_readlane((int)hk, j));
  }
  __device__ __forceinline__ uint32_t i(int j) const {
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)(PACKED ? hk : hi), j);
    return PACKED ? x & 0xFFFFu : x;
  }
  __device__ __forceinline__ void set(uint32_t key, uint32_t ix) {
    if constexpr (PACKED) hk = key << 16 | ix;
    else hk = key, hi = ix;
    int a = (int)(threadIdx.x & 63), d = 0;
    uint64_t m = 0;
#pragma unroll
    for (int st = 0; st < 6; ++st) {  // 64 slots: depth <= 6
      m |= a > 0 ? 1ull << a : 0ull;
      d += a > 0 ? 1 : 0;
      a = a > 0 ? (a - 1) >> 1 : 0;
    }
    anc = m;
    dep = d;
  }
  // std::__adjust_heap + std::__push_heap from slot `top` with value (vk, vi), wave-parallel.
  // The only serial chain is: sibling keys by DPP wave shifts -> "my parent chose me" bits ->
  // one ballot B -> the path (each lane: are all links from top down to it in B, one mask test
  // against its ancestor bits) -> m, one ballot.  Both children's entries are fetched with
  // ds_bpermute at the start, off that chain.  (Round 3: a readlane chase of the path and
  // bpermutes of the children's keys before it, ~630 cycles per pop in tools/heap_probe.hip.)
  __device__ __forceinline__ void adjust(int top, int len, uint32_t vk, uint32_t vi) {
    const int lane = (int)(threadIdx.x & 63);
    const int c1 = min(2 * lane + 1, 63), c2 = min(2 * lane + 2, 63);
    const uint32_t pl = (uint32_t)__builtin_amdgcn_ds_bpermute(c1 * 4, (int)hk);
    const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute(c2 * 4, (int)hk);
    uint32_t il = 0, ir = 0;
    if constexpr (!PACKED) {
      il = (uint32_t)__builtin_amdgcn_ds_bpermute(c1 * 4, (int)hi);
      ir = (uint32_t)__builtin_amdgcn_ds_bpermute(c2 * 4, (int)hi);
    }
    const uint32_t key = key_of(hk);
    const uint32_t kn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x130, 0xF, 0xF, false);  // wave_shl:1: lane + 1
    const uint32_t kp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x138, 0xF, 0xF, false);  // wave_shr:1: lane - 1
    const int p = (lane - 1) >> 1;                              // parent of this lane
    // (bitwise, not short-circuit: && / || here compiled to exec-mask branches)
    const unsigned two = p < (len - 1) / 2 ? 1u : 0u;           // the parent has both children
    const unsigned lone = (len & 1) == 0 && p == (len - 2) / 2 ? 1u : 0u;  // only the left one
    const unsigned in = lane >= 1 && lane < len ? 1u : 0u;
    // the right child unless it is strictly smaller than the left (std::__adjust_heap)
    const unsigned cl = lone | (two & (kn < key ? 1u : 0u));   // left child (odd lane) chosen
    const unsigned cr = two & (key < kp ? 0u : 1u);             // right child (even lane) chosen
    const uint64_t B = __builtin_amdgcn_ballot_w64((in & ((lane & 1) ? cl : cr)) != 0u);
    // on the path from `top`: a descendant of top (or top) whose links below top are all in B
    uint64_t links = anc;
    int d = dep;
    bool desc = true;
    if (top != 0) {  // wave-uniform: make_heap's sift-downs
      const uint64_t at = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)anc, top) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(anc >> 32), top) << 32);
      links = anc & ~at;
      d = dep - __builtin_amdgcn_readlane(dep, top);
      desc = (anc >> top) & 1ull;
    }
    const unsigned onpath = desc && (B & links) == links ? 1u : 0u;
    const int m = __popcll(__builtin_amdgcn_ballot_w64(
        (onpath & (d >= 1 ? 1u : 0u) & (key < vk ? 0u : 1u)) != 0u));
    const bool left = (B >> c1) & 1ull;  // this slot's chosen child (path slots above the leaf)
    const uint32_t ck = (uint32_t)vreg((int)(left ? pl : pr));
    const bool up = (onpath & (d < m ? 1u : 0u)) != 0u, here = (onpath & (d == m ? 1u : 0u)) != 0u;
    const uint32_t v = PACKED ? (vk << 16 | vi) : vk;
    hk = up ? ck : here ? v : hk;
    if constexpr (!PACKED) hi = up ? (uint32_t)vreg((int)(left ? il : ir)) : here ? vi : hi;
  }
};

// The register heap of wave_heap_select (middle <= 64), in two steps so that a block can build
// it in one wave while its other waves prefilter the candidates (heap_candidates):
// std::make_heap over the first `middle` slots ...
template <bool PK, typename K, typename I>
__device__ __forceinline__ void reg_heap_make(RegHeap<PK>& h, const K* key, const I* idx,
                                              int middle) {
  const int lane = threadIdx.x & 63;
  h.set(lane < middle ? (uint32_t)key[lane] : 0u, lane < middle ? (uint32_t)idx[lane] : 0u);
  if (middle >= 2)
    for (int parent = (middle - 2) / 2; parent >= 0; --parent)
      h.adjust(parent, middle, h.k(parent), h.i(parent));
}
// ... then the scan of positions [middle, len) -- or only the ascending candidate positions
// `cand[0..ncand)` -- with its pops, and the heap's slots stored to key / idx[0..middle).
template <bool PK, typename K, typename I>
__device__ __forceinline__ void reg_heap_scan(RegHeap<PK>& h, K* key, I* idx, int middle, int len,
                                              const uint16_t* cand, int ncand) {
  const int lane = threadIdx.x & 63;
  uint32_t top = h.k(0);
  // the scan, eight rows of 64 candidates per LDS round trip (the loads do not depend on the
  // heap; only the ballots and pops do).  idx[i] == i on entry (every caller), so a candidate's
  // index is its position.
  constexpr int R = 8;
  const int end = cand ? ncand : len, first = cand ? 0 : middle;
  for (int base = first; base < end; base += 64 * R) {
    uint32_t kq[R], pq[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = base + q * 64 + lane;
      pq[q] = cand ? (uint32_t)cand[min(i, end - 1)] : (uint32_t)i;
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = base + q * 64 + lane;
      kq[q] = i < end ? (uint32_t)key[pq[q]] : 0xFFFFFFFFu;
    }
    // lanes past the end hold ~0, never below top (16-bit keys are below 2^16); the rows'
    // ballots against the current top first: most groups late in the row hold no candidate
    uint64_t cm[R], any = 0;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      cm[q] = __builtin_amdgcn_ballot_w64(kq[q] < top);
      any |= cm[q];
    }
    if (!any) continue;
#pragma unroll
    for (int q = 0; q < R; ++q) {
      // top only decreases: a row's candidates against the current top are a subset of cm[q]
      uint64_t c = cm[q] & __builtin_amdgcn_ballot_w64(kq[q] < top);
      while (c) {
        const int l = (int)__builtin_ctzll(c);
        // std::__pop_heap(first, middle, i): the old top goes to position i (never read again:
        // only the heap's slots are the result), element i sifts in from the root
        h.adjust(0, middle, (uint32_t)__builtin_amdgcn_readlane((int)kq[q], l),
                 (uint32_t)__builtin_amdgcn_readlane((int)pq[q], l));
        top = h.k(0);
        c &= ~((2ull << l) - 1ull) & __builtin_amdgcn_ballot_w64(kq[q] < top);
      }
    }
  }
  if (lane < middle) {
    key[lane] = (K)h.key_of(h.hk);
    idx[lane] = (I)(PK ? (h.hk & 0xFFFFu) : h.hi);
  }
}

template <typename K, typename I>
__device__ __forceinline__ void wave_heap_select(K* key, I* idx, int middle, int len) {
  const int lane = threadIdx.x & 63;
  if (middle <= 64) {  // the heap in registers (RegHeap): make_heap, then the scan with its pops
    constexpr bool PK = sizeof(K) == 2 && sizeof(I) == 2;
    RegHeap<PK> h;
    reg_heap_make(h, key, idx, middle);
    reg_heap_scan(h, key, idx, middle, len, nullptr, 0);
    wave_sync();
    return;
  }
  if (lane == 0) make_heap(key, idx, middle);
  wave_sync();
  uint32_t top = (uint32_t)key[0];
  for (int base = middle; base < len; base += 64) {
    const int i = base + lane;
    const uint32_t ki = i < len ? (uint32_t)key[i] : 0xFFFFFFFFu;
    uint64_t cand = __builtin_amdgcn_ballot_w64(i < len && ki < top);
    while (cand) {
      const int l = (int)__builtin_ctzll(cand);
      if (lane == 0) pop_heap(key, idx, middle, base + l);
      wave_sync();
      top = (uint32_t)key[0];
      cand &= ~((2ull << l) - 1ull) & __builtin_amdgcn_ballot_w64(ki < top);
    }
  }
  wave_sync();
}

// The partition chain of libstdc++ introsort (topk = false) / introselect (topk = true),
// following only the segment [lo, hi) that straddles position k, run by NT cooperating lanes
// (the whole 1024-thread block, or one wave once the segment is short).  One level is
// std::__move_median_to_first + std::__unguarded_partition(lo+1, hi, pivot=lo) computed in
// parallel:
//   g_t = t-th position (ascending) in [lo+1,hi) with !(key < p)            ("ge")
//   s_t = t-th position (descending) with !(p < key), then the pivot slot lo ("le")
// libstdc++ swaps g_t <-> s_t for every t with g_t < s_t -- a prefix t <= m -- and returns
// cut = min(g_{m+1}, s_m).  With A(x) = #ge before x and Lin(x) = #le in [lo+1, x]:
//   g_t < s_t  <=>  A(g_t) + Lin(g_t) < tot_le
// (tests/native/select_model.cpp validates the chain against libstdc++), so m is counted in
// the same pass that scatters the s rank -> position table.  Positions are laid out j-major
// (lane + 64*j within a wave's stripe) so ge/le flags are wave ballots; every j-loop is fully
// unrolled and loads are issued before dependent stores, keeping LDS latency off the chain.
// Returns 0 when the first-k set is final, 1 when the block hands a short segment to one wave.
#ifdef KVC_STAMPS
#define KVC_TICK(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define KVC_TICK(v) (void)0
#endif

// Uniform (wave-invariant) value into an SGPR, so that the arithmetic on it runs on the scalar
// unit instead of costing a 4-cycle wave64 VALU slot in every wave.
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// inclusive prefix sum within each 16-lane row (4 DPP adds); lanes 0..15 = the 16 waves
__device__ __forceinline__ int row_scan16(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);  // row_shr:8
  return v;
}
// popcount of a wave-uniform mask on the VALU (v_bcnt reading the SGPRs; the result in every
// lane): a scalar s_bcnt1 of a mask a VALU compare has just written waits for that compare
__device__ __forceinline__ int vpopc(uint64_t m) {
  int r;
  asm("v_bcnt_u32_b32 %0, %1, 0\n\tv_bcnt_u32_b32 %0, %2, %0"
      : "=&v"(r)
      : "s"((uint32_t)m), "s"((uint32_t)(m >> 32)));
  return r;
}
// lanes below this one with their bit set in `mask`, plus `base` (v_mbcnt_lo/hi: 2 VALU)
__device__ __forceinline__ int mbcnt(uint64_t mask, int base) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, (uint32_t)base));
}

// f(integral_constant<int, I>) for I in [B, E): a loop the compiler cannot leave rolled.
template <int B, int E, typename F>
__device__ __forceinline__ void unroll_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>());
    unroll_for<B + 1, E>(f);
  }
}

// P1 of a level: the ge / le counts of one wave's stripe, counted per lane on the VALU (packed
// ge | le << 16) and summed once per pass (a 16-lane DPP scan, four readlanes).  Ballot counts
// (s_bcnt + s_add per row on the scalar unit, which all 32 waves of a CU share) cost the
// selection 2 % (SELECT_GATHER 0.1525 -> 0.1494 ms at the headline, 0.187 -> 0.183 snapkv,
// 0.128 -> 0.124 h2o; profiles/r03_zz_valu_counts_ab.jsonl): the kernel is bound by the CU's
// total issue work and the scalar unit carried the larger share.
// WHOLE: every position of the stripe is below hi (unclamped loads with immediate offsets; rows
// j >= J of a JM-row body read at most JM/2 rows past the stripe -- the smallest body, 1 --
// inside the selection arrays).  Otherwise loads are clamped and lanes past hi masked off.
// Position ch is counted with the key it holds (the pivot value); the caller corrects the owner
// wave's counts for the virtual median move.
// A level body of bound JM runs levels with JM/2 < J <= JM, so rows j < JM/2 need no J check --
// except the smallest body (kLevelJmMin), which runs every J <= JM
template <int JM>
__device__ constexpr int jm_rows_past() {
  return JM <= kLevelJmMin ? 1 : JM / 2;
}
template <typename KeyT, int JM, bool WHOLE>
__device__ __forceinline__ void p1_counts(const KeyT* key, int pos0, int J, int hi, uint32_t p,
                                          int& cge, int& cle) {
  constexpr int JB = JM < 16 ? JM : 16;
  uint32_t pc = 0;  // per-lane counts: ge | le << 16 (at most 64 per lane)
  unroll_for<0, JM / JB>([&](auto bc) {
    constexpr int j0 = decltype(bc)::value * JB;
    if (j0 > 0 && j0 >= J) return;
    KeyT kv[JB];
    unroll_for<0, JB>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int pos = pos0 + (j0 + q) * 64;
      kv[q] = key[WHOLE ? pos : min(pos, hi - 1)];
    });
    unroll_for<0, JB>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int j = j0 + q;
      if (j >= jm_rows_past<JM>() && j >= J) return;
      bool ge = (uint32_t)kv[q] >= p, le = (uint32_t)kv[q] <= p;
      if constexpr (!WHOLE) {
        const bool inb = pos0 + j * 64 < hi;
        ge = ge && inb;
        le = le && inb;
      }
      pc += (ge ? 1u : 0u) + (le ? 0x10000u : 0u);
    });
  });
  const int rs = row_scan16((int)pc);  // per 16-lane row; the four row totals on the scalar unit
  const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(rs, 15) +
                       (uint32_t)__builtin_amdgcn_readlane(rs, 31) +
                       (uint32_t)__builtin_amdgcn_readlane(rs, 47) +
                       (uint32_t)__builtin_amdgcn_readlane(rs, 63);
  cge += (int)(tot & 0xFFFFu);
  cle += (int)(tot >> 16);
}

// Candidate prefilter of std::__heap_select(first, middle, last) for middle <= 64, by NT
// threads: position i >= middle enters the heap iff key[i] < top_i, and top_i -- the heap's max
// -- is the middle-th smallest key of [0, i) (the heap always holds the `middle` smallest keys
// seen, as a multiset).  Any `middle`-element subset of [0, i) bounds it from above, so with the
// scan range cut into one chunk per wave, U_w = min(max of the first `middle` keys, the
// middle-th smallest key of each earlier chunk) >= top_i for every i of chunk w, and {i in chunk
// w : key[i] < U_w} holds every entering position.  Writes those positions, ascending, to `cand`
// (capacity ccap) and returns their count, or -1 (nothing written) when they do not fit or a
// chunk exceeds 20 rows of 64; ends with a barrier.  The heap scan then visits only them:
// ~1 800 of 15 936 positions for the h2o heavy hitters (k = 64).
template <int NT, bool EXACT = true, typename K>
__device__ int heap_candidates(const K* key, int middle, int len, uint16_t* cand, int ccap,
                               int* wbuf, int* cbuf, int w0 = 0) {
  constexpr int NW = NT / 64, JM = 20;  // 16 384 positions over 15 chunk waves: 17 rows
  static_assert(NW <= 16, "one 16-lane DPP row holds the wave values");
  const int lane = threadIdx.x & 63, wid = uni((int)(threadIdx.x >> 6));
  const int span = len - middle;
  const int rows = (span + 64 * (NW - w0) - 1) / (64 * (NW - w0));  // rows per chunk (uniform)
  if (rows > JM) return -1;
  // waves below w0 (busy elsewhere until the first barrier) hold no chunk
  const int c0 = wid < w0 ? len : middle + (wid - w0) * rows * 64, c1 = min(c0 + rows * 64, len);
  uint32_t kv[JM];
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int pos = c0 + j * 64 + lane;
    const bool v = j < rows && pos < c1;
    kv[j] = v ? (uint32_t)key[pos] : 0xFFFFFFFFu;
    mn = v ? min(mn, kv[j]) : mn;
    mx = v ? max(mx, kv[j]) : mx;
  }
  uint32_t q0 = lane < middle ? (uint32_t)key[lane] : 0u;  // max of the first `middle` keys
  if (!EXACT) mx = mn;  // loose bound: the largest lane minimum (>= 64 keys lie at or below it)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    if (EXACT) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    q0 = max(q0, (uint32_t)__shfl_xor((int)q0, o, 64));
  }
  // this chunk's middle-th smallest key: the smallest v with #(key <= v) >= middle (bisection on
  // the VALU, one wave reduction per step); loose: every lane holds a key (a full first row)
  uint32_t lo = EXACT ? (uint32_t)uni((int)mn) : (uint32_t)uni((int)mx), hi = (uint32_t)uni((int)mx);
  const bool has = EXACT ? c1 - c0 >= middle : c1 - c0 >= 64;
  while (EXACT && has && lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int cl = 0;
#pragma unroll
    for (int j = 0; j < JM; ++j) cl += kv[j] <= mid ? 1 : 0;  // invalid slots hold ~0u
    const int rs = row_scan16(cl);
    const int c = __builtin_amdgcn_readlane(rs, 15) + __builtin_amdgcn_readlane(rs, 31) +
                  __builtin_amdgcn_readlane(rs, 47) + __builtin_amdgcn_readlane(rs, 63);
    if (c >= middle) hi = mid;
    else lo = mid + 1;
  }
  if (lane == 0) wbuf[wid] = has ? (int)lo : -1;  // -1: no bound (0xFFFFFFFF)
  __syncthreads();
  uint32_t U = (uint32_t)uni((int)q0);
  for (int w = 0; w < wid; ++w) U = min(U, (uint32_t)wbuf[w]);
  int c = 0;
#pragma unroll
  for (int j = 0; j < JM; ++j) c += __popcll(__builtin_amdgcn_ballot_w64(kv[j] < U));
  if (lane == 0) cbuf[wid] = c;
  __syncthreads();
  int before = 0, total = 0;
  for (int w = 0; w < NW; ++w) {
    const int cw = cbuf[w];
    before += w < wid ? cw : 0;
    total += cw;
  }
  if (total > ccap) {
    __syncthreads();  // wbuf / cbuf are free again
    return -1;
  }
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const uint64_t b = __builtin_amdgcn_ballot_w64(kv[j] < U);
    if (kv[j] < U) cand[before + mbcnt(b, 0)] = (uint16_t)(c0 + j * 64 + lane);
    before += __popcll(b);
  }
  __syncthreads();
  return total;
}

// P2 of a level, rank window 0: scatter the s and g rank -> position tables for ranks <= cap
// and count the swaps (nsw), from re-read keys.  With F(x) = A(x) + Lin(x) (non-decreasing in
// x), a ge position is swapped iff F < tot_le and an le position iff F > tot_le, and only the
// swapped g's and s's plus g_{m+1} are ever read back.  So a whole stripe (MODE):
//   P2_FULL  straddles F = tot_le: records every ge and le rank <= cap, counts its swaps;
//   P2_LEFT  ends at F <= tot_le: every ge swapped (nsw = its ge count, set by the caller), no
//            le swapped -- records the g ranks only;
//   P2_RIGHT starts at F >= tot_le: no ge swapped, every le swapped -- records the s ranks and
//            its first ge position (g_{m+1} when no earlier stripe has an unswapped ge).
// FAST: a whole stripe without the median slot.  Otherwise (always P2_FULL) lanes past hi are
// masked and the median slot ch carries klo's flags (kge / kle): the owner wave moves the
// median physically only after this pass.
enum { P2_FULL = 0, P2_LEFT = 1, P2_RIGHT = 2 };
// P2's running rank bases: scalar popcounts (s_bcnt1 + s_add on the CU's one scalar unit, then a
// v_mov into mbcnt's base operand), or with KVC_P2_VBASE the VALU (two v_bcnt per row, the base
// a VGPR mbcnt reads directly)
#ifndef KVC_P2_VBASE
#define KVC_P2_VBASE 0
#endif
__device__ __forceinline__ int p2_count(uint64_t m) {
  if constexpr (KVC_P2_VBASE) return vpopc(m);
  else return __popcll(m);
}
// ISINK: the lane sinks start at spos + ssink / gpos + gsink (level 0's tables in the idx region
// sink into the shared tables); otherwise they are the 64 entries before each table
template <typename KeyT, int JM, bool FAST, int MODE = P2_FULL, bool ISINK = false>
__device__ __forceinline__ void p2_window0(const KeyT* key, uint16_t* spos, uint16_t* gpos,
                                           int lane, int pos0, int wbeg, int J, int hi,
                                           uint32_t p, int ch, bool kge, bool kle, int rge1,
                                           int rle, int tot_le, int cap, int& nsw,
                                           int ssink = -64, int gsink = -64) {
  static_assert(FAST || MODE == P2_FULL, "partial stripes take the full pass");
  const int ssl = ISINK ? ssink + lane : lane - 64, gsl = ISINK ? gsink + lane : lane - 64;
  // keys in flight per lane (register budget: 64 VGPRs); 4 and 16 measured the same
  // (profiles/r03_c_p2_keys_in_flight_ab.jsonl)
  constexpr int JB = JM < 8 ? JM : 8;
  const int t1 = tot_le + 1;
  const int cap1 = cap + 1;  // the dump slot (slots 1..cap are the window's ranks)
  const int g1 = rge1;  // P2_RIGHT: rank of the stripe's first ge position
  int ff = kBig;        // P2_RIGHT: the stripe's first ge position (wave-uniform)
  unroll_for<0, JM / JB>([&](auto bc) {
    constexpr int j0 = decltype(bc)::value * JB;
    if (j0 > 0 && j0 >= J) return;
    KeyT kv[JB];
    unroll_for<0, JB>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int pos = pos0 + (j0 + q) * 64;
      kv[q] = key[FAST ? pos : min(pos, hi - 1)];
    });
    unroll_for<0, JB>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int j = j0 + q;
      if (j >= jm_rows_past<JM>() && j >= J) return;
      const int pj = pos0 + j * 64;
      bool ge = (uint32_t)kv[q] >= p, le = (uint32_t)kv[q] <= p;
      if constexpr (!FAST) {
        const bool inb = pj < hi, isch = pj == ch;
        ge = inb && (isch ? kge : ge);
        le = inb && (isch ? kle : le);
      }
      // Scatter slots are plain selects (v_min + v_cndmask): a rank past the window goes to the
      // never-read slot cap + 1, a lane without the flag to its sink.  (Written as
      // `flag && rank <= cap ? rank : sink`, the compiler emitted two exec-mask branches per row
      // of 64 positions -- 7 scalar instructions on the CU's one scalar unit.)
      if constexpr (MODE == P2_LEFT) {
        const uint64_t bg = __builtin_amdgcn_ballot_w64(ge);
        const int a1 = vreg(min(mbcnt(bg, rge1), cap1));
        gpos[ge ? a1 : gsl] = (uint16_t)pj;
        rge1 += p2_count(bg);
      } else if constexpr (MODE == P2_RIGHT) {
        const uint64_t bl = __builtin_amdgcn_ballot_w64(le);
        const int sr = vreg(min(t1 - 1 - mbcnt(bl, rle), cap1));  // s rank of an le position
        spos[le ? sr : ssl] = (uint16_t)pj;
        rle += p2_count(bl);
        if (ff == kBig) {
          const uint64_t bg = __builtin_amdgcn_ballot_w64(ge);
          if (bg) ff = pj - lane + (int)__builtin_ctzll(bg);
        }
      } else {
        const uint64_t bg = __builtin_amdgcn_ballot_w64(ge), bl = __builtin_amdgcn_ballot_w64(le);
        const int a1 = vreg(mbcnt(bg, rge1));                   // g rank: A + 1
        const int sr = vreg(t1 - (mbcnt(bl, rle) + (le ? 1 : 0)));  // s rank: tot_le - Lin + 1
        spos[le ? min(sr, cap1) : ssl] = (uint16_t)pj;
        gpos[ge ? min(a1, cap1) : gsl] = (uint16_t)pj;
        // g_t < s_t  <=>  A + Lin < tot_le  <=>  a1 < sr: swapped (a prefix t <= m of the g's)
        nsw += __popcll(bg & __builtin_amdgcn_ballot_w64(a1 < sr));
        rge1 += p2_count(bg);
        rle += p2_count(bl);
      }
    });
  });
  if constexpr (MODE == P2_RIGHT) {
    if (ff != kBig && g1 <= cap && lane == 0) gpos[g1] = (uint16_t)ff;
  }
}

// The chain's last levels, once the segment [lo, hi) holds at most 64 positions, run by one wave
// with the segment in registers: lane i holds position lo + i (key, index).  A level is the same
// libstdc++ step as partition_level (std::__move_median_to_first + std::__unguarded_partition:
// g_t <-> s_t for the prefix t <= m with g_t < s_t, cut = min(g_{m+1}, s_m)), computed from two
// ballots: the g / s rank -> lane tables are built by forward permutes (ds_permute) and each
// swapped lane fetches its partner's entry by a backward permute -- no LDS memory round trips,
// no rank-table stores.  The final stable insertion sort ranks the segment's lanes against each
// other, and every lane writes its entry back once.  depth == 0 (the introsort / introselect
// depth limit) writes the registers back and takes the serial heap path, as run_chain does.
// Returns with the segment's final arrangement in key / idx (only the first-k SET matters).
template <typename KeyT>
__device__ __forceinline__ void wave_tiny_chain(KeyT* key, uint16_t* idx, int k, bool topk,
                                                int thr, int lo, int hi, int depth,
                                                uint32_t* status) {
  const int lane = threadIdx.x & 63;
  const int m = hi - lo;  // <= 64
  const bool own = lane < m;
  uint32_t kk = own ? (uint32_t)key[lo + lane] : 0xFFFFFFFFu;
  uint32_t ii = own ? (uint32_t)idx[lo + lane] : 0u;
  int slo = 0, shi = m;          // the segment, relative to lo
  const int kr = k - lo;         // k relative to lo
  int dest = lane;               // where this lane's entry is written back
  bool heap = false;
  while (true) {
    if (slo == kr || shi == kr) break;  // a partition boundary sits at k
    if (shi - slo <= thr) {  // final stable insertion sort: rank within [slo, shi)
      const bool in = lane >= slo && lane < shi;
      int r = 0;
      for (int j = slo; j < shi; ++j) {  // uniform trip count
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)kk, j);
        r += (kj < kk || (kj == kk && j < lane)) ? 1 : 0;
      }
      dest = in ? slo + r : lane;
      break;
    }
    if (depth == 0) {  // depth limit: the serial heap algorithms on LDS
      heap = true;
      break;
    }
    --depth;
    // std::__move_median_to_first(slo, slo + 1, mid, shi - 1)
    const int a = slo + 1, b = slo + (shi - slo) / 2, c = shi - 1;
    const uint32_t ka = (uint32_t)__builtin_amdgcn_readlane((int)kk, a);
    const uint32_t kb = (uint32_t)__builtin_amdgcn_readlane((int)kk, b);
    const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)kk, c);
    int ch;
    if (ka < kb) {
      if (kb < kc) ch = b; else if (ka < kc) ch = c; else ch = a;
    } else if (ka < kc) {
      ch = a;
    } else if (kb < kc) {
      ch = c;
    } else {
      ch = b;
    }
    const uint32_t p = ch == a ? ka : ch == b ? kb : kc;
    const uint32_t klo = (uint32_t)__builtin_amdgcn_readlane((int)kk, slo);
    const uint32_t ich = (uint32_t)__builtin_amdgcn_readlane((int)ii, ch);
    const uint32_t ilo = (uint32_t)__builtin_amdgcn_readlane((int)ii, slo);
    kk = lane == slo ? p : lane == ch ? klo : kk;
    ii = lane == slo ? ich : lane == ch ? ilo : ii;
    // std::__unguarded_partition(slo + 1, shi, pivot = slo)
    const bool inr = lane > slo && lane < shi;
    const bool ge = inr && kk >= p, le = inr && kk <= p;
    const uint64_t GE = __builtin_amdgcn_ballot_w64(ge), LE = __builtin_amdgcn_ballot_w64(le);
    const int tot_le = __popcll(LE);
    const int A = mbcnt(GE, 0);                    // ge lanes below
    const int lin = mbcnt(LE, 0) + (le ? 1 : 0);   // le lanes in (slo, lane]
    const bool sg = ge && A + lin < tot_le;        // g_t (t = A + 1) with g_t < s_t: swapped
    const uint64_t SG = __builtin_amdgcn_ballot_w64(sg);
    const int msw = __popcll(SG);
    // the rank -> lane tables below use lane 63 as the sink of lanes with nothing to record:
    // sound because the swapped pairs are disjoint in (slo, shi), so msw <= 31 ranks (lanes
    // 0..30).  Checked (one scalar compare per level), never expected to fire.
    if (msw > 31 && status && lane == 0) atomicOr(status, (uint32_t)KVC_DEV_INTERNAL);
    const int srk = tot_le - lin + 1;              // s rank of an le lane
    const bool ss = le && srk <= msw;              // s_t, t <= m: swapped
    // rank -> lane tables: lane t - 1 of gt / st receives g_t / s_t (others write lane 63,
    // never read: m <= 31)
    const int gt = __builtin_amdgcn_ds_permute((sg ? A : 63) * 4, lane);
    const int st = __builtin_amdgcn_ds_permute((ss ? srk - 1 : 63) * 4, lane);
    const int tab = gt | (st << 8);
    const int t1 = sg ? A : ss ? srk - 1 : 0;      // this lane's rank - 1
    const int pt = __builtin_amdgcn_ds_bpermute(t1 * 4, tab);
    const int partner = sg ? (pt >> 8) : ss ? (pt & 0xFF) : lane;
    if constexpr (sizeof(KeyT) == 2) {
      const uint32_t w = __builtin_amdgcn_ds_bpermute(partner * 4, (int)(kk << 16 | ii));
      kk = w >> 16;
      ii = w & 0xFFFFu;
    } else {
      const uint32_t nk = __builtin_amdgcn_ds_bpermute(partner * 4, (int)kk);
      ii = __builtin_amdgcn_ds_bpermute(partner * 4, (int)ii);
      kk = nk;
    }
    // cut = min(g_{m+1}, s_m): the first unswapped ge lane, the lowest swapped le lane
    const uint64_t GN = GE & ~SG;
    const int gnext = GN ? (int)__builtin_ctzll(GN) : kBig;
    const uint64_t SS = __builtin_amdgcn_ballot_w64(ss);
    const int cut = min(gnext, SS ? (int)__builtin_ctzll(SS) : kBig);
    const bool right = topk ? cut <= kr - 1 : kr > cut;
    slo = right ? cut : slo;
    shi = right ? shi : cut;
  }
  if (own) {
    key[lo + dest] = (KeyT)kk;
    idx[lo + dest] = (uint16_t)ii;
  }
  if (heap) {
    wave_sync();
    if (lane == 0) {
      if (topk) {
        heap_select(key + lo + slo, idx + lo + slo, kr - slo, shi - slo);
        kv_swap(key, idx, lo + slo, k - 1);
      } else {
        make_heap(key + lo + slo, idx + lo + slo, shi - slo);
        sort_heap(key + lo + slo, idx + lo + slo, shi - slo);
      }
    }
  }
  wave_sync();
}

// One partition level over [lo, hi) with at most JM positions per lane (compile-time bound; the
// passes stop at the segment's own J with a scalar branch).  Returns cut.  See run_chain for
// the algorithm.  P1 and P2 are issue-bound at the long levels (16 waves of 16 rows of 64
// positions), so per-position work is a handful of VALU ops: flags are compare ballots
// (recomputed from the keys in P2 rather than carried), wave counts are scalar popcounts, and
// wave-uniform work -- median of 3, cross-wave prefix sums, swap count, g_{m+1} -- runs on SGPRs.
//
// ITAB (level 0 of a 1 024-thread row, lo = 0, indices still the identity; ihalf = n_cap / 2):
// the rank tables are the two halves of the idx region, whose n_cap / 2 - 1 ranks cover every m
// the level can reach (m <= (hi - lo - 1) / 2): one window.  The median move and P4 then swap keys
// only; after every table read (a barrier) the indices are rebuilt: the identity with the
// median's transposition (lo <-> ch), then (another barrier) each swapped pair's entries from
// the pair kept in registers -- the same arrangement as physical index swaps, without P4's
// index loads and without the second window (and its flag pass).
template <typename KeyT, int NT, int JM, bool ITAB = false>
__device__ __forceinline__ int partition_level(KeyT* key, uint16_t* idx, uint16_t* spos,
                                               uint16_t* gpos, SelScalars<KeyT>& sc, int lo,
                                               int hi, int cap, uint64_t* acc,
                                               bool use_tc = false, uint32_t tcv = 0,
                                               bool desc = false, int ihalf = 0) {
  static_assert(!ITAB || (NT > 64 && sizeof(KeyT) == 2), "ITAB: level 0 of 16-bit block rows");
  constexpr int NW = NT / 64;
  typedef typename std::conditional<(JM > 32), uint64_t, uint32_t>::type MaskT;
  const int lane = threadIdx.x & 63;
  const int wid = (NT == 64) ? 0 : uni((int)(threadIdx.x >> 6));
  const int tid = wid * 64 + lane;
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  KVC_TICK(t0);
  const int J = (hi - lo - 1 + NT - 1) / NT;  // <= JM
  const int wbeg = lo + 1 + wid * J * 64;
  const int pos0 = wbeg + lane;
  // ---- median of 3 (std::__move_median_to_first), on the scalar unit; the swap into lo is
  // virtual until the owner wave of position ch has read its P2 keys ----
  const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
  const uint32_t ka = (uint32_t)uni((int)key[a]), kb = (uint32_t)uni((int)key[b]);
  const uint32_t kc = (uint32_t)uni((int)key[c]), klo = (uint32_t)uni((int)key[lo]);
  int ch;
  if (ka < kb) {
    if (kb < kc) ch = b; else if (ka < kc) ch = c; else ch = a;
  } else if (ka < kc) {
    ch = a;
  } else if (kb < kc) {
    ch = c;
  } else {
    ch = b;
  }
  const uint32_t p = (ch == a) ? ka : (ch == b) ? kb : kc;
  const bool kge = klo >= p, kle = klo <= p;  // flags of the key that moves into slot ch
  const int nval = hi - wbeg;                 // positions of this wave's stripe below hi
  const bool whole = nval >= J * 64;
  const bool owner = ch >= wbeg && ch < wbeg + J * 64;
  uint64_t ta = 0, tb = 0, tc = 0;  // diagnostic build: P1 sub-phases of a J = 16 level
  KVC_TICK(ta);
  // ---- P1: wave ge / le counts ----
  int cge = 0, cle = 0;
  if (use_tc) {
    // level 0 of a plain-norm row (lo = 0, hi = n): SCORE counted every 64-token tile against
    // this pivot (score_tile).  This stripe [wbeg, wbeg + 64 J), wbeg = 1 + 64 T0, is tiles
    // T0 .. T0 + J - 1 without position 64 T0 (the previous stripe's last, or the pivot slot lo)
    // and with position 64 (T0 + J) (its own last, in the next tile).  Same counts as the pass
    // below, including slot ch counted with the pivot's key (corrected for the median move).
    // tcv: lane l < J holds tile T0 + l's counts (loaded at the start of select_body, its
    // latency under the key load)
    const int T0 = wid * J;
    const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane(row_scan16((int)tcv), 15);
    uint32_t g = sum & 0xFFFFu, l = sum >> 16;
    if (desc) {  // descending keys are complemented: ge <-> le of the ascending counts
      const uint32_t t = g;
      g = l;
      l = t;
    }
    const int x0 = T0 * kTile, x1 = (T0 + J) * kTile;
    if (x0 < hi) {
      const uint32_t k0 = (uint32_t)uni((int)key[x0]);
      g -= k0 >= p ? 1u : 0u;
      l -= k0 <= p ? 1u : 0u;
    }
    if (x1 < hi) {
      const uint32_t k1 = (uint32_t)uni((int)key[x1]);
      g += k1 >= p ? 1u : 0u;
      l += k1 <= p ? 1u : 0u;
    }
    cge = (int)g;
    cle = (int)l;
  } else if (whole)
    p1_counts<KeyT, JM, true>(key, pos0, J, hi, p, cge, cle);
  else if (nval > 0)
    p1_counts<KeyT, JM, false>(key, pos0, J, hi, p, cge, cle);
  if (owner) {  // slot ch was counted with the pivot's flags (both set); it holds klo
    cge -= kge ? 0 : 1;
    cle -= kle ? 0 : 1;
  }
  KVC_TICK(tb);
  int ge_before = 0, le_before = 0, tot_le = cle, tot_ge = cge;
  if constexpr (NW > 1) {
    static_assert(NW <= 16, "cross-wave scans use one 16-lane DPP row");
    if (lane == 0)  // sums < 2^16 (positions < 65536): packed
      sc.wa[wid] = (int)((uint32_t)cge | ((uint32_t)cle << 16));
    KVC_TICK(tc);
#ifdef KVC_STAMPS
    if (lane == 0) {  // diagnostic: this wave's level start and P1 end (low 32 bits)
      sc.wb[wid] = (int)(uint32_t)t0;
      sc.fnan[wid] = (int)(uint32_t)tc;
    }
#endif
    __syncthreads();  // B_a
    const int scan = row_scan16(lane < NW ? sc.wa[lane] : 0);
    // unpack unsigned: the le half reaches bit 31 for segments longer than 32767 positions
    const uint32_t before = wid ? (uint32_t)__builtin_amdgcn_readlane(scan, wid - 1) : 0u;
    ge_before = (int)(before & 0xFFFFu);
    le_before = (int)(before >> 16);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(scan, NW - 1);
    tot_le = (int)(tot >> 16);
    tot_ge = (int)(tot & 0xFFFFu);
  }
  // ITAB: the level's tables in the idx region, sinks in the shared tables
  uint16_t* const shs = spos;
  bool it = false;
  int ssink = -64, gsink = -64;
  if constexpr (ITAB) {
    it = true;
    {
      ssink = (int)(spos - idx);
      gsink = (int)(gpos - (idx + ihalf));
      spos = idx;
      gpos = idx + ihalf;
      cap = ihalf - 1;
    }
  }
  KVC_TICK(t1);
  // ---- P2, rank window 0: s / g rank tables, swap count m, g_{m+1} (stores only) ----
  int nsw = 0;
  if (whole && !owner) {
    if (ge_before + cge + le_before + cle <= tot_le) {  // every ge swapped, no le
      p2_window0<KeyT, JM, true, P2_LEFT, ITAB>(key, spos, gpos, lane, pos0, wbeg, J, hi, p, ch,
                                                kge, kle, ge_before + 1, le_before, tot_le, cap,
                                                nsw, ssink, gsink);
      nsw = cge;
    } else if (ge_before + le_before >= tot_le) {  // no ge swapped, every le
      p2_window0<KeyT, JM, true, P2_RIGHT, ITAB>(key, spos, gpos, lane, pos0, wbeg, J, hi, p, ch,
                                                 kge, kle, ge_before + 1, le_before, tot_le, cap,
                                                 nsw, ssink, gsink);
    } else {
      p2_window0<KeyT, JM, true, P2_FULL, ITAB>(key, spos, gpos, lane, pos0, wbeg, J, hi, p, ch,
                                                kge, kle, ge_before + 1, le_before, tot_le, cap,
                                                nsw, ssink, gsink);
    }
  } else if (nval > 0)
    p2_window0<KeyT, JM, false, P2_FULL, ITAB>(key, spos, gpos, lane, pos0, wbeg, J, hi, p, ch,
                                               kge, kle,
                                ge_before + 1, le_before, tot_le, cap, nsw, ssink, gsink);
  // the median move, made physical by the only wave that reads slot ch (after its P2 loads)
  if (owner && lane == 0) {
    if (ITAB && it) {  // keys only: the idx region holds the tables
      const KeyT t = key[lo];
      key[lo] = key[ch];
      key[ch] = t;
    } else {
      kv_swap(key, idx, lo, ch);
    }
  }
  int msw;
#ifdef KVC_STAMPS
  uint64_t tp2 = 0;
  KVC_TICK(tp2);
  uint32_t wstart[NW > 1 ? NW : 1], wp1[NW > 1 ? NW : 1];
  if constexpr (NW > 1) {
    if (acc && tid == 0 && JM == 16 && J == 16)
      for (int w = 0; w < NW; ++w) {
        wstart[w] = (uint32_t)sc.wb[w];
        wp1[w] = (uint32_t)sc.fnan[w];
      }
    __syncthreads();  // diagnostic: the P1 stamps are read before P2 stamps overwrite them
    if (lane == 0) sc.fnan[wid] = (int)(uint32_t)tp2;
  }
#endif
  if constexpr (NW > 1) {
    if (lane == 0) sc.wm[wid] = nsw;
    __syncthreads();  // B_b
    msw = __builtin_amdgcn_readlane(row_scan16(lane < NW ? sc.wm[lane] : 0), NW - 1);
  } else {
    wave_sync();
    msw = nsw;
  }
  // g_{m+1}, the first unswapped ge position (none when every ge position is swapped)
  int gnext = msw >= tot_ge ? kBig : msw < cap ? uni((int)gpos[msw + 1]) : kBig;
  KVC_TICK(t2);
  // ---- m >= cap (rare): the level's flags, from the keys before any swap (the median slot is
  // physical now), kept in registers for the later windows' scatters (the swapped pairs are
  // disjoint, so earlier windows' swaps do not change them), and g_{m+1} from a flag pass ----
  MaskT gem = 0, lem = 0;
  if (msw >= cap) {
    for (int j = 0; j < J; ++j) {
      const int pos = pos0 + j * 64;
      const bool inb = pos < hi;
      const uint32_t kk = (uint32_t)key[min(pos, hi - 1)];
      gem |= (inb && kk >= p) ? ((MaskT)1 << j) : (MaskT)0;
      lem |= (inb && kk <= p) ? ((MaskT)1 << j) : (MaskT)0;
    }
    int rge = ge_before, rle = le_before, ff = kBig;
    for (int j = 0; j < J && ff == kBig; ++j) {
      const bool ge = (gem >> j) & 1, le = (lem >> j) & 1;
      const uint64_t bg = __builtin_amdgcn_ballot_w64(ge), bl = __builtin_amdgcn_ballot_w64(le);
      const bool cond = mbcnt(bg, rge) + mbcnt(bl, rle) + (le ? 1 : 0) < tot_le;
      const uint64_t bf = bg & ~__builtin_amdgcn_ballot_w64(cond);
      if (bf) ff = wbeg + j * 64 + (int)__builtin_ctzll(bf);
      rge += __popcll(bg);
      rle += __popcll(bl);
    }
    if constexpr (NW > 1) {
      if (lane == 0) sc.wb[wid] = ff == kBig ? 0xFFFF : ff;  // ff < 65535
      __syncthreads();  // every wave has its flags before the first swap
      const uint32_t x = lane < NW ? (uint32_t)sc.wb[lane] : 0xFFFFu;
      // waves in position order: the first one with an unswapped ge position wins
      const uint64_t fb = __builtin_amdgcn_ballot_w64(x != 0xFFFFu);
      gnext = fb ? __builtin_amdgcn_readlane((int)x, (int)__builtin_ctzll(fb)) : kBig;
    } else {
      wave_sync();
      gnext = ff;
    }
  }
  if (ITAB && it) {
    // ---- P4, one window: the m pairs, ranks t = 1 + tid + q NT (q < JM / 2: m <= NT J / 2),
    // kept packed (g | s << 16) for the index rebuild; keys swapped now ----
    constexpr int QM = JM / 2 > 0 ? JM / 2 : 1;
    // q-rows with a rank for this wave (uniform): the rest keep pr = 0 and touch nothing
    const int nq = msw >= 1 + wid * 64 ? uni(min(QM, (msw - 1 - wid * 64) / NT + 1)) : 0;
    uint32_t pr[QM];
    KeyT kg[QM], ks[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) pr[q] = 0u;
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q >= nq) break;
      const int t = 1 + tid + q * NT;
      const bool v = t <= msw;
      const int ti = v ? t : 0;
      const int g = gpos[ti], sv = spos[ti];
      pr[q] = v ? ((uint32_t)g | (uint32_t)sv << 16) : 0u;  // lo = 0: a self swap of slot 0
    }
    // the cut's s_m, read before the tables are overwritten
    const int sm = msw > 0 ? uni((int)spos[msw]) : kBig;
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q >= nq) break;
      kg[q] = key[pr[q] & 0xFFFFu];
      ks[q] = key[pr[q] >> 16];
    }
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q >= nq) break;
      key[pr[q] & 0xFFFFu] = ks[q];
      key[pr[q] >> 16] = kg[q];
    }
    __syncthreads();  // every table entry is read
    // identity indices with the median's transposition lo <-> ch: 16-B stores, then the two
    // entries by the thread that stored them (same-thread LDS order)
    for (int v = tid; v < (hi + 7) / 8; v += NT) {
      const uint32_t b = (uint32_t)v * 8;
      reinterpret_cast<uint4*>(idx)[v] =
          make_uint4(b | (b + 1) << 16, (b + 2) | (b + 3) << 16, (b + 4) | (b + 5) << 16,
                     (b + 6) | (b + 7) << 16);
      if (v == (lo >> 3)) idx[lo] = (uint16_t)ch;
      if (v == (ch >> 3)) idx[ch] = (uint16_t)lo;
    }
    __syncthreads();
    // the swapped pairs' entries: idx[g] = old idx[s], idx[s] = old idx[g] (old = identity with
    // lo <-> ch; lo is never swapped).  Lanes without a pair write the shared tables' sinks.
    uint16_t* sink = shs + lane;
#pragma unroll
    for (int q = 0; q < QM; ++q) {
      if (q >= nq) break;
      const int g = (int)(pr[q] & 0xFFFFu), sv = (int)(pr[q] >> 16);
      const bool v = pr[q] != 0u;
      (v ? idx + g : sink)[0] = (uint16_t)(sv == ch ? lo : sv);
      (v ? idx + sv : sink)[0] = (uint16_t)(g == ch ? lo : g);
    }
    __syncthreads();  // B_c
    KVC_TICK(t3);
#ifdef KVC_STAMPS
    if (acc && tid == 0) {
      acc[0] += t1 - t0;
      acc[1] += t2 - t1;
      acc[2] += t3 - t2;
      acc[3] += 1;
      acc[4] += (uint64_t)msw;
      acc[25] = (t1 - t0) | ((t2 - t1) << 20) | ((t3 - t2) << 40);
    }
#endif
    return min(gnext, sm);
  }
  int wb = 0;
  while (true) {
    // ---- P4: this window's swaps (disjoint pairs g_t <-> s_t), spread evenly over the NT
    // lanes: rank-table loads, then key/idx loads, then stores ----
    // Lanes past the window's last rank swap the pivot slot lo with itself (lo is never a
    // swapped g_t or s_t: every g_t > lo, and a swapped s_t > g_t), so the loads and stores need
    // no exec-mask branches; q-rows with no rank left for the wave are skipped uniformly.
    const int wend = min(msw, wb + cap);
    for (int base = wb + 1; base <= wend; base += NT * 4) {
      if (base + wid * 64 > wend) break;  // no rank left for this wave
      const int nq = uni(min(4, (wend - base - wid * 64) / NT + 1));  // q-rows with a rank
      int gp[4], sp[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nq) break;
        const int t = base + tid + q * NT;
        const bool v = t <= wend;
        const int ti = v ? t - wb : 0;
        const int g = gpos[ti], sv = spos[ti];
        gp[q] = v ? g : lo;
        sp[q] = v ? sv : lo;
      }
      KeyT kg[4], ks[4];
      uint16_t ig[4], is[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nq) break;
        kg[q] = key[gp[q]];
        ks[q] = key[sp[q]];
        ig[q] = idx[gp[q]];
        is[q] = idx[sp[q]];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nq) break;
        key[gp[q]] = ks[q];
        key[sp[q]] = kg[q];
        idx[gp[q]] = is[q];
        idx[sp[q]] = ig[q];
      }
    }
    if (wend >= msw) break;
    group_sync<NT>();  // the next window overwrites the tables
    wb += cap;
    // ---- scatter of window wb from the flags (ranks (wb, wb + cap]) ----
    int rge = ge_before, rle = le_before;
    for (int j = 0; j < J; ++j) {
      const bool ge = (gem >> j) & 1, le = (lem >> j) & 1;
      const uint64_t bg = __builtin_amdgcn_ballot_w64(ge), bl = __builtin_amdgcn_ballot_w64(le);
      const int A = mbcnt(bg, rge);                   // ge positions before this one
      const int lin = mbcnt(bl, rle) + (le ? 1 : 0);  // le positions in [lo+1, pos]
      const bool cond = A + lin < tot_le;
      const uint16_t pj = (uint16_t)(pos0 + j * 64);
      const int sr = tot_le - lin + 1 - wb;  // s rank within the window
      spos[(le && sr >= 1 && sr <= cap) ? sr : lane - 64] = pj;
      const int gr = A + 1 - wb;             // swapped (cond): g rank A + 1 <= m
      gpos[(ge && cond && gr >= 1 && gr <= cap) ? gr : lane - 64] = pj;
      rge += __popcll(bg);
      rle += __popcll(bl);
    }
    group_sync<NT>();
  }
  group_sync<NT>();  // B_c
  KVC_TICK(t3);
#ifdef KVC_STAMPS
  if (acc && tid == 0) {
    acc[0] += t1 - t0;
    acc[1] += t2 - t1;
    acc[2] += t3 - t2;
    acc[3] += 1;
    acc[4] += (uint64_t)msw;
    if (NT > 64) acc[25] = (t1 - t0) | ((t2 - t1) << 20) | ((t3 - t2) << 40);  // level split
#ifdef KVC_SNAP_STAMPS
    if (false) {  // slots 26..29 hold the snapkv scoring stamps (tools/select_stamps.py with SEL_SNAP_STAMPS)
#else
    if (NT > 64 && JM == 16 && J == 16) {  // level 0 of a 16 384-position row (slots 26..29):
#endif
      // wave start skew, longest wave P1 (start -> counts written), last P1 end after the first
      // start, last P2 end after B_a (wave 0's t1)
      uint32_t s0 = wstart[0], s1 = wstart[0], p1m = 0, e1 = 0, e2 = 0;
      for (int w = 0; w < NW; ++w) {
        s0 = min(s0, wstart[w]);
        s1 = max(s1, wstart[w]);
      }
      for (int w = 0; w < NW; ++w) {
        p1m = max(p1m, wp1[w] - wstart[w]);
        e1 = max(e1, wp1[w] - s0);
        e2 = max(e2, (uint32_t)sc.fnan[w] - (uint32_t)t1);
      }
      acc[21] = s1 - s0;
      acc[22] = p1m;
      acc[23] = e1;
      acc[24] = e2;
    }
  }
#endif
  return min(gnext, msw > 0 ? uni((int)spos[msw - wb]) : kBig);
}

// The partition chain of libstdc++ introsort (topk = false) / introselect (topk = true),
// following only the segment [lo, hi) that straddles position k, run by NT cooperating lanes
// (the whole 1024-thread block, or one wave once the segment is short).  One level is
// std::__move_median_to_first + std::__unguarded_partition(lo+1, hi, pivot=lo) computed in
// parallel:
//   g_t = t-th position (ascending) in [lo+1,hi) with !(key < p)            ("ge")
//   s_t = t-th position (descending) with !(p < key), then the pivot slot lo ("le")
// libstdc++ swaps g_t <-> s_t for every t with g_t < s_t -- a prefix t <= m -- and returns
// cut = min(g_{m+1}, s_m).  With A(x) = #ge before x and Lin(x) = #le in [lo+1, x]:
//   g_t < s_t  <=>  A(g_t) + Lin(g_t) < tot_le
// so m is counted in the same pass that scatters the s rank -> position table (spos).
// Positions are laid out j-major (lane + 64*j within a wave's stripe) so flags are wave ballots;
// each level runs a body specialised on its positions-per-lane bound (1..16, or 64 for the
// global-memory variant of zones longer than kZoneMax).
// Returns 0 when the first-k set is final, 1 when the block hands a short segment to one wave.
template <typename KeyT, int NT, int MAXJ, bool L0T = true>
__device__ __forceinline__ int run_chain(KeyT* key, uint16_t* idx, uint16_t* spos, uint16_t* gpos,
                         SelScalars<KeyT>& sc, int k, bool topk, int thr, int cap, int& lo,
                         int& hi, int& depth, int& level, int wave_seg,
                         uint64_t* acc = nullptr, uint32_t* status = nullptr,
                         bool l0use = false, uint32_t l0tc = 0, bool desc = false,
                         int ihalf = 0, bool l0plain = false) {
  const int tid = (NT == 64) ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  while (true) {
    if (lo == k || hi == k) return 0;  // a partition boundary sits at k: the set is final
    if constexpr (NT == 64 && kTinyChain) {
      if (hi - lo <= 64 && hi - lo > thr) {  // the last levels from registers
        wave_tiny_chain(key, idx, k, topk, thr, lo, hi, depth, status);
        return 0;
      }
    }
    if (hi - lo <= thr) {              // final (stable) insertion sort of the segment
      if (tid < 64) wave_stable_sort(key, idx, lo, hi);
      group_sync<NT>();
      return 0;
    }
    if (NT > 64 && hi - lo <= wave_seg) return 1;
    if (depth == 0) {  // depth limit: libstdc++ switches to heap algorithms
      if (tid == 0) {
        if (topk) {
          heap_select(key + lo, idx + lo, k - lo, hi - lo);
          kv_swap(key, idx, lo, k - 1);
        } else {
          make_heap(key + lo, idx + lo, hi - lo);
          sort_heap(key + lo, idx + lo, hi - lo);
        }
      }
      group_sync<NT>();
      return 0;
    }
    --depth;
    const int J = (hi - lo - 1 + NT - 1) / NT;
    // SCORE's level-0 tile counts (plain-norm rows; the first level covers the whole zone)
    const bool tc = l0use && level == 0 && lo == 0;
    int cut;
#ifdef KVC_STAMPS
    const uint64_t tl0 = __builtin_amdgcn_s_memtime();
#endif
    // level 0 of a plain-norm row keeps its rank tables in the idx region (ihalf = n_cap / 2:
    // n_cap / 2 - 1 ranks per table) when the shared tables could need a second window
    // (partition_level).  Only those rows: their level-0 swap counts sit around the shared cap
    // (m median 3 667 of cap 3 840 at the headline: 44 % of rows took a second window), while
    // the extra barriers and index rebuild measured slower on snapkv rows
    // (profiles/r06_f_itab_ab.jsonl)
    const bool itab = L0T && kL0Itab && NT == kSelThreads && sizeof(KeyT) == 2 && ihalf > 0 &&
                      (l0plain || kL0ItabAll) && level == 0 && lo == 0 && J > 4 &&
                      (hi - 1) / 2 > cap && hi <= 2 * ihalf;
    if constexpr (L0T && kL0Itab && NT == kSelThreads && sizeof(KeyT) == 2) {
      if (KVC_ITAB_COLD ? __builtin_expect(itab, 0) : itab) {
        if (J <= 8)
          cut = partition_level<KeyT, NT, 8, true>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                                   l0tc, desc, ihalf);
        else
          cut = partition_level<KeyT, NT, 16, true>(key, idx, spos, gpos, sc, lo, hi, cap, acc,
                                                    tc, l0tc, desc, ihalf);
      }
    }
    if (itab) {
    } else if (J <= 1 && kLevelJmMin <= 1)
      cut = partition_level<KeyT, NT, 1>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                         l0tc, desc);
    else if (J <= 2 && kLevelJmMin <= 2)
      cut = partition_level<KeyT, NT, 2>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                         l0tc, desc);
    else if (J <= 4 && kLevelJmMin <= 4)
      cut = partition_level<KeyT, NT, 4>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                         l0tc, desc);
    else if (J <= 8 && kLevelJmMin <= 8)
      cut = partition_level<KeyT, NT, 8>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                         l0tc, desc);
    else if (MAXJ <= 16 || J <= 16)
      cut = partition_level<KeyT, NT, 16>(key, idx, spos, gpos, sc, lo, hi, cap, acc, tc,
                                          l0tc, desc);
    else if (J <= 32)
      cut = partition_level<KeyT, NT, (MAXJ < 32 ? 16 : 32)>(key, idx, spos, gpos, sc, lo, hi, cap,
                                                               acc, tc, l0tc, desc);
    else
      cut = partition_level<KeyT, NT, (MAXJ < 64 ? 16 : 64)>(key, idx, spos, gpos, sc, lo, hi, cap,
                                                               acc, tc, l0tc, desc);
#ifdef KVC_STAMPS
    // per block level (first 8): cycles, and segment length  (slots 16.. of the row)
    if (acc && NT > 64 && tid == 0 && level < 5) {
      acc[11 + 2 * level] = __builtin_amdgcn_s_memtime() - tl0;
      acc[12 + 2 * level] = acc[25];  // P1 | P2 << 20 | P4 << 40 of this level
    }
#endif
    cut = uni(cut);  // uniform by construction; stated, so that lo / hi stay in SGPRs
    // std::__introselect: if (cut <= nth) first = cut; else last = cut;
    // std::__introsort_loop: recurse right, loop on the left part (k <= cut: keep the left).
    // Value selects, not branches: a store through a selected pointer to lo / hi would put
    // them in scratch memory.
    const bool right = topk ? cut <= k - 1 : k > cut;
    lo = right ? cut : lo;
    hi = right ? hi : cut;
    ++level;
  }
}

// Exclusive prefix sum of one int per thread over the NT threads of the block (wave scans as
// four 16-lane DPP row scans, wave totals through `buf`); one barrier.
template <int NT>
__device__ __forceinline__ int block_exclusive_scan(int v, int* buf, int lane, int wid) {
  static_assert(NT / 64 <= 16, "one 16-lane DPP row holds the wave totals");
  const int rs = row_scan16(v);  // inclusive within each 16-lane row
  const int r0 = __builtin_amdgcn_readlane(rs, 15), r1 = __builtin_amdgcn_readlane(rs, 31);
  const int r2 = __builtin_amdgcn_readlane(rs, 47), r3 = __builtin_amdgcn_readlane(rs, 63);
  const int row = lane >> 4;
  const int excl = rs - v + (row > 0 ? r0 : 0) + (row > 1 ? r1 : 0) + (row > 2 ? r2 : 0);
  if constexpr (NT == 64) {
    return excl;
  } else {
    if (lane == 0) buf[wid] = r0 + r1 + r2 + r3;
    __syncthreads();
    const int ws = row_scan16(lane < NT / 64 ? buf[lane] : 0);
    const int w = uni(wid);
    return excl + (w ? __builtin_amdgcn_readlane(ws, w - 1) : 0);
  }
}


// Atomic += 1 on an int in LDS (`p` a generic pointer into the workgroup's LDS: its low 32
// bits are the LDS address).  A ds_add_u32 without return; callers wait (lgkmcnt) before the
// barrier that publishes the sums.  (The compiler's own lowering of an atomic through such a
// pointer emits an address-space test gfx950's VALU compare cannot encode.)
__device__ __forceinline__ void lds_add1(int* p) {
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1) : "memory");
}

// Block-wide sum of one int per wave (waves of NT threads).  Callers alternate two buffers, so
// consecutive calls need one barrier each (a wave can only rewrite a buffer after every wave has
// passed the barrier of the call in between, i.e. finished reading it).
template <int NT>
__device__ __forceinline__ int block_sum_waves(int v, int* buf, int lane, int wid) {
  static_assert(NT / 64 <= 16, "one 16-lane DPP row holds the wave sums");
  if (lane == 0) buf[wid] = v;
  __syncthreads();
  const int s = row_scan16(lane < NT / 64 ? buf[lane] : 0);  // lanes 0..NW-1 = waves
  return __builtin_amdgcn_readlane(s, NT / 64 - 1);
}

// No-straddling-tie fast path (32-bit keys): the k-th smallest key T by bisection over the key
// values (the row's keys held in registers, one ballot count per step), with c_le = #keys <= T.
// If c_le == k, every key <= T is kept and every other key is not, whatever order libstdc++'s
// sort / nth_element / partial_sort would leave tied elements in -- the first-k SET is fixed by
// the values alone.  fp32 norms essentially never tie at the boundary, so
// this replaces the partition chain for them; bf16 / fp16 rows (tied in nearly every head) skip
// it.  Returns true (and emits) when it applies.
// With `radix`, `hist` (512 ints of LDS scratch: the rank tables, unused before the chain) T is found by
// a radix select over the offsets key - min instead: 8-bit digits from the top, one 256-bin LDS
// histogram of the keys still in the k-th key's bucket per digit (two buffers, each zeroed a pass
// ahead), wave 0 locating the bucket -- two barriers per 8 bits instead of one per bit.
template <int NT, int JM, typename KeyT, bool TO_LDS>
__device__ __forceinline__ bool select_fast_untied(const KeyT* key, int n, int k, SelScalars<KeyT>& sc,
                                   int32_t* out, uint16_t* sel, int* hist, bool radix) {
  const int tid = threadIdx.x, lane = tid & 63, wid = (NT == 64) ? 0 : uni(tid >> 6);
  const int J = (n + NT - 1) / NT;
  if (J > JM) return false;
  const int wbeg = wid * J * 64;
  // the row's keys in registers (every loop below is fully unrolled and predicated on j < J:
  // a runtime trip count would turn kv[] into indexed register accesses)
  uint32_t kv[JM];
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool v = j < J && pos < n;
    kv[j] = v ? (uint32_t)key[min(pos, n - 1)] : 0xFFFFFFFFu;
    mn = v ? min(mn, kv[j]) : mn;
    mx = v ? max(mx, kv[j]) : mx;
  }
  // block min / max of the keys: the bisection range
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  }
  if (lane == 0) {
    sc.wa[wid] = (int)mn;
    sc.wb[wid] = (int)mx;
  }
  __syncthreads();
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    lo = min(lo, (uint32_t)sc.wa[w]);
    hi = max(hi, (uint32_t)sc.wb[w]);
  }
  lo = (uint32_t)uni((int)lo);
  hi = (uint32_t)uni((int)hi);
  __syncthreads();  // sc.wa / sc.wb are the count buffers below
  int c_le = n, parity = 0;
  if (radix) {
    const uint32_t span = hi - lo;
    int rem = span ? 32 - __builtin_clz(span) : 0;  // offset bits still undecided
    uint32_t prefix = 0;  // the decided high bits of the k-th key's offset
    int below = 0;        // #keys whose offset lies below the bucket `prefix`
    for (int i = tid; i < 512; i += NT) hist[i] = 0;
    __syncthreads();
    while (rem > 0) {
      const int w = min(8, rem), sh = rem - w;
      int* h = hist + 256 * parity;
#pragma unroll
      for (int j = 0; j < JM; ++j) {
        const int pos = wbeg + j * 64 + lane;
        const uint32_t d = kv[j] - lo;
        if (j < J && pos < n && (uint32_t)((uint64_t)d >> rem) == prefix)
          lds_add1(h + ((d >> sh) & ((1u << w) - 1u)));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the other buffer's last reader (wave 0, previous pass) finished before the last barrier
      for (int i = tid; i < 256; i += NT) hist[256 * (parity ^ 1) + i] = 0;
      __syncthreads();
      if (wid == 0) {
        const int c0 = h[4 * lane], c1 = h[4 * lane + 1], c2 = h[4 * lane + 2],
                  c3 = h[4 * lane + 3];
        const int s4 = c0 + c1 + c2 + c3;
        const int ex = block_exclusive_scan<64>(s4, nullptr, lane, 0);
        const int need = k - below;  // >= 1: the k-th key lies in this bucket
        const uint64_t b = __builtin_amdgcn_ballot_w64(ex + s4 >= need);
        if (lane == (b ? __builtin_ctzll(b) : 63)) {
          int c = ex, bin = 4 * lane, cnt = c0;
          if (c + c0 < need) {
            c += c0; ++bin; cnt = c1;
            if (c + c1 < need) {
              c += c1; ++bin; cnt = c2;
              if (c + c2 < need) { c += c2; ++bin; cnt = c3; }
            }
          }
          // published in slots the emission below never writes (it writes sc.wm[wid] while a
          // lagging wave may still read this pass's values)
          sc.wa[0] = bin;
          sc.wb[0] = below + c;
          sc.fnan[0] = cnt;
        }
      }
      __syncthreads();
      prefix = (prefix << w) | (uint32_t)sc.wa[0];
      below = sc.wb[0];
      c_le = below + sc.fnan[0];
      rem = sh;
      parity ^= 1;
    }
    lo = lo + prefix;
  }
  // smallest v with #(key <= v) >= k; invariant c_le = #(key <= hi) (= n at hi = max key)
  while (!radix && lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int cl = 0;  // per-lane count (VALU), one wave reduction per step
#pragma unroll
    for (int j = 0; j < JM; ++j) cl += (kv[j] <= mid) ? 1 : 0;  // invalid slots hold ~0u
    const int rs = row_scan16(cl);
    const int c = __builtin_amdgcn_readlane(rs, 15) + __builtin_amdgcn_readlane(rs, 31) +
                  __builtin_amdgcn_readlane(rs, 47) + __builtin_amdgcn_readlane(rs, 63);
    const int tot = block_sum_waves<NT>(c, parity ? sc.wb : sc.wa, lane, wid);
    parity ^= 1;
    if (tot >= k) {
      hi = mid;
      c_le = tot;
    } else {
      lo = mid + 1;
    }
  }
  if (c_le != k) {
    __syncthreads();  // the chain reuses sc
    return false;
  }
  // ---- emit {pos : key[pos] <= T} ascending ----
  const uint32_t T = lo;
  uint32_t fm = 0;  // kept flags by j
  int c = 0;
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool f = j < J && pos < n && kv[j] <= T;
    fm |= f ? (1u << j) : 0u;
    c += __popcll(__builtin_amdgcn_ballot_w64(f));
  }
  if (lane == 0) sc.wm[wid] = c;
  __syncthreads();
  int run = 0;
  for (int w = 0; w < wid; ++w) run += sc.wm[w];
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool f = (fm >> j) & 1u;
    const uint64_t bf = __builtin_amdgcn_ballot_w64(f);
    if (f) {
      const int r = run + __popcll(bf & lanemask_lt(lane));
      if constexpr (TO_LDS) sel[r] = (uint16_t)pos;
      else out[r] = pos;
    }
    run += __popcll(bf);
  }
  return true;
}

// KVC_ALGO_STABLE (opt-in, not the reference's tie order): the first k of a STABLE sort of the
// row's keys -- every key below T, the k-th smallest key, then the first k - #(key < T) keys
// equal to T in position order.  T by a radix select (8-bit digits of key - min from the top, a
// 256-bin LDS histogram per digit in `hist`, 512 ints: one digit for a bf16 norm row, whose keys
// span < 256 codes) or, for rows whose scratch is shorter, by bisection over the key range; then
// one flag pass and the ascending emission (output slot of a kept position = #(key < T before
// it) + min(#(key == T before it), need)).  Lane positions wid*J*64 + j*64 + lane, j < J <= JM:
// every pass re-reads the keys from LDS with its JM loads issued back to back (nothing but two
// flag words held across barriers).  `sel` must not alias the keys.
template <int NT, int JM, typename KeyT, bool TO_LDS>
__device__ __forceinline__ void stable_select(const KeyT* key, int n, int k, SelScalars<KeyT>& sc,
                                              int32_t* out, uint16_t* sel, int* hist, bool radix,
                                              uint64_t* stamps = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wid = (NT == 64) ? 0 : uni(tid >> 6);
  const int J = (n + NT - 1) / NT;
  const int base = wid * J * 64 + lane;
  const int jv = base < n ? min(J, (n - base + 63) >> 6) : 0;  // this lane's valid j
  constexpr int CH = JM < 16 ? JM : 16;  // loads issued together per pass step
  uint32_t mn = 0xFFFFFFFFu, mx = 0u;
#pragma unroll
  for (int j0 = 0; j0 < JM; j0 += CH) {
    uint32_t x[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) x[j] = j0 + j < jv ? (uint32_t)key[base + (j0 + j) * 64] : 0u;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      mn = j0 + j < jv ? min(mn, x[j]) : mn;
      mx = j0 + j < jv ? max(mx, x[j]) : mx;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
    mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
  }
  if (lane == 0) {
    sc.wa[wid] = (int)mn;
    sc.wb[wid] = (int)mx;
  }
  if (radix)
    for (int i = tid; i < 512; i += NT) hist[i] = 0;
  __syncthreads();
  uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    lo = min(lo, (uint32_t)sc.wa[w]);
    hi = max(hi, (uint32_t)sc.wb[w]);
  }
  lo = (uint32_t)uni((int)lo);
  hi = (uint32_t)uni((int)hi);
  KVC_STAMP(2);
  int parity = 0;
  if (radix) {
    // the first pass publishes in sc.wa[1] / sc.wb[1], the next in [2] ... (read after its
    // barrier; no slot is rewritten), so the min / max words above may still be being read
    int rem = hi - lo ? 32 - __builtin_clz(hi - lo) : 0;  // offset bits still undecided
    uint32_t prefix = 0;
    int below = 0, slot = 1;
    while (rem > 0) {
      const int w = min(8, rem), sh = rem - w;
      int* h = hist + 256 * parity;
#pragma unroll
      for (int j0 = 0; j0 < JM; j0 += CH) {
        uint32_t x[CH];
#pragma unroll
        for (int j = 0; j < CH; ++j) x[j] = j0 + j < jv ? (uint32_t)key[base + (j0 + j) * 64] : 0u;
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const uint32_t d = x[j] - lo;
          if (j0 + j < jv && (rem == 32 ? 0u : d >> rem) == prefix)
            lds_add1(h + ((d >> sh) & ((1u << w) - 1u)));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the other buffer's last reader (wave 0, previous pass) finished before the last barrier
      for (int i = tid; i < 256; i += NT) hist[256 * (parity ^ 1) + i] = 0;
      __syncthreads();
      if (wid == 0) {
        const int c0 = h[4 * lane], c1 = h[4 * lane + 1], c2 = h[4 * lane + 2],
                  c3 = h[4 * lane + 3];
        const int s4 = c0 + c1 + c2 + c3;
        const int ex = block_exclusive_scan<64>(s4, nullptr, lane, 0);
        const int need = k - below;  // >= 1: the k-th key lies in this bucket
        const uint64_t b = __builtin_amdgcn_ballot_w64(ex + s4 >= need);
        if (lane == (b ? __builtin_ctzll(b) : 63)) {
          int c = ex, bin = 4 * lane;
          if (c + c0 < need) {
            c += c0; ++bin;
            if (c + c1 < need) {
              c += c1; ++bin;
              if (c + c2 < need) { c += c2; ++bin; }
            }
          }
          sc.wa[slot] = bin;
          sc.wb[slot] = below + c;
        }
      }
      __syncthreads();
      prefix = (prefix << w) | (uint32_t)sc.wa[slot];
      below = sc.wb[slot];
      ++slot;  // <= 4 passes: slots 1..4 of 16
      rem = sh;
      parity ^= 1;
    }
    lo = lo + prefix;
  } else {
    __syncthreads();  // sc.wa / sc.wb are the bisection's count buffers
  }
  // smallest v with #(key <= v) >= k (bisection; the radix select leaves lo at it)
  while (!radix && lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    int cl = 0;
#pragma unroll
    for (int j0 = 0; j0 < JM; j0 += CH) {
      uint32_t x[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) x[j] = j0 + j < jv ? (uint32_t)key[base + (j0 + j) * 64] : 0u;
#pragma unroll
      for (int j = 0; j < CH; ++j) cl += (j0 + j < jv && x[j] <= mid) ? 1 : 0;
    }
    const int rs = row_scan16(cl);
    const int c = __builtin_amdgcn_readlane(rs, 15) + __builtin_amdgcn_readlane(rs, 31) +
                  __builtin_amdgcn_readlane(rs, 47) + __builtin_amdgcn_readlane(rs, 63);
    const int tot = block_sum_waves<NT>(c, parity ? sc.wb : sc.wa, lane, wid);
    parity ^= 1;
    if (tot >= k) hi = mid;
    else lo = mid + 1;
  }
  KVC_STAMP(3);
  const uint32_t T = lo;
  typedef typename std::conditional<(JM > 32), uint64_t, uint32_t>::type FlagT;
  FlagT ltm = 0, eqm = 0;  // this lane's flags by j
  int clt = 0, ceq = 0;
#pragma unroll
  for (int j0 = 0; j0 < JM; j0 += CH) {
    uint32_t x[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) x[j] = j0 + j < jv ? (uint32_t)key[base + (j0 + j) * 64] : 0u;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const bool flt = j0 + j < jv && x[j] < T, feq = j0 + j < jv && x[j] == T;
      ltm |= flt ? (FlagT)1 << (j0 + j) : (FlagT)0;
      eqm |= feq ? (FlagT)1 << (j0 + j) : (FlagT)0;
      clt += __popcll(__builtin_amdgcn_ballot_w64(flt));
      ceq += __popcll(__builtin_amdgcn_ballot_w64(feq));
    }
  }
  if (lane == 0) sc.wm[wid] = clt | (ceq << 16);  // each <= kZoneMax < 2^16
  __syncthreads();
  int rlt = 0, req = 0, tlt = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int x = sc.wm[w];
    rlt += w < wid ? (x & 0xFFFF) : 0;
    req += w < wid ? (x >> 16) : 0;
    tlt += x & 0xFFFF;
  }
  const int need = k - tlt;  // 1 <= need <= #(key == T)
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const bool flt = (ltm >> j) & 1u, feq = (eqm >> j) & 1u;
    const uint64_t bl = __builtin_amdgcn_ballot_w64(flt), be = __builtin_amdgcn_ballot_w64(feq);
    const int lb = rlt + __popcll(bl & lanemask_lt(lane));
    const int eb = req + __popcll(be & lanemask_lt(lane));
    if (flt || (feq && eb < need)) {
      const int r = lb + min(eb, need);
      if constexpr (TO_LDS) sel[r] = (uint16_t)(base + j * 64);
      else out[r] = base + j * 64;
    }
    rlt += __popcll(bl);
    req += __popcll(be);
  }
}

// Reference-exact selection for one (layer, b, h) row whose zone norms are at `nrow`; working
// arrays at `arrays` (SelArrays layout for n_cap positions and `cap`-rank windows: LDS, or a
// global scratch row for zones longer than kZoneMax) and scalars in `sc`; NT threads (the
// workgroup) cooperate.  Emits the kept zone-local indices in ascending order to `out` (global
// int32) or, with TO_LDS, to `sel` (LDS u16, may alias the key region: keys are dead by then).
// Returns false (and ORs KVC_DEV_SELECT_BOUNDS into *status) when the row exceeds this kernel's
// zone capacity -- nothing is selected then.
template <int KC, bool TO_LDS, int MAXN, int NT, bool HH = false, bool STABLE = false,
          bool L0T = true>
__device__ __forceinline__ bool select_body(const kvc_layer_t* __restrict__ ly, int dt, int order,
                            int algo, const char* __restrict__ nrow, int32_t* out, uint16_t* sel,
                            char* arrays, int n_cap, int cap,
                            SelScalars<typename DTypeTraits<KC>::key_t>& sc,
                            int wave_seg, uint64_t* stamps, uint32_t* status,
                            const uint32_t* trow = nullptr, const char* pf_k = nullptr,
                            const char* pf_v = nullptr, int pf_rowb = 0) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  constexpr int ESZ = DTypeTraits<KC>::esz;
  constexpr int MAXJ = (MAXN + NT - 1) / NT;  // positions per lane, level 0
  const SelArrays<KeyT> A(arrays, n_cap, cap);
  KeyT* key = A.key;
  uint16_t* idx = A.idx;
  uint16_t* spos = A.spos;
  KVC_STAMP(0);
  const int n = ly->zone_len;
  const int k = ly->n_select;
  if (n > MAXN || n > n_cap) {  // a dispatch bug, never silent: flag it, select nothing
    if (threadIdx.x == 0 && status) atomicOr(status, (uint32_t)KVC_DEV_SELECT_BOUNDS);
    return false;
  }
  if (k <= 0 || n <= 0) return true;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (k >= n) {  // keep everything (e.g. h2o_l2 when the middle is no longer than heavy_hitter)
    for (int i = tid; i < n; i += NT) {
      if constexpr (TO_LDS) sel[i] = (uint16_t)i;
      else out[i] = i;
    }
    return true;
  }
  const bool desc = order == KVC_DESC;
  const bool topk = algo == KVC_ALGO_TOPK;
  const bool partial = topk && (int64_t)k * 64 <= n;  // aten TopKImpl.h: use_partial_sort
  const int thr = topk ? 3 : 16;  // introselect / introsort segment threshold
  // SCORE's level-0 tile counts of a plain-norm row (score_tile), loaded with the keys (below)
  // so that the load's latency passes under the key load: lane l < J0 of wave w holds tile
  // w J0 + l, J0 = level 0's positions per lane (partition_level).  Loaded in the plain-norm
  // branch only: the snapkv scoring keeps the VGPR.
  const bool l0use = kL0TileCounts && !STABLE && MAXJ <= 16 && trow &&
                     ly->score_mode == KVC_SCORE_NORM;
  uint32_t l0tc = 0;

  // ---- keys ----
  if (ly->score_mode == KVC_SCORE_SNAPKV) {
    // scratch for the unpooled scores from the idx region on: n u16 (bf16), or n floats over
    // idx + the rank tables (fp32 rows always get full n/2-rank tables: >= 4n bytes)
    char* tmp = reinterpret_cast<char*>(idx);
    if constexpr (ESZ == 2 && MAXN <= kZoneMax) {
      constexpr int MAXV = (MAXN / 8 + NT - 1) / NT;
      bool idx_done = false;
      with_dt<KC>(dt, [&](auto D) {
        idx_done = snapkv_keys16<D.value, NT, MAXV>(nrow, trow, n, ly->pool_kernel, desc,
                                                    reinterpret_cast<uint16_t*>(key), idx,
                                                    reinterpret_cast<uint16_t*>(tmp), sc, stamps);
      });
      if (!idx_done) {
        __syncthreads();  // the scores (in the idx region) are dead
        for (int v = tid; v < (n + 7) / 8; v += NT) {
          const uint32_t b = (uint32_t)v * 8;
          reinterpret_cast<uint4*>(idx)[v] =
              make_uint4(b | (b + 1) << 16, (b + 2) | (b + 3) << 16, (b + 4) | (b + 5) << 16,
                         (b + 6) | (b + 7) << 16);
        }
      }
    } else {
      with_dt<KC>(dt, [&](auto D) {
        snapkv_keys<D.value, KeyT, NT>(nrow, n, ly->pool_kernel, desc, key, tmp, sc);
      });
      __syncthreads();
      for (int i = tid; i < n; i += NT) idx[i] = (uint16_t)i;
    }
  } else {
    // 16-B loads, all issued before the first use (norm rows are padded to 64 elements, so a
    // whole vector past n stays inside the row); keys/indices written as 16-B LDS stores
    if (l0use) {
      const int J0 = (n - 1 + NT - 1) / NT, t = wid * J0 + lane;
      l0tc = lane < J0 && t < (n + kTile - 1) / kTile ? trow[t] : 0u;
    }
    constexpr int VEC = 16 / ESZ;
    constexpr int MAXV = ((MAXN < kZoneMax ? MAXN : kZoneMax) / VEC + NT - 1) / NT;  // per batch
    const int nvec = (n + VEC - 1) / VEC;
    for (int v0 = 0; v0 < nvec; v0 += MAXV * NT) {  // one batch for n <= kZoneMax
    uint4 buf[MAXV];
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      const int v = v0 + tid + q * NT;
      if (v < nvec) buf[q] = reinterpret_cast<const uint4*>(nrow)[v];
    }
#pragma unroll
    for (int q = 0; q < MAXV; ++q) {
      const int v = v0 + tid + q * NT;
      if (v < nvec) {
        const uint32_t w[4] = {buf[q].x, buf[q].y, buf[q].z, buf[q].w};
        uint32_t kw[4], iw[4];
        if constexpr (KC != KVC_F32) {
          // packed key map (key_h16x2): key_h16's order and ties, other codes -- every key of
          // the row is made here, and the selection only compares keys with each other
          const uint32_t inf = inf_bits16(dt);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            kw[e] = key_h16x2(w[e], desc, inf);
            iw[e] = (uint32_t)(v * 8 + 2 * e) | ((uint32_t)(v * 8 + 2 * e + 1) << 16);
          }
          *reinterpret_cast<uint4*>(key + v * 8) = make_uint4(kw[0], kw[1], kw[2], kw[3]);
          *reinterpret_cast<uint4*>(idx + v * 8) = make_uint4(iw[0], iw[1], iw[2], iw[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) kw[e] = key_f32(w[e], desc);
          *reinterpret_cast<uint4*>(key + v * 4) = make_uint4(kw[0], kw[1], kw[2], kw[3]);
          *reinterpret_cast<uint2*>(idx + v * 4) =
              make_uint2((uint32_t)(v * 4) | ((uint32_t)(v * 4 + 1) << 16),
                         (uint32_t)(v * 4 + 2) | ((uint32_t)(v * 4 + 3) << 16));
        }
      }
    }
    }
  }
  __syncthreads();
  KVC_STAMP(1);

  // ---- KVC_ALGO_STABLE: the first k of a stable sort (ties in position order) ----
  if constexpr (STABLE) {
    static_assert(MAXJ <= 64, "stable selection: positions per lane (flag words)");
    if constexpr (MAXN > kZoneMax) {
      // the global-scratch variant (zones up to kZoneMaxGlobal): the histograms in LDS
      __shared__ int stable_hist[512];
      stable_select<NT, MAXJ, KeyT, TO_LDS>(key, n, k, sc, out, sel, stable_hist, true, stamps);
    } else {
      // the radix histograms (512 ints) over the idx region and the rank tables, unused here
      // (sel, when in LDS, is the idx region too: written only after the last histogram read);
      // shorter rows bisect over the key range instead
      const bool radix = (size_t)n_cap * 2 + (size_t)(cap + 72) * 4 >= 2048;
      stable_select<NT, MAXJ, KeyT, TO_LDS>(key, n, k, sc, out, sel, reinterpret_cast<int*>(idx),
                                            radix, stamps);
    }
    KVC_STAMP(4);
    return true;
  }

  // ---- reference-exact k-selection ----
  if constexpr (sizeof(KeyT) == 4 && MAXJ <= 16) {  // fp32 keys: untied boundary -> values only
    // (`sel` may alias the key region: the keys are read into registers before any store)
    // the rank tables (>= 2 KiB from n_cap = 1024 on) hold the radix histograms
    const bool radix = (size_t)(cap + 72) * 4 >= 2048;
    if (select_fast_untied<NT, MAXJ, KeyT, TO_LDS>(key, n, k, sc, out, sel,
                                                   reinterpret_cast<int*>(idx + n_cap), radix)) {
      KVC_STAMP(31);  // diagnostic build: fast path taken
      return true;
    }
  }
  if (partial) {  // std::partial_sort's heap select
    bool done = false;
    if constexpr (HH && NT > 64) {  // heavy-hitter kernels only: see heap_candidates
      if (k <= 64 && n >= 4096) {
        // wave 0 builds the register heap while the other waves prefilter the scan's candidates
        // into the rank tables (unused by the heap select); then wave 0 scans only those
        constexpr bool PK = sizeof(KeyT) == 2;
        RegHeap<PK> h;
        if (wid == 0) reg_heap_make(h, key, idx, k);
        uint16_t* cand = idx + n_cap;
        const int nc = heap_candidates<NT>(key, k, n, cand, (cap + 72) * 2, sc.wa, sc.wb, 1);
        if (wid == 0) reg_heap_scan(h, key, idx, k, n, nc >= 0 ? cand : nullptr, nc);
        done = true;
      }
    }
    if (!done && wid == 0) wave_heap_select(key, idx, k, n);
  } else {
    int lo = 0, hi = n, depth = 2 * floor_log2(n), level = 0;
    uint64_t* accb = nullptr;
    uint64_t* accw = nullptr;
#ifdef KVC_STAMPS
    if (stamps) {
      accb = stamps + blockIdx.x * 32 + 5;
      accw = stamps + blockIdx.x * 32 + 10;
      if (tid == 0)
        for (int q = 0; q < 21; ++q) accb[q] = 0;
    }
#endif
    const int st = run_chain<KeyT, NT, MAXJ, L0T>(
        key, idx, spos, A.gpos, sc, k, topk, thr, cap, lo, hi, depth, level, wave_seg, accb, status,
        l0use, l0tc, desc, MAXJ <= 16 ? n_cap / 2 : 0, !STABLE && ly->score_mode == KVC_SCORE_NORM);
    KVC_STAMP(2);
    if (st == 1 && wid == 0)
      run_chain<KeyT, 64, 16>(key, idx, spos, A.gpos, sc, k, topk, thr, cap, lo, hi, depth,
                              level, wave_seg, accw, status);
    if constexpr (kSgPrefetch && TO_LDS && NT > 64) {
      // while wave 0 finishes the chain, the other waves touch the K / V rows of the positions
      // already known to be kept (idx[0, lo): stable, wave 0 only rearranges [lo, hi)), so that
      // the row's copy finds them in the caches (diagnostic A/B: KVC_SG_PREFETCH)
      if (st == 1 && wid > 0 && pf_rowb > 0) {
        const int64_t kss = ly->k_stride[2] * ESZ, vss = ly->v_stride[2] * ESZ;
        for (int u = tid - 64; u < lo * 4; u += NT - 64) {
          const int p = ly->zone_start + (int)idx[u >> 2];
          const char* a = ((u & 2) ? pf_v + p * vss : pf_k + p * kss) + ((u & 1) ? pf_rowb - 4 : 0);
          const uint32_t x = *reinterpret_cast<const volatile uint32_t*>(a);
          asm volatile("" ::"v"(x));
        }
      }
    }
  }
  __syncthreads();
  KVC_STAMP(3);

  // ---- emit the kept set {idx[0..k)} as ascending zone-local indices: a bitmap of the kept
  // positions over the (dead) key region, one block scan of per-thread popcounts, and each
  // thread writing the positions of its words.  Every bitmap word is in registers before the
  // scan's barrier, so `sel` (which aliases the key region) is only written after it.
  uint32_t* bm = reinterpret_cast<uint32_t*>(key);
  const int nw = (n + 31) >> 5;
  for (int w = tid; w < nw; w += NT) bm[w] = 0u;
  __syncthreads();
  for (int i = tid; i < k; i += NT) {
    const int x = idx[i];
    atomicOr(&bm[x >> 5], 1u << (x & 31));
  }
  __syncthreads();
  constexpr int MAXW = (MAXN / 32 + NT - 1) / NT;  // bitmap words per thread
  uint32_t wv[MAXW];
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < MAXW; ++q) {
    const int w = tid * MAXW + q;
    wv[q] = w < nw ? bm[w] : 0u;
    cnt += __popc(wv[q]);
  }
  int r = block_exclusive_scan<NT>(cnt, sc.wa, lane, wid);
#pragma unroll
  for (int q = 0; q < MAXW; ++q) {
    const int base = (tid * MAXW + q) * 32;
    for (uint32_t b = wv[q]; b; b &= b - 1u, ++r) {
      const int pos = base + (int)__builtin_ctz(b);
      if constexpr (TO_LDS) sel[r] = (uint16_t)pos;
      else out[r] = pos;
    }
  }
  KVC_STAMP(4);
  return true;
}


// One workgroup of NT threads per (layer, b, h) row.  NT = 256 for zones up to 4 096
// positions, arrays in dynamic LDS sized by the call's longest zone (n_cap): several rows per
// CU.  NT = 1 024 beyond, arrays in static LDS laid out for kZoneMax (compile-time addresses)
// with rank windows of kSelCapBig: two rows per CU for bf16.
template <typename KeyT>
constexpr int kSelCapBig = sel_cap(kZoneMax, (int)sizeof(KeyT), kBigBudget);
template <typename KeyT>
constexpr int kSelBytesBig = (int)sel_bytes(kZoneMax, (int)sizeof(KeyT), kSelCapBig<KeyT>);

// 8 waves per SIMD: two 1024-thread rows per CU (fp32 rows of the big kernel: one per CU, LDS).
// HH: the heavy-hitter instance (kvc_heavy_hitters), whose heap selects prefilter their scan.
template <int KC, int NT, bool HH = false, bool STABLE = false>
__global__ void __launch_bounds__(NT, sel_waves_per_eu(KC, NT, HH))
    select_kernel(const LayerChunk T, int BH, int dt, int order, int algo,
                  const char* __restrict__ norms, int64_t norm_stride,
                  int32_t* __restrict__ out_idx, int64_t idx_stride, int wave_seg, int n_cap,
                  int cap, uint64_t* stamps, uint32_t* status, const uint32_t* __restrict__ tmax) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  constexpr int ESZ = DTypeTraits<KC>::esz;
  constexpr int MAXN = NT == kSelThreads ? kZoneMax : NT * 16;
  __shared__ SelScalars<KeyT> sc;
  const kvc_layer_t* ly = T.l + blockIdx.x / BH;
  const int row = ly->row0 + (int)(blockIdx.x % BH);  // global workspace row
  const uint32_t* trow = tmax ? tmax + (int64_t)row * (norm_stride / kTile) : nullptr;
  if constexpr (NT == kSelThreads) {
    // LDS: key[kZoneMax] | idx[kZoneMax] (u16) | spos | gpos (u16 rank windows) -- SelArrays
    __shared__ __attribute__((aligned(16))) char smem[kSelBytesBig<KeyT>];
    select_body<KC, false, MAXN, NT, HH, STABLE>(ly, dt, order, algo,
                                     norms + (int64_t)row * norm_stride * ESZ,
                                     out_idx + (int64_t)row * idx_stride, nullptr, smem, kZoneMax,
                                     kSelCapBig<KeyT>, sc, wave_seg, stamps, status, trow);
  } else {
    extern __shared__ __attribute__((aligned(16))) char dsmem[];
    select_body<KC, false, MAXN, NT, HH, STABLE>(ly, dt, order, algo,
                                     norms + (int64_t)row * norm_stride * ESZ,
                                     out_idx + (int64_t)row * idx_stride, nullptr, dsmem, n_cap,
                                     cap, sc, wave_seg, stamps, status, trow);
  }
}

// Zones longer than kZoneMax (up to kZoneMaxGlobal): the same selection with its arrays in a
// per-row global scratch (L2 / Infinity-Cache resident; a workgroup barrier orders the
// workgroup's global accesses like LDS ones -- all its waves share one CU's L1).
template <int KC, bool STABLE = false>
__global__ void __launch_bounds__(kSelThreads)
    select_global_kernel(const LayerChunk T, int BH, int dt, int order, int algo,
                         const char* __restrict__ norms, int64_t norm_stride,
                         int32_t* __restrict__ out_idx, int64_t idx_stride, int wave_seg,
                         char* __restrict__ scratch, int64_t scratch_row_bytes, int n_cap,
                         uint32_t* status) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  constexpr int ESZ = DTypeTraits<KC>::esz;
  __shared__ SelScalars<KeyT> sc;
  const kvc_layer_t* ly = T.l + blockIdx.x / BH;
  const int row = ly->row0 + (int)(blockIdx.x % BH);
  select_body<KC, false, kZoneMaxGlobal, kSelThreads, false, STABLE>(
      ly, dt, order, algo, norms + (int64_t)row * norm_stride * ESZ,
      out_idx + (int64_t)row * idx_stride, nullptr, scratch + (int64_t)row * scratch_row_bytes,
      n_cap, n_cap / 2 + 1, sc, wave_seg, nullptr, status);
}

// Zones longer than kZoneMaxGlobal (up to kZoneMaxLong): the same partition chain with u32
// positions and full rank tables in a per-row global scratch
//   key[n_cap] | idx[n_cap] (u32) | spos[n_cap/2 + 2] (u32) | gpos[n_cap/2 + 2] (u32)
// Too many positions per lane to keep a level's flags in registers, so each pass re-derives
// them from the keys (the keys do not change between a level's passes: the median move and the
// swaps run after the last one); counts are plain ints.  Rare, long rows: simplicity over speed.
__host__ __device__ constexpr size_t sel_long_bytes(int n_cap, int key_size) {
  return (size_t)n_cap * key_size + (size_t)n_cap * 4 + 2 * (size_t)(n_cap / 2 + 2) * 4;
}

struct LongScalars {
  int ge[kSelWaves];
  int le[kSelWaves];
  int nsw[kSelWaves];
  int ff[kSelWaves];
};

// One level over [lo, hi) (see run_chain for the algorithm); returns cut.
template <typename KeyT>
__device__ int partition_long(KeyT* key, uint32_t* idx, uint32_t* spos, uint32_t* gpos,
                              LongScalars& sc, int lo, int hi) {
  const int tid = threadIdx.x, lane = tid & 63, wid = uni(tid >> 6);
  const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
  const uint32_t ka = (uint32_t)uni((int)key[a]), kb = (uint32_t)uni((int)key[b]);
  const uint32_t kc = (uint32_t)uni((int)key[c]), klo = (uint32_t)uni((int)key[lo]);
  int ch;  // std::__move_median_to_first(lo, a, b, c)
  if (ka < kb) {
    if (kb < kc) ch = b; else if (ka < kc) ch = c; else ch = a;
  } else if (ka < kc) {
    ch = a;
  } else if (kb < kc) {
    ch = c;
  } else {
    ch = b;
  }
  const uint32_t p = (ch == a) ? ka : (ch == b) ? kb : kc;
  const int J = (hi - lo - 1 + kSelThreads - 1) / kSelThreads;
  const int wbeg = lo + 1 + wid * J * 64;
  const int half = (hi - lo) / 2 + 1;  // swapped ranks m <= (n - 1) / 2
  // ---- P1: wave counts of ge / le positions ----
  int cge = 0, cle = 0;
  for (int j = 0; j < J; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool inb = pos < hi;
    const uint32_t kk = inb ? (pos == ch ? klo : (uint32_t)key[pos]) : 0u;
    cge += __popcll(__builtin_amdgcn_ballot_w64(inb && kk >= p));
    cle += __popcll(__builtin_amdgcn_ballot_w64(inb && kk <= p));
  }
  if (lane == 0) {
    sc.ge[wid] = cge;
    sc.le[wid] = cle;
  }
  __syncthreads();
  int ge_before = 0, le_before = 0, tot_le = 0;
  for (int w = 0; w < kSelWaves; ++w) {
    const int g = sc.ge[w], l = sc.le[w];
    ge_before += w < wid ? g : 0;
    le_before += w < wid ? l : 0;
    tot_le += l;
  }
  // ---- P2: rank -> position tables, swap count, first unswapped ge ----
  int rge = ge_before, rle = le_before, nsw = 0, ff = kBig;
  for (int j = 0; j < J; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool inb = pos < hi;
    const uint32_t kk = inb ? (pos == ch ? klo : (uint32_t)key[pos]) : 0u;
    const bool ge = inb && kk >= p, le = inb && kk <= p;
    const uint64_t bg = __builtin_amdgcn_ballot_w64(ge), bl = __builtin_amdgcn_ballot_w64(le);
    const int A = mbcnt(bg, rge);
    const int lin = mbcnt(bl, rle) + (le ? 1 : 0);
    const bool cond = A + lin < tot_le;
    const int sr = tot_le - lin + 1;
    if (le && sr <= half) spos[sr] = (uint32_t)pos;
    if (ge && cond) gpos[A + 1] = (uint32_t)pos;
    const uint64_t bc = __builtin_amdgcn_ballot_w64(cond);
    nsw += __popcll(bg & bc);
    const uint64_t bf = bg & ~bc;
    ff = min(ff, bf ? wbeg + j * 64 + (int)__builtin_ctzll(bf) : kBig);
    rge += __popcll(bg);
    rle += __popcll(bl);
  }
  if (lane == 0) {
    sc.nsw[wid] = nsw;
    sc.ff[wid] = ff;
  }
  __syncthreads();
  int msw = 0, gnext = kBig;
  for (int w = 0; w < kSelWaves; ++w) {
    msw += sc.nsw[w];
    gnext = min(gnext, sc.ff[w]);  // stripes ascend with the wave id
  }
  if (tid == 0) kv_swap(key, idx, lo, ch);  // the median move, made physical
  __syncthreads();
  // ---- P4: the m disjoint swaps g_t <-> s_t ----
  for (int t = tid + 1; t <= msw; t += kSelThreads) {
    const int g = (int)gpos[t], sv = (int)spos[t];
    const KeyT kg = key[g], ks = key[sv];
    const uint32_t ig = idx[g], is = idx[sv];
    key[g] = ks;
    key[sv] = kg;
    idx[g] = is;
    idx[sv] = ig;
  }
  const int cut = min(gnext, msw > 0 ? (int)spos[msw] : kBig);
  __syncthreads();  // tables and counters are reused by the next level
  return cut;
}

template <int KC>
__global__ void __launch_bounds__(kSelThreads)
    select_long_kernel(const LayerChunk T, int BH, int dt, int order, int algo,
                       const char* __restrict__ norms, int64_t norm_stride,
                       int32_t* __restrict__ out_idx, int64_t idx_stride,
                       char* __restrict__ scratch, int64_t scratch_row_bytes, int n_cap,
                       uint32_t* status) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  constexpr int ESZ = DTypeTraits<KC>::esz;
  __shared__ SelScalars<KeyT> ssc;
  __shared__ LongScalars sc;
  const kvc_layer_t* ly = T.l + blockIdx.x / BH;
  const int row = ly->row0 + (int)(blockIdx.x % BH);
  const int n = ly->zone_len, k = ly->n_select;
  if (n > n_cap || n > kZoneMaxLong) {
    if (threadIdx.x == 0 && status) atomicOr(status, (uint32_t)KVC_DEV_SELECT_BOUNDS);
    return;
  }
  if (k <= 0 || n <= 0) return;
  const char* nrow = norms + (int64_t)row * norm_stride * ESZ;
  int32_t* out = out_idx + (int64_t)row * idx_stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (k >= n) {
    for (int i = tid; i < n; i += kSelThreads) out[i] = i;
    return;
  }
  char* base = scratch + (int64_t)row * scratch_row_bytes;
  KeyT* key = reinterpret_cast<KeyT*>(base);
  uint32_t* idx = reinterpret_cast<uint32_t*>(base + (size_t)n_cap * sizeof(KeyT));
  uint32_t* spos = idx + n_cap;
  uint32_t* gpos = spos + (n_cap / 2 + 2);
  const bool desc = order == KVC_DESC;
  if (ly->score_mode == KVC_SCORE_SNAPKV) {  // unpooled scores in the idx region first
    with_dt<KC>(dt, [&](auto D) {
      snapkv_keys<D.value, KeyT, kSelThreads>(nrow, n, ly->pool_kernel, desc, key,
                                              reinterpret_cast<char*>(idx), ssc);
    });
    __syncthreads();
  } else {
    for (int i = tid; i < n; i += kSelThreads) {
      if constexpr (KC == KVC_F32)
        key[i] = key_f32(reinterpret_cast<const uint32_t*>(nrow)[i], desc);
      else
        key[i] = key_h16(reinterpret_cast<const uint16_t*>(nrow)[i], desc, inf_bits16(dt));
    }
  }
  for (int i = tid; i < n; i += kSelThreads) idx[i] = (uint32_t)i;
  __syncthreads();
  const bool topk = algo == KVC_ALGO_TOPK;
  if (topk && (int64_t)k * 64 <= n) {  // std::partial_sort's heap select (one wave)
    if (wid == 0) wave_heap_select(key, idx, k, n);
  } else {
    const int thr = topk ? 3 : 16;
    int lo = 0, hi = n, depth = 2 * floor_log2(n);
    while (true) {
      if (lo == k || hi == k) break;
      if (hi - lo <= thr) {
        if (tid == 0) insertion_sort(key, idx, lo, hi);
        break;
      }
      if (depth == 0) {
        if (tid == 0) {
          if (topk) {
            heap_select(key + lo, idx + lo, k - lo, hi - lo);
            kv_swap(key, idx, lo, k - 1);
          } else {
            make_heap(key + lo, idx + lo, hi - lo);
            sort_heap(key + lo, idx + lo, hi - lo);
          }
        }
        break;
      }
      --depth;
      const int cut = partition_long<KeyT>(key, idx, spos, gpos, sc, lo, hi);
      if (topk) {
        if (cut <= k - 1) lo = cut; else hi = cut;
      } else {
        if (k <= cut) hi = cut; else lo = cut;
      }
    }
  }
  __syncthreads();
  // ---- emit {idx[0..k)} ascending: u16 flags over the (dead) key region, two counted passes
  uint16_t* flag = reinterpret_cast<uint16_t*>(key);
  for (int i = tid; i < n; i += kSelThreads) flag[i] = 0;
  __syncthreads();
  for (int i = tid; i < k; i += kSelThreads) flag[idx[i]] = 1;
  __syncthreads();
  const int J = (n + kSelThreads - 1) / kSelThreads;
  const int wbeg = wid * J * 64;
  int c = 0;
  for (int j = 0; j < J; ++j) {
    const int pos = wbeg + j * 64 + lane;
    c += __popcll(__builtin_amdgcn_ballot_w64(pos < n && flag[pos] != 0));
  }
  if (lane == 0) sc.ge[wid] = c;
  __syncthreads();
  int run = 0;
  for (int w = 0; w < wid; ++w) run += sc.ge[w];
  for (int j = 0; j < J; ++j) {
    const int pos = wbeg + j * 64 + lane;
    const bool f = pos < n && flag[pos] != 0;
    const uint64_t bf = __builtin_amdgcn_ballot_w64(f);
    if (f) out[run + __popcll(bf & lanemask_lt(lane))] = pos;
    run += __popcll(bf);
  }
}

// ---------------------------------------------------------------------------------------------
// GATHER
// ---------------------------------------------------------------------------------------------
// Output rows a GATHER launch copies (KVC_FLAG_GATHER_FIXED / _SELECTED): all, the sink and
// tail rows, or the selected rows -- as a count of "virtual" rows and the map to output rows.
enum { PART_ALL = 0, PART_FIXED = 1, PART_SELECTED = 2 };
__host__ __device__ __forceinline__ int part_rows(const kvc_layer_t& y, int part) {
  return part == PART_FIXED ? y.sink_len + y.tail_len
                            : part == PART_SELECTED ? y.n_select : y.sink_len + y.n_select +
                                                                       y.tail_len;
}
__device__ __forceinline__ int part_row(int v, int sink, int nsel, int part) {
  return part == PART_FIXED ? (v < sink ? v : v + nsel) : part == PART_SELECTED ? v + sink : v;
}

// One block of the copy: kGatherTokens output rows of K and V of workspace row `grow`
// (layer * BH + b * H + h), token block `by`.
template <int DT, int NC, bool NTS>
__device__ __forceinline__ void gather_block(const kvc_layer_t* __restrict__ L, int H, int BH,
                                             const int32_t* __restrict__ gidx,
                                             int64_t idx_stride, int shared, uint32_t* status,
                                             int part, int grow, int by) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  constexpr int ITERS = (kGatherTokens * NC + kGatherThreads - 1) / kGatherThreads;
  const kvc_layer_t* ly = L + grow / BH;
  const int r = grow - (grow / BH) * BH;
  const int n_out = ly->n_out;
  const int nv = part_rows(*ly, part);  // rows this launch copies
  const int t0 = by * kGatherTokens;
  if (t0 >= nv) return;
  const int nu = min(kGatherTokens, nv - t0) * NC;
  const int b = r / H, h = r - (r / H) * H;
  const int sink = ly->sink_len, nsel = ly->n_select;
  const char* kb = static_cast<const char*>(ly->k) +
                   ((int64_t)b * ly->k_stride[0] + (int64_t)h * ly->k_stride[1]) * ESZ;
  const char* vb = static_cast<const char*>(ly->v) +
                   ((int64_t)b * ly->v_stride[0] + (int64_t)h * ly->v_stride[1]) * ESZ;
  const int64_t kss = ly->k_stride[2] * ESZ, vss = ly->v_stride[2] * ESZ;
  // index row of (layer, b, h); KVC_FLAG_SHARED_INDEX: (layer, b)'s row serves every head
  const int32_t* irow = gidx + (int64_t)((ly->row0 + r) / (shared ? H : 1)) * idx_stride;
  const int64_t obase = (int64_t)r * n_out * NC * 16;
  char* ko = static_cast<char*>(ly->k_out) + obase;
  char* vo = static_cast<char*>(ly->v_out) + obase;
  uint4 xk[ITERS], xv[ITERS];
  bool gat[ITERS];
  int64_t oofs[ITERS];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int u = threadIdx.x + i * kGatherThreads;
    gat[i] = false;
    oofs[i] = 0;
    if (u < nu) {
      const int t = part_row(t0 + u / NC, sink, nsel, part), c = u - (u / NC) * NC;
      oofs[i] = ((int64_t)t * NC + c) * 16;
      int src;
      if (t < sink) {
        src = t;
      } else if (t < sink + nsel) {
        int zi = irow[t - sink];
        if ((zi < 0 || zi >= ly->zone_len) && status)  // never read outside the zone: clamp
          atomicOr(status, (uint32_t)KVC_DEV_INDEX_RANGE);
        zi = min(max(zi, 0), ly->zone_len - 1);
        src = ly->zone_start + zi;
        gat[i] = true;
      } else {
        src = ly->tail_start + (t - sink - nsel);
      }
      xk[i] = *reinterpret_cast<const uint4*>(kb + src * kss + c * 16);
      xv[i] = *reinterpret_cast<const uint4*>(vb + src * vss + c * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int u = threadIdx.x + i * kGatherThreads;
    if (u < nu) {
      uint4 a = xk[i], bq = xv[i];
      if (gat[i]) {  // torch.gather's NaN rewrite (gathered segment only)
        a = canon_nan_dt<DT>(a);
        bq = canon_nan_dt<DT>(bq);
      }
      if constexpr (NTS) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4{a.x, a.y, a.z, a.w},
                                    reinterpret_cast<u32x4*>(ko + oofs[i]));
        __builtin_nontemporal_store(u32x4{bq.x, bq.y, bq.z, bq.w},
                                    reinterpret_cast<u32x4*>(vo + oofs[i]));
      } else {
        *reinterpret_cast<uint4*>(ko + oofs[i]) = a;
        *reinterpret_cast<uint4*>(vo + oofs[i]) = bq;
      }
    }
  }
}

// grid = (rows, output-token blocks), one block each -- or, with loop_rows > 0, a capped 1-D grid
// whose blocks stride over the rows * nby blocks (the fixed rows of h2o_attention copied beside
// its heavy-hitter selection: a few resident workgroups per CU leave room for the selection's).
template <int DT, int NC, bool NTS>
__global__ void __launch_bounds__(kGatherThreads)
    gather_kernel(const LayerChunk T, int H, int BH, const int32_t* __restrict__ gidx,
                  int64_t idx_stride, int shared, uint32_t* status, int part, int loop_rows,
                  int nby) {
  if (loop_rows == 0) {
    gather_block<DT, NC, NTS>(T.l, H, BH, gidx, idx_stride, shared, status, part, blockIdx.x,
                              blockIdx.y);
    return;
  }
  const int nvb = loop_rows * nby;
  for (int vb = blockIdx.x; vb < nvb; vb += gridDim.x)
    gather_block<DT, NC, NTS>(T.l, H, BH, gidx, idx_stride, shared, status, part, vb % loop_rows,
                              vb / loop_rows);
}

// ---------------------------------------------------------------------------------------------
// Row copy shared by the select+gather kernel
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ bool layer_selects(const kvc_layer_t& y) {
  return y.n_select > 0 && y.n_select < y.zone_len;
}

// Copy one output row (sink ++ selected ++ tail) of K and V with the whole workgroup.
// sel: ascending zone-local kept indices in LDS, or nullptr when no selection ran.
// Thread tid copies 16-B chunk tid % NC of output tokens tid / NC + i * (NT / NC): the same
// coalesced units as a flat unit loop (consecutive threads, consecutive 16-B units) with the
// chunk and its address offsets fixed per thread; the last NT % NC threads idle.
// part: PART_ALL, or PART_SELECTED / PART_FIXED (the row's copy split between the selecting
// workgroup and a copy-only one, part_rows / part_row).
template <int DT, int NC, int NT = kSelThreads, bool NTS = false>
__device__ __forceinline__ void gather_row(const kvc_layer_t* __restrict__ ly, int r, int H,
                                           const uint16_t* sel, int part = PART_ALL) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  constexpr int BATCH = 4;
  constexpr int TPI = NT / NC;  // tokens per pass
  static_assert(TPI >= 1, "a row's chunks must fit the workgroup");
  const int tq = (int)threadIdx.x / NC, c = (int)threadIdx.x - tq * NC;
  if (tq >= TPI) return;
  const int n_out = ly->n_out;
  const int b = r / H, h = r - (r / H) * H;
  const int sink = ly->sink_len, nsel = ly->n_select;
  const int nv = part_rows(*ly, part);  // rows this workgroup copies
  const char* kb = static_cast<const char*>(ly->k) +
                   ((int64_t)b * ly->k_stride[0] + (int64_t)h * ly->k_stride[1]) * ESZ + c * 16;
  const char* vb = static_cast<const char*>(ly->v) +
                   ((int64_t)b * ly->v_stride[0] + (int64_t)h * ly->v_stride[1]) * ESZ + c * 16;
  const int64_t kss = ly->k_stride[2] * ESZ, vss = ly->v_stride[2] * ESZ;
  char* ko = static_cast<char*>(ly->k_out) + (int64_t)r * n_out * NC * 16 + c * 16;
  char* vo = static_cast<char*>(ly->v_out) + (int64_t)r * n_out * NC * 16 + c * 16;
  for (int tb = tq; tb < nv; tb += TPI * BATCH) {
    uint4 xk[BATCH], xv[BATCH];
    bool gat[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int v = tb + i * TPI;
      const int t = part_row(v, sink, nsel, part);
      gat[i] = false;
      if (v < nv) {
        int src;
        if (t < sink) {
          src = t;
        } else if (t < sink + nsel) {
          int zi = sel ? (int)sel[t - sink] : t - sink;
          zi = min(max(zi, 0), ly->zone_len - 1);
          src = ly->zone_start + zi;
          gat[i] = true;
        } else {
          src = ly->tail_start + (t - sink - nsel);
        }
        if constexpr (kSgNtl) {  // kept rows are read once: non-temporal
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kb + src * kss));
          const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vb + src * vss));
          xk[i] = make_uint4(a.x, a.y, a.z, a.w);
          xv[i] = make_uint4(q.x, q.y, q.z, q.w);
        } else {
          xk[i] = *reinterpret_cast<const uint4*>(kb + src * kss);
          xv[i] = *reinterpret_cast<const uint4*>(vb + src * vss);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int v = tb + i * TPI;
      const int t = part_row(v, sink, nsel, part);
      if (v < nv) {
        uint4 a = xk[i], q = xv[i];
        if (gat[i]) {
          a = canon_nan_dt<DT>(a);
          q = canon_nan_dt<DT>(q);
        }
        const int64_t off = (int64_t)t * (NC * 16);
        if constexpr (NTS) {  // written once: non-temporal
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(u32x4{a.x, a.y, a.z, a.w},
                                      reinterpret_cast<u32x4*>(ko + off));
          __builtin_nontemporal_store(u32x4{q.x, q.y, q.z, q.w},
                                      reinterpret_cast<u32x4*>(vo + off));
        } else {
          *reinterpret_cast<uint4*>(ko + off) = a;
          *reinterpret_cast<uint4*>(vo + off) = q;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// SELECT + GATHER: one workgroup per (layer, b, h) row selects into LDS and copies the row's
// output (sink ++ selected ++ tail of K and V) straight from the LDS index list.  With two
// workgroups per CU, one row's copy (HBM-bound) overlaps the other's selection (LDS/issue-
// bound), and the index list never round-trips through global memory.  Layout and thread
// counts as select_kernel; rows without a selection only copy.
// ---------------------------------------------------------------------------------------------
// L0T: level 0 may keep its rank tables in the idx region (run_chain); the instance without that
// code runs launches where it does not pay (launch_chunk)
template <int KC, int NT, int NC, bool STABLE = false, bool L0T = true>
__global__ void __launch_bounds__(NT, sel_waves_per_eu(KC, NT))
    select_gather_kernel(const LayerChunk T, int H, int BH, int dt, int order, int algo,
                         const char* __restrict__ norms, int64_t norm_stride, int wave_seg,
                         int n_cap, int cap, uint32_t* status, int split_rows,
                         const uint32_t* __restrict__ tmax) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  constexpr int ESZ = DTypeTraits<KC>::esz;
  constexpr int MAXN = NT == kSelThreads ? kZoneMax : NT * 16;
  __shared__ SelScalars<KeyT> sc;
  // split_rows > 0 (few rows: fewer than the CUs): workgroups [split_rows, 2 split_rows) copy the
  // sink / tail rows of row blockIdx - split_rows on otherwise idle CUs while the row's own
  // workgroup selects; the selecting workgroup then copies only the selected rows
  const bool copier = split_rows > 0 && (int)blockIdx.x >= split_rows;
  const int wg = copier ? (int)blockIdx.x - split_rows : (int)blockIdx.x;
  const kvc_layer_t* ly = T.l + wg / BH;
  const int r = wg % BH;
  if (ly->n_out == 0) return;
  const bool selects = layer_selects(*ly);
  if constexpr (NT == kSelThreads) {
    n_cap = kZoneMax;
    cap = kSelCapBig<KeyT>;
  }
  if (copier) {
    // a row over the selecting workgroup's capacity is flagged there and left wholly unwritten
    // (KVC_DEV_SELECT_BOUNDS): its sink / tail rows are not copied either
    if (selects && ly->zone_len <= MAXN && ly->zone_len <= n_cap)
      with_dt<KC>(dt, [&](auto D) {
        gather_row<D.value, NC, NT, kSgNts>(ly, r, H, nullptr, PART_FIXED);
      });
    return;
  }
  const char* nrow = norms + (int64_t)(ly->row0 + r) * norm_stride * ESZ;
  char* arrays;
  if constexpr (NT == kSelThreads) {
    __shared__ __attribute__((aligned(16))) char smem[kSelBytesBig<KeyT>];
    arrays = smem;
  } else {
    extern __shared__ __attribute__((aligned(16))) char dsmem[];
    arrays = dsmem;
  }
  // the kept positions: over the key region, dead after the chain (the stable selection reads
  // its keys to the end: the idx region then)
  uint16_t* sel = reinterpret_cast<uint16_t*>(arrays + (STABLE ? (size_t)n_cap * sizeof(KeyT) : 0));
  if (selects) {
    const uint32_t* trow =
        tmax ? tmax + (int64_t)(ly->row0 + r) * (norm_stride / kTile) : nullptr;
    const int b = r / H, h = r - (r / H) * H;
    const char* pk = static_cast<const char*>(ly->k) +
                     ((int64_t)b * ly->k_stride[0] + (int64_t)h * ly->k_stride[1]) * ESZ;
    const char* pv = static_cast<const char*>(ly->v) +
                     ((int64_t)b * ly->v_stride[0] + (int64_t)h * ly->v_stride[1]) * ESZ;
    const bool ok = select_body<KC, true, MAXN, NT, false, STABLE, L0T>(
        ly, dt, order, algo, nrow, nullptr, sel, arrays, n_cap, cap, sc, wave_seg, nullptr, status,
        trow, pk, pv, NC * 16);
    if (!ok) return;  // flagged in *status; the row's output is left unwritten (the copier
                      // workgroup of a split row skips it too)
    __syncthreads();
  }
  with_dt<KC>(dt, [&](auto D) {
    gather_row<D.value, NC, NT, kSgNts>(ly, r, H, selects ? sel : nullptr,
                                      split_rows > 0 && selects ? PART_SELECTED : PART_ALL);
  });
}

// ---------------------------------------------------------------------------------------------
// h2o_attention heavy hitters: torch's CPU sums restated per output column
// ---------------------------------------------------------------------------------------------
// aten cascade_sum (SumKernel.cpp) adds the rows of one output column in one of two orders:
//   cascade (multi_row_sum): four accumulator levels; rows go one by one into level 0, and after
//     every 2^p rows (p = max(4, CeilLog2(n) / 4)) level j-1 is folded into level j while the row
//     counter's j-th p-bit digit is zero; result ((a0 + a1) + a2) + a3.
//   ilp4 (row_sum): four interleaved lanes (row i -> lane i % 4), each a cascade over n / 4 rows,
//     leftover rows into lane 0, then ((l0 + l1) + l2) + l3.
// Which columns take ilp4 depends on the loop calls the reference made (col_class).
__device__ __forceinline__ int ceil_log2_i(int x) { return x <= 2 ? 1 : 32 - __clz(x - 1); }

template <typename LD>
__device__ __forceinline__ float cascade_sum(const LD& ld, int n, int off, int mul) {
  const int lp = max(4, ceil_log2_i(n) / 4);
  const int step = 1 << lp, mask = step - 1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int i = 0;
  while (i + step <= n) {
    if (step == 16) {  // the common level size: loads first, then the dependent adds
      float x[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) x[t] = ld(off + (i + t) * mul);
#pragma unroll
      for (int t = 0; t < 16; ++t) a0 = a0 + x[t];
      i += 16;
    } else {
      for (int t = 0; t < step; ++t, ++i) a0 = a0 + ld(off + i * mul);
    }
    a1 = a1 + a0;
    a0 = 0.f;
    if ((i & (mask << lp)) == 0) {
      a2 = a2 + a1;
      a1 = 0.f;
      if ((i & (mask << (2 * lp))) == 0) {
        a3 = a3 + a2;
        a2 = 0.f;
      }
    }
  }
  for (; i < n; ++i) a0 = a0 + ld(off + i * mul);
  a0 = a0 + a1;
  a0 = a0 + a2;
  return a0 + a3;
}

template <typename LD>
__device__ __forceinline__ float ilp4_sum(const LD& ld, int n) {
  const int n4 = n >> 2;
  float p0 = cascade_sum(ld, n4, 0, 4);
  const float p1 = cascade_sum(ld, n4, 1, 4);
  const float p2 = cascade_sum(ld, n4, 2, 4);
  const float p3 = cascade_sum(ld, n4, 3, 4);
  for (int i = 4 * n4; i < n; ++i) p0 = p0 + ld(i);
  p0 = p0 + p1;
  p0 = p0 + p2;
  return p0 + p3;
}

// Does column j of `cols` take the ilp4 order?  The reference's loop calls cover the columns in
// chunks: one call [0, cols) (chunk == 0), or parallel_dim_reduction's thread chunks of `chunk`
// columns with bounds rounded down to `rnd` columns (128 bytes; the final end stays cols).  In a
// call of L columns the vectorised loop (L >= vec_min = one Vectorized<scalar_t>) sums whole
// groups of `group` columns (four Vectorized<float>) with the cascade and the rest with row_sum;
// a shorter call sums groups of four columns with the cascade and the rest with row_sum.
__device__ __forceinline__ bool col_ilp(int j, int cols, int chunk, int rnd, int group,
                                        int vec_min) {
  int s = 0, e = cols;
  if (chunk > 0) {
    const int T = (cols + chunk - 1) / chunk;  // threads that start below cols
    int t = j / chunk;
    while (t + 1 < T && ((t + 1) * chunk) / rnd * rnd <= j) ++t;
    s = (t * chunk) / rnd * rnd;
    e = t + 1 < T ? ((t + 1) * chunk) / rnd * rnd : cols;
  }
  const int L = e - s;
  const int g = L >= vec_min ? group : 4;
  return j - s >= L / g * g;
}

template <int DT>
__device__ __forceinline__ uint32_t store_bits(float f) {
  if constexpr (DT == KVC_F32)
    return f32_to_bits(f);
  else
    return bits16_dt<DT>(f);
}
template <int DT>
__device__ __forceinline__ void store_dt(void* base, int64_t i, float f) {
  if constexpr (DT == KVC_F32)
    reinterpret_cast<float*>(base)[i] = f;
  else
    reinterpret_cast<uint16_t*>(base)[i] = (uint16_t)bits16_dt<DT>(f);
}

struct AttnChunk {
  kvc_attn_layer_t l[kArgLayers];
};
struct HHChunk {
  kvc_hh_layer_t l[kArgLayers];
};
constexpr int kColThreads = 256;

// update_attention_scores (h2o_attention.py:100-151) for every layer of the chunk: grid
// (layer * batch * heads rows, column blocks); one thread per key column:
//   imp = dt(0 + sum_q attn[b,h,q,j])                     attn.sum(dim=2)           (:116)
//   acc_new = dt(base + imp), base = dt(acc_old*decay) for j < old_len, else 0  (:118-151)
// Reads of attn are coalesced across the block's columns (q rows of stride attn_stride[2]).
// ODT: dtype of acc_old.  ODT != DT (the carried accumulation and the new attention differ in
// dtype, every layer carried): base is rounded to ODT, and acc_new is fp32 -- torch's promotion
// of two different float dtypes through torch.cat / + (:129-151) -- holding fp32(base) + fp32(imp).
// V consecutive elements of dtype DT at element offset i of `base` as floats: one 16-B load when
// the span is whole and 16-B aligned, else element by element (n valid, the rest 0).
template <int DT, int V>
__device__ __forceinline__ void load_vec(const char* base, int64_t i, int n, float (&x)[V]) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  constexpr int PER = 16 / ESZ;  // elements per 16-B load
  const char* p = base + i * ESZ;
  if (n == V && V % PER == 0 && ((uintptr_t)p & 15u) == 0) {
#pragma unroll
    for (int c = 0; c < V / PER; ++c) {
      const uint4 w = reinterpret_cast<const uint4*>(p)[c];
      const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        if constexpr (DT == KVC_F32) x[c * PER + e] = bits_to_f32(u[e]);
        else if constexpr (DT == KVC_BF16)
          x[c * PER + e] = bf16_to_f32((u[e / 2] >> (16 * (e & 1))) & 0xFFFFu);
        else x[c * PER + e] = f16_to_f32((u[e / 2] >> (16 * (e & 1))) & 0xFFFFu);
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) x[e] = e < n ? load_dt<DT>(p, e) : 0.f;
  }
}

// The first n of V floats stored as dtype DT at element offset i of `base` (rounded as
// store_dt): 16-B stores when the span is whole and aligned.
template <int DT, int V>
__device__ __forceinline__ void store_vec(void* base, int64_t i, int n, const float (&x)[V]) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  char* p = static_cast<char*>(base) + i * ESZ;
  constexpr int PER = 16 / ESZ;  // elements per 16-B store
  if (n == V && V % PER == 0 && ((uintptr_t)p & 15u) == 0) {
#pragma unroll
    for (int c = 0; c < V / PER; ++c) {
      uint32_t u[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if constexpr (DT == KVC_F32) u[w] = f32_to_bits(x[c * PER + w]);
        else u[w] = store_bits<DT>(x[c * PER + 2 * w]) | (store_bits<DT>(x[c * PER + 2 * w + 1]) << 16);
      }
      *reinterpret_cast<uint4*>(p + c * 16) = make_uint4(u[0], u[1], u[2], u[3]);
    }
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e)
      if (e < n) store_dt<DT>(base, i + e, x[e]);
  }
}

// ODT: dtype of acc_old.  ODT != DT (the carried accumulation and the new attention differ in
// dtype, every layer carried): base is rounded to ODT, and acc_new is fp32 -- torch's promotion
// of two different float dtypes through torch.cat / + (:129-151) -- holding fp32(base) + fp32(imp).
// One thread per kAccCols consecutive key columns (16-B loads and stores where aligned): with one
// column per thread a 32-layer decode step's [32, 16 384] rows took 65 536 workgroups and the
// launch ~130 us, bound by workgroup turnover, not bytes.
constexpr int kAccCols = 8;
template <int DT, int ODT>
__global__ void __launch_bounds__(kColThreads)
    attn_accum_kernel(const AttnChunk T, int H, int BH, float decay, int group, int vec_min) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  constexpr int NDT = ODT == DT ? DT : KVC_F32;  // acc_new's dtype
  constexpr int V = kAccCols;
  const kvc_attn_layer_t* ly = T.l + blockIdx.x / BH;
  const int r = (int)(blockIdx.x % BH);
  const int j0 = ((int)blockIdx.y * kColThreads + (int)threadIdx.x) * V;
  const int k = ly->key_len;
  if (j0 >= k) return;
  const int n = min(V, k - j0);
  const int b = r / H, h = r - (r / H) * H;
  const char* a = static_cast<const char*>(ly->attn) +
                  ((int64_t)b * ly->attn_stride[0] + (int64_t)h * ly->attn_stride[1]) * ESZ;
  const int64_t qs = ly->attn_stride[2] * ESZ;
  const int q = ly->q_len;
  float s[V];
  if (q == 1) {  // no reduction: the elementwise out = 0 + x
    load_vec<DT, V>(a, j0, n, s);
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = 0.f + s[e];
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int j = j0 + e;
      if (e >= n) {
        s[e] = 0.f;
        continue;
      }
      const auto ld = [&](int i) { return load_dt<DT>(a + (int64_t)i * qs, j); };
      // the accumulating store adds to the zero-filled output
      s[e] = col_ilp(j, k, ly->col_chunk, 128 / ESZ, group, vec_min) ? 0.f + ilp4_sum(ld, q)
                                                                      : 0.f + cascade_sum(ld, q, 0, 1);
    }
  }
  float base[V];
  const int nold = min(n, ly->old_len - j0);  // carried columns of this thread (may be <= 0)
  if (nold > 0)
    load_vec<ODT, V>(static_cast<const char*>(ly->acc_old), (int64_t)r * ly->old_len + j0, nold,
                     base);
  float out[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const float bse = e < nold ? round_dt<ODT>(base[e] * decay) : 0.f;
    out[e] = bse + round_dt<DT>(s[e]);
  }
  store_vec<NDT, V>(ly->acc_new, (int64_t)r * k + j0, n, out);
}

// get_heavy_hitter_indices' head sum (h2o_attention.py:194-198) for every layer of the chunk:
// grid (layer * batch rows, column blocks); row l*batch + b of `sums` (dtype, row stride
// `stride`) receives dt(0 + sum_h acc[b, h, m0 + j]) for j < zone_len.
template <int DT>
__global__ void __launch_bounds__(kColThreads)
    head_sum_kernel(const HHChunk T, int H, int B, int group, int vec_min, char* sums,
                    int64_t stride) {
  constexpr int ESZ = DTypeTraits<DT>::esz;
  const int l = (int)(blockIdx.x / B), b = (int)(blockIdx.x % B);
  const kvc_hh_layer_t* ly = T.l + l;
  const int j = (int)blockIdx.y * kColThreads + (int)threadIdx.x;
  const int m = ly->zone_len;
  if (j >= m) return;
  const char* a = static_cast<const char*>(ly->acc) +
                  ((int64_t)b * H * ly->acc_len + ly->zone_start + j) * ESZ;
  const int64_t hs = (int64_t)ly->acc_len * ESZ;
  const auto ld = [&](int i) { return load_dt<DT>(a + (int64_t)i * hs, 0); };
  float s;
  if (H == 1)
    s = 0.f + ld(0);
  else if (col_ilp(j, m, ly->col_chunk, 128 / ESZ, group, vec_min))
    s = 0.f + ilp4_sum(ld, H);
  else
    s = 0.f + cascade_sum(ld, H, 0, 1);
  store_dt<DT>(sums + (int64_t)blockIdx.x * stride * ESZ, j, s);
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static inline int esize(int dtype) { return dtype == KVC_F32 ? 4 : 2; }
// Calls f(std::integral_constant<int, DT>) for the call's storage dtype (validated by plan_impl).
template <typename F>
static int with_dtype(int dtype, F&& f) {
#ifdef KVC_ISA_PROBE  // diagnostic compile for ISA inspection: bf16 instantiations only
  return dtype == KVC_BF16 ? f(std::integral_constant<int, KVC_BF16>()) : KVC_E_DTYPE;
#else
  if (dtype == KVC_BF16) return f(std::integral_constant<int, KVC_BF16>());
  if (dtype == KVC_F16) return f(std::integral_constant<int, KVC_F16>());
  return f(std::integral_constant<int, KVC_F32>());
#endif
}
static inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
// one row of the global selection scratch (SelArrays for n_cap positions), 256-B aligned rows
static inline size_t sel_scratch_row_bytes(int n_cap, int dtype) {
  if (n_cap > kZoneMaxGlobal) return round_up(sel_long_bytes(n_cap, esize(dtype)), 256);
  return round_up(sel_bytes(n_cap, esize(dtype), n_cap / 2 + 1), 256);
}

static int plan_impl(const kvc_params_t* p, kvc_layer_t* layers, int nl, kvc_plan_info_t* info,
                     bool fill) {
  if (!p || nl < 0 || (nl > 0 && !layers)) return KVC_E_ARG;
  if (p->dtype != KVC_BF16 && p->dtype != KVC_F16 && p->dtype != KVC_F32) return KVC_E_DTYPE;
  if (p->batch < 1 || p->heads < 1 || p->head_dim < 1) return KVC_E_ARG;
  if (p->order != KVC_ASC && p->order != KVC_DESC) return KVC_E_ARG;
  if (p->algo != KVC_ALGO_SORT && p->algo != KVC_ALGO_TOPK && p->algo != KVC_ALGO_STABLE)
    return KVC_E_ARG;
  if ((p->flags & ~(KVC_FLAG_SPLIT_SELECT_GATHER | KVC_FLAG_SHARED_INDEX | KVC_FLAG_GATHER_FIXED |
                    KVC_FLAG_GATHER_SELECTED)) || p->reserved != 0)
    return KVC_E_ARG;  // unknown flag bits / reserved field: refuse rather than ignore
  if ((p->flags & KVC_FLAG_GATHER_FIXED) && (p->flags & KVC_FLAG_GATHER_SELECTED))
    return KVC_E_ARG;
  if ((p->flags & KVC_FLAG_SHARED_INDEX) && !p->external_index) return KVC_E_ARG;
  // the two gather parts of one call share its index region: with the engine's own selection
  // each launch would also SCORE and SELECT into the same workspace (a race when the two run
  // concurrently, as the flags intend) -- so only external indices may be split
  if ((p->flags & (KVC_FLAG_GATHER_FIXED | KVC_FLAG_GATHER_SELECTED)) && !p->external_index)
    return KVC_E_ARG;
  const int es = esize(p->dtype);
  const int rowb = p->head_dim * es;
  if (rowb % 16) return KVC_E_HEADDIM;
  const int nc = rowb / 16;
  // 64..1024-byte rows: every pythia geometry (D 32/64/80/128/256) in bf16, fp16 and fp32
  if (nc != 4 && nc != 8 && nc != 10 && nc != 16 && nc != 20 && nc != 32 && nc != 64)
    return KVC_E_HEADDIM;
  const int64_t BH = (int64_t)p->batch * p->heads;
  if (BH * nl > 0x7FFFFFFF) return KVC_E_ARG;
  int64_t tiles = 0, units = 0, max_zone = 0, max_sel = 0;
  bool snap = false;  // a snapkv row is scored: the per-tile maxima region
  for (int l = 0; l < nl; ++l) {
    kvc_layer_t& y = layers[l];
    const int S = y.seq_len;
    if (S < 0 || y.zone_start < 0 || y.zone_len < 0 || (int64_t)y.zone_start + y.zone_len > S ||
        y.n_select < 0 || y.n_select > y.zone_len || y.sink_len < 0 || y.sink_len > S ||
        y.tail_start < 0 || y.tail_len < 0 || (int64_t)y.tail_start + y.tail_len > S ||
        (y.score_mode != KVC_SCORE_NORM && y.score_mode != KVC_SCORE_SNAPKV))
      return KVC_E_ARG;
    const int64_t n_out = (int64_t)y.sink_len + y.n_select + y.tail_len;
    if (n_out > 0x7FFFFFFF || 2 * BH * n_out * nc > 0x7FFFFFFF) return KVC_E_ARG;
    const bool needs_select = y.n_select > 0 && y.n_select < y.zone_len;
    if (needs_select && y.zone_len > kZoneMaxLong) return KVC_E_TOO_LONG;
    // stable selections: LDS, or the u16-position global scratch (not the u32 long variant)
    if (needs_select && p->algo == KVC_ALGO_STABLE && !p->external_index &&
        y.zone_len > kZoneMaxGlobal)
      return KVC_E_TOO_LONG;
    if (n_out > 0) {
      if (!y.k || !y.v || !y.k_out || !y.v_out) return KVC_E_ARG;
      if (!aligned16(y.k) || !aligned16(y.v) || !aligned16(y.k_out) || !aligned16(y.v_out))
        return KVC_E_ALIGN;
      const int64_t* ks = y.k_stride;
      const int64_t* vs = y.v_stride;
      if ((p->batch > 1 && ((ks[0] * es) % 16 || (vs[0] * es) % 16)) ||
          (p->heads > 1 && ((ks[1] * es) % 16 || (vs[1] * es) % 16)) ||
          (S > 1 && ((ks[2] * es) % 16 || (vs[2] * es) % 16)))
        return KVC_E_ALIGN;
    }
    const int64_t tl = needs_select ? BH * ((y.zone_len + kTile - 1) / kTile) : 0;
    const int64_t ul = 2 * BH * n_out * nc;
    if (fill) {
      y.n_out = (int32_t)n_out;
      y.row0 = (int32_t)(l * BH);
      y.tile0 = (int32_t)tiles;
      y.unit0 = units;
    } else if (y.n_out != n_out || y.row0 != l * BH || y.tile0 != tiles || y.unit0 != units) {
      return KVC_E_ARG;
    }
    if (needs_select && y.zone_len > max_zone) max_zone = y.zone_len;
    snap |= needs_select && y.score_mode == KVC_SCORE_SNAPKV;
    if (y.n_select > max_sel) max_sel = y.n_select;
    tiles += tl;
    units += ul;
    if (tiles > 0x7FFFFFFF) return KVC_E_ARG;
  }
  if (info) {
    const int64_t rows = BH * nl;
    info->rows = rows;
    info->score_tiles = tiles;
    info->gather_units = units;
    info->norm_row_stride = (int64_t)round_up((size_t)max_zone, kTile);
    info->index_row_stride = (int64_t)round_up((size_t)(max_sel > 0 ? max_sel : 1), 16);
    size_t off = 0;
    info->norm_offset = off;
    off = round_up(off + (size_t)rows * info->norm_row_stride * es, 256);
    info->index_offset = off;
    off = round_up(off + (size_t)rows * info->index_row_stride * 4, 256);
    if (max_zone > kZoneMax)  // selection scratch rows for zones longer than the LDS limit
      off += (size_t)rows * sel_scratch_row_bytes((int)info->norm_row_stride, p->dtype);
    // SCORE's per-64-token-tile statistics (u32 each; tmax_offset()): the norm maximum of a
    // snapkv row's tile; for a plain-norm row, level 0's ge / le counts in the KVC_L0_TILE_COUNTS
    // build (reserved either way: the layout does not depend on the build option)
    if (snap || max_zone > 0)
      off += (size_t)rows * (size_t)(info->norm_row_stride / kTile) * 4;
#ifdef KVC_STAMPS
    off += (size_t)rows * 256;  // diagnostic stamp slots (32 x u64 per select row)
#endif
    info->workspace_bytes = off;
  }
  return KVC_OK;
}

// Offset of the snapkv per-tile maxima region (rows x norm_row_stride / 64 u32): after the index
// region and the long-zone selection scratch (plan_impl's layout).
static inline size_t tmax_offset(const kvc_plan_info_t& info, int dtype) {
  size_t off = round_up(info.index_offset + (size_t)info.rows * info.index_row_stride * 4, 256);
  if (info.norm_row_stride > kZoneMax)
    off += (size_t)info.rows * sel_scratch_row_bytes((int)info.norm_row_stride, dtype);
  return off;
}

// Every launch goes through hipLaunchKernel, whose return value is this launch's own status (a
// caller's pending HIP error is neither consumed nor reported as ours).
template <typename... P, typename... A>
static int launch_k(void (*kern)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t s,
                    A&&... a) {
  std::tuple<P...> args(std::forward<A>(a)...);
  void* ptrs[sizeof...(P)];
  std::apply([&](auto&... x) {
    int i = 0;
    ((ptrs[i++] = static_cast<void*>(&x)), ...);
  }, args);
  return hipLaunchKernel(reinterpret_cast<const void*>(kern), grid, block, ptrs, lds, s) ==
                 hipSuccess
             ? KVC_OK
             : KVC_E_HIP;
}

// Calls f(std::integral_constant<int, NC>()) for a row width in 16-B chunks (validated by
// plan_impl: 64..1024-byte rows).
template <typename F>
static int with_nc(int nc, F&& f) {
#ifdef KVC_ISA_PROBE  // D = 128 bf16 rows only
  return nc == 16 ? f(std::integral_constant<int, 16>()) : KVC_E_HEADDIM;
#else
  switch (nc) {
    case 4: return f(std::integral_constant<int, 4>());
    case 8: return f(std::integral_constant<int, 8>());
    case 10: return f(std::integral_constant<int, 10>());
    case 16: return f(std::integral_constant<int, 16>());
    case 20: return f(std::integral_constant<int, 20>());
    case 32: return f(std::integral_constant<int, 32>());
    case 64: return f(std::integral_constant<int, 64>());
    default: return KVC_E_HEADDIM;
  }
#endif
}

// Keys are read once (non-temporal loads) and outputs written once (non-temporal stores): they
// would otherwise evict useful lines from the Infinity Cache.
template <int DT, int NC>
static int launch_score(const LayerChunk& T, int nl, int H, int64_t tile_base,
                        int64_t chunk_tiles, char* norms, int64_t nstride, uint32_t* tmax,
                        hipStream_t s) {
  constexpr int per_wg = score_waves(NC);  // one tile per wave
  const unsigned grid = (unsigned)((chunk_tiles + per_wg - 1) / per_wg);
  return launch_k(score_kernel<DT, NC, true>, dim3(grid), dim3(per_wg * 64), 0, s, T, nl, H,
                  tile_base, chunk_tiles, norms, nstride, tmax, nstride / kTile);
}

// `work` = max n_out over the chunk's layers; grid = (rows, token blocks)
// KVC_FLAG_GATHER_FIXED launches (copies meant to run beside a selection on another stream) use
// at most this many workgroups: two of four waves per CU
// (A/B: an uncapped grid starves the heap select beside it -- the S = 16 384 h2o_attention call
// 0.155 -> 0.216 ms, 1 024 blocks 0.208; tools/ab_variants.txt fgfull / fg1024)
#ifndef KVC_FIXED_GATHER_BLOCKS
#define KVC_FIXED_GATHER_BLOCKS 512
#endif
constexpr int kFixedGatherBlocks = KVC_FIXED_GATHER_BLOCKS;
template <int DT, int NC>
static int launch_gather(const LayerChunk& T, int nl, int H, int BH, const int32_t* idx,
                         int64_t istride, int shared, uint32_t* status, int64_t work, int part,
                         hipStream_t s) {
  const int rows = nl * BH, nby = (int)((work + kGatherTokens - 1) / kGatherTokens);
  if (part == PART_FIXED && (int64_t)rows * nby > kFixedGatherBlocks)
    return launch_k(gather_kernel<DT, NC, true>, dim3(kFixedGatherBlocks), dim3(kGatherThreads), 0,
                    s, T, H, BH, idx, istride, shared, status, part, rows, nby);
  return launch_k(gather_kernel<DT, NC, true>, dim3((unsigned)rows, (unsigned)nby),
                  dim3(kGatherThreads), 0, s, T, H, BH, idx, istride, shared, status, part, 0, nby);
}

// SELECT over the rows of a chunk (BH rows per layer, workspace row ly->row0 + blockIdx % BH):
// the LDS kernels (512-thread rows for zones up to kSmallZone, else 1 024-thread rows) or, for
// zones longer than kZoneMax, the global-scratch kernels (u32 positions beyond kZoneMaxGlobal).
template <int KC, bool HH = false>
static int launch_select(const LayerChunk& T, int cn, int BH, int dt, int order, int algo,
                         const char* norms, int64_t nstride, int32_t* idx, int64_t istride,
                         bool long_zone, char* scratch, uint64_t* stamps, uint32_t* status,
                         hipStream_t s, const uint32_t* tmax = nullptr) {
  typedef typename DTypeTraits<KC>::key_t KeyT;
  const dim3 rows_grid((unsigned)(cn * BH));
  const int n_cap = (int)nstride;  // longest zone of the call, rounded to 64
  if (long_zone) {
    const int64_t rb = (int64_t)sel_scratch_row_bytes(n_cap, KC);
    if (n_cap > kZoneMaxGlobal)  // u32 positions (the call's longest zone decides)
      return launch_k(select_long_kernel<KC>, rows_grid, dim3(kSelThreads), 0, s, T, BH, dt,
                      order, algo, norms, nstride, idx, istride, scratch, rb, n_cap, status);
    if (algo == KVC_ALGO_STABLE)
      return launch_k(select_global_kernel<KC, true>, rows_grid, dim3(kSelThreads), 0, s, T, BH,
                      dt, order, algo, norms, nstride, idx, istride, kWaveSeg, scratch, rb, n_cap,
                      status);
    return launch_k(select_global_kernel<KC>, rows_grid, dim3(kSelThreads), 0, s, T, BH, dt,
                    order, algo, norms, nstride, idx, istride, kWaveSeg, scratch, rb, n_cap,
                    status);
  }
  const int ks = (int)sizeof(KeyT);
  const auto go = [&](auto stable) {
    constexpr bool ST = decltype(stable)::value;
    if (n_cap <= kSmallZone) {
      const int cap = sel_cap(n_cap, ks, kSmallBudget);
      return launch_k(select_kernel<KC, kSelThreadsSmall, HH, ST>, rows_grid,
                      dim3(kSelThreadsSmall), sel_bytes(n_cap, ks, cap), s, T, BH, dt, order, algo,
                      norms, nstride, idx, istride, kWaveSegSmall, n_cap, cap, stamps, status,
                      tmax);
    }
    return launch_k(select_kernel<KC, kSelThreads, HH, ST>, rows_grid, dim3(kSelThreads), 0, s, T,
                    BH, dt, order, algo, norms, nstride, idx, istride, kWaveSeg, n_cap, 0, stamps,
                    status, tmax);
  };
  if (algo == KVC_ALGO_STABLE) return go(std::true_type());
  return go(std::false_type());
}

// One chunk of <= kArgLayers layers: SCORE, then SELECT_GATHER (or SELECT and GATHER as two
// kernels with KVC_FLAG_SPLIT_SELECT_GATHER, or GATHER alone for copy-only / external-index
// calls), each kernel with the chunk's table by value.
template <int DT, int NC>
static int launch_chunk(const kvc_params_t* p, const kvc_plan_info_t& info, const kvc_layer_t* layers,
                        int nl, int c0, int cn, char* w, hipStream_t s) {
  typedef typename DTypeTraits<DT>::key_t KeyT;
  constexpr int KC = DT == KVC_F32 ? KVC_F32 : KVC_BF16;  // selection binary: the key class
  const int H = p->heads, BH = p->batch * p->heads;
  char* norms = w + info.norm_offset;
  int32_t* idx = reinterpret_cast<int32_t*>(w + info.index_offset);
  const int64_t nstride = info.norm_row_stride, istride = info.index_row_stride;
#ifdef KVC_STAMPS
  uint64_t* stamps = reinterpret_cast<uint64_t*>(w + info.workspace_bytes - info.rows * 256);
#else
  uint64_t* stamps = nullptr;
#endif
  LayerChunk T;
  memcpy(T.l, layers + c0, (size_t)cn * sizeof(kvc_layer_t));
  const int64_t tile_base = layers[c0].tile0;
  const int64_t tile_end = c0 + cn < nl ? (int64_t)layers[c0 + cn].tile0 : info.score_tiles;
  const int part = (p->flags & KVC_FLAG_GATHER_FIXED)      ? PART_FIXED
                   : (p->flags & KVC_FLAG_GATHER_SELECTED) ? PART_SELECTED
                                                           : PART_ALL;
  bool sel = false, long_zone = false, snap = false;
  int64_t max_out = 0, max_part = 0;
  for (int l = c0; l < c0 + cn; ++l) {
    sel |= layers[l].n_select > 0;
    snap |= layer_selects(layers[l]) && layers[l].score_mode == KVC_SCORE_SNAPKV;
    long_zone |= layer_selects(layers[l]) && layers[l].zone_len > kZoneMax;
    max_out = layers[l].n_out > max_out ? layers[l].n_out : max_out;
    const int64_t pr = part_rows(layers[l], part);
    max_part = pr > max_part ? pr : max_part;
  }
  const bool ext = p->external_index != 0;
  uint32_t* status = p->device_status;
  // snapkv rows: SCORE's per-tile norm maxima (plan_impl reserved them), read by the selection
  uint32_t* tmax = (snap || (kL0TileCounts && info.norm_row_stride > 0)) && !ext
                       ? reinterpret_cast<uint32_t*>(w + tmax_offset(info, p->dtype))
                       : nullptr;
  uint32_t* tmax_sel = tmax;  // snapkv rows read their maxima, plain rows their level-0 counts
  int rc = KVC_OK;
  if ((p->phases & KVC_PHASE_SCORE) && tile_end > tile_base && !ext)
    rc = launch_score<DT, NC>(T, cn, H, tile_base, tile_end - tile_base, norms, nstride, tmax, s);
  if (rc != KVC_OK) return rc;
  const int n_cap = (int)nstride;  // longest zone of the call, rounded to 64
  if ((p->phases & KVC_PHASE_SELECT) && sel && !ext) {
    const bool fuse_sg = (p->phases & KVC_PHASE_GATHER) && max_out > 0 && !stamps &&
                         !long_zone && part == PART_ALL &&
                         !(p->flags & KVC_FLAG_SPLIT_SELECT_GATHER);
    if (fuse_sg) {  // this chunk's gather happens inside the select kernel
      const int rows = cn * BH;
      const dim3 rows_grid((unsigned)rows);
      const int ks = (int)sizeof(KeyT);
      const auto go = [&](auto stable) {
        constexpr bool ST = decltype(stable)::value;
        if (n_cap <= kSmallZone) {
          const int cap = sel_cap(n_cap, ks, kSmallBudget);
          return launch_k(select_gather_kernel<KC, kSelThreadsSmall, NC, ST>, rows_grid,
                          dim3(kSelThreadsSmall), sel_bytes(n_cap, ks, cap), s, T, H, BH, DT,
                          p->order, p->algo, norms, nstride, kWaveSegSmall, n_cap, cap, status, 0,
                          tmax_sel);
        }
        // fewer rows than CUs (e.g. 4 layers per GPU of an 8-way layer split): one row per CU
        // and idle CUs -- the sink / tail rows get copy-only workgroups of their own
        bool fixed = false, plain = false;
        for (int l = c0; l < c0 + cn; ++l) {
          fixed |= layer_selects(layers[l]) && layers[l].sink_len + layers[l].tail_len > 0;
          plain |= layer_selects(layers[l]) && layers[l].score_mode == KVC_SCORE_NORM;
        }
        const int split = fixed && rows <= kSplitCopyRows ? rows : 0;
        const dim3 grid((unsigned)(split ? 2 * rows : rows));
        // Level 0's idx-region rank tables (run_chain) pay on launches with plain-norm rows;
        // snapkv-only launches run faster in the instance without that code
        // (profiles/r06_h_l0t_instance_ab.jsonl: headline snapkv 0.1770 -> 0.1715 ms; with one
        // row per CU the tables still win for cfg4 ranks, 0.0467 -> 0.0427, and lose 2 us for
        // cfg5 pyramid ones)
        if constexpr (!ST) {
          if (plain)
            return launch_k(select_gather_kernel<KC, kSelThreads, NC, ST, true>, grid,
                            dim3(kSelThreads), 0, s, T, H, BH, DT, p->order, p->algo, norms,
                            nstride, kWaveSeg, n_cap, 0, status, split, tmax_sel);
        }
        return launch_k(select_gather_kernel<KC, kSelThreads, NC, ST, false>, grid,
                        dim3(kSelThreads), 0, s, T, H, BH, DT, p->order, p->algo, norms, nstride,
                        kWaveSeg, n_cap, 0, status, split, tmax_sel);
      };
      return p->algo == KVC_ALGO_STABLE ? go(std::true_type()) : go(std::false_type());
    }
    char* scratch = w + round_up(info.index_offset + (size_t)info.rows * istride * 4, 256);
    uint64_t* st = stamps ? stamps + (size_t)layers[c0].row0 * 32 : nullptr;
    rc = launch_select<KC>(T, cn, BH, DT, p->order, p->algo, norms, nstride, idx, istride,
                           long_zone, scratch, st, status, s, tmax_sel);
  }
  if (rc != KVC_OK) return rc;
  if ((p->phases & KVC_PHASE_GATHER) && max_part > 0)
    rc = launch_gather<DT, NC>(T, cn, H, BH, idx, istride,
                               (p->flags & KVC_FLAG_SHARED_INDEX) ? 1 : 0, status, max_part, part,
                               s);
  return rc;
}

// kvc_debug_select_capacity: the 512-thread SELECT / SELECT_GATHER kernels of one chunk with a
// caller-chosen zone capacity (the device-side bounds check's test hook)
static int debug_select_impl(const kvc_params_t* p, const kvc_layer_t* layers, int nl, char* w,
                             size_t wbytes, int zone_cap, hipStream_t s) {
  kvc_plan_info_t info;
  int rc = plan_impl(p, const_cast<kvc_layer_t*>(layers), nl, &info, false);
  if (rc != KVC_OK) return rc;
  if (nl < 1 || nl > kArgLayers || zone_cap < kTile || zone_cap > kSmallZone ||
      zone_cap % kTile || p->external_index || p->algo == KVC_ALGO_STABLE ||
      (p->phases != KVC_PHASE_SELECT && p->phases != (KVC_PHASE_SELECT | KVC_PHASE_GATHER)))
    return KVC_E_ARG;
  if (!w || wbytes < info.workspace_bytes) return KVC_E_WORKSPACE;
  LayerChunk T;
  memcpy(T.l, layers, (size_t)nl * sizeof(kvc_layer_t));
  const int H = p->heads, BH = p->batch * p->heads;
  const char* norms = w + info.norm_offset;
  int32_t* idx = reinterpret_cast<int32_t*>(w + info.index_offset);
  const dim3 grid((unsigned)(nl * BH));
  const int nc = p->head_dim * esize(p->dtype) / 16;
  return with_dtype(p->dtype, [&](auto dt) {
    constexpr int DT = decltype(dt)::value;
    constexpr int KC = DT == KVC_F32 ? KVC_F32 : KVC_BF16;
    const int ks = (int)sizeof(typename DTypeTraits<KC>::key_t);
    const int cap = sel_cap(zone_cap, ks, kSmallBudget);
    const size_t lds = sel_bytes(zone_cap, ks, cap);
    if (p->phases == KVC_PHASE_SELECT)
      return launch_k(select_kernel<KC, kSelThreadsSmall>, grid, dim3(kSelThreadsSmall), lds, s,
                      T, BH, DT, p->order, p->algo, norms, info.norm_row_stride, idx,
                      info.index_row_stride, kWaveSegSmall, zone_cap, cap,
                      static_cast<uint64_t*>(nullptr), p->device_status,
                      static_cast<const uint32_t*>(nullptr));
    return with_nc(nc, [&](auto ncv) {
      return launch_k(select_gather_kernel<KC, kSelThreadsSmall, decltype(ncv)::value>, grid,
                      dim3(kSelThreadsSmall), lds, s, T, H, BH, DT, p->order, p->algo, norms,
                      info.norm_row_stride, kWaveSegSmall, zone_cap, cap, p->device_status, 0,
                      static_cast<const uint32_t*>(nullptr));
    });
  });
}

// ---- h2o_attention host side ----------------------------------------------------------------
static int attn_params_check(const kvc_attn_params_t* p, bool accumulate = false) {
  if (!p) return KVC_E_ARG;
  if (p->dtype != KVC_BF16 && p->dtype != KVC_F16 && p->dtype != KVC_F32) return KVC_E_DTYPE;
  if (p->batch < 1 || p->heads < 1) return KVC_E_ARG;
  // flags: kvc_attn_accumulate's KVC_ATTN_OLD_DTYPE(d) only (d a dtype other than p->dtype)
  // flags: KVC_ATTN_HH_STABLE (both entry points: one params struct serves a decode step's
  // accumulate and heavy-hitter calls) | kvc_attn_accumulate's KVC_ATTN_OLD_DTYPE(d), bits 0-1,
  // d a dtype other than p->dtype
  const int od = p->flags & 3;
  if ((p->flags & ~(3 | KVC_ATTN_HH_STABLE)) || (od && (!accumulate || od == KVC_ATTN_OLD_DTYPE(p->dtype))))
    return KVC_E_ARG;
  if (p->vec_bytes < 16 || p->vec_bytes > 64 || p->vec_bytes % 16) return KVC_E_ARG;
  if ((int64_t)p->batch * p->heads > 0x7FFFFFFF / kArgLayers) return KVC_E_ARG;
  return KVC_OK;
}

static int accumulate_impl(const kvc_attn_params_t* p, const kvc_attn_layer_t* layers, int nl,
                           hipStream_t s) {
  int rc = attn_params_check(p, true);
  if (rc != KVC_OK) return rc;
  if (nl < 0 || (nl > 0 && !layers)) return KVC_E_ARG;
  const int es = esize(p->dtype);
  const int od = p->flags & 3;                 // KVC_ATTN_OLD_DTYPE bits
  const int odt = od ? od - 1 : p->dtype;      // acc_old's dtype
  const int oes = esize(odt), nes = od ? 4 : es;
  for (int l = 0; l < nl; ++l) {
    const kvc_attn_layer_t& y = layers[l];
    if (!y.attn || !y.acc_new || y.q_len < 1 || y.key_len < 1 || y.old_len < 0 ||
        y.old_len > y.key_len || (y.old_len > 0 && !y.acc_old) || y.col_chunk < 0 ||
        (od && y.old_len == 0) || (uintptr_t)y.attn % es ||
        (uintptr_t)y.acc_new % nes || (uintptr_t)y.acc_old % oes)
      return KVC_E_ARG;
    if ((y.key_len + kColThreads * kAccCols - 1) / (kColThreads * kAccCols) > 65535)
      return KVC_E_TOO_LONG;
  }
  const int H = p->heads, BH = p->batch * p->heads;
  const int group = 4 * (p->vec_bytes / 4), vec_min = p->vec_bytes / es;
  for (int c0 = 0; c0 < nl && rc == KVC_OK; c0 += kArgLayers) {
    const int cn = nl - c0 < kArgLayers ? nl - c0 : kArgLayers;
    AttnChunk T;
    memcpy(T.l, layers + c0, (size_t)cn * sizeof(kvc_attn_layer_t));
    int kmax = 0;
    for (int l = 0; l < cn; ++l) kmax = T.l[l].key_len > kmax ? T.l[l].key_len : kmax;
    const int cols = kColThreads * kAccCols;
    const dim3 grid((unsigned)(cn * BH), (unsigned)((kmax + cols - 1) / cols));
    rc = with_dtype(p->dtype, [&](auto dt) {
      return with_dtype(odt, [&](auto od) {
        return launch_k(attn_accum_kernel<decltype(dt)::value, decltype(od)::value>, grid,
                        dim3(kColThreads), 0, s, T, H, BH, p->decay, group, vec_min);
      });
    });
  }
  return rc;
}

// Workspace of kvc_heavy_hitters: head-summed rows [layers * batch, nstride] of dtype, then the
// global selection scratch rows when a zone is longer than kZoneMax.
static int hh_layout(const kvc_attn_params_t* p, const kvc_hh_layer_t* layers, int nl,
                     int64_t* nstride, size_t* sums_bytes, size_t* total) {
  int rc = attn_params_check(p);
  if (rc != KVC_OK) return rc;
  if (nl < 0 || (nl > 0 && !layers)) return KVC_E_ARG;
  int64_t mmax = 1;
  for (int l = 0; l < nl; ++l) {
    const kvc_hh_layer_t& y = layers[l];
    if (!y.acc || y.acc_len < 1 || y.zone_start < 0 || y.zone_len < 1 ||
        (int64_t)y.zone_start + y.zone_len > y.acc_len || y.n_select < 0 ||
        y.n_select > y.zone_len || y.col_chunk < 0 || y.reserved != 0 ||
        (uintptr_t)y.acc % esize(p->dtype))
      return KVC_E_ARG;
    if (y.zone_len > kZoneMaxLong) return KVC_E_TOO_LONG;
    if ((p->flags & KVC_ATTN_HH_STABLE) && y.n_select < y.zone_len && y.zone_len > kZoneMaxGlobal)
      return KVC_E_TOO_LONG;  // the stable selection's longest zone, as kvc_plan
    mmax = y.zone_len > mmax ? y.zone_len : mmax;
  }
  const int64_t rows = (int64_t)nl * p->batch;
  *nstride = (int64_t)round_up((size_t)mmax, kTile);
  *sums_bytes = round_up((size_t)rows * *nstride * esize(p->dtype), 256);
  *total = *sums_bytes;
  if (mmax > kZoneMax) *total += (size_t)rows * sel_scratch_row_bytes((int)*nstride, p->dtype);
  return KVC_OK;
}

static int heavy_hitters_impl(const kvc_attn_params_t* p, const kvc_hh_layer_t* layers, int nl,
                              int32_t* out, int64_t ostride, char* w, size_t wbytes,
                              hipStream_t s) {
  int64_t nstride;
  size_t sums_bytes, total;
  int rc = hh_layout(p, layers, nl, &nstride, &sums_bytes, &total);
  if (rc != KVC_OK) return rc;
  if (nl == 0) return KVC_OK;
  if (!w || wbytes < total) return KVC_E_WORKSPACE;
  if (!out) return KVC_E_ARG;
  for (int l = 0; l < nl; ++l)
    if (layers[l].n_select > ostride) return KVC_E_ARG;
  const int B = p->batch, H = p->heads, es = esize(p->dtype);
  const int group = 4 * (p->vec_bytes / 4), vec_min = p->vec_bytes / es;
  for (int c0 = 0; c0 < nl && rc == KVC_OK; c0 += kArgLayers) {
    const int cn = nl - c0 < kArgLayers ? nl - c0 : kArgLayers;
    HHChunk T;
    memcpy(T.l, layers + c0, (size_t)cn * sizeof(kvc_hh_layer_t));
    LayerChunk S;  // the selection rows: zone = the head-summed row, chunk-local row0
    memset(&S, 0, sizeof(S));
    int mmax = 0;
    bool long_zone = false;
    for (int l = 0; l < cn; ++l) {
      S.l[l].zone_len = T.l[l].zone_len;
      S.l[l].n_select = T.l[l].n_select;
      S.l[l].seq_len = T.l[l].zone_len;
      S.l[l].score_mode = KVC_SCORE_NORM;
      S.l[l].row0 = l * B;
      mmax = T.l[l].zone_len > mmax ? T.l[l].zone_len : mmax;
      long_zone |= T.l[l].zone_len > kZoneMax;
    }
    char* sums = w + (size_t)c0 * B * nstride * es;
    char* scratch = w + sums_bytes + (size_t)c0 * B * sel_scratch_row_bytes((int)nstride, p->dtype);
    int32_t* o = out + (int64_t)c0 * B * ostride;
    const dim3 grid((unsigned)(cn * B), (unsigned)((mmax + kColThreads - 1) / kColThreads));
    rc = with_dtype(p->dtype, [&](auto dt) {
      constexpr int DT = decltype(dt)::value;
      constexpr int KC = DT == KVC_F32 ? KVC_F32 : KVC_BF16;
      int r = launch_k(head_sum_kernel<DT>, grid, dim3(kColThreads), 0, s, T, H, B, group,
                       vec_min, sums, nstride);
      if (r != KVC_OK) return r;
      // torch.topk(largest=True) + torch.sort: the descending TOPK selection, ascending indices
      const int algo = (p->flags & KVC_ATTN_HH_STABLE) ? KVC_ALGO_STABLE : KVC_ALGO_TOPK;
      return launch_select<KC, true>(S, cn, B, DT, KVC_DESC, algo, sums, nstride, o, ostride,
                               long_zone, scratch, nullptr, p->device_status, s);
    });
  }
  return rc;
}

}  // namespace kvc

extern "C" {

int kvc_version(void) { return KVC_ABI_VERSION; }
size_t kvc_layer_struct_size(void) { return sizeof(kvc_layer_t); }
int kvc_max_zone_len(void) { return kvc::kZoneMaxLong; }

#ifndef KVC_SOURCE_DIGEST
#define KVC_SOURCE_DIGEST "unknown"
#endif
const char* kvc_source_digest(void) { return KVC_SOURCE_DIGEST; }

const char* kvc_status_string(int s) {
  switch (s) {
    case KVC_OK: return "ok";
    case KVC_E_ARG: return "invalid argument";
    case KVC_E_DTYPE: return "unsupported dtype (bf16/fp16/fp32 only)";
    case KVC_E_HEADDIM: return "unsupported head_dim";
    case KVC_E_ALIGN: return "pointer or stride not 16-byte aligned";
    case KVC_E_TOO_LONG: return "scored zone longer than kvc_max_zone_len()";
    case KVC_E_WORKSPACE: return "workspace too small";
    case KVC_E_HIP: return "HIP launch failure";
    default: return "unknown status";
  }
}

int kvc_plan(const kvc_params_t* params, kvc_layer_t* layers, int num_layers,
             kvc_plan_info_t* info) {
  return kvc::plan_impl(params, layers, num_layers, info, true);
}

int kvc_launch(const kvc_params_t* p, const kvc_layer_t* layers, int nl, void* ws,
               size_t ws_bytes, kvc_stream_t stream) {
  using namespace kvc;
  kvc_plan_info_t info;
  int rc = plan_impl(p, const_cast<kvc_layer_t*>(layers), nl, &info, false);
  if (rc != KVC_OK) return rc;
  if (nl == 0) return KVC_OK;
  if (!ws || ws_bytes < info.workspace_bytes) return KVC_E_WORKSPACE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(ws);
  const int nc = p->head_dim * esize(p->dtype) / 16;
  for (int c0 = 0; c0 < nl && rc == KVC_OK; c0 += kArgLayers) {
    const int cn = nl - c0 < kArgLayers ? nl - c0 : kArgLayers;
    rc = with_dtype(p->dtype, [&](auto dt) {
      return with_nc(nc, [&](auto ncv) {
        return launch_chunk<decltype(dt)::value, decltype(ncv)::value>(p, info, layers, nl, c0,
                                                                       cn, w, s);
      });
    });
  }
  return rc;
}

int kvc_compress(const kvc_params_t* params, kvc_layer_t* layers, int num_layers, void* ws,
                 size_t ws_bytes, kvc_stream_t stream) {
  kvc_plan_info_t info;
  const int rc = kvc::plan_impl(params, layers, num_layers, &info, true);
  if (rc != KVC_OK) return rc;
  return kvc_launch(params, layers, num_layers, ws, ws_bytes, stream);
}

int kvc_debug_select_capacity(const kvc_params_t* params, const kvc_layer_t* layers,
                              int num_layers, void* workspace, size_t workspace_bytes,
                              int zone_cap, kvc_stream_t stream) {
  return kvc::debug_select_impl(params, layers, num_layers, static_cast<char*>(workspace),
                                workspace_bytes, zone_cap, reinterpret_cast<hipStream_t>(stream));
}

int kvc_attn_accumulate(const kvc_attn_params_t* params, const kvc_attn_layer_t* layers,
                        int num_layers, kvc_stream_t stream) {
  return kvc::accumulate_impl(params, layers, num_layers, reinterpret_cast<hipStream_t>(stream));
}

int kvc_hh_workspace(const kvc_attn_params_t* params, const kvc_hh_layer_t* layers,
                     int num_layers, size_t* bytes) {
  int64_t nstride;
  size_t sums, total;
  if (!bytes) return KVC_E_ARG;
  const int rc = kvc::hh_layout(params, layers, num_layers, &nstride, &sums, &total);
  if (rc == KVC_OK) *bytes = total;
  return rc;
}

int kvc_heavy_hitters(const kvc_attn_params_t* params, const kvc_hh_layer_t* layers,
                      int num_layers, int32_t* out_idx, int64_t out_row_stride, void* workspace,
                      size_t workspace_bytes, kvc_stream_t stream) {
  return kvc::heavy_hitters_impl(params, layers, num_layers, out_idx, out_row_stride,
                                 static_cast<char*>(workspace), workspace_bytes,
                                 reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
