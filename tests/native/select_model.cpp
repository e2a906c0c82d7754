// Host model of the select kernel's algorithm (test infrastructure): the same chain of Hoare
// partitions from rank lists that select_kernel computes in parallel, executed serially, with the
// serial steps taken from the kernel's own header (csrc/kvc_serial.h, __host__ __device__).
// tests/test_select_model.py checks it against real libstdc++ std::sort / std::nth_element /
// std::partial_sort, including adversarial inputs that force the heap fallbacks.
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "kvc_serial.h"

extern "C" int model_select(const uint32_t* keys_in, int n, int k, int topk, int32_t* out,
                            int* path) {
  using namespace kvc;
  std::vector<uint32_t> key(keys_in, keys_in + n);
  std::vector<uint32_t> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = (uint32_t)i;
  uint32_t* K = key.data();
  uint32_t* I = idx.data();
  *path = 0;  // 0 partitions only, 1 partial_sort heap select, 2 depth-limit heap fallback
  if (k > 0 && k < n) {
    const bool partial = topk && (int64_t)k * 64 <= n;
    const int thr = topk ? 3 : 16;
    int lo = 0, hi = n, depth = 2 * floor_log2(n);
    if (partial) {
      heap_select(K, I, k, n);
      *path = 1;
    } else {
      while (!(lo == k || hi == k)) {
        if (hi - lo <= thr) {
          insertion_sort(K, I, lo, hi);
          break;
        }
        if (depth == 0) {
          *path = 2;
          if (topk) {
            heap_select(K + lo, I + lo, k - lo, hi - lo);
            kv_swap(K, I, lo, k - 1);
          } else {
            make_heap(K + lo, I + lo, hi - lo);
            sort_heap(K + lo, I + lo, hi - lo);
          }
          break;
        }
        --depth;
        move_median_to_first(K, I, lo, lo + 1, lo + (hi - lo) / 2, hi - 1);
        const uint32_t p = K[lo];
        std::vector<int> G, S;
        for (int i = lo + 1; i < hi; ++i)
          if (!(K[i] < p)) G.push_back(i);
        for (int i = hi - 1; i > lo; --i)
          if (!(p < K[i])) S.push_back(i);
        S.push_back(lo);
        int m = 0;
        while (m < (int)G.size() && m < (int)S.size() && G[m] < S[m]) ++m;
        const int gn = m < (int)G.size() ? G[m] : 0x7FFFFFFF;
        const int sm = m > 0 ? S[m - 1] : 0x7FFFFFFF;
        const int cut = std::min(gn, sm);
        for (int t = 0; t < m; ++t) kv_swap(K, I, G[t], S[t]);
        if (topk) {
          if (cut <= k - 1) lo = cut; else hi = cut;
        } else {
          if (k <= cut) hi = cut; else lo = cut;
        }
      }
    }
  }
  const int kk = k < n ? k : n;
  std::vector<int32_t> sel(I, I + (kk > 0 ? kk : 0));
  std::sort(sel.begin(), sel.end());
  for (int i = 0; i < (int)sel.size(); ++i) out[i] = sel[i];
  return 0;
}

extern "C" uint32_t model_key_bf16(uint32_t b, int desc) { return kvc::key_bf16(b, desc != 0); }
extern "C" uint32_t model_key_f32(uint32_t b, int desc) { return kvc::key_f32(b, desc != 0); }
extern "C" uint32_t model_f32_to_bf16(float f) { return kvc::f32_to_bf16_rne(f); }
extern "C" uint32_t model_canon_nan(uint32_t w) { return kvc::canon_nan_bf16x2(w); }
extern "C" uint32_t model_key_f16(uint32_t b, int desc) { return kvc::key_f16(b, desc != 0); }
extern "C" uint32_t model_f32_to_f16(float f) { return kvc::f32_to_f16_rne(f); }
extern "C" float model_f16_to_f32(uint32_t h) { return kvc::f16_to_f32(h); }
extern "C" uint32_t model_canon_nan_f16(uint32_t w) { return kvc::canon_nan_f16x2(w); }

