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

// Lane-by-lane CPU mirror of select_kernel's run_chain (the parallel formulation: aligned
// per-lane chunks, virtual median swap, packed ge/le scan, m = #{ge : A + Lin < tot_le},
// g_{m+1} = first ge failing it).  NT lanes simulated serially per pass.
namespace {
template <typename KeyT>
int chain_v2(std::vector<KeyT>& key, std::vector<uint16_t>& idx, int k, bool topk, int NT,
             int wave_seg, int& lo, int& hi, int& depth, int* path) {
  using namespace kvc;
  const int VK = 16 / (int)sizeof(KeyT);
  const int thr = topk ? 3 : 16;
  std::vector<uint16_t> spos(key.size() + 8, 0);
  while (true) {
    if (lo == k || hi == k) return 0;
    if (hi - lo <= thr) { insertion_sort(key.data(), idx.data(), lo, hi); return 0; }
    if (NT > 64 && hi - lo <= wave_seg) return 1;
    if (depth == 0) {
      *path = 2;
      if (topk) { heap_select(key.data() + lo, idx.data() + lo, k - lo, hi - lo); kv_swap(key.data(), idx.data(), lo, k - 1); }
      else { make_heap(key.data() + lo, idx.data() + lo, hi - lo); sort_heap(key.data() + lo, idx.data() + lo, hi - lo); }
      return 0;
    }
    --depth;
    const int a = lo + 1, b = lo + (hi - lo) / 2, c = hi - 1;
    const KeyT ka = key[a], kb = key[b], kc = key[c], klo = key[lo];
    int ch;
    if (ka < kb) { if (kb < kc) ch = b; else if (ka < kc) ch = c; else ch = a; }
    else if (ka < kc) ch = a; else if (kb < kc) ch = c; else ch = b;
    const KeyT p = (ch == a) ? ka : (ch == b) ? kb : kc;
    const int base = (lo + 1) & ~(VK - 1);
    int E = (hi - base + NT - 1) / NT;
    E = (E + VK - 1) / VK * VK;
    if (E > 32) return -1;
    std::vector<uint32_t> gem(NT, 0), lem(NT, 0), excl(NT, 0);
    uint32_t run = 0;
    for (int t = 0; t < NT; ++t) {
      const int c0 = base + t * E;
      for (int j = 0; j < E; ++j) {
        const int pos = c0 + j;
        if (pos >= hi) break;
        KeyT kk = key[pos];
        if (pos == ch) kk = klo;
        const bool valid = pos > lo && pos < hi;
        gem[t] |= (uint32_t)(valid && !(kk < p)) << j;
        lem[t] |= (uint32_t)(valid && !(p < kk)) << j;
      }
      excl[t] = run;
      run += (uint32_t)__builtin_popcount(gem[t]) | ((uint32_t)__builtin_popcount(lem[t]) << 16);
    }
    const int tot_le = (int)(run >> 16);
    kv_swap(key.data(), idx.data(), lo, ch);
    spos[tot_le + 1] = (uint16_t)lo;
    int msw = 0, gnext = 0x7FFFFFFF;
    for (int t = 0; t < NT; ++t) {
      const int ge_excl = (int)(excl[t] & 0xFFFF), le_excl = (int)(excl[t] >> 16);
      for (int j = 0; j < E; ++j) {
        const uint32_t bit = 1u << j;
        if (!((gem[t] | lem[t]) & bit)) continue;
        const int pos = base + t * E + j;
        const int lin = le_excl + __builtin_popcount(lem[t] & (bit | (bit - 1u)));
        if (lem[t] & bit) spos[tot_le - lin + 1] = (uint16_t)pos;
        if (gem[t] & bit) {
          const int A = ge_excl + __builtin_popcount(gem[t] & (bit - 1u));
          if (A + lin < tot_le) ++msw; else gnext = std::min(gnext, pos);
        }
      }
    }
    for (int t = 0; t < NT; ++t) {
      const int ge_excl = (int)(excl[t] & 0xFFFF);
      for (int j = 0; j < E; ++j) {
        const uint32_t bit = 1u << j;
        if (!(gem[t] & bit)) continue;
        const int tt = ge_excl + __builtin_popcount(gem[t] & (bit - 1u)) + 1;
        if (tt > msw) break;
        kv_swap(key.data(), idx.data(), base + t * E + j, (int)spos[tt]);
      }
    }
    const int cut = std::min(gnext, msw > 0 ? (int)spos[msw] : 0x7FFFFFFF);
    if (topk) { if (cut <= k - 1) lo = cut; else hi = cut; }
    else { if (k <= cut) hi = cut; else lo = cut; }
  }
}
}  // namespace

extern "C" int model_select_v2(const uint32_t* keys_in, int n, int k, int topk, int key16,
                               int32_t* out, int* path) {
  using namespace kvc;
  *path = 0;
  std::vector<uint16_t> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = (uint16_t)i;
  std::vector<int32_t> sel;
  auto finish = [&](auto& key) {
    for (int i = 0; i < k; ++i) sel.push_back(idx[i]);
  };
  if (key16) {
    std::vector<uint16_t> key(keys_in, keys_in + n);
    if (topk && (int64_t)k * 64 <= n) { heap_select(key.data(), idx.data(), k, n); *path = 1; }
    else if (k > 0 && k < n) {
      int lo = 0, hi = n, depth = 2 * floor_log2(n);
      int st = chain_v2<uint16_t>(key, idx, k, topk, 1024, 1024, lo, hi, depth, path);
      if (st < 0) return -1;
      if (st == 1 && chain_v2<uint16_t>(key, idx, k, topk, 64, 1024, lo, hi, depth, path) < 0) return -1;
    }
    finish(key);
  } else {
    std::vector<uint32_t> key(keys_in, keys_in + n);
    if (topk && (int64_t)k * 64 <= n) { heap_select(key.data(), idx.data(), k, n); *path = 1; }
    else if (k > 0 && k < n) {
      int lo = 0, hi = n, depth = 2 * floor_log2(n);
      int st = chain_v2<uint32_t>(key, idx, k, topk, 1024, 1024, lo, hi, depth, path);
      if (st < 0) return -1;
      if (st == 1 && chain_v2<uint32_t>(key, idx, k, topk, 64, 1024, lo, hi, depth, path) < 0) return -1;
    }
    finish(key);
  }
  std::sort(sel.begin(), sel.end());
  for (int i = 0; i < (int)sel.size(); ++i) out[i] = sel[i];
  return 0;
}
