// Host model of the select kernel's algorithm (test infrastructure): the same chain of Hoare
// partitions from rank lists that select_kernel computes in parallel, executed serially, with the
// serial steps taken from the kernel's own header (csrc/kvc_serial.h, __host__ __device__).
// tests/test_select_model.py checks it against real libstdc++ std::sort / std::nth_element /
// std::partial_sort, including adversarial inputs that force the heap fallbacks.
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "kvc_serial.h"

// Lane-by-lane model of wave_tiny_chain's level (csrc/kvc.hip): the segment [lo, hi) of at
// most 64 positions in "lanes" (lane i = position lo + i); the median move, the ge / le ballots,
// the g / s ranks from mbcnt counts, the rank -> lane tables of the forward permutes and the
// partner fetch of the backward permutes, exactly as the kernel computes them.  Returns cut.
static int tiny_level(uint32_t* K, uint32_t* I, int lo, int hi) {
  int m = hi - lo;
  uint32_t kk[64], ii[64];
  for (int l = 0; l < 64; ++l) {
    kk[l] = l < m ? K[lo + l] : 0xFFFFFFFFu;
    ii[l] = l < m ? I[lo + l] : 0u;
  }
  const int slo = 0, shi = m;
  const int a = slo + 1, b = slo + (shi - slo) / 2, c = shi - 1;
  const uint32_t ka = kk[a], kb = kk[b], kc = kk[c];
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
  const uint32_t klo = kk[slo], ich = ii[ch], ilo = ii[slo];
  kk[ch] = klo; kk[slo] = p;
  ii[ch] = ilo; ii[slo] = ich;
  uint64_t GE = 0, LE = 0;
  bool ge[64], le[64];
  for (int l = 0; l < 64; ++l) {
    const bool inr = l > slo && l < shi;
    ge[l] = inr && kk[l] >= p;
    le[l] = inr && kk[l] <= p;
    GE |= (uint64_t)ge[l] << l;
    LE |= (uint64_t)le[l] << l;
  }
  const int tot_le = __builtin_popcountll(LE);
  int A[64], lin[64], srk[64];
  bool sg[64], ss[64];
  uint64_t SG = 0;
  for (int l = 0; l < 64; ++l) {
    const uint64_t below = l ? (~0ull >> (64 - l)) : 0ull;
    A[l] = __builtin_popcountll(GE & below);
    lin[l] = __builtin_popcountll(LE & below) + (le[l] ? 1 : 0);
    sg[l] = ge[l] && A[l] + lin[l] < tot_le;
    SG |= (uint64_t)sg[l] << l;
  }
  const int msw = __builtin_popcountll(SG);
  uint64_t SS = 0;
  int gt[64], st[64];
  for (int l = 0; l < 64; ++l) gt[l] = st[l] = -1;
  for (int l = 0; l < 64; ++l) {  // forward permutes (dump lane 63)
    srk[l] = tot_le - lin[l] + 1;
    ss[l] = le[l] && srk[l] <= msw;
    SS |= (uint64_t)ss[l] << l;
    gt[sg[l] ? A[l] : 63] = l;
    st[ss[l] ? srk[l] - 1 : 63] = l;
  }
  uint32_t nk[64], ni[64];
  for (int l = 0; l < 64; ++l) {
    int partner = l;
    if (sg[l]) partner = st[A[l]];
    else if (ss[l]) partner = gt[srk[l] - 1];
    nk[l] = kk[partner];
    ni[l] = ii[partner];
  }
  for (int l = 0; l < m; ++l) {
    K[lo + l] = nk[l];
    I[lo + l] = ni[l];
  }
  const uint64_t GN = GE & ~SG;
  const int gnext = GN ? __builtin_ctzll(GN) : 0x7FFFFFFF;
  const int cut = std::min(gnext, SS ? __builtin_ctzll(SS) : 0x7FFFFFFF);
  return cut == 0x7FFFFFFF ? cut : lo + cut;
}

static int g_tiny = 0;  // model_select: segments of 16 < n <= 64 (> thr) through tiny_level
extern "C" void model_set_tiny(int on) { g_tiny = on; }

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
        if (g_tiny && hi - lo <= 64) {
          const int cut = tiny_level(K, I, lo, hi);
          if (topk) {
            if (cut <= k - 1) lo = cut; else hi = cut;
          } else {
            if (k <= cut) hi = cut; else lo = cut;
          }
          continue;
        }
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


// ---- the select kernel's register heap (RegHeap in csrc/kvc.hip), 64 lanes simulated ---------
// adjust() as the kernel computes it: per lane its chosen child from its children's keys, the
// path from `top` by a chase of chosen children, the stop depth m as a count over path nodes,
// then path depths < m take their chosen child's entry and depth m the value.  Checked slot by
// slot against kvc_serial.h's serial adjust_heap (itself checked against libstdc++ above).
namespace {
struct ModelRegHeap {
  uint32_t hk[64] = {0}, hi[64] = {0};
  void adjust(int top, int len, uint32_t vk, uint32_t vi) {
    int ch[64], depth[64];
    uint32_t ck[64], ci[64];
    for (int lane = 0; lane < 64; ++lane) {
      const int l = std::min(2 * lane + 1, 63), r = std::min(2 * lane + 2, 63);
      const bool two = lane < (len - 1) / 2;
      const bool lone = (len & 1) == 0 && lane == (len - 2) / 2;
      const bool left = lone || (two && hk[r] < hk[l]);
      ch[lane] = two || lone ? (left ? l : r) : -1;
      ck[lane] = left ? hk[l] : hk[r];
      ci[lane] = left ? hi[l] : hi[r];
      depth[lane] = -1;
    }
    for (int cur = top, d = 0; cur >= 0; ++d) {
      depth[cur] = d;
      cur = ch[cur];
    }
    int m = 0;
    for (int lane = 0; lane < 64; ++lane) m += depth[lane] >= 1 && !(hk[lane] < vk);
    for (int lane = 0; lane < 64; ++lane) {
      const bool up = depth[lane] >= 0 && depth[lane] < m, here = depth[lane] == m;
      hk[lane] = up ? ck[lane] : here ? vk : hk[lane];
      hi[lane] = up ? ci[lane] : here ? vi : hi[lane];
    }
  }
};
uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
}  // namespace

// Random rows (n up to 3000, 1..`levels` distinct keys: tie-heavy for small values), every
// middle 1..64: the register heap's make_heap + scan + pops against kvc_serial.h heap_select,
// compared slot by slot (key and index).  Returns the number of mismatching rows.
extern "C" int model_regheap_check(uint64_t seed, int cases) {
  int bad = 0;
  for (int c = 0; c < cases; ++c) {
    const int n = 2 + (int)(splitmix(seed) % 3000);
    const int middle = 1 + (int)(splitmix(seed) % std::min(64, n - 1));
    const uint32_t levels = 1 + (uint32_t)(splitmix(seed) % (c % 3 == 0 ? 4 : 65536));
    std::vector<uint32_t> key(n), idx(n);
    for (int i = 0; i < n; ++i) {
      key[i] = (uint32_t)(splitmix(seed) % levels);
      idx[i] = (uint32_t)i;
    }
    std::vector<uint32_t> sk = key, si = idx;
    kvc::heap_select(sk.data(), si.data(), middle, n);
    ModelRegHeap h;
    for (int j = 0; j < middle; ++j) {
      h.hk[j] = key[j];
      h.hi[j] = idx[j];
    }
    if (middle >= 2)
      for (int parent = (middle - 2) / 2; parent >= 0; --parent)
        h.adjust(parent, middle, h.hk[parent], h.hi[parent]);
    for (int i = middle; i < n; ++i)
      if (key[i] < h.hk[0]) h.adjust(0, middle, key[i], idx[i]);
    for (int j = 0; j < middle; ++j)
      if (h.hk[j] != sk[j] || h.hi[j] != si[j]) {
        ++bad;
        break;
      }
  }
  return bad;
}
