// handoff_probe.hip -- what splitting one selection row over two workgroups would pay on the
// 8-way rank geometry (one 1 024-thread selection workgroup per CU, most CUs idle), measured on
// the box ("The 8-way split's per-rank floor").
//
//   pingpong  pairs of 1 024-thread workgroups (16 waves, 80 KiB of LDS each: one per CU, as a
//             selection row) pass an 8-byte tagged word back and forth R times through the L2s
//             (agent-scope relaxed sc1 stores / sc1 load polls: the guide's handoff-1to1 form);
//             partner on the same XCD (blockIdx + 8) or on another (blockIdx + 17); optionally
//             with every other CU streaming HBM reads (the loaded-chip case).  -> us per hop
//   p1split   level 0's first pass of the selection chain (P1: the ge / le counts of a
//             15 936-position bf16-key row against its median-of-3 pivot, 16 waves x J rows of
//             64 positions, packed per-lane counters, one DPP row scan, a block reduction) by
//             ONE workgroup over the whole row, against TWO workgroups on one XCD each counting
//             half and the second handing its counts to the first (one 8-byte tagged word).
//             -> us from the counting workgroup's start to the row's counts known, both forms
//             (rows of 128 workgroups = the cfg4 rank's 4 layers x 32 heads)
// Every poll is bounded (a missing partner ends the wait with an error flag, never a hang).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/handoff_probe.hip -o tools/handoff_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kThreads = 1024;
constexpr int kLds = 80 * 1024;  // one selection row's worth: one such workgroup per CU
constexpr int kMaxPoll = 1 << 20;

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz
__device__ __forceinline__ void put(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t get(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// poll until the word's tag (high 32 bits) equals `tag`; returns its low 32 bits (or ~0 on timeout)
__device__ uint32_t wait_tag(uint64_t* p, uint32_t tag, uint32_t* err) {
  for (int i = 0; i < kMaxPoll; ++i) {
    const uint64_t w = get(p);
    if ((uint32_t)(w >> 32) == tag) return (uint32_t)w;
    if ((i & 1023) == 1023 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return 0xFFFFFFFFu;  // another wait already timed out: give up
  }
  atomicOr(err, 1u);
  return 0xFFFFFFFFu;
}

// blocks [0, npairs) ping; block b + off pongs; other blocks stream `buf` (if stream) until the
// pingers are done (bounded passes)
__global__ void __launch_bounds__(kThreads) pingpong(uint64_t* words, int npairs, int off, int rounds,
                                                     const uint4* buf, size_t nvec, int stream,
                                                     uint64_t* out, uint32_t* err, uint32_t* done) {
  extern __shared__ char lds[];
  const int b = blockIdx.x;
  const bool ping = b < npairs, pong = b >= off && b - off < npairs && b - off >= 0 && !ping;
  if (threadIdx.x == 0) lds[0] = 0;
  if (ping || pong) {
    const int pr = ping ? b : b - off;
    uint64_t* mine = words + 2 * pr + (ping ? 0 : 1);
    uint64_t* theirs = words + 2 * pr + (ping ? 1 : 0);
    if (threadIdx.x == 0) {
      const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
      uint64_t t0 = 0;
      for (int r = 1; r <= rounds; ++r) {
        if (ping) {
          if (r == 2) t0 = rt();  // round 1 waits for the partner's dispatch
          put(mine, ((uint64_t)r << 32) | xcc);
          wait_tag(theirs, r, err);
        } else {
          wait_tag(theirs, r, err);
          put(mine, ((uint64_t)r << 32) | xcc);
          if (r == 1) out[2 * pr + 1] = xcc;  // the ponger's own XCC id
        }
      }
      if (ping) {
        out[2 * pr] = (rt() - t0) | ((uint64_t)xcc << 56);
        atomicAdd(done, 1u);
      }
    }
    return;
  }
  if (!stream) return;
  // streaming block: 16-B loads over the buffer until every pinger is done
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int pass = 0; pass < 64; ++pass) {
    for (size_t i = (size_t)b * kThreads + threadIdx.x; i < nvec;
         i += (size_t)(gridDim.x) * kThreads) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + i));
      acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)npairs) break;
  }
  if (acc.x == 0x12345678u && acc.y == 7u) atomicOr(err, 2u);  // keep the loads
}

// P1 of level 0 over positions [lo, hi) of a row of bf16 keys (u16), pivot p: ge | le << 16 of
// this block's positions (per-lane packed counters, DPP-free wave sum via shuffles, LDS block sum)
// (key[i] holds position lo + i)
__device__ uint32_t count_range(const uint16_t* key, int lo, int hi, uint32_t p, uint32_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = hi - lo, J = (n + kThreads - 1) / kThreads;
  const int pos0 = lo + wid * J * 64 + lane;
  uint32_t pc = 0;
  for (int j = 0; j < J; ++j) {
    const int pos = pos0 + j * 64;
    const uint32_t k = pos < hi ? key[pos - lo] : 0u;
    pc += (pos < hi && k >= p ? 1u : 0u) + (pos < hi && k <= p ? 0x10000u : 0u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pc += (uint32_t)__shfl_xor((int)pc, o, 64);
  if (lane == 0) wsum[wid] = pc;
  __syncthreads();
  uint32_t t = 0;
  for (int w = 0; w < kThreads / 64; ++w) t += wsum[w];
  return t;
}

// rows of n bf16 norms (u16 bits, contiguous); split = 0: block r counts row r; split = 1: blocks
// r and r + 8 * (r / 8) + 8 ... pairs on one XCD count halves, the second hands its counts over
__global__ void __launch_bounds__(kThreads) p1(const uint16_t* norms, int n, int rows, int split,
                                              uint64_t* words, uint32_t tag, uint64_t* out,
                                              uint32_t* counts, uint32_t* err) {
  extern __shared__ char lds[];
  uint16_t* key = reinterpret_cast<uint16_t*>(lds);
  __shared__ uint32_t wsum[kThreads / 64];
  int row, half;
  if (!split) {
    row = blockIdx.x;
    half = -1;
  } else {  // blocks 16g + i (i < 8) and 16g + 8 + i share an XCD under round-robin placement
    const int g = blockIdx.x / 16, i = blockIdx.x % 16;
    row = g * 8 + (i & 7);
    half = i >> 3;
  }
  if (row >= rows) return;
  const uint16_t* src = norms + (size_t)row * n;
  const int lo = half == 1 ? n / 2 : 0, hi = half == 0 ? n / 2 : n;
  for (int i = lo + threadIdx.x; i < hi; i += kThreads) key[i - lo] = src[i];  // the row's (half) keys
  // median of three (positions 1, n/2, n-1), from global (the halves hold only one side)
  const uint32_t ka = src[1], kb = src[n / 2], kc = src[n - 1];
  const uint32_t p = ka < kb ? (kb < kc ? kb : (ka < kc ? kc : ka)) : (ka < kc ? ka : (kb < kc ? kc : kb));
  __syncthreads();
  const uint64_t t0 = rt();
  uint32_t c = count_range(key, lo, hi, p, wsum);
  if (half == 1) {  // hand the counts to the other half's block
    if (threadIdx.x == 0) put(words + row, ((uint64_t)tag << 32) | c);
    return;
  }
  if (half == 0 && threadIdx.x == 0) c += wait_tag(words + row, tag, err);
  if (threadIdx.x == 0) {
    out[row] = rt() - t0;
    counts[row] = c;
  }
}

static std::vector<uint16_t> bf16_norm_rows(int rows, int n) {  // bf16 norms of ~N(0,1) keys
  std::vector<uint16_t> v((size_t)rows * n);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& x : v) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const float f = 11.3f + 0.7f * ((float)(s % 20001) / 10000.0f - 1.0f) * 1.7f;
    uint32_t u;
    memcpy(&u, &f, 4);
    x = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
  }
  return v;
}

static void pct(std::vector<double> v, double* med, double* p90) {
  std::sort(v.begin(), v.end());
  *med = v[v.size() / 2];
  *p90 = v[(size_t)(v.size() * 0.9)];
}

int main(int argc, char** argv) {
  CK(hipFuncSetAttribute((const void*)pingpong, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  CK(hipFuncSetAttribute((const void*)p1, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  uint64_t *words, *out;
  uint32_t *err, *done, *counts;
  CK(hipMalloc(&words, 4096 * sizeof(uint64_t)));
  CK(hipMalloc(&out, 4096 * sizeof(uint64_t)));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&done, 4));
  CK(hipMalloc(&counts, 4096 * 4));
  const size_t nvec = (size_t)1 << 26;  // 1 GiB streamed by the loaded-chip variant
  uint4* buf;
  CK(hipMalloc(&buf, nvec * 16));
  CK(hipMemset(buf, 1, nvec * 16));
  // ---- ping-pong ----
  const int npairs = 8, rounds = 200;
  for (int stream = 0; stream < 2; ++stream) {
    for (int o : {8, 17}) {  // partner blockIdx + 8 (same XCD), + 17 (another XCD)
      const int grid = stream ? 256 : o + npairs;
      CK(hipMemset(words, 0, 4096 * sizeof(uint64_t)));
      CK(hipMemset(err, 0, 4));
      CK(hipMemset(done, 0, 4));
      hipLaunchKernelGGL(pingpong, dim3(grid), dim3(kThreads), kLds, 0, words, npairs, o, rounds,
                         buf, nvec, stream, out, err, done);
      CK(hipDeviceSynchronize());
      uint64_t h[32];
      uint32_t e;
      CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      std::vector<double> hop;
      int same = 0;
      for (int i = 0; i < npairs; ++i) {
        const uint64_t ticks = h[2 * i] & ((1ull << 56) - 1);
        hop.push_back(ticks * 10.0 / 1000.0 / (2.0 * (rounds - 1)));  // 100 MHz ticks -> us per hop
        same += (int)((h[2 * i] >> 56) == (h[2 * i + 1] & 0xFF));
      }
      double med, p90;
      pct(hop, &med, &p90);
      printf("{\"probe\": \"pingpong\", \"partner\": \"blockIdx + %d\", \"pairs_on_same_xcd\": %d, "
             "\"pairs\": %d, \"streaming_chip\": %s, \"us_per_hop_median\": %.3f, "
             "\"us_per_hop_p90\": %.3f, \"err\": %u}\n",
             o, same, npairs, stream ? "true" : "false", med, p90, e);
    }
  }
  // ---- P1 of level 0: one workgroup per row vs two per row (same XCD) + hand-off ----
  const int n = 15936, rows = 128;  // the cfg4 rank: 4 layers x 32 heads, h2o middle
  std::vector<uint16_t> host = bf16_norm_rows(rows, n);
  uint16_t* norms;
  CK(hipMalloc(&norms, host.size() * 2));
  CK(hipMemcpy(norms, host.data(), host.size() * 2, hipMemcpyHostToDevice));
  std::vector<uint32_t> ref(rows);
  for (int split = 0; split < 2; ++split) {
    std::vector<double> us;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemset(err, 0, 4));
      const int grid = split ? 2 * rows : rows;
      hipLaunchKernelGGL(p1, dim3(grid), dim3(kThreads), kLds, 0, norms, n, rows, split, words,
                         (uint32_t)(100 + rep + 10 * split), out, counts, err);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> t(rows);
      std::vector<uint32_t> c(rows);
      uint32_t e;
      CK(hipMemcpy(t.data(), out, rows * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(c.data(), counts, rows * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      if (e) { fprintf(stderr, "p1 split=%d: poll timeout\n", split); return 2; }
      if (!split) ref = c;
      else if (c != ref) { fprintf(stderr, "p1 split counts differ\n"); return 3; }
      for (auto x : t) us.push_back(x * 10.0 / 1000.0);
    }
    double med, p90;
    pct(us, &med, &p90);
    printf("{\"probe\": \"p1_level0\", \"row\": %d, \"rows\": %d, \"workgroups_per_row\": %d, "
           "\"us_start_to_counts_median\": %.3f, \"us_p90\": %.3f, \"counts_equal\": true}\n",
           n, rows, split ? 2 : 1, med, p90);
  }
  return 0;
}
