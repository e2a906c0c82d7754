// row_gather_probe.hip -- HBM read traffic of gathering 160-byte token rows (pythia-2.8b's
// head_dim 80 in bf16: BASELINE cfg2 fix512-s4096-d80) with different load shapes (GPU box only).
// The engine's copy (gather_row, csrc/kvc.hip) reads 1.51x its algorithmic bytes on that geometry
// (profiles/r04_j_pmc_traffic_fix512_s4096_d80.json).  A 160-B row at a 32-B-aligned offset spans
// two 128-B lines and three 64-B sectors; this probe measures which shape of loads fetches what.
//
// Workload: K and V [32 layers x 32 heads x 4096 x 80] bf16 (1.34 GB: past the 256 MiB Infinity
// Cache), 512 ascending random positions per (layer, head) row -- the shape of a fix512 selection
// -- gathered into contiguous [512, 80] outputs.  One kernel per load shape (one workgroup of 256
// threads per row, 4 token rows in flight per thread):
//   v16    16-B lanes, 10 lanes per row (the engine's gather_row layout)
//   v16nt  the same with non-temporal loads
//   v8     8-B lanes, 20 lanes per row
//   w32    32-B lanes (two 16-B loads each), 5 lanes per row
//   s64    the row's three 64-B sectors (192 B, 12 16-B lanes; 32 B beyond the row are read too)
//   l128   the row's two 128-B lines (256 B, 16 lanes)
//   v16o   v16 with the rows' order reversed within each 64-row batch (same lines, other order)
// Every variant writes the 160-B output rows (the sector / line variants extract them from the
// loaded chunks by lane shuffles), checked against v16's output.  Run it under
//   rocprofv3 --pmc FETCH_SIZE -- tools/row_gather_probe   (and TCC_EA0_RDREQ / _32B counters)
// to read each kernel's fetched bytes; stdout reports the best-of-10 time of each variant.
// Build:  hipcc --offload-arch=gfx950 -O3 tools/row_gather_probe.hip -o tools/row_gather_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

constexpr int L = 32, H = 32, S = 4096, D = 80, K = 512;
constexpr int ROWB = D * 2;            // 160 bytes per token row
constexpr int ROWS = L * H;            // gather rows (layer, head)
constexpr int NT = 256;                // threads per workgroup
constexpr int BATCH = 4;               // token rows in flight per thread

enum { V16 = 0, V16NT, V8, W32, S64, L128, V16O, NVAR };
static const char* kNames[NVAR] = {"v16", "v16nt", "v8", "w32", "s64", "l128", "v16o"};

__device__ __forceinline__ uint4 ld16(const char* p, bool nt) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  if (nt) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const uint4*>(p);
}

// out row t of workgroup row r = X[r][pos[r][t]] for X = K, V
template <int VAR>
__global__ void __launch_bounds__(NT) gather(const char* __restrict__ k, const char* __restrict__ v,
                                             const int* __restrict__ pos, char* __restrict__ ko,
                                             char* __restrict__ vo) {
  const int r = blockIdx.x;
  const char* kb = k + (size_t)r * S * ROWB;
  const char* vb = v + (size_t)r * S * ROWB;
  char* kob = ko + (size_t)r * K * ROWB;
  char* vob = vo + (size_t)r * K * ROWB;
  const int* pr = pos + r * K;
  const int tid = threadIdx.x;
  if constexpr (VAR == V16 || VAR == V16NT || VAR == V16O) {
    constexpr int NC = ROWB / 16, TPI = NT / NC;  // 10 lanes per row, 25 rows per pass
    const int tq = tid / NC, c = tid - tq * NC;
    if (tq >= TPI) return;
    for (int tb = tq; tb < K; tb += TPI * BATCH) {
      uint4 xk[BATCH], xv[BATCH];
      int tt[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        int t = tb + i * TPI;
        if (VAR == V16O && t < K) t = (t & ~63) + 63 - (t & 63) < K ? (t & ~63) + 63 - (t & 63) : t;
        tt[i] = t;
        if (t < K) {
          const int p = pr[t];
          xk[i] = ld16(kb + (size_t)p * ROWB + c * 16, VAR == V16NT);
          xv[i] = ld16(vb + (size_t)p * ROWB + c * 16, VAR == V16NT);
        }
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        if (tt[i] < K) {
          *reinterpret_cast<uint4*>(kob + (size_t)tt[i] * ROWB + c * 16) = xk[i];
          *reinterpret_cast<uint4*>(vob + (size_t)tt[i] * ROWB + c * 16) = xv[i];
        }
      }
    }
  } else if constexpr (VAR == V8) {
    constexpr int NC = ROWB / 8, TPI = NT / NC;  // 20 lanes per row
    const int tq = tid / NC, c = tid - tq * NC;
    if (tq >= TPI) return;
    for (int tb = tq; tb < K; tb += TPI * BATCH) {
      uint2 xk[BATCH], xv[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        if (t < K) {
          const int p = pr[t];
          xk[i] = *reinterpret_cast<const uint2*>(kb + (size_t)p * ROWB + c * 8);
          xv[i] = *reinterpret_cast<const uint2*>(vb + (size_t)p * ROWB + c * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        if (t < K) {
          *reinterpret_cast<uint2*>(kob + (size_t)t * ROWB + c * 8) = xk[i];
          *reinterpret_cast<uint2*>(vob + (size_t)t * ROWB + c * 8) = xv[i];
        }
      }
    }
  } else if constexpr (VAR == W32) {
    constexpr int NC = ROWB / 32, TPI = NT / NC;  // 5 lanes per row
    const int tq = tid / NC, c = tid - tq * NC;
    if (tq >= TPI) return;
    for (int tb = tq; tb < K; tb += TPI * BATCH) {
      uint4 xk[BATCH][2], xv[BATCH][2];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        if (t < K) {
          const int p = pr[t];
          xk[i][0] = ld16(kb + (size_t)p * ROWB + c * 32, false);
          xk[i][1] = ld16(kb + (size_t)p * ROWB + c * 32 + 16, false);
          xv[i][0] = ld16(vb + (size_t)p * ROWB + c * 32, false);
          xv[i][1] = ld16(vb + (size_t)p * ROWB + c * 32 + 16, false);
        }
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        if (t < K) {
          *reinterpret_cast<uint4*>(kob + (size_t)t * ROWB + c * 32) = xk[i][0];
          *reinterpret_cast<uint4*>(kob + (size_t)t * ROWB + c * 32 + 16) = xk[i][1];
          *reinterpret_cast<uint4*>(vob + (size_t)t * ROWB + c * 32) = xv[i][0];
          *reinterpret_cast<uint4*>(vob + (size_t)t * ROWB + c * 32 + 16) = xv[i][1];
        }
      }
    }
  } else {
    // S64: 12 lanes per row over the row's 64-B-aligned 192-byte span; L128: 16 lanes over its
    // 128-B-aligned 256-byte span.  Lane c holds span chunk c; output chunk j (of 10) is span
    // chunk j + off/16 -- fetched from its lane by ds_bpermute.  Rows are grouped per 16 lanes
    // (4 rows per wave), so that every row's lanes lie in one wave.
    constexpr int NC = VAR == S64 ? 12 : 16, SPAN = NC * 16, AL = VAR == S64 ? 64 : 128;
    constexpr int TPW = 4, TPI = NT / 64 * TPW;  // 16 rows per pass
    const int lane = tid & 63, wv = tid >> 6, slot = lane >> 4, c = lane & 15;
    for (int tb = wv * TPW + slot; tb < K; tb += TPI * BATCH) {
      uint4 xk[BATCH], xv[BATCH];
      int off[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        off[i] = 0;
        xk[i] = xv[i] = make_uint4(0, 0, 0, 0);
        if (t < K) {
          const size_t a = (size_t)pr[t] * ROWB;
          const size_t a0 = a / AL * AL;
          off[i] = (int)(a - a0);
          if (c < NC && a0 + c * 16 + 16 <= (size_t)S * ROWB) {
            xk[i] = ld16(kb + a0 + c * 16, false);
            xv[i] = ld16(vb + a0 + c * 16, false);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int t = tb + i * TPI;
        // output chunk c (c < 10) of this row comes from span chunk c + off / 16, same 16 lanes
        const int src = (lane & ~15) + min(c + off[i] / 16, 15);
        uint4 ok, ov;
        ok.x = __builtin_amdgcn_ds_bpermute(src * 4, (int)xk[i].x);
        ok.y = __builtin_amdgcn_ds_bpermute(src * 4, (int)xk[i].y);
        ok.z = __builtin_amdgcn_ds_bpermute(src * 4, (int)xk[i].z);
        ok.w = __builtin_amdgcn_ds_bpermute(src * 4, (int)xk[i].w);
        ov.x = __builtin_amdgcn_ds_bpermute(src * 4, (int)xv[i].x);
        ov.y = __builtin_amdgcn_ds_bpermute(src * 4, (int)xv[i].y);
        ov.z = __builtin_amdgcn_ds_bpermute(src * 4, (int)xv[i].z);
        ov.w = __builtin_amdgcn_ds_bpermute(src * 4, (int)xv[i].w);
        if (t < K && c < 10) {
          *reinterpret_cast<uint4*>(kob + (size_t)t * ROWB + c * 16) = ok;
          *reinterpret_cast<uint4*>(vob + (size_t)t * ROWB + c * 16) = ov;
        }
      }
    }
    (void)SPAN;
  }
}

typedef void (*Kern)(const char*, const char*, const int*, char*, char*);
static const Kern kKerns[NVAR] = {gather<V16>, gather<V16NT>, gather<V8>, gather<W32>,
                                  gather<S64>, gather<L128>, gather<V16O>};

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main(int argc, char** argv) {
  const size_t in_bytes = (size_t)ROWS * S * ROWB, out_bytes = (size_t)ROWS * K * ROWB;
  char *k, *v, *ko, *vo, *ref;
  int* pos;
  CHECK(hipMalloc(&k, in_bytes));
  CHECK(hipMalloc(&v, in_bytes));
  CHECK(hipMalloc(&ko, out_bytes));
  CHECK(hipMalloc(&vo, out_bytes));
  CHECK(hipMalloc(&ref, 2 * out_bytes));
  CHECK(hipMalloc(&pos, (size_t)ROWS * K * sizeof(int)));
  // inputs: byte pattern from the address (so gathered rows are checkable)
  {
    std::vector<uint32_t> hv(in_bytes / 4 / ROWS);
    for (int r = 0; r < ROWS; ++r) {
      for (size_t i = 0; i < hv.size(); ++i) hv[i] = (uint32_t)(r * 2654435761u) ^ (uint32_t)i;
      CHECK(hipMemcpy(k + (size_t)r * S * ROWB, hv.data(), S * ROWB, hipMemcpyHostToDevice));
      for (size_t i = 0; i < hv.size(); ++i) hv[i] = ~hv[i];
      CHECK(hipMemcpy(v + (size_t)r * S * ROWB, hv.data(), S * ROWB, hipMemcpyHostToDevice));
    }
  }
  {
    std::vector<int> hp((size_t)ROWS * K), perm(S);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int r = 0; r < ROWS; ++r) {
      for (int i = 0; i < S; ++i) perm[i] = i;
      for (int i = 0; i < K; ++i) {  // partial Fisher-Yates
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const int j = i + (int)(x % (uint64_t)(S - i));
        std::swap(perm[i], perm[j]);
      }
      std::sort(perm.begin(), perm.begin() + K);
      memcpy(&hp[(size_t)r * K], perm.data(), K * sizeof(int));
    }
    CHECK(hipMemcpy(pos, hp.data(), hp.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  printf("{\"rows\": %d, \"k\": %d, \"row_bytes\": %d, \"alg_read_bytes\": %zu, \"variants\": [",
         ROWS, K, ROWB, 2 * out_bytes);
  for (int q = 0; q < NVAR; ++q) {
    float best = 1e30f;
    for (int rep = 0; rep < reps; ++rep) {
      CHECK(hipMemset(ko, 0, out_bytes));
      CHECK(hipMemset(vo, 0, out_bytes));
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(kKerns[q], dim3(ROWS), dim3(NT), 0, 0, k, v, pos, ko, vo);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    bool ok = true;
    if (q == 0) {
      CHECK(hipMemcpy(ref, ko, out_bytes, hipMemcpyDeviceToDevice));
      CHECK(hipMemcpy(ref + out_bytes, vo, out_bytes, hipMemcpyDeviceToDevice));
      // spot-check v16 against the host pattern: row 5, token 7
      std::vector<int> hp(K);
      CHECK(hipMemcpy(hp.data(), pos + 5 * K, K * sizeof(int), hipMemcpyDeviceToHost));
      uint32_t got[ROWB / 4];
      CHECK(hipMemcpy(got, ko + ((size_t)5 * K + 7) * ROWB, ROWB, hipMemcpyDeviceToHost));
      for (int i = 0; i < ROWB / 4; ++i)
        ok &= got[i] == ((uint32_t)(5 * 2654435761u) ^ (uint32_t)((size_t)hp[7] * ROWB / 4 + i));
    } else {
      std::vector<char> h1(out_bytes), h2(out_bytes);
      CHECK(hipMemcpy(h1.data(), ko, out_bytes, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(h2.data(), ref, out_bytes, hipMemcpyDeviceToHost));
      ok &= memcmp(h1.data(), h2.data(), out_bytes) == 0;
      CHECK(hipMemcpy(h1.data(), vo, out_bytes, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(h2.data(), ref + out_bytes, out_bytes, hipMemcpyDeviceToHost));
      ok &= memcmp(h1.data(), h2.data(), out_bytes) == 0;
    }
    printf("%s{\"variant\": \"%s\", \"best_ms\": %.5f, \"alg_TBps\": %.3f, \"output_ok\": %s}",
           q ? ", " : "", kNames[q], best, 4.0 * out_bytes / (best * 1e-3) / 1e12,
           ok ? "true" : "false");
    fflush(stdout);
  }
  printf("]}\n");
  return 0;
}
