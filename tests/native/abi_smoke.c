/* abi_smoke.c -- a native C caller of the engine: only include/kvc.h, libkvc.so and the HIP
 * runtime API (no Python, no torch).  Test infrastructure (tests/test_native_abi.py).
 *
 *   abi_smoke plan                       host-only kvc_plan checks (no GPU needed)
 *   abi_smoke run DIR H S D K DESC [ALGO]
 *                                        reads DIR/k.bin, DIR/v.bin (bf16 [1,H,S,D]), runs
 *                                        fix_size_l2(keep K, keep_ratio 0) on one layer with
 *                                        kvc_plan + kvc_launch, writes DIR/k_out.bin, v_out.bin
 *                                        (ALGO: kvc_algo, default KVC_ALGO_SORT; KVC_ALGO_STABLE
 *                                        selects with the opt-in stable tie order)
 *
 * The mapping of one fix_size_l2 layer onto the C ABI is INTEGRATION.md's: zone [0, S),
 * n_select = K, no sink / tail, order ASC (keep_low) or DESC (keep_high), algo SORT
 * (reference kvcompress/methods/fix_size_l2.py:99-150). */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kvc.h"

#define CHECK(c, msg)                                 \
  do {                                                \
    if (!(c)) {                                       \
      fprintf(stderr, "abi_smoke: %s\n", (msg));     \
      return 1;                                       \
    }                                                 \
  } while (0)

static kvc_layer_t layer_of(void* k, void* v, void* ko, void* vo, int H, int S, int D, int K) {
  kvc_layer_t l;
  memset(&l, 0, sizeof(l));
  l.k = k;
  l.v = v;
  l.k_out = ko;
  l.v_out = vo;
  l.k_stride[0] = l.v_stride[0] = (int64_t)H * S * D;
  l.k_stride[1] = l.v_stride[1] = (int64_t)S * D;
  l.k_stride[2] = l.v_stride[2] = D;
  l.seq_len = S;
  l.zone_start = 0;
  l.zone_len = S;
  l.n_select = K;
  l.score_mode = KVC_SCORE_NORM;
  return l;
}

static kvc_params_t params_of(int H, int D, int desc, int algo) {
  kvc_params_t p;
  memset(&p, 0, sizeof(p));
  p.dtype = KVC_BF16;
  p.batch = 1;
  p.heads = H;
  p.head_dim = D;
  p.order = desc ? KVC_DESC : KVC_ASC;
  p.algo = algo;
  p.phases = KVC_PHASE_ALL;
  return p;
}

static int plan_checks(void) {
  CHECK(kvc_version() == KVC_ABI_VERSION, "ABI version");
  CHECK(kvc_layer_struct_size() == sizeof(kvc_layer_t), "layer struct size");
  CHECK(kvc_max_zone_len() == (1 << 24), "max zone");
  CHECK(kvc_source_digest() != NULL && strlen(kvc_source_digest()) > 0, "source digest");
  void* fake = (void*)(uintptr_t)4096; /* kvc_plan never dereferences tensor pointers */
  kvc_layer_t l = layer_of(fake, fake, fake, fake, 32, 16384, 128, 512);
  kvc_params_t p = params_of(32, 128, 0, KVC_ALGO_SORT);
  kvc_plan_info_t info;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_OK, "plan of the headline layer");
  CHECK(l.n_out == 512 && l.row0 == 0 && l.tile0 == 0, "plan-filled fields");
  CHECK(info.rows == 32 && info.workspace_bytes > 0, "plan info");
  p.head_dim = 100;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_HEADDIM, "bad head_dim rejected");
  p = params_of(32, 128, 0, KVC_ALGO_SORT);
  p.dtype = 7;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_DTYPE, "bad dtype rejected");
  p = params_of(32, 128, 0, KVC_ALGO_SORT);
  l.k = (void*)(uintptr_t)4098;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_ALIGN, "misaligned pointer rejected");
  l.k = fake;
  l.n_select = 16385;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_ARG, "n_select > zone rejected");
  l.n_select = 512;
  CHECK(kvc_launch(&p, &l, 1, NULL, 0, NULL) == KVC_E_WORKSPACE, "missing workspace rejected");
  p.flags = 16;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_ARG, "unknown flag bit rejected");
  p.flags = 0;
  p.reserved = 1;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_ARG, "non-zero reserved field rejected");
  p.reserved = 0;
  p.algo = KVC_ALGO_STABLE;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_OK, "stable selection planned");
  p.algo = 3;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_E_ARG, "unknown algorithm rejected");
  p.algo = KVC_ALGO_SORT;
  CHECK(strcmp(kvc_status_string(KVC_E_ALIGN), "pointer or stride not 16-byte aligned") == 0,
        "status string");
  printf("abi_smoke plan: ok\n");
  return 0;
}

static void* read_file(const char* path, size_t bytes) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  void* buf = malloc(bytes);
  const size_t got = buf ? fread(buf, 1, bytes, f) : 0;
  fclose(f);
  if (got != bytes) {
    free(buf);
    return NULL;
  }
  return buf;
}

static int write_file(const char* path, const void* buf, size_t bytes) {
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  const size_t put = fwrite(buf, 1, bytes, f);
  fclose(f);
  return put == bytes ? 0 : 1;
}

static int run(const char* dir, int H, int S, int D, int K, int desc, int algo) {
  char path[4096];
  const size_t in_bytes = (size_t)H * S * D * 2, out_bytes = (size_t)H * K * D * 2;
  snprintf(path, sizeof(path), "%s/k.bin", dir);
  void* hk = read_file(path, in_bytes);
  snprintf(path, sizeof(path), "%s/v.bin", dir);
  void* hv = read_file(path, in_bytes);
  CHECK(hk && hv, "reading inputs");
  void *dk, *dv, *dko, *dvo, *ws;
  CHECK(hipMalloc(&dk, in_bytes) == hipSuccess && hipMalloc(&dv, in_bytes) == hipSuccess &&
            hipMalloc(&dko, out_bytes) == hipSuccess && hipMalloc(&dvo, out_bytes) == hipSuccess,
        "hipMalloc");
  CHECK(hipMemcpy(dk, hk, in_bytes, hipMemcpyHostToDevice) == hipSuccess &&
            hipMemcpy(dv, hv, in_bytes, hipMemcpyHostToDevice) == hipSuccess,
        "upload");
  kvc_layer_t l = layer_of(dk, dv, dko, dvo, H, S, D, K);
  kvc_params_t p = params_of(H, D, desc, algo);
  kvc_plan_info_t info;
  CHECK(kvc_plan(&p, &l, 1, &info) == KVC_OK, "kvc_plan");
  CHECK(hipMalloc(&ws, info.workspace_bytes) == hipSuccess, "workspace");
  hipStream_t s;
  CHECK(hipStreamCreate(&s) == hipSuccess, "stream");
  const int rc = kvc_launch(&p, &l, 1, ws, info.workspace_bytes, (kvc_stream_t)s);
  CHECK(rc == KVC_OK, kvc_status_string(rc));
  CHECK(hipStreamSynchronize(s) == hipSuccess, "kernels failed");
  CHECK(hipMemcpy(hk, dko, out_bytes, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(hv, dvo, out_bytes, hipMemcpyDeviceToHost) == hipSuccess,
        "download");
  snprintf(path, sizeof(path), "%s/k_out.bin", dir);
  CHECK(write_file(path, hk, out_bytes) == 0, "writing k_out");
  snprintf(path, sizeof(path), "%s/v_out.bin", dir);
  CHECK(write_file(path, hv, out_bytes) == 0, "writing v_out");
  hipStreamDestroy(s);
  hipFree(ws);
  hipFree(dk);
  hipFree(dv);
  hipFree(dko);
  hipFree(dvo);
  free(hk);
  free(hv);
  printf("abi_smoke run: ok (%d heads, S=%d, D=%d, keep %d)\n", H, S, D, K);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && strcmp(argv[1], "plan") == 0) return plan_checks();
  if ((argc == 8 || argc == 9) && strcmp(argv[1], "run") == 0)
    return run(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
               atoi(argv[7]), argc == 9 ? atoi(argv[8]) : KVC_ALGO_SORT);
  fprintf(stderr, "usage: abi_smoke plan | run DIR H S D K DESC [ALGO]\n");
  return 2;
}
