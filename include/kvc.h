/*
 * kvc.h -- C ABI of the MI355X-native KV-cache compression engine.
 *
 * This library is the native half of the drop-in replacement for the reference's
 * kvcompress/methods hot path (od-liu/CS3602-LLM-Inference-Acceleration).  One call compresses a
 * batch of layers; each layer's output is built from three segments of its input sequence:
 *
 *     out = K[:, :, sink]  ++  K[:, :, zone][selected]  ++  K[:, :, tail]      (same for V)
 *
 * which covers every compressing branch of the eight in-scope methods.  Each entry below names the
 * reference lines (in /root/reference/kvcompress/methods/) whose norm -> argsort/topk -> sort ->
 * gather -> cat sequence one call replaces:
 *   fix_size_l2   fix_size_l2.py:99-150   zone [0,S-P), select keep, tail = last P
 *   l2_compress   l2_compress.py:62-90    zone [0,S),   select ceil(kr*S)
 *   h2o_l2        h2o_l2.py:99-151        sink start, zone middle, tail recent
 *   snapkv_lite   snapkv_lite.py:83-152   zone prefix (snapkv scoring, topk), tail obs window
 *   pyramid_kv    pyramid_kv.py:115-183   sink, zone middle, tail recent (per-layer size)
 *   adaptive_l2   adaptive_l2.py:81-145 (hard limit), :147-199 (gradual)
 *   streaming_llm streaming_llm.py:99-109 sink + tail, no selection (pure copy);
 *                 evict_for_space streaming_llm.py:154-168 likewise
 * recent_only (recent_only.py:65-66) returns views and never reaches the engine.
 *
 * The reference does this with torch CPU/GPU ops (torch.norm -> argsort/topk -> sort -> gather
 * -> cat); the engine reproduces their results bit-exactly, including libstdc++'s introsort /
 * introselect tie order, torch.norm's 8-lane FMA order, and torch.gather's bf16 NaN rewrite.
 *
 * Phases (stream-ordered on `stream`, one kernel each per chunk of <= 64 layers; SELECT and
 * GATHER run as one select_gather kernel unless params.flags has KVC_FLAG_SPLIT_SELECT_GATHER):
 *   SCORE  : key L2 norms of every zone token           -> workspace norm region
 *   SELECT : per (layer,b,h) row: snapkv scoring (opt.), reference-exact k-selection,
 *            ascending zone-local indices                -> workspace index region (int32)
 *   GATHER : segment copy of K and V into k_out / v_out (caller-allocated, contiguous)
 *
 * Ownership: the caller allocates outputs and the workspace; the library never allocates,
 * frees or synchronises.  Entry points are reentrant (no global mutable state, no environment
 * variables read) and may be used concurrently on different devices/streams.  All functions
 * return a kvc_status (0 = ok); a HIP launch failure is reported from that launch's own return
 * value, and a caller's pending HIP error is left untouched.
 */
#ifndef KVC_H
#define KVC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history:
 *   3  kvc_params_t.flags / reserved / device_status; the h2o_attention entries.
 *   4  KVC_ALGO_STABLE and KVC_ATTN_HH_STABLE (opt-in stable tie policy); KVC_FLAG_GATHER_FIXED /
 *      KVC_FLAG_GATHER_SELECTED are refused (KVC_E_ARG) without external_index, where a v3
 *      library accepted them; device status bit KVC_DEV_INTERNAL. */
#define KVC_ABI_VERSION 4

typedef struct ihipStream_t* kvc_stream_t; /* a hipStream_t; NULL = legacy default stream */

/* KVC_F16: IEEE half (what transformers >= 5 loads pythia checkpoints as: dtype="auto").  Its
 * norm follows torch's non-vectorised CPU reduction (one fp32 accumulator in dim order), not the
 * 8-lane order of bf16/fp32 -- see DESIGN.md. */
enum kvc_dtype { KVC_F32 = 0, KVC_BF16 = 1, KVC_F16 = 2 };
/* KVC_ASC keeps the smallest keys (argsort ascending, "keep_low");
 * KVC_DESC keeps the largest (argsort descending / topk largest, "keep_high", snapkv). */
enum kvc_order { KVC_ASC = 0, KVC_DESC = 1 };
/* KVC_ALGO_SORT: set of argsort(stable=False)[:k] = libstdc++ std::sort (introsort)
 * KVC_ALGO_TOPK: set of torch.topk = std::nth_element (introselect), or std::partial_sort
 *                (heap select) when k*64 <= n, exactly as aten TopKImpl.h chooses.
 * KVC_ALGO_STABLE (opt-in, not the reference's tie order): set of argsort(stable=True)[:k] --
 *                every key strictly before the k-th one and the first of the tied keys in
 *                position order; the same set for sort and topk callers.  A radix select with
 *                no partition chain.  Zones of at most 65 536 positions (else KVC_E_TOO_LONG). */
enum kvc_algo { KVC_ALGO_SORT = 0, KVC_ALGO_TOPK = 1, KVC_ALGO_STABLE = 2 };
enum kvc_score { KVC_SCORE_NORM = 0, KVC_SCORE_SNAPKV = 1 };
enum kvc_phase {
  KVC_PHASE_SCORE = 1,
  KVC_PHASE_SELECT = 2,
  KVC_PHASE_GATHER = 4,
  KVC_PHASE_ALL = 7
};
enum kvc_flag {
  KVC_FLAG_SPLIT_SELECT_GATHER = 1, /* SELECT writes the index region, then a GATHER kernel    */
  KVC_FLAG_SHARED_INDEX = 2,        /* external_index: index row (layer*batch + b) serves every
                                       head of (layer, b) -- h2o_attention's heavy hitters, one
                                       index list per layer (h2o_attention.py:326-333)        */
  KVC_FLAG_GATHER_FIXED = 4,        /* GATHER copies only the sink and tail rows of each output
                                       (the rows no selection decides), layout unchanged      */
  KVC_FLAG_GATHER_SELECTED = 8      /* GATHER copies only the selected rows.  With the previous
                                       flag: one call's copy in two launches, e.g. the fixed rows
                                       on a second stream while the selection runs.  At most one
                                       of the two, and only with external_index (the parts
                                       read the caller's indices; KVC_E_ARG otherwise)         */
};
/* Bits the kernels OR into *params.device_status (when not NULL).  The word is sticky: the
 * library never clears it; the caller zeroes it and reads it after the stream has drained. */
enum kvc_device_status {
  KVC_DEV_SELECT_BOUNDS = 1, /* a selection row exceeded its kernel's zone capacity: nothing
                                is selected and none of that row's output rows is written
                                (never expected: kvc_launch picks kernels by the planned zone
                                lengths)                                                       */
  KVC_DEV_INDEX_RANGE = 2,   /* an external index lay outside its zone and was clamped        */
  KVC_DEV_INTERNAL = 4       /* an internal invariant of a selection failed (e.g. the register
                                tail of the partition chain saw more swaps than a 64-lane
                                segment allows): that row's output is unspecified (never
                                expected; checked so a violation cannot pass silently)        */
};
enum kvc_status {
  KVC_OK = 0,
  KVC_E_ARG = -1,       /* malformed layer table / params                             */
  KVC_E_DTYPE = -2,     /* dtype is not bf16 / fp16 / fp32                            */
  KVC_E_HEADDIM = -3,   /* head_dim*elem_size not in {64,128,160,256,320,512,1024} B  */
  KVC_E_ALIGN = -4,     /* a base pointer or stride is not 16-byte aligned            */
  KVC_E_TOO_LONG = -5,  /* a scored zone is longer than kvc_max_zone_len() (2^24), or a
                           KVC_ALGO_STABLE selection zone longer than 65 536            */
  KVC_E_WORKSPACE = -6, /* workspace smaller than kvc_plan() reported                 */
  KVC_E_HIP = -7        /* a HIP launch failed                                        */
};

/* One layer.  Inputs K,V: [batch, heads, seq_len, head_dim], last dim contiguous, arbitrary
 * element strides for the other three dims.  Outputs: contiguous [batch, heads, n_out, head_dim]
 * with n_out = sink_len + n_select + tail_len. */
typedef struct kvc_layer {
  const void* k;
  const void* v;
  void* k_out;
  void* v_out;
  int64_t k_stride[3]; /* element strides of dims batch, heads, seq */
  int64_t v_stride[3];
  int32_t seq_len;     /* S */
  int32_t zone_start;  /* scored zone [zone_start, zone_start + zone_len) */
  int32_t zone_len;
  int32_t n_select;    /* tokens kept from the zone: 0 <= n_select <= zone_len */
  int32_t sink_len;    /* segment A: source rows [0, sink_len)                   */
  int32_t tail_start;  /* segment C: source rows [tail_start, tail_start+tail_len) */
  int32_t tail_len;
  int32_t pool_kernel; /* KVC_SCORE_SNAPKV: avg_pool1d kernel; <= 1 means no pooling */
  int32_t score_mode;  /* enum kvc_score */
  /* ---- filled in by kvc_plan() ---- */
  int32_t n_out;
  int32_t row0;  /* first workspace row of this layer (rows = layer*batch*heads + b*heads + h) */
  int32_t tile0; /* first 64-token SCORE tile of this layer */
  int64_t unit0; /* first GATHER unit (one 16-byte chunk of one output row of K or V) */
} kvc_layer_t;

typedef struct kvc_params {
  int32_t dtype;
  int32_t batch;
  int32_t heads;
  int32_t head_dim;
  int32_t order;          /* enum kvc_order */
  int32_t algo;           /* enum kvc_algo  */
  int32_t phases;         /* OR of enum kvc_phase */
  int32_t external_index; /* 1: GATHER reads indices the caller wrote into the index region */
  int32_t flags;          /* OR of enum kvc_flag (other bits: KVC_E_ARG) */
  int32_t reserved;       /* must be 0 (else KVC_E_ARG) */
  uint32_t* device_status;/* optional device word for enum kvc_device_status bits (or NULL) */
} kvc_params_t;

typedef struct kvc_plan_info {
  size_t norm_offset;      /* workspace byte offset of the norm region                    */
  size_t index_offset;     /* workspace byte offset of the int32 index region             */
  size_t workspace_bytes;  /* total workspace the launch needs                              */
  int64_t norm_row_stride; /* elements (of dtype) per row in the norm region               */
  int64_t index_row_stride;/* int32 entries per row in the index region                   */
  int64_t rows;            /* num_layers * batch * heads                                   */
  int64_t score_tiles;     /* SCORE work items                                             */
  int64_t gather_units;    /* GATHER work items                                            */
} kvc_plan_info_t;

/* ABI/library identification. */
int kvc_version(void);
size_t kvc_layer_struct_size(void);
int kvc_max_zone_len(void);
const char* kvc_status_string(int status);
/* SHA-256 (hex) of the sources this library was compiled from (csrc/kvc.hip, csrc/kvc_common.h,
 * csrc/kvc_serial.h, include/kvc.h, in that order), or "unknown" for builds that do not set it --
 * lets a caller (and tests/test_abi.py) check that a shipped binary matches its source tree. */
const char* kvc_source_digest(void);

/* Validates the table, fills the kvc_plan() fields of every layer (host memory) and the
 * workspace layout.  Pure host function. */
int kvc_plan(const kvc_params_t* params, kvc_layer_t* layers, int num_layers,
             kvc_plan_info_t* info);

/* Launches the requested phases.  `layers` is the host table filled by kvc_plan(); the kernels
 * receive it by value in their kernel arguments (no copy is enqueued). */
int kvc_launch(const kvc_params_t* params, const kvc_layer_t* layers, int num_layers,
               void* workspace, size_t workspace_bytes, kvc_stream_t stream);

/* Convenience: kvc_plan + kvc_launch.  `layers` is updated in place. */
int kvc_compress(const kvc_params_t* params, kvc_layer_t* layers, int num_layers,
                 void* workspace, size_t workspace_bytes, kvc_stream_t stream);

/* Diagnostic entry (tests of the device status channel; no reference counterpart).  Runs the
 * 512-thread SELECT (params->phases == KVC_PHASE_SELECT) or SELECT_GATHER (KVC_PHASE_SELECT |
 * KVC_PHASE_GATHER) kernel of a planned table (at most 64 layers) as kvc_launch would, but with
 * the kernels' zone capacity set to `zone_cap` (a multiple of 64, <= 8192) instead of the
 * table's longest zone.  A row whose zone is longer than that capacity selects nothing, writes
 * no index and no K/V output row, and ORs KVC_DEV_SELECT_BOUNDS into params->device_status --
 * the path a dispatch bug would take.  kvc_launch itself always passes a sufficient capacity. */
int kvc_debug_select_capacity(const kvc_params_t* params, const kvc_layer_t* layers,
                              int num_layers, void* workspace, size_t workspace_bytes,
                              int zone_cap, kvc_stream_t stream);


/* ---------------------------------------------------------------------------------------------
 * h2o_attention heavy hitters (reference: kvcompress/methods/h2o_attention.py).  The reference's
 * H2OAttentionManager keeps per layer an accumulated attention tensor acc [B,H,len]:
 *   update_attention_scores (:84-153)  acc = (acc*decay, zero-extended | zeros) + attn.sum(dim=2)
 *   get_heavy_hitter_indices (:156-213) top-k of acc[:, :, m0:m1].sum(dim=1), sorted ascending
 * Both sums follow torch's CPU reduction order (aten cascade_sum: four-level cascade per column,
 * four interleaved lanes -- row_sum -- for the columns the SIMD loop leaves over, which depend on
 * the reference process's thread chunks: col_chunk below); the top-k is the reference-exact
 * std::nth_element / std::partial_sort set (KVC_ALGO_TOPK, descending).
 * ------------------------------------------------------------------------------------------- */
typedef struct kvc_attn_params {
  int32_t dtype;        /* enum kvc_dtype of attn / acc */
  int32_t batch;
  int32_t heads;
  int32_t vec_bytes;    /* SIMD width of the reference's CPU sum kernel: 32 on x86 (sum_stub has
                           no AVX512 variant) */
  float decay;          /* decay_factor as the fp32 value torch multiplies by (:136, :146) */
  int32_t flags;        /* kvc_heavy_hitters: 0 or KVC_ATTN_HH_STABLE.  kvc_attn_accumulate: 0, or
                           KVC_ATTN_OLD_DTYPE(d) when every layer's acc_old (old_len > 0 in every
                           layer) is of enum kvc_dtype d != dtype -- the reference then promotes
                           through `acc * decay`, torch.cat and `+` (:129-151): base is rounded to
                           d, and acc_new is FLOAT32 = fp32(base) + fp32(attn.sum), unrounded --
                           and/or KVC_ATTN_HH_STABLE, which it ignores (one struct per step) */
  uint32_t* device_status; /* optional, as kvc_params_t */
} kvc_attn_params_t;

#define KVC_ATTN_OLD_DTYPE(d) ((int32_t)(d) + 1) /* kvc_attn_params.flags, bits 0-1 */
/* kvc_attn_params.flags bit 2 (opt-in): kvc_heavy_hitters selects the first n_select of a STABLE
 * descending sort of the head sums (KVC_ALGO_STABLE's tie order) instead of torch.topk's; zones
 * of at most 65 536 positions (else KVC_E_TOO_LONG). */
#define KVC_ATTN_HH_STABLE 4

/* One layer of update_attention_scores (:100-154). */
typedef struct kvc_attn_layer {
  const void* attn;       /* [batch, heads, q_len, key_len], last dim contiguous */
  int64_t attn_stride[3]; /* element strides of batch, heads, q */
  const void* acc_old;    /* [batch, heads, old_len] contiguous (NULL when old_len == 0) */
  void* acc_new;          /* [batch, heads, key_len] contiguous, written */
  int32_t q_len;          /* >= 1 */
  int32_t key_len;        /* >= 1 */
  int32_t old_len;        /* 0: first update or reset (:118-123, :138-144); else <= key_len:
                             columns [0, old_len) carry acc_old * decay (:129-137, :145-146) */
  int32_t col_chunk;      /* columns per reference thread chunk of the q-sum; 0 = one chunk */
} kvc_attn_layer_t;

/* One layer of get_heavy_hitter_indices (:183-213). */
typedef struct kvc_hh_layer {
  const void* acc;        /* [batch, heads, acc_len] contiguous */
  int32_t acc_len;
  int32_t zone_start;     /* middle_start (:187) */
  int32_t zone_len;       /* middle_end - middle_start >= 1 (:188, :205) */
  int32_t n_select;       /* min(heavy_hitter_size, zone_len) (:206) */
  int32_t col_chunk;      /* columns per reference thread chunk of the head sum; 0 = one */
  int32_t reserved;       /* 0 */
} kvc_hh_layer_t;

/* acc_new of every layer (one kernel per chunk of layers). */
int kvc_attn_accumulate(const kvc_attn_params_t* params, const kvc_attn_layer_t* layers,
                        int num_layers, kvc_stream_t stream);

/* Workspace kvc_heavy_hitters needs for this table. */
int kvc_hh_workspace(const kvc_attn_params_t* params, const kvc_hh_layer_t* layers,
                     int num_layers, size_t* bytes);

/* Heavy hitters of every layer: row (layer*batch + b) of out_idx (int32, row stride
 * out_row_stride >= max n_select) receives the n_select ascending zone-local indices of
 * torch.topk(head_sum, n_select) (:198-211).  With out_idx = the index region of a
 * KVC_FLAG_SHARED_INDEX gather plan, kvc_launch then compacts K/V (:305-361). */
int kvc_heavy_hitters(const kvc_attn_params_t* params, const kvc_hh_layer_t* layers,
                      int num_layers, int32_t* out_idx, int64_t out_row_stride, void* workspace,
                      size_t workspace_bytes, kvc_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KVC_H */
