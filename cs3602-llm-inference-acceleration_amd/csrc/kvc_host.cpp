// kvc_host.cpp -- native host path of a repeated compress call (torch C++ extension).
//
// A per-token decode step calls the same compress function with the same shapes every token
// (reference kvcompress/evaluate.py:154-166), and for a fixed call shape the reference's per-layer
// branch logic (e.g. pyramid_kv.py:82-183) is a pure function of (kwargs, per-layer S).  The
// Python side (kvcompress/_engine.py, CallMemo) runs a call shape once through the method's own
// code, records what it did per layer -- input passed through, a dim-2 slice (view), or an engine
// output -- plus the planned engine launch, and from the next identical call on hands the layer
// list to this module, which in one C++ call
//   scan() : reads every layer's shape / dtype / device / contiguity / alignment into the memo key
//   run()  : fills the planned layer table's pointers, allocates the call's outputs (one
//            caching-allocator block, contiguous [B,H,n_out,D] views), enqueues kvc_launch on the
//            caller's stream and builds the result list (same objects, slices, outputs).
// No arithmetic happens here; the kernels and the ABI are libkvc.so's (include/kvc.h).
#include <hip/hip_runtime_api.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <cstring>
#include <map>
#include <vector>

#include "kvc.h"

namespace py = pybind11;

namespace {

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return KVC_BF16;
    case at::kHalf: return KVC_F16;
    case at::kFloat: return KVC_F32;
    default: return -1;
  }
}

bool as_tensor(PyObject* o, at::Tensor& out) {
  if (!THPVariable_Check(o)) return false;
  out = THPVariable_Unpack(o);
  return true;
}

// (K, V) of list item i, or false when it is not a 2-sequence of tensors
bool layer_of(PyObject* item, at::Tensor& k, at::Tensor& v) {
  if (!PyTuple_Check(item) && !PyList_Check(item)) return false;
  if (PySequence_Fast_GET_SIZE(item) != 2) return false;
  PyObject** it = PySequence_Fast_ITEMS(item);
  return as_tensor(it[0], k) && as_tensor(it[1], v);
}

bool plain(const at::Tensor& t, int64_t row_bytes) {
  return t.is_contiguous() && (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15u) == 0 &&
         row_bytes % 16 == 0;
}

}  // namespace

// (B, H, D, dtype, device, S_0 .. S_{L-1}) when every layer is a plain (K, V) pair on one ROCm
// device -- 4-D, K.shape == V.shape, one (B, H, D) and dtype (bf16 / fp16 / fp32), contiguous,
// 16-byte aligned rows -- else None (the call then takes the method's Python path).
py::object scan(py::list kv) {
  const Py_ssize_t n = PyList_GET_SIZE(kv.ptr());
  if (n == 0) return py::none();
  py::tuple sig(n + 5);
  int64_t B = -1, H = -1, D = -1;
  int dt = -1, dev = -1;
  at::Tensor k, v;
  for (Py_ssize_t i = 0; i < n; ++i) {
    if (!layer_of(PyList_GET_ITEM(kv.ptr(), i), k, v)) return py::none();
    if (k.dim() != 4 || !k.is_cuda() || !v.is_cuda() || k.sizes() != v.sizes() ||
        k.scalar_type() != v.scalar_type() || k.get_device() != v.get_device())
      return py::none();
    if (i == 0) {
      B = k.size(0), H = k.size(1), D = k.size(3);
      dt = dtype_code(k);
      dev = k.get_device();
      if (dt < 0) return py::none();
    } else if (k.size(0) != B || k.size(1) != H || k.size(3) != D || dtype_code(k) != dt ||
               k.get_device() != dev) {
      return py::none();
    }
    const int64_t rb = D * (int64_t)k.element_size();
    if (!plain(k, rb) || !plain(v, rb)) return py::none();
    sig[i + 5] = py::int_(k.size(2));
  }
  sig[0] = py::int_(B);
  sig[1] = py::int_(H);
  sig[2] = py::int_(D);
  sig[3] = py::int_(dt);
  sig[4] = py::int_(dev);
  return std::move(sig);
}

// The outputs of a recorded call (one caching-allocator block: all K outputs, then all V
// outputs) and its layer table with every pointer filled in.
struct Prepared {
  std::vector<at::Tensor> ko, vo;
  std::vector<kvc_layer_t> table;
};

Prepared prepare(PyObject* kv, const std::vector<at::Tensor>& ks, const std::vector<at::Tensor>& vs,
                 const py::detail::unchecked_reference<int64_t, 2>& act, int64_t table_addr,
                 int64_t n_jobs, const std::vector<int64_t>& n_outs) {
  const Py_ssize_t L = PyList_GET_SIZE(kv);
  Prepared o;
  o.ko.resize(n_jobs);
  o.vo.resize(n_jobs);
  if (n_jobs > 0) {
    std::vector<at::Tensor>& ko = o.ko;
    std::vector<at::Tensor>& vo = o.vo;
    const at::Tensor& k0 = ks[0];
    const int64_t B = k0.size(0), H = k0.size(1), D = k0.size(3);
    int64_t total = 0;
    for (int64_t j = 0; j < n_jobs; ++j) total += 2 * B * H * n_outs[j] * D;
    at::Tensor buf = at::empty({total}, k0.options());
    std::vector<kvc_layer_t>& table = o.table;
    table.resize(n_jobs);
    std::memcpy(table.data(), reinterpret_cast<const void*>(table_addr),
                sizeof(kvc_layer_t) * n_jobs);
    int64_t off = 0;
    for (int64_t j = 0; j < n_jobs; ++j) {  // all K outputs, then all V outputs
      const int64_t n = n_outs[j];
      ko[j] = buf.as_strided({B, H, n, D}, {H * n * D, n * D, D, 1}, off);
      off += B * H * n * D;
    }
    for (int64_t j = 0; j < n_jobs; ++j) {
      const int64_t n = n_outs[j];
      vo[j] = buf.as_strided({B, H, n, D}, {H * n * D, n * D, D, 1}, off);
      off += B * H * n * D;
    }
    for (Py_ssize_t i = 0; i < L; ++i) {
      if (act(i, 0) != 2) continue;
      const int64_t j = act(i, 1);
      if (j < 0 || j >= n_jobs) throw std::invalid_argument("kvc_host: bad job index");
      table[j].k = ks[i].data_ptr();
      table[j].v = vs[i].data_ptr();
      table[j].k_out = ko[j].data_ptr();
      table[j].v_out = vo[j].data_ptr();
    }
  }
  return o;
}

void launch(const Prepared& o, int64_t params_addr, int64_t ws, int64_t ws_bytes,
            int64_t stream) {
  if (o.table.empty()) return;
  const int rc = kvc_launch(reinterpret_cast<const kvc_params_t*>(params_addr), o.table.data(),
                            (int)o.table.size(), reinterpret_cast<void*>(ws), (size_t)ws_bytes,
                            reinterpret_cast<kvc_stream_t>(stream));
  if (rc != KVC_OK)
    throw std::runtime_error(std::string("kvc_launch failed: ") + kvc_status_string(rc));
}

// The result list of a recorded call: per layer the input itself, a dim-2 slice, or its outputs.
py::list result_list(PyObject* kv, const std::vector<at::Tensor>& ks,
                     const std::vector<at::Tensor>& vs,
                     const py::detail::unchecked_reference<int64_t, 2>& act, const Prepared& o) {
  const Py_ssize_t L = PyList_GET_SIZE(kv);
  const std::vector<at::Tensor>& ko = o.ko;
  const std::vector<at::Tensor>& vo = o.vo;
  py::list out(L);
  for (Py_ssize_t i = 0; i < L; ++i) {
    const int64_t a = act(i, 0);
    if (a == 0) {
      out[i] = py::reinterpret_borrow<py::object>(PyList_GET_ITEM(kv, i));
    } else if (a == 1) {
      const int64_t s = act(i, 1), len = act(i, 2);
      out[i] = py::make_tuple(ks[i].slice(2, s, s + len), vs[i].slice(2, s, s + len));
    } else {
      const int64_t j = act(i, 1);
      out[i] = py::make_tuple(ko[j], vo[j]);
    }
  }
  return out;
}

void unpack_layers(PyObject* kv, std::vector<at::Tensor>& ks, std::vector<at::Tensor>& vs) {
  const Py_ssize_t L = PyList_GET_SIZE(kv);
  ks.resize(L);
  vs.resize(L);
  for (Py_ssize_t i = 0; i < L; ++i)
    if (!layer_of(PyList_GET_ITEM(kv, i), ks[i], vs[i]))
      throw std::invalid_argument("kvc_host: layer is not a (K, V) pair");
}

// Replays a recorded call on a list that scan() matched to it.
//   actions : int64 [L, 3] -- (0, -, -) the input pair itself; (1, start, len) K/V[:, :, start:
//             start+len] (views); (2, job, -) the engine outputs of table row `job`
//   table   : address of the planned kvc_layer_t rows (pointer columns are filled here), count
//   n_outs  : output rows of each table row
//   params  : address of the kvc_params_t the plan was made with
py::list run(py::list kv, py::array_t<int64_t, py::array::c_style> actions, int64_t table_addr,
             int64_t n_jobs, std::vector<int64_t> n_outs, int64_t params_addr, int64_t ws,
             int64_t ws_bytes, int64_t stream) {
  const Py_ssize_t L = PyList_GET_SIZE(kv.ptr());
  auto act = actions.unchecked<2>();
  if (act.shape(0) != L || act.shape(1) != 3 || (int64_t)n_outs.size() != n_jobs)
    throw std::invalid_argument("kvc_host.run: recorded call does not match the layer list");
  std::vector<at::Tensor> ks, vs;
  unpack_layers(kv.ptr(), ks, vs);
  const Prepared o = prepare(kv.ptr(), ks, vs, act, table_addr, n_jobs, n_outs);
  launch(o, params_addr, ws, ws_bytes, stream);
  return result_list(kv.ptr(), ks, vs, act, o);
}

// Per device: a second stream and two events (no timing, no system fence) with which run_h2o
// copies the selection-independent output rows beside the heavy-hitter selection.  Created on
// first use, kept for the life of the process.
struct SideStream {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

const SideStream& side_stream() {
  static std::map<int, SideStream> per_device;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("kvc_host: hipGetDevice failed");
  SideStream& s = per_device[dev];
  if (!s.side) {
    const unsigned ef = hipEventDisableTiming | hipEventDisableSystemFence;
    if (hipStreamCreateWithFlags(&s.side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s.fork, ef) != hipSuccess ||
        hipEventCreateWithFlags(&s.join, ef) != hipSuccess)
      throw std::runtime_error("kvc_host: side stream / event creation failed");
  }
  return s;
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("kvc_host: ") + what + " failed");
}

// ---- h2o_attention (reference kvcompress/methods/h2o_attention.py:84-363) ---------------------
// A decode step of h2o_attention_compress with a manager is three engine calls: accumulate the
// new attention rows (:84-153), the heavy hitters of every layer (:156-213) written into the
// index region of a shared-index gather plan, and that gather (:305-361).  For a repeated call
// shape the tables are fixed up to their pointers; kvcompress/methods/h2o_attention.py plans
// them and these two functions key and replay them.

// Memo key of (kv, attention, accumulated) -- scan(kv), then per attention layer (dtype, B, H, q,
// k, strides 0..2, device) or -1 when it is None, then per accumulated tensor (dtype, shape,
// device) or -1 -- or None when an input needs the Python path (a layer that is not a plain
// tensor pair, an attention row that is not last-dim contiguous and element aligned, a
// non-contiguous accumulated tensor).
py::object scan_h2o(py::list kv, py::object attns, py::list accs) {
  py::object base = scan(kv);
  if (base.is_none()) return py::none();
  PyObject* seq = PySequence_Fast(attns.ptr(), "attention_scores must be a sequence");
  if (!seq) throw py::error_already_set();
  py::object hold = py::reinterpret_steal<py::object>(seq);
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  if (PyList_GET_SIZE(accs.ptr()) != n) return py::none();
  std::vector<int64_t> sig;
  sig.reserve(n * 15);
  at::Tensor t;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* o = PySequence_Fast_GET_ITEM(seq, i);
    if (o == Py_None) {
      sig.push_back(-1);
      continue;
    }
    if (!as_tensor(o, t) || t.dim() != 4 || !t.is_cuda() || dtype_code(t) < 0 ||
        t.stride(3) != 1 || reinterpret_cast<uintptr_t>(t.data_ptr()) % t.element_size())
      return py::none();
    sig.insert(sig.end(), {dtype_code(t), t.size(0), t.size(1), t.size(2), t.size(3),
                           t.stride(0), t.stride(1), t.stride(2), (int64_t)t.get_device()});
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* o = PyList_GET_ITEM(accs.ptr(), i);
    if (o == Py_None) {
      sig.push_back(-1);
      continue;
    }
    if (!as_tensor(o, t) || t.dim() != 3 || !t.is_cuda() || !t.is_contiguous())
      return py::none();
    sig.insert(sig.end(), {dtype_code(t), t.size(0), t.size(1), t.size(2),
                           (int64_t)t.get_device()});
  }
  py::tuple b = base.cast<py::tuple>();
  py::tuple out(b.size() + sig.size());
  for (size_t i = 0; i < b.size(); ++i) out[i] = b[i];
  for (size_t i = 0; i < sig.size(); ++i) out[b.size() + i] = py::int_(sig[i]);
  return std::move(out);
}

// Replays a planned h2o_attention step on inputs scan_h2o() matched to it.
//   a_layers : attention layer of each kvc_attn_layer_t row of the planned table at a_table (the
//              pointer columns are filled here: attn, acc_old of rows with old_len > 0, and
//              acc_new -- views of one fresh allocation, returned)
//   hh_rows  : accumulate row whose acc_new each kvc_hh_layer_t row of hh_table reads
//   idx, idx_stride : the gather plan's index region, where kvc_heavy_hitters writes
//   the rest : as run()
// Returns (result list, [acc_new of each accumulate row]).
//   fixed_params, sel_params : when non-zero, the gather runs as two launches (kvc_params with
//              KVC_FLAG_GATHER_FIXED / _SELECTED): the sink and recent rows on a side stream,
//              forked from `stream` after the accumulate (which they would slow down) and joined
//              after the selected rows' launch, so they copy while the heavy hitters are selected
py::tuple run_h2o(py::list kv, py::object attns, py::list accs, std::vector<int64_t> a_layers,
                  int64_t a_table, int64_t a_params, std::vector<int64_t> hh_rows,
                  int64_t hh_table, int64_t hh_ws, int64_t hh_ws_bytes, int64_t idx,
                  int64_t idx_stride, py::array_t<int64_t, py::array::c_style> actions,
                  int64_t table_addr, int64_t n_jobs, std::vector<int64_t> n_outs,
                  int64_t params_addr, int64_t ws, int64_t ws_bytes, int64_t stream,
                  int64_t fixed_params, int64_t sel_params) {
  const Py_ssize_t L = PyList_GET_SIZE(kv.ptr());
  auto act = actions.unchecked<2>();
  if (act.shape(0) != L || act.shape(1) != 3 || (int64_t)n_outs.size() != n_jobs ||
      a_layers.empty() || (fixed_params == 0) != (sel_params == 0))
    throw std::invalid_argument("kvc_host.run_h2o: recorded call does not match the inputs");
  std::vector<at::Tensor> ks, vs;
  unpack_layers(kv.ptr(), ks, vs);
  const Prepared o = prepare(kv.ptr(), ks, vs, act, table_addr, n_jobs, n_outs);
  const hipStream_t main = reinterpret_cast<hipStream_t>(stream);
  const SideStream* side = nullptr;
  PyObject* seq = PySequence_Fast(attns.ptr(), "attention_scores must be a sequence");
  if (!seq) throw py::error_already_set();
  py::object hold = py::reinterpret_steal<py::object>(seq);
  const Py_ssize_t n_att = PySequence_Fast_GET_SIZE(seq);
  const size_t na = a_layers.size();
  std::vector<kvc_attn_layer_t> at(na);
  std::memcpy(at.data(), reinterpret_cast<const void*>(a_table), sizeof(kvc_attn_layer_t) * na);
  std::vector<at::Tensor> att(na);
  int64_t total = 0;
  for (size_t r = 0; r < na; ++r) {
    const int64_t li = a_layers[r];
    if (li < 0 || li >= n_att || !as_tensor(PySequence_Fast_GET_ITEM(seq, li), att[r]))
      throw std::invalid_argument("kvc_host.run_h2o: attention layer is not a tensor");
    total += att[r].size(0) * att[r].size(1) * (int64_t)at[r].key_len;
  }
  at::Tensor buf = at::empty({total}, att[0].options());
  py::list acc_out(na);
  std::vector<at::Tensor> acc_new(na);
  int64_t off = 0;
  at::Tensor old;
  for (size_t r = 0; r < na; ++r) {
    const int64_t B = att[r].size(0), H = att[r].size(1), k = at[r].key_len;
    acc_new[r] = buf.as_strided({B, H, k}, {H * k, k, 1}, off);
    off += B * H * k;
    at[r].attn = att[r].data_ptr();
    at[r].acc_new = acc_new[r].data_ptr();
    at[r].acc_old = nullptr;
    if (at[r].old_len > 0) {
      if (!as_tensor(PyList_GET_ITEM(accs.ptr(), a_layers[r]), old))
        throw std::invalid_argument("kvc_host.run_h2o: accumulated attention missing");
      at[r].acc_old = old.data_ptr();
    }
    acc_out[r] = acc_new[r];
  }
  int rc = kvc_attn_accumulate(reinterpret_cast<const kvc_attn_params_t*>(a_params), at.data(),
                               (int)na, reinterpret_cast<kvc_stream_t>(stream));
  if (rc != KVC_OK)
    throw std::runtime_error(std::string("kvc_attn_accumulate failed: ") + kvc_status_string(rc));
  // Joins the side stream back into `main` on every exit path once the side copy is enqueued:
  // if a later launch throws, the outputs it writes are freed to the caching allocator (on
  // `main`) only after the copy has finished.
  struct Join {
    const SideStream* s = nullptr;
    hipStream_t main;
    bool armed = false;
    void operator()() {
      if (!armed) return;
      armed = false;
      check_hip(hipEventRecord(s->join, s->side), "hipEventRecord");
      check_hip(hipStreamWaitEvent(main, s->join, 0), "hipStreamWaitEvent");
    }
    ~Join() {
      if (armed) {  // unwinding: best effort, never throw from a destructor
        (void)hipEventRecord(s->join, s->side);
        (void)hipStreamWaitEvent(main, s->join, 0);
      }
    }
  } join;
  join.main = main;
  if (fixed_params && !o.table.empty()) {  // the sink / recent rows, beside the heavy hitters
    side = &side_stream();
    join.s = side;
    check_hip(hipEventRecord(side->fork, main), "hipEventRecord");
    check_hip(hipStreamWaitEvent(side->side, side->fork, 0), "hipStreamWaitEvent");
    join.armed = true;
    launch(o, fixed_params, ws, ws_bytes, reinterpret_cast<int64_t>(side->side));
  }
  const size_t nh = hh_rows.size();
  std::vector<kvc_hh_layer_t> ht(nh);
  std::memcpy(ht.data(), reinterpret_cast<const void*>(hh_table), sizeof(kvc_hh_layer_t) * nh);
  for (size_t j = 0; j < nh; ++j) {
    if (hh_rows[j] < 0 || hh_rows[j] >= (int64_t)na)
      throw std::invalid_argument("kvc_host.run_h2o: bad heavy-hitter row");
    ht[j].acc = acc_new[hh_rows[j]].data_ptr();
  }
  rc = kvc_heavy_hitters(reinterpret_cast<const kvc_attn_params_t*>(a_params), ht.data(), (int)nh,
                         reinterpret_cast<int32_t*>(idx), idx_stride,
                         reinterpret_cast<void*>(hh_ws), (size_t)hh_ws_bytes,
                         reinterpret_cast<kvc_stream_t>(stream));
  if (rc != KVC_OK)
    throw std::runtime_error(std::string("kvc_heavy_hitters failed: ") + kvc_status_string(rc));
  launch(o, side ? sel_params : params_addr, ws, ws_bytes, stream);
  join();
  return py::make_tuple(result_list(kv.ptr(), ks, vs, act, o), acc_out);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "kvcompress native host path (scan / run of a recorded compress call)";
  m.def("scan", &scan, "memo key of a plain (K, V) layer list, or None");
  m.def("run", &run, "replay a recorded compress call: one kvc_launch, outputs, result list");
  m.def("scan_h2o", &scan_h2o, "memo key of an h2o_attention step's inputs, or None");
  m.def("run_h2o", &run_h2o, "replay a planned h2o_attention step: accumulate, heavy hitters, "
        "gather");
}
