// Bindings of the one-sided threshold lane (transport/onesided.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../kernels/onesided_kernels.h"
#include "../transport/onesided.h"

namespace py = pybind11;

namespace akka {

namespace {
// Minimal DLPack (v0.x ABI) to hand a window row to torch without a copy.
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;

// The tensor holds a strong reference to the Python object that owns the lane
// (manager_ctx): a window row handed to torch keeps the lane -- and so the
// window memory -- alive after the allreduce object is dropped.  torch may free
// the tensor on a thread without the GIL.
void dl_delete(DLManagedTensor* t) {
  delete[] t->dl_tensor.shape;
  if (t->manager_ctx != nullptr && Py_IsInitialized() && !_Py_IsFinalizing()) {  // (at exit: leak, never block)
    const PyGILState_STATE g = PyGILState_Ensure();
    Py_DECREF(static_cast<PyObject*>(t->manager_ctx));
    PyGILState_Release(g);
  }
  delete t;
}

// A capsule over device memory the lane owns; `owner` is kept alive by it.
py::capsule window_capsule(void* data, int32_t device, int64_t n, bool bf16, const py::object& owner) {
  auto* t = new DLManagedTensor();
  t->dl_tensor.data = data;
  t->dl_tensor.device = {kDLROCM, device};
  t->dl_tensor.ndim = 1;
  t->dl_tensor.dtype = bf16 ? DLDataType{4, 16, 1} : DLDataType{2, 32, 1};
  t->dl_tensor.shape = new int64_t[1]{n};
  t->dl_tensor.strides = nullptr;
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = owner.inc_ref().ptr();
  t->deleter = dl_delete;
  return py::capsule(t, "dltensor", [](PyObject* cap) {
    // consumed capsules are renamed "used_dltensor" (the consumer owns them)
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* m = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}
const char* kStatNames[] = {
    "rounds",           "skipped_rounds",     "scatter_pushed",  "scatter_outdated", "scatter_conflict",
    "gather_pushed",    "gather_outdated",    "gather_conflict", "reduce_threshold", "reduce_forced",
    "complete_threshold", "complete_forced",  "timeouts",        "landed_chunks",    "missing_chunks",
    "dead_skips",       "reduce_contribs",    "reduce_abandoned",
};
const char* kReasons[] = {"wait", "threshold", "unreachable", "catch_up", "host_force", "timeout", "abandoned"};
}  // namespace

void bind_onesided(py::module_& m) {
  py::class_<OneSidedLane>(m, "OneSidedLane")
      .def(py::init([](int32_t device, int64_t S, int32_t N, int64_t C, int32_t me, const std::string& dtype,
                       float th_reduce, float th_complete, int32_t max_lag, int32_t rows, int64_t part_bytes,
                       int64_t timeout_ms, int32_t threads, int32_t role_wgs, int32_t cu_keep, bool fenced,
                       bool window_output) {
             OneSidedParams p;
             p.th_reduce = th_reduce;
             p.th_complete = th_complete;
             p.max_lag = max_lag;
             p.rows = rows;
             p.part_bytes = part_bytes;
             p.timeout_ms = timeout_ms;
             p.threads = threads;
             p.role_wgs = role_wgs;
             p.cu_keep = cu_keep;
             p.fenced = fenced;
             p.window_output = window_output;
             const DType dt = (dtype == "bfloat16" || dtype == "bf16") ? DType::BF16 : DType::F32;
             return std::make_unique<OneSidedLane>(device, S, N, C, me, dt, p);
           }),
           py::arg("device"), py::arg("S"), py::arg("N"), py::arg("C"), py::arg("me"), py::arg("dtype") = "float32",
           py::arg("th_reduce") = 1.f, py::arg("th_complete") = 1.f, py::arg("max_lag") = 1, py::arg("rows") = 0,
           py::arg("part_bytes") = 0, py::arg("timeout_ms") = 30000, py::arg("threads") = 256,
           py::arg("role_wgs") = 0, py::arg("cu_keep") = 0, py::arg("fenced") = false,
           py::arg("window_output") = false)
      .def("gather_row_dlpack",
           [](py::object self, int32_t row, const std::string& dtype, int32_t device) {
             const auto& l = self.cast<const OneSidedLane&>();
             AKKA_CHECK(l.on_gpu() && l.window_output(), "onesided lane: no window output");
             AKKA_CHECK(row >= 0 && row < l.rows(), "onesided lane: no such row");
             return window_capsule(l.gather_row(row), device, l.geometry().S, dtype == "bfloat16", self);
           })
      .def("set_fenced", &OneSidedLane::set_fenced)
      .def_property_readonly("fenced", &OneSidedLane::fenced)
      .def("handle", [](const OneSidedLane& l) { return py::bytes(l.handle()); })
      .def("timeline", [](OneSidedLane& l) {
        std::vector<uint64_t> v;
        {
          py::gil_scoped_release nogil;
          v = l.timeline();
        }
        return v;
      })
      .def("open", [](OneSidedLane& l, std::vector<std::string> handles) {
        py::gil_scoped_release nogil;
        l.open(handles);
      })
      .def("unlink", &OneSidedLane::unlink)
      .def("add_peer",
           [](OneSidedLane& l, int32_t q, py::bytes h) {
             std::string hs(h);
             py::gil_scoped_release nogil;
             l.add_peer(q, hs);
           })
      .def("members", &OneSidedLane::members)
      .def("round",
           [](OneSidedLane& l, uintptr_t stream, uintptr_t in, uintptr_t out, uintptr_t counts, int32_t kcols) {
             py::gil_scoped_release nogil;  // the CPU backend waits for other processes
             return l.round(stream, reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out),
                            reinterpret_cast<int32_t*>(counts), kcols);
           })
      .def("status",
           [](const OneSidedLane& l, int64_t call) {
             const os::CallStatus c = l.status(call);
             py::dict d;
             d["call"] = call;
             d["round"] = c.round;
             d["reason"] = c.round >= 0 && c.reason >= 0 && c.reason < 7 ? kReasons[c.reason] : "pending";
             d["landed_chunks"] = c.landed_chunks;
             d["forced_chunks"] = c.forced_chunks;
             return d;
           })
      .def("stats",
           [](OneSidedLane& l) {
             std::vector<uint64_t> v;
             {
               py::gil_scoped_release nogil;
               v = l.stats();
             }
             py::dict d;
             for (size_t i = 0; i < sizeof(kStatNames) / sizeof(kStatNames[0]); ++i) d[kStatNames[i]] = v[i];
             return d;
           })
      .def("cu_stream", &OneSidedLane::cu_stream)
      .def("stats_nowait",
           [](OneSidedLane& l) {
             std::vector<uint64_t> v;
             {
               py::gil_scoped_release nogil;
               v = l.stats_nowait();
             }
             py::dict d;
             for (size_t i = 0; i < sizeof(kStatNames) / sizeof(kStatNames[0]); ++i) d[kStatNames[i]] = v[i];
             return d;
           })
      .def("peek_flags",
           [](OneSidedLane& l) {
             py::gil_scoped_release nogil;
             return l.peek_flags();
           })
      .def("peek_part",
           [](OneSidedLane& l, int32_t phase, int32_t row, int32_t src, int32_t k, int32_t j) {
             std::string s;
             {
               py::gil_scoped_release nogil;
               s = l.peek_part(phase, row, src, k, j);
             }
             return py::bytes(s);
           })
      .def("begin",
           [](OneSidedLane& l, uintptr_t in, uintptr_t out, uintptr_t counts, int32_t kcols) {
             return l.begin(reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out),
                            reinterpret_cast<int32_t*>(counts), kcols);
           })
      .def("progress", &OneSidedLane::progress)
      .def("active", &OneSidedLane::active)
      .def("set_hold", &OneSidedLane::set_hold)
      .def("outbox",
           [](const OneSidedLane& l) {
             py::list out;
             for (const auto& e : l.outbox()) {
               py::dict d;
               d["phase"] = e[0] == 0 ? "scatter" : "gather";
               d["dst"] = e[1];
               d["chunk"] = e[2];
               d["part"] = e[3];
               d["round"] = e[4];
               d["count"] = e[5];
               out.append(d);
             }
             return out;
           })
      .def("deliver", &OneSidedLane::deliver)
      .def("outbox_bytes", [](const OneSidedLane& l, int64_t i) { return py::bytes(l.outbox_bytes(i)); })
      .def("inject",
           [](OneSidedLane& l, int32_t phase, int32_t dst, int32_t k, int32_t j, uint32_t r, uint32_t cnt,
              py::bytes data, int32_t stage) { l.inject(phase, dst, k, j, r, cnt, std::string(data), stage); },
           py::arg("phase"), py::arg("dst"), py::arg("chunk"), py::arg("part"), py::arg("round"),
           py::arg("count") = 0, py::arg("data") = py::bytes(""), py::arg("stage") = 0)
      .def("drop", &OneSidedLane::drop)
      .def("note_replays", &OneSidedLane::note_replays)
      .def("error", &OneSidedLane::error)
      .def("clear_error", &OneSidedLane::clear_error)
      .def("set_dead", &OneSidedLane::set_dead)
      .def("force_below", &OneSidedLane::force_below)
      .def("retire", &OneSidedLane::retire, py::arg("stream") = 0)
      .def("info", [](const OneSidedLane& l) {
        py::dict d;
        d["backend"] = l.on_gpu() ? "gpu" : "cpu";
        d["rows"] = l.rows();
        d["parts"] = l.parts();
        d["part_elems"] = l.part_elems();
        d["need_reduce"] = l.need_reduce();
        d["need_complete"] = l.need_complete();
        d["window_bytes"] = int64_t(l.window_bytes());
        d["memory"] = l.memory_kind();
        d["calls"] = l.calls();
        d["total_chunks"] = l.geometry().total_chunks();
        d["threads"] = l.threads();
        d["ranks_on_this_gpu"] = l.shared_ranks();
        d["lane_cus"] = l.lane_cus();
        d["clock_khz"] = l.clock_khz();
        d["pieces_per_part"] = l.pieces();
        d["handoff"] = l.fenced() ? "fenced" : "lite";
        d["window_output"] = l.window_output();
        const auto g = l.role_grid();
        d["role_wgs"] = py::dict(py::arg("push") = g[0], py::arg("reduce") = g[1], py::arg("copy") = g[2]);
        return d;
      });
  m.def("onesided_layout", [](int32_t N, int32_t D, int32_t Kmax, int32_t P) {
    // every exported / local word index of the layout (CPU test: disjoint, in range)
    os::Layout L;
    L.init(N, D, Kmax, P);
    std::vector<int64_t> exported, local;
    for (int32_t d = 0; d < D; ++d)
      for (int32_t s = 0; s < N; ++s)
        for (int32_t k = 0; k < Kmax; ++k)
          for (int32_t j = 0; j < P; ++j) {
            exported.push_back(L.stag(d, s, k, j));
            exported.push_back(L.stag(d, s, k, j) + 1);
            exported.push_back(L.gtag(d, s, k, j));
            exported.push_back(L.gtag(d, s, k, j) + 1);
          }
    for (int32_t d = 0; d < D; ++d) {
      for (int32_t k = 0; k < Kmax; ++k) {
        exported.push_back(L.fired(d, k));
        exported.push_back(L.sread(d, k));
      }
      exported.push_back(L.gread(d));
    }
    for (int32_t k = 0; k < Kmax; ++k) {
      local.push_back(L.dec(k));
      local.push_back(L.dec(k) + 1);
      local.push_back(L.kctr(k));
      local.push_back(L.odone(k));
      for (int32_t j = 0; j < P; ++j) {
        local.push_back(L.okq(k, j));
        local.push_back(L.pctr(k, j));
        local.push_back(L.pdone(k, j));
      }
    }
    exported.push_back(L.done());
    for (int32_t s = 0; s < N; ++s) {
      exported.push_back(L.seen(s));
      exported.push_back(L.fin(s));
    }
    for (int32_t b = 0; b < N; ++b)
      for (int32_t k = 0; k < Kmax; ++k) local.push_back(L.cmask(b, k));
    for (int32_t i = 0; i < os::Layout::kStateWords; ++i) local.push_back(L.state(i));
    py::dict r;
    r["exported"] = exported;
    r["local"] = local;
    r["flag_words"] = L.flag_words;
    r["local_words"] = L.local_words;
    return r;
  });
  m.def("onesided_rules", [](uint32_t t, uint32_t r) { return os::tag_state(t, r); });
  m.def("onesided_completion_verdict", &os::completion_verdict);
  m.def(
      "onesided_reduce_role_bench",
      [](int32_t N, int64_t block, int64_t chunk, int64_t part, int32_t nsub, const std::string& dtype,
         int32_t threads, int32_t grid, int32_t iters, int32_t device) {
        py::gil_scoped_release nogil;
        return os::onesided_reduce_role_bench(N, block, chunk, part, nsub, dtype == "float32" ? 0 : 1, threads, grid,
                                              iters, device);
      },
      py::arg("N"), py::arg("block"), py::arg("chunk"), py::arg("part"), py::arg("nsub"), py::arg("dtype") = "float32",
      py::arg("threads") = 1024, py::arg("grid") = 256, py::arg("iters") = 10, py::arg("device") = 0);
  m.def("onesided_evaluate", &os::evaluate);
  m.def("onesided_select_round", &os::select_round);
}

}  // namespace akka
