// Diagnostic bindings: raw IPC export / open of one allocation of a chosen
// kind and size (scripts/ipc_open_ab.py: which allocations hipIpcOpenMemHandle
// opens, and how long it takes).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cstring>
#include <string>

#include "../engine/common.h"
#include "../kernels/ipc_kernels.h"
#include "../transport/link_probe.h"

namespace py = pybind11;

namespace akka {

namespace {
void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw AkkaError(std::string("akka probe: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

void bind_probe(py::module_& m) {
  py::class_<LinkProbe>(m, "LinkProbe")
      .def(py::init<int32_t, int32_t, int32_t, int64_t>(), py::arg("device"), py::arg("rank"), py::arg("nranks"),
           py::arg("bytes"))
      .def("handle", [](const LinkProbe& p) { return py::bytes(p.handle()); })
      .def("open", &LinkProbe::open)
      .def("unlink", &LinkProbe::unlink)
      .def("bytes", &LinkProbe::bytes)
      .def("push", [](LinkProbe& p, std::vector<int32_t> peers, int32_t iters) {
        py::gil_scoped_release nogil;
        return p.push(peers, iters);
      })
      .def("pull", [](LinkProbe& p, std::vector<int32_t> peers, int32_t iters) {
        py::gil_scoped_release nogil;
        return p.pull(peers, iters);
      });
  m.def("ipc_probe_export", [](int32_t device, int64_t bytes, const std::string& kind) {
    check(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    if (kind == "fine") check(hipExtMallocWithFlags(&p, size_t(bytes), hipDeviceMallocFinegrained), "alloc fine");
    else if (kind == "uncached") check(hipExtMallocWithFlags(&p, size_t(bytes), hipDeviceMallocUncached), "alloc uncached");
    else if (kind == "coarse") check(hipMalloc(&p, size_t(bytes)), "hipMalloc");
    else throw AkkaError("akka probe: kind must be fine, uncached or coarse");
    check(hipMemset(p, 0x5a, size_t(bytes)), "hipMemset");
    check(hipDeviceSynchronize(), "sync");
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
    return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), reinterpret_cast<uintptr_t>(p));
  });
  m.def("ipc_probe_open", [](int32_t device, py::bytes handle) {
    std::string s = handle;
    AKKA_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "probe: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, s.data(), sizeof(h));
    check(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    {
      py::gil_scoped_release nogil;
      check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    }
    const double s_open = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    unsigned char b = 0;
    check(hipMemcpy(&b, p, 1, hipMemcpyDeviceToHost), "read back");
    return py::make_tuple(reinterpret_cast<uintptr_t>(p), s_open, int(b));
  });
  m.def("ipc_reduce_role_bench", [](int32_t N, int64_t block, int64_t portion_bytes, const std::string& dtype,
                                    bool plain, int32_t iters, int32_t threads, int32_t device, const std::string& kind,
                                    bool lite, int32_t max_wgs) {
    const int32_t wk = kind == "coarse" ? 1 : kind == "uncached" ? 2 : 0;
    py::gil_scoped_release nogil;
    return ipc_reduce_role_bench(N, block, portion_bytes, dtype == "bfloat16" ? DType::BF16 : DType::F32, plain, iters,
                                 threads, device, wk, lite, max_wgs);
  }, py::arg("N"), py::arg("block"), py::arg("portion_bytes") = int64_t(512) << 10, py::arg("dtype") = "float32",
     py::arg("plain") = false, py::arg("iters") = 20, py::arg("threads") = 256, py::arg("device") = 0,
     py::arg("kind") = "fine", py::arg("lite") = false, py::arg("max_wgs") = 1024);
  m.def("ipc_probe_close", [](uintptr_t p) { check(hipIpcCloseMemHandle(reinterpret_cast<void*>(p)), "close"); });
  m.def("ipc_probe_free", [](uintptr_t p) { check(hipFree(reinterpret_cast<void*>(p)), "free"); });
}

}  // namespace akka
