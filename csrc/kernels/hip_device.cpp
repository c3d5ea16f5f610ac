// HIP implementation of the Device interface (MI355X, gfx950).
//
// Two streams per worker: `comm` carries the RCCL groups (and the counts
// upload), `compute` the chunk reduces and copies; they synchronise through
// events only, so a reduce of chunk k overlaps the xGMI transfer of step k+1.
// Pinned staging memory is hipHostMalloc'd.  Reduce launches of consecutive
// chunks with identical source layouts are merged before launch (a worker
// whose whole round is self-contained, e.g. N=1, issues ONE kernel per round).
#include <hip/hip_runtime.h>

#include <mutex>

#include "../engine/device.h"
#include "kernels.h"

namespace akka {

#define AKKA_HIP(call)                                                                        \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      throw AkkaError(std::string("akka: ") + #call + " failed: " + hipGetErrorString(e_));   \
  } while (0)

namespace {

class HipDevice final : public Device {
 public:
  HipDevice(int32_t dev, bool high_priority_comm) : dev_(dev) {
    AKKA_HIP(hipSetDevice(dev));
    int lo = 0, hi = 0;
    AKKA_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    AKKA_HIP(hipStreamCreateWithPriority(&comm_, hipStreamNonBlocking, high_priority_comm ? hi : lo));
    AKKA_HIP(hipStreamCreateWithPriority(&compute_, hipStreamNonBlocking, lo));
    impl_ = reduce_impl_from_env();
  }
  ~HipDevice() override {
    hipSetDevice(dev_);
    hipStreamSynchronize(comm_);
    hipStreamSynchronize(compute_);
    if (exported_) return;  // see Device::mark_streams_exported
    hipStreamDestroy(comm_);
    hipStreamDestroy(compute_);
  }
  void mark_streams_exported() override { exported_ = true; }

  bool is_host() const override { return false; }
  int32_t device_index() const override { return dev_; }

  void* alloc(size_t bytes) override {
    void* p = nullptr;
    AKKA_HIP(hipSetDevice(dev_));
    AKKA_HIP(hipMalloc(&p, bytes ? bytes : 16));
    return p;
  }
  void release(void* p) override {
    if (p) hipFree(p);
  }
  void* alloc_pinned(size_t bytes) override {
    void* p = nullptr;
    AKKA_HIP(hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault));
    return p;
  }
  void release_pinned(void* p) override {
    if (p) hipHostFree(p);
  }

  StreamH comm_stream() override { return comm_; }
  StreamH compute_stream() override { return compute_; }
  StreamH create_stream() override {
    // Normal priority on purpose: HIP serves high-priority streams from a
    // small pool of hardware queues, and a per-peer stream parked on a peer
    // (p2p waiting for a straggler) must not share a queue with other streams.
    AKKA_HIP(hipSetDevice(dev_));
    hipStream_t s;
    AKKA_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return s;
  }
  void destroy_stream(StreamH s) override {
    flush_if(s);
    hipStreamSynchronize(static_cast<hipStream_t>(s));
    hipStreamDestroy(static_cast<hipStream_t>(s));
  }

  EventH create_event() override {
    hipEvent_t e;
    AKKA_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }
  void destroy_event(EventH e) override { hipEventDestroy(static_cast<hipEvent_t>(e)); }
  void record(EventH e, StreamH s) override {
    flush_if(s);
    AKKA_HIP(hipEventRecord(static_cast<hipEvent_t>(e), static_cast<hipStream_t>(s)));
  }
  void wait(StreamH s, EventH e) override {
    flush_if(s);
    // An event that already completed needs no barrier packet on the stream
    // (each cross-stream wait costs the command processor several us).  Not
    // while capturing: an event recorded inside the capture has no eager
    // record, so it would read as complete and the graph would lose an edge.
    if (!capturing_ && hipEventQuery(static_cast<hipEvent_t>(e)) == hipSuccess) return;
    AKKA_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e), 0));
  }
  bool query(EventH e) override {
    flush_all();
    hipError_t r = hipEventQuery(static_cast<hipEvent_t>(e));
    if (r == hipSuccess) return true;
    if (r == hipErrorNotReady) return false;
    AKKA_HIP(r);
    return false;
  }
  void sync_event(EventH e) override {
    flush_all();
    AKKA_HIP(hipEventSynchronize(static_cast<hipEvent_t>(e)));
  }
  void sync_stream(StreamH s) override {
    flush_if(s);
    AKKA_HIP(hipStreamSynchronize(static_cast<hipStream_t>(s)));
  }
  bool stream_idle(StreamH s) override {
    if (capturing_) return false;  // (a captured stream's ops have not run: the graph needs the edge)
    flush_if(s);
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(static_cast<hipStream_t>(s), &cst) != hipSuccess || cst != hipStreamCaptureStatusNone)
      return false;
    return hipStreamQuery(static_cast<hipStream_t>(s)) == hipSuccess;
  }

  bool begin_capture(StreamH s) override {
    flush_all();
    AKKA_HIP(hipStreamBeginCapture(static_cast<hipStream_t>(s), hipStreamCaptureModeRelaxed));
    capturing_ = true;
    return true;
  }
  GraphH end_capture(StreamH s, bool discard) override {
    flush_all();
    capturing_ = false;
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(static_cast<hipStream_t>(s), &g);
    if (e != hipSuccess || !g || discard) {
      if (g) hipGraphDestroy(g);
      if (e != hipSuccess && !discard) AKKA_HIP(e);
      return nullptr;
    }
    hipGraphExec_t ex = nullptr;
    e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    AKKA_HIP(e);
    return ex;
  }
  void launch_graph(GraphH g, StreamH s) override {
    flush_if(s);
    AKKA_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(g), static_cast<hipStream_t>(s)));
  }
  void destroy_graph(GraphH g) override {
    if (g) hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
  }

  void reduce(StreamH s, const ReduceSpec* specs, int32_t n, DType dt) override {
    for (int32_t i = 0; i < n; ++i) {
      const ReduceSpec& sp = specs[i];
      if (pending_.size() && pending_stream_ == s && pending_dt_ == dt && mergeable(pending_.back(), sp)) {
        pending_.back().n += sp.n;
        continue;
      }
      flush_if(s);
      flush_all();
      pending_.push_back(sp);
      pending_stream_ = s;
      pending_dt_ = dt;
    }
  }
  void copy(StreamH s, void* dst, const void* src, size_t bytes, CopyKind kind) override {
    if (bytes == 0 || dst == src) return;
    flush_if(s);
    hipMemcpyKind k = hipMemcpyDefault;
    switch (kind) {
      case CopyKind::HostToDevice:
        k = hipMemcpyHostToDevice;
        break;
      case CopyKind::DeviceToHost:
        k = hipMemcpyDeviceToHost;
        break;
      case CopyKind::DeviceToDevice:
        k = hipMemcpyDeviceToDevice;
        break;
      default:
        k = hipMemcpyDefault;
    }
    AKKA_HIP(hipMemcpyAsync(dst, src, bytes, k, static_cast<hipStream_t>(s)));
  }
  bool host_notify(StreamH s, std::function<void()> fn) override {
    flush_if(s);
    auto* heap = new std::function<void()>(std::move(fn));
    hipError_t e = hipLaunchHostFunc(
        static_cast<hipStream_t>(s),
        [](void* arg) {
          auto* f = static_cast<std::function<void()>*>(arg);
          (*f)();
          delete f;
        },
        heap);
    if (e != hipSuccess) {
      delete heap;
      return false;
    }
    return true;
  }
  void zero(StreamH s, void* dst, size_t bytes) override {
    if (!bytes) return;
    flush_if(s);
    AKKA_HIP(hipMemsetAsync(dst, 0, bytes, static_cast<hipStream_t>(s)));
  }

  void fill_i32(StreamH s, int32_t* dst, int32_t value, size_t n) override {
    if (!n) return;
    // A counts row issued right behind a pending reduce on the same stream
    // rides along in that launch (block 0 writes it): one dispatch per round.
    if (!pending_.empty() && pending_stream_ == s && !pending_.back().fill && n <= 65536) {
      pending_.back().fill = dst;
      pending_.back().fill_value = value;
      pending_.back().fill_n = int32_t(n);
      return;
    }
    flush_if(s);
    AKKA_HIP(hipMemsetD32Async(dst, value, n, static_cast<hipStream_t>(s)));
  }
  void poison_counts_if(StreamH s, const uint32_t* flag, int32_t* counts, size_t n) override {
    if (!n) return;
    flush_if(s);
    launch_poison_counts(static_cast<hipStream_t>(s), flag, counts, int64_t(n));
  }
  void fill_counts_unless(StreamH s, const uint32_t* flag, int32_t* counts, int32_t value, size_t n) override {
    if (!n) return;
    flush_if(s);
    launch_fill_counts(static_cast<hipStream_t>(s), flag, counts, value, int64_t(n));
  }
  void flush(StreamH s) override { flush_if(s); }

 private:
  bool mergeable(const ReduceSpec& a, const ReduceSpec& b) const {
    if (a.nsrc != b.nsrc || a.fill || b.fill) return false;
    const size_t es = dtype_size(pending_dt_);
    const size_t off = size_t(a.n) * es;
    if (static_cast<char*>(a.dst) + off != b.dst) return false;
    for (int i = 0; i < a.nsrc; ++i) {
      // dst-as-accumulator passes (split_reduce) never merge
      if (a.srcs[i] == a.dst) return false;
      if (static_cast<const char*>(a.srcs[i]) + off != b.srcs[i]) return false;
    }
    return true;
  }
  void flush_if(StreamH s) {
    if (!pending_.empty() && pending_stream_ == s) flush_all();
  }
  void flush_all() {
    if (pending_.empty()) return;
    for (const auto& sp : pending_) launch_reduce(static_cast<hipStream_t>(pending_stream_), sp, pending_dt_, impl_);
    pending_.clear();
  }

  int32_t dev_;
  hipStream_t comm_ = nullptr;
  hipStream_t compute_ = nullptr;
  bool exported_ = false;
  ReduceImpl impl_;
  bool capturing_ = false;
  std::vector<ReduceSpec> pending_;
  StreamH pending_stream_ = nullptr;
  DType pending_dt_ = DType::F32;
};

}  // namespace

std::unique_ptr<Device> make_hip_device(int32_t device_index, bool high_priority_comm) {
  return std::make_unique<HipDevice>(device_index, high_priority_comm);
}

}  // namespace akka
