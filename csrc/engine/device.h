// Device abstraction: the data plane and the stream-scheduled link are written
// once against this interface and run either on a HIP device (production,
// gfx950 kernels + HIP streams/events) or on the host (CPU dev boxes, the
// spec-test probe, and the multi-rank p2p simulator that checks the RCCL
// schedule without a GPU).
//
// The reference has no device boundary at all: every buffer is a JVM array and
// every copy is System.arraycopy (AllReduceBuffer.scala:25-32,
// ReducedDataBuffer.scala:38); the N-way chunk sum is a scalar JVM loop
// (ScatteredDataBuffer.scala:20-32).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "common.h"

namespace akka {

using StreamH = void*;
using EventH = void*;
using GraphH = void*;  // an instantiated (executable) graph

// Sources per reduce launch; more sources are folded in extra passes.
constexpr int kMaxReduceSrc = 16;

// dst[0:n) = sum_i srcs[i][0:n)   (fp32 accumulate; dst may alias srcs[0])
struct ReduceSpec {
  void* dst = nullptr;
  const void* srcs[kMaxReduceSrc] = {};
  int32_t nsrc = 0;
  int64_t n = 0;
  // Optional piggy-backed int32 fill (a counts row) done by the same launch.
  int32_t* fill = nullptr;
  int32_t fill_value = 0;
  int32_t fill_n = 0;
};

// A byte range an op reads or writes (stream race checking, racecheck.h).
struct Access {
  const void* ptr;
  size_t bytes;
  bool write;
  const char* tag;
};

enum class CopyKind : int32_t { Default = 0, HostToDevice = 1, DeviceToHost = 2, DeviceToDevice = 3, HostToHost = 4 };

class Device {
 public:
  virtual ~Device() = default;
  virtual bool is_host() const = 0;
  virtual int32_t device_index() const { return -1; }

  virtual void* alloc(size_t bytes) = 0;
  virtual void release(void* p) = 0;
  // Page-locked host staging memory (plain host memory on the host device).
  virtual void* alloc_pinned(size_t bytes) = 0;
  virtual void release_pinned(void* p) = 0;

  virtual StreamH comm_stream() = 0;
  virtual StreamH compute_stream() = 0;
  // comm/compute were handed to a framework that may still reference them
  // after this device is gone (torch ExternalStream + record_stream: the
  // caching allocator records events on them when blocks are freed): never
  // destroy them.
  virtual void mark_streams_exported() {}
  // Extra streams (per-peer streams of the reactive transport).
  virtual StreamH create_stream() = 0;
  virtual void destroy_stream(StreamH s) = 0;

  virtual EventH create_event() = 0;
  virtual void destroy_event(EventH e) = 0;
  virtual void record(EventH e, StreamH s) = 0;
  virtual void wait(StreamH s, EventH e) = 0;
  virtual bool query(EventH e) = 0;
  virtual void sync_event(EventH e) = 0;
  virtual void sync_stream(StreamH s) = 0;
  // Every op enqueued on `s` so far has completed (a hand-over point of `s`
  // needs no event).  Conservative: false when unknown.
  virtual bool stream_idle(StreamH) { return false; }

  virtual void reduce(StreamH s, const ReduceSpec* specs, int32_t nspecs, DType dt) = 0;
  virtual void copy(StreamH s, void* dst, const void* src, size_t bytes, CopyKind kind) = 0;
  virtual void zero(StreamH s, void* dst, size_t bytes) = 0;
  virtual void fill_i32(StreamH s, int32_t* dst, int32_t value, size_t n) = 0;
  // counts[0..n) = 0 if *flag != 0 when the stream gets there (a failed
  // one-sided round).  Host devices never run those rounds.
  virtual void poison_counts_if(StreamH, const uint32_t* /*flag*/, int32_t* /*counts*/, size_t /*n*/) {}
  // counts[0..n) = (*flag != 0 ? 0 : value) when the stream gets there: the
  // counts fill of an exact round and its poison check as one operation.
  virtual void fill_counts_unless(StreamH s, const uint32_t* flag, int32_t* counts, int32_t value, size_t n) {
    fill_i32(s, counts, value, n);
    poison_counts_if(s, flag, counts, n);
  }
  // Issue any work held back on `s` (reduce launches kept open for merging).
  virtual void flush(StreamH) {}

  // Stream capture into graphs (HIP graphs).  While capturing, wait() must
  // never be elided and nothing may synchronize.  Host devices: unsupported.
  virtual bool begin_capture(StreamH) { return false; }
  // Ends the capture on `s`; returns the instantiated graph, or nullptr (and
  // discards the capture) if `discard` or the capture failed.
  virtual GraphH end_capture(StreamH, bool /*discard*/) { return nullptr; }
  virtual void launch_graph(GraphH, StreamH) { throw AkkaError("launch_graph: unsupported device"); }
  virtual void destroy_graph(GraphH) {}

  // Run `fn` on a host thread once the stream reaches this point (HIP:
  // hipLaunchHostFunc; `fn` must not call HIP).  Default: unsupported.
  virtual bool host_notify(StreamH, std::function<void()>) { return false; }

  // Host-device only: deferred execution queue used by the p2p simulator.
  virtual void enqueue_host_op(StreamH, std::function<bool()>) {
    throw AkkaError("enqueue_host_op: not a host device");
  }

  // Stream race checking (host device with AKKA_RACECHECK=1, racecheck.h).
  // models_streams(): callers may hand the engine streams of this device as
  // the producer of inputs / the allocator of outputs (their events count).
  virtual bool models_streams() const { return false; }
  // An op at this point of `s` that touches these bytes (transports and
  // callers declare what the device ops cannot see, e.g. p2p buffers).
  virtual void declare_access(StreamH, const std::vector<Access>&) {}
  virtual std::vector<std::string> race_reports() const { return {}; }
  virtual int64_t race_count() const { return 0; }
};

// Reduce specs with more than kMaxReduceSrc sources: fold into passes where
// pass p>0 accumulates into dst (dst is its own first source).
std::vector<ReduceSpec> split_reduce(void* dst, const std::vector<const void*>& srcs, int64_t n);

std::unique_ptr<Device> make_host_device(bool deferred);
// Defined in hip_device.cpp (HIP build only).
std::unique_ptr<Device> make_hip_device(int32_t device_index, bool high_priority_comm);

}  // namespace akka
