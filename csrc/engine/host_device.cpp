// Host implementation of the Device interface.
//
// Immediate mode executes every op at the call (the spec-test probe path and
// CPU-only clusters).  Deferred mode appends ops to one in-order queue per
// device; the p2p simulator (sim_p2p.cpp) drains the queues of N simulated
// ranks together, so grouped send/recv rendezvous, matching order and deadlock
// freedom of the RCCL schedule are exercised on a CPU box.
#include <cmath>
#include <cstdlib>
#include <deque>
#include <map>

#include "device.h"
#include "racecheck.h"

namespace akka {

static inline float bf16_to_f32(uint16_t v) {
  uint32_t u = uint32_t(v) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
static inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return uint16_t((u >> 16) | 0x40);  // keep NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

static void host_reduce(const ReduceSpec& s, DType dt) {
  if (dt == DType::F32) {
    float* d = static_cast<float*>(s.dst);
    std::vector<float> acc(static_cast<size_t>(s.n), 0.0f);
    for (int32_t i = 0; i < s.nsrc; ++i) {
      const float* p = static_cast<const float*>(s.srcs[i]);
      for (int64_t j = 0; j < s.n; ++j) acc[j] += p[j];
    }
    std::memcpy(d, acc.data(), size_t(s.n) * 4);
  } else {
    uint16_t* d = static_cast<uint16_t*>(s.dst);
    std::vector<float> acc(static_cast<size_t>(s.n), 0.0f);
    for (int32_t i = 0; i < s.nsrc; ++i) {
      const uint16_t* p = static_cast<const uint16_t*>(s.srcs[i]);
      for (int64_t j = 0; j < s.n; ++j) acc[j] += bf16_to_f32(p[j]);
    }
    for (int64_t j = 0; j < s.n; ++j) d[j] = f32_to_bf16(acc[j]);
  }
}

std::vector<ReduceSpec> split_reduce(void* dst, const std::vector<const void*>& srcs, int64_t n) {
  std::vector<ReduceSpec> out;
  size_t i = 0;
  bool first = true;
  do {
    ReduceSpec s;
    s.dst = dst;
    s.n = n;
    if (!first) s.srcs[s.nsrc++] = dst;
    while (i < srcs.size() && s.nsrc < kMaxReduceSrc) s.srcs[s.nsrc++] = srcs[i++];
    out.push_back(s);
    first = false;
  } while (i < srcs.size());
  return out;
}

namespace {

// Host event: record() bumps `recorded` at enqueue time and the stream op sets
// `completed` when it runs; wait() captures the target generation at enqueue
// time (CUDA/HIP semantics: a wait refers to the most recent record).
struct HostEvent {
  int64_t recorded = 0;
  int64_t completed = 0;
};

class HostDevice final : public Device {
 public:
  explicit HostDevice(bool deferred) : deferred_(deferred) {
    queues_[reinterpret_cast<StreamH>(1)];
    queues_[reinterpret_cast<StreamH>(2)];
    const char* rc = std::getenv("AKKA_RACECHECK");
    if (rc && *rc && *rc != '0') rc_ = std::make_unique<RaceChecker>();
  }
  ~HostDevice() override = default;

  bool is_host() const override { return true; }
  void* alloc(size_t bytes) override {
    void* p = std::calloc(bytes ? bytes : 1, 1);
    AKKA_CHECK(p, "host alloc failed");
    return p;
  }
  void release(void* p) override { std::free(p); }
  void* alloc_pinned(size_t bytes) override { return alloc(bytes); }
  void release_pinned(void* p) override { std::free(p); }

  StreamH comm_stream() override { return reinterpret_cast<StreamH>(1); }
  StreamH compute_stream() override { return reinterpret_cast<StreamH>(2); }
  StreamH create_stream() override {
    StreamH s = reinterpret_cast<StreamH>(next_stream_++);
    queues_[s];
    return s;
  }
  void destroy_stream(StreamH s) override { queues_.erase(s); }

  EventH create_event() override { return new HostEvent(); }
  void destroy_event(EventH e) override {
    if (rc_) rc_->forget_event(e);
    delete static_cast<HostEvent*>(e);
  }
  void record(EventH e, StreamH s) override {
    auto* ev = static_cast<HostEvent*>(e);
    const int64_t gen = ++ev->recorded;
    if (rc_) {
      rc_->tick(s);
      rc_->record(e, s);
    }
    run(s, [ev, gen]() {
      if (ev->completed < gen) ev->completed = gen;
      return true;
    });
  }
  void wait(StreamH s, EventH e) override {
    auto* ev = static_cast<HostEvent*>(e);
    const int64_t target = ev->recorded;
    if (rc_) rc_->wait(s, e);  // ordering holds even when the wait is elided below
    if (ev->completed >= target) return;
    run(s, [ev, target]() { return ev->completed >= target; });
  }
  bool query(EventH e) override {
    auto* ev = static_cast<HostEvent*>(e);
    const bool done = ev->completed >= ev->recorded;
    if (done && rc_) rc_->host_join_event(e);  // the host saw it: later ops follow it
    return done;
  }
  void sync_event(EventH e) override {
    auto* ev = static_cast<HostEvent*>(e);
    if (deferred_) {
      while (ev->completed < ev->recorded && step()) {
      }  // best effort: a simulated rank cannot block on its peers
    }
    if (rc_ && ev->completed >= ev->recorded) rc_->host_join_event(e);
  }
  void sync_stream(StreamH s) override {
    if (deferred_) {
      while (!queue_of(s).empty() && step()) {
      }
      AKKA_CHECK(queue_of(s).empty(),
                 "host device sync would block: the simulated stream waits on a peer (drive the simulator instead)");
    }
    if (rc_) rc_->host_join_stream(s);
  }

  bool models_streams() const override { return rc_ != nullptr; }
  void declare_access(StreamH s, const std::vector<Access>& acc) override {
    if (!rc_) return;
    rc_->tick(s);
    rc_->access(s, acc);
  }
  std::vector<std::string> race_reports() const override {
    return rc_ ? rc_->reports() : std::vector<std::string>{};
  }
  int64_t race_count() const override { return rc_ ? rc_->races() : 0; }

  void reduce(StreamH s, const ReduceSpec* specs, int32_t n, DType dt) override {
    std::vector<ReduceSpec> v(specs, specs + n);
    if (rc_) {
      const size_t es = dt == DType::F32 ? 4 : 2;
      std::vector<Access> acc;
      for (const auto& sp : v) {
        for (int32_t i = 0; i < sp.nsrc; ++i)
          if (sp.srcs[i] != sp.dst) acc.push_back({sp.srcs[i], size_t(sp.n) * es, false, "reduce.src"});
        acc.push_back({sp.dst, size_t(sp.n) * es, true, "reduce.dst"});
        if (sp.fill) acc.push_back({sp.fill, size_t(sp.fill_n) * 4, true, "reduce.fill"});
      }
      declare_access(s, acc);
    }
    run(s, [v, dt]() {
      for (const auto& sp : v) {
        host_reduce(sp, dt);
        if (sp.fill)
          for (int32_t i = 0; i < sp.fill_n; ++i) sp.fill[i] = sp.fill_value;
      }
      return true;
    });
  }
  void copy(StreamH s, void* dst, const void* src, size_t bytes, CopyKind kind) override {
    if (dst == src || bytes == 0) return;
    if (rc_) {
      // a host->device copy reads its (pinned, host-owned) source at issue
      if (kind == CopyKind::HostToDevice) declare_access(s, {{dst, bytes, true, "copy.dst"}});
      else declare_access(s, {{src, bytes, false, "copy.src"}, {dst, bytes, true, "copy.dst"}});
    }
    if (deferred_ && kind == CopyKind::HostToDevice) {
      // Host->device copies read their (pinned / message-owned) source when
      // issued; snapshot it so the deferred queue models that contract.
      auto snap = std::make_shared<std::vector<char>>(static_cast<const char*>(src),
                                                      static_cast<const char*>(src) + bytes);
      run(s, [=]() {
        std::memcpy(dst, snap->data(), bytes);
        return true;
      });
      return;
    }
    run(s, [=]() {
      std::memmove(dst, src, bytes);
      return true;
    });
  }
  void zero(StreamH s, void* dst, size_t bytes) override {
    if (rc_) declare_access(s, {{dst, bytes, true, "zero"}});
    run(s, [=]() {
      std::memset(dst, 0, bytes);
      return true;
    });
  }
  void fill_i32(StreamH s, int32_t* dst, int32_t value, size_t n) override {
    if (rc_) declare_access(s, {{dst, n * sizeof(int32_t), true, "fill_i32"}});
    run(s, [=]() {
      for (size_t i = 0; i < n; ++i) dst[i] = value;
      return true;
    });
  }
  void enqueue_host_op(StreamH s, std::function<bool()> op) override {
    AKKA_CHECK(deferred_, "enqueue_host_op requires a deferred host device");
    queue_of(s).push_back(std::move(op));
  }

  // Simulator hooks.  step(): run every stream's head ops until each blocks;
  // `rotate` changes which stream goes first (schedule fuzzing).
  bool step(uint32_t rotate = 0) {
    bool progress = false;
    const size_t n = queues_.size();
    std::vector<std::deque<std::function<bool()>>*> qs;
    qs.reserve(n);
    for (auto& kv : queues_) qs.push_back(&kv.second);
    for (size_t i = 0; i < n; ++i) {
      auto& q = *qs[(i + rotate) % n];
      while (!q.empty()) {
        if (!q.front()()) break;
        q.pop_front();
        progress = true;
      }
    }
    return progress;
  }
  bool idle() const {
    for (const auto& kv : queues_)
      if (!kv.second.empty()) return false;
    return true;
  }

 private:
  std::deque<std::function<bool()>>& queue_of(StreamH s) { return queues_[s]; }
  void run(StreamH s, std::function<bool()> f) {
    if (deferred_) {
      queue_of(s).push_back(std::move(f));
    } else {
      f();
    }
  }

  bool deferred_;
  std::unique_ptr<RaceChecker> rc_;  // AKKA_RACECHECK=1
  std::map<StreamH, std::deque<std::function<bool()>>> queues_;
  uintptr_t next_stream_ = 16;
};

}  // namespace

std::unique_ptr<Device> make_host_device(bool deferred) { return std::make_unique<HostDevice>(deferred); }

// Exposed to sim_p2p.cpp.
bool host_device_step(Device* d, uint32_t rotate) { return static_cast<HostDevice*>(d)->step(rotate); }
bool host_device_idle(Device* d) { return static_cast<HostDevice*>(d)->idle(); }

}  // namespace akka
