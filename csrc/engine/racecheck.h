// Stream race checker for the host (simulated) device.
//
// The engine orders its GPU work with streams and events only; a missing wait
// is a data race that real hardware shows rarely and nondeterministically (the
// round-2 counts-fill race: profiles/r02/hazard/).  On the CPU simulator every
// stream op is known at enqueue time, so happens-before can be checked
// exactly, independent of how the simulated queues happen to interleave:
//
//   * every stream carries a vector clock; an op on stream s ticks s's own
//     component; record(e, s) snapshots s's clock into e; wait(s, e) joins e's
//     clock into s (HIP/CUDA semantics: a wait refers to the latest record);
//   * host synchronisation (sync_stream / sync_event / a query that returned
//     true) joins that clock into the host's, and every op enqueued later on
//     any stream starts from at least the host's clock;
//   * each op declares the byte ranges it reads and writes; a shadow map keeps,
//     per range, the last write and the reads since, each as (stream, clock).
//     An access conflicts with an earlier one on another stream unless the
//     earlier one happens-before it (its stream's component in the new op's
//     clock is at least the earlier op's tick).  Read/read never conflicts.
//
// Reports name both ops (tags given by the device op kinds, e.g. "fill_i32",
// "reduce.dst", "p2p.recv", "caller.write") and their streams.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "device.h"

namespace akka {

class RaceChecker {
 public:
  using VC = std::vector<int64_t>;

  // A new op on stream s: tick s, join the host clock; returns the op's clock.
  const VC& tick(StreamH s);
  // Check `acc` (done by the op just ticked on s) and update the shadow map.
  void access(StreamH s, const std::vector<Access>& acc);
  void record(void* event, StreamH s);         // event clock := s clock (after a tick)
  void wait(StreamH s, void* event);           // s clock |= event clock
  void host_join_stream(StreamH s);            // host clock |= s clock
  void host_join_event(void* event);           // host clock |= event clock
  void forget_event(void* event) { events_.erase(event); }

  const std::vector<std::string>& reports() const { return reports_; }
  int64_t races() const { return races_; }
  void clear() {
    reports_.clear();
    races_ = 0;
  }

 private:
  struct Stamp {
    int32_t stream = -1;  // stream index
    int64_t clock = 0;
    const char* tag = "";
  };
  struct Cell {  // shadow state of bytes [start, end)
    uintptr_t end = 0;
    Stamp write;                 // last write (stream -1: none)
    std::vector<Stamp> reads;    // reads since the last write, one per stream (latest)
  };
  int32_t index(StreamH s);
  static void join(VC& a, const VC& b);
  bool before(const Stamp& prev, const VC& now) const {
    return prev.stream < 0 || (size_t(prev.stream) < now.size() && now[size_t(prev.stream)] >= prev.clock);
  }
  void report(const Stamp& prev, bool prev_write, int32_t cur_stream, const Access& a, uintptr_t lo, uintptr_t hi);
  void split(uintptr_t at);

  std::map<StreamH, int32_t> ids_;
  std::vector<VC> clocks_;  // per stream index
  VC host_;
  std::map<void*, VC> events_;
  std::map<uintptr_t, Cell> shadow_;
  std::vector<std::string> reports_;
  int64_t races_ = 0;
};

}  // namespace akka
