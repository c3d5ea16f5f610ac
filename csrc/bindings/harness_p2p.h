// Harness p2p endpoints for the Python layer (not production transports):
//  * PyCallbackP2P / PyAsyncCallbackP2P -- groups delegated to Python
//    callables (torch.distributed gloo across CPU processes), blocking or
//    posted-and-polled;
//  * LoopbackP2P / LoopbackPairP2P -- N ranks of one process on one GPU
//    (host rendezvous, or asynchronous per-pair with stream wait/write-value).
// They live next to the bindings because they call into Python or release
// the GIL; RCCL (rccl_p2p.cpp) is what runs between GPUs.
#pragma once

#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <set>
#include <vector>

#include "../transport/p2p.h"

namespace akka {

namespace py = pybind11;

// Grouped p2p delegated to a Python callable: ops = [(send, peer, ptr, bytes)].
// Used with torch.distributed (gloo) to run the production schedule across
// real processes on CPU-only machines.
class PyCallbackP2P final : public P2P {
 public:
  PyCallbackP2P(py::function fn, int32_t rank, int32_t n, Device* dev = nullptr)
      : fn_(std::move(fn)), rank_(rank), n_(n), dev_(dev) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "callback"; }
  void group(StreamH s, const std::vector<P2POp>& ops) override {
    py::list l;
    std::vector<Access> acc;
    for (const auto& op : ops) {
      l.append(py::make_tuple(op.send, op.peer, reinterpret_cast<uintptr_t>(op.buf), op.bytes, op.channel));
      acc.push_back({op.buf, op.bytes, !op.send, op.send ? "p2p.send" : "p2p.recv"});
    }
    if (dev_) dev_->declare_access(s, acc);  // stream race checking (no-op unless on)
    fn_(l);
  }

 private:
  py::function fn_;
  int32_t rank_, n_;
  Device* dev_;
};

// Asynchronous grouped p2p through two Python callables (reactive transport
// across CPU processes, torch.distributed gloo): when the stream reaches the
// group, `post(ops)` starts the isend/irecv and returns a handle; the stream
// op then completes once `test(handle)` is true.  Groups on one stream run in
// order (one outstanding group per pair stream), different pair streams
// overlap -- the same contract as RCCL pair communicators on MI355X.
class PyAsyncCallbackP2P final : public P2P {
 public:
  PyAsyncCallbackP2P(py::function post, py::function test, int32_t rank, int32_t n, Device* dev)
      : post_(std::move(post)), test_(std::move(test)), rank_(rank), n_(n), dev_(dev) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "async-callback"; }
  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    struct State {
      py::list ops;
      py::object handle;
      bool posted = false;
    };
    auto st = std::make_shared<State>();
    for (const auto& op : ops)
      st->ops.append(py::make_tuple(op.send, op.peer, reinterpret_cast<uintptr_t>(op.buf), op.bytes, op.channel));
    py::function post = post_, test = test_;
    // Runs from WorkerCore::poll / start (Python callers: the GIL is held).
    dev_->enqueue_host_op(stream, [st, post, test]() {
      if (!st->posted) {
        st->handle = post(st->ops);
        st->posted = true;
      }
      if (!test(st->handle).cast<bool>()) return false;
      st->handle = py::none();
      return true;
    });
  }

 private:
  py::function post_, test_;
  int32_t rank_, n_;
  Device* dev_;
};

// ---------------------------------------------------------------------------
// GPU loopback p2p: N ranks of ONE process on ONE GPU, each with its own HIP
// streams.  A group is a host rendezvous of all ranks (the GIL is released
// while waiting); receives are device copies on the receiver's stream after
// the sender's "posted" event, and a sender's stream continues only after its
// receivers' "copied" events.  Every event is recorded before anyone waits on
// it, so this exercises the real stream/event ordering of the GPU data plane
// and StreamLink at N > 1 without RCCL (which needs one GPU per rank).
struct LoopbackHub {
  explicit LoopbackHub(int32_t n) : n(n), ops(n), streams(n, nullptr), posted(n, nullptr), copied(n, nullptr) {
    for (int32_t i = 0; i < n; ++i) {
      hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(&posted[i]), hipEventDisableTiming);
      hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(&copied[i]), hipEventDisableTiming);
    }
  }
  ~LoopbackHub() {
    for (int32_t i = 0; i < n; ++i) {
      hipEventDestroy(static_cast<hipEvent_t>(posted[i]));
      hipEventDestroy(static_cast<hipEvent_t>(copied[i]));
    }
  }
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const int64_t gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen; }))
      throw AkkaError("akka: loopback p2p rendezvous timed out (ranks issued different schedules)");
  }
  int32_t n;
  std::mutex mu;
  std::condition_variable cv;
  int32_t arrived = 0;
  int64_t generation = 0;
  std::vector<std::vector<P2POp>> ops;
  std::vector<StreamH> streams;
  std::vector<EventH> posted, copied;
  int64_t bytes = 0;
};

struct PyLoopbackHub {
  std::shared_ptr<LoopbackHub> hub;
};

class LoopbackP2P final : public P2P {
 public:
  LoopbackP2P(std::shared_ptr<LoopbackHub> hub, int32_t rank) : hub_(std::move(hub)), rank_(rank) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return hub_->n; }
  const char* name() const override { return "loopback"; }
  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    py::gil_scoped_release nogil;
    LoopbackHub& h = *hub_;
    hipStream_t s = static_cast<hipStream_t>(stream);
    check(hipEventRecord(static_cast<hipEvent_t>(h.posted[rank_]), s));
    {
      std::lock_guard<std::mutex> lk(h.mu);
      h.ops[rank_] = ops;
      h.streams[rank_] = stream;
    }
    h.barrier();  // every rank posted this group
    // my receives: j-th recv from p <-> j-th send from p to me, in this group
    std::vector<int32_t> taken(h.n, 0);
    int64_t moved = 0;
    for (const auto& op : ops) {
      if (op.send) continue;
      const auto& pops = h.ops[op.peer];
      int32_t seen = 0;
      const P2POp* match = nullptr;
      for (const auto& q : pops) {
        if (q.send && q.peer == rank_ && seen++ == taken[op.peer]) {
          match = &q;
          break;
        }
      }
      AKKA_CHECK(match, "loopback p2p: recv from " + std::to_string(op.peer) + " has no matching send");
      AKKA_CHECK(match->bytes == op.bytes, "loopback p2p: size mismatch");
      ++taken[op.peer];
      check(hipStreamWaitEvent(s, static_cast<hipEvent_t>(h.posted[op.peer]), 0));
      if (op.bytes) check(hipMemcpyAsync(op.buf, match->buf, op.bytes, hipMemcpyDeviceToDevice, s));
      moved += int64_t(op.bytes);
    }
    check(hipEventRecord(static_cast<hipEvent_t>(h.copied[rank_]), s));
    {
      std::lock_guard<std::mutex> lk(h.mu);
      h.bytes += moved;
    }
    h.barrier();  // every receiver enqueued its copies + recorded `copied`
    std::vector<bool> seen_peer(h.n, false);
    for (const auto& op : ops)
      if (op.send && !seen_peer[op.peer]) {
        seen_peer[op.peer] = true;
        check(hipStreamWaitEvent(s, static_cast<hipEvent_t>(h.copied[op.peer]), 0));
      }
    h.barrier();  // nobody re-records posted/copied before all waits are enqueued
  }

 private:
  static void check(hipError_t e) {
    if (e != hipSuccess) throw AkkaError(std::string("akka: loopback p2p: ") + hipGetErrorString(e));
  }
  std::shared_ptr<LoopbackHub> hub_;
  int32_t rank_;
};

// ---------------------------------------------------------------------------
// Asynchronous per-pair loopback p2p (reactive transport harness): a group
// holds ops to one peer and never blocks the host.  The first side of a pair
// to post records a "posted" event and parks its stream on a signal word
// (hipStreamWaitValue32); the second side, on its own stream, waits for the
// first side's event, performs both directions' copies and releases the first
// side with hipStreamWriteValue32.  Groups of a pair match in posting order,
// like RCCL p2p on a pair communicator -- so a peer that never posts stalls
// only its own pair's streams, which is exactly what the reactive link has to
// tolerate.
struct PairHub {
  static constexpr int32_t kCh = 2;  // channels (independent matching orders) per pair
  explicit PairHub(int32_t n)
      : n(n), posts(size_t(n) * n * kCh), flags(size_t(n) * n * kCh, nullptr), seq(size_t(n) * n * kCh, 0) {
    // One coherent pinned block, one 64-byte line per signal word: the CP's
    // wait-value packets poll it, the peer stream's write-value packet sets it.
    if (hipHostMalloc(&block, flags.size() * 64, hipHostMallocCoherent) != hipSuccess)
      throw AkkaError("akka: pair loopback: cannot allocate signal memory");
    std::memset(block, 0, flags.size() * 64);
    for (size_t i = 0; i < flags.size(); ++i) flags[i] = reinterpret_cast<uint32_t*>(static_cast<char*>(block) + i * 64);
  }
  // index of (a, b, channel) in flags/seq, and of the unordered pair in posts
  size_t dir(int32_t a, int32_t b, int32_t ch) const { return (size_t(a) * n + size_t(b)) * kCh + size_t(ch); }
  size_t pair(int32_t a, int32_t b, int32_t ch) const {
    return (size_t(std::min(a, b)) * n + size_t(std::max(a, b))) * kCh + size_t(ch);
  }
  ~PairHub() {
    for (auto* e : events) hipEventDestroy(e);
    if (block) hipHostFree(block);
  }
  struct Post {
    int32_t rank;
    StreamH stream;
    std::vector<P2POp> ops;
    hipEvent_t posted;
    uint32_t seq;
  };
  hipEvent_t event() {
    if (!free_events.empty()) {
      hipEvent_t e = free_events.back();
      free_events.pop_back();
      return e;
    }
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) throw AkkaError("akka: hipEventCreate");
    events.push_back(e);
    return e;
  }
  int32_t n;
  std::mutex mu;
  std::vector<std::deque<Post>> posts;  // [pair(lo,hi,ch)] unmatched posts of that pair (one side at a time)
  std::vector<uint32_t*> flags;         // [dir(a,b,ch)]: a's stream waits here for its groups with b
  std::vector<uint32_t> seq;            // [dir(a,b,ch)]: groups a posted towards b
  void* block = nullptr;
  std::vector<hipEvent_t> events, free_events;
  std::set<std::pair<int32_t, int32_t>> dead;  // (me, peer) aborted by me
  int64_t bytes = 0;
};

struct PyPairHub {
  std::shared_ptr<PairHub> hub;
};

class LoopbackPairP2P final : public P2P {
 public:
  LoopbackPairP2P(std::shared_ptr<PairHub> hub, int32_t rank) : hub_(std::move(hub)), rank_(rank) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return hub_->n; }
  const char* name() const override { return "loopback-pair"; }
  bool abort_peer(int32_t peer) override {
    // Release both directions of the pair for good: a stream parked on the
    // dead peer moves on (its copies never happen), and the unmatched posts
    // are dropped.
    PairHub& h = *hub_;
    std::lock_guard<std::mutex> lk(h.mu);
    for (int32_t ch = 0; ch < PairHub::kCh; ++ch) {
      const size_t key = h.pair(rank_, peer, ch);
      for (auto& p : h.posts[key]) h.free_events.push_back(p.posted);
      h.posts[key].clear();
      __atomic_store_n(h.flags[h.dir(rank_, peer, ch)], 0x7fffffffu, __ATOMIC_SEQ_CST);
      __atomic_store_n(h.flags[h.dir(peer, rank_, ch)], 0x7fffffffu, __ATOMIC_SEQ_CST);
    }
    h.dead.insert({rank_, peer});
    return true;
  }
  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    if (ops.empty()) return;
    PairHub& h = *hub_;
    const int32_t peer = ops.front().peer;
    const int32_t ch = ops.front().channel;
    for (const auto& op : ops)
      AKKA_CHECK(op.peer == peer && op.channel == ch, "pair group holds ops to more than one peer / channel");
    AKKA_CHECK(ch >= 0 && ch < PairHub::kCh, "pair loopback: bad channel");
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(h.mu);
    AKKA_CHECK(!h.dead.count({rank_, peer}), "pair loopback: group to an aborted peer");
    auto& q = h.posts[h.pair(rank_, peer, ch)];
    if (q.empty() || q.front().rank == rank_) {
      PairHub::Post p{rank_, stream, ops, h.event(), ++h.seq[h.dir(rank_, peer, ch)]};
      check(hipEventRecord(p.posted, s));
      check(hipStreamWaitValue32(s, h.flags[h.dir(rank_, peer, ch)], p.seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
      q.push_back(std::move(p));
      return;
    }
    PairHub::Post other = std::move(q.front());
    q.pop_front();
    check(hipStreamWaitEvent(s, other.posted, 0));
    h.free_events.push_back(other.posted);  // the wait captured its record
    int64_t moved = 0;
    moved += copy_dir(other.ops, ops, s);  // other's sends -> my recvs
    moved += copy_dir(ops, other.ops, s);  // my sends -> other's recvs
    check(hipStreamWriteValue32(s, h.flags[h.dir(other.rank, rank_, ch)], other.seq, 0));
    h.bytes += moved;
  }

 private:
  // j-th send in `from` (to the other side) matches the j-th recv in `to`.
  static int64_t copy_dir(const std::vector<P2POp>& from, const std::vector<P2POp>& to, hipStream_t s) {
    std::vector<const P2POp*> sends, recvs;
    for (const auto& op : from)
      if (op.send) sends.push_back(&op);
    for (const auto& op : to)
      if (!op.send) recvs.push_back(&op);
    AKKA_CHECK(sends.size() == recvs.size(), "pair loopback: send/recv count mismatch");
    int64_t moved = 0;
    for (size_t j = 0; j < sends.size(); ++j) {
      AKKA_CHECK(sends[j]->bytes == recvs[j]->bytes, "pair loopback: size mismatch");
      if (sends[j]->bytes)
        check(hipMemcpyAsync(recvs[j]->buf, sends[j]->buf, sends[j]->bytes, hipMemcpyDeviceToDevice, s));
      moved += int64_t(sends[j]->bytes);
    }
    return moved;
  }
  static void check(hipError_t e) {
    if (e != hipSuccess) throw AkkaError(std::string("akka: pair loopback p2p: ") + hipGetErrorString(e));
  }
  std::shared_ptr<PairHub> hub_;
  int32_t rank_;
};

}  // namespace akka
