// Round engine: the per-worker threshold-allreduce state machine.
//
// Behavioural twin of the reference AllreduceWorker actor
// (src/main/scala/sample/cluster/allreduce/AllreduceWorker.scala:7-301):
//   InitWorkers      W:35-90    -> Engine::init
//   StartAllreduce   W:92-114   -> Engine::start          (incl. catch-up W:100-106)
//   ScatterBlock     W:116-126, W:170-186 -> Engine::on_scatter
//   ReduceBlock      W:128-138, W:149-168 -> Engine::on_reduce
//   Terminated       W:141-146  -> Engine::on_peer_terminated
//   scatter/broadcast/complete  W:212-285
//
// Single-threaded by contract (like an actor's receive): one progress thread
// per rank drives it.  Data movement is delegated to a DataPlane (memory +
// kernels) and a Link (transport); this class owns only round/threshold
// bookkeeping, so it is identical for the host probe, the TCP cluster and the
// RCCL/xGMI production path.
//
// Deliberate fixes of reference quirks, each covered by a test:
//  1. catch-up cannot double-complete: a forced round whose self-delivery
//     already completed it is not completed again, and chunks already reduced
//     are not re-broadcast;
//  2. thresholds fire once on reaching the cut-off (>=) and count DISTINCT
//     sources, so duplicate deliveries can neither overshoot nor stall a round;
//  3/4. exact integer partitioning (see geometry.h);
//  5. completion uses an O(1) per-row counter;
//  6. a worker without a master simply does not report completion;
//  future-round messages are handled in place after an implicit start (the
//  reference re-enqueues them at the mailbox tail, breaking per-pair FIFO).
#pragma once

#include <deque>
#include <functional>
#include <set>
#include <string>
#include <vector>

#include "dataplane.h"

namespace akka {

struct InitParams {
  int32_t id = -1;            // destId
  int32_t worker_num = 0;     // workerNum (N)
  float th_reduce = 1.0f;     // fraction of scattered copies needed to reduce a chunk
  float th_complete = 1.0f;   // fraction of reduced chunks needed to complete a round
  int32_t max_lag = 0;        // rounds a worker may fall behind
  int64_t data_size = 0;
  int64_t max_chunk_size = 1;
};

struct PeerEntry {
  int32_t id;
  bool local;  // true: this worker itself (messages short-circuit, W:228-232)
};

// Transport seen by the engine.  Sends to a *local* peer never reach the link.
class Link {
 public:
  virtual ~Link() = default;
  virtual void send_scatter(int32_t dest, int32_t chunk, int32_t round, const Payload& p) = 0;
  virtual void send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) = 0;
  // Called once the engine finished the outermost event it was handling.
  virtual void pump() {}
  // Called after scatter() of a round (all of its sends issued).
  virtual void on_scattered(int32_t /*round*/) {}
  // May the engine finalize (flush) `round` right now?  A scheduled link says
  // no while receives for the round are still being issued; it then calls
  // Engine::flush_deferred(round) itself.
  virtual bool may_finalize(int32_t /*round*/) { return true; }
  // Exact-threshold fast lane: the engine offers a round whose outcome is
  // fixed (thReduce = thComplete = 1, all N peers known, no state of the round
  // seen yet): every chunk is the sum of all N inputs with count N.  A link
  // that can move and reduce the whole round by itself (collectives) does so
  // and returns true; the engine then completes the round without per-chunk
  // bookkeeping.  False: the engine runs the ordinary message flow.
  virtual bool bulk_round(int32_t /*round*/) { return false; }
  // True if bulk_round always takes exact rounds (its schedule for them
  // differs from the message flow's, so every rank must take it).
  virtual bool takes_exact_rounds() const { return false; }
  // The control plane reported peer `id` dead (WorkerTerminated): end the
  // transfers owed to / expected from it; it is no longer in the peer map.
  virtual void on_peer_lost(int32_t /*id*/) {}
};

// Embedding layer callbacks (Python, CLI, bench).
class EngineHost {
 public:
  virtual ~EngineHost() = default;
  // AllReduceInputRequest(round) -> bind input via DataPlane::bind_input.
  virtual void fetch(int32_t round) = 0;
  // Bind the round's output + counts buffers via DataPlane::bind_output.
  virtual void alloc_output(int32_t round) = 0;
  // AllReduceOutput for `round` is final in stream order (data sink).
  virtual void deliver(int32_t round) = 0;
  // CompleteAllreduce(id, round) to the master (W:276).
  virtual void notify_complete(int32_t round) = 0;
  // The engine no longer references the round's input (an outdated round it
  // scattered only for the benefit of slower peers).
  virtual void release(int32_t round) { (void)round; }
  virtual void log(int32_t level, const std::string& msg) { (void)level; (void)msg; }
};

struct EngineStats {
  int64_t scatters_in = 0, reduces_in = 0, outdated_dropped = 0, future_started = 0;
  int64_t chunks_reduced = 0, forced_reduces = 0, rounds_completed = 0, rounds_forced = 0;
  int64_t errors = 0;
  int64_t bulk_rounds = 0;  // rounds run through Link::bulk_round
};

class Engine {
 public:
  Engine(EngineHost* host, Link* link);
  ~Engine();

  // InitWorkers (W:35-90).  The data plane is created by the embedding layer
  // (it needs the device) after the first init; pass it via attach().
  // Returns true on first init (buffers must be attached), false on re-init
  // (only the peer map is replaced, W:87-89).
  bool init(const InitParams& p, const std::vector<PeerEntry>& peers);
  void attach(DataPlane* dp);

  void start(int32_t round);
  void on_scatter(int32_t src, int32_t dest, int32_t chunk, int32_t round, const Payload& p);
  void on_reduce(int32_t src, int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p);
  void on_peer_terminated(int32_t id);
  void flush_deferred(int32_t round);
  void set_link(Link* link) { link_ = link; }
  // Bind the round's output buffers now (a scheduled link receives into them).
  void ensure_output(int32_t round);

  // --- introspection ------------------------------------------------------
  bool initialized() const { return id_ >= 0 && dp_ != nullptr; }
  int32_t id() const { return id_; }
  int32_t round() const { return round_; }
  int32_t max_round() const { return max_round_; }
  int32_t max_scattered() const { return max_scattered_; }
  std::vector<int32_t> completed() const { return {completed_.begin(), completed_.end()}; }
  bool is_completed(int32_t r) const { return r < round_ || completed_.count(r) > 0; }
  std::vector<PeerEntry> peers() const { return peers_; }
  const InitParams& params() const { return params_; }
  const Geometry& geometry() const { return g_; }
  int32_t min_scatter_required() const { return min_scatter_; }
  int32_t min_reduced_required() const { return min_reduced_; }
  int32_t scatter_count(int32_t round, int32_t chunk) const;
  int32_t reduced_arrivals(int32_t round) const;
  const EngineStats& stats() const { return stats_; }
  DataPlane* dataplane() const { return dp_; }

 private:
  struct Row {
    int32_t round = -1;
    // phase 1, my block: [K_me][N] landed flags, per-chunk distinct arrivals, reduced bit
    std::vector<uint8_t> sc_mask;
    std::vector<int32_t> sc_count;
    std::vector<uint8_t> sc_reduced;
    // phase 2, whole vector: [N][kmax] landed flags + contributor counts
    std::vector<uint8_t> rd_landed;
    int32_t rd_arrivals = 0;
    bool done = false;
  };
  struct Pending {
    int kind;  // 0 start, 1 scatter, 2 reduce
    int32_t src, dest, chunk, round, count;
    Payload p;
    std::vector<uint8_t> owned;
  };
  class Scope;

  Row& row(int32_t round);
  const Row* find_row(int32_t round) const;
  bool present(int32_t id, bool* local) const;
  void do_start(int32_t r);
  void do_scatter_msg(int32_t src, int32_t dest, int32_t chunk, int32_t round, const Payload& p);
  void do_reduce_msg(int32_t src, int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p);
  void scatter(int32_t r);
  bool bulk_eligible(int32_t r) const;
  void complete_bulk(int32_t r);
  void reduce_and_broadcast(int32_t r, int32_t chunk, bool forced);
  void complete(int32_t r);
  void finalize_round(int32_t r);
  void leave_scope();

  EngineHost* host_;
  Link* link_;
  DataPlane* dp_ = nullptr;
  InitParams params_;
  Geometry g_;
  int32_t id_ = -1;
  int32_t N_ = 0;
  std::vector<PeerEntry> peers_;  // sorted by id
  int32_t round_ = -1, max_round_ = -1, max_scattered_ = -1;
  std::set<int32_t> completed_;
  std::set<int32_t> awaiting_finalize_;
  int32_t L_ = 1;
  int32_t kme_ = 0, kmax_ = 1;
  int32_t min_scatter_ = 1, min_reduced_ = 1;
  std::vector<Row> rows_;
  std::deque<Pending> pending_;
  int depth_ = 0;
  EngineStats stats_;
};

}  // namespace akka
