// ReactiveLink: the straggler-tolerant GPU data path.
//
// StreamLink (stream_link.h) enqueues a round's whole schedule as symmetric
// all-peer groups on one comm stream, so a rank proceeds at the pace of its
// slowest peer: fast on a healthy node, but the threshold parameters
// (thReduce / thComplete) only decide *what* is summed, never *when*.
// The reference's point is the opposite: each ScatterBlock / ReduceBlock is an
// independent message (W:212-238, W:252-268) and a worker reduces / completes
// as soon as the threshold number of them arrived (SB:9-13, RB:60-66), so a
// slow or dead peer does not stall the others.
//
// MI355X mapping of that message model:
//   * one HIP stream per peer and one point-to-point RCCL communicator per
//     pair (rccl_pair_p2p.cpp): transfers to different peers never wait for
//     each other, and each xGMI link carries its own peer's traffic;
//   * per (round, peer) two grouped exchanges on that pair's stream:
//       P1(r): my input slice of block p -> p,  p's slice of my block -> ring
//       P2(r): my reduced block + wire counts -> p,  p's reduced block -> landing
//     issued in the same order by both sides of every pair
//     (P1(0), P2(0), P1(1), P2(1), ...), so matching never depends on timing;
//   * arrival is an event completing on the pair stream: poll() queries the
//     in-flight events and hands completed arrivals to the unchanged Engine,
//     which applies the reference's thresholds, reduces on the compute stream,
//     completes rounds and runs catch-up -- without waiting for stragglers;
//   * P2(r) is issued once my block is fully reduced or the round completed
//     (then unreduced chunks go out with wire count 0 = "not reduced");
//   * the data plane runs in staged mode (per-round send slots + a landing
//     row), so transfers still in flight after a round completed never touch
//     memory the caller owns.  A frozen peer pins one send slot per round; the
//     pool grows up to `max_slots`, after which the oldest finished round's
//     slot is reclaimed by a GPU-side wait (the bounded-staleness limit).
// Counts travel in-band as count+1 (0 = chunk not reduced), copied to pinned
// host memory behind the receive so the host reads them at poll time.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../engine/engine.h"
#include "p2p.h"

namespace akka {

struct ReactiveLinkStats {
  int64_t groups = 0, bytes_sent = 0, p1_arrivals = 0, p2_arrivals = 0, unreduced_chunks = 0, polls = 0,
          reclaim_waits = 0, peers_lost = 0, transfers_dropped = 0;
};

class ReactiveLink final : public Link {
 public:
  ReactiveLink(Engine* engine, P2P* p2p, int32_t max_slots = 16);
  ~ReactiveLink() override;
  // Creates the per-peer streams and switches the data plane to staged mode.
  void bind(DataPlane* dp);

  void send_scatter(int32_t, int32_t, int32_t, const Payload&) override {}  // whole-block P1 from the staged input
  void send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) override;
  void on_scattered(int32_t round) override;
  void pump() override;
  bool may_finalize(int32_t round) override;
  void on_peer_lost(int32_t id) override;

  // Query in-flight transfers and deliver the completed ones to the engine.
  // Returns true if anything completed.
  bool poll();
  int32_t in_flight() const { return int32_t(pending_.size()); }
  // Block (without spinning) until a transfer may have completed since the
  // last call, or `timeout_us` elapsed.  Uses host notifications queued behind
  // every group; returns immediately if the device cannot notify.
  void wait_activity(int64_t timeout_us);
  const ReactiveLinkStats& stats() const { return stats_; }
  std::vector<StreamH> peer_streams() const { return streams_; }

 private:
  struct RoundState {
    bool scattered = false;
    bool closable = false;  // my block fully reduced, or the round completed
    std::vector<int32_t> wire;  // [kme] count+1, 0 = not reduced
    int32_t reduced = 0;
    int32_t open = 0;  // in-flight transfers of this round
    bool p2_issued = false;
    bool completed = false;
  };
  struct Pending {
    int32_t round = 0;
    int32_t peer = 0;
    int32_t phase = 0;
    EventH ev = nullptr;
    int32_t* counts = nullptr;  // pinned, phase 2
  };

  RoundState& st(int32_t r);
  // Peers this rank exchanges with in a round: in the engine's peer map at
  // issue time and not lost.  (Both sides of a pair must agree, which holds
  // when membership changes at a round boundary: InitWorkers / death.)
  bool exchanges_with(int32_t p) const;
  std::vector<uint8_t> lost_;  // [N]
  void issue_ready();
  void issue_p1(int32_t r);
  void issue_p2(int32_t r);
  bool reclaim(int32_t round);
  void retire(int32_t r);
  EventH get_event();
  void put_event(EventH e);
  int32_t* get_pinned();

  Engine* engine_;
  P2P* p2p_;
  DataPlane* dp_ = nullptr;
  Device* dev_ = nullptr;
  int32_t N_ = 0, me_ = 0, L_ = 0, kme_ = 0, kmax_ = 0, max_slots_ = 16;
  std::vector<StreamH> streams_;  // [N], null for me
  std::map<int32_t, RoundState> rounds_;
  int32_t next_round_ = 0;
  bool next_is_p2_ = false;
  bool issuing_ = false;
  std::deque<Pending> pending_;
  std::vector<EventH> events_, free_events_;
  std::vector<int32_t*> pinned_, free_pinned_;
  int32_t* recv_dev_ = nullptr;    // [L][N][kmax]
  ReactiveLinkStats stats_;
  // completion notifications (host callbacks from the pair streams)
  struct Notifier {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t count = 0;
  };
  std::shared_ptr<Notifier> notifier_ = std::make_shared<Notifier>();
  uint64_t seen_ = 0;
  bool notify_ok_ = true;
  void arm(StreamH s);
};

}  // namespace akka
