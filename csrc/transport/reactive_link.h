// ReactiveLink: the straggler-tolerant GPU data path.
//
// StreamLink (stream_link.h) enqueues a round's whole schedule as symmetric
// all-peer groups on one comm stream, so a rank proceeds at the pace of its
// slowest peer: fast on a healthy node, but the threshold parameters
// (thReduce / thComplete) only decide *what* is summed, never *when*.
// The reference's point is the opposite: each ScatterBlock / ReduceBlock is an
// independent message of at most maxChunkSize floats (W:212-238, W:252-268),
// and a worker reduces a chunk the moment its threshold number of copies
// arrived and broadcasts it at once (W:177-181, SB:9-13); a round completes
// when enough reduced chunks arrived (RB:60-66).  A slow or dead peer does
// not stall the others.
//
// MI355X mapping of that message model:
//   * per peer one HIP stream and a point-to-point RCCL communicator
//     (rccl_p2p.cpp): transfers to different peers never wait for each
//     other, each xGMI link carries its own peer's traffic;
//   * chunks move in transfer groups of gm consecutive chunks (gm = 1 when a
//     chunk is >= 16 MiB; small maxChunkSize is batched so a group carries
//     >= 16 MiB -- fixed bounds, the same on every rank):
//       P1(r,g): chunks of group g of my input slice of block p -> p,
//                those of p's slice of my block -> ring slot       (channel 0)
//       P2(r,g): my reduced chunks of group g + their counts -> p,
//                p's reduced chunks + counts -> landing row        (channel 1)
//     and every chunk is still delivered, reduced and counted on its own;
//     Both sides of a pair issue the same total order -- P1(r, all chunks)
//     at scatter time, then P2(r, k) in chunk order as chunks get reduced,
//     then P1(r+1) ... -- so matching never depends on timing (the two phases
//     also use separate matching channels);
//   * arrival is an event completing on the pair stream, per chunk: poll()
//     hands completed arrivals to the unchanged Engine, which applies the
//     reference's thresholds, reduces chunk k on the compute stream, completes
//     rounds and runs catch-up -- without waiting for stragglers;
//   * P2(r,g) is issued as soon as my chunks of group g are reduced (each
//     count rides in its reduce launch: a 4-byte fill merged into it), or once
//     the round completed (then unreduced chunks go out with count 0);
//   * the data plane runs in staged mode (per-round send slots + a landing
//     row), so transfers still in flight after a round completed never touch
//     memory the caller owns.  A frozen peer pins one send slot per round; the
//     pool grows up to `max_slots`, after which the oldest finished round's
//     slot is reclaimed by a GPU-side wait (the bounded-staleness limit).
// Counts travel in-band as count+1 (0 = chunk not reduced), copied to pinned
// host memory behind each receive so the host reads them at poll time.
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
  // P2 chunks issued while P1 chunks of the same round were still in flight
  // (the per-chunk pipeline at work)
  int64_t p2_overlapped = 0;
};

class ReactiveLink final : public Link {
 public:
  ReactiveLink(Engine* engine, P2P* p2p, int32_t max_slots = 16);
  ~ReactiveLink() override;
  // Creates the per-peer streams and switches the data plane to staged mode.
  void bind(DataPlane* dp);

  void send_scatter(int32_t, int32_t, int32_t, const Payload&) override {}  // P1 chunks come from the staged input
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
  // the groups; returns immediately if the device cannot notify.
  void wait_activity(int64_t timeout_us);
  const ReactiveLinkStats& stats() const { return stats_; }
  std::vector<StreamH> peer_streams() const { return s1_; }

 private:
  struct RoundState {
    bool scattered = false;
    bool completed = false;
    bool p1_issued = false;
    std::vector<int32_t> wire;    // [kme] count+1, 0 = not reduced
    std::vector<EventH> ready;    // [kme] compute event after chunk k's reduce + count fill
    int32_t p2_next = 0;          // first chunk index whose P2 groups are not issued
    int32_t open = 0;             // in-flight transfers of this round
    int32_t p1_open = 0;          // of which phase 1
    bool p2_done = false;         // every P2 chunk issued
  };
  struct Pending {
    int32_t round = 0;
    int32_t peer = 0;
    int32_t phase = 0;
    int32_t chunk = 0;      // first chunk of the group
    int32_t chunk_end = 0;  // one past its last chunk
    EventH ev = nullptr;
    int32_t* count = nullptr;  // pinned row, phase 2
  };

  RoundState& st(int32_t r);
  // Peers this rank exchanges with in a round: in the engine's peer map at
  // issue time and not lost.  (Both sides of a pair must agree, which holds
  // when membership changes at a round boundary: InitWorkers / death.)
  bool exchanges_with(int32_t p) const;
  void issue_ready();
  void issue_p1(int32_t r);
  // Issue P2 chunks of round r that are ready; true once all are issued.
  bool issue_p2(int32_t r);
  bool reclaim(int32_t round);
  void retire(int32_t r);
  EventH get_event();
  void put_event(EventH e);
  int32_t* get_count_slot();
  int32_t chunks_with(int32_t p) const;  // chunk indices exchanged per round with peer p
  int64_t span_len(int32_t block, int32_t k0, int32_t k1) const;
  int32_t gm_ = 1;  // chunks per transfer group

  Engine* engine_;
  P2P* p2p_;
  DataPlane* dp_ = nullptr;
  Device* dev_ = nullptr;
  int32_t N_ = 0, me_ = 0, L_ = 0, kme_ = 0, kmax_ = 0, max_slots_ = 16;
  std::vector<StreamH> s1_, s2_;  // [N] phase-1 / phase-2 pair streams (one stream per peer today), null for me
  std::vector<uint8_t> lost_;     // [N]
  std::map<int32_t, RoundState> rounds_;
  int32_t p1_round_ = 0;  // next round whose P1 is not issued (== p2_round_ or p2_round_ + 1)
  int32_t p2_round_ = 0;  // round whose P2 chunks are being issued
  bool issuing_ = false;
  std::deque<Pending> pending_;
  std::vector<EventH> events_, free_events_;
  std::vector<int32_t*> pinned_blocks_, free_counts_;
  int32_t* recv_dev_ = nullptr;  // [L][N][kmax]
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
