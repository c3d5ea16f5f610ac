// StreamLink: the production data path.  Turns the engine's per-chunk sends
// into a symmetric, pipelined schedule of grouped p2p steps on the comm
// stream, with the chunk reduce on the compute stream in between.
//
// Reference data path (what this replaces):
//   scatter:   W:212-238  one ScatterBlock per (peer, chunk) over Akka/TCP
//   reduce:    W:177-181 + SB:20-32  at the reduce threshold
//   broadcast: W:252-268  one ReduceBlock per peer
// MI355X mapping (step s of round r, one RCCL group on the comm stream):
//   { scatter chunk s of block j -> worker j,   for every peer j     (phase 1)
//     recv my chunk s from every peer into the scatter ring slot
//     broadcast my reduced chunk s-LAG -> every peer                  (phase 2)
//     recv chunk s-LAG of block j from j straight into the output }
// All 7 xGMI links of a GPU carry traffic in both phases at once, and the
// reduce of chunk s (compute stream) overlaps step s+1's transfers; LAG=2 keeps
// the comm stream from ever waiting on a reduce.  The last step also carries
// each rank's per-chunk contributor counts (the ReduceBlock.count field).
//
// "Arrival" is stream-ordered: right after a step's group is enqueued the link
// reports its receives to the engine as landed; everything the engine does in
// response (reduce, broadcast, completion) is enqueued behind the group, so the
// host never blocks on the GPU and the round/threshold state machine is the
// same code as in every other transport.
#pragma once

#include <deque>
#include <map>
#include <set>

#include "../engine/engine.h"
#include "p2p.h"

namespace akka {

struct StreamLinkStats {
  int64_t groups = 0, ops = 0, bytes_sent = 0, rounds = 0, unreduced_chunks = 0;
  int64_t bulk_rounds = 0, collective_rounds = 0;
};

// Which schedule runs an exact-threshold round (thReduce = thComplete = 1):
//  P2P        the chunk-pipelined step schedule below, like every other round;
//  Collective the bulk lane: RCCL reduce-scatter + all-gather over the whole
//             buffer when the geometry is even (S == N * step), otherwise a
//             whole-block direct exchange (one grouped p2p per phase around
//             one N-way reduce);
//  Auto       Collective when the transport has native collectives and the
//             geometry is even, else P2P.
// Threshold rounds (< 1) always take the step schedule.
enum class Lane : int32_t { Auto = 0, P2P = 1, Collective = 2 };

class StreamLink final : public Link {
 public:
  StreamLink(Engine* engine, P2P* p2p, int32_t lag);
  void bind(DataPlane* dp) { dp_ = dp; }

  void send_scatter(int32_t dest, int32_t chunk, int32_t round, const Payload& p) override;
  void send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) override;
  void on_scattered(int32_t round) override;
  void pump() override;
  bool may_finalize(int32_t round) override;
  bool bulk_round(int32_t round) override;

  void set_lane(Lane l) { lane_ = l; }
  Lane lane() const { return lane_; }
  const StreamLinkStats& stats() const { return stats_; }
  int32_t lag() const { return lag_; }

 private:
  struct Out {
    const void* ptr = nullptr;
    int64_t len = 0;
  };
  struct RoundQ {
    std::map<std::pair<int32_t, int32_t>, Out> scatter;  // (chunk, dest)
    std::map<std::pair<int32_t, int32_t>, Out> bcast;    // (chunk, dest)
    std::map<int32_t, EventH> bcast_ready;               // chunk -> compute event after its reduce
  };
  void schedule(int32_t round);
  void mark_scheduled(int32_t round);

  Engine* engine_;
  P2P* p2p_;
  DataPlane* dp_ = nullptr;
  int32_t lag_;
  std::map<int32_t, RoundQ> q_;
  std::deque<int32_t> ready_;
  std::set<int32_t> in_flight_;
  std::set<int32_t> scheduled_;
  bool pumping_ = false;
  Lane lane_ = Lane::Auto;
  StreamLinkStats stats_;
};

}  // namespace akka
