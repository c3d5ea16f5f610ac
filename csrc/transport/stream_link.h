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
#include <string>
#include <tuple>

#include "../engine/engine.h"
#include "ipc_lane.h"
#include "p2p.h"

namespace akka {

struct StreamLinkStats {
  int64_t groups = 0, ops = 0, bytes_sent = 0, rounds = 0, unreduced_chunks = 0;
  // bulk rounds by lane: collective = RCCL reduce-scatter + all-gather or the
  // whole-block exchange; exact_step_rounds = the exact p2p step template
  int64_t bulk_rounds = 0, collective_rounds = 0, exact_step_rounds = 0, graph_captures = 0, graph_replays = 0;
  int64_t ipc_rounds = 0;
};

// Which schedule runs an exact-threshold round (thReduce = thComplete = 1):
//  P2P        the chunk-pipelined step schedule below, like every other round;
//  Collective the bulk lane: RCCL reduce-scatter + all-gather over the whole
//             buffer when the geometry is even (S == N * step), otherwise a
//             whole-block direct exchange (one grouped p2p per phase around
//             one N-way reduce);
//  Auto       P2P: the framework's own schedule.  (Until round 2 Auto picked
//             RCCL's collectives when the geometry was even; they are now a
//             comparator that runs only when asked for by name.)
//  Ipc        one-sided xGMI loads/stores between mapped windows (ipc_lane.h),
//             once set_ipc() handed the link an opened IpcLane.
// Exact rounds never go through the engine's per-chunk message flow: their
// outcome is fixed (every chunk = sum of all N, count N), so the link runs
// them from a per-geometry op template with no engine callbacks, no op maps
// and no counts exchange (exact_steps).  Threshold rounds (< 1) take the
// message-driven step schedule (schedule()).  Which path a round takes is a
// function of the round's parameters only, identical on every rank (the
// schedules must match pairwise).
enum class Lane : int32_t { Auto = 0, P2P = 1, Collective = 2, Ipc = 3 };

class StreamLink final : public Link {
 public:
  StreamLink(Engine* engine, P2P* p2p, int32_t lag);
  ~StreamLink() override;
  void bind(DataPlane* dp) { dp_ = dp; }

  void send_scatter(int32_t dest, int32_t chunk, int32_t round, const Payload& p) override;
  void send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) override;
  void on_scattered(int32_t round) override;
  void pump() override;
  bool may_finalize(int32_t round) override;
  bool bulk_round(int32_t round) override;
  bool takes_exact_rounds() const override { return dp_ && dp_->geometry().N > 1; }

  void set_lane(Lane l) { lane_ = l; }
  // The one-sided lane's windows (created + opened by the caller); nullptr drops it.
  void set_ipc(std::unique_ptr<IpcLane> ipc);
  IpcLane* ipc() const { return ipc_.get(); }
  // Replay exact p2p-lane rounds from captured HIP graphs (off by default).
  void set_graphs(bool on);
  bool graphs() const { return graphs_; }
  const std::string& graph_error() const { return graph_error_; }
  int32_t exact_unit_chunks() const { return unit_chunks_; }
  // Minimum bytes of an exact-round transfer unit (< 0: AKKA_EXACT_UNIT_BYTES
  // or 16 MiB).  Rebuilds the template at the next exact round; like set_lane,
  // every rank must switch at the same round.
  void set_exact_unit_bytes(int64_t bytes);
  Lane lane() const { return lane_; }
  const StreamLinkStats& stats() const { return stats_; }
  int32_t lag() const { return lag_; }

 private:
  struct Out {
    const void* ptr = nullptr;
    int64_t len = 0;
  };
  // One op of the exact step template: base 0 = round input, 1 = ring row
  // of the round, 2 = round output; `off` in bytes from that base.
  struct OpT {
    bool send;
    int32_t peer;
    int8_t base;
    int64_t off;
    size_t bytes;
  };
  void build_exact_template();
  void exact_steps(int32_t round);
  void exact_body(int32_t round, char* const base[3], bool captured);
  // HIP-graph cache of exact rounds, keyed by their three base pointers
  // (input, ring row, output): a round seen twice is captured, later rounds
  // with the same buffers replay the graph (one launch instead of one RCCL
  // group + two event hops + one reduce launch per step).
  struct GraphEntry {
    GraphH exec = nullptr;
    int32_t seen = 0;
    uint64_t last_use = 0;
  };
  std::map<std::tuple<char*, char*, char*>, GraphEntry> graphs_map_;
  bool graphs_ = false;
  uint64_t tick_ = 0;
  int64_t exact_groups_ = 0, exact_ops_ = 0, exact_bytes_ = 0;
  std::string graph_error_;
  void collective_round(int32_t round, bool native);
  void ipc_round(int32_t round);
  std::unique_ptr<IpcLane> ipc_;
  StreamH ipc_last_stream_ = nullptr;  // stream of the lane's last engine-path round
  bool ipc_last_stream_set_ = false;
  std::vector<std::vector<OpT>> exact_;  // [step] -> ops
  Geometry gx_;                          // exact rounds' transfer units (unit_chunks_ chunks each)
  int32_t unit_chunks_ = 1;
  int64_t unit_bytes_ = -1;
  void drop_graphs();
  std::vector<P2POp> scratch_;
  std::vector<EventH> reduced_ev_;
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
