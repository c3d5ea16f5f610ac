// Grouped point-to-point transport.
//
// The reference's data plane is Akka remoting: every ScatterBlock/ReduceBlock
// is an independent TCP message into an unbounded mailbox.  On
// MI355X the data plane is RCCL send/recv over xGMI: a group of sends/recvs to
// all peers runs concurrently, one peer per xGMI link.  RCCL p2p is a
// rendezvous (a send completes only against the matching recv, matched in
// issue order per peer pair), so the schedule that issues the groups
// (stream_link.h) must be symmetric across ranks; SimP2P checks exactly that
// on the CPU.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../engine/device.h"

namespace akka {

struct P2POp {
  bool send = false;
  int32_t peer = -1;
  void* buf = nullptr;
  size_t bytes = 0;
  // Independent ordering domain (pair transports): channel 0 and 1 of a pair
  // match separately, so phase-2 chunks never queue behind phase-1 chunks
  // (RCCL: one pair communicator per channel).  Global transports: 0 only.
  int32_t channel = 0;
};

// What the transport itself reports about its communicator(s): for RCCL the
// values come from ncclCommCount / ncclCommUserRank / ncclCommCuDevice, not
// from the arguments it was built with (the bench prints them as proof that
// RCCL really saw N ranks).
struct P2PInfo {
  std::string kind;
  int32_t nranks = 0;
  int32_t rank = -1;
  int32_t device = -1;
  int32_t comms = 0;  // communicators held (global + pair comms)
};

class P2P {
 public:
  virtual ~P2P() = default;
  virtual int32_t rank() const = 0;
  virtual int32_t nranks() const = 0;
  // Enqueue one group of ops on `stream` (RCCL: ncclGroupStart .. ncclGroupEnd).
  virtual void group(StreamH stream, const std::vector<P2POp>& ops) = 0;
  virtual const char* name() const = 0;
  virtual P2PInfo info() const { return P2PInfo{name(), nranks(), rank(), -1, 0}; }
  // Surface asynchronous transport errors (RCCL: ncclCommGetAsyncError on
  // every communicator).  Links call it once per round, not per group.
  virtual void check() {}

  // Whole-buffer collectives over all ranks (the exact-threshold fast lane,
  // stream_link.h): `count` elements per rank.  reduce_scatter: recv = sum
  // over ranks of send[rank*count ..]; all_gather: recv[r*count ..] = rank r's
  // send (in place when send == recv + rank*count).  Default: unsupported.
  // A peer died (the control plane said so): end every transfer with it that
  // is queued or in flight, so streams parked on it move on, and never match
  // with it again.  RCCL pair communicators: ncclCommAbort of that pair's
  // communicator.  Transports whose communicator spans all ranks cannot
  // abort one peer (they are rebuilt over the survivors instead): false.
  virtual bool abort_peer(int32_t /*peer*/) { return false; }
  // New membership epoch (the control plane's re-InitWorkers after a death or
  // a join): drop the old communicator and build one over `members` (engine
  // ids, ascending; comm rank = index) from a fresh unique id.  Transports
  // keyed by engine ids directly need nothing: false.
  virtual bool rebuild(const std::vector<uint8_t>& /*uid*/, const std::vector<int32_t>& /*members*/) {
    return false;
  }

  // Transports over mapped peer memory (ipc_p2p.cpp): this rank's handle,
  // to be exchanged with every rank, then open() with all of them.
  virtual std::string handle() const { throw AkkaError(std::string("akka: ") + name() + " p2p has no handle"); }
  virtual void open(const std::vector<std::string>&) {
    throw AkkaError(std::string("akka: ") + name() + " p2p has nothing to open");
  }
  virtual bool has_collectives() const { return false; }
  virtual void reduce_scatter(StreamH, const void*, void*, size_t, DType) {
    throw AkkaError(std::string("akka: ") + name() + " p2p has no reduce_scatter");
  }
  virtual void all_gather(StreamH, const void*, void*, size_t, DType) {
    throw AkkaError(std::string("akka: ") + name() + " p2p has no all_gather");
  }
};

// No two-sided transport: a job whose exact rounds all run on the one-sided
// ipc lane (ipc_lane.h).  Any message-driven schedule fails loudly.
class NullP2P final : public P2P {
 public:
  NullP2P(int32_t rank, int32_t nranks) : rank_(rank), nranks_(nranks) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return nranks_; }
  void group(StreamH, const std::vector<P2POp>&) override {
    throw AkkaError("akka: this job has no p2p transport (ipc-only data plane): only exact rounds on the ipc lane");
  }
  const char* name() const override { return "none"; }

 private:
  int32_t rank_, nranks_;
};

// ---- CPU simulator ------------------------------------------------------------
class SimHub;
std::shared_ptr<SimHub> make_sim_hub(int32_t nranks, bool collectives = false);
// Endpoint for `rank`; ops are queued on the rank's deferred host device.
std::unique_ptr<P2P> make_sim_p2p(std::shared_ptr<SimHub> hub, int32_t rank, Device* dev);
// Drive all ranks' deferred devices until every queue is empty.  Throws with a
// diagnostic if no rank can make progress (a schedule deadlock).
void sim_run(const std::shared_ptr<SimHub>& hub, const std::vector<Device*>& devices, int64_t max_iters);
int64_t sim_bytes_moved(const std::shared_ptr<SimHub>& hub);
int64_t sim_events(const std::shared_ptr<SimHub>& hub);
// Step every stream of the given (deferred host) devices once; returns progress.
bool sim_step(const std::shared_ptr<SimHub>& hub, const std::vector<Device*>& devices, uint32_t rotate);

// ---- RCCL ---------------------------------------------------------------------
std::vector<uint8_t> rccl_unique_id();
// `members`: engine ids in the communicator (empty = all nranks); the
// communicator rank of engine id m is its index in `members`.
std::unique_ptr<P2P> make_rccl_p2p(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device,
                                   const std::vector<int32_t>& members = {});
// Round-robin tournament (circle method) used to split the global communicator
// into pair communicators: in round t (0 <= t < P-1, P = N rounded up to even)
// rank x is paired with tournament_partner(N, t, x); a partner >= N means x
// sits this round out (odd N).  Every unordered pair meets exactly once.
inline int32_t tournament_partner(int32_t n, int32_t t, int32_t x) {
  const int32_t P = (n % 2) ? n + 1 : n;
  if (x == P - 1) return t;
  if (x == t) return P - 1;
  return ((2 * t - x) % (P - 1) + (P - 1)) % (P - 1);
}
inline int32_t tournament_rounds(int32_t n) { return ((n % 2) ? n + 1 : n) - 1; }

// Per-pair communicators (reactive transport): a group holds ops to one peer
// on one channel; two communicators per pair (channel 0: phase 1, channel 1:
// phase 2).
std::unique_ptr<P2P> make_rccl_pair_p2p(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks,
                                        int32_t device);
const char* rccl_version_string();
// ---- mapped peer memory (xGMI) ---------------------------------------------------
// Grouped send/recv through mailboxes in every rank's window (ipc_p2p.cpp);
// handle() / open() exchange the windows before the first group.
std::unique_ptr<P2P> make_ipc_p2p(int32_t rank, int32_t nranks, int32_t device);

// One-GPU shape rehearsal (1-rank comm posing as rank/nranks, ops to self).
std::unique_ptr<P2P> make_rccl_shape_p2p(int32_t rank, int32_t nranks, int32_t device);

}  // namespace akka
