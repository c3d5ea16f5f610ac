// RCCL point-to-point over xGMI (the production data plane).
//
// One communicator spanning all workers (rank = worker id).  Each schedule
// step is one ncclGroupStart/End holding a send and a recv per peer, so RCCL
// runs the transfers to all N-1 peers concurrently -- on a fully connected
// 8x MI355X node, one xGMI link per peer.  The unique id travels over the
// control plane (InitWorkers / torch TCPStore), see akka_allreduce_amd/parallel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <sstream>

#include "p2p.h"

namespace akka {

#define AKKA_NCCL(call)                                                                          \
  do {                                                                                           \
    ncclResult_t r_ = (call);                                                                    \
    if (r_ != ncclSuccess)                                                                       \
      throw AkkaError(std::string("akka: ") + #call + " failed: " + ncclGetErrorString(r_));     \
  } while (0)

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  AKKA_NCCL(ncclGetUniqueId(&id));
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id));
}

const char* rccl_version_string() {
  static std::string s;
  if (s.empty()) {
    int v = 0;
    ncclGetVersion(&v);
    std::ostringstream os;
    os << v / 10000 << "." << (v / 100) % 100 << "." << v % 100;
    s = os.str();
  }
  return s.c_str();
}

namespace {

// Ask RCCL what it actually built: rank count, this rank, device.  A mismatch
// (e.g. two ranks resolved to one card, or a stale unique id joining another
// job) fails here, at init, instead of as a hang in the first group.
void verify_comm(ncclComm_t c, int32_t want_n, int32_t want_rank, int32_t want_dev, const char* what) {
  int n = -1, r = -1, d = -1;
  AKKA_NCCL(ncclCommCount(c, &n));
  AKKA_NCCL(ncclCommUserRank(c, &r));
  AKKA_NCCL(ncclCommCuDevice(c, &d));
  if (n != want_n || r != want_rank || (want_dev >= 0 && d != want_dev)) {
    std::ostringstream os;
    os << "akka: RCCL " << what << " communicator reports nranks=" << n << " rank=" << r << " device=" << d
       << ", expected nranks=" << want_n << " rank=" << want_rank << " device=" << want_dev;
    throw AkkaError(os.str());
  }
}

void check_async(ncclComm_t c, const char* what) {
  if (!c) return;
  ncclResult_t async = ncclSuccess;
  AKKA_NCCL(ncclCommGetAsyncError(c, &async));
  if (async != ncclSuccess && async != ncclInProgress)
    throw AkkaError(std::string("akka: RCCL async error on ") + what + " communicator: " + ncclGetErrorString(async));
}

class RcclP2P final : public P2P {
 public:
  RcclP2P(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device,
          const std::vector<int32_t>& members)
      : rank_(rank), n_(nranks), device_(device) {
    if (hipSetDevice(device) != hipSuccess) throw AkkaError("akka: hipSetDevice failed");
    connect(uid, members);
  }
  ~RcclP2P() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "rccl"; }

  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    AKKA_NCCL(ncclGroupStart());
    for (const auto& op : ops) {
      const int32_t cr = comm_rank(op.peer);
      if (op.send) AKKA_NCCL(ncclSend(op.buf, op.bytes, ncclUint8, cr, comm_, s));
      else AKKA_NCCL(ncclRecv(op.buf, op.bytes, ncclUint8, cr, comm_, s));
    }
    AKKA_NCCL(ncclGroupEnd());
  }
  P2PInfo info() const override {
    int n = -1, r = -1, d = -1;
    ncclCommCount(comm_, &n);
    ncclCommUserRank(comm_, &r);
    ncclCommCuDevice(comm_, &d);
    return P2PInfo{name(), n, r, d, 1};
  }
  void check() override { check_async(comm_, "global"); }

  bool rebuild(const std::vector<uint8_t>& uid, const std::vector<int32_t>& members) override {
    if (comm_) {
      // A member may be dead with kernels of ours still parked on it: abort
      // (destroy would wait for them).  Rounds in flight at that moment are lost.
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
    connect(uid, members);
    return true;
  }

  bool has_collectives() const override { return int32_t(members_.size()) == n_; }
  void reduce_scatter(StreamH stream, const void* send, void* recv, size_t count, DType dt) override {
    AKKA_CHECK(has_collectives(), "reduce_scatter needs every rank in the communicator");
    AKKA_NCCL(ncclReduceScatter(send, recv, count, nccl_type(dt), ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void all_gather(StreamH stream, const void* send, void* recv, size_t count, DType dt) override {
    AKKA_CHECK(has_collectives(), "all_gather needs every rank in the communicator");
    AKKA_NCCL(ncclAllGather(send, recv, count, nccl_type(dt), comm_, static_cast<hipStream_t>(stream)));
  }

 private:
  void connect(const std::vector<uint8_t>& uid, const std::vector<int32_t>& members) {
    AKKA_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    members_ = members;
    if (members_.empty())
      for (int32_t i = 0; i < n_; ++i) members_.push_back(i);
    comm_rank_.assign(size_t(n_), -1);
    int32_t mine = -1;
    for (size_t i = 0; i < members_.size(); ++i) {
      const int32_t m = members_[i];
      AKKA_CHECK(m >= 0 && m < n_ && comm_rank_[size_t(m)] < 0, "bad communicator member list");
      comm_rank_[size_t(m)] = int32_t(i);
      if (m == rank_) mine = int32_t(i);
    }
    AKKA_CHECK(mine >= 0, "this rank is not a member of the communicator it should join");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (hipSetDevice(device_) != hipSuccess) throw AkkaError("akka: hipSetDevice failed");
    AKKA_NCCL(ncclCommInitRank(&comm_, int(members_.size()), id, mine));
    verify_comm(comm_, int32_t(members_.size()), mine, device_, "global");
  }
  int32_t comm_rank(int32_t peer) const {
    AKKA_CHECK(peer >= 0 && peer < n_ && comm_rank_[size_t(peer)] >= 0,
               "p2p op to worker " + std::to_string(peer) + ", which is not in the communicator");
    return comm_rank_[size_t(peer)];
  }
  static ncclDataType_t nccl_type(DType dt) { return dt == DType::BF16 ? ncclBfloat16 : ncclFloat32; }
  int32_t rank_, n_;
  int32_t device_ = -1;
  ncclComm_t comm_ = nullptr;
  std::vector<int32_t> members_;
  std::vector<int32_t> comm_rank_;  // [n] engine id -> communicator rank (-1: not a member)
};

// One two-rank communicator per peer pair, split off the global one.  A group
// may only hold ops to a single peer; it runs on that pair's communicator, so
// transfers to different peers (issued on different streams) are independent
// -- a slow peer stalls only its own pair (reactive_link.h).
class RcclPairP2P final : public P2P {
 public:
  RcclPairP2P(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device)
      : rank_(rank), n_(nranks) {
    AKKA_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) throw AkkaError("akka: hipSetDevice failed");
    AKKA_NCCL(ncclCommInitRank(&global_, nranks, id, rank));
    verify_comm(global_, nranks, rank, device, "global");
    // Round-robin tournament (circle method): P-1 rounds of disjoint pairs,
    // one ncclCommSplit per channel each; with odd N a dummy player sits one
    // rank out.  Every rank runs the same sequence of splits.
    for (int32_t ch = 0; ch < kChannels; ++ch) {
      pair_[ch].assign(size_t(nranks), nullptr);
      for (int32_t t = 0; t < tournament_rounds(nranks); ++t) {
        const int32_t partner = tournament_partner(nranks, t, rank);
        const bool real = partner < nranks && partner != rank;
        ncclComm_t c = nullptr;
        AKKA_NCCL(ncclCommSplit(global_, real ? std::min(rank, partner) : NCCL_SPLIT_NOCOLOR, rank, &c, nullptr));
        if (real) pair_[ch][size_t(partner)] = c;
      }
      for (int32_t p = 0; p < nranks; ++p) {
        if (p == rank) continue;
        AKKA_CHECK(pair_[ch][size_t(p)], "pair communicator missing for peer " + std::to_string(p));
        // split key = global rank: the lower global rank is pair rank 0
        verify_comm(pair_[ch][size_t(p)], 2, rank < p ? 0 : 1, device, "pair");
      }
    }
  }
  ~RcclPairP2P() override {
    for (auto& v : pair_)
      for (ncclComm_t c : v)
        if (c) ncclCommDestroy(c);
    if (global_) ncclCommDestroy(global_);
  }
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "rccl-pair"; }

  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    if (ops.empty()) return;
    const int32_t peer = ops.front().peer;
    const int32_t ch = ops.front().channel;
    AKKA_CHECK(peer >= 0 && peer < n_ && peer != rank_, "pair group: bad peer");
    AKKA_CHECK(ch >= 0, "pair group: bad channel");
    // The reactive link issues both phases of a pair on ONE stream in one
    // total order both sides share, so one communicator per pair serves both
    // channels (fewer RCCL communicators to build at N = 8).
    ncclComm_t c = pair_[std::min(ch, kChannels - 1)][size_t(peer)];
    AKKA_CHECK(c, "pair group to peer " + std::to_string(peer) + " after its communicator was aborted");
    const int32_t prank = peer < rank_ ? 0 : 1;  // split key = global rank
    hipStream_t s = static_cast<hipStream_t>(stream);
    AKKA_NCCL(ncclGroupStart());
    for (const auto& op : ops) {
      AKKA_CHECK(op.peer == peer, "pair group holds ops to more than one peer");
      if (op.send) AKKA_NCCL(ncclSend(op.buf, op.bytes, ncclUint8, prank, c, s));
      else AKKA_NCCL(ncclRecv(op.buf, op.bytes, ncclUint8, prank, c, s));
    }
    AKKA_NCCL(ncclGroupEnd());
  }
  bool abort_peer(int32_t peer) override {
    if (peer < 0 || peer >= n_ || peer == rank_) return false;
    for (auto& v : pair_) {
      ncclComm_t& c = v[size_t(peer)];
      if (c) {
        // Kernels parked on the dead peer exit; the pair streams move on.  The
        // communicators are gone: every later group to that peer is an error.
        ncclCommAbort(c);
        c = nullptr;
      }
    }
    aborted_.push_back(peer);
    return true;
  }
  P2PInfo info() const override {
    int n = -1, r = -1, d = -1;
    ncclCommCount(global_, &n);
    ncclCommUserRank(global_, &r);
    ncclCommCuDevice(global_, &d);
    int32_t comms = 1;
    for (const auto& v : pair_)
      for (ncclComm_t c : v) comms += c ? 1 : 0;
    return P2PInfo{name(), n, r, d, comms};
  }
  void check() override {
    // the global communicator spans the dead rank too: only the pairs matter
    // once a peer was aborted
    if (aborted_.empty()) check_async(global_, "global");
    for (const auto& v : pair_)
      for (ncclComm_t c : v) check_async(c, "pair");
  }

 private:
  static constexpr int32_t kChannels = 1;
  int32_t rank_, n_;
  ncclComm_t global_ = nullptr;
  std::vector<ncclComm_t> pair_[kChannels];  // [channel][peer]
  std::vector<int32_t> aborted_;
};

// Shape rehearsal on ONE GPU: a 1-rank RCCL communicator that presents
// itself as rank `rank` of `nranks` and sends every op to itself.  In an
// exact round of an even geometry the k-th send and the k-th receive of a
// group have the same size, so RCCL matches them pairwise; the bytes are
// meaningless but the host path (engine, link, ncclGroupStart/End with the
// N-rank group shape) and the GPU p2p kernels are the real ones.  Used to
// measure the host cost per round of the N=8 schedule on a 1-GPU box.
class RcclShapeP2P final : public P2P {
 public:
  RcclShapeP2P(int32_t rank, int32_t nranks, int32_t device) : rank_(rank), n_(nranks) {
    if (hipSetDevice(device) != hipSuccess) throw AkkaError("akka: hipSetDevice failed");
    ncclUniqueId id;
    AKKA_NCCL(ncclGetUniqueId(&id));
    AKKA_NCCL(ncclCommInitRank(&comm_, 1, id, 0));
    verify_comm(comm_, 1, 0, device, "shape");
  }
  ~RcclShapeP2P() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "rccl-shape"; }
  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    AKKA_NCCL(ncclGroupStart());
    for (const auto& op : ops) {
      if (op.send) AKKA_NCCL(ncclSend(op.buf, op.bytes, ncclUint8, 0, comm_, s));
      else AKKA_NCCL(ncclRecv(op.buf, op.bytes, ncclUint8, 0, comm_, s));
    }
    AKKA_NCCL(ncclGroupEnd());
  }
  void check() override { check_async(comm_, "shape"); }

 private:
  int32_t rank_, n_;
  ncclComm_t comm_ = nullptr;
};

}  // namespace

std::unique_ptr<P2P> make_rccl_shape_p2p(int32_t rank, int32_t nranks, int32_t device) {
  return std::make_unique<RcclShapeP2P>(rank, nranks, device);
}

std::unique_ptr<P2P> make_rccl_pair_p2p(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks,
                                        int32_t device) {
  return std::make_unique<RcclPairP2P>(uid, rank, nranks, device);
}

std::unique_ptr<P2P> make_rccl_p2p(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device,
                                   const std::vector<int32_t>& members) {
  return std::make_unique<RcclP2P>(uid, rank, nranks, device, members);
}

}  // namespace akka
