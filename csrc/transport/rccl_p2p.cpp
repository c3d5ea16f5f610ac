// RCCL point-to-point over xGMI (the production data plane).
//
// One communicator spanning all workers (rank = worker id).  Each schedule
// step is one ncclGroupStart/End holding a send and a recv per peer, so RCCL
// runs the transfers to all N-1 peers concurrently -- on a fully connected
// 8x MI355X node, one xGMI link per peer.  The unique id travels over the
// control plane (InitWorkers / torch TCPStore), see akka_allreduce_amd/parallel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

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

class RcclP2P final : public P2P {
 public:
  RcclP2P(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device)
      : rank_(rank), n_(nranks) {
    AKKA_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) throw AkkaError("akka: hipSetDevice failed");
    AKKA_NCCL(ncclCommInitRank(&comm_, nranks, id, rank));
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
      if (op.send) AKKA_NCCL(ncclSend(op.buf, op.bytes, ncclUint8, op.peer, comm_, s));
      else AKKA_NCCL(ncclRecv(op.buf, op.bytes, ncclUint8, op.peer, comm_, s));
    }
    AKKA_NCCL(ncclGroupEnd());
    ncclResult_t async = ncclSuccess;
    AKKA_NCCL(ncclCommGetAsyncError(comm_, &async));
    AKKA_CHECK(async == ncclSuccess, std::string("RCCL async error: ") + ncclGetErrorString(async));
  }

 private:
  int32_t rank_, n_;
  ncclComm_t comm_ = nullptr;
};

}  // namespace

std::unique_ptr<P2P> make_rccl_p2p(const std::vector<uint8_t>& uid, int32_t rank, int32_t nranks, int32_t device) {
  return std::make_unique<RcclP2P>(uid, rank, nranks, device);
}

}  // namespace akka
