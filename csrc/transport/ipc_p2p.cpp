// IpcP2P: the P2P interface (grouped send / recv, matched in issue order per
// pair and channel) over mapped peer memory instead of RCCL.
//
// Every rank's window holds mailboxes, one ring of slots per (source rank,
// channel); a send copies its bytes into the receiver's mailbox over xGMI and
// raises per-slot flags there, the matching recv copies them out into its
// destination and hands the slot back (ipc_kernels.h for the layout).  A group
// is ONE kernel launch in which every (direction, peer, channel) queue runs
// concurrently -- the same progress guarantee as an RCCL group, so the
// schedules of StreamLink and ReactiveLink run on it unchanged, with their
// thresholds, catch-up and per-peer streams.  Waits are bounded and also end
// when the host aborts a peer (abort_peer): a dead rank costs its partners a
// dropped transfer, never a hung GPU.
//
// Why: (1) the whole transport stack runs without RCCL, so several ranks can
// share one GPU (RCCL refuses two ranks on one device) and every schedule --
// including the straggler-tolerant one -- is tested across real processes on
// a one-GPU box; (2) on a node it is a second p2p engine next to RCCL's, with
// no proxy and no channel setup.  The reference's Akka remoting hop (W:212-268
// ScatterBlock / ReduceBlock messages) mapped onto xGMI stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>

#include "../kernels/ipc_kernels.h"
#include "ipc_lane.h"
#include "ipc_p2p.h"
#include "p2p.h"

namespace akka {

#define AKKA_P2P_HIP(call)                                                                       \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      throw AkkaError(std::string("akka ipc p2p: ") + #call + " failed: " + hipGetErrorString(e_)); \
  } while (0)

namespace {

constexpr char kMagic[8] = {'A', 'K', 'P', '2', 'P', '0', '1', 0};
constexpr int32_t kChannels = 2;

struct Blob {
  char magic[8];
  int32_t rank, nranks, nslots, wpp;
  int64_t piece;
  hipIpcMemHandle_t mbox, flags;
};

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoll(v) : dflt;
}

class IpcP2P final : public P2P {
 public:
  IpcP2P(int32_t rank, int32_t nranks, int32_t device) : rank_(rank), n_(nranks), device_(device) {
    AKKA_CHECK(n_ >= 1 && n_ <= kIpcMaxRanks, "ipc p2p: 1..16 ranks");
    AKKA_P2P_HIP(hipSetDevice(device_));
    piece_ = std::max<int64_t>(1 << 16, env_i64("AKKA_IPC_P2P_PIECE_BYTES", int64_t(4) << 20)) / 16 * 16;
    nslots_ = int32_t(std::clamp<int64_t>(env_i64("AKKA_IPC_P2P_SLOTS", 4), 2, 64));
    // workgroups per piece: 32 keeps more copies in flight (-6 % per 256 MiB round
    // vs 8 on 4 ranks sharing a card, profiles/r02/ipc_p2p)
    wpp_ = int32_t(std::clamp<int64_t>(env_i64("AKKA_IPC_P2P_WGS", 32), 1, 64));
    // A group's workgroups must all be resident at once; keep the grid within
    // half of what the device holds (the other half: other kernels, other
    // ranks sharing the card in tests) by giving each queue fewer workgroups
    // than parts when needed (each then serves several parts).
    grid_cap_ = std::max(1, ipc_p2p_resident_wgs(device_) / 2);
    mbox_bytes_ = size_t(n_) * kChannels * size_t(nslots_) * size_t(piece_);
    flag_bytes_ = ipc_p2p_flag_bytes(n_, kChannels, nslots_, wpp_);
    mbox_ = static_cast<char*>(ipc_alloc_window(mbox_bytes_, &mem_kind_));  // fine-grained (ipc_lane.h)
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flag_bytes_, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      AKKA_P2P_HIP(hipMalloc(reinterpret_cast<void**>(&flags_), flag_bytes_));
    }
    AKKA_P2P_HIP(hipMemset(flags_, 0, flag_bytes_));
    // error word + dead-peer table live in host memory the kernels write / read
    AKKA_P2P_HIP(hipHostMalloc(reinterpret_cast<void**>(&host_), sizeof(uint32_t) * (1 + kIpcMaxRanks),
                               hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(host_, 0, sizeof(uint32_t) * (1 + kIpcMaxRanks));
    AKKA_P2P_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_dev_), host_, 0));
    AKKA_P2P_HIP(hipDeviceSynchronize());
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || khz <= 0) khz = 100000;
    timeout_ = uint64_t(std::max<int64_t>(1, env_i64("AKKA_IPC_TIMEOUT_MS", 60000))) * uint64_t(khz);
    peer_mbox_.assign(size_t(n_), nullptr);
    peer_flags_.assign(size_t(n_), nullptr);
    peer_mbox_[size_t(rank_)] = mbox_;
    peer_flags_[size_t(rank_)] = flags_;
    send_seq_.assign(size_t(n_) * kChannels, 0);
    recv_seq_.assign(size_t(n_) * kChannels, 0);
  }
  ~IpcP2P() override {
    hipSetDevice(device_);
    hipDeviceSynchronize();
    for (int32_t p = 0; p < n_; ++p) {
      if (p == rank_) continue;
      if (peer_mbox_[size_t(p)]) hipIpcCloseMemHandle(peer_mbox_[size_t(p)]);
      if (peer_flags_[size_t(p)]) hipIpcCloseMemHandle(peer_flags_[size_t(p)]);
    }
    if (mbox_) hipFree(mbox_);
    if (flags_) hipFree(flags_);
    if (host_) hipHostFree(host_);
  }

  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return n_; }
  const char* name() const override { return "ipc"; }
  P2PInfo info() const override { return P2PInfo{"ipc", n_, rank_, device_, 0}; }
  const std::string& memory_kind() const { return mem_kind_; }

  std::string handle() const override {
    Blob b;
    std::memset(&b, 0, sizeof(b));
    std::memcpy(b.magic, kMagic, sizeof(kMagic));
    b.rank = rank_;
    b.nranks = n_;
    b.nslots = nslots_;
    b.wpp = wpp_;
    b.piece = piece_;
    AKKA_P2P_HIP(hipIpcGetMemHandle(&b.mbox, mbox_));
    AKKA_P2P_HIP(hipIpcGetMemHandle(&b.flags, flags_));
    return std::string(reinterpret_cast<const char*>(&b), sizeof(b));
  }

  void open(const std::vector<std::string>& handles) override {
    AKKA_CHECK(!ready_, "ipc p2p: already open");
    AKKA_CHECK(int32_t(handles.size()) == n_, "ipc p2p: need one handle per rank");
    AKKA_P2P_HIP(hipSetDevice(device_));
    for (int32_t p = 0; p < n_; ++p) {
      const std::string& h = handles[size_t(p)];
      AKKA_CHECK(h.size() == sizeof(Blob), "ipc p2p: malformed handle");
      Blob b;
      std::memcpy(&b, h.data(), sizeof(b));
      AKKA_CHECK(std::memcmp(b.magic, kMagic, sizeof(kMagic)) == 0, "ipc p2p: not a mailbox handle");
      AKKA_CHECK(b.rank == p && b.nranks == n_ && b.nslots == nslots_ && b.wpp == wpp_ && b.piece == piece_,
                 "ipc p2p: rank " + std::to_string(p) + " was configured differently");
      if (p == rank_) continue;
      void* m = nullptr;
      void* f = nullptr;
      AKKA_P2P_HIP(hipIpcOpenMemHandle(&m, b.mbox, hipIpcMemLazyEnablePeerAccess));
      AKKA_P2P_HIP(hipIpcOpenMemHandle(&f, b.flags, hipIpcMemLazyEnablePeerAccess));
      peer_mbox_[size_t(p)] = static_cast<char*>(m);
      peer_flags_[size_t(p)] = static_cast<uint32_t*>(f);
    }
    ready_ = true;
  }

  void group(StreamH stream, const std::vector<P2POp>& ops) override {
    AKKA_CHECK(ready_, "ipc p2p: open() the peer mailboxes first");
    IpcP2PPlan plan = plan_ipc_p2p_group(ops, n_, piece_, kChannels, host_ + 1, send_seq_, recv_seq_);
    if (plan.ops.empty()) return;
    IpcP2PArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int32_t p = 0; p < n_; ++p) {
      a.mbox[p] = peer_mbox_[size_t(p)];
      a.flags[p] = peer_flags_[size_t(p)];
    }
    a.err = host_dev_;
    a.dead = host_dev_ + 1;
    a.piece = piece_;
    a.nslots = nslots_;
    a.wpp = wpp_;
    a.nch = kChannels;
    a.N = n_;
    a.me = rank_;
    a.timeout = timeout_;
    a.nops = int32_t(plan.ops.size());
    a.nqueues = int32_t(plan.qstart.size()) - 1;
    a.wpg = std::clamp(grid_cap_ / std::max(1, a.nqueues), 1, wpp_);
    std::copy(plan.ops.begin(), plan.ops.end(), a.ops);
    for (size_t i = 0; i < plan.qstart.size(); ++i) a.qstart[i] = int16_t(plan.qstart[i]);
    launch_ipc_p2p_group(static_cast<hipStream_t>(stream), a);
    AKKA_P2P_HIP(hipGetLastError());
    ++groups_;
    bytes_ += plan.bytes_sent;
  }

  void check() override {
    if (__atomic_load_n(host_, __ATOMIC_ACQUIRE) != 0)
      throw AkkaError("akka ipc p2p: a transfer timed out or its peer was aborted (AKKA_IPC_TIMEOUT_MS)");
  }
  bool abort_peer(int32_t peer) override {
    if (peer < 0 || peer >= n_ || peer == rank_) return false;
    __atomic_store_n(host_ + 1 + peer, 1u, __ATOMIC_RELEASE);
    return true;
  }

 private:
  int32_t rank_, n_, device_;
  int64_t piece_ = 0;
  int32_t nslots_ = 4, wpp_ = 32, grid_cap_ = 1024;
  size_t mbox_bytes_ = 0, flag_bytes_ = 0;
  char* mbox_ = nullptr;
  std::string mem_kind_;
  uint32_t* flags_ = nullptr;
  uint32_t* host_ = nullptr;      // [0] error, [1 + p] peer p aborted
  uint32_t* host_dev_ = nullptr;  // the same, as the device sees it
  uint64_t timeout_ = 0;
  bool ready_ = false;
  std::vector<char*> peer_mbox_;
  std::vector<uint32_t*> peer_flags_;
  std::vector<uint32_t> send_seq_, recv_seq_;  // [peer][channel] next piece sequence number
  int64_t groups_ = 0, bytes_ = 0;
};

}  // namespace

IpcP2PPlan plan_ipc_p2p_group(const std::vector<P2POp>& ops, int32_t nranks, int64_t piece, int32_t nch,
                              const uint32_t* dead, std::vector<uint32_t>& send_seq, std::vector<uint32_t>& recv_seq) {
  AKKA_CHECK(piece > 0 && nch > 0, "ipc p2p plan: bad piece / channel count");
  AKKA_CHECK(send_seq.size() == size_t(nranks) * size_t(nch) && recv_seq.size() == send_seq.size(),
             "ipc p2p plan: sequence tables do not match nranks x channels");
  // queues in order of first appearance; ops keep their issue order inside
  std::map<std::tuple<int, int, int>, size_t> qindex;
  std::vector<std::vector<const P2POp*>> queues;
  for (const P2POp& op : ops) {
    if (op.bytes == 0) continue;
    AKKA_CHECK(op.peer >= 0 && op.peer < nranks, "ipc p2p: peer out of range");
    if (dead && dead[op.peer]) continue;  // aborted peer: its transfers are dropped
    const int ch = std::min<int>(op.channel, nch - 1);
    auto key = std::make_tuple(op.send ? 1 : 0, op.peer, ch);
    auto it = qindex.find(key);
    if (it == qindex.end()) {
      it = qindex.emplace(key, queues.size()).first;
      queues.emplace_back();
    }
    queues[it->second].push_back(&op);
  }
  IpcP2PPlan plan;
  size_t nops = 0;
  for (const auto& q : queues) nops += q.size();
  AKKA_CHECK(nops <= size_t(kIpcP2PMaxOps), "ipc p2p: more than " + std::to_string(kIpcP2PMaxOps) + " ops in one group");
  for (const auto& q : queues) {
    plan.qstart.push_back(int32_t(plan.ops.size()));
    for (const P2POp* op : q) {
      const int ch = std::min<int>(op->channel, nch - 1);
      uint32_t& seq = (op->send ? send_seq : recv_seq)[size_t(op->peer) * size_t(nch) + size_t(ch)];
      IpcP2POp o;
      std::memset(&o, 0, sizeof(o));
      o.buf = static_cast<char*>(op->buf);
      o.bytes = int64_t(op->bytes);
      o.seq = seq;
      o.send = op->send ? 1 : 0;
      o.peer = int8_t(op->peer);
      o.ch = int8_t(ch);
      plan.ops.push_back(o);
      seq += uint32_t((int64_t(op->bytes) + piece - 1) / piece);
      if (op->send) plan.bytes_sent += int64_t(op->bytes);
    }
  }
  if (!plan.ops.empty()) plan.qstart.push_back(int32_t(plan.ops.size()));
  return plan;
}

std::unique_ptr<P2P> make_ipc_p2p(int32_t rank, int32_t nranks, int32_t device) {
  return std::make_unique<IpcP2P>(rank, nranks, device);
}

}  // namespace akka
