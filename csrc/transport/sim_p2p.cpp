// CPU simulator of RCCL grouped p2p semantics (rendezvous, per-pair in-order
// matching, whole-group completion) over deferred host devices.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <tuple>
#include <sstream>

#include "p2p.h"

namespace akka {

bool host_device_step(Device* d, uint32_t rotate);
bool host_device_idle(Device* d);

struct SimSend {
  const void* buf;
  size_t bytes;
  bool consumed = false;
};

// One simulated RCCL collective (reduce-scatter / all-gather) across the ranks.
struct SimColl {
  std::vector<const void*> send;
  std::vector<void*> recv;
  int32_t deposited = 0, computed = 0, released = 0;
};

class SimHub {
 public:
  explicit SimHub(int32_t n, bool collectives = false)
      : n_(n), collectives(collectives), coll_seq(size_t(n), 0) {}
  int32_t n_;
  // native collectives (like an RCCL communicator spanning every rank):
  // opt-in, so the exact-round collective lane can be simulated too
  bool collectives;
  std::vector<int64_t> coll_seq;  // per rank: collectives issued so far (same order on every rank)
  std::map<int64_t, std::shared_ptr<SimColl>> colls;
  // fifo[src, dst, channel]: sends posted by src to dst not yet consumed, in order.
  std::map<std::tuple<int32_t, int32_t, int32_t>, std::deque<std::shared_ptr<SimSend>>> fifo;
  // (me, peer): `me` aborted its transfers with `peer` (abort_peer).
  std::set<std::pair<int32_t, int32_t>> aborted;
  int64_t bytes = 0;
  int64_t groups = 0;
  int64_t events = 0;  // posts + matches: progress that completes no queue op yet
};

std::shared_ptr<SimHub> make_sim_hub(int32_t nranks, bool collectives) {
  return std::make_shared<SimHub>(nranks, collectives);
}
int64_t sim_bytes_moved(const std::shared_ptr<SimHub>& hub) { return hub->bytes; }
int64_t sim_events(const std::shared_ptr<SimHub>& hub) { return hub->events; }

namespace {

float sim_bf16_to_f32(uint16_t v) {
  uint32_t u = uint32_t(v) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
uint16_t sim_f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return uint16_t((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return uint16_t(u >> 16);
}

class SimP2P final : public P2P {
 public:
  SimP2P(std::shared_ptr<SimHub> hub, int32_t rank, Device* dev) : hub_(std::move(hub)), rank_(rank), dev_(dev) {}
  int32_t rank() const override { return rank_; }
  int32_t nranks() const override { return hub_->n_; }
  const char* name() const override { return "sim"; }
  bool abort_peer(int32_t peer) override {
    // like ncclCommAbort of the pair communicator: queued and future ops
    // with `peer` complete at once without moving data
    hub_->aborted.insert({rank_, peer});
    hub_->events++;
    return true;
  }

  bool has_collectives() const override { return hub_->collectives; }

  // ncclReduceScatter: recv[0:count) = sum over ranks (ascending) of send[me*count ..].
  void reduce_scatter(StreamH s, const void* send, void* recv, size_t count, DType dt) override {
    const size_t es = dtype_size(dt);
    dev_->declare_access(s, {{send, size_t(hub_->n_) * count * es, false, "rccl.reduce_scatter.send"},
                             {recv, count * es, true, "rccl.reduce_scatter.recv"}});
    collective(s, send, recv, [count, dt, es](const SimColl& c, int32_t me, int32_t n) {
      std::vector<float> acc(count, 0.f);
      for (int32_t k = 0; k < n; ++k) {
        const char* src = static_cast<const char*>(c.send[size_t(k)]) + size_t(me) * count * es;
        for (size_t i = 0; i < count; ++i) {
          if (dt == DType::F32) {
            float v;
            std::memcpy(&v, src + i * 4, 4);
            acc[i] += v;
          } else {
            uint16_t h;
            std::memcpy(&h, src + i * 2, 2);
            acc[i] += sim_bf16_to_f32(h);
          }
        }
      }
      char* dst = static_cast<char*>(c.recv[size_t(me)]);
      for (size_t i = 0; i < count; ++i) {
        if (dt == DType::F32) std::memcpy(dst + i * 4, &acc[i], 4);
        else {
          const uint16_t h = sim_f32_to_bf16(acc[i]);
          std::memcpy(dst + i * 2, &h, 2);
        }
      }
    });
  }
  // ncclAllGather: recv[k*count ..] = rank k's send[0:count) (send may sit inside recv).
  void all_gather(StreamH s, const void* send, void* recv, size_t count, DType dt) override {
    const size_t es = dtype_size(dt);
    dev_->declare_access(s, {{send, count * es, false, "rccl.all_gather.send"},
                             {recv, size_t(hub_->n_) * count * es, true, "rccl.all_gather.recv"}});
    collective(s, send, recv, [count, es](const SimColl& c, int32_t me, int32_t n) {
      char* dst = static_cast<char*>(c.recv[size_t(me)]);
      for (int32_t k = 0; k < n; ++k)
        std::memmove(dst + size_t(k) * count * es, c.send[size_t(k)], count * es);
    });
  }

  void group(StreamH s, const std::vector<P2POp>& ops) override {
    std::vector<Access> acc;
    for (const auto& op : ops) {
      AKKA_CHECK(op.peer >= 0 && op.peer < hub_->n_ && op.peer != rank_, "sim p2p: bad peer");
      acc.push_back({op.buf, op.bytes, !op.send, op.send ? "p2p.send" : "p2p.recv"});
    }
    dev_->declare_access(s, acc);
    struct State {
      bool posted = false;
      std::vector<std::shared_ptr<SimSend>> sends;
      std::vector<bool> recv_done;
    };
    auto st = std::make_shared<State>();
    auto hub = hub_;
    const int32_t me = rank_;
    dev_->enqueue_host_op(s, [st, hub, me, ops]() {
      if (!st->posted) {
        for (const auto& op : ops) {
          if (!op.send) continue;
          auto snd = std::make_shared<SimSend>(SimSend{op.buf, op.bytes});
          hub->fifo[{me, op.peer, op.channel}].push_back(snd);
          st->sends.push_back(snd);
        }
        st->recv_done.assign(ops.size(), false);
        st->posted = true;
        if (std::getenv("AKKA_SIM_TRACE")) {
          std::fprintf(stderr, "[sim] rank %d posts group %lld:", me, (long long)hub->groups);
          for (const auto& op : ops) std::fprintf(stderr, " %s%d:%zu", op.send ? "S" : "R", op.peer, op.bytes);
          std::fprintf(stderr, "\n");
        }
        hub->groups++;
        hub->events++;
      }
      // Receives match the oldest unconsumed send of their pair, in op order.
      bool all = true;
      for (size_t i = 0; i < ops.size(); ++i) {
        const auto& op = ops[i];
        if (op.send || st->recv_done[i]) continue;
        if (hub->aborted.count({me, op.peer})) {
          st->recv_done[i] = true;
          continue;
        }
        // Earlier recvs from the same peer in this group must match first.
        bool blocked = false;
        for (size_t j = 0; j < i; ++j)
          if (!ops[j].send && ops[j].peer == op.peer && ops[j].channel == op.channel && !st->recv_done[j])
            blocked = true;
        if (blocked) {
          all = false;
          continue;
        }
        auto& q = hub->fifo[{op.peer, me, op.channel}];
        if (q.empty()) {
          all = false;
          continue;
        }
        auto snd = q.front();
        if (snd->bytes != op.bytes) {
          std::ostringstream os;
          os << "sim p2p: size mismatch " << op.peer << "->" << me << " send " << snd->bytes << " B vs recv "
             << op.bytes << " B";
          throw AkkaError(os.str());
        }
        if (op.bytes) std::memcpy(op.buf, snd->buf, op.bytes);
        hub->bytes += int64_t(op.bytes);
        snd->consumed = true;
        q.pop_front();
        st->recv_done[i] = true;
        hub->events++;
      }
      size_t si = 0;
      for (const auto& op : ops) {
        if (!op.send) continue;
        const auto& snd = st->sends[si++];
        if (!snd->consumed && !hub->aborted.count({me, op.peer})) all = false;
      }
      return all;
    });
  }

 private:
  // Every rank deposits its buffers; once all did, each computes its own
  // result (reading the others' send buffers); a rank's op completes only
  // when every rank computed, so no send buffer is reused while read.
  template <typename F>
  void collective(StreamH s, const void* send, void* recv, F compute) {
    AKKA_CHECK(hub_->collectives, "sim p2p: native collectives are off for this hub");
    const int64_t seq = hub_->coll_seq[size_t(rank_)]++;
    struct St {
      int phase = 0;
      std::shared_ptr<SimColl> c;
    };
    auto st = std::make_shared<St>();
    auto hub = hub_;
    const int32_t me = rank_, n = hub_->n_;
    dev_->enqueue_host_op(s, [st, hub, me, n, seq, send, recv, compute]() {
      if (st->phase == 0) {
        auto& c = hub->colls[seq];
        if (!c) {
          c = std::make_shared<SimColl>();
          c->send.assign(size_t(n), nullptr);
          c->recv.assign(size_t(n), nullptr);
        }
        st->c = c;
        c->send[size_t(me)] = send;
        c->recv[size_t(me)] = recv;
        ++c->deposited;
        st->phase = 1;
        hub->events++;
      }
      if (st->phase == 1) {
        if (st->c->deposited < n) return false;
        compute(*st->c, me, n);
        ++st->c->computed;
        st->phase = 2;
        hub->events++;
      }
      if (st->c->computed < n) return false;
      if (++st->c->released == n) hub->colls.erase(seq);
      hub->events++;
      return true;
    });
  }

  std::shared_ptr<SimHub> hub_;
  int32_t rank_;
  Device* dev_;
};

}  // namespace

std::unique_ptr<P2P> make_sim_p2p(std::shared_ptr<SimHub> hub, int32_t rank, Device* dev) {
  AKKA_CHECK(dev->is_host(), "sim p2p needs a deferred host device");
  return std::make_unique<SimP2P>(std::move(hub), rank, dev);
}

bool sim_step(const std::shared_ptr<SimHub>& hub, const std::vector<Device*>& devices, uint32_t rotate) {
  const int64_t ev0 = hub->events;
  bool progress = false;
  for (Device* d : devices) progress |= host_device_step(d, rotate);
  return progress || hub->events != ev0;
}

void sim_run(const std::shared_ptr<SimHub>& hub, const std::vector<Device*>& devices, int64_t max_iters) {
  for (int64_t it = 0; it < max_iters; ++it) {
    bool progress = false, idle = true;
    const int64_t ev0 = hub->events;
    for (Device* d : devices) {
      progress |= host_device_step(d, uint32_t(it));
      idle &= host_device_idle(d);
    }
    if (idle) return;
    progress |= hub->events != ev0;
    if (!progress) {
      std::ostringstream os;
      os << "sim p2p: deadlock - no rank can progress; pending sends per pair:";
      for (auto& kv : hub->fifo)
        if (!kv.second.empty())
          os << " " << std::get<0>(kv.first) << "->" << std::get<1>(kv.first) << "/c" << std::get<2>(kv.first) << ":"
             << kv.second.size();
      for (size_t i = 0; i < devices.size(); ++i)
        if (!host_device_idle(devices[i])) os << " [rank " << i << " blocked]";
      throw AkkaError(os.str());
    }
  }
  throw AkkaError("sim p2p: iteration limit reached");
}

}  // namespace akka
