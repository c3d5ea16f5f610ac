#include "reactive_link.h"

#include <algorithm>
#include <chrono>
#include <cstring>

namespace akka {

ReactiveLink::ReactiveLink(Engine* engine, P2P* p2p, int32_t max_slots)
    : engine_(engine), p2p_(p2p), max_slots_(max_slots) {}

ReactiveLink::~ReactiveLink() {
  if (!dev_) return;
  // A lost peer's stream is left alone (never synchronized or destroyed):
  // whatever it still holds can only wait for a rank that is gone.
  try {
    for (size_t p = 0; p < streams_.size(); ++p)
      if (streams_[p] && !lost_[p]) dev_->sync_stream(streams_[p]);
  } catch (...) {
  }
  for (size_t p = 0; p < streams_.size(); ++p)
    if (streams_[p] && !lost_[p]) dev_->destroy_stream(streams_[p]);
  for (EventH e : events_) dev_->destroy_event(e);
  for (int32_t* p : pinned_) dev_->release_pinned(p);
  if (recv_dev_) dev_->release(recv_dev_);
}

void ReactiveLink::bind(DataPlane* dp) {
  AKKA_CHECK(!dp_, "reactive link already bound");
  dp_ = dp;
  dev_ = dp->device();
  const Geometry& g = dp->geometry();
  N_ = g.N;
  me_ = dp->me();
  L_ = dp->ring_rows();
  kme_ = g.num_chunks(me_);
  kmax_ = dp->kmax();
  AKKA_CHECK(N_ >= 2, "the reactive transport needs at least two workers");
  AKKA_CHECK(p2p_->nranks() == N_ && p2p_->rank() == me_, "p2p endpoint does not match the worker geometry");
  streams_.assign(size_t(N_), nullptr);
  lost_.assign(size_t(N_), 0);
  for (int32_t p = 0; p < N_; ++p)
    if (p != me_) streams_[size_t(p)] = dev_->create_stream();
  recv_dev_ = static_cast<int32_t*>(dev_->alloc(size_t(L_) * N_ * kmax_ * sizeof(int32_t)));
  dp->enable_staging(std::max(max_slots_, L_ + 1), [this](int32_t round) { return reclaim(round); });
}

ReactiveLink::RoundState& ReactiveLink::st(int32_t r) {
  auto it = rounds_.find(r);
  if (it != rounds_.end()) return it->second;
  RoundState& s = rounds_[r];
  s.wire.assign(size_t(std::max(kme_, 1)), 0);
  if (kme_ == 0) s.closable = true;  // empty block: nothing of mine to reduce
  return s;
}

EventH ReactiveLink::get_event() {
  if (!free_events_.empty()) {
    EventH e = free_events_.back();
    free_events_.pop_back();
    return e;
  }
  EventH e = dev_->create_event();
  events_.push_back(e);
  return e;
}
void ReactiveLink::put_event(EventH e) { free_events_.push_back(e); }

int32_t* ReactiveLink::get_pinned() {
  if (!free_pinned_.empty()) {
    int32_t* p = free_pinned_.back();
    free_pinned_.pop_back();
    return p;
  }
  int32_t* p = static_cast<int32_t*>(dev_->alloc_pinned(size_t(kmax_) * sizeof(int32_t)));
  pinned_.push_back(p);
  return p;
}

void ReactiveLink::send_reduce(int32_t /*dest*/, int32_t chunk, int32_t round, int32_t count, const Payload&) {
  // Called once per (chunk, remote peer); the data already sits in the landing
  // row (DataPlane staged mode) -- only record the chunk's count once.
  if (round < next_round_) return;  // P2 already out (cannot happen: no reduces after completion)
  RoundState& s = st(round);
  if (s.p2_issued) return;
  int32_t& w = s.wire[size_t(chunk)];
  if (w == 0) {
    w = count + 1;
    if (++s.reduced == kme_) s.closable = true;
  }
}

void ReactiveLink::on_scattered(int32_t round) { st(round).scattered = true; }

bool ReactiveLink::may_finalize(int32_t round) {
  // The round completed: P2 goes out with whatever is reduced by now.  (Its
  // send slot is released at the next pump, after finalize read it.)
  auto it = rounds_.find(round);
  if (it != rounds_.end()) {
    it->second.closable = true;
    it->second.completed = true;
  } else if (round >= next_round_) {
    RoundState& s = st(round);
    s.closable = true;
    s.completed = true;
  }
  return true;
}

void ReactiveLink::pump() {
  issue_ready();
  for (auto it = rounds_.begin(); it != rounds_.end() && it->first < next_round_;) {
    const int32_t r = it->first;
    ++it;
    retire(r);
  }
}

void ReactiveLink::issue_ready() {
  if (issuing_ || !dp_) return;
  issuing_ = true;
  try {
    for (;;) {
      auto it = rounds_.find(next_round_);
      if (it == rounds_.end()) break;
      if (!next_is_p2_) {
        if (!it->second.scattered) break;
        issue_p1(next_round_);
        next_is_p2_ = true;
      } else {
        if (!it->second.closable) break;
        issue_p2(next_round_);
        next_is_p2_ = false;
        ++next_round_;
      }
    }
  } catch (...) {
    issuing_ = false;
    throw;
  }
  issuing_ = false;
}

bool ReactiveLink::exchanges_with(int32_t p) const {
  if (p == me_ || lost_[size_t(p)]) return false;
  for (const auto& pe : engine_->peers())
    if (pe.id == p) return true;
  return false;
}

void ReactiveLink::on_peer_lost(int32_t id) {
  if (id < 0 || id >= N_ || id == me_ || lost_[size_t(id)]) return;
  lost_[size_t(id)] = 1;
  ++stats_.peers_lost;
  // End what is queued / in flight with the dead peer (RCCL: abort of the
  // pair communicator), then forget it: its arrivals are never delivered, so
  // its contributions count as missing (the thresholds decide), and nothing
  // -- slot reclaim included -- ever waits for its transfers again.
  p2p_->abort_peer(id);
  for (auto it = pending_.begin(); it != pending_.end();) {
    if (it->peer != id) {
      ++it;
      continue;
    }
    auto rs = rounds_.find(it->round);
    if (rs != rounds_.end()) --rs->second.open;
    // the event / pinned row may still be referenced by the dead stream: not recycled
    ++stats_.transfers_dropped;
    it = pending_.erase(it);
  }
  for (auto it = rounds_.begin(); it != rounds_.end() && it->first < next_round_;) {
    const int32_t r = it->first;
    ++it;
    retire(r);
  }
}

void ReactiveLink::issue_p1(int32_t r) {
  const Geometry& g = dp_->geometry();
  const size_t es = dp_->esize();
  const int64_t my_len = g.block_len(me_);
  // Covers the staging copy of r and every reduce that read ring row r%L for
  // an older round.
  EventH rel = dp_->row_release_event(r);
  RoundState& s = st(r);
  std::vector<P2POp> ops;
  for (int32_t i = 1; i < N_; ++i) {
    const int32_t p = (me_ + i) % N_;
    if (!exchanges_with(p)) continue;
    StreamH ps = streams_[size_t(p)];
    dev_->wait(ps, rel);
    ops.clear();
    const int64_t plen = g.block_len(p);
    if (plen > 0) ops.push_back({true, p, const_cast<void*>(dp_->staged_input(r, p)), size_t(plen) * es});
    if (my_len > 0) ops.push_back({false, p, dp_->scatter_slot(r, p, 0), size_t(my_len) * es});
    if (!ops.empty()) {
      p2p_->group(ps, ops);
      ++stats_.groups;
      if (plen > 0) stats_.bytes_sent += plen * int64_t(es);
    }
    Pending pd;
    pd.round = r;
    pd.peer = p;
    pd.phase = 1;
    pd.ev = get_event();
    dev_->record(pd.ev, ps);
    arm(ps);
    pending_.push_back(pd);
    ++s.open;
  }
}

void ReactiveLink::issue_p2(int32_t r) {
  const Geometry& g = dp_->geometry();
  const size_t es = dp_->esize();
  const int64_t my_len = g.block_len(me_);
  const size_t row = size_t(r % L_);
  RoundState& s = st(r);
  StreamH cs = dev_->compute_stream();
  int32_t* wdev = dp_->wire_dev(r);
  void* mine = dp_->mine_at(r, 0);
  if (kme_ > 0) {
    // The slot's pinned row is only rewritten after its previous round's
    // transfers (which follow this upload in stream order) finished.
    int32_t* wh = dp_->wire_host(r);
    std::memcpy(wh, s.wire.data(), size_t(kme_) * sizeof(int32_t));
    for (int32_t k = 0; k < kme_; ++k)
      if (s.wire[size_t(k)] == 0) ++stats_.unreduced_chunks;
    dev_->copy(cs, wdev, wh, size_t(kme_) * sizeof(int32_t), CopyKind::HostToDevice);
  }
  // Everything my block's sends read (reduces, wire counts) and everything
  // that read the landing row for round r-L (its finalize) is on the compute
  // stream before this point.
  EventH ready = get_event();
  dev_->record(ready, cs);
  std::vector<P2POp> ops;
  for (int32_t i = 1; i < N_; ++i) {
    const int32_t p = (me_ + i) % N_;
    if (!exchanges_with(p)) continue;
    StreamH ps = streams_[size_t(p)];
    dev_->wait(ps, ready);
    const int32_t kp = g.num_chunks(p);
    const int64_t plen = g.block_len(p);
    int32_t* rdev = recv_dev_ + (row * N_ + size_t(p)) * kmax_;
    ops.clear();
    if (my_len > 0) {
      ops.push_back({true, p, mine, size_t(my_len) * es});
      ops.push_back({true, p, wdev, size_t(kme_) * sizeof(int32_t)});
    }
    if (plen > 0) {
      ops.push_back({false, p, dp_->landing_at(r, p, 0), size_t(plen) * es});
      ops.push_back({false, p, rdev, size_t(kp) * sizeof(int32_t)});
    }
    if (!ops.empty()) {
      p2p_->group(ps, ops);
      ++stats_.groups;
      if (my_len > 0) stats_.bytes_sent += my_len * int64_t(es) + kme_ * int64_t(sizeof(int32_t));
    }
    Pending pd;
    pd.round = r;
    pd.peer = p;
    pd.phase = 2;
    if (kp > 0) {
      pd.counts = get_pinned();
      dev_->copy(ps, pd.counts, rdev, size_t(kp) * sizeof(int32_t), CopyKind::DeviceToHost);
    }
    pd.ev = get_event();
    dev_->record(pd.ev, ps);
    arm(ps);
    pending_.push_back(pd);
    ++s.open;
  }
  put_event(ready);  // the waits above captured its record
  s.p2_issued = true;
  p2p_->check();  // RCCL async errors on the pair communicators: once per round
}

bool ReactiveLink::reclaim(int32_t round) {
  // The data plane wants to reuse `round`'s send slot for a newer round: make
  // the compute stream (which writes the slot next) wait for the transfers
  // that still read it.  Everything issuable is issued first so those waits
  // exist; a round whose P2 cannot be issued yet is not reclaimable.
  issue_ready();
  if (round >= next_round_) return false;
  for (const Pending& pd : pending_) {
    if (pd.round == round) {
      dev_->wait(dev_->compute_stream(), pd.ev);
      ++stats_.reclaim_waits;
    }
  }
  rounds_.erase(round);  // its arrivals are outdated; nothing else to release
  return true;
}

void ReactiveLink::retire(int32_t r) {
  auto it = rounds_.find(r);
  if (it == rounds_.end() || !it->second.p2_issued || it->second.open > 0 || !it->second.completed) return;
  rounds_.erase(it);
  dp_->release_slot(r);
}

void ReactiveLink::arm(StreamH s) {
  if (!notify_ok_ || dev_->is_host()) return;
  std::shared_ptr<Notifier> n = notifier_;  // outlives the link if a callback fires late
  notify_ok_ = dev_->host_notify(s, [n]() {
    {
      std::lock_guard<std::mutex> lk(n->mu);
      ++n->count;
    }
    n->cv.notify_all();
  });
}

void ReactiveLink::wait_activity(int64_t timeout_us) {
  if (!notify_ok_ || !dev_ || dev_->is_host() || pending_.empty()) return;
  std::unique_lock<std::mutex> lk(notifier_->mu);
  notifier_->cv.wait_for(lk, std::chrono::microseconds(timeout_us), [&] { return notifier_->count != seen_; });
  seen_ = notifier_->count;
}

bool ReactiveLink::poll() {
  if (!dp_) return false;
  ++stats_.polls;
  std::vector<Pending> done;
  for (auto it = pending_.begin(); it != pending_.end();) {
    if (dev_->query(it->ev)) {
      done.push_back(*it);
      it = pending_.erase(it);
    } else {
      ++it;
    }
  }
  if (done.empty()) return false;
  const Geometry& g = dp_->geometry();
  for (const Pending& pd : done) {
    put_event(pd.ev);
    {
      auto rs = rounds_.find(pd.round);
      if (rs != rounds_.end()) --rs->second.open;
    }
    if (pd.phase == 1) {
      ++stats_.p1_arrivals;
      for (int32_t k = 0; k < kme_; ++k) {
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(me_, k);
        p.on_host = dev_->is_host();
        engine_->on_scatter(pd.peer, me_, k, pd.round, p);
      }
    } else {
      ++stats_.p2_arrivals;
      const int32_t kp = g.num_chunks(pd.peer);
      std::vector<int32_t> counts(pd.counts, pd.counts + kp);
      if (pd.counts) free_pinned_.push_back(pd.counts);
      for (int32_t k = 0; k < kp; ++k) {
        const int32_t w = counts[size_t(k)];
        if (w <= 0) continue;  // the owner never reduced this chunk
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(pd.peer, k);
        p.on_host = dev_->is_host();
        if (w == 1 && pd.round >= engine_->round()) {
          // Reduced from zero contributions: reads as zeros (a forced reduce of
          // a round whose landing row may already have been reused).
          dev_->zero(dev_->compute_stream(), dp_->landing_at(pd.round, pd.peer, k), size_t(p.len) * dp_->esize());
        }
        engine_->on_reduce(pd.peer, me_, k, pd.round, w - 1, p);
      }
    }
    if (pd.round < next_round_) retire(pd.round);
  }
  return true;
}

}  // namespace akka
