#include "reactive_link.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

namespace akka {

namespace {
constexpr int32_t kPhase1 = 0;  // pair channel of phase 1 (scatter)
constexpr int32_t kPhase2 = 1;  // pair channel of phase 2 (reduced chunks + counts)
constexpr int32_t kCountRows = 64;  // pinned count rows allocated at a time
}  // namespace

ReactiveLink::ReactiveLink(Engine* engine, P2P* p2p, int32_t max_slots)
    : engine_(engine), p2p_(p2p), max_slots_(max_slots) {}

ReactiveLink::~ReactiveLink() {
  if (!dev_) return;
  // A lost peer's streams are left alone (never synchronized or destroyed):
  // whatever they still hold can only wait for a rank that is gone.
  try {
    for (size_t p = 0; p < s1_.size(); ++p) {
      if (lost_[p]) continue;
      if (s1_[p]) dev_->sync_stream(s1_[p]);
      if (s2_[p] && s2_[p] != s1_[p]) dev_->sync_stream(s2_[p]);
    }
  } catch (...) {
  }
  for (size_t p = 0; p < s1_.size(); ++p) {
    if (lost_[p]) continue;
    if (s1_[p]) dev_->destroy_stream(s1_[p]);
    if (s2_[p] && s2_[p] != s1_[p]) dev_->destroy_stream(s2_[p]);
  }
  for (EventH e : events_) dev_->destroy_event(e);
  for (int32_t* p : pinned_blocks_) dev_->release_pinned(p);
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
  s1_.assign(size_t(N_), nullptr);
  s2_.assign(size_t(N_), nullptr);
  lost_.assign(size_t(N_), 0);
  // One stream per peer for both phases: a second stream per peer doubles the
  // hardware queues a process needs, and past ~16 mapped queues per device
  // the scheduler time-slices them (measured on the 3-rank loopback: ~1.5 ms
  // per parked group).  Phase-2 chunks therefore run behind the pair's
  // phase-1 chunks of the same round in stream order (they are still issued,
  // reduced and delivered per chunk); the two phases keep separate matching
  // channels.
  for (int32_t p = 0; p < N_; ++p)
    if (p != me_) s1_[size_t(p)] = s2_[size_t(p)] = dev_->create_stream();
  // Transfer groups: gm_ consecutive chunks per exchange, so that a group
  // carries at least AKKA_REACTIVE_GROUP_BYTES (default 16 MiB) -- every chunk
  // is still received, reduced and delivered to the engine on its own; only
  // the number of p2p groups (host enqueue + arrival polling per group) drops
  // for small maxChunkSize.  A function of the geometry: identical on every rank.
  int64_t min_bytes = int64_t(16) << 20;
  if (const char* v = std::getenv("AKKA_REACTIVE_GROUP_BYTES")) min_bytes = std::max<int64_t>(0, std::atoll(v));
  const int64_t cbytes = std::max<int64_t>(1, g.C * int64_t(dp->esize()));
  gm_ = int32_t(std::clamp<int64_t>((min_bytes + cbytes - 1) / cbytes, 1, std::max(kmax_, 1)));
  recv_dev_ = static_cast<int32_t*>(dev_->alloc(size_t(L_) * N_ * kmax_ * sizeof(int32_t)));
  dp->enable_staging(std::max(max_slots_, L_ + 1), [this](int32_t round) { return reclaim(round); });
}

ReactiveLink::RoundState& ReactiveLink::st(int32_t r) {
  auto it = rounds_.find(r);
  if (it != rounds_.end()) return it->second;
  RoundState& s = rounds_[r];
  s.wire.assign(size_t(std::max(kme_, 1)), 0);
  s.ready.assign(size_t(std::max(kme_, 1)), nullptr);
  return s;
}

int64_t ReactiveLink::span_len(int32_t block, int32_t k0, int32_t k1) const {
  // elements of chunks [k0, k1) of `block` (consecutive chunks are contiguous)
  const Geometry& g = dp_->geometry();
  if (k1 <= k0) return 0;
  return g.chunk_start(block, k1 - 1) + g.chunk_len(block, k1 - 1) - g.chunk_start(block, k0);
}

int32_t ReactiveLink::chunks_with(int32_t p) const {
  return std::max(kme_, dp_->geometry().num_chunks(p));
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

int32_t* ReactiveLink::get_count_slot() {
  // a pinned row of gm_ counts (one per chunk of a transfer group)
  if (free_counts_.empty()) {
    int32_t* b = static_cast<int32_t*>(dev_->alloc_pinned(size_t(kCountRows) * size_t(gm_) * sizeof(int32_t)));
    pinned_blocks_.push_back(b);
    for (int32_t i = kCountRows - 1; i >= 0; --i) free_counts_.push_back(b + size_t(i) * size_t(gm_));
  }
  int32_t* p = free_counts_.back();
  free_counts_.pop_back();
  return p;
}

void ReactiveLink::send_reduce(int32_t /*dest*/, int32_t chunk, int32_t round, int32_t count, const Payload&) {
  // Called once per (chunk, remote peer) right after the engine reduced the
  // chunk into the round's send slot: record its count once -- written into
  // the slot's device count row by a 4-byte fill that merges into the reduce
  // launch -- and the point the chunk's P2 groups wait for.
  if (round < p2_round_) return;  // P2 of the round already out (cannot happen: no reduces after completion)
  RoundState& s = st(round);
  if (chunk < s.p2_next || s.wire[size_t(chunk)] != 0) return;
  s.wire[size_t(chunk)] = count + 1;
  StreamH cs = dev_->compute_stream();
  dev_->fill_i32(cs, dp_->wire_dev(round) + chunk, count + 1, 1);
  s.ready[size_t(chunk)] = get_event();
  dev_->record(s.ready[size_t(chunk)], cs);
}

void ReactiveLink::on_scattered(int32_t round) { st(round).scattered = true; }

bool ReactiveLink::may_finalize(int32_t round) {
  // The round completed: its remaining P2 chunks go out with whatever is
  // reduced by now (count 0 for the rest).  Its send slot is released once
  // every transfer of the round finished.
  if (round >= p2_round_ || rounds_.count(round)) st(round).completed = true;
  return true;
}

void ReactiveLink::pump() {
  issue_ready();
  for (auto it = rounds_.begin(); it != rounds_.end() && it->first < p2_round_;) {
    const int32_t r = it->first;
    ++it;
    retire(r);
  }
}

void ReactiveLink::issue_ready() {
  if (issuing_ || !dp_) return;
  issuing_ = true;
  try {
    // Per pair stream: P1(r) chunks, then P2(r) chunks as they get ready,
    // then P1(r+1) ...  -- one total order both sides of every pair share,
    // so the pair's stream never waits on a group its peer queued later.
    for (;;) {
      if (p1_round_ == p2_round_) {
        auto it = rounds_.find(p1_round_);
        if (it == rounds_.end() || !it->second.scattered) break;
        issue_p1(p1_round_);
        ++p1_round_;
      }
      if (!rounds_.count(p2_round_)) break;
      if (!issue_p2(p2_round_)) break;
      ++p2_round_;
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
  // pair communicators), then forget it: its arrivals are never delivered, so
  // its contributions count as missing (the thresholds decide), and nothing
  // -- slot reclaim included -- ever waits for its transfers again.
  p2p_->abort_peer(id);
  for (auto it = pending_.begin(); it != pending_.end();) {
    if (it->peer != id) {
      ++it;
      continue;
    }
    auto rs = rounds_.find(it->round);
    if (rs != rounds_.end()) {
      --rs->second.open;
      if (it->phase == 1) --rs->second.p1_open;
    }
    // the event / pinned count may still be referenced by the dead stream: not recycled
    ++stats_.transfers_dropped;
    it = pending_.erase(it);
  }
  for (auto it = rounds_.begin(); it != rounds_.end() && it->first < p2_round_;) {
    const int32_t r = it->first;
    ++it;
    retire(r);
  }
}

void ReactiveLink::issue_p1(int32_t r) {
  const Geometry& g = dp_->geometry();
  const size_t es = dp_->esize();
  // Covers the staging copy of r and every reduce that read ring row r%L for
  // an older round.
  EventH rel = dp_->row_release_event(r);
  RoundState& s = st(r);
  std::vector<P2POp> ops;
  for (int32_t i = 1; i < N_; ++i) {
    const int32_t p = (me_ + i) % N_;
    if (!exchanges_with(p)) continue;
    StreamH ps = s1_[size_t(p)];
    dev_->wait(ps, rel);
    const int32_t kp = g.num_chunks(p);
    const char* in = static_cast<const char*>(dp_->staged_input(r, p));
    const int32_t kall = chunks_with(p);
    for (int32_t k0 = 0; k0 < kall; k0 += gm_) {
      const int32_t k1 = std::min(k0 + gm_, kall);
      ops.clear();
      if (k0 < kp) {  // chunks [k0, min(k1, kp)) of block p: contiguous in the staged input
        const int64_t len = span_len(p, k0, std::min(k1, kp));
        ops.push_back({true, p, const_cast<char*>(in) + size_t(g.chunk_start(p, k0)) * es, size_t(len) * es, kPhase1});
        stats_.bytes_sent += len * int64_t(es);
      }
      if (k0 < kme_)  // p's chunks [k0, min(k1, kme)) of my block: contiguous in its ring slot
        ops.push_back({false, p, dp_->scatter_slot(r, p, k0), size_t(span_len(me_, k0, std::min(k1, kme_))) * es,
                       kPhase1});
      p2p_->group(ps, ops);
      ++stats_.groups;
      Pending pd;
      pd.round = r;
      pd.peer = p;
      pd.phase = 1;
      pd.chunk = k0;
      pd.chunk_end = k1;
      pd.ev = get_event();
      dev_->record(pd.ev, ps);
      // one host notification per pair and round (the last group): a host
      // callback blocks its stream until it ran, and many per round
      // serialise on the runtime's callback thread; earlier groups are
      // picked up by the waiter's periodic poll
      if (k1 == kall) arm(ps);
      pending_.push_back(pd);
      ++s.open;
      ++s.p1_open;
    }
  }
  s.p1_issued = true;
}

bool ReactiveLink::issue_p2(int32_t r) {
  RoundState& s = st(r);
  if (s.p2_done) return true;
  // The landing row r%L was last read by round r-L's finalize (compute
  // stream): that round must have completed (it has, whenever one of my
  // chunks of r was reduced; with an empty block of my own this is the check).
  if (r - L_ >= 0 && !engine_->is_completed(r - L_)) return false;
  const Geometry& g = dp_->geometry();
  const size_t es = dp_->esize();
  StreamH cs = dev_->compute_stream();
  const size_t row = size_t(r % L_);
  if (s.p2_next == 0) {
    // receive-only groups (chunks past the end of my block) wait on this
    EventH landing = get_event();
    dev_->record(landing, cs);
    for (int32_t i = 1; i < N_; ++i) {
      const int32_t p = (me_ + i) % N_;
      if (exchanges_with(p)) dev_->wait(s2_[size_t(p)], landing);
    }
    put_event(landing);
  }
  std::vector<P2POp> ops;
  while (s.p2_next < kmax_) {
    const int32_t k0 = s.p2_next;
    const int32_t k1 = std::min(k0 + gm_, kmax_);
    // the group goes out once every chunk of mine in it is reduced (or the
    // round completed: the rest then carry count 0) -- fixed group bounds,
    // so both sides of a pair build the same groups
    const int32_t m1 = std::min(k1, kme_);
    bool ready = true;
    for (int32_t k = k0; k < m1 && ready; ++k) ready = s.wire[size_t(k)] != 0 || s.completed;
    if (!ready) break;
    EventH rdy = nullptr;
    if (k0 < kme_) {
      for (int32_t k = k0; k < m1; ++k)
        if (s.wire[size_t(k)] == 0) {  // round completed before this chunk reached its threshold
          dev_->fill_i32(cs, dp_->wire_dev(r) + k, 0, 1);
          ++stats_.unreduced_chunks;
        }
      // everything the group's sends read (reduces, count fills) is on the
      // compute stream before this point
      rdy = get_event();
      dev_->record(rdy, cs);
    }
    bool issued = false;
    for (int32_t i = 1; i < N_; ++i) {
      const int32_t p = (me_ + i) % N_;
      if (!exchanges_with(p) || k0 >= chunks_with(p)) continue;
      StreamH ps = s2_[size_t(p)];
      const int32_t kp = g.num_chunks(p);
      int32_t* rdev = recv_dev_ + (row * size_t(N_) + size_t(p)) * size_t(kmax_);
      ops.clear();
      if (k0 < kme_) {
        dev_->wait(ps, rdy);
        const int64_t len = span_len(me_, k0, m1);
        ops.push_back({true, p, dp_->mine_at(r, k0), size_t(len) * es, kPhase2});
        ops.push_back({true, p, dp_->wire_dev(r) + k0, size_t(m1 - k0) * sizeof(int32_t), kPhase2});
        stats_.bytes_sent += len * int64_t(es) + int64_t(m1 - k0) * int64_t(sizeof(int32_t));
      }
      const int32_t p1 = std::min(k1, kp);
      if (k0 < kp) {
        ops.push_back({false, p, dp_->landing_at(r, p, k0), size_t(span_len(p, k0, p1)) * es, kPhase2});
        ops.push_back({false, p, rdev + k0, size_t(p1 - k0) * sizeof(int32_t), kPhase2});
      }
      p2p_->group(ps, ops);
      ++stats_.groups;
      Pending pd;
      pd.round = r;
      pd.peer = p;
      pd.phase = 2;
      pd.chunk = k0;
      pd.chunk_end = k1;
      if (k0 < kp) {
        pd.count = get_count_slot();
        dev_->copy(ps, pd.count, rdev + k0, size_t(p1 - k0) * sizeof(int32_t), CopyKind::DeviceToHost);
      }
      pd.ev = get_event();
      dev_->record(pd.ev, ps);
      if (k1 >= chunks_with(p)) arm(ps);  // see issue_p1
      pending_.push_back(pd);
      ++s.open;
      issued = true;
    }
    if (issued && s.p1_open > 0) ++stats_.p2_overlapped;
    if (rdy) put_event(rdy);  // the waits above captured its record
    for (int32_t k = k0; k < m1; ++k)
      if (s.ready[size_t(k)]) {
        put_event(s.ready[size_t(k)]);
        s.ready[size_t(k)] = nullptr;
      }
    s.p2_next = k1;
  }
  if (s.p2_next < kmax_) return false;
  s.p2_done = true;
  p2p_->check();  // RCCL async errors on the pair communicators: once per round
  return true;
}

bool ReactiveLink::reclaim(int32_t round) {
  // The data plane wants to reuse `round`'s send slot for a newer round: make
  // the compute stream (which writes the slot next) wait for the transfers
  // that still read it.  Everything issuable is issued first so those waits
  // exist; a round whose P2 is not fully issued yet is not reclaimable.
  issue_ready();
  if (round >= p2_round_ || round >= p1_round_) return false;
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
  if (it == rounds_.end()) return;
  const RoundState& s = it->second;
  if (!s.p2_done || !s.p1_issued || s.open > 0 || !s.completed) return;
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
      if (rs != rounds_.end()) {
        --rs->second.open;
        if (pd.phase == 1) --rs->second.p1_open;
      }
    }
    if (pd.phase == 1) {
      for (int32_t k = pd.chunk; k < std::min(pd.chunk_end, kme_); ++k) {
        ++stats_.p1_arrivals;
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(me_, k);
        p.on_host = dev_->is_host();
        engine_->on_scatter(pd.peer, me_, k, pd.round, p);
      }
    } else if (pd.count) {
      const int32_t kp = g.num_chunks(pd.peer);
      std::vector<int32_t> w(pd.count, pd.count + (std::min(pd.chunk_end, kp) - pd.chunk));
      free_counts_.push_back(pd.count);
      for (int32_t k = pd.chunk; k < std::min(pd.chunk_end, kp); ++k) {
        ++stats_.p2_arrivals;
        const int32_t wk = w[size_t(k - pd.chunk)];
        if (wk <= 0) continue;  // 0: the owner never reduced this chunk
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(pd.peer, k);
        p.on_host = dev_->is_host();
        if (wk == 1 && pd.round >= engine_->round()) {
          // Reduced from zero contributions: reads as zeros (a forced reduce of
          // a round whose landing row may already have been reused).
          dev_->zero(dev_->compute_stream(), dp_->landing_at(pd.round, pd.peer, k), size_t(p.len) * dp_->esize());
        }
        engine_->on_reduce(pd.peer, me_, k, pd.round, wk - 1, p);
      }
    }
    if (pd.round < p2_round_) retire(pd.round);
  }
  return true;
}

}  // namespace akka
