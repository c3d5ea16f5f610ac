#include "engine.h"

#include <algorithm>
#include <exception>

namespace akka {

class Engine::Scope {
 public:
  explicit Scope(Engine* e) : e_(e), uncaught_(std::uncaught_exceptions()) { ++e_->depth_; }
  ~Scope() noexcept(false) {
    if (--e_->depth_ == 0 && std::uncaught_exceptions() == uncaught_) e_->leave_scope();
  }

 private:
  Engine* e_;
  int uncaught_;
};

Engine::Engine(EngineHost* host, Link* link) : host_(host), link_(link) {}
Engine::~Engine() = default;

bool Engine::init(const InitParams& p, const std::vector<PeerEntry>& peers) {
  if (id_ != -1) {
    // Re-init only replaces the peer map (W:87-89).
    peers_ = peers;
    std::sort(peers_.begin(), peers_.end(), [](const PeerEntry& a, const PeerEntry& b) { return a.id < b.id; });
    return false;
  }
  AKKA_CHECK(p.worker_num >= 1, "workerNum must be >= 1");
  AKKA_CHECK(p.id >= 0 && p.id < p.worker_num, "destId out of range");
  AKKA_CHECK(p.max_lag >= 0, "maxLag must be >= 0");
  params_ = p;
  id_ = p.id;
  N_ = p.worker_num;
  peers_ = peers;
  std::sort(peers_.begin(), peers_.end(), [](const PeerEntry& a, const PeerEntry& b) { return a.id < b.id; });
  g_ = Geometry(p.data_size, p.worker_num, p.max_chunk_size);
  L_ = p.max_lag + 1;  // ring of maxLag+1 rows (W:64, W:74)
  kme_ = g_.num_chunks(id_);
  kmax_ = std::max(1, g_.max_block_len_chunks());
  // Cut-offs computed like the reference (float32 product, truncated), then
  // clamped into [1, total]: a zero cut-off never fires under the reference's
  // `==` test, which is a stall, not a feature.
  min_scatter_ = std::clamp(float_threshold(p.th_reduce, N_), 1, N_);
  int64_t total = g_.total_chunks();
  min_reduced_ = int32_t(std::clamp<int64_t>(float_threshold(p.th_complete, total), 1, std::max<int64_t>(total, 1)));
  round_ = 0;
  max_round_ = -1;
  max_scattered_ = -1;
  completed_.clear();
  rows_.assign(size_t(L_), Row{});
  return true;
}

void Engine::attach(DataPlane* dp) {
  AKKA_CHECK(id_ >= 0, "attach before init");
  AKKA_CHECK(dp->geometry().S == g_.S && dp->geometry().N == g_.N && dp->geometry().C == g_.C,
             "data plane geometry does not match InitWorkers");
  AKKA_CHECK(dp->ring_rows() == L_, "data plane ring depth must be maxLag+1");
  dp_ = dp;
  // Replay messages that arrived before initialisation, in arrival order (the
  // reference busy-requeues them to itself, W:95-97/120-123/132-135).
  std::deque<Pending> q;
  q.swap(pending_);
  Scope s(this);
  for (auto& m : q) {
    Payload p = m.p;
    if (!m.owned.empty()) p.ptr = m.owned.data();
    if (m.kind == 0) do_start(m.round);
    else if (m.kind == 1) do_scatter_msg(m.src, m.dest, m.chunk, m.round, p);
    else do_reduce_msg(m.src, m.dest, m.chunk, m.round, m.count, p);
  }
}

bool Engine::present(int32_t id, bool* local) const {
  for (const auto& pe : peers_) {
    if (pe.id == id) {
      *local = pe.local;
      return true;
    }
  }
  return false;
}

Engine::Row& Engine::row(int32_t r) {
  Row& rw = rows_[size_t(r % L_)];
  if (rw.round != r) {
    AKKA_CHECK(rw.round < r, "round " + std::to_string(r) + " maps to a ring row held by newer round " +
                                 std::to_string(rw.round));
    AKKA_CHECK(rw.round < round_ || completed_.count(rw.round) || rw.round < 0,
               "ring row still held by live round " + std::to_string(rw.round));
    rw.round = r;
    rw.sc_mask.assign(size_t(std::max(kme_, 1)) * N_, 0);
    rw.sc_count.assign(size_t(std::max(kme_, 1)), 0);
    rw.sc_reduced.assign(size_t(std::max(kme_, 1)), 0);
    rw.rd_landed.assign(size_t(N_) * kmax_, 0);
    rw.rd_arrivals = 0;
    rw.done = false;
  }
  return rw;
}

const Engine::Row* Engine::find_row(int32_t r) const {
  if (r < 0 || rows_.empty()) return nullptr;
  const Row& rw = rows_[size_t(r % L_)];
  return rw.round == r ? &rw : nullptr;
}

int32_t Engine::scatter_count(int32_t r, int32_t chunk) const {
  const Row* rw = find_row(r);
  if (!rw || chunk < 0 || chunk >= kme_) return 0;
  return rw->sc_count[size_t(chunk)];
}

int32_t Engine::reduced_arrivals(int32_t r) const {
  const Row* rw = find_row(r);
  return rw ? rw->rd_arrivals : 0;
}

void Engine::ensure_output(int32_t r) {
  if (!dp_->has_output(r)) host_->alloc_output(r);
  AKKA_CHECK(dp_->has_output(r), "alloc_output did not bind an output for round " + std::to_string(r));
}

// ---------------------------------------------------------------------------
// External events

void Engine::start(int32_t r) {
  if (!initialized()) {
    Pending m{0, -1, -1, -1, r, 0, {}, {}};
    pending_.push_back(std::move(m));
    return;
  }
  Scope s(this);
  do_start(r);
}

void Engine::on_scatter(int32_t src, int32_t dest, int32_t chunk, int32_t r, const Payload& p) {
  // Pre-init payload messages are queued by the embedding layer, which owns
  // their bytes (the reference busy-requeues them, W:120-123).
  AKKA_CHECK(initialized(), "ScatterBlock delivered before InitWorkers");
  Scope s(this);
  do_scatter_msg(src, dest, chunk, r, p);
}

void Engine::on_reduce(int32_t src, int32_t dest, int32_t chunk, int32_t r, int32_t count, const Payload& p) {
  AKKA_CHECK(initialized(), "ReduceBlock delivered before InitWorkers");
  Scope s(this);
  do_reduce_msg(src, dest, chunk, r, count, p);
}

void Engine::on_peer_terminated(int32_t id) {
  // Reachable here (the control plane tells workers about deaths); the
  // reference's handler never fires because workers never watch peers (W:141-146).
  peers_.erase(std::remove_if(peers_.begin(), peers_.end(), [id](const PeerEntry& p) { return p.id == id; }),
               peers_.end());
  if (link_ && id != id_) {
    Scope s(this);  // the link may deliver / retire rounds: pump afterwards
    link_->on_peer_lost(id);
  }
}

void Engine::flush_deferred(int32_t r) {
  if (!awaiting_finalize_.count(r)) return;
  Scope s(this);
  awaiting_finalize_.erase(r);
  const Row* rw = find_row(r);
  AKKA_CHECK(rw, "deferred round lost its ring row");
  dp_->finalize(r, rw->rd_landed);
  host_->deliver(r);
}

// ---------------------------------------------------------------------------
// Handlers

void Engine::do_start(int32_t r) {
  max_round_ = std::max(max_round_, r);
  // Catch-up: a worker more than maxLag rounds behind force-completes its
  // oldest rounds with whatever arrived (W:100-106).
  while (round_ < max_round_ - params_.max_lag) {
    const int32_t r0 = round_;
    for (int32_t k = 0; k < kme_; ++k) {
      if (round_ != r0) break;  // a self-delivered chunk completed r0 (quirk 1)
      Row& rw = row(r0);
      if (!rw.sc_reduced[size_t(k)]) reduce_and_broadcast(r0, k, /*forced=*/true);
    }
    if (!completed_.count(r0)) {
      ++stats_.rounds_forced;
      complete(r0);
    }
    AKKA_CHECK(round_ > r0, "catch-up made no progress");
  }
  while (max_scattered_ < max_round_) {
    const int32_t next = max_scattered_ + 1;
    host_->fetch(next);
    AKKA_CHECK(dp_->has_input(next), "fetch did not bind an input for round " + std::to_string(next));
    if (bulk_eligible(next) && link_->bulk_round(next)) {
      max_scattered_ = next;
      complete_bulk(next);
      continue;
    }
    scatter(next);
    max_scattered_ = next;
    if (link_) link_->on_scattered(next);
    // Catch-up re-scatters rounds it already force-completed (W:107-111, T17):
    // peers still behind can use them; locally the input can go now.
    if (next < round_ || completed_.count(next)) host_->release(next);
  }
  for (auto it = completed_.begin(); it != completed_.end();) {
    if (*it < round_) it = completed_.erase(it);
    else ++it;
  }
}

void Engine::scatter(int32_t r) {
  // Rotated from self: idx = (i + id) % N (W:213-214).  The reference loops
  // `0 until peers.size`, skipping some known peers when membership is
  // non-contiguous; looping over all N ids fixes that and is identical for a
  // contiguous map.
  for (int32_t i = 0; i < N_; ++i) {
    const int32_t idx = (i + id_) % N_;
    bool local = false;
    if (!present(idx, &local)) continue;
    const int32_t kn = g_.num_chunks(idx);
    for (int32_t k = 0; k < kn; ++k) {
      Payload p = dp_->input_chunk(r, idx, k);
      if (local) do_scatter_msg(id_, idx, k, r, p);
      else if (link_) link_->send_scatter(idx, k, r, p);
    }
  }
}

bool Engine::bulk_eligible(int32_t r) const {
  // The outcome of round r is fixed with exact thresholds and the full
  // membership.  The decision must not depend on local timing: a scheduled
  // link runs exact rounds with their own pairwise-matched schedule, so every
  // rank has to take it for the same rounds.  Local state that would make
  // this rank deviate (older rounds still open, part of r already received)
  // is an error rather than a silent switch to a different schedule.
  // (N = 1 too: the whole round is one local pass, no per-chunk bookkeeping)
  if (!link_ || int32_t(peers_.size()) != N_) return false;
  if (min_scatter_ != N_ || int64_t(min_reduced_) != g_.total_chunks()) return false;
  const bool clean = r == round_ && r == max_round_ && !completed_.count(r) && find_row(r) == nullptr;
  if (!clean && N_ == 1) return false;  // (catch-up at N = 1: the message flow, as before)
  if (!clean) {
    // outbox / reactive links run the message flow for every round anyway
    AKKA_CHECK(!link_->takes_exact_rounds(),
               "round " + std::to_string(r) + " is exact but cannot run as a whole (older rounds open or part of it "
               "already received): the scheduled transport needs rounds started in order");
    return false;
  }
  return true;
}

void Engine::complete_bulk(int32_t r) {
  // Same end state as the message flow of an exact round: every chunk of my
  // block reduced from all N sources, every reduced chunk landed with count N.
  Row& rw = row(r);
  std::fill(rw.sc_mask.begin(), rw.sc_mask.end(), uint8_t(1));
  std::fill(rw.sc_count.begin(), rw.sc_count.end(), N_);
  std::fill(rw.sc_reduced.begin(), rw.sc_reduced.end(), uint8_t(1));
  for (int32_t j = 0; j < N_; ++j)
    for (int32_t k = 0; k < g_.num_chunks(j); ++k) {
      rw.rd_landed[size_t(j) * kmax_ + k] = 1;
      dp_->set_count(r, j, k, N_);
    }
  rw.rd_arrivals = int32_t(g_.total_chunks());
  stats_.scatters_in += int64_t(kme_) * N_;
  stats_.reduces_in += g_.total_chunks();
  stats_.chunks_reduced += kme_;
  ++stats_.bulk_rounds;
  complete(r);
}

void Engine::do_scatter_msg(int32_t src, int32_t dest, int32_t chunk, int32_t r, const Payload& p) {
  ++stats_.scatters_in;
  AKKA_CHECK(dest == id_, "ScatterBlock for worker " + std::to_string(dest) + " routed to " + std::to_string(id_));
  AKKA_CHECK(src >= 0 && src < N_, "ScatterBlock srcId out of range");
  if (r < round_ || completed_.count(r)) {  // outdated (W:172-173)
    ++stats_.outdated_dropped;
    return;
  }
  if (r <= max_round_) {
    AKKA_CHECK(chunk >= 0 && chunk < kme_, "ScatterBlock chunkId out of range");
    Row& rw = row(r);
    dp_->store_scatter(r, src, chunk, p);
    uint8_t& m = rw.sc_mask[size_t(chunk) * N_ + src];
    if (!m) {
      m = 1;
      ++rw.sc_count[size_t(chunk)];
    }
    if (!rw.sc_reduced[size_t(chunk)] && rw.sc_count[size_t(chunk)] >= min_scatter_)
      reduce_and_broadcast(r, chunk, /*forced=*/false);
  } else {
    // Future round: implicit StartAllreduce(r), then handle (W:182-185).
    ++stats_.future_started;
    do_start(r);
    do_scatter_msg(src, dest, chunk, r, p);
  }
}

void Engine::reduce_and_broadcast(int32_t r, int32_t chunk, bool forced) {
  Row& rw = row(r);
  ensure_output(r);
  std::vector<int32_t> srcs;
  for (int32_t s = 0; s < N_; ++s)
    if (rw.sc_mask[size_t(chunk) * N_ + s]) srcs.push_back(s);
  const int32_t count = rw.sc_count[size_t(chunk)];
  Payload p = dp_->reduce(r, chunk, srcs);
  rw.sc_reduced[size_t(chunk)] = 1;
  ++stats_.chunks_reduced;
  if (forced) ++stats_.forced_reduces;
  // Broadcast in the same rotated order (W:254-255).
  for (int32_t i = 0; i < N_; ++i) {
    const int32_t idx = (i + id_) % N_;
    bool local = false;
    if (!present(idx, &local)) continue;
    if (local) do_reduce_msg(id_, idx, chunk, r, count, p);
    else if (link_) link_->send_reduce(idx, chunk, r, count, p);
  }
}

void Engine::do_reduce_msg(int32_t src, int32_t dest, int32_t chunk, int32_t r, int32_t count, const Payload& p) {
  ++stats_.reduces_in;
  // Validation of W:150-154.
  AKKA_CHECK(p.len <= params_.max_chunk_size, "Reduced block of size " + std::to_string(p.len) +
                                                  " is larger than expected.. Max msg size is " +
                                                  std::to_string(params_.max_chunk_size));
  AKKA_CHECK(dest == id_, "Message with destination " + std::to_string(dest) + " was incorrectly routed to node " +
                              std::to_string(id_));
  AKKA_CHECK(src >= 0 && src < N_, "ReduceBlock srcId out of range");
  if (r < round_ || completed_.count(r)) {  // outdated (W:155-156)
    ++stats_.outdated_dropped;
    return;
  }
  if (r <= max_round_) {
    AKKA_CHECK(chunk >= 0 && chunk < g_.num_chunks(src), "ReduceBlock chunkId out of range");
    Row& rw = row(r);
    ensure_output(r);
    dp_->store_reduced(r, src, chunk, p);
    if (count >= 0) dp_->set_count(r, src, chunk, count);
    uint8_t& l = rw.rd_landed[size_t(src) * kmax_ + chunk];
    if (!l) {
      l = 1;
      ++rw.rd_arrivals;
    }
    if (!rw.done && rw.rd_arrivals >= min_reduced_) complete(r);
  } else {
    ++stats_.future_started;
    do_start(r);
    do_reduce_msg(src, dest, chunk, r, count, p);
  }
}

void Engine::complete(int32_t r) {
  Row& rw = row(r);
  rw.done = true;
  ensure_output(r);
  finalize_round(r);
  host_->notify_complete(r);
  completed_.insert(r);
  ++stats_.rounds_completed;
  if (round_ == r) {
    do {
      ++round_;
    } while (completed_.count(round_));
  }
}

void Engine::finalize_round(int32_t r) {
  if (link_ && !link_->may_finalize(r)) {
    awaiting_finalize_.insert(r);
    return;
  }
  const Row& rw = rows_[size_t(r % L_)];
  // Every count arrived with its ReduceBlock header: all rows are host-known.
  std::vector<int32_t> all(static_cast<size_t>(N_), 0);
  for (int32_t j = 0; j < N_; ++j) all[size_t(j)] = j;
  // (bulk rounds whose writes all end on the comm stream finalize there)
  dp_->upload_counts(r, all, dp_->exec_on_comm(r) || dp_->exec_on_producer(r) ? dp_->exec_stream(r)
                                                                                  : dp_->device()->compute_stream());
  dp_->finalize(r, rw.rd_landed);
  host_->deliver(r);
}

void Engine::leave_scope() {
  if (link_) link_->pump();
}

}  // namespace akka
