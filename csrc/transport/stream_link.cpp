#include "stream_link.h"

#include <algorithm>

namespace akka {

StreamLink::StreamLink(Engine* engine, P2P* p2p, int32_t lag) : engine_(engine), p2p_(p2p), lag_(lag) {
  AKKA_CHECK(lag >= 1, "broadcast lag must be >= 1 (a chunk is reduced after its scatter step)");
}

void StreamLink::send_scatter(int32_t dest, int32_t chunk, int32_t round, const Payload& p) {
  q_[round].scatter[{chunk, dest}] = Out{p.ptr, p.len};
}

void StreamLink::send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t /*count*/, const Payload& p) {
  RoundQ& rq = q_[round];
  rq.bcast[{chunk, dest}] = Out{p.ptr, p.len};
  // One event per reduced chunk: the comm stream waits for it before the step
  // that broadcasts the chunk.  The count travels in-band at the last step.
  if (!rq.bcast_ready.count(chunk)) rq.bcast_ready[chunk] = dp_->record_compute();
}

void StreamLink::on_scattered(int32_t round) { ready_.push_back(round); }

bool StreamLink::may_finalize(int32_t round) {
  // Only after every receive of the round has been issued: a round may reach
  // its completion threshold while its later steps are still being enqueued
  // (or, with tiny thresholds, during scatter() before any step exists).
  return scheduled_.count(round) > 0;
}

void StreamLink::pump() {
  if (pumping_) return;
  pumping_ = true;
  try {
    while (!ready_.empty()) {
      int32_t r = ready_.front();
      ready_.pop_front();
      schedule(r);
    }
  } catch (...) {
    pumping_ = false;
    throw;
  }
  pumping_ = false;
}

void StreamLink::schedule(int32_t r) {
  AKKA_CHECK(dp_, "stream link has no data plane");
  const Geometry& g = dp_->geometry();
  const int32_t me = dp_->me();
  const int32_t N = g.N;
  if (N == 1) {  // nothing to move: the round was reduced in place during scatter()
    engine_->ensure_output(r);
    dp_->upload_counts(r, {me}, dp_->exec_stream(r));
    mark_scheduled(r);
    return;
  }
  AKKA_CHECK(p2p_->nranks() == N && p2p_->rank() == me, "p2p communicator does not match the worker geometry");
  auto peers = engine_->peers();
  AKKA_CHECK(int32_t(peers.size()) == N, "scheduled transport needs the full peer map (all N workers)");
  const size_t es = dp_->esize();
  const int32_t kme = g.num_chunks(me);
  const int32_t kmax = dp_->kmax();
  const int32_t steps = g.max_block_len_chunks() + lag_;

  in_flight_.insert(r);
  engine_->ensure_output(r);
  RoundQ& rq = q_[r];
  StreamH comm = dp_->device()->comm_stream();
  // The ring row for r was last read by round r-L's reduces (compute stream).
  dp_->comm_wait(dp_->row_release_event(r));
  dp_->wait_input(r, comm);  // scatter sends read the input
  dp_->mark_comm_used(r);

  std::vector<P2POp> ops;
  for (int32_t s = 0; s < steps; ++s) {
    ops.clear();
    const int32_t kb = s - lag_;
    bool bcast_step = kb >= 0 && kb < kme;
    bool unreduced = false;
    if (bcast_step) {
      auto it = rq.bcast_ready.find(kb);
      if (it == rq.bcast_ready.end()) {
        // The round reached thComplete before this chunk reached thReduce:
        // later scatters were outdated (W:172-173), so it is never reduced.
        // The symmetric schedule still moves the bytes: zeros with in-band
        // count 0 -- what the reference's output shows for a chunk that
        // never arrived (RB:41-47).
        AKKA_CHECK(engine_->is_completed(r), "round " + std::to_string(r) + ": chunk " + std::to_string(kb) +
                                                 " was not reduced by its broadcast step (threshold never reached?)");
        unreduced = true;
        dp_->device()->zero(dp_->exec_stream(r), dp_->output_at(r, me, kb), size_t(g.chunk_len(me, kb)) * es);
        dp_->comm_wait(dp_->record_compute());
        ++stats_.unreduced_chunks;
      } else {
        dp_->comm_wait(it->second);
      }
    }
    const bool last = (s == steps - 1);
    if (last) dp_->upload_counts(r, {me}, comm);
    for (int32_t i = 1; i < N; ++i) {
      const int32_t peer = (me + i) % N;
      const int32_t kp = g.num_chunks(peer);
      if (s < kp) {
        auto it = rq.scatter.find({s, peer});
        AKKA_CHECK(it != rq.scatter.end(), "missing scatter payload for peer " + std::to_string(peer));
        ops.push_back({true, peer, const_cast<void*>(it->second.ptr), size_t(it->second.len) * es});
      }
      if (s < kme) ops.push_back({false, peer, dp_->scatter_slot(r, peer, s), size_t(g.chunk_len(me, s)) * es});
      if (bcast_step && unreduced) {
        ops.push_back({true, peer, dp_->output_at(r, me, kb), size_t(g.chunk_len(me, kb)) * es});
      } else if (bcast_step) {
        auto it = rq.bcast.find({kb, peer});
        AKKA_CHECK(it != rq.bcast.end(), "missing broadcast payload for peer " + std::to_string(peer));
        ops.push_back({true, peer, const_cast<void*>(it->second.ptr), size_t(it->second.len) * es});
      }
      if (kb >= 0 && kb < kp) ops.push_back({false, peer, dp_->output_at(r, peer, kb), size_t(g.chunk_len(peer, kb)) * es});
      if (last) {
        if (kme > 0) ops.push_back({true, peer, dp_->counts_row(r, me), size_t(kme) * sizeof(int32_t)});
        if (kp > 0) ops.push_back({false, peer, dp_->counts_row(r, peer), size_t(kp) * sizeof(int32_t)});
      }
    }
    if (!ops.empty()) {
      p2p_->group(comm, ops);
      stats_.groups++;
      stats_.ops += int64_t(ops.size());
      for (const auto& op : ops)
        if (op.send) stats_.bytes_sent += int64_t(op.bytes);
    }
    EventH landed = dp_->record_comm();
    (void)kmax;
    // Stream-ordered arrival: report what this step received.
    if (s < kme && N > 1) {
      dp_->compute_wait(landed);
      for (int32_t i = 1; i < N; ++i) {
        const int32_t peer = (me + i) % N;
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(me, s);
        p.on_host = false;
        engine_->on_scatter(peer, me, s, r, p);
      }
    }
    if (kb >= 0) {
      for (int32_t i = 1; i < N; ++i) {
        const int32_t peer = (me + i) % N;
        if (kb >= g.num_chunks(peer)) continue;
        Payload p;
        p.kind = PayloadKind::Landed;
        p.len = g.chunk_len(peer, kb);
        p.on_host = false;
        engine_->on_reduce(peer, me, kb, r, /*count in-band*/ -1, p);
      }
    }
  }
  p2p_->check();  // RCCL async errors: once per round, not per group
  in_flight_.erase(r);
  q_.erase(r);
  stats_.rounds++;
  mark_scheduled(r);
}

void StreamLink::mark_scheduled(int32_t r) {
  scheduled_.insert(r);
  while (scheduled_.size() > 4096) scheduled_.erase(scheduled_.begin());
  engine_->flush_deferred(r);
}

}  // namespace akka
