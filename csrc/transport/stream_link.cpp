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

bool StreamLink::bulk_round(int32_t r) {
  if (lane_ == Lane::P2P || !dp_) return false;
  const Geometry& g = dp_->geometry();
  const int32_t N = g.N;
  const int32_t me = dp_->me();
  if (N < 2) return false;  // a local round is already one pass
  const bool native = p2p_->has_collectives() && g.S == int64_t(N) * g.step;
  if (lane_ == Lane::Auto && !native) return false;
  AKKA_CHECK(p2p_->nranks() == N && p2p_->rank() == me, "p2p communicator does not match the worker geometry");
  const size_t es = dp_->esize();
  Device* dev = dp_->device();
  engine_->ensure_output(r);
  StreamH comm = dev->comm_stream();
  dp_->comm_wait(dp_->row_release_event(r));  // the direct exchange lands in ring row r%L
  dp_->wait_input(r, comm);
  dp_->mark_comm_used(r);
  const char* in = static_cast<const char*>(dp_->input_chunk(r, 0, 0).ptr);
  char* out = static_cast<char*>(dp_->output_at(r, 0, 0));
  char* mine = out + size_t(g.block_start(me)) * es;
  const int64_t my_len = g.block_len(me);
  if (native) {
    // phase 1 = reduce-scatter of the N blocks, phase 2 = all-gather of the
    // reduced blocks (in place): RCCL's own xGMI schedules, two calls a round
    p2p_->reduce_scatter(comm, in, mine, size_t(g.step), dp_->dtype());
    p2p_->all_gather(comm, mine, out, size_t(g.step), dp_->dtype());
    stats_.groups += 2;
    stats_.bytes_sent += int64_t(2) * (N - 1) * g.step * int64_t(es);
    ++stats_.collective_rounds;
  } else {
    // Whole-block direct exchange: the reference's scatter / reduce /
    // broadcast (W:212-268) with one message per peer and phase.
    std::vector<P2POp> ops;
    for (int32_t i = 1; i < N; ++i) {
      const int32_t peer = (me + i) % N;
      const int64_t plen = g.block_len(peer);
      if (plen > 0) ops.push_back({true, peer, const_cast<char*>(in) + size_t(g.block_start(peer)) * es, size_t(plen) * es});
      if (my_len > 0) ops.push_back({false, peer, dp_->scatter_slot(r, peer, 0), size_t(my_len) * es});
    }
    if (!ops.empty()) {
      p2p_->group(comm, ops);
      stats_.groups++;
      stats_.ops += int64_t(ops.size());
    }
    if (my_len > 0) {
      StreamH cs = dev->compute_stream();
      dp_->compute_wait(dp_->record_comm());
      dp_->wait_input(r, cs);
      std::vector<const void*> srcs;
      srcs.push_back(in + size_t(g.block_start(me)) * es);
      for (int32_t i = 1; i < N; ++i) srcs.push_back(dp_->scatter_slot(r, (me + i) % N, 0));
      auto specs = split_reduce(mine, srcs, my_len);
      dev->reduce(cs, specs.data(), int32_t(specs.size()), dp_->dtype());
      dp_->comm_wait(dp_->record_compute());
    }
    ops.clear();
    for (int32_t i = 1; i < N; ++i) {
      const int32_t peer = (me + i) % N;
      const int64_t plen = g.block_len(peer);
      if (my_len > 0) ops.push_back({true, peer, mine, size_t(my_len) * es});
      if (plen > 0) ops.push_back({false, peer, out + size_t(g.block_start(peer)) * es, size_t(plen) * es});
    }
    if (!ops.empty()) {
      p2p_->group(comm, ops);
      stats_.groups++;
      stats_.ops += int64_t(ops.size());
    }
    for (int32_t i = 1; i < N; ++i)
      stats_.bytes_sent += (g.block_len((me + i) % N) + my_len) * int64_t(es);
  }
  p2p_->check();
  stats_.rounds++;
  stats_.bulk_rounds++;
  mark_scheduled(r);
  return true;
}

void StreamLink::mark_scheduled(int32_t r) {
  scheduled_.insert(r);
  while (scheduled_.size() > 4096) scheduled_.erase(scheduled_.begin());
  engine_->flush_deferred(r);
}

}  // namespace akka
