#include "stream_link.h"

#include <algorithm>
#include <cstdlib>

namespace akka {

StreamLink::StreamLink(Engine* engine, P2P* p2p, int32_t lag) : engine_(engine), p2p_(p2p), lag_(lag) {
  AKKA_CHECK(lag >= 1, "broadcast lag must be >= 1 (a chunk is reduced after its scatter step)");
}

StreamLink::~StreamLink() {
  if (graphs_map_.empty() || !dp_) return;
  Device* dev = dp_->device();
  try {
    dev->sync_stream(dev->comm_stream());
  } catch (...) {
  }
  for (auto& kv : graphs_map_) dev->destroy_graph(kv.second.exec);
}

void StreamLink::set_graphs(bool on) {
  graphs_ = on && dp_ && !dp_->device()->is_host();
  if (!graphs_) drop_graphs();
}

void StreamLink::drop_graphs() {
  if (graphs_map_.empty()) return;
  Device* dev = dp_->device();
  dev->sync_stream(dev->comm_stream());
  for (auto& kv : graphs_map_) dev->destroy_graph(kv.second.exec);
  graphs_map_.clear();
}

void StreamLink::set_exact_unit_bytes(int64_t bytes) {
  if (bytes == unit_bytes_) return;
  unit_bytes_ = bytes;
  exact_.clear();  // rebuilt by the next exact round
  drop_graphs();   // captured with the old template
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
  // Partial membership (W:213-216, SPEC:141-172): the step schedule runs over
  // the peers in the current peer map.  Both sides of a pair must agree, which
  // holds when the map changes at a round boundary (InitWorkers, death).
  std::vector<uint8_t> present(size_t(N), 0);
  bool any_peer = false;
  for (const auto& pe : engine_->peers())
    if (pe.id >= 0 && pe.id < N) {
      present[size_t(pe.id)] = 1;
      any_peer |= pe.id != me;
    }
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
    // (no remote peer in the map: my reduced chunks have nobody to go to)
    bool bcast_step = any_peer && kb >= 0 && kb < kme;
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
      if (!present[size_t(peer)]) continue;
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
        if (!present[size_t(peer)]) continue;
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
        if (!present[size_t(peer)] || kb >= g.num_chunks(peer)) continue;
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
  AKKA_CHECK(dp_, "stream link has no data plane");
  const Geometry& g = dp_->geometry();
  const int32_t N = g.N;
  if (N < 2) {
    // N = 1: input -> output in one launch on the producer's stream (bind_input
    // put the round there), the counts fill riding in it (HipDevice::fill_i32);
    // none of the per-chunk scatter / reduce / broadcast bookkeeping, whose
    // host cost grows with the chunk count (profiles/r06/small_rounds/)
    engine_->ensure_output(r);
    // claim the round's ring row first: claiming it later (complete_bulk's
    // set_count) flushes the pending reduce, and the counts fill could no
    // longer ride in it -- a second launch per round
    dp_->set_count(r, 0, 0, 1);
    const StreamH s = dp_->exec_stream(r);
    dp_->wait_input(r, s);
    const void* in = dp_->input_chunk(r, 0, 0).ptr;
    void* out = dp_->output_at(r, 0, 0);
    if (in != out && g.S > 0) {
      auto specs = split_reduce(out, {in}, g.S);
      dp_->device()->reduce(s, specs.data(), int32_t(specs.size()), dp_->dtype());
    }
    stats_.rounds++;
    stats_.bulk_rounds++;
    mark_scheduled(r);
    return true;
  }
  AKKA_CHECK(p2p_->nranks() == N && p2p_->rank() == dp_->me(), "p2p communicator does not match the worker geometry");
  const bool native = p2p_->has_collectives() && g.S == int64_t(N) * g.step;
  // Auto = the framework's own p2p schedule (gfx950 reduce); RCCL's
  // reduce-scatter + all-gather runs only when asked for by name.
  dp_->set_poison_flag(lane_ == Lane::Ipc && ipc_ ? ipc_->error_word_device() : nullptr);
  // every write of a bulk round ends in comm-stream order (ipc kernels; the
  // step schedule's last broadcasts wait for every reduce; RCCL's
  // collectives): its counts and done point go there too, no stream hop
  dp_->set_exec_comm(r);
  if (lane_ == Lane::Ipc) ipc_round(r);
  else if (lane_ == Lane::Collective) collective_round(r, native);
  else exact_steps(r);
  p2p_->check();
  stats_.rounds++;
  stats_.bulk_rounds++;
  mark_scheduled(r);
  return true;
}

void StreamLink::set_ipc(std::unique_ptr<IpcLane> ipc) {
  if (ipc_ && dp_) {
    dp_->device()->sync_stream(dp_->device()->comm_stream());
    if (ipc_last_stream_set_ && ipc_last_stream_ != dp_->device()->comm_stream()) {
      // the last round ran on a caller's stream: wait for it through an event
      // recorded there now (the stream handle is the caller's, still alive
      // while its rounds are in flight)
      EventH e = dp_->pooled_event_public();
      dp_->device()->record(e, ipc_last_stream_);
      dp_->device()->sync_event(e);
    }
  }
  ipc_ = std::move(ipc);
  ipc_last_stream_set_ = false;
}

void StreamLink::ipc_round(int32_t r) {
  AKKA_CHECK(ipc_ && ipc_->ready(), "ipc lane selected but its windows are not open (ipc_open)");
  // a wait of an earlier round timed out (a peer missing or too late): like
  // an RCCL async error, it ends the lane's rounds with an exception
  AKKA_CHECK(ipc_->error_now() == 0,
             "ipc lane: a wait of an earlier round timed out (peer missing?); its rounds are not trustworthy");
  Device* dev = dp_->device();
  engine_->ensure_output(r);
  StreamH comm = dev->comm_stream();
  // A synchronous call runs its round on the caller's own stream: the ipc
  // kernels need no stream of the engine's, and the caller waits anyway --
  // no input event, no done event (the direct rounds' cost, through the
  // engine's bookkeeping).  Async calls keep the comm stream (overlap).
  StreamH s = comm;
  if (dp_->caller_waits(r)) s = dp_->run_on_caller(r);
  // Rounds of the lane run one at a time: a round on another stream than
  // the previous one's orders behind it first (windows are reused)
  if (ipc_last_stream_set_ && ipc_last_stream_ != s) {
    EventH e = dp_->pooled_event_public();
    dev->record(e, ipc_last_stream_);
    dev->wait(s, e);
  }
  ipc_last_stream_ = s;
  ipc_last_stream_set_ = true;
  // (no ring row: the ipc kernels move the bytes through the lane's own
  // windows, so the round does not wait for the compute stream's readers)
  if (s == comm) {
    dp_->wait_input(r, comm);
    dp_->mark_comm_used(r);
  }
  // the round's counts (N everywhere, 0 if a wait failed) are written by the
  // round's last kernel: no fill launch behind it (profiles/r05/engine_path/)
  int32_t* counts = dp_->has_counts(r) ? dp_->counts_row(r, 0) : nullptr;
  if (counts) dp_->set_counts_by_lane(r);
  ipc_->round(s, dp_->input_chunk(r, 0, 0).ptr, dp_->output_at(r, 0, 0), nullptr, 0, counts,
              int64_t(dp_->geometry().N) * dp_->kmax(), dp_->geometry().N);
  const Geometry& g = dp_->geometry();
  stats_.bytes_sent += int64_t(2) * (g.S - g.block_len(dp_->me())) * int64_t(dp_->esize());
  ++stats_.ipc_rounds;
}

void StreamLink::collective_round(int32_t r, bool native) {
  const Geometry& g = dp_->geometry();
  const int32_t N = g.N;
  const int32_t me = dp_->me();
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
    return;
  }
  ++stats_.collective_rounds;
  // Whole-block direct exchange: the reference's scatter / reduce / broadcast
  // (W:212-268) with one message per peer and phase.
  std::vector<P2POp>& ops = scratch_;
  ops.clear();
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
    for (int32_t src = 0; src < N; ++src)  // ascending source id, like the message flow
      srcs.push_back(src == me ? static_cast<const void*>(in + size_t(g.block_start(me)) * es)
                               : dp_->scatter_slot(r, src, 0));
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
  for (int32_t i = 1; i < N; ++i) stats_.bytes_sent += (g.block_len((me + i) % N) + my_len) * int64_t(es);
}

void StreamLink::build_exact_template() {
  // The exact round's step schedule depends only on the geometry and the lag:
  // built once, then every round only adds three base pointers.  Same groups
  // and per-pair order as schedule() minus the counts exchange (all N).
  const Geometry& g0 = dp_->geometry();
  const int32_t me = dp_->me();
  const int32_t N = g0.N;
  const size_t es = dp_->esize();
  // Transfer unit: m consecutive chunks moved as one (>= 16 MiB per unit, or
  // AKKA_EXACT_UNIT_BYTES).  The outcome of an exact round does not depend on
  // how its bytes are cut, and every p2p op costs the host 4-7 us inside
  // ncclGroupEnd (profiles/r02/host): fewer, larger steps.  A function of the
  // geometry only, so every rank builds the same groups.
  int64_t min_bytes = int64_t(16) << 20;
  if (unit_bytes_ >= 0) min_bytes = unit_bytes_;
  else if (const char* v = std::getenv("AKKA_EXACT_UNIT_BYTES")) min_bytes = std::max<int64_t>(0, std::atoll(v));
  min_bytes = std::min<int64_t>(min_bytes, int64_t(1) << 50);
  const int64_t cbytes = std::max<int64_t>(1, g0.C * int64_t(es));
  unit_chunks_ = int32_t(std::clamp<int64_t>((min_bytes + cbytes - 1) / cbytes, 1,
                                             std::max(1, g0.max_block_len_chunks())));
  gx_ = Geometry(g0.S, N, g0.C * unit_chunks_);
  const Geometry& g = gx_;
  const int32_t kme = g.num_chunks(me);
  const int32_t steps = g.max_block_len_chunks() + lag_;
  const char* ring0 = static_cast<const char*>(dp_->scatter_slot(0, 0, 0));
  exact_.assign(size_t(steps), {});
  for (int32_t s = 0; s < steps; ++s) {
    auto& v = exact_[size_t(s)];
    const int32_t kb = s - lag_;
    const bool bcast = kb >= 0 && kb < kme;
    for (int32_t i = 1; i < N; ++i) {
      const int32_t peer = (me + i) % N;
      const int32_t kp = g.num_chunks(peer);
      if (s < kp) v.push_back({true, peer, 0, g.chunk_offset(peer, s) * int64_t(es), size_t(g.chunk_len(peer, s)) * es});
      if (s < kme)  // unit s starts at chunk s*m of the slot
        v.push_back({false, peer, 1, static_cast<const char*>(dp_->scatter_slot(0, peer, s * unit_chunks_)) - ring0,
                     size_t(g.chunk_len(me, s)) * es});
      if (bcast) v.push_back({true, peer, 2, g.chunk_offset(me, kb) * int64_t(es), size_t(g.chunk_len(me, kb)) * es});
      if (kb >= 0 && kb < kp)
        v.push_back({false, peer, 2, g.chunk_offset(peer, kb) * int64_t(es), size_t(g.chunk_len(peer, kb)) * es});
    }
  }
  reduced_ev_.assign(size_t(std::max(kme, 1)), nullptr);
  exact_groups_ = exact_ops_ = exact_bytes_ = 0;
  for (const auto& v : exact_) {
    if (!v.empty()) ++exact_groups_;
    exact_ops_ += int64_t(v.size());
    for (const auto& t : v)
      if (t.send) exact_bytes_ += int64_t(t.bytes);
  }
}

void StreamLink::exact_steps(int32_t r) {
  if (exact_.empty()) build_exact_template();
  Device* dev = dp_->device();
  engine_->ensure_output(r);
  StreamH comm = dev->comm_stream();
  dp_->comm_wait(dp_->row_release_event(r));  // ring row r%L was last read by round r-L's reduces
  dp_->wait_input(r, comm);
  dp_->mark_comm_used(r);
  char* base[3] = {const_cast<char*>(static_cast<const char*>(dp_->input_chunk(r, 0, 0).ptr)),
                   static_cast<char*>(dp_->scatter_slot(r, 0, 0)), static_cast<char*>(dp_->output_at(r, 0, 0))};
  ++stats_.exact_step_rounds;
  if (graphs_) {
    auto key = std::make_tuple(base[0], base[1], base[2]);
    GraphEntry& ge = graphs_map_[key];
    ge.last_use = ++tick_;
    if (ge.exec) {
      // the whole round is in comm-stream order: everything after it (the
      // next round's ring reuse, finalize's join) orders behind the launch
      dev->launch_graph(ge.exec, comm);
      ++stats_.graph_replays;
      stats_.groups += exact_groups_;
      stats_.ops += exact_ops_;
      stats_.bytes_sent += exact_bytes_;
      return;
    }
    if (++ge.seen >= 2) {
      if (graphs_map_.size() > 16) {  // LRU: keep the cache bounded (fresh buffers every round never repeat)
        auto victim = graphs_map_.end();
        for (auto it = graphs_map_.begin(); it != graphs_map_.end(); ++it)
          if (it->first != key && (victim == graphs_map_.end() || it->second.last_use < victim->second.last_use))
            victim = it;
        if (victim != graphs_map_.end()) {
          if (victim->second.exec) {
            dev->sync_stream(comm);
            dev->destroy_graph(victim->second.exec);
          }
          graphs_map_.erase(victim);
        }
      }
      GraphEntry& g2 = graphs_map_[key];
      GraphH exec = nullptr;
      dev->begin_capture(comm);
      try {
        exact_body(r, base, /*captured=*/true);
        exec = dev->end_capture(comm, false);
      } catch (const std::exception& e) {
        dev->end_capture(comm, true);
        graph_error_ = e.what();
        set_graphs(false);  // capture unsupported here: stay eager from now on
        exact_body(r, base, false);
        return;
      }
      g2.exec = exec;
      ++stats_.graph_captures;
      dev->launch_graph(exec, comm);
      stats_.groups += exact_groups_;
      stats_.ops += exact_ops_;
      stats_.bytes_sent += exact_bytes_;
      return;
    }
  }
  exact_body(r, base, false);
  stats_.groups += exact_groups_;
  stats_.ops += exact_ops_;
  stats_.bytes_sent += exact_bytes_;
}

void StreamLink::exact_body(int32_t r, char* const base[3], bool captured) {
  const Geometry& g = gx_;  // transfer units (build_exact_template)
  const int32_t me = dp_->me();
  const int32_t N = g.N;
  const size_t es = dp_->esize();
  const int32_t kme = g.num_chunks(me);
  Device* dev = dp_->device();
  StreamH comm = dev->comm_stream();
  StreamH cs = dev->compute_stream();
  // Eager: the compute stream waits for the input's producer.  Captured: the
  // compute branch forks from the comm stream inside the graph, which starts
  // after the comm stream's (eager) input wait.
  if (!captured && kme > 0) dp_->wait_input(r, cs);
  std::vector<P2POp>& ops = scratch_;
  std::vector<const void*> srcs(static_cast<size_t>(N), nullptr);
  for (size_t s = 0; s < exact_.size(); ++s) {
    const int32_t kb = int32_t(s) - lag_;
    if (kb >= 0 && kb < kme) dp_->comm_wait(reduced_ev_[size_t(kb)]);
    ops.clear();
    for (const OpT& t : exact_[s]) ops.push_back({t.send, t.peer, base[t.base] + t.off, t.bytes});
    if (!ops.empty()) p2p_->group(comm, ops);
    if (int32_t(s) < kme) {
      // unit s of my block landed from every peer: reduce it (compute stream)
      dp_->compute_wait(dp_->record_comm());
      const int32_t k = int32_t(s);
      for (int32_t src = 0; src < N; ++src)  // ascending source id, like the message flow
        srcs[size_t(src)] = src == me ? static_cast<const void*>(base[0] + g.chunk_offset(me, k) * int64_t(es))
                                      : dp_->scatter_slot(r, src, k * unit_chunks_);
      auto specs = split_reduce(base[2] + g.chunk_offset(me, k) * int64_t(es), srcs, g.chunk_len(me, k));
      dev->reduce(cs, specs.data(), int32_t(specs.size()), dp_->dtype());
      reduced_ev_[size_t(k)] = dp_->record_compute();
    }
  }
  // A capture must end with every forked stream joined back (the last
  // broadcast step already waited for the last reduce; this covers kme == 0).
  if (captured && kme > 0) dp_->comm_wait(dp_->record_compute());
}

void StreamLink::mark_scheduled(int32_t r) {
  scheduled_.insert(r);
  while (scheduled_.size() > 4096) scheduled_.erase(scheduled_.begin());
  engine_->flush_deferred(r);
}

}  // namespace akka
