// Data plane: where chunks live and the two compute ops on them.
//
// Replaces the reference's buffer layer (buffer/AllReduceBuffer.scala,
// ScatteredDataBuffer.scala, ReducedDataBuffer.scala) with a layout built for
// zero-copy device transport:
//
//  * scatter ring  [L][N][myBlockLen]   -- peers' contributions to MY block
//    (ScatteredDataBuffer's temporalBuffer, AllReduceBuffer.scala:11-21).
//    My own contribution is never copied: its slot aliases the round's input
//    tensor (the reference short-circuits self messages, W:228-232).
//  * output row    [S] per round         -- the reduced vector at its final
//    offsets, bound per round by the embedding layer (a fresh torch tensor),
//    so ReducedDataBuffer.getWithCounts' concatenation (RB:26-53) is free:
//    peers' reduced chunks are received straight into place.
//  * counts        [N][Kmax] int32       -- contributor count per (block, chunk);
//    the per-element expansion of RB:41-47 is a lazy kernel (count_expand).
//
// All bookkeeping (arrival masks, thresholds, landed flags) lives in the Engine;
// the data plane only owns memory, streams and kernels.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <vector>

#include "device.h"
#include "geometry.h"

namespace akka {

class DataPlane {
 public:
  DataPlane(Device* dev, const Geometry& g, int32_t me, int32_t ring_rows, DType dt);
  ~DataPlane();
  DataPlane(const DataPlane&) = delete;
  DataPlane& operator=(const DataPlane&) = delete;

  Device* device() const { return dev_; }
  const Geometry& geometry() const { return g_; }
  int32_t me() const { return me_; }
  DType dtype() const { return dt_; }
  size_t esize() const { return dtype_size(dt_); }
  int32_t ring_rows() const { return L_; }
  int32_t kmax() const { return kmax_; }

  // --- per-round bindings (memory owned by the embedding layer) ------------
  // `ready_stream` is the stream that produced `input`; it may be the null
  // stream (handle 0), so `has_stream` says whether there is one at all.
  // defer_record: record the input-ready event only when a stream first
  // waits for it (a synchronous call whose round may run on the producer's
  // own stream needs none: one marker less per round).  Only for rounds whose
  // consumers all wait inside the call that binds them (fast_round).
  void bind_input(int32_t round, const void* input, StreamH ready_stream, bool has_stream, bool defer_record = false);
  // `alloc_stream` (optional): the stream in whose order output/counts were
  // allocated (a caching allocator may hand out memory that earlier work on
  // that stream still uses).  Every other stream that writes them waits for
  // that point first (wait_input).  Without one, the input's ready point
  // stands in (the fast path binds the output just before the input).
  void bind_output(int32_t round, void* output, int32_t* counts, StreamH alloc_stream = nullptr,
                   bool has_stream = false);
  bool has_input(int32_t round) const;
  bool has_output(int32_t round) const;
  bool has_counts(int32_t round) const;
  void unbind(int32_t round);

  // --- views ---------------------------------------------------------------
  Payload input_chunk(int32_t round, int32_t block, int32_t k) const;
  Payload output_chunk(int32_t round, int32_t block, int32_t k) const;
  void* scatter_slot(int32_t round, int32_t src, int32_t k) const;
  void* output_at(int32_t round, int32_t block, int32_t k) const;
  int32_t* counts_row(int32_t round, int32_t block) const;

  // --- phase 1 receive side + the chunk N-way sum ----------------------------
  void store_scatter(int32_t round, int32_t src, int32_t k, const Payload& p);
  // Sum the listed sources' copies of my chunk k into the output row; returns a
  // ReducedView payload of the result (what gets broadcast).
  Payload reduce(int32_t round, int32_t k, const std::vector<int32_t>& srcs);

  // --- phase 2 receive side --------------------------------------------------
  void store_reduced(int32_t round, int32_t src, int32_t k, const Payload& p);
  void set_count(int32_t round, int32_t block, int32_t k, int32_t count);
  // Error word of the lane that moves the next rounds (nullptr: none): a
  // round finalized while it is set gets all-zero counts (ipc lane failure).
  void set_poison_flag(const uint32_t* f) { poison_flag_ = f; }
  // Copy host-known counts of the given blocks into the round's counts tensor.
  void upload_counts(int32_t round, const std::vector<int32_t>& blocks, StreamH s);

  // Zero data+count of chunks that never landed (landed: [N][kmax] flags), join
  // the comm and compute streams and record the round's done event.
  void finalize(int32_t round, const std::vector<uint8_t>& landed);
  // Make `stream` wait for the round's done event (stream-ordered hand-off).
  void stream_wait_done(int32_t round, StreamH stream);
  // Host-blocking wait for the round (used by the host/outbox paths).
  void sync_done(int32_t round);

  // Copy a payload to host bytes (probe/TCP transports). Synchronous.
  void read_payload(const Payload& p, void* host_dst) const;

  // Stream hooks for the scheduled link.
  EventH pooled_event_public() { return pooled_event(); }
  EventH record_compute();
  EventH record_comm();
  void compute_wait(EventH e) { dev_->wait(dev_->compute_stream(), e); }
  void comm_wait(EventH e) { dev_->wait(dev_->comm_stream(), e); }
  // Stream that runs the round's reduces/copies/finalize: the compute stream,
  // or -- for a purely local round (N == 1) -- the input producer's stream.
  StreamH exec_stream(int32_t round) const;
  bool exec_on_producer(int32_t round) const;
  // A bulk (whole exact) round whose every write ends in comm-stream order
  // (ipc kernels, the exact step schedule, RCCL's collectives): its counts and
  // finalize run on the comm stream too, so the round needs no comm -> compute
  // -> comm event hop before its done point (profiles/r05/engine_path/).
  void set_exec_comm(int32_t round);
  // The lane's own kernels write this round's counts (and apply the poison
  // flag themselves): upload_counts / finalize leave them alone.
  void set_counts_by_lane(int32_t round);
  // The caller's stream will wait for this round (a synchronous call).
  void set_caller_waits(int32_t round);
  bool caller_waits(int32_t round) const;
  // Run the round on the stream that produced its input (the caller's): it
  // is then in that stream's order with no event hop either way, like a
  // purely local round.  Needs caller_waits() and a producer stream.
  StreamH run_on_caller(int32_t round);
  bool exec_on_comm(int32_t round) const;
  // Make `s` wait (once per round) for the stream that produced the input and
  // for the point where the output/counts memory was handed over: every
  // stream that reads the input or writes the output/counts calls it first.
  void wait_input(int32_t round, StreamH s);
  // The comm stream wrote into this round's output (finalize must join it).
  void mark_comm_used(int32_t round);
  // Event after the last compute op that reads ring row of `round`.
  EventH row_release_event(int32_t round);

  // --- staged mode (reactive transport) ------------------------------------
  // With per-peer streams a round can complete while some of its sends and
  // receives are still in flight (the threshold semantics: a straggler's
  // transfers finish later).  So nothing in flight may touch memory the
  // caller owns:
  //  * send side -- a per-round *send slot* from a pool: the staged input
  //    (copied at bind time), my reduced block, my wire counts.  A slot stays
  //    busy until its round completed and all its transfers finished; while a
  //    peer is frozen the pool grows (up to `max_slots`), so fast ranks keep
  //    going for that many rounds before the oldest slot must be reclaimed by
  //    waiting (`reclaim(round)`: the link makes the compute stream wait for
  //    that round's outstanding transfers).
  //  * receive side -- peers' reduced blocks land in a ring row (receives on a
  //    pair stream are ordered, so ring reuse is safe); finalize() copies the
  //    landed chunks into the user's output.
  void enable_staging(int32_t max_slots, std::function<bool(int32_t)> reclaim);
  bool staging() const { return staging_on_; }
  const void* staged_input(int32_t round, int32_t block);
  void* mine_at(int32_t round, int32_t k);
  int32_t* wire_dev(int32_t round);
  int32_t* wire_host(int32_t round);
  void* landing_at(int32_t round, int32_t block, int32_t k) const;
  // The link is done with the round's send slot (completed + transfers done).
  void release_slot(int32_t round);
  int32_t slots_allocated() const { return int32_t(slots_.size()); }
  int32_t slots_busy() const;

 private:
  struct Binding {
    const void* input = nullptr;
    void* output = nullptr;
    int32_t* counts = nullptr;
    EventH input_ready = nullptr;  // recorded on the producer stream
    bool input_waited_compute = false;
    bool input_waited_comm = false;
    bool input_pending = false;    // input_ready not recorded yet (bind_input defer_record)
    bool input_idle = false;       // the producer stream was idle at bind time: nothing to wait for
    EventH output_ready = nullptr;  // recorded on the stream that allocated output/counts
    bool output_waited_compute = false;
    bool output_waited_comm = false;
    bool comm_used = false;  // the comm stream wrote into this round (join at finalize)
    StreamH exec = nullptr;  // stream running this round's compute when exec_on_producer
    bool exec_on_producer = false;
    bool exec_on_comm = false;     // set_exec_comm: counts + finalize on the comm stream
    bool counts_poisoned = false;  // the counts fill already applied the poison flag
    bool counts_by_lane = false;   // set_counts_by_lane
    bool caller_waits = false;     // set_caller_waits
    StreamH ready = nullptr;       // the producer stream given at bind_input (has_ready)
    bool has_ready = false;
    EventH done = nullptr;
    // Producer-stream rounds record `done` only when someone asks for it: the
    // round is already in that stream's order, and a marker between two
    // back-to-back reduce launches costs the command processor a few us.  A
    // later record on the same stream covers this round (and possibly more).
    bool done_lazy = false;
    bool finalized = false;
  };
  EventH done_event(Binding& b);
  struct Row {
    int32_t round = -1;
    std::vector<uint8_t> self_alias;  // [K_me]: slot[me] of chunk k aliases the input
    EventH released = nullptr;        // compute-stream event after last reader
    EventH staging_done = nullptr;    // comm-stream event after last counts upload
  };

  Row& row_for(int32_t round);
  const Binding& binding(int32_t round) const;
  Binding& binding_mut(int32_t round);

  EventH pooled_event();
  EventH binding_event();

  Device* dev_;
  Geometry g_;
  int32_t me_;
  int32_t L_;
  DType dt_;
  int32_t kme_;
  int32_t kmax_;
  int64_t my_len_;
  int64_t mis_el_ = 0;       // my block's offset mod 16 B, in elements
  int64_t slot_stride_ = 0;  // scatter slot / own-block buffer stride (elements, 16-B multiple)
  int64_t row_stride_ = 0;   // landing row stride (elements, 16-B multiple)
  void* scatter_ring_ = nullptr;   // [L][N][slot_stride]
  int32_t* staging_ = nullptr;     // pinned [L][N][kmax]
  std::vector<Row> rows_;
  std::map<int32_t, Binding> bind_;
  std::vector<EventH> events_;     // all events created (destroyed at teardown)
  std::vector<EventH> free_events_;
  std::vector<EventH> spare_events_;  // recycled per-round (input_ready / done) events
  // staged mode
  struct SendSlot {
    int32_t round = -1;
    void* input = nullptr;      // [S]
    void* mine = nullptr;       // [my block]
    int32_t* wire = nullptr;    // device [kmax]
    int32_t* wire_h = nullptr;  // pinned [kmax]
  };
  SendSlot& slot(int32_t round);
  SendSlot new_slot();
  bool staging_on_ = false;
  // Fault injection for the race checker's own test (AKKA_FAULT_SKIP_OUTPUT_WAIT=1):
  // counts upload / finalize skip the wait for the caller's hand-over point,
  // i.e. the round-2 counts-fill race comes back.
  bool fault_skip_output_wait_ = false;
  const uint32_t* poison_flag_ = nullptr;
  int32_t max_slots_ = 0;
  std::vector<SendSlot> slots_;
  std::map<int32_t, size_t> slot_of_;
  std::vector<int32_t*> retired_pinned_;
  void* land_ring_ = nullptr;  // [L][S]
  std::function<bool(int32_t)> reclaim_;
};

}  // namespace akka
