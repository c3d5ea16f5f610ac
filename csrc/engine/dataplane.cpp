#include "dataplane.h"

#include <cstdlib>

#include <algorithm>

namespace akka {

namespace {
constexpr size_t kEventPool = 4096;
}

DataPlane::DataPlane(Device* dev, const Geometry& g, int32_t me, int32_t ring_rows, DType dt)
    : dev_(dev), g_(g), me_(me), L_(ring_rows), dt_(dt) {
  AKKA_CHECK(me >= 0 && me < g.N, "worker id out of range");
  AKKA_CHECK(ring_rows >= 1, "ring must have at least one row");
  if (const char* f = std::getenv("AKKA_FAULT_SKIP_OUTPUT_WAIT")) fault_skip_output_wait_ = *f && *f != '0';
  kme_ = g_.num_chunks(me_);
  kmax_ = std::max(1, g_.max_block_len_chunks());
  my_len_ = g_.block_len(me_);
  // 16-B vector loads need every pointer of a chunk reduce to share one
  // alignment: slot data starts at the same offset mod 16 B as my block does
  // in the caller's tensors (block_start * esize), and slot / row strides are
  // multiples of 16 B (kernels.hip peels the common misaligned head).
  const int64_t vec_el = int64_t(16 / esize());
  mis_el_ = g_.block_start(me_) % vec_el;
  slot_stride_ = (std::max<int64_t>(my_len_, 1) + mis_el_ + vec_el - 1) / vec_el * vec_el;
  row_stride_ = (std::max<int64_t>(g_.S, 1) + vec_el - 1) / vec_el * vec_el;
  size_t ring_bytes = size_t(L_) * size_t(g_.N) * size_t(slot_stride_) * esize();
  scatter_ring_ = dev_->alloc(ring_bytes);
  staging_ = static_cast<int32_t*>(dev_->alloc_pinned(size_t(L_) * g_.N * kmax_ * sizeof(int32_t)));
  std::memset(staging_, 0, size_t(L_) * g_.N * kmax_ * sizeof(int32_t));
  rows_.resize(L_);
  for (auto& r : rows_) {
    r.self_alias.assign(std::max(kme_, 1), 0);
    r.released = dev_->create_event();
    r.staging_done = dev_->create_event();
    events_.push_back(r.released);
    events_.push_back(r.staging_done);
  }
}

DataPlane::~DataPlane() {
  try {
    dev_->sync_stream(dev_->compute_stream());
    dev_->sync_stream(dev_->comm_stream());
  } catch (...) {
  }
  for (EventH e : events_) dev_->destroy_event(e);  // includes every binding/spare event
  dev_->release(scatter_ring_);
  dev_->release_pinned(staging_);
  for (auto& sl : slots_) {
    dev_->release(sl.input);
    dev_->release(sl.mine);
    dev_->release(sl.wire);
    dev_->release_pinned(sl.wire_h);
  }
  for (int32_t* p : retired_pinned_) dev_->release_pinned(p);
  if (land_ring_) dev_->release(land_ring_);
}

void DataPlane::enable_staging(int32_t max_slots, std::function<bool(int32_t)> reclaim) {
  AKKA_CHECK(!staging_on_, "staging already enabled");
  AKKA_CHECK(max_slots >= L_ + 1, "send slot pool must exceed the ring depth");
  land_ring_ = dev_->alloc(size_t(L_) * size_t(row_stride_) * esize());
  max_slots_ = max_slots;
  reclaim_ = std::move(reclaim);
  staging_on_ = true;
  // Preallocate the whole pool when it is small (<= 8 GiB): growing it while a
  // peer lags would put hipMalloc/hipHostMalloc on the fast ranks' round path.
  const size_t slot_bytes = (size_t(std::max<int64_t>(g_.S, 1)) + size_t(slot_stride_)) * esize();
  const int32_t pre = slot_bytes * size_t(max_slots) <= (size_t(8) << 30) ? max_slots : L_ + 2;
  for (int32_t i = 0; i < pre; ++i) slots_.push_back(new_slot());
}

DataPlane::SendSlot DataPlane::new_slot() {
  SendSlot s;
  s.input = dev_->alloc(size_t(std::max<int64_t>(g_.S, 1)) * esize());
  s.mine = dev_->alloc(size_t(slot_stride_) * esize());
  s.wire = static_cast<int32_t*>(dev_->alloc(size_t(kmax_) * sizeof(int32_t)));
  s.wire_h = static_cast<int32_t*>(dev_->alloc_pinned(size_t(kmax_) * sizeof(int32_t)));
  return s;
}

int32_t DataPlane::slots_busy() const { return int32_t(slot_of_.size()); }

DataPlane::SendSlot& DataPlane::slot(int32_t round) {
  AKKA_CHECK(staging_on_, "send slots need staged mode");
  auto it = slot_of_.find(round);
  if (it != slot_of_.end()) return slots_[it->second];
  size_t idx = slots_.size();
  for (size_t i = 0; i < slots_.size(); ++i)
    if (slots_[i].round < 0) {
      idx = i;
      break;
    }
  if (idx == slots_.size()) {
    if (int32_t(slots_.size()) < max_slots_) {
      slots_.push_back(new_slot());
    } else {
      // Pool exhausted (a peer is far behind): reclaim the oldest slot whose
      // round is over by making the compute stream wait for its transfers.
      int32_t victim = -1;
      for (auto& kv : slot_of_) {
        const Binding* b = nullptr;
        auto bi = bind_.find(kv.first);
        if (bi != bind_.end()) b = &bi->second;
        if (kv.first < round && (!b || b->finalized) && reclaim_(kv.first)) {
          victim = kv.first;
          break;
        }
      }
      AKKA_CHECK(victim >= 0, "send slot pool exhausted with no finished round to reclaim");
      idx = slot_of_[victim];
      slot_of_.erase(victim);
      // Its wire upload may not have executed yet: never rewrite that pinned row.
      retired_pinned_.push_back(slots_[idx].wire_h);
      slots_[idx].wire_h = static_cast<int32_t*>(dev_->alloc_pinned(size_t(kmax_) * sizeof(int32_t)));
    }
  }
  SendSlot& s = slots_[idx];
  s.round = round;
  slot_of_[round] = idx;
  return s;
}

void DataPlane::release_slot(int32_t round) {
  auto it = slot_of_.find(round);
  if (it == slot_of_.end()) return;
  slots_[it->second].round = -1;
  slot_of_.erase(it);
}

const void* DataPlane::staged_input(int32_t round, int32_t block) {
  return static_cast<const char*>(slot(round).input) + size_t(g_.block_start(block)) * esize();
}

void* DataPlane::mine_at(int32_t round, int32_t k) {
  return static_cast<char*>(slot(round).mine) + (size_t(mis_el_) + size_t(k) * size_t(g_.C)) * esize();
}

int32_t* DataPlane::wire_dev(int32_t round) { return slot(round).wire; }
int32_t* DataPlane::wire_host(int32_t round) { return slot(round).wire_h; }

void* DataPlane::landing_at(int32_t round, int32_t block, int32_t k) const {
  AKKA_CHECK(staging_on_, "landing_at: staging is off");
  size_t off = size_t(round % L_) * size_t(row_stride_) + size_t(g_.chunk_offset(block, k));
  return static_cast<char*>(land_ring_) + off * esize();
}

EventH DataPlane::pooled_event() {
  // Circular pool: link/step events are waited on right after being recorded,
  // and the host never runs more than ring_rows rounds ahead, so reuse after
  // kEventPool records is safe.
  if (events_.size() < kEventPool + 2 * rows_.size()) {
    EventH e = dev_->create_event();
    events_.push_back(e);
    free_events_.push_back(e);
    return e;
  }
  EventH e = free_events_.front();
  std::rotate(free_events_.begin(), free_events_.begin() + 1, free_events_.end());
  return e;
}

EventH DataPlane::record_compute() {
  EventH e = pooled_event();
  dev_->record(e, dev_->compute_stream());
  return e;
}
EventH DataPlane::record_comm() {
  EventH e = pooled_event();
  dev_->record(e, dev_->comm_stream());
  return e;
}

DataPlane::Row& DataPlane::row_for(int32_t round) {
  AKKA_CHECK(round >= 0, "negative round");
  Row& r = rows_[size_t(round % L_)];
  if (r.round != round) {
    AKKA_CHECK(r.round < round, "ring row reused by an older round");
    // The previous occupant's counts upload reads this row's staging area.
    if (r.round >= 0) dev_->sync_event(r.staging_done);
    std::fill(r.self_alias.begin(), r.self_alias.end(), 0);
    std::memset(staging_ + size_t(round % L_) * g_.N * kmax_, 0, size_t(g_.N) * kmax_ * sizeof(int32_t));
    r.round = round;
  }
  return r;
}

EventH DataPlane::row_release_event(int32_t round) {
  // Recorded on demand (not after every reduce, which would split the merged
  // reduce launches): everything issued on the compute stream so far, which
  // includes every reduce that read this ring row for an older round.
  Row& r = rows_[size_t(round % L_)];
  dev_->record(r.released, dev_->compute_stream());
  return r.released;
}

const DataPlane::Binding& DataPlane::binding(int32_t round) const {
  auto it = bind_.find(round);
  AKKA_CHECK(it != bind_.end(), "round " + std::to_string(round) + " has no bound buffers");
  return it->second;
}
DataPlane::Binding& DataPlane::binding_mut(int32_t round) {
  return const_cast<Binding&>(static_cast<const DataPlane*>(this)->binding(round));
}

void DataPlane::bind_input(int32_t round, const void* input, StreamH ready_stream, bool has_stream, bool defer_record) {
  Binding& b = bind_[round];
  b.input = input;
  b.input_pending = false;
  b.input_idle = false;
  b.ready = ready_stream;
  b.has_ready = has_stream && (!dev_->is_host() || dev_->models_streams());
  b.input_waited_compute = b.input_waited_comm = false;
  if (staging_on_) {
    // Stage the input on the compute stream; afterwards nothing reads the
    // caller's tensor, so every consumer is ordered by the compute stream.
    const StreamH cs = dev_->compute_stream();
    if (has_stream && (!dev_->is_host() || dev_->models_streams())) {
      if (!b.input_ready) b.input_ready = binding_event();
      dev_->record(b.input_ready, ready_stream);
      dev_->wait(cs, b.input_ready);
    }
    void* dst = const_cast<void*>(staged_input(round, 0));
    // HostToDevice on the host device: the simulator snapshots the source at
    // issue, like a stream-ordered copy whose source the caller may then free.
    dev_->copy(cs, dst, input, size_t(g_.S) * esize(),
               dev_->is_host() ? CopyKind::HostToDevice : CopyKind::DeviceToDevice);
    b.input = dst;
    b.input_waited_compute = b.input_waited_comm = true;
    return;
  }
  if (has_stream && (!dev_->is_host() || dev_->models_streams())) {
    if (g_.N == 1) {
      // A purely local round (no peers, no comm stream) runs its reduce on the
      // producer's own stream: no cross-stream event hop per round.
      b.exec = ready_stream;
      b.exec_on_producer = true;
      return;
    }
    if (!b.input_ready) b.input_ready = binding_event();
    if (defer_record) b.input_pending = true;  // recorded by the first wait_input, if any
    // an async call on an idle stream: everything that wrote the input (or
    // last used the output / counts memory) has completed -- no marker on the
    // caller's stream, no barrier on the engine's (back-to-back async rounds)
    else if (dev_->stream_idle(ready_stream)) b.input_idle = true;
    else dev_->record(b.input_ready, ready_stream);
  }
}

StreamH DataPlane::exec_stream(int32_t round) const {
  auto it = bind_.find(round);
  if (it != bind_.end() && it->second.exec_on_producer) return it->second.exec;
  if (it != bind_.end() && it->second.exec_on_comm) return dev_->comm_stream();
  return dev_->compute_stream();
}

void DataPlane::set_exec_comm(int32_t round) {
  Binding& b = binding_mut(round);
  if (!b.exec_on_producer) b.exec_on_comm = true;
}

void DataPlane::set_counts_by_lane(int32_t round) { binding_mut(round).counts_by_lane = true; }

void DataPlane::set_caller_waits(int32_t round) { binding_mut(round).caller_waits = true; }

bool DataPlane::caller_waits(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.caller_waits && it->second.has_ready && !staging_on_;
}

StreamH DataPlane::run_on_caller(int32_t round) {
  Binding& b = binding_mut(round);
  AKKA_CHECK(b.caller_waits && b.has_ready, "run_on_caller: the round has no waiting caller stream");
  b.exec = b.ready;
  b.exec_on_producer = true;
  b.exec_on_comm = false;
  b.input_pending = false;  // the round runs in the producer's order: nothing waits for the input event
  return b.exec;
}

bool DataPlane::exec_on_comm(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.exec_on_comm;
}

bool DataPlane::exec_on_producer(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.exec_on_producer;
}

EventH DataPlane::binding_event() {
  // Per-round events are recycled: once a round is unbound nobody waits on
  // its input/done events again, so re-recording them later is safe.
  if (!spare_events_.empty()) {
    EventH e = spare_events_.back();
    spare_events_.pop_back();
    return e;
  }
  EventH e = dev_->create_event();
  events_.push_back(e);
  return e;
}

void DataPlane::bind_output(int32_t round, void* output, int32_t* counts, StreamH alloc_stream, bool has_stream) {
  Binding& b = bind_[round];
  b.output = output;
  b.counts = counts;
  if (has_stream && (!dev_->is_host() || dev_->models_streams()) && g_.N > 1) {  // N == 1: everything runs on the producer stream
    if (!b.output_ready) b.output_ready = binding_event();
    dev_->record(b.output_ready, alloc_stream);
    b.output_waited_compute = b.output_waited_comm = false;
  }
  if (!b.done) b.done = binding_event();
  b.finalized = false;
  // (exec_on_comm may already be set: bulk rounds bind their output lazily,
  // after the link chose the comm stream; a fresh round's binding starts clear)
  b.counts_poisoned = false;
}

bool DataPlane::has_input(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.input != nullptr;
}
bool DataPlane::has_counts(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.counts != nullptr;
}

bool DataPlane::has_output(int32_t round) const {
  auto it = bind_.find(round);
  return it != bind_.end() && it->second.output != nullptr;
}

void DataPlane::unbind(int32_t round) {
  auto it = bind_.find(round);
  if (it == bind_.end()) return;
  if (it->second.input_ready) spare_events_.push_back(it->second.input_ready);
  if (it->second.output_ready) spare_events_.push_back(it->second.output_ready);
  if (it->second.done) spare_events_.push_back(it->second.done);
  bind_.erase(it);
}

void DataPlane::wait_input(int32_t round, StreamH s) {
  // Each consumer stream waits for the input's producer once per round, and
  // only if it actually reads the input (N=1 never touches the comm stream).
  Binding& b = binding_mut(round);
  const bool comm = s == dev_->comm_stream();
  // fault injection (AKKA_FAULT_SKIP_OUTPUT_WAIT): the stream that fills an
  // exact round's counts (the comm stream since round 5) skips the caller's
  // hand-over point -- the round-2 counts-fill race, re-created for the checker
  if (b.output_ready && !(fault_skip_output_wait_ && comm && b.exec_on_comm)) {
    bool& od = comm ? b.output_waited_comm : b.output_waited_compute;
    if (!od) {
      dev_->wait(s, b.output_ready);
      od = true;
    }
  }
  if (!b.input_ready || b.input_idle) return;
  if (b.input_pending) {
    dev_->record(b.input_ready, b.ready);
    b.input_pending = false;
  }
  bool& done = comm ? b.input_waited_comm : b.input_waited_compute;
  if (done) return;
  dev_->wait(s, b.input_ready);
  done = true;
}

void DataPlane::mark_comm_used(int32_t round) { binding_mut(round).comm_used = true; }

Payload DataPlane::input_chunk(int32_t round, int32_t block, int32_t k) const {
  const Binding& b = binding(round);
  AKKA_CHECK(b.input, "round " + std::to_string(round) + " has no input");
  Payload p;
  p.ptr = static_cast<const char*>(b.input) + size_t(g_.chunk_offset(block, k)) * esize();
  p.len = g_.chunk_len(block, k);
  p.kind = PayloadKind::InputView;
  p.on_host = dev_->is_host();
  return p;
}

Payload DataPlane::output_chunk(int32_t round, int32_t block, int32_t k) const {
  Payload p;
  p.ptr = !staging_on_ ? output_at(round, block, k)
          : block == me_ ? const_cast<DataPlane*>(this)->mine_at(round, k) : landing_at(round, block, k);
  p.len = g_.chunk_len(block, k);
  p.kind = PayloadKind::ReducedView;
  p.on_host = dev_->is_host();
  return p;
}

void* DataPlane::scatter_slot(int32_t round, int32_t src, int32_t k) const {
  size_t row = size_t(round % L_);
  size_t off = (row * size_t(g_.N) + size_t(src)) * size_t(slot_stride_) + size_t(mis_el_) + size_t(k) * size_t(g_.C);
  return static_cast<char*>(scatter_ring_) + off * esize();
}

void* DataPlane::output_at(int32_t round, int32_t block, int32_t k) const {
  const Binding& b = binding(round);
  AKKA_CHECK(b.output, "round " + std::to_string(round) + " has no output buffer");
  return static_cast<char*>(b.output) + size_t(g_.chunk_offset(block, k)) * esize();
}

int32_t* DataPlane::counts_row(int32_t round, int32_t block) const {
  const Binding& b = binding(round);
  AKKA_CHECK(b.counts, "round has no counts buffer");
  return b.counts + size_t(block) * kmax_;
}

void DataPlane::store_scatter(int32_t round, int32_t src, int32_t k, const Payload& p) {
  AKKA_CHECK(k >= 0 && k < kme_, "scatter chunk id out of range");
  int64_t want = g_.chunk_len(me_, k);
  // AllReduceBuffer.store throws ArrayIndexOutOfBounds past the block end
  // (AB:27-30, tested by SBS:32-42); a short payload is a silent partial store.
  AKKA_CHECK(p.len <= want, "scatter payload of " + std::to_string(p.len) + " elements overruns chunk " +
                                std::to_string(k) + " (" + std::to_string(want) + " elements)");
  Row& r = row_for(round);
  if (src == me_ && p.kind == PayloadKind::InputView) {
    r.self_alias[size_t(k)] = 1;
    return;
  }
  if (src == me_) r.self_alias[size_t(k)] = 0;
  if (p.kind == PayloadKind::Landed) return;
  void* dst = scatter_slot(round, src, k);
  CopyKind ck = p.on_host ? CopyKind::HostToDevice : CopyKind::DeviceToDevice;
  dev_->copy(exec_stream(round), dst, p.ptr, size_t(p.len) * esize(), ck);
}

Payload DataPlane::reduce(int32_t round, int32_t k, const std::vector<int32_t>& srcs) {
  AKKA_CHECK(k >= 0 && k < kme_, "reduce chunk id out of range");
  Row& r = row_for(round);
  Binding& b = binding_mut(round);
  int64_t n = g_.chunk_len(me_, k);
  void* dst = staging_on_ ? mine_at(round, k) : output_at(round, me_, k);
  std::vector<const void*> ptrs;
  ptrs.reserve(srcs.size());
  const StreamH cs = exec_stream(round);
  for (int32_t s : srcs) {
    if (s == me_ && r.self_alias[size_t(k)]) {
      wait_input(round, cs);
      ptrs.push_back(static_cast<const char*>(b.input) + size_t(g_.chunk_offset(me_, k)) * esize());
    } else {
      ptrs.push_back(scatter_slot(round, s, k));
    }
  }
  if (ptrs.empty()) {
    dev_->zero(cs, dst, size_t(n) * esize());
  } else {
    auto specs = split_reduce(dst, ptrs, n);
    dev_->reduce(cs, specs.data(), int32_t(specs.size()), dt_);
  }
  return output_chunk(round, me_, k);
}

void DataPlane::store_reduced(int32_t round, int32_t src, int32_t k, const Payload& p) {
  AKKA_CHECK(src >= 0 && src < g_.N, "reduced block src out of range");
  AKKA_CHECK(k >= 0 && k < g_.num_chunks(src), "reduced chunk id out of range");
  int64_t want = g_.chunk_len(src, k);
  AKKA_CHECK(p.len <= want, "reduced payload overruns chunk");
  if (p.kind == PayloadKind::Landed) return;
  void* dst = !staging_on_ ? output_at(round, src, k) : src == me_ ? mine_at(round, k) : landing_at(round, src, k);
  if (p.ptr == dst) return;
  CopyKind ck = p.on_host ? CopyKind::HostToDevice : CopyKind::DeviceToDevice;
  dev_->copy(exec_stream(round), dst, p.ptr, size_t(p.len) * esize(), ck);
}

void DataPlane::set_count(int32_t round, int32_t block, int32_t k, int32_t count) {
  row_for(round);
  staging_[(size_t(round % L_) * g_.N + size_t(block)) * kmax_ + size_t(k)] = count;
}

void DataPlane::upload_counts(int32_t round, const std::vector<int32_t>& blocks, StreamH s) {
  Row& r = row_for(round);
  const Binding& b = binding(round);
  if (!b.counts || b.counts_by_lane) return;
  // the counts memory is the caller's: write it only after the point where
  // the caller's stream handed it over (an exact round's compute stream has
  // not waited for anything of the caller's yet)
  if (!b.exec_on_producer && !fault_skip_output_wait_) wait_input(round, s);
  bool copied = false;
  if (int32_t(blocks.size()) == g_.N && g_.N > 1) {
    // every block, one value everywhere (exact rounds: all N): ONE 32-bit
    // fill of the whole [N][kmax] table instead of a fill per block (each a
    // separate ~5 us launch on the compute stream, seen in the N=8 trace);
    // entries past a block's last chunk are never read
    const int32_t* row = staging_ + size_t(round % L_) * g_.N * kmax_;
    const int32_t v = row[0];
    bool same = true;
    for (int32_t j = 0; j < g_.N && same; ++j)
      for (int32_t k = 0; k < g_.num_chunks(j) && same; ++k) same = row[size_t(j) * kmax_ + k] == v;
    if (same) {
      if (poison_flag_ && b.exec_on_comm && s == dev_->comm_stream()) {
        // the lane's error word decides the value when the stream gets there
        // (v, or 0 after a failed wait): fill + poison in one launch, in the
        // order of the stream that ran the lane's kernels
        dev_->fill_counts_unless(s, poison_flag_, b.counts, v, size_t(g_.N) * kmax_);
        binding_mut(round).counts_poisoned = true;
      } else {
        dev_->fill_i32(s, b.counts, v, size_t(g_.N) * kmax_);
      }
      if (s == dev_->comm_stream()) binding_mut(round).comm_used = true;
      return;
    }
  }
  for (int32_t blk : blocks) {
    const int32_t* src = staging_ + (size_t(round % L_) * g_.N + size_t(blk)) * kmax_;
    const int32_t kb = std::max(1, g_.num_chunks(blk));
    bool uniform = true;
    for (int32_t k = 1; k < kb && uniform; ++k) uniform = src[k] == src[0];
    if (uniform) {
      // exact thresholds: every chunk has the same count -> a 32-bit fill,
      // no host staging read on the stream
      dev_->fill_i32(s, b.counts + size_t(blk) * kmax_, src[0], size_t(kb));
    } else {
      dev_->copy(s, b.counts + size_t(blk) * kmax_, src, size_t(kmax_) * sizeof(int32_t), CopyKind::HostToDevice);
      copied = true;
    }
  }
  if (s == dev_->comm_stream()) binding_mut(round).comm_used = true;
  if (copied) dev_->record(r.staging_done, s);
}

void DataPlane::finalize(int32_t round, const std::vector<uint8_t>& landed) {
  Binding& b = binding_mut(round);
  AKKA_CHECK(landed.size() == size_t(g_.N) * kmax_, "landed mask has wrong shape");
  const StreamH cs = exec_stream(round);
  // cs writes the caller's output/counts below
  if (!b.exec_on_producer && !fault_skip_output_wait_) wait_input(round, cs);
  // Join: everything the comm stream wrote into this round's output (a round
  // executing on the comm stream is already in its order).
  if (b.comm_used && !b.exec_on_comm) {
    EventH ce = record_comm();
    dev_->wait(cs, ce);
  }
  if (staging_on_) {
    // Copy landed chunks (landing row / my send slot) -> output, coalescing
    // runs of consecutive landed chunks within a block.
    int64_t run0 = -1, run1 = -1;
    const char* base = nullptr;  // source address of element run0
    auto flush = [&]() {
      if (run0 < 0) return;
      dev_->copy(cs, static_cast<char*>(b.output) + size_t(run0) * esize(), base, size_t(run1 - run0) * esize(),
                 dev_->is_host() ? CopyKind::HostToHost : CopyKind::DeviceToDevice);
      run0 = run1 = -1;
    };
    for (int32_t j = 0; j < g_.N; ++j, flush())
      for (int32_t k = 0; k < g_.num_chunks(j); ++k) {
        if (!landed[size_t(j) * kmax_ + k]) {
          flush();
          continue;
        }
        int64_t o = g_.chunk_offset(j, k), e = o + g_.chunk_len(j, k);
        if (run0 >= 0 && run1 == o) run1 = e;
        else {
          flush();
          run0 = o;
          run1 = e;
          base = static_cast<const char*>(j == me_ ? mine_at(round, k) : landing_at(round, j, k));
        }
      }
    flush();
  }
  for (int32_t j = 0; j < g_.N; ++j) {
    int32_t kj = g_.num_chunks(j);
    int32_t k = 0;
    while (k < kj) {
      if (landed[size_t(j) * kmax_ + k]) {
        ++k;
        continue;
      }
      int32_t k0 = k;
      while (k < kj && !landed[size_t(j) * kmax_ + k]) ++k;
      // Missing reduced chunks read as 0 with count 0 (RB:41-47, RBS:95-119).
      int64_t off = g_.chunk_offset(j, k0);
      int64_t end = g_.chunk_offset(j, k - 1) + g_.chunk_len(j, k - 1);
      dev_->zero(cs, static_cast<char*>(b.output) + size_t(off) * esize(), size_t(end - off) * esize());
      if (b.counts) dev_->zero(cs, b.counts + size_t(j) * kmax_ + k0, size_t(k - k0) * sizeof(int32_t));
    }
  }
  // a round of a lane that failed (a wait timed out / the lane was aborted)
  // never comes back as exact: its counts read 0 everywhere
  if (poison_flag_ && b.counts && !b.counts_poisoned && !b.counts_by_lane)
    dev_->poison_counts_if(cs, poison_flag_, b.counts, size_t(g_.N) * kmax_);
  if (b.exec_on_producer) {
    dev_->flush(cs);  // the round's launch must not wait for the next round to merge into
    b.done_lazy = true;
  } else {
    dev_->record(b.done, cs);
    // async callers record their event on the compute stream (worker.py
    // _deliver / the DDP hook's async_stream): it follows the comm stream's
    // done point -- off the comm stream's path, which never waits for it
    if (b.exec_on_comm) dev_->wait(dev_->compute_stream(), b.done);
  }
  b.finalized = true;
}

EventH DataPlane::done_event(Binding& b) {
  if (b.done_lazy) {
    dev_->record(b.done, b.exec);
    b.done_lazy = false;
  }
  return b.done;
}

void DataPlane::stream_wait_done(int32_t round, StreamH stream) {
  Binding& b = binding_mut(round);
  AKKA_CHECK(b.finalized, "round not finalized");
  if (b.exec_on_producer && stream == b.exec) return;  // already in that stream's order
  dev_->wait(stream, done_event(b));
}

void DataPlane::sync_done(int32_t round) {
  Binding& b = binding_mut(round);
  AKKA_CHECK(b.finalized, "round not finalized");
  dev_->sync_event(done_event(b));
}

void DataPlane::read_payload(const Payload& p, void* host_dst) const {
  if (p.len == 0) return;
  size_t bytes = size_t(p.len) * esize();
  if (dev_->is_host() || p.on_host) {
    std::memcpy(host_dst, p.ptr, bytes);
    return;
  }
  // Device view: the producing op is on the compute stream (reduce) or the
  // input's producer (already waited for by input_chunk).
  dev_->sync_stream(dev_->compute_stream());
  dev_->copy(dev_->compute_stream(), host_dst, p.ptr, bytes, CopyKind::DeviceToHost);
  dev_->sync_stream(dev_->compute_stream());
}

}  // namespace akka
