// pybind11 module `akka_allreduce_amd._native`.
//
// Exposes one worker core (engine + data plane + link) per rank, the kernels
// (for tests/bench), RCCL bootstrap helpers and the CPU p2p simulator.
// Python owns all round memory (torch tensors) and passes raw pointers +
// stream handles; nothing here depends on libtorch, so the module builds with
// plain hipcc in seconds and loads on CPU-only machines.
#include <hip/hip_runtime.h>
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <set>

#include "../engine/engine.h"
#include "../kernels/kernels.h"
#include "../runtime/frames.h"
#include "../runtime/watchdog.h"
#include "../transport/ipc_p2p.h"
#include "../transport/p2p.h"
#include "../transport/reactive_link.h"
#include "harness_p2p.h"
#include "../transport/stream_link.h"

namespace py = pybind11;
using namespace akka;

namespace akka {
bool host_device_step(Device* d, uint32_t rotate);  // host_device.cpp
void bind_onesided(py::module_& m);                 // bind_onesided.cpp
void bind_probe(py::module_& m);                    // bind_probe.cpp
}

namespace {

struct PySimHub {
  std::shared_ptr<SimHub> hub;
};

struct OutMsg {
  int32_t kind;  // 1 scatter, 2 reduce
  int32_t src, dest, chunk, round, count;
  std::string data;  // the payload's bytes (py::bytes on access)
};

class OutboxLink final : public Link {
 public:
  explicit OutboxLink(int32_t me) : me_(me) {}
  void bind(DataPlane* dp) { dp_ = dp; }
  void send_scatter(int32_t dest, int32_t chunk, int32_t round, const Payload& p) override {
    box_.push_back(make(1, dest, chunk, round, 0, p));
  }
  void send_reduce(int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) override {
    box_.push_back(make(2, dest, chunk, round, count, p));
  }
  std::vector<OutMsg> drain() {
    std::vector<OutMsg> out;
    out.swap(box_);
    return out;
  }
  size_t size() const { return box_.size(); }

 private:
  OutMsg make(int32_t kind, int32_t dest, int32_t chunk, int32_t round, int32_t count, const Payload& p) {
    if (p.kind == PayloadKind::InputView) dp_->wait_input(round, dp_->device()->compute_stream());
    std::string buf(size_t(p.len) * dp_->esize(), '\0');
    dp_->read_payload(p, buf.data());
    return OutMsg{kind, me_, dest, chunk, round, count, std::move(buf)};
  }
  int32_t me_;
  DataPlane* dp_ = nullptr;
  std::vector<OutMsg> box_;
};

class WorkerCore final : public EngineHost {
 public:
  WorkerCore(py::object host, std::string link, int32_t device, std::string dtype, bool deferred, int32_t lag)
      : host_(std::move(host)), link_kind_(std::move(link)), device_idx_(device), deferred_(deferred), lag_(lag) {
    if (dtype == "float32" || dtype == "f32" || dtype == "fp32") dt_ = DType::F32;
    else if (dtype == "bfloat16" || dtype == "bf16") dt_ = DType::BF16;
    else throw AkkaError("akka: unsupported dtype " + dtype);
    AKKA_CHECK(link_kind_ == "outbox" || link_kind_ == "stream" || link_kind_ == "reactive",
               "link must be 'outbox', 'stream' or 'reactive'");
    engine_ = std::make_unique<Engine>(this, nullptr);
  }
  ~WorkerCore() override {
    // Order: link and data plane reference the device and the engine.
    stream_link_.reset();
    reactive_link_.reset();
    dp_.reset();
    p2p_.reset();  // (a shared transport lives on in the engines that still hold it)
    adopted_p2p_.reset();
    dev_.reset();
  }

  // ---- control -------------------------------------------------------------
  bool init(int32_t id, int32_t n, float th_reduce, float th_complete, int32_t max_lag, int64_t data_size,
            int64_t max_chunk, std::vector<std::pair<int32_t, bool>> peers) {
    InitParams p;
    p.id = id;
    p.worker_num = n;
    p.th_reduce = th_reduce;
    p.th_complete = th_complete;
    p.max_lag = max_lag;
    p.data_size = data_size;
    p.max_chunk_size = max_chunk;
    std::vector<PeerEntry> pe;
    for (auto& kv : peers) pe.push_back({kv.first, kv.second});
    bool first = engine_->init(p, pe);
    if (!first) return false;
    if (!dev_) {  // (adopt_transport may have handed us a shared device)
      if (device_idx_ < 0) dev_ = make_host_device(deferred_);
      else {
        // AKKA_COMM_PRIORITY=normal: the comm stream at normal priority
        // (measurement knob: which hardware queue pool the round lands in)
        const char* pr = std::getenv("AKKA_COMM_PRIORITY");
        dev_ = make_hip_device(device_idx_, !(pr && std::strcmp(pr, "normal") == 0));
      }
    }
    dp_ = std::make_unique<DataPlane>(dev_.get(), engine_->geometry(), id, max_lag + 1, dt_);
    if (link_kind_ == "outbox") {
      outbox_ = std::make_unique<OutboxLink>(id);
      outbox_->bind(dp_.get());
      engine_->set_link(outbox_.get());
    }
    return true;
  }
  // Must be called after init for link == "stream", before attach.
  void connect_rccl(py::bytes uid, int32_t rank, int32_t nranks, std::vector<int32_t> members) {
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    AKKA_CHECK(dev_ && !dev_->is_host(), "RCCL transport needs a HIP device");
    if (link_kind_ == "reactive") {
      AKKA_CHECK(members.empty() || int32_t(members.size()) == nranks,
                 "the reactive transport's pair communicators are built over all workers");
      p2p_ = make_rccl_pair_p2p(v, rank, nranks, device_idx_);
      make_reactive_link();
      return;
    }
    p2p_ = make_rccl_p2p(v, rank, nranks, device_idx_, members);
    make_stream_link();
  }
  // Membership epoch from a re-InitWorkers (new unique id + member list).
  bool rebuild_transport(py::bytes uid, std::vector<int32_t> members) {
    AKKA_CHECK(p2p_, "rebuild_transport before the transport was connected");
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    py::gil_scoped_release nogil;  // ncclCommInitRank waits for every member
    return p2p_->rebuild(v, members);
  }
  // Host-cost rehearsal of the N-rank schedule on one GPU (rccl_p2p.cpp
  // RcclShapeP2P): the bytes are meaningless, the host path is the real one.
  void connect_rccl_shape(int32_t rank, int32_t nranks) {
    AKKA_CHECK(dev_ && !dev_->is_host(), "RCCL transport needs a HIP device");
    AKKA_CHECK(link_kind_ == "stream", "shape rehearsal runs the scheduled transport");
    p2p_ = make_rccl_shape_p2p(rank, nranks, device_idx_);
    make_stream_link();
  }
  void connect_sim(const PySimHub& hub, int32_t rank) {
    AKKA_CHECK(dev_ && dev_->is_host() && deferred_, "sim transport needs a deferred host device");
    p2p_ = make_sim_p2p(hub.hub, rank, dev_.get());
    if (link_kind_ == "reactive") make_reactive_link();
    else make_stream_link();
  }
  void connect_callback(py::function fn, int32_t rank, int32_t nranks) {
    AKKA_CHECK(dev_ && dev_->is_host() && !deferred_, "callback p2p runs on an immediate host device");
    p2p_ = std::make_unique<PyCallbackP2P>(std::move(fn), rank, nranks, dev_.get());
    make_stream_link();
  }
  void connect_loopback(const PyLoopbackHub& hub, int32_t rank) {
    AKKA_CHECK(dev_ && !dev_->is_host(), "loopback p2p needs a HIP device");
    p2p_ = std::make_unique<LoopbackP2P>(hub.hub, rank);
    make_stream_link();
  }
  void connect_loopback_pair(const PyPairHub& hub, int32_t rank) {
    AKKA_CHECK(dev_ && !dev_->is_host(), "pair loopback p2p needs a HIP device");
    AKKA_CHECK(link_kind_ == "reactive", "pair loopback serves the reactive link");
    p2p_ = std::make_unique<LoopbackPairP2P>(hub.hub, rank);
    make_reactive_link();
  }
  void connect_async_callback(py::function post, py::function test, int32_t rank, int32_t nranks) {
    AKKA_CHECK(dev_ && dev_->is_host() && deferred_, "async callback p2p runs on a deferred host device");
    AKKA_CHECK(link_kind_ == "reactive", "async callback p2p serves the reactive link");
    p2p_ = std::make_unique<PyAsyncCallbackP2P>(std::move(post), std::move(test), rank, nranks, dev_.get());
    self_drive_ = true;
    make_reactive_link();
  }
  // Grouped send/recv over mapped peer memory instead of RCCL (ipc_p2p.cpp);
  // then p2p_handle() to every rank and p2p_open(all handles).
  void connect_ipc_p2p(int32_t rank, int32_t nranks) {
    AKKA_CHECK(dev_ && !dev_->is_host(), "ipc p2p needs a HIP device");
    p2p_ = make_ipc_p2p(rank, nranks, device_idx_);
    if (link_kind_ == "reactive") make_reactive_link();
    else make_stream_link();
  }
  py::bytes p2p_handle() {
    AKKA_CHECK(p2p_, "p2p_handle: no transport");
    return py::bytes(p2p_->handle());
  }
  void p2p_open(std::vector<std::string> handles) {
    AKKA_CHECK(p2p_, "p2p_open: no transport");
    py::gil_scoped_release nogil;
    p2p_->open(handles);
  }
  // ipc-only data plane: no two-sided transport; exact rounds on the ipc lane.
  void connect_none(int32_t rank, int32_t nranks) {
    AKKA_CHECK(dev_ && !dev_->is_host(), "the ipc-only data plane needs a HIP device");
    AKKA_CHECK(link_kind_ == "stream", "the ipc lane belongs to the scheduled (stream) transport");
    p2p_ = std::make_unique<NullP2P>(rank, nranks);
    make_stream_link();
  }
  // Several engines of one job (e.g. one per DDP bucket size) share ONE
  // transport: the device (its comm / compute streams) and the P2P object
  // (RCCL communicator, ipc-only null transport, gloo callbacks).  Every
  // engine's rounds are then ordered on the same streams, in the order the
  // caller issues them -- identical on every rank -- which is what RCCL
  // needs of ops sharing a communicator and what lets engines share window
  // memory (IpcLane::share).  Call adopt_transport before init, then
  // connect_adopted instead of a connect_* call.
  void adopt_transport(WorkerCore& other) {
    AKKA_CHECK(!dev_ && !p2p_, "adopt_transport: call it before init");
    AKKA_CHECK(other.dev_ && other.p2p_, "adopt_transport: the other engine has no connected transport");
    AKKA_CHECK(other.link_kind_ == link_kind_ && other.device_idx_ == device_idx_ && other.deferred_ == deferred_,
               "adopt_transport: the engines differ in link kind or device");
    // Only the scheduled link orders every engine's groups on one comm stream
    // in the call order all ranks share.  Reactive links issue their phase-2
    // groups from per-peer streams when chunks become ready (timing-dependent,
    // rank-dependent order): two of them on one pair communicator could match
    // a send of one engine with a receive of the other.
    AKKA_CHECK(link_kind_ == "stream", "adopt_transport: only the scheduled (stream) link can be shared");
    dev_ = other.dev_;
    adopted_p2p_ = other.p2p_;
  }
  void connect_adopted() {
    AKKA_CHECK(adopted_p2p_, "connect_adopted: adopt_transport first");
    AKKA_CHECK(adopted_p2p_->nranks() == engine_->geometry().N && adopted_p2p_->rank() == engine_->id(),
               "connect_adopted: the shared transport was built for another rank / size");
    p2p_ = adopted_p2p_;
    if (link_kind_ == "reactive") make_reactive_link();
    else make_stream_link();
  }
  // Identity of the transport object (engines sharing one report the same).
  uintptr_t transport_id() const { return reinterpret_cast<uintptr_t>(p2p_.get()); }
  // ---- one-sided xGMI lane (ipc_lane.h) ----
  // `capacity`: size the windows for a buffer of that many elements; `share`:
  // an engine on the same (adopted) transport whose open lane's windows this
  // one reuses when they are large enough (IpcLane).
  py::bytes ipc_handle(int64_t capacity, WorkerCore* share) {
    AKKA_CHECK(stream_link_ && dp_, "ipc_handle: scheduled (stream) transport, after init");
    const IpcLane* other = (share && share->stream_link_) ? share->stream_link_->ipc() : nullptr;
    if (!ipc_pending_)
      ipc_pending_ = std::make_unique<IpcLane>(dev_.get(), dp_->geometry(), dp_->me(), dt_, capacity, other);
    return py::bytes(ipc_pending_->handle());
  }
  void ipc_open(std::vector<std::string> handles) {
    AKKA_CHECK(ipc_pending_, "ipc_open: call ipc_handle first");
    {
      py::gil_scoped_release nogil;
      ipc_pending_->open(handles);
    }
    stream_link_->set_ipc(std::move(ipc_pending_));
  }
  uint32_t ipc_error() {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_error: the ipc lane is not open");
    py::gil_scoped_release nogil;
    return stream_link_->ipc()->error();
  }
  void ipc_set_mode(const std::string& mode, bool fused, int32_t threads, int32_t lite) {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_set_mode: the ipc lane is not open");
    AKKA_CHECK(mode == "pull" || mode == "bcast", "ipc mode must be 'pull' or 'bcast'");
    AKKA_CHECK(threads == 0 || threads == 256 || threads == 512 || threads == 1024,
               "ipc workgroup size must be 256, 512 or 1024 (0: keep)");
    stream_link_->ipc()->set_bcast(mode == "bcast");
    stream_link_->ipc()->set_fused(fused);
    if (threads) stream_link_->ipc()->set_threads(threads);
    if (lite >= 0) stream_link_->ipc()->set_lite(lite != 0);
  }
  // Exact ipc round straight on `stream`, none of the engine's round
  // bookkeeping (exact rounds: every count is N) -- the graph-capturable
  // path, with device-resident round ids (ipc_device_rounds(true)).
  // `counts` ([n] int32, optional): the fixed counts table the caller hands
  // out with direct rounds; a failed wait zeroes it on the device.  A wait of
  // an earlier round that failed makes this call raise, like the engine path
  // (StreamLink::ipc_round).
  // `finish`: the round's last workgroup writes `counts` (N everywhere, 0 after
  // a failed wait) like an engine-path round, instead of zeroing it only on
  // failure (measurement knob, bench/small_rounds.py).
  void ipc_round_direct(uintptr_t in, uintptr_t out, uintptr_t stream, uintptr_t counts, int64_t n, bool finish) {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_round_direct: the ipc lane is not open");
    AKKA_CHECK(stream_link_->ipc()->device_rounds(), "ipc_round_direct: switch device rounds on first");
    AKKA_CHECK(stream_link_->ipc()->error_now() == 0,
               "ipc lane: a wait of an earlier round timed out (peer missing?); its rounds are not trustworthy");
    int32_t* c = reinterpret_cast<int32_t*>(counts);
    if (finish && c)
      stream_link_->ipc()->round(reinterpret_cast<StreamH>(stream), reinterpret_cast<const void*>(in),
                                 reinterpret_cast<void*>(out), nullptr, 0, c, n, engine_->geometry().N);
    else
      stream_link_->ipc()->round(reinterpret_cast<StreamH>(stream), reinterpret_cast<const void*>(in),
                                 reinterpret_cast<void*>(out), c, c ? n : 0);
  }
  // The lane's error word as far as the kernels got (no synchronisation).
  uint32_t ipc_error_now() {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_error_now: the ipc lane is not open");
    return stream_link_->ipc()->error_now();
  }
  void ipc_device_rounds(bool on) {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_device_rounds: the ipc lane is not open");
    py::gil_scoped_release nogil;
    stream_link_->ipc()->set_device_rounds(on);
  }
  uint32_t ipc_current_round() {
    AKKA_CHECK(stream_link_ && stream_link_->ipc(), "ipc_current_round: the ipc lane is not open");
    py::gil_scoped_release nogil;
    return stream_link_->ipc()->current_round();
  }
  void ipc_close() {
    ipc_pending_.reset();
    if (stream_link_) stream_link_->set_ipc(nullptr);
  }
  void connect_local() {  // N == 1: stream link without peers
    AKKA_CHECK(engine_->geometry().N == 1, "connect_local is for single-worker jobs");
    make_stream_link(/*any_kind=*/true);
  }
  void attach() {
    AKKA_CHECK(dp_, "attach before init");
    if (link_kind_ == "stream") AKKA_CHECK(stream_link_, "stream link not connected");
    if (link_kind_ == "reactive") AKKA_CHECK(stream_link_ || reactive_link_, "reactive link not connected");
    engine_->attach(dp_.get());
  }

  void start(int32_t r) { engine_->start(r); }
  // Reactive transport: deliver completed transfers to the engine.
  bool poll() {
    if (!reactive_link_) return false;
    if (!self_drive_) return reactive_link_->poll();
    // Host streams driven by this process (async callback p2p): run the
    // stream queues and the link until neither moves.
    bool any = false;
    for (int i = 0; i < 64; ++i) {
      bool moved = host_device_step(dev_.get(), 0);
      moved |= reactive_link_->poll();
      if (!moved) break;
      any = true;
    }
    return any;
  }
  int32_t in_flight() const { return reactive_link_ ? reactive_link_->in_flight() : 0; }
  void wait_activity(int64_t timeout_us) {
    if (!reactive_link_ || self_drive_) return;
    py::gil_scoped_release nogil;
    reactive_link_->wait_activity(timeout_us);
  }
  bool reactive() const { return reactive_link_ != nullptr; }
  void scatter_in(int32_t src, int32_t dest, int32_t chunk, int32_t round, uintptr_t ptr, int64_t len, bool on_host) {
    Payload p{reinterpret_cast<const void*>(ptr), len, PayloadKind::External, on_host};
    engine_->on_scatter(src, dest, chunk, round, p);
  }
  void reduce_in(int32_t src, int32_t dest, int32_t chunk, int32_t round, int32_t count, uintptr_t ptr, int64_t len,
                 bool on_host) {
    Payload p{reinterpret_cast<const void*>(ptr), len, PayloadKind::External, on_host};
    engine_->on_reduce(src, dest, chunk, round, count, p);
  }
  void peer_terminated(int32_t id) { engine_->on_peer_terminated(id); }

  // ---- memory bindings -----------------------------------------------------
  void bind_input(int32_t round, uintptr_t ptr, uintptr_t stream, bool has_stream) {
    dp_->bind_input(round, reinterpret_cast<const void*>(ptr), reinterpret_cast<StreamH>(stream), has_stream);
  }
  void bind_output(int32_t round, uintptr_t out, uintptr_t counts, uintptr_t stream, bool has_stream) {
    dp_->bind_output(round, reinterpret_cast<void*>(out), reinterpret_cast<int32_t*>(counts),
                     reinterpret_cast<StreamH>(stream), has_stream);
  }
  void unbind(int32_t round) { dp_->unbind(round); }

  // ---- stream race checking (host device, AKKA_RACECHECK=1) --------------------
  bool models_streams() const { return dev_ && dev_->models_streams(); }
  uintptr_t create_stream() {
    AKKA_CHECK(dev_, "no device");
    return reinterpret_cast<uintptr_t>(dev_->create_stream());
  }
  // A caller op on `stream` that reads or writes [ptr, ptr + bytes).
  void declare_access(uintptr_t stream, uintptr_t ptr, size_t bytes, bool write, const std::string& tag) {
    AKKA_CHECK(dev_, "no device");
    const char* t = tags_.insert(tag).first->c_str();
    dev_->declare_access(reinterpret_cast<StreamH>(stream), {{reinterpret_cast<const void*>(ptr), bytes, write, t}});
  }
  std::vector<std::string> race_reports() const { return dev_ ? dev_->race_reports() : std::vector<std::string>{}; }
  int64_t race_count() const { return dev_ ? dev_->race_count() : 0; }
  void sync_stream(uintptr_t stream) {
    AKKA_CHECK(dev_, "no device");
    dev_->sync_stream(reinterpret_cast<StreamH>(stream));
  }
  void stream_wait_done(int32_t round, uintptr_t stream) {
    dp_->stream_wait_done(round, reinterpret_cast<StreamH>(stream));
  }
  void sync_done(int32_t round) { dp_->sync_done(round); }
  bool exec_on_producer(int32_t round) const { return dp_->exec_on_producer(round); }
  void sync_all() {
    if (!dev_) return;
    dev_->sync_stream(dev_->compute_stream());
    dev_->sync_stream(dev_->comm_stream());
  }
  void count_mean(uintptr_t dst, uintptr_t src, uintptr_t counts, uintptr_t stream) {
    const Geometry& g = engine_->geometry();
    AKKA_CHECK(dev_ && !dev_->is_host(), "count_mean: device path only");
    launch_count_mean(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<void*>(dst),
                      reinterpret_cast<const void*>(src), reinterpret_cast<const int32_t*>(counts), g.S, g.step, g.N,
                      g.C, dp_->kmax(), dt_);
  }
  void expand_counts(uintptr_t out, uintptr_t counts, uintptr_t stream) {
    const Geometry& g = engine_->geometry();
    AKKA_CHECK(dev_ && !dev_->is_host(), "expand_counts: device path only");
    launch_count_expand(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<int32_t*>(out),
                        reinterpret_cast<const int32_t*>(counts), g.S, g.step, g.N, g.C, dp_->kmax());
  }

  std::pair<uintptr_t, uintptr_t> streams() const {
    AKKA_CHECK(dev_, "streams() before init");
    dev_->mark_streams_exported();
    return {reinterpret_cast<uintptr_t>(dev_->comm_stream()), reinterpret_cast<uintptr_t>(dev_->compute_stream())};
  }
  std::vector<OutMsg> drain() { return outbox_ ? outbox_->drain() : std::vector<OutMsg>{}; }

  // The outbox as wire frames (csrc/runtime/frames.h), one byte string per
  // destination in first-emission order, each destination's messages in
  // emission order (per-pair FIFO): the CPU data plane's sends without a
  // Python message object per chunk.
  std::vector<std::pair<int32_t, py::bytes>> drain_frames() {
    std::vector<std::pair<int32_t, py::bytes>> res;
    if (!outbox_) return res;
    std::vector<OutMsg> msgs = outbox_->drain();
    if (msgs.empty()) return res;
    const char* dt = dt_ == DType::F32 ? "float32" : "bfloat16";
    std::vector<int32_t> order;
    std::map<int32_t, std::string> by;
    for (const OutMsg& m : msgs) {
      auto it = by.find(m.dest);
      if (it == by.end()) {
        order.push_back(m.dest);
        it = by.emplace(m.dest, std::string()).first;
      }
      frames::append_data_frame(it->second, m.kind, m.data.data(), m.data.size(), dt, m.src, m.dest, m.chunk,
                                m.round, m.count);
    }
    for (int32_t d : order) res.emplace_back(d, py::bytes(by[d]));
    return res;
  }

  // One arriving frame BODY, if it is a ScatterBlock / ReduceBlock of this
  // worker's dtype: parsed in place and handed to the engine with a pointer
  // into the frame.  False: anything else (the caller decodes it in Python).
  bool apply_frame(py::bytes body) {
    char* p = nullptr;
    Py_ssize_t n = 0;
    if (PyBytes_AsStringAndSize(body.ptr(), &p, &n) != 0) throw py::error_already_set();
    return apply_frame_raw(p, size_t(n));
  }
  bool apply_frame_raw(const char* p, size_t n) {
    frames::DataFrame f;
    if (!frames::parse_data_frame(p, n, f)) return false;
    const char* dt = dt_ == DType::F32 ? "float32" : "bfloat16";
    const size_t es = dt_ == DType::F32 ? 4 : 2;
    if (f.dtype != dt || f.nbytes % es != 0) return false;
    const Payload pl{f.value, int64_t(f.nbytes / es), PayloadKind::External, true};
    if (f.kind == 1) engine_->on_scatter(int32_t(f.src), int32_t(f.dest), int32_t(f.chunk), int32_t(f.round), pl);
    else engine_->on_reduce(int32_t(f.src), int32_t(f.dest), int32_t(f.chunk), int32_t(f.round), int32_t(f.count), pl);
    return true;
  }
  Device* device() const { return dev_.get(); }

  // ---- introspection -------------------------------------------------------
  py::dict state() const {
    py::dict d;
    d["id"] = engine_->id();
    d["round"] = engine_->round();
    d["max_round"] = engine_->max_round();
    d["max_scattered"] = engine_->max_scattered();
    d["completed"] = engine_->completed();
    d["initialized"] = engine_->initialized();
    std::vector<int32_t> ids;
    for (auto& p : engine_->peers()) ids.push_back(p.id);
    d["peers"] = ids;
    if (engine_->id() >= 0) {
      const Geometry& g = engine_->geometry();
      d["step"] = g.step;
      d["kmax"] = std::max(1, g.max_block_len_chunks());
      d["min_scatter_required"] = engine_->min_scatter_required();
      d["min_reduced_required"] = engine_->min_reduced_required();
      d["ring_rows"] = engine_->params().max_lag + 1;
    }
    const EngineStats& s = engine_->stats();
    py::dict st;
    st["scatters_in"] = s.scatters_in;
    st["reduces_in"] = s.reduces_in;
    st["outdated_dropped"] = s.outdated_dropped;
    st["future_started"] = s.future_started;
    st["chunks_reduced"] = s.chunks_reduced;
    st["forced_reduces"] = s.forced_reduces;
    st["rounds_completed"] = s.rounds_completed;
    st["rounds_forced"] = s.rounds_forced;
    st["bulk_rounds"] = s.bulk_rounds;
    d["stats"] = st;
    if (stream_link_) {
      py::dict ls;
      ls["groups"] = stream_link_->stats().groups;
      ls["ops"] = stream_link_->stats().ops;
      ls["bytes_sent"] = stream_link_->stats().bytes_sent;
      ls["rounds"] = stream_link_->stats().rounds;
      ls["unreduced_chunks"] = stream_link_->stats().unreduced_chunks;
      ls["lag"] = stream_link_->lag();
      ls["bulk_rounds"] = stream_link_->stats().bulk_rounds;
      ls["collective_rounds"] = stream_link_->stats().collective_rounds;
      ls["exact_step_rounds"] = stream_link_->stats().exact_step_rounds;
      ls["exact_unit_chunks"] = stream_link_->exact_unit_chunks();
      ls["graph_captures"] = stream_link_->stats().graph_captures;
      ls["graph_replays"] = stream_link_->stats().graph_replays;
      ls["graphs"] = stream_link_->graphs();
      if (!stream_link_->graph_error().empty()) ls["graph_error"] = stream_link_->graph_error();
      const Lane ln = stream_link_->lane();
      ls["lane"] = ln == Lane::Auto ? "auto" : ln == Lane::P2P ? "p2p" : ln == Lane::Ipc ? "ipc" : "collective";
      ls["ipc_rounds"] = stream_link_->stats().ipc_rounds;
      if (IpcLane* ipc = stream_link_->ipc()) {
        py::dict is;
        is["portions"] = ipc->nportions();
        is["portion_bytes"] = ipc->portion_elems() * int64_t(dtype_size(dt_));
        is["window_bytes"] = int64_t(ipc->window_bytes());
        is["shares_windows"] = ipc->shares_windows();
        is["windows_id"] = int64_t(ipc->windows_id());
        is["max_wgs"] = ipc->max_wgs();
        is["ranks_on_this_gpu"] = ipc->ranks_on_this_gpu();
        is["rounds"] = ipc->stats().rounds;
        is["bcast_rounds"] = ipc->stats().bcast_rounds;
        is["mode"] = ipc->bcast() ? "bcast" : "pull";
        is["fused"] = ipc->fused();
        is["lite"] = ipc->lite();
        is["memory"] = ipc->memory_kind();
        is["bytes_pushed"] = ipc->stats().bytes_pushed;
        is["bytes_pulled"] = ipc->stats().bytes_pulled;
        ls["ipc"] = is;
      }
      d["link"] = ls;
    }
    if (reactive_link_) {
      const auto& rs = reactive_link_->stats();
      py::dict ls;
      ls["groups"] = rs.groups;
      ls["bytes_sent"] = rs.bytes_sent;
      ls["p1_arrivals"] = rs.p1_arrivals;
      ls["p2_arrivals"] = rs.p2_arrivals;
      ls["unreduced_chunks"] = rs.unreduced_chunks;
      ls["polls"] = rs.polls;
      ls["reclaim_waits"] = rs.reclaim_waits;
      ls["peers_lost"] = rs.peers_lost;
      ls["transfers_dropped"] = rs.transfers_dropped;
      ls["p2_overlapped"] = rs.p2_overlapped;
      ls["slots"] = dp_->slots_allocated();
      ls["slots_busy"] = dp_->slots_busy();
      ls["in_flight"] = reactive_link_->in_flight();
      d["link"] = ls;
    }
    return d;
  }
  // What the transport reports about itself (RCCL: ncclCommCount/UserRank/
  // CuDevice) -- None before a transport is connected.
  py::object p2p_info() const {
    if (!p2p_) return py::none();
    P2PInfo i = p2p_->info();
    py::dict d;
    d["kind"] = i.kind;
    d["nranks"] = i.nranks;
    d["rank"] = i.rank;
    d["device"] = i.device;
    d["comms"] = i.comms;
    return std::move(d);
  }
  // Exact-round lane of the scheduled transport (stream_link.h Lane).
  void set_lane(const std::string& lane) {
    AKKA_CHECK(stream_link_, "set_lane: scheduled (stream) transport only");
    if (lane == "auto") stream_link_->set_lane(Lane::Auto);
    else if (lane == "p2p") stream_link_->set_lane(Lane::P2P);
    else if (lane == "collective") stream_link_->set_lane(Lane::Collective);
    else if (lane == "ipc") {
      AKKA_CHECK(stream_link_->ipc() && stream_link_->ipc()->ready(), "set_lane('ipc'): open the ipc windows first");
      stream_link_->set_lane(Lane::Ipc);
    }
    else throw AkkaError("akka: lane must be 'auto', 'p2p', 'collective' or 'ipc'");
  }
  void set_exact_unit_bytes(int64_t bytes) {
    AKKA_CHECK(stream_link_, "set_exact_unit_bytes: scheduled (stream) transport only");
    stream_link_->set_exact_unit_bytes(bytes);
  }
  void set_graphs(bool on) {
    AKKA_CHECK(stream_link_, "set_graphs: scheduled (stream) transport only");
    stream_link_->set_graphs(on);
  }
  void p2p_check() {
    if (p2p_) p2p_->check();
  }
  int32_t scatter_count(int32_t round, int32_t chunk) const { return engine_->scatter_count(round, chunk); }
  int32_t reduced_arrivals(int32_t round) const { return engine_->reduced_arrivals(round); }

  // ---- fast path ---------------------------------------------------------------
  // One collective-style round with caller-owned buffers: input, output and
  // counts are bound natively, so the engine's fetch / alloc_output / deliver
  // callbacks never enter Python.  Returns the rounds delivered during the call
  // (the caller builds their outputs); they are already unbound.  With
  // `stream_wait` the caller's stream is made to wait for each delivered round.
  std::vector<int32_t> fast_round(int32_t r, uintptr_t in, uintptr_t out, uintptr_t counts, uintptr_t stream,
                                  bool stream_wait) {
    AKKA_CHECK(dp_ && dev_ && stream_link_, "fast_round: scheduled (stream) transport only");
    AKKA_CHECK(!deferred_, "fast_round: deferred host streams complete rounds outside the call");
    pre_[r] = Prebound{in, out, counts, stream, stream_wait};
    fast_delivered_.clear();
    // collective use has nobody to tell CompleteAllreduce: skip that Python
    // callback per round (notify_complete); one attribute lookup per call
    fast_no_master_ = host_.attr("master").is_none();
    try {
      engine_->start(r);
    } catch (...) {
      pre_.erase(r);
      fast_no_master_ = false;
      throw;
    }
    fast_no_master_ = false;
    std::vector<int32_t> got;
    got.swap(fast_delivered_);
    for (int32_t d : got) dp_->unbind(d);
    return got;
  }

  // ---- EngineHost -------------------------------------------------------------
  void fetch(int32_t round) override {
    auto it = pre_.find(round);
    if (it == pre_.end()) {
      host_.attr("_fetch")(round);
      return;
    }
    // host devices: a modelled caller stream (stream race checking) counts too
    // (a synchronous call: its round completes inside this call, so the
    // input-ready marker can wait until a stream of the engine needs it --
    // none does when the round runs on the caller's stream)
    dp_->bind_input(round, reinterpret_cast<const void*>(it->second.in), reinterpret_cast<StreamH>(it->second.stream),
                    !dev_->is_host() || (dev_->models_streams() && it->second.stream != 0),
                    it->second.stream_wait && !dev_->is_host());
    // a synchronous call: the caller's stream waits for the round anyway, so
    // a lane that needs no stream of its own may run the round right there
    if (it->second.stream_wait && !dev_->is_host()) dp_->set_caller_waits(round);
  }
  void alloc_output(int32_t round) override {
    auto it = pre_.find(round);
    if (it == pre_.end()) {
      host_.attr("_alloc_output")(round);
      return;
    }
    dp_->bind_output(round, reinterpret_cast<void*>(it->second.out), reinterpret_cast<int32_t*>(it->second.counts));
  }
  void deliver(int32_t round) override {
    auto it = pre_.find(round);
    if (it == pre_.end()) {
      host_.attr("_deliver")(round);
      return;
    }
    if (it->second.stream_wait) dp_->stream_wait_done(round, reinterpret_cast<StreamH>(it->second.stream));
    pre_.erase(it);
    fast_delivered_.push_back(round);
  }
  void notify_complete(int32_t round) override {
    // (deliver() has already moved a prebound round to fast_delivered_)
    if (fast_no_master_ && std::find(fast_delivered_.begin(), fast_delivered_.end(), round) != fast_delivered_.end())
      return;  // nobody to tell (collective use)
    if (pre_.count(round) && host_.attr("master").is_none()) return;
    host_.attr("_notify_complete")(round);
  }
  void release(int32_t round) override {
    if (pre_.count(round)) return;  // caller-owned input: nothing to drop
    host_.attr("_release")(round);
  }

 private:
  void make_reactive_link() {
    AKKA_CHECK(engine_->geometry().N >= 2, "reactive link needs N >= 2");
    // send-slot pool depth = bounded staleness while a peer lags (default 16)
    int32_t slots = 16;
    if (const char* v = std::getenv("AKKA_REACTIVE_SLOTS")) slots = std::max(2, std::atoi(v));
    reactive_link_ = std::make_unique<ReactiveLink>(engine_.get(), p2p_.get(), slots);
    reactive_link_->bind(dp_.get());
    engine_->set_link(reactive_link_.get());
  }
  void make_stream_link(bool any_kind = false) {
    AKKA_CHECK(any_kind || link_kind_ == "stream", "worker was not created with link='stream'");
    stream_link_ = std::make_unique<StreamLink>(engine_.get(), p2p_.get(), lag_);
    stream_link_->bind(dp_.get());
    engine_->set_link(stream_link_.get());
  }

  struct Prebound {
    uintptr_t in, out, counts, stream;
    bool stream_wait;
  };
  std::unordered_map<int32_t, Prebound> pre_;
  std::unique_ptr<IpcLane> ipc_pending_;  // created by ipc_handle, moved into the link by ipc_open
  std::vector<int32_t> fast_delivered_;
  bool fast_no_master_ = false;  // inside fast_round, with no master to notify

  py::object host_;
  std::string link_kind_;
  int32_t device_idx_;
  bool deferred_;
  std::set<std::string> tags_;  // stable storage of declared access tags
  int32_t lag_;
  DType dt_ = DType::F32;
  std::shared_ptr<Device> dev_;  // shared between engines that adopt one transport
  std::unique_ptr<DataPlane> dp_;
  std::shared_ptr<P2P> p2p_;
  std::shared_ptr<P2P> adopted_p2p_;
  std::unique_ptr<StreamLink> stream_link_;
  std::unique_ptr<ReactiveLink> reactive_link_;
  bool self_drive_ = false;
  std::unique_ptr<OutboxLink> outbox_;
  std::unique_ptr<Engine> engine_;
};

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// The frames of one connection, split natively: data frames a worker core
// takes are applied in place without returning to Python; the first frame it
// does not take (another message type, another dtype, no core) is handed back
// -- frames stay in order.  One Python call per recv instead of one per chunk
// (csrc/runtime/frames.h: the reference's ~400 messages per worker per round).
class FrameSplitter {
 public:
  void append(py::bytes chunk) {
    char* p = nullptr;
    Py_ssize_t n = 0;
    if (PyBytes_AsStringAndSize(chunk.ptr(), &p, &n) != 0) throw py::error_already_set();
    if (pos_ > 0 && pos_ == buf_.size()) {
      buf_.clear();
      pos_ = 0;
    }
    buf_.append(p, size_t(n));
  }
  // Applies frames to `core` until one it does not take; returns that body
  // (bytes), or None once no complete frame is left.  A frame whose apply
  // raised is consumed and the error re-raised.
  py::object run(WorkerCore* core) {
    while (buf_.size() - pos_ >= 4) {
      const unsigned char* h = reinterpret_cast<const unsigned char*>(buf_.data() + pos_);
      const size_t n = (size_t(h[0]) << 24) | (size_t(h[1]) << 16) | (size_t(h[2]) << 8) | size_t(h[3]);
      // a corrupt stream: ValueError, which makes the runtime close the
      // connection (as wire.FrameReader does) instead of retrying forever
      if (n > (size_t(1) << 31)) throw py::value_error("frame of " + std::to_string(n) + " bytes exceeds limit");
      if (buf_.size() - pos_ < 4 + n) break;
      const char* body = buf_.data() + pos_ + 4;
      pos_ += 4 + n;
      if (core != nullptr && core->apply_frame_raw(body, n)) continue;
      py::bytes out(body, n);
      compact();
      return out;
    }
    compact();
    return py::none();
  }
  size_t pending() const { return buf_.size() - pos_; }

 private:
  void compact() {
    if (pos_ > (size_t(1) << 16) && pos_ * 2 > buf_.size()) {
      buf_.erase(0, pos_);
      pos_ = 0;
    }
  }
  std::string buf_;
  size_t pos_ = 0;
};

}  // namespace


PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X-native threshold allreduce core (engine, gfx950 kernels, RCCL/xGMI transport)";
  py::register_exception<AkkaError>(m, "AkkaError", PyExc_RuntimeError);
  bind_onesided(m);
  bind_probe(m);

  // the native data-frame codec alone (tests: interop with wire.py both ways)
  m.def("frame_encode", [](int32_t kind, py::bytes value, const std::string& dtype, int32_t src, int32_t dest,
                           int32_t chunk, int32_t round, int32_t count) {
    std::string v = value, out;
    frames::append_data_frame(out, kind, v.data(), v.size(), dtype.c_str(), src, dest, chunk, round, count);
    return py::bytes(out);
  });
  m.def("frame_parse", [](py::bytes body) -> py::object {
    std::string b = body;
    frames::DataFrame f;
    if (!frames::parse_data_frame(b.data(), b.size(), f)) return py::none();
    py::dict d;
    d["kind"] = f.kind;
    d["value"] = py::bytes(f.value, f.nbytes);
    d["dtype"] = f.dtype;
    d["src"] = f.src;
    d["dest"] = f.dest;
    d["chunk"] = f.chunk;
    d["round"] = f.round;
    d["count"] = f.count;
    return d;
  });
  py::class_<FrameSplitter>(m, "FrameSplitter")
      .def(py::init<>())
      .def("append", &FrameSplitter::append)
      .def("run", &FrameSplitter::run, py::arg("core").none(true))
      .def_property_readonly("pending", &FrameSplitter::pending);
  py::class_<OutMsg>(m, "OutMsg")
      .def_readonly("kind", &OutMsg::kind)
      .def_readonly("src", &OutMsg::src)
      .def_readonly("dest", &OutMsg::dest)
      .def_readonly("chunk", &OutMsg::chunk)
      .def_readonly("round", &OutMsg::round)
      .def_readonly("count", &OutMsg::count)
      .def_property_readonly("data", [](const OutMsg& o) { return py::bytes(o.data); });

  py::class_<PyLoopbackHub>(m, "LoopbackHub")
      .def(py::init([](int32_t n) { return PyLoopbackHub{std::make_shared<LoopbackHub>(n)}; }))
      .def("bytes_moved", [](const PyLoopbackHub& h) { return h.hub->bytes; });

  py::class_<PyPairHub>(m, "PairLoopbackHub")
      .def(py::init([](int32_t n) { return PyPairHub{std::make_shared<PairHub>(n)}; }))
      .def("bytes_moved", [](const PyPairHub& h) {
        std::lock_guard<std::mutex> lk(h.hub->mu);
        return h.hub->bytes;
      })
      .def("release_all", [](const PyPairHub& h) {
        // Un-park every stream waiting for a peer that will never post (test
        // teardown after a failure): no hang at stream destruction.
        std::lock_guard<std::mutex> lk(h.hub->mu);
        for (auto* f : h.hub->flags) __atomic_store_n(f, 0x7fffffffu, __ATOMIC_SEQ_CST);
      });

  py::class_<PySimHub>(m, "SimHub")
      .def(py::init([](int32_t n, bool collectives) { return PySimHub{make_sim_hub(n, collectives)}; }),
           py::arg("n"), py::arg("collectives") = false)
      .def("bytes_moved", [](const PySimHub& h) { return sim_bytes_moved(h.hub); });

  py::class_<WorkerCore>(m, "WorkerCore")
      .def(py::init<py::object, std::string, int32_t, std::string, bool, int32_t>(), py::arg("host"),
           py::arg("link") = "outbox", py::arg("device") = -1, py::arg("dtype") = "float32",
           py::arg("deferred") = false, py::arg("lag") = 2)
      .def("init", &WorkerCore::init)
      .def("connect_rccl", &WorkerCore::connect_rccl, py::arg("uid"), py::arg("rank"), py::arg("nranks"),
           py::arg("members") = std::vector<int32_t>{})
      .def("rebuild_transport", &WorkerCore::rebuild_transport)
      .def("connect_sim", &WorkerCore::connect_sim)
      .def("connect_rccl_shape", &WorkerCore::connect_rccl_shape)
      .def("connect_local", &WorkerCore::connect_local)
      .def("connect_callback", &WorkerCore::connect_callback)
      .def("connect_loopback", &WorkerCore::connect_loopback)
      .def("connect_loopback_pair", &WorkerCore::connect_loopback_pair)
      .def("connect_async_callback", &WorkerCore::connect_async_callback)
      .def("attach", &WorkerCore::attach)
      .def("start", &WorkerCore::start)
      .def("poll", &WorkerCore::poll)
      .def("in_flight", &WorkerCore::in_flight)
      .def("wait_activity", &WorkerCore::wait_activity)
      .def("reactive", &WorkerCore::reactive)
      .def("scatter_in", &WorkerCore::scatter_in)
      .def("reduce_in", &WorkerCore::reduce_in)
      .def("peer_terminated", &WorkerCore::peer_terminated)
      .def("fast_round", &WorkerCore::fast_round)
      .def("bind_input", &WorkerCore::bind_input)
      .def("bind_output", &WorkerCore::bind_output, py::arg("round"), py::arg("out"), py::arg("counts"),
           py::arg("stream") = 0, py::arg("has_stream") = false)
      .def("unbind", &WorkerCore::unbind)
      .def("models_streams", &WorkerCore::models_streams)
      .def("create_stream", &WorkerCore::create_stream)
      .def("declare_access", &WorkerCore::declare_access)
      .def("race_reports", &WorkerCore::race_reports)
      .def("race_count", &WorkerCore::race_count)
      .def("sync_stream", &WorkerCore::sync_stream)
      .def("stream_wait_done", &WorkerCore::stream_wait_done)
      .def("sync_done", &WorkerCore::sync_done)
      .def("exec_on_producer", &WorkerCore::exec_on_producer)
      .def("sync_all", &WorkerCore::sync_all)
      .def("expand_counts", &WorkerCore::expand_counts)
      .def("count_mean", &WorkerCore::count_mean)
      .def("drain", &WorkerCore::drain)
      .def("drain_frames", &WorkerCore::drain_frames)
      .def("apply_frame", &WorkerCore::apply_frame)
      .def("streams", &WorkerCore::streams)
      .def("state", &WorkerCore::state)
      .def("p2p_info", &WorkerCore::p2p_info)
      .def("p2p_check", &WorkerCore::p2p_check)
      .def("set_lane", &WorkerCore::set_lane)
      .def("set_graphs", &WorkerCore::set_graphs)
      .def("set_exact_unit_bytes", &WorkerCore::set_exact_unit_bytes)
      .def("connect_none", &WorkerCore::connect_none)
      .def("connect_ipc_p2p", &WorkerCore::connect_ipc_p2p)
      .def("adopt_transport", &WorkerCore::adopt_transport)
      .def("connect_adopted", &WorkerCore::connect_adopted)
      .def("transport_id", &WorkerCore::transport_id)
      .def("p2p_handle", &WorkerCore::p2p_handle)
      .def("p2p_open", &WorkerCore::p2p_open)
      .def("ipc_handle", &WorkerCore::ipc_handle, py::arg("capacity") = 0, py::arg("share") = nullptr)
      .def("ipc_open", &WorkerCore::ipc_open)
      .def("ipc_error", &WorkerCore::ipc_error)
      .def("ipc_close", &WorkerCore::ipc_close)
      .def("ipc_round_direct", &WorkerCore::ipc_round_direct, py::arg("in_ptr"), py::arg("out_ptr"), py::arg("stream"),
           py::arg("counts") = 0, py::arg("n") = 0, py::arg("finish") = false)
      .def("ipc_error_now", &WorkerCore::ipc_error_now)
      .def("ipc_device_rounds", &WorkerCore::ipc_device_rounds)
      .def("ipc_current_round", &WorkerCore::ipc_current_round)
      .def("ipc_set_mode", &WorkerCore::ipc_set_mode, py::arg("mode"), py::arg("fused") = false,
           py::arg("threads") = 0, py::arg("lite") = -1)
      .def("scatter_count", &WorkerCore::scatter_count)
      .def("reduced_arrivals", &WorkerCore::reduced_arrivals);

  m.def("sim_step", [](const PySimHub& hub, std::vector<WorkerCore*> cores, uint32_t rotate) {
    std::vector<Device*> devs;
    for (auto* c : cores) devs.push_back(c->device());
    return sim_step(hub.hub, devs, rotate);
  }, py::arg("hub"), py::arg("cores"), py::arg("rotate") = 0);
  m.def("sim_run", [](const PySimHub& hub, std::vector<WorkerCore*> cores, int64_t max_iters) {
    std::vector<Device*> devs;
    for (auto* c : cores) devs.push_back(c->device());
    sim_run(hub.hub, devs, max_iters);
  }, py::arg("hub"), py::arg("cores"), py::arg("max_iters") = 100000000);

  m.def("rccl_unique_id", []() {
    auto v = rccl_unique_id();
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  m.def("rccl_version", []() { return std::string(rccl_version_string()); });
  m.def("watchdog_arm", &watchdog_arm, py::arg("seconds"), py::arg("line"), py::arg("to_stdout"),
        py::arg("debug_path") = "", py::arg("exit_code") = 3, py::arg("tail_bytes") = 4096,
        py::arg("beacon_path") = "",
        "Native phase watchdog (runtime/watchdog.h): on expiry write `line` and _exit(exit_code)");
  m.def("watchdog_disarm", &watchdog_disarm);
  m.def("watchdog_set_out_fd", &watchdog_set_out_fd);
  m.def("watchdog_install_sigterm", &watchdog_install_sigterm);
  m.def("watchdog_track_child", &watchdog_track_child, py::arg("pid"));
  m.def("watchdog_untrack_child", &watchdog_untrack_child, py::arg("pid"));
  m.def("json_escape", &json_escape);
  m.def("hw_queue_probe", [](int32_t kmax, int32_t wait_ms) {
    // How many streams can be parked on a wait-value before a fresh stream
    // stops making progress (= the HW queues streams really get).  Returns the
    // first k at which a memset on a fresh stream did not finish in wait_ms,
    // or kmax+1.  Every parked stream is released before returning.
    py::gil_scoped_release nogil;
    uint32_t* flag = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent) != hipSuccess)
      throw AkkaError("probe: hipHostMalloc failed");
    *flag = 0;
    void* buf = nullptr;
    if (hipMalloc(&buf, 1 << 20) != hipSuccess) throw AkkaError("probe: hipMalloc failed");
    std::vector<hipStream_t> parked;
    int32_t result = kmax + 1;
    for (int32_t k = 1; k <= kmax; ++k) {
      hipStream_t s;
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
      hipStreamWaitValue32(s, flag, 1, hipStreamWaitValueGte, 0xFFFFFFFFu);
      parked.push_back(s);
      hipStream_t f;
      hipStreamCreateWithFlags(&f, hipStreamNonBlocking);
      hipEvent_t e;
      hipEventCreateWithFlags(&e, hipEventDisableTiming);
      hipMemsetAsync(buf, k & 0xff, 1 << 20, f);
      hipEventRecord(e, f);
      auto t0 = std::chrono::steady_clock::now();
      bool done = false;
      while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(wait_ms)) {
        if (hipEventQuery(e) == hipSuccess) {
          done = true;
          break;
        }
      }
      if (!done) {
        result = k;
        __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
        hipEventSynchronize(e);
      }
      hipEventDestroy(e);
      parked.push_back(f);
      if (!done) break;
    }
    __atomic_store_n(flag, 1u, __ATOMIC_SEQ_CST);
    for (auto s : parked) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
    hipFree(buf);
    hipHostFree(flag);
    return result;
  }, py::arg("kmax") = 40, py::arg("wait_ms") = 200);
  m.def("tournament", [](int32_t n) {
    std::vector<std::vector<int32_t>> rounds;
    for (int32_t t = 0; t < tournament_rounds(n); ++t) {
      std::vector<int32_t> partner(static_cast<size_t>(n), 0);
      for (int32_t x = 0; x < n; ++x) partner[size_t(x)] = tournament_partner(n, t, x);
      rounds.push_back(partner);
    }
    return rounds;
  }, "partner[x] per ncclCommSplit round of the pair-communicator setup (>= n: sits out)");

  // Raw grouped-p2p endpoint (tests / microbenchmarks of the RCCL data plane).
  py::class_<P2P>(m, "P2PEndpoint")
      .def("rank", &P2P::rank)
      .def("nranks", &P2P::nranks)
      .def("info", [](const P2P& p) {
        P2PInfo i = p.info();
        py::dict d;
        d["kind"] = i.kind;
        d["nranks"] = i.nranks;
        d["rank"] = i.rank;
        d["device"] = i.device;
        d["comms"] = i.comms;
        return d;
      })
      .def("check", &P2P::check)
      .def("has_collectives", &P2P::has_collectives)
      .def("rebuild", [](P2P& p, py::bytes uid, std::vector<int32_t> members) {
        std::string s = uid;
        return p.rebuild(std::vector<uint8_t>(s.begin(), s.end()), members);
      })
      .def("reduce_scatter", [](P2P& p, uintptr_t stream, uintptr_t send, uintptr_t recv, size_t count,
                                const std::string& dtype) {
        p.reduce_scatter(reinterpret_cast<StreamH>(stream), reinterpret_cast<const void*>(send),
                         reinterpret_cast<void*>(recv), count, dtype == "bfloat16" ? DType::BF16 : DType::F32);
      })
      .def("all_gather", [](P2P& p, uintptr_t stream, uintptr_t send, uintptr_t recv, size_t count,
                            const std::string& dtype) {
        p.all_gather(reinterpret_cast<StreamH>(stream), reinterpret_cast<const void*>(send),
                     reinterpret_cast<void*>(recv), count, dtype == "bfloat16" ? DType::BF16 : DType::F32);
      })
      .def("group", [](P2P& p, uintptr_t stream, const std::vector<std::tuple<bool, int32_t, uintptr_t, size_t>>& ops) {
        std::vector<P2POp> v;
        v.reserve(ops.size());
        for (const auto& o : ops)
          v.push_back({std::get<0>(o), std::get<1>(o), reinterpret_cast<void*>(std::get<2>(o)), std::get<3>(o)});
        p.group(reinterpret_cast<StreamH>(stream), v);
      });
  m.def("rccl_endpoint", [](py::bytes uid, int32_t rank, int32_t nranks, int32_t device, bool pairs,
                            std::vector<int32_t> members) {
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    return pairs ? make_rccl_pair_p2p(v, rank, nranks, device) : make_rccl_p2p(v, rank, nranks, device, members);
  }, py::arg("uid"), py::arg("rank"), py::arg("nranks"), py::arg("device"), py::arg("pairs") = false,
     py::arg("members") = std::vector<int32_t>{});

  // ---- kernels (tests / microbench) ----------------------------------------------
  m.def("reduce", [](uintptr_t dst, std::vector<uintptr_t> srcs, int64_t n, std::string dtype, uintptr_t stream,
                     std::string impl) {
    DType dt = (dtype == "bfloat16" || dtype == "bf16") ? DType::BF16 : DType::F32;
    ReduceImpl im = reduce_impl_from_name(impl.c_str());
    std::vector<const void*> ptrs;
    for (auto p : srcs) ptrs.push_back(reinterpret_cast<const void*>(p));
    AKKA_CHECK(!ptrs.empty(), "reduce: no sources");
    for (const auto& spec : split_reduce(reinterpret_cast<void*>(dst), ptrs, n)) launch_reduce(as_stream(stream), spec, dt, im);
  }, py::arg("dst"), py::arg("srcs"), py::arg("n"), py::arg("dtype") = "float32", py::arg("stream") = 0,
        py::arg("impl") = "auto");
  m.def("count_expand", [](uintptr_t out, uintptr_t counts, int64_t S, int64_t step, int32_t N, int64_t C,
                           int32_t kmax, uintptr_t stream) {
    launch_count_expand(as_stream(stream), reinterpret_cast<int32_t*>(out), reinterpret_cast<const int32_t*>(counts),
                        S, step, N, C, kmax);
  });
  m.def("count_mean", [](uintptr_t dst, uintptr_t src, uintptr_t counts, int64_t S, int64_t step, int32_t N,
                         int64_t C, int32_t kmax, std::string dtype, uintptr_t stream, bool axpy, float alpha,
                         uintptr_t shadow) {
    launch_count_mean(as_stream(stream), reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src),
                      reinterpret_cast<const int32_t*>(counts), S, step, N, C, kmax,
                      dtype == "bfloat16" ? DType::BF16 : DType::F32, axpy, alpha, reinterpret_cast<void*>(shadow));
  }, py::arg("dst"), py::arg("src"), py::arg("counts"), py::arg("S"), py::arg("step"), py::arg("N"), py::arg("C"),
     py::arg("kmax"), py::arg("dtype"), py::arg("stream"), py::arg("axpy") = false, py::arg("alpha") = 0.f,
     py::arg("shadow") = 0);
  m.def("colsum_bf16", [](uintptr_t out, uintptr_t in, int64_t M, int64_t ncol, uintptr_t part, uintptr_t tickets,
                          int32_t splits, uintptr_t stream, bool lite, uintptr_t act, uintptr_t gout) {
    launch_colsum_bf16(as_stream(stream), reinterpret_cast<float*>(out), reinterpret_cast<const void*>(in), M, ncol,
                       reinterpret_cast<float*>(part), reinterpret_cast<uint32_t*>(tickets), splits, lite,
                       reinterpret_cast<const void*>(act), reinterpret_cast<void*>(gout));
  }, py::arg("out"), py::arg("in"), py::arg("M"), py::arg("ncol"), py::arg("part"), py::arg("tickets"),
     py::arg("splits"), py::arg("stream"), py::arg("lite") = true, py::arg("act") = 0, py::arg("gout") = 0);
  m.def("colsum_row_splits", &colsum_row_splits);
  m.def("xent_fwd", [](uintptr_t x, uintptr_t y, int64_t B, int64_t C, uintptr_t lse, uintptr_t rowloss, uintptr_t out,
                       uintptr_t ticket, uintptr_t stream) {
    launch_xent_fwd(as_stream(stream), reinterpret_cast<const void*>(x), reinterpret_cast<const int64_t*>(y), B, C,
                    reinterpret_cast<float*>(lse), reinterpret_cast<float*>(rowloss), reinterpret_cast<float*>(out),
                    reinterpret_cast<uint32_t*>(ticket));
  });
  m.def("xent_bwd", [](uintptr_t x, uintptr_t y, int64_t B, int64_t C, uintptr_t lse, uintptr_t stat, uintptr_t go,
                       uintptr_t gx, uintptr_t stream) {
    launch_xent_bwd(as_stream(stream), reinterpret_cast<const void*>(x), reinterpret_cast<const int64_t*>(y), B, C,
                    reinterpret_cast<const float*>(lse), reinterpret_cast<const float*>(stat),
                    reinterpret_cast<const float*>(go), reinterpret_cast<void*>(gx));
  });
  m.def("geometry", [](int64_t S, int32_t N, int64_t C) {
    Geometry g(S, N, C);
    py::dict d;
    std::vector<std::pair<int64_t, int64_t>> blocks;
    std::vector<int32_t> nch;
    for (int32_t j = 0; j < N; ++j) {
      blocks.push_back({g.block_start(j), g.block_end(j)});
      nch.push_back(g.num_chunks(j));
    }
    d["step"] = g.step;
    d["blocks"] = blocks;
    d["num_chunks"] = nch;
    d["total_chunks"] = g.total_chunks();
    return d;
  });
  m.def("float_threshold", &float_threshold);
  // CPU checks of the ipc transports' host logic (tests/test_ipc_layout.py)
  m.def("ipc_p2p_plan", [](std::vector<std::tuple<bool, int32_t, int64_t, int32_t>> ops, int32_t nranks,
                           int64_t piece, std::vector<uint32_t> dead, std::vector<uint32_t> send_seq,
                           std::vector<uint32_t> recv_seq) {
    std::vector<P2POp> v;
    for (auto& t : ops) v.push_back({std::get<0>(t), std::get<1>(t), nullptr, size_t(std::get<2>(t)), std::get<3>(t)});
    dead.resize(size_t(nranks), 0);
    IpcP2PPlan plan = plan_ipc_p2p_group(v, nranks, piece, 2, dead.data(), send_seq, recv_seq);
    py::list queues;
    for (size_t q = 0; q + 1 < plan.qstart.size(); ++q) {
      py::list ql;
      for (int32_t i = plan.qstart[q]; i < plan.qstart[q + 1]; ++i) {
        const IpcP2POp& o = plan.ops[size_t(i)];
        ql.append(py::make_tuple(bool(o.send), int(o.peer), int(o.ch), o.bytes, o.seq));
      }
      queues.append(ql);
    }
    return py::make_tuple(queues, send_seq, recv_seq, plan.bytes_sent);
  });
  m.def("ipc_layout", [](int32_t N, int32_t np, int32_t nslots, int32_t wpp) {
    py::dict d;
    std::vector<int64_t> lane, p2p;
    for (int32_t src = 0; src < N; ++src)
      for (int32_t j = 0; j < np; ++j) lane.push_back(ipc_flag_push(src, j, np));
    for (int32_t j = 0; j < np; ++j)
      for (int32_t part = 0; part < kIpcReduceSplit; ++part) lane.push_back(ipc_flag_reduced(j, part, N, np));
    for (int32_t src = 0; src < N; ++src)
      for (int32_t j = 0; j < np; ++j)
        for (int32_t part = 0; part < kIpcReduceSplit; ++part) lane.push_back(ipc_flag_gather(src, j, part, N, np));
    lane.push_back(ipc_flag_error(N, np));
    for (int32_t r = 0; r < N; ++r)
      for (int32_t ch = 0; ch < 2; ++ch)
        for (int32_t sl = 0; sl < nslots; ++sl)
          for (int32_t w = 0; w < wpp; ++w) {
            p2p.push_back(ipc_p2p_flag_written(r, ch, sl, w, 2, nslots, wpp));
            p2p.push_back(ipc_p2p_flag_consumed(r, ch, sl, w, N, 2, nslots, wpp));
          }
    d["lane_flags"] = lane;
    d["lane_flag_bytes"] = int64_t(ipc_flag_bytes(N, np));
    d["p2p_flags"] = p2p;
    d["p2p_flag_bytes"] = int64_t(ipc_p2p_flag_bytes(N, 2, nslots, wpp));
    d["stride"] = kIpcFlagStride;
    d["window_slots"] = ipc_window_slots(N);
    return d;
  });
  m.attr("build_arch") = "gfx950";
}
