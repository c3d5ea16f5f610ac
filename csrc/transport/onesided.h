// OneSidedLane: threshold rounds as one-sided stores into mapped peer windows
// (protocol: kernels/onesided_protocol.h; gfx950 kernels: kernels/onesided.hip).
//
// The reference's data plane is fire-and-forget messages into unbounded
// mailboxes (AllreduceWorker.scala:227-232, 259-264): a fast worker never
// waits for a slow one, late messages are dropped (W:155-156, 172-173), and
// maxLag catch-up bounds staleness (W:100-106).  Two-sided transports (RCCL
// p2p) cannot do that -- every send needs the peer's matching receive, so a
// straggler eventually throttles everybody.  Here every rank exports a window
// (scatter rows, gather rows, flag words) and peers STORE into it over xGMI:
// no send ever waits, and the receiver-side thresholds decide what is used.
//
// Two backends run the same protocol functions:
//  * GPU (device >= 0): windows are fine-grained HBM exported with IPC
//    handles, the round is one role-partitioned launch on the caller's
//    stream (its last workgroup out finishes the call) (onesided_kernels.h): each chunk of my block is
//    reduced and pushed the moment its threshold is met, each peer chunk is
//    copied out the moment it lands;
//  * CPU (device < 0): windows are POSIX shared memory, the round is a
//    progress loop over the same roles in the calling thread -- the
//    multi-process CPU tests of the same semantics.  Its pushes can be HELD
//    (an outbox of messages with their bytes, delivered or dropped one by
//    one): a harness then replays the reference spec's arrival orders
//    (AllreduceSpec.scala) against the lane, deterministically.
//
// Setup is collective, like the exact ipc lane: handle() on every rank, the
// handles go to every rank out of band, open(all handles); then unlink()
// (CPU) once every rank opened (a killed rank then leaves nothing behind).
#pragma once

#include <array>
#include <cstdint>
#include <deque>
#include <string>
#include <vector>

#include "../engine/common.h"
#include "../engine/geometry.h"
#include "../kernels/onesided_protocol.h"

namespace akka {

struct OneSidedParams {
  float th_reduce = 1.f, th_complete = 1.f;
  int32_t max_lag = 1;
  int32_t rows = 0;                      // ring depth D (0: max(3, maxLag + 2))
  int64_t part_bytes = 0;  // <= 0: the default part size (kAutoPartBytes)
  int64_t timeout_ms = 30000;            // bound of every wait (then forced + error)
  int32_t threads = 256;                 // workgroup size of the round launch (256 or 1024)
  int32_t role_wgs = 0;                  // workgroups per data role (push / reduce / copy); 0: automatic
  // Keep the round launch on `cu_keep` of every 8 CUs (a CU-masked stream).
  // Ranks sharing one GPU that also run compute kernels (a DP step): a round
  // waiting on its peers cannot hold every SIMD while a PEER's kernels that
  // need a whole SIMD's registers (fp32 MFMA GEMMs) wait for one (the mask
  // costs the shared-card round ~0.25 ms at 64 MiB, profiles/r04/README.md).
  // A rank on a GPU of its own: the bounded footprint that lets an async
  // round overlap the backward on the other CUs (the role grid is sized for
  // the kept CUs).  0: no mask.
  int32_t cu_keep = 0;
  // Hand-off mode of window bytes (os::Args::fenced): false "lite"
  // (write-through + drain), true "fenced" (plain stores + system release /
  // acquire).  AKKA_OS_HANDOFF=fenced|lite overrides it at construction.
  bool fenced = false;
  // Exact rounds only: a call without a caller buffer returns the gather row
  // of its call id in this rank's own window -- the peers' reduced parts
  // land there at their final offsets, so no copy (Python: the output of
  // call c stays valid until call c + 1).  Taken when the thresholds are 1
  // and a block's byte size is a 16-byte multiple; window_output() says.
  bool window_output = false;
};

class OneSidedLane {
 public:
  OneSidedLane(int32_t device, int64_t S, int32_t N, int64_t C, int32_t me, DType dt, const OneSidedParams& p);
  ~OneSidedLane();
  OneSidedLane(const OneSidedLane&) = delete;
  OneSidedLane& operator=(const OneSidedLane&) = delete;

  std::string handle() const;
  // An empty handle (q != me) is a rank not in the peer map yet (partial
  // membership, W:213-216): it is never pushed to nor waited for (dead)
  // until add_peer() maps its window.
  void open(const std::vector<std::string>& handles);
  // Re-init with a larger peer map (W:87-89): map a rank that was absent at
  // open() and treat it as live from the next call on.  Between rounds only
  // (GPU: synchronises the device).  A rank mapped once stays mapped: a
  // departed rank is marked dead (set_dead), not remapped.
  void add_peer(int32_t q, const std::string& handle);
  // Ranks whose windows are mapped (me included).
  std::vector<int32_t> members() const;
  // CPU: remove this rank's shared-memory name (every peer mapped it already).
  void unlink();
  bool ready() const { return ready_; }

  // One call = one round of this rank: in[S] -> out[S], counts[N][kcols]
  // (per chunk).  GPU: enqueued on `stream`; CPU: runs to completion.
  // Returns the call id (status()).
  int64_t round(uintptr_t stream, const void* in, void* out, int32_t* counts, int32_t kcols);
  // The call's record (host memory, no sync): round = -1 while it runs;
  // throws if the record was already reused by a call 64 or more later.
  os::CallStatus status(int64_t call) const;
  std::vector<uint64_t> stats();  // GPU: synchronises the device first
  uint32_t error() const;
  void clear_error();
  // A peer marked dead is never waited for again (and never written to).
  void set_dead(int32_t peer, bool dead);
  // Every wait of a round r < v ends at once with what landed (forced).
  void force_below(uint32_t v);
  // This rank serves no further round: peers stop waiting for its copies of
  // rounds >= its next one (the end of a job; GPU: enqueued on `stream`).
  void retire(uintptr_t stream);
  // Calls a captured (graphed) call ran in addition to round()'s own: keeps
  // the host's call ids in step with the device's sequence.
  void note_replays(int64_t n) { calls_ += n; }
  // Switch the hand-off mode between calls (every later call; both modes
  // share the tags, so ranks may switch independently).
  void set_fenced(bool on) { p_.fenced = on; }
  bool fenced() const { return p_.fenced; }
  bool window_output() const { return wo_; }
  // Base of my own gather row `row` (window output: call c's output is row c % D).
  void* gather_row(int32_t row) const { return gd_[size_t(row)]; }

  // ---- CPU backend, step by step (the deterministic replay harness) ----------
  // begin(): start a round (non-blocking), returns its call id; progress():
  // one pass over every role, true once the round completed.
  int64_t begin(const void* in, void* out, int32_t* counts, int32_t kcols);
  bool progress();
  bool active() const { return cr_.active; }
  // Held pushes stay in the outbox (with their bytes) until delivered.
  void set_hold(bool hold) { hold_ = hold; }
  // outbox entries: (phase 0 scatter / 1 gather, dst, chunk, part, round, count)
  std::vector<std::array<int64_t, 6>> outbox() const;
  // Perform / discard outbox entry i (gates evaluated at delivery, as the
  // reference's receiver checks a message when it arrives).
  void deliver(int64_t i);
  void drop(int64_t i);
  std::string outbox_bytes(int64_t i) const;
  // Play this rank as a TestKit-style peer (AllreduceSpec.scala:812-818): a
  // push of arbitrary bytes from this rank, through the same gates.
  // GPU lanes: the host performs the push into the receiver's device window
  // (blocking copies on a side stream) -- the receiver's kernel may be
  // running; its decisions are the real os_round_kernel's.
  // stage (GPU lanes): 0 the whole push; 1 only its gate (a writer that
  // passed it and has not stored yet: the "writing r" marker stays); 2 the
  // bytes and the "done" tag of a push whose gate already passed
  void inject(int32_t phase, int32_t dst, int32_t k, int32_t j, uint32_t r, uint32_t cnt, const std::string& bytes,
              int32_t stage = 0);
  // stats() without synchronising the device (GPU: read while a call runs).
  std::vector<uint64_t> stats_nowait();
  // Test access to this rank's own window (GPU: copies on the side stream,
  // while a call may run): the flag words, and part j of chunk k of source
  // (SD, phase 0) or block (GD, phase 1) `src` in ring row `row`.
  std::vector<uint32_t> peek_flags();
  std::string peek_part(int32_t phase, int32_t row, int32_t src, int32_t k, int32_t j);

  bool on_gpu() const { return device_ >= 0; }
  int32_t rows() const { return D_; }
  int32_t parts() const { return P_; }
  int64_t part_elems() const { return part_len_; }
  int32_t need_reduce() const { return need_r_; }
  int32_t need_complete() const { return need_c_; }
  int32_t pieces() const { return nsub_; }
  int32_t threads() const { return nt_; }
  int32_t shared_ranks() const { return shared_ranks_; }
  // CUs the round launch may use (cu_keep; 0: all)
  int32_t lane_cus() const { return lane_cus_; }
  // the CU-masked stream (hipStream_t as an integer; 0 without cu_keep): a
  // call enqueued on it runs there directly, without the fork / join
  uintptr_t cu_stream() const { return reinterpret_cast<uintptr_t>(cu_stream_); }
  // AKKA_OS_TIMELINE=1 at construction: per workgroup [entry, round known,
  // role done] of the last call (waits for the device), and the clock rate
  std::vector<uint64_t> timeline();
  int64_t clock_khz() const { return clock_khz_; }
  std::array<int32_t, 3> role_grid() const { return {gp_, gr_, gq_}; }
  size_t window_bytes() const { return win_bytes_; }
  const std::string& memory_kind() const { return mem_kind_; }
  const Geometry& geometry() const { return g_; }
  int64_t calls() const { return calls_; }

 private:
  struct HostWords {  // host memory (GPU: mapped into the device)
    uint32_t err;
    uint32_t force;
    uint32_t dead[os::kMaxRanks];
    uint32_t pad[14];
    os::CallStatus status[os::kStatusSlots];
  };
  struct Msg {
    int32_t phase, dst, k, j;
    uint32_t r, cnt;
    std::vector<char> bytes;
    int32_t stage = 0;  // inject() on a GPU lane: 0 all, 1 gate only, 2 bytes + tag only
  };
  struct CpuRound {
    bool active = false;
    uint32_t r = 0;
    int32_t row = 0;
    int64_t call = 0;
    const char* in = nullptr;
    char* out = nullptr;
    int32_t* counts = nullptr;
    int32_t kcols = 0;
    std::vector<uint8_t> decided;
    int64_t deadline_ms = 0;
  };
  static constexpr int64_t kDefaultRoleWgs = 256;
  static constexpr int64_t kAutoPartBytes = int64_t(256) << 10;  // default part size (part_bytes <= 0)
  // wgs: reduce = 2 x wgs; push / copy = wgs unless given
  void size_roles(int64_t wgs, int64_t push_wgs = 0, int64_t copy_wgs = 0);
  void gpu_call(uintptr_t stream, const char* in, char* out, int32_t* counts, int32_t kcols);
  int32_t make_cu_stream(int32_t keep);
  // CPU roles
  void push(int32_t phase, int32_t dst, int32_t k, int32_t j, uint32_t r, uint32_t cnt, const char* src);
  void exec(const Msg& m, const char* src);
  void exec_gpu(const Msg& m);
  bool try_decide(int32_t k, bool timed_out);
  bool try_complete(bool timed_out);
  void flush();
  void dump(const char* role, int32_t k) const;
  void map_peer(int32_t q, const std::string& handle);
  void write_tables(void* stream = nullptr);  // GPU: the device's pointer tables from pfl_ / psd_ / pgd_
  void wait_own_calls() const;  // GPU: this lane's last call finished (its status record names it)

  int32_t device_;
  Geometry g_;
  int32_t me_;
  DType dt_;
  size_t es_;
  OneSidedParams p_;
  os::Layout L_;
  int32_t D_ = 0, P_ = 1, Kmax_ = 0, need_r_ = 1, need_c_ = 1;
  int32_t nsub_ = 1, nt_ = 256, gp_ = 1, gr_ = 0, gq_ = 1, shared_ranks_ = 1;
  // OneSidedParams::cu_keep: the round launch goes to a CU-masked stream,
  // joined to the caller's stream by events
  void* cu_stream_ = nullptr;  // hipStream_t
  void* ev_in_ = nullptr;      // hipEvent_t
  void* ev_out_ = nullptr;     // hipEvent_t
  int32_t lane_cus_ = 0;
  unsigned long long* tl_dev_ = nullptr;  // AKKA_OS_TIMELINE=1: [grid][3]
  int64_t tl_words_ = 0;
  int64_t clock_khz_ = 0;
  std::string my_bus_;
  int64_t slot_ = 0, part_len_ = 64;
  size_t flag_bytes_ = 0, row_bytes_ = 0, win_bytes_ = 0;
  std::string mem_kind_;
  bool ready_ = false;
  std::vector<uint8_t> absent_;  // [N]: not mapped yet (partial membership)
  bool wo_ = false;              // window output (OneSidedParams::window_output, granted)
  int64_t calls_ = 0;
  uint64_t timeout_ticks_ = 0;

  // own window
  uint32_t* flags_ = nullptr;
  std::vector<char*> sd_, gd_;  // [D]
  // peers' windows as mapped here (own included)
  std::vector<uint32_t*> pfl_;            // [N]
  std::vector<std::vector<char*>> psd_, pgd_;  // [D][N]
  std::vector<void*> opened_;             // GPU: IPC mappings to close

  // local state
  uint32_t* loc_ = nullptr;             // GPU: uncached device memory; CPU: loc_host_
  unsigned long long* stats_dev_ = nullptr;
  void* tab_dev_ = nullptr;             // GPU: os::Tables
  HostWords* hw_ = nullptr;             // host
  HostWords* hw_dev_ = nullptr;         // device view of hw_ (GPU)
  std::vector<uint32_t> loc_host_;
  std::vector<unsigned long long> stats_host_;
  std::array<unsigned long long, os::kNumStats> inj_stats_{};  // GPU: injected pushes' gate outcomes
  void* side_stream_ = nullptr;  // hipStream_t (non-blocking): inject / stats_nowait copies

  // CPU progress state
  CpuRound cr_;
  std::deque<Msg> outbox_;
  bool hold_ = false;
  std::vector<float> acc_;
  std::vector<char> part_;

  // CPU shared memory
  std::string shm_name_;
  char* shm_base_ = nullptr;
  size_t shm_bytes_ = 0;
  std::vector<std::pair<char*, size_t>> peer_maps_;
  bool unlinked_ = false;
};

}  // namespace akka
