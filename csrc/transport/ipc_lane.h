// IpcLane: exact rounds as one-sided xGMI loads/stores between the GPUs of a
// node (kernels: csrc/kernels/ipc.hip, protocol in ipc_kernels.h).
//
// Why a lane of its own: on one node every MI355X maps every other one's HBM
// over xGMI, so an exact round (thresholds 1, every chunk from every peer)
// needs no message matching at all.  Each rank owns a window
//   [slot 0 | ... | slot N-1]  [reduced | gather 0 | ... | gather N-1]
// (two allocations; each slot >= one block; ipc_kernels.h)
// plus a small flag area (uncached).  Rank q pushes block p of its input into
// slot q of rank p's window, rank p sums its N slots into its output block and
// `reduced` row, and every rank pulls the reduced rows of the others (or, in
// bcast mode, rank p stores them into everyone's gather slot [p]) -- all
// seven links of a rank busy in both phases, driven by the CUs, with round-id
// flags per portion instead of RCCL groups: three kernel launches per round
// and no host work beyond them.  The reference's scatter / reduce / broadcast
// (W:212-268) for the exact case; thresholds < 1 keep the p2p schedule.
//
// Setup is collective: every rank creates its window (handle()), the handles
// are exchanged out of band (torch.distributed, any backend) and every rank
// opens the others' (open()).  Rounds are numbered 1, 2, ... per lane: every
// rank must run the same exact rounds on this lane, in the same order (the
// same contract as the other lanes).  Waits inside the kernels are bounded:
// a missing peer turns into error() != 0, never a hung GPU.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../engine/device.h"
#include "../engine/geometry.h"

namespace akka {

// Device memory another GPU writes into and this one reads (or the reverse)
// over xGMI.  Coarse-grained memory (plain hipMalloc) is only coherent at
// kernel boundaries of ONE device: a line of it cached in this GPU's L2 is not
// invalidated when a peer overwrites the memory behind it.  The windows are
// therefore fine-grained by default (AKKA_IPC_MEM = fine | uncached | coarse);
// `kind` reports what was allocated.
void* ipc_alloc_window(size_t bytes, std::string* kind);

// Largest allocation the lanes export (one allocation, one IPC handle).
// hipIpcOpenMemHandle of an allocation of 2^31 bytes or more hangs on the
// ROCm 7.2 / MI355X pool, whatever its memory kind (fine, uncached and coarse
// all hang at 2048 MiB and all open at 2047 MiB in 0.3 ms:
// profiles/r03/ipc_open/) -- a 2 GiB boundary, so every part stays below it.
constexpr size_t kIpcMaxWindowBytes = size_t(2047) << 20;

struct IpcLaneStats {
  int64_t rounds = 0, bcast_rounds = 0, bytes_pushed = 0, bytes_pulled = 0;
};

// The big part of a rank's window (inbound slots | reduced row + gather
// slots) and every peer's as mapped in this process.  Lanes of engines that
// share one transport (same device streams, rounds issued in the same order
// on every rank) share it: every round of any of them starts only after this
// rank's previous round finished reading peers' windows and every peer
// finished reading this rank's slots (the lanes' flag protocol), so one set of
// windows serves every geometry that fits (IpcLane's `share`).
struct IpcWindows {
  Device* dev = nullptr;
  int32_t N = 0, me = 0;
  size_t in_bytes = 0, out_bytes = 0;
  char* data = nullptr;
  char* gdata = nullptr;
  std::vector<char*> peer_data, peer_gdata;  // [N] (own = data / gdata)
  std::vector<void*> opened;
  std::string kind;
  bool open = false;
  ~IpcWindows();
};

class IpcLane {
 public:
  // `capacity` (elements, 0: S): size the windows for a buffer this large, so
  // that later lanes of smaller (or equal) geometry can share them; `share`:
  // use that lane's windows when they are large enough (then this lane only
  // allocates and exchanges its own flag area).
  IpcLane(Device* dev, const Geometry& g, int32_t me, DType dt, int64_t capacity = 0,
          const IpcLane* share = nullptr);
  ~IpcLane();
  IpcLane(const IpcLane&) = delete;
  IpcLane& operator=(const IpcLane&) = delete;

  // This rank's window handle (data + flags), with the geometry it was built for.
  std::string handle() const;
  // Open every other rank's window; handles[i] is rank i's handle().
  void open(const std::vector<std::string>& handles);
  bool ready() const { return ready_; }
  // Phase 2 by remote writes (the reducer stores its rows into every peer's
  // gather slot) instead of remote reads.  Every rank must use the same mode
  // in a round; modes may change between rounds.
  void set_bcast(bool on) { bcast_ = on; }
  bool bcast() const { return bcast_; }
  // One launch per round with push / reduce / phase-2 roles (pipelined by
  // portion) instead of three kernels.
  void set_fused(bool on) { fused_ = on; }
  bool fused() const { return fused_; }
  // Workgroup size of the round kernels (256 / 512 / 1024; default
  // AKKA_IPC_THREADS or 256).  Larger groups keep more loads / stores in
  // flight per CU when one rank has the GPU to itself.
  void set_threads(int32_t t) { threads_ = (t == 512 || t == 1024) ? t : 256; }
  int32_t threads() const { return threads_; }
  // Fence-free hand-offs (xgmi_device.h "lite"): window bytes stored
  // write-through (sc0 sc1), flags after a drain, consumers' system-coherent
  // loads in place of the acquire -- no buffer_wbl2 / buffer_inv per item.
  // Every rank must use the same setting in a round (AKKA_IPC_LITE).
  void set_lite(bool on) { lite_ = on; }
  bool lite() const { return lite_; }
  // Enqueue one exact round on `s`: in[S] from every rank summed into out[S].
  // `fail_counts` (optional, [fail_n] int32): zeroed by the kernel that
  // finds a wait failed -- the fixed counts table of direct rounds then reads
  // 0 for this and every later round (the lane is dead; calls raise).
  void round(StreamH s, const void* in, void* out, int32_t* fail_counts = nullptr, int64_t fail_n = 0,
             int32_t* counts_out = nullptr, int64_t counts_n = 0, int32_t counts_value = 0);
  // Device-resident round ids (graph capture): on, the round id lives in a
  // device word that a bump launch in front of every round advances -- a
  // captured round replays with a fresh id.  Switching copies the id across
  // (off: synchronises to read it back).  Every rank switches at the same round.
  void set_device_rounds(bool on);
  bool device_rounds() const { return round_dev_on_; }
  uint32_t current_round();  // host view (off) / device word (on: synchronises)
  // The error word (a wait timed out): error() after draining the device,
  // error_now() as far as the kernels got (no synchronisation).
  uint32_t error();
  uint32_t error_now() const;
  // device view of the host-mapped error word (the poison flag of the rounds)
  const uint32_t* error_word_device() const { return err_dev_; }
  int32_t nportions() const { return nportions_; }
  int64_t portion_elems() const { return portion_; }
  size_t window_bytes() const { return win_ ? win_->in_bytes + win_->out_bytes : 0; }
  const std::string& memory_kind() const { return win_->kind; }
  bool shares_windows() const { return shared_windows_; }
  // Identity of the window memory (lanes sharing windows report the same).
  uintptr_t windows_id() const { return reinterpret_cast<uintptr_t>(win_.get()); }
  int32_t max_wgs() const { return max_wgs_; }
  int32_t ranks_on_this_gpu() const { return sharers_; }
  const IpcLaneStats& stats() const { return stats_; }

 private:
  Device* dev_;
  Geometry g_;
  int32_t me_;
  DType dt_;
  size_t es_;
  int64_t slot_ = 0, portion_ = 0;
  int32_t nportions_ = 0;
  size_t flag_bytes_ = 0;
  std::shared_ptr<IpcWindows> win_;  // inbound slots + reduced / gather rows (maybe shared)
  bool shared_windows_ = false;
  uint32_t* flags_ = nullptr;        // this lane's own flag area (never shared)
  uint32_t* err_host_ = nullptr;  // host-mapped error word
  uint32_t* err_dev_ = nullptr;
  std::vector<uint32_t*> peer_flags_; // [N]
  std::vector<void*> opened_flags_;
  uint32_t round_ = 0;
  uint32_t* round_dev_ = nullptr;  // uncached device word (device rounds)
  uint32_t* fin_ctr_ = nullptr;    // uncached: the round's counts finisher ticket (IpcArgs::fin_ctr)
  bool round_dev_on_ = false;
  int32_t max_wgs_ = 1024, sharers_ = 1;
  int32_t threads_ = 256;  // workgroup size of the round kernels (AKKA_IPC_THREADS)
  uint64_t timeout_ticks_ = 0;
  bool ready_ = false;
  bool bcast_ = false, fused_ = false, lite_ = false;
  std::string mem_kind_;
  IpcLaneStats stats_;
};

}  // namespace akka
