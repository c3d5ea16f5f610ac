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

// Largest part of a window the lane builds (one allocation, one IPC handle).
constexpr size_t kIpcMaxWindowBytes = size_t(1920) << 20;

struct IpcLaneStats {
  int64_t rounds = 0, bcast_rounds = 0, bytes_pushed = 0, bytes_pulled = 0;
};

class IpcLane {
 public:
  IpcLane(Device* dev, const Geometry& g, int32_t me, DType dt);
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
  // Enqueue one exact round on `s`: in[S] from every rank summed into out[S].
  void round(StreamH s, const void* in, void* out);
  // The error word (a wait timed out): error() after draining the device,
  // error_now() as far as the kernels got (no synchronisation).
  uint32_t error();
  uint32_t error_now() const;
  // device view of the host-mapped error word (the poison flag of the rounds)
  const uint32_t* error_word_device() const { return err_dev_; }
  int32_t nportions() const { return nportions_; }
  int64_t portion_elems() const { return portion_; }
  size_t window_bytes() const { return data_bytes_; }
  const std::string& memory_kind() const { return mem_kind_; }
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
  size_t data_bytes_ = 0, flag_bytes_ = 0, in_bytes_ = 0, out_bytes_ = 0;
  char* data_ = nullptr;   // inbound slots
  char* gdata_ = nullptr;  // reduced row + gather slots
  uint32_t* flags_ = nullptr;
  uint32_t* err_host_ = nullptr;  // host-mapped error word
  uint32_t* err_dev_ = nullptr;
  std::vector<char*> peer_data_;      // [N] mapped windows (own = data_)
  std::vector<char*> peer_gdata_;     // [N] mapped reduced / gather parts (own = gdata_)
  std::vector<uint32_t*> peer_flags_; // [N]
  uint32_t round_ = 0;
  int32_t max_wgs_ = 1024, sharers_ = 1;
  int32_t threads_ = 256;  // workgroup size of the round kernels (AKKA_IPC_THREADS)
  uint64_t timeout_ticks_ = 0;
  bool ready_ = false;
  bool bcast_ = false, fused_ = false;
  std::string mem_kind_;
  IpcLaneStats stats_;
};

}  // namespace akka
