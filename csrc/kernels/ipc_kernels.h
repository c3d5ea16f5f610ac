// One-sided xGMI exact round (ipc.hip): every rank maps every other rank's
// window (hipIpcOpenMemHandle) and the round runs as three kernels on one
// stream, no RCCL and no host round trip:
//   push    my input's block p  -> rank p's window slot [me]   (xGMI stores)
//   reduce  slots [0..N) of my block (+ my own input block)    -> my output
//           block and my window's `reduced` row               (local HBM)
//   pull    rank p's `reduced` row -> my output's block p       (xGMI loads)
// or, in bcast mode, reduce also stores its rows into every peer's gather
// slot [me] (xGMI stores) and a local `gather` copies them into the output --
// phase 2 as remote writes instead of remote reads.
// Each block is cut into portions; a portion moves under its own round-id
// flag (one producer workgroup -> one consumer workgroup), so no grid-wide
// barrier exists anywhere and a slow portion delays only its own consumer.
// The reference's scatter / reduce / broadcast of a round, W:212-268, with
// every chunk arriving from every peer (thresholds 1).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../engine/common.h"

namespace akka {

constexpr int kIpcMaxRanks = 16;
constexpr int kIpcFlagStride = 16;  // uint32 words: one 64-B line per flag
constexpr int kIpcReduceSplit = 4;  // reduce workgroups (parts) per portion

// Window of a rank, in slots of `slot` elements, as two allocations (each
// one IPC mapping, so a window may reach twice the largest mapping size):
//   data:  [0, N)   slot[src]: src's contribution to my block (pushed by src)
//   gdata: 0        reduced: my reduced block (pulled by the others, pull mode)
//          [1, N+1) gather[src]: src's reduced block (pushed by src, bcast mode)
// Flags hold round ids (stores, never counts), so the two phase-2 modes can
// alternate between rounds.
struct IpcArgs {
  char* data[kIpcMaxRanks];       // inbound slots of every rank, mapped in this process (own = local)
  char* gdata[kIpcMaxRanks];      // reduced row + gather slots of every rank, mapped likewise
  uint32_t* flags[kIpcMaxRanks];  // flag area of every rank, mapped in this process
  int64_t bstart[kIpcMaxRanks];   // block start / length (elements)
  int64_t blen[kIpcMaxRanks];
  int64_t slot;       // elements per window slot (>= every block, 64-element multiple)
  int64_t portion;    // elements per portion (a multiple of 1024)
  int32_t nportions;  // portions per slot
  int32_t max_wgs;    // grid cap of the kernels that wait (reduce, pull / gather)
  int32_t bcast = 0;  // phase 2: 0 = every rank pulls the reduced rows, 1 = the reducer pushes them
  int32_t fused = 0;  // 1: push, reduce and phase 2 as roles of ONE launch (pipelined by portion)
  int32_t N = 0, me = 0;
  int32_t threads = 256;    // workgroup size of the round's kernels (256 / 512 / 1024)
  int32_t plain_slots = 0;  // measurement only: plain slot loads behind the acquire instead of sc0 sc1 loads
  int32_t lite = 0;         // fence-free hand-offs: write-through window stores + drained flags (xgmi_device.h)
  uint32_t round = 0;       // this round's id (1, 2, ... identical on every rank)
  // device-resident round id (graph-capturable rounds): when set, the round's
  // kernels read the id here instead of `round`; a bump launch in front of
  // the round advances it, so a captured round replays with a fresh id
  const uint32_t* round_dev = nullptr;
  uint64_t timeout = 0;     // per wait, in wall-clock ticks (100 MHz)
  const char* in = nullptr;  // round input [S]
  char* out = nullptr;       // round output [S]
  uint32_t* err = nullptr;   // host-mapped error word: set on a timed-out wait (read by the host each round)
  // direct rounds' fixed counts table [fail_n]: zeroed by a failed wait, so
  // an output of a failed round never reads as exact (nullptr: engine rounds,
  // whose counts are poisoned behind the round instead)
  int32_t* fail_counts = nullptr;
  int64_t fail_n = 0;
  // engine-path rounds: the round's counts table [counts_n], written by the
  // last workgroup of the round's last kernel -- counts_value everywhere, or
  // 0 when a wait of this round failed (no counts fill launch behind the
  // round).  fin_ctr: this lane's finisher ticket (uncached, reset by the
  // finisher)
  int32_t* counts_out = nullptr;
  int64_t counts_n = 0;
  int32_t counts_value = 0;
  uint32_t* fin_ctr = nullptr;
};

// Flag words of one rank's flag area (uint32 index).
__host__ __device__ inline int64_t ipc_flag_push(int32_t src, int32_t j, int32_t np) {
  return (int64_t(src) * np + j) * kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_flag_reduced(int32_t j, int32_t part, int32_t N, int32_t np) {
  return (int64_t(N) * np + int64_t(j) * kIpcReduceSplit + part) * kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_flag_gather(int32_t src, int32_t j, int32_t part, int32_t N, int32_t np) {
  return (int64_t(N) * np + int64_t(kIpcReduceSplit) * np + (int64_t(src) * np + j) * kIpcReduceSplit + part) *
         kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_flag_error(int32_t N, int32_t np) {
  return (int64_t(N) * np + int64_t(kIpcReduceSplit) * np * (1 + N)) * kIpcFlagStride;
}
__host__ __device__ inline size_t ipc_flag_bytes(int32_t N, int32_t np) {
  return size_t(ipc_flag_error(N, np) + kIpcFlagStride) * sizeof(uint32_t);
}
__host__ __device__ inline int64_t ipc_window_slots(int32_t N) { return 2 * int64_t(N) + 1; }

// ---- two-sided p2p over mapped mailboxes (csrc/transport/ipc_p2p.cpp) ----
// Every rank's window holds, per (source rank, channel), `nslots` mailbox
// slots of `piece` bytes.  An op of B bytes moves as ceil(B / piece) pieces
// with consecutive sequence numbers per (pair, channel, direction); piece q
// uses slot q % nslots.  Each piece is split over `wpp` workgroups, and every
// (slot, workgroup) pair has its own round-id style flags:
//   written [src][ch][slot][w]  in the receiver's area, set by the sender;
//   consumed[dst][ch][slot][w]  in the sender's area, set by the receiver.
// A sender waits for `consumed` of piece q - nslots before reusing the slot.
constexpr int kIpcP2PMaxOps = 80;

struct IpcP2POp {
  char* buf;       // local source (send) or destination (recv)
  int64_t bytes;   // > 0
  uint32_t seq;    // first piece's sequence number
  int8_t send, peer, ch, pad;
  int64_t pad2;
};

struct IpcP2PArgs {
  char* mbox[kIpcMaxRanks];       // mailbox region of every rank, mapped here (own = local)
  uint32_t* flags[kIpcMaxRanks];  // flag area of every rank, mapped here
  uint32_t* err;                  // host-pinned: set on a timed-out wait or a dead peer
  const uint32_t* dead;           // host-pinned [N]: peers aborted by the host
  int64_t piece;
  int32_t nslots, wpp, nch, N, me, nops, nqueues;
  int32_t wpg;  // workgroups per queue actually launched (<= wpp; each serves parts w, w + wpg, ...)
  uint64_t timeout;
  int16_t qstart[kIpcP2PMaxOps + 1];  // ops of queue i: [qstart[i], qstart[i+1]), in issue order
  IpcP2POp ops[kIpcP2PMaxOps];
};

__host__ __device__ inline int64_t ipc_p2p_box(int32_t rank, int32_t ch, int32_t slot, int32_t nch, int32_t nslots) {
  return (int64_t(rank) * nch + ch) * nslots + slot;
}
__host__ __device__ inline int64_t ipc_p2p_flag_written(int32_t src, int32_t ch, int32_t slot, int32_t w, int32_t nch,
                                                        int32_t nslots, int32_t wpp) {
  return (ipc_p2p_box(src, ch, slot, nch, nslots) * wpp + w) * kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_p2p_flag_consumed(int32_t dst, int32_t ch, int32_t slot, int32_t w,
                                                         int32_t N, int32_t nch, int32_t nslots, int32_t wpp) {
  return (int64_t(N) * nch * nslots * wpp + ipc_p2p_box(dst, ch, slot, nch, nslots) * wpp + w) * kIpcFlagStride;
}
__host__ __device__ inline size_t ipc_p2p_flag_bytes(int32_t N, int32_t nch, int32_t nslots, int32_t wpp) {
  return size_t(2) * N * nch * nslots * wpp * kIpcFlagStride * sizeof(uint32_t);
}

// One group: every queue (ops sharing direction, peer and channel) gets `wpp`
// workgroups that walk its ops in order; all queues run concurrently (the
// group semantics of a grouped send/recv).
void launch_ipc_p2p_group(hipStream_t s, const IpcP2PArgs& a);
// Workgroups of the group kernel the device can hold at once (occupancy x
// CUs): every workgroup of a group must be resident together (a queue's
// workgroup may wait on a peer's, which waits on another of this group).
int32_t ipc_p2p_resident_wgs(int32_t device);

// Microbenchmark of the exact round's reduce role alone (ipc.hip): ms per launch.
// win_kind: 0 fine-grained, 1 coarse, 2 uncached window memory; max_wgs: the
// grid cap in 256-thread workgroups (IpcArgs::max_wgs).
double ipc_reduce_role_bench(int32_t N, int64_t block, int64_t portion_bytes, DType dt, bool plain, int32_t iters,
                             int32_t threads, int32_t device, int32_t win_kind = 0, bool lite = false,
                             int32_t max_wgs = 1024);

// Enqueue one round on `s`: push, reduce, then pull (bcast = 0) or, with
// bcast = 1, the reducer writes its rows into every peer's gather slot and a
// local gather copies them out.
void launch_ipc_round(hipStream_t s, const IpcArgs& a, DType dt);
// round_dev += 1 (one thread), in stream order before a device-round round.
void launch_ipc_round_bump(hipStream_t s, uint32_t* round_dev);

}  // namespace akka
