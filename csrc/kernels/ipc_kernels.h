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

// Window of a rank, in slots of `slot` elements:
//   [0, N)        slot[src]: src's contribution to my block (pushed by src)
//   N             reduced: my reduced block (pulled by the others, pull mode)
//   [N+1, 2N+1)   gather[src]: src's reduced block (pushed by src, bcast mode)
// Flags hold round ids (stores, never counts), so the two phase-2 modes can
// alternate between rounds.
struct IpcArgs {
  char* data[kIpcMaxRanks];       // window base of every rank, mapped in this process (own = local)
  uint32_t* flags[kIpcMaxRanks];  // flag area of every rank, mapped in this process
  int64_t bstart[kIpcMaxRanks];   // block start / length (elements)
  int64_t blen[kIpcMaxRanks];
  int64_t slot;       // elements per window slot (>= every block, 64-element multiple)
  int64_t portion;    // elements per portion (a multiple of 1024)
  int32_t nportions;  // portions per slot
  int32_t max_wgs;    // grid cap of the kernels that wait (reduce, pull / gather)
  int32_t bcast = 0;  // phase 2: 0 = every rank pulls the reduced rows, 1 = the reducer pushes them
  int32_t N = 0, me = 0;
  uint32_t round = 0;       // this round's id (1, 2, ... identical on every rank)
  uint64_t timeout = 0;     // per wait, in wall-clock ticks (100 MHz)
  const char* in = nullptr;  // round input [S]
  char* out = nullptr;       // round output [S]
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

// Enqueue one round on `s`: push, reduce, then pull (bcast = 0) or, with
// bcast = 1, the reducer writes its rows into every peer's gather slot and a
// local gather copies them out.
void launch_ipc_round(hipStream_t s, const IpcArgs& a, DType dt);

}  // namespace akka
