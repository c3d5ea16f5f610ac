// One-sided xGMI exact round (ipc.hip): every rank maps every other rank's
// window (hipIpcOpenMemHandle) and the round runs as three kernels on one
// stream, no RCCL and no host round trip:
//   push    my input's block p  -> rank p's window slot [me]   (xGMI stores)
//   reduce  slots [0..N) of my block (+ my own input block)    -> my output
//           block and my window's `reduced` row               (local HBM)
//   pull    rank p's `reduced` row -> my output's block p       (xGMI loads)
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

struct IpcArgs {
  char* data[kIpcMaxRanks];       // window base of every rank, mapped in this process (own = local)
  uint32_t* flags[kIpcMaxRanks];  // flag area of every rank, mapped in this process
  int64_t bstart[kIpcMaxRanks];   // block start / length (elements)
  int64_t blen[kIpcMaxRanks];
  int64_t slot;       // elements per window slot (>= every block, 64-element multiple)
  int64_t portion;    // elements per portion (a multiple of 1024)
  int32_t nportions;  // portions per slot
  int32_t max_wgs;    // grid cap of the kernels that wait (reduce, pull)
  int32_t N = 0, me = 0;
  uint32_t round = 0;       // this round's id (1, 2, ... identical on every rank)
  uint64_t timeout = 0;     // per wait, in wall-clock ticks (100 MHz)
  const char* in = nullptr;  // round input [S]
  char* out = nullptr;       // round output [S]
};

// Flag words of one rank's flag area (uint32 index).
__host__ __device__ inline int64_t ipc_flag_push(int32_t src, int32_t j, int32_t nportions) {
  return (int64_t(src) * nportions + j) * kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_flag_reduced(int32_t j, int32_t N, int32_t nportions) {
  return (int64_t(N) * nportions + j) * kIpcFlagStride;
}
__host__ __device__ inline int64_t ipc_flag_error(int32_t N, int32_t nportions) {
  return (int64_t(N + 1) * nportions) * kIpcFlagStride;
}
__host__ __device__ inline size_t ipc_flag_bytes(int32_t N, int32_t nportions) {
  return size_t(ipc_flag_error(N, nportions) + kIpcFlagStride) * sizeof(uint32_t);
}

// Enqueue push, reduce and pull of one round on `s`.
void launch_ipc_round(hipStream_t s, const IpcArgs& a, DType dt);

}  // namespace akka
