// gfx950 kernels of the one-sided threshold lane (onesided.hip); protocol in
// onesided_protocol.h, host side in transport/onesided.{h,cpp}.
//
// One call (one round of this rank) is six launches on the caller's stream:
//   begin    1 workgroup   pick the round (catch-up over what peers announced)
//   push     (N-1)*K*P     phase 1: my input's block p -> rank p's SD[row][me]
//   decide   K_me          per chunk of my block: wait (bounded) until
//                          floor(thReduce*N) copies landed or the round is
//                          forced; record the landed mask
//   reduce   K_me*P        masked sum -> my output block and every peer's
//                          GD[row][me] (phase 2, remote stores)
//   cdecide  1             wait until floor(thComplete*total) reduced chunks
//                          landed in my GD[row] or the round is forced
//   copy     (N-1)*K*P     landed chunks GD -> output, the rest 0 / count 0
// Only decide and cdecide wait, and their grids are tiny, so no workgroup
// ever waits on a workgroup that might not be resident.  Senders never wait.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "onesided_protocol.h"

namespace akka {
namespace os {

// Pointer tables of every rank's window as mapped in THIS process (device
// memory, written once by open()).
struct Tables {
  char* sd[kMaxRows][kMaxRanks];  // scatter rows: [N][slot] elements each
  char* gd[kMaxRows][kMaxRanks];  // gather rows: [N][slot] elements each
  uint32_t* fl[kMaxRanks];        // flag areas
  int64_t bstart[kMaxRanks], blen[kMaxRanks];
  int32_t nch[kMaxRanks];
};

struct Args {
  const Tables* tab = nullptr;
  uint32_t* loc = nullptr;                 // local state (Layout local words)
  unsigned long long* stats = nullptr;     // kNumStats counters
  Layout L;
  int64_t C = 1, slot = 0, part_len = 64;  // elements
  int32_t me = 0, kme = 0, need_r = 1, need_c = 1, max_lag = 0;  // kme: chunks of my block
  int32_t kcols = 1;                       // columns of the counts table [N][kcols]
  int32_t call_slot = 0, threads = 256;
  uint64_t timeout = 0;                    // per wait, wall-clock ticks
  const char* in = nullptr;                // round input [S]
  char* out = nullptr;                     // round output [S]
  int32_t* counts = nullptr;               // [N][kcols] per-chunk contributor counts
  uint32_t* err = nullptr;                 // host-mapped: set on a timed-out wait
  const uint32_t* dead = nullptr;          // host-mapped [kMaxRanks]: peers marked dead
  const uint32_t* force = nullptr;         // host-mapped: rounds < *force are forced
  CallStatus* status = nullptr;            // host-mapped [kStatusSlots]
};

// Enqueue one call on `s` (dtype: 0 fp32, 1 bf16).
void launch_onesided_call(hipStream_t s, const Args& a, int32_t dtype);
// Announce to every peer that this rank serves no further round (fin words).
void launch_onesided_retire(hipStream_t s, const Args& a);

}  // namespace os
}  // namespace akka
