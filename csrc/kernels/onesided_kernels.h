// gfx950 kernels of the one-sided threshold lane (onesided.hip); protocol in
// onesided_protocol.h, host side in transport/onesided.{h,cpp}.
//
// One call (one round of this rank) is ONE launch on the caller's stream,
// roles by workgroup id (onesided_protocol.h, "One call"):
//   [0]                  begin: round selection, announcements
//   [1, 1+gp)            push: (N-1)*K*P parts, fire and forget
//   [.., +kme)           decide: one workgroup per chunk of my block
//   [.., +gr)            reduce: kme*P*nsub pieces, each starts when its chunk
//                        is decided
//   [.., +1)             complete: the thComplete decision, counts
//   [.., +gq)            copy: landed peer parts -> output; parts outside the
//                        completion set -> 0
// The last workgroup out finishes the call (announcements withdrawn, stats,
// status record, call id + 1).
// Deadlock-free without co-residency: workgroups are dispatched in id order,
// every role waits only on roles with lower ids (or on peers' pushers, which
// never wait), and every wait is bounded by the lane's timeout.
// The call id and the round live in device memory (kCallSeq, kCur): the
// launches' arguments are the same every call, so a call can be captured in
// a HIP graph and replayed.
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
  uint32_t* loc = nullptr;                 // local state (Layout local words), uncached device memory
  unsigned long long* stats = nullptr;     // kNumStats counters
  Layout L;
  int64_t C = 1, slot = 0, part_len = 64;  // elements
  int32_t me = 0, kme = 0, need_r = 1, need_c = 1, max_lag = 0;  // kme: chunks of my block
  int32_t kcols = 1;                       // columns of the counts table [N][kcols]
  int32_t threads = 1024;
  int32_t gp = 1, gr = 1, gq = 1;          // push / reduce / copy workgroups
  int32_t nsub = 1;                        // reduce pieces per part
  // my own output block is written through (sc0 sc1) instead of streamed:
  // when a round can complete without my chunk (thComplete < 1), a copy
  // workgroup on another XCD zeroes it after its reduce pieces -- two XCDs'
  // L2s holding the same dirty lines would write back in any order
  int32_t own_wt = 0;
  // hand-off mode of window bytes: 0 "lite" (write-through stores + drain
  // before the flag, system-coherent loads), 1 "fenced" (plain stores, a
  // system-scope release before every flag, a system-scope acquire after
  // every observed flag: the HIP memory model's protocol, xgmi_device.h)
  int32_t fenced = 0;
  // window output: the call's output is the gather row (call id % D) of my
  // own window (exact rounds; `out` unused), see os_round_kernel
  int32_t wo = 0;
  uint64_t timeout = 0;                 // per wait, wall-clock ticks
  const char* in = nullptr;                // round input [S]
  char* out = nullptr;                     // round output [S]
  int32_t* counts = nullptr;               // [N][kcols] per-chunk contributor counts
  uint32_t* err = nullptr;                 // host-mapped: set on a timed-out wait
  const uint32_t* dead = nullptr;          // host-mapped [kMaxRanks]: peers marked dead
  const uint32_t* force = nullptr;         // host-mapped: rounds < *force are forced
  CallStatus* status = nullptr;            // host-mapped [kStatusSlots]
  // measurement (AKKA_OS_TIMELINE=1): per workgroup [entry, round known,
  // role done] wall-clock ticks of the last call; nullptr otherwise
  unsigned long long* tl = nullptr;
};

// Enqueue one call on `s` (dtype: 0 fp32, 1 bf16).
void launch_onesided_call(hipStream_t s, const Args& a, int32_t dtype);
// Announce to every peer that this rank serves no further round (fin words).
void launch_onesided_retire(hipStream_t s, const Args& a);
// Workgroups of the round launch for these role sizes.
inline int32_t onesided_grid(const Args& a) { return 1 + a.gp + a.kme + a.gr + 1 + a.gq; }

// Microbenchmark of the reduce role alone (one process, local windows, every
// decision pre-set, no peer gated): N sources of `block` elements, `parts`
// (elements) per part, `nsub` pieces each.  Returns ms per launch.
double onesided_reduce_role_bench(int32_t N, int64_t block, int64_t chunk, int64_t part, int32_t nsub, int32_t dtype,
                                  int32_t threads, int32_t grid, int32_t iters, int32_t device);

}  // namespace os
}  // namespace akka
