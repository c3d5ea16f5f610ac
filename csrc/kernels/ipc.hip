// gfx950 kernels of the one-sided xGMI exact round (ipc_kernels.h).
//
// Memory-model protocol (HIP / LLVM AMDGPU, system scope because producer and
// consumer sit on different devices and the bytes cross xGMI):
//   producer: its stores -> s_waitcnt vmcnt(0) in every wave -> workgroup
//             barrier -> lane 0: release fence (system) -> s_waitcnt vmcnt(0)
//             -> relaxed system-scope store (or add) of the flag word;
//   consumer: lane 0 polls the flag with relaxed system-scope loads (with
//             s_sleep) -> acquire fence (system) -> s_waitcnt vmcnt(0) ->
//             workgroup barrier -> plain loads of the payload.
// The explicit s_waitcnt after the release fence is there on purpose: the
// compiler may drop its own when it proves the scoreboard empty, letting the
// flag overtake the write-back (docs/DESIGN.md section 4f rule 2).
// Every wait is bounded (wall clock, `timeout` ticks): on expiry the waiting
// workgroup sets this rank's error word and the abort word of EVERY rank's
// flag area (wait_flag), skips its data work and still signals, so every grid
// drains and no GPU is ever left spinning.  Every rank's later waits fail on
// the abort word, its round's counts are poisoned to 0 behind the round
// (DataPlane::finalize), and its next round on the lane raises.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "ipc_kernels.h"
#include "xgmi_device.h"

namespace akka {
namespace {

constexpr int kThreads = 256;      // default workgroup size (AKKA_IPC_THREADS: 256 / 512 / 1024)
constexpr int kMaxThreads = 1024;  // launch bound of the one-sided round kernels
constexpr int kReduceSplit = kIpcReduceSplit;
using namespace xgmi;

// Lane 0 only.  true once *f reached `want` and no rank aborted the lane.
// On timeout this rank ABORTS the lane: the abort word of every rank's flag
// area is set before this workgroup signals anything (its release orders the
// stores), so a peer that sees one of this rank's flags also sees the abort
// and never consumes data this rank did not produce.  A peer's abort, or an
// earlier timeout of this rank, makes every later wait fail too; the failed
// round's counts are then poisoned to 0 (DataPlane::finalize) and the next
// round on the lane raises.
// Lane 0: this rank's round failed -- error word, and the direct rounds'
// counts table reads 0 from now on (vector stores, one lane).
__device__ void fail_round(const IpcArgs& a) {
  sys_store(a.err, 1u);
  for (int64_t i = 0; i < a.fail_n; ++i) a.fail_counts[i] = 0;
}

__device__ bool wait_flag(const IpcArgs& a, uint32_t* f, uint32_t want, uint64_t deadline) {
  uint32_t* abort_me = a.flags[a.me] + ipc_flag_error(a.N, a.nportions);
  uint32_t spins = 0;
  while (true) {
    if (reached(sys_load(f), want)) {
      // a producer that aborted stored the abort before its flag (release)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (sys_load(abort_me) != 0) {
        fail_round(a);
        return false;
      }
      return true;
    }
    if ((++spins & 63) == 0) {
      if (sys_load(a.err) != 0 || sys_load(abort_me) != 0) {
        fail_round(a);
        return false;
      }
      if (wall_clock64() > deadline) {
        fail_round(a);
        for (int32_t p = 0; p < a.N; ++p) sys_store(a.flags[p] + ipc_flag_error(a.N, a.nportions), 1u);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// This round's id: a kernel argument, or (graph-capturable rounds) the
// device word the bump launch in front of the round advanced.
__device__ inline uint32_t round_of(const IpcArgs& a) { return a.round_dev ? sys_load(a.round_dev) : a.round; }

__device__ inline void signal(uint32_t* f, uint32_t v) {  // lane 0, after release_wg
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Sum of the N sources of `n` elements, ascending source rank (source `me`
// is the round input, the others are window slots), to `o`, to `r` (pull
// mode) or, with gather_off >= 0 (bcast mode), to every peer's window at
// byte offset gather_off.
// Vector body with the source count NS known at compile time: every thread
// issues all NS x U 16-byte loads of an iteration before the first add (the
// standalone reduce kernel's structure, kernels.hip), U = 16 / NS vectors per
// source, so ~16 loads are in flight per lane whatever N is.  Slot loads are
// system-coherent buffer loads (sc0 sc1), or -- `plain_slots`, measured
// against them -- plain loads behind the workgroup's system-scope acquire.
// Same summation order as the runtime-N body (ascending source), so the
// result is bitwise identical.
template <typename T, int NS>
__device__ void reduce_vec_n(const IpcArgs& a, const char* mine, const char* slots, int64_t slot_bytes, char* o,
                             char* r, int64_t gather_off, int64_t n) {
  constexpr int PV = Elt<T>::kPerVec;
  constexpr int U = NS >= 16 ? 1 : (16 / NS);
  const int me = a.me;
  const bool bc = gather_off >= 0;
  const bool plain = a.plain_slots != 0;
  const int64_t nv = n / PV;
  const int bd = int(blockDim.x);
  for (int64_t i0 = threadIdx.x; i0 < nv; i0 += int64_t(U) * bd) {
    uint4 v[NS][U];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s == me || plain) {
        const uint4* src = reinterpret_cast<const uint4*>(s == me ? mine : slots + int64_t(s) * slot_bytes);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + int64_t(u) * bd;
          v[s][u] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
      } else {
        const auto rs = sys_rsrc(slots + int64_t(s) * slot_bytes, n * int64_t(sizeof(T)));
#pragma unroll
        for (int u = 0; u < U; ++u) v[s][u] = load_sys16(rs, (i0 + int64_t(u) * bd) * 16);  // 0 past the end
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + int64_t(u) * bd;
      float acc[PV];
#pragma unroll
      for (int e = 0; e < PV; ++e) acc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) Elt<T>::add(acc, v[s][u]);
      if (i < nv) {
        const uint4 w = Elt<T>::pack(acc);
        // my output: read by this rank only, after the round -- streamed past
        // the caches so it does not evict the slots still to be read
        store_nt16(reinterpret_cast<uint4*>(o) + i, w);
        // window bytes (read by peers): write-through with `lite`, else plain + release
        if (bc) {
#pragma unroll
          for (int p = 0; p < NS; ++p) {
            if (p == me) continue;
            if (a.lite) store_sys16(sys_rsrc(a.gdata[p] + gather_off, nv * 16), i * 16, w);
            else reinterpret_cast<uint4*>(a.gdata[p] + gather_off)[i] = w;
          }
        } else if (a.lite) {
          store_sys16(sys_rsrc(r, nv * 16), i * 16, w);
        } else {
          reinterpret_cast<uint4*>(r)[i] = w;
        }
      }
    }
  }
}

// Returns whether the window bytes it stored need a release fence before the
// flag (plain stores), i.e. false only for the write-through `lite` bodies.
// NS > 0: the kernel was instantiated for N == NS (one kernel per node rank
// count, so each gets the registers of its own body only); NS == 0: any N.
template <typename T, int NS>
__device__ bool reduce_span(const IpcArgs& a, const char* mine, const char* slots, int64_t slot_bytes, char* o,
                            char* r, int64_t gather_off, int64_t n) {
  constexpr int ES = sizeof(T);
  constexpr int PV = Elt<T>::kPerVec;
  const int N = a.N, me = a.me;
  const bool bc = gather_off >= 0;
  bool vec = ((uintptr_t(mine) | uintptr_t(slots) | uintptr_t(slot_bytes) | uintptr_t(o) | uintptr_t(r) |
               uintptr_t(bc ? gather_off : 0) | uintptr_t(n * ES)) & 15) == 0;
  if (vec) {
    if constexpr (NS > 0) {
      reduce_vec_n<T, NS>(a, mine, slots, slot_bytes, o, r, gather_off, n);
      return !a.lite;
    }
    const int64_t nv = n / PV;
    for (int64_t i0 = threadIdx.x; i0 < nv; i0 += kUnroll * int(blockDim.x)) {
      float acc[kUnroll][PV];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int e = 0; e < PV; ++e) acc[u][e] = 0.f;
      for (int s = 0; s < N; ++s) {
        uint4 v[kUnroll];
        if (s == me) {  // my own input: ordinary memory of this rank
          const uint4* src = reinterpret_cast<const uint4*>(mine);
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + int64_t(u) * int(blockDim.x);
            v[u] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
          }
        } else {  // slot s: written by rank s
          const auto r = sys_rsrc(slots + int64_t(s) * slot_bytes, n * ES);
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) v[u] = load_sys16(r, (i0 + int64_t(u) * int(blockDim.x)) * 16);  // 0 past the end
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) Elt<T>::add(acc[u], v[u]);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t i = i0 + int64_t(u) * int(blockDim.x);
        if (i < nv) {
          const uint4 w = Elt<T>::pack(acc[u]);
          reinterpret_cast<uint4*>(o)[i] = w;
          if (bc) {
            for (int p = 0; p < N; ++p)
              if (p != me) reinterpret_cast<uint4*>(a.gdata[p] + gather_off)[i] = w;
          } else {
            reinterpret_cast<uint4*>(r)[i] = w;
          }
        }
      }
    }
  } else {
    for (int64_t i = threadIdx.x; i < n; i += int(blockDim.x)) {
      float acc = 0.f;
      for (int s = 0; s < N; ++s)
        acc += s == me ? Elt<T>::load1(mine + i * ES)
                       : Elt<T>::load1_sys(sys_rsrc(slots + int64_t(s) * slot_bytes, n * ES), i * ES);
      Elt<T>::store1(o + i * ES, acc);
      if (bc) {
        for (int p = 0; p < N; ++p)
          if (p != me) Elt<T>::store1(a.gdata[p] + gather_off + i * ES, acc);
      } else {
        Elt<T>::store1(r + i * ES, acc);
      }
    }
  }
  return true;  // plain window stores (runtime-N or scalar body): release before the flag
}

// ---- the three phases of a round, one work item each ----------------------

// Portion j of my input's block p -> rank p's slot [me], then its push flag.
template <int ES>
__device__ void push_item(const IpcArgs& a, int32_t j, int32_t p) {
  const int64_t e0 = int64_t(j) * a.portion;
  const int64_t n = max(int64_t(0), min(a.portion, a.blen[p] - e0));
  char* dst = a.data[p] + (int64_t(a.me) * a.slot + e0) * ES;
  const char* src = a.in + (a.bstart[p] + e0) * ES;
  const bool lite = a.lite && ((uintptr_t(dst) | uintptr_t(src) | uintptr_t(n * ES)) & 15) == 0;
  if (n > 0) {
    if (lite) copy_out_sys(dst, src, n * ES);  // write-through: no release fence needed
    else copy_bytes(dst, src, n * ES);
  }
  if (lite) drain_wg();
  else release_wg();
  if (threadIdx.x == 0) signal(a.flags[p] + ipc_flag_push(a.me, j, a.nportions), round_of(a));
  __syncthreads();
}

// After the flag waits: every lane's verdict combined; without `lite` lane 0
// also runs the system-scope acquire (with `lite` every read of the handed-off
// bytes is a system-coherent load, which needs none).
__device__ inline bool settle_waits(const IpcArgs& a, bool ok) {
  ok = __syncthreads_and(ok ? 1 : 0) != 0;
  if (!a.lite) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  return ok;
}

// Part `part` of portion j of my block: wait for every peer's push of it, sum,
// write my output block and my `reduced` row (pull mode) or every peer's
// gather slot [me] (bcast mode), then signal.
template <typename T, int NS>
__device__ void reduce_item(const IpcArgs& a, int32_t j, int32_t part) {
  constexpr int ES = sizeof(T);
  const int32_t me = a.me, N = a.N, np = a.nportions;
  uint32_t* fl = a.flags[me];
  // each item's part of its portion (a multiple of 64 elements)
  const int64_t per = ((a.portion / kReduceSplit) + 63) / 64 * 64;
  bool ok = true;
  {
    // every peer's push flag polled by a lane of its own: the waits overlap
    const int32_t s = int32_t(threadIdx.x);
    if (s < N && s != me) ok = wait_flag(a, fl + ipc_flag_push(s, j, np), round_of(a), wall_clock64() + a.timeout);
  }
  ok = settle_waits(a, ok);
  const int64_t e0 = int64_t(j) * a.portion;
  const int64_t n = max(int64_t(0), min(a.portion, a.blen[me] - e0));
  const int64_t p0 = min(n, part * per), p1 = min(n, p0 + per);
  bool fenced = !a.lite;
  if (ok && p1 > p0) {
    const int64_t e = e0 + p0;
    fenced = reduce_span<T, NS>(a, a.in + (a.bstart[me] + e) * ES, a.data[me] + e * ES, a.slot * ES,
                                a.out + (a.bstart[me] + e) * ES, a.gdata[me] + e * ES,
                                a.bcast ? (int64_t(1 + me) * a.slot + e) * ES : int64_t(-1), p1 - p0);
  }
  if (fenced) release_wg();  // (uniform: the alignment of an item is the same for every thread)
  else drain_wg();
  if (threadIdx.x == 0) {
    if (a.bcast) {
      for (int32_t p = 0; p < N; ++p)
        if (p != me) signal(a.flags[p] + ipc_flag_gather(me, j, part, N, np), round_of(a));
    } else {
      signal(fl + ipc_flag_reduced(j, part, N, np), round_of(a));
    }
  }
  __syncthreads();  // `ok` is rewritten by the next item
}

// Rank p's reduced portion j (all its parts) -> my output's block p.  Pull
// mode reads it from rank p's window over xGMI; bcast mode finds it in my
// gather slot [p] (rank p wrote it there), the copy is local.
template <int ES>
__device__ void phase2_item(const IpcArgs& a, int32_t j, int32_t p) {
  const int32_t me = a.me, N = a.N, np = a.nportions;
  bool ok = true;
  {
    const int32_t part = int32_t(threadIdx.x);  // one lane per reduce part: the waits overlap
    if (part < kReduceSplit)
      ok = wait_flag(a, a.bcast ? a.flags[me] + ipc_flag_gather(p, j, part, N, np)
                                : a.flags[p] + ipc_flag_reduced(j, part, N, np),
                     round_of(a), wall_clock64() + a.timeout);
  }
  ok = settle_waits(a, ok);
  const int64_t e0 = int64_t(j) * a.portion;
  const int64_t n = max(int64_t(0), min(a.portion, a.blen[p] - e0));
  const char* src = a.bcast ? a.gdata[me] + (int64_t(1 + p) * a.slot + e0) * ES
                            : a.gdata[p] + e0 * ES;
  if (ok && n > 0) copy_in(a.out + (a.bstart[p] + e0) * ES, src, n * ES);
  __syncthreads();  // `ok` is rewritten by the next item
}

// Items in portion-major order (all peers of portion 0, then portion 1, ...),
// peers rotated from me + 1 so every link is busy at once.
__device__ inline int32_t item_peer(const IpcArgs& a, int32_t w) { return (a.me + 1 + w % (a.N - 1)) % a.N; }

// ---- three kernels on one stream -----------------------------------------
// push never waits; reduce and phase 2 loop over their items under a grid cap
// so that workgroups parked on flags never fill the machine (ranks sharing a
// card in tests need room for each other's push kernels).

template <int ES>
__global__ __launch_bounds__(kMaxThreads) void ipc_push_kernel(IpcArgs a) {
  const int32_t items = a.nportions * (a.N - 1);
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) push_item<ES>(a, w / (a.N - 1), item_peer(a, w));
}

// One instantiation per (dtype, rank count, launch bound): a 1024-thread bound
// caps a thread at 128 VGPRs, a 256-thread one lets the N-source body keep
// every load in registers (occupancy then follows its real VGPR count).
template <typename T, int NS, int LB>
__global__ __launch_bounds__(LB) void ipc_reduce_kernel(IpcArgs a) {
  const int32_t items = a.nportions * kReduceSplit;
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) reduce_item<T, NS>(a, w / kReduceSplit, w % kReduceSplit);
}

// Every workgroup of the round's LAST kernel, at its end: the last one out
// writes the round's counts (N, or 0 after a failed wait of this round --
// every wait of the round ended before its workgroup took a ticket) and
// resets the ticket for the next round (same stream: nothing overlaps).
__device__ void finish_counts(const IpcArgs& a) {
  if (!a.counts_out) return;
  __shared__ int32_t last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.fin_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = prev + 1u == gridDim.x ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  const int32_t v = sys_load(a.err) != 0 ? 0 : a.counts_value;
  for (int64_t i = threadIdx.x; i < a.counts_n; i += blockDim.x) a.counts_out[i] = v;
  if (threadIdx.x == 0) sys_store(a.fin_ctr, 0u);
}

template <int ES>
__global__ __launch_bounds__(kMaxThreads) void ipc_phase2_kernel(IpcArgs a) {
  const int32_t items = a.nportions * (a.N - 1);
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) phase2_item<ES>(a, w / (a.N - 1), item_peer(a, w));
  finish_counts(a);
}

// ---- one fused launch -----------------------------------------------------
// Roles by workgroup id: [0, gp) push, [gp, gp + gr) reduce, the rest phase 2.
// A reducer starts on portion j as soon as its pushes landed and phase 2 moves
// portion j while later portions are still being pushed, so the links stay
// busy across the reduce.  Deadlock-free without co-residency: workgroups are
// dispatched in id order (per XCD), pushers never wait, reducers wait only on
// (remote) pushers and phase-2 workgroups only on (remote) reducers -- every
// role depends on roles with lower ids only.
template <typename T, int NS>
__global__ __launch_bounds__(kMaxThreads) void ipc_fused_kernel(IpcArgs a, int32_t gp, int32_t gr) {
  constexpr int ES = sizeof(T);
  const int32_t b = blockIdx.x;
  if (b < gp) {
    const int32_t items = a.nportions * (a.N - 1);
    for (int32_t w = b; w < items; w += gp) push_item<ES>(a, w / (a.N - 1), item_peer(a, w));
  } else if (b < gp + gr) {
    const int32_t items = a.nportions * kReduceSplit;
    for (int32_t w = b - gp; w < items; w += gr) reduce_item<T, NS>(a, w / kReduceSplit, w % kReduceSplit);
  } else {
    const int32_t gq = int32_t(gridDim.x) - gp - gr;
    const int32_t items = a.nportions * (a.N - 1);
    for (int32_t w = b - gp - gr; w < items; w += gq) phase2_item<ES>(a, w / (a.N - 1), item_peer(a, w));
  }
  finish_counts(a);
}

template <typename T, int NS>
void launch_reduce(hipStream_t s, const IpcArgs& a, unsigned grid, unsigned nt) {
  if (nt <= unsigned(kThreads))
    hipLaunchKernelGGL((ipc_reduce_kernel<T, NS, kThreads>), dim3(grid), dim3(nt), 0, s, a);
  else
    hipLaunchKernelGGL((ipc_reduce_kernel<T, NS, kMaxThreads>), dim3(grid), dim3(nt), 0, s, a);
}

// Calls f(std::integral_constant<int, NS>) with NS = N for the node's rank
// counts (2..8, 16) and NS = 0 (runtime N) otherwise.
template <typename F>
void with_ns(int32_t N, F&& f) {
  switch (N) {
    case 2: return f(std::integral_constant<int, 2>{});
    case 3: return f(std::integral_constant<int, 3>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 5: return f(std::integral_constant<int, 5>{});
    case 6: return f(std::integral_constant<int, 6>{});
    case 7: return f(std::integral_constant<int, 7>{});
    case 8: return f(std::integral_constant<int, 8>{});
    case 16: return f(std::integral_constant<int, 16>{});
    default: return f(std::integral_constant<int, 0>{});
  }
}

template <typename T, int NS>
void launch_round(hipStream_t s, const IpcArgs& a) {
  constexpr int ES = sizeof(T);
  // workgroup size and the waiting kernels' grid cap (given in 256-thread
  // workgroups: the cap bounds parked WAVES, whatever the workgroup size)
  const int32_t nt = (a.threads == 512 || a.threads == 1024) ? a.threads : kThreads;
  const int32_t cap = std::max(1, (a.max_wgs > 0 ? a.max_wgs : 1024) * kThreads / nt);
  const int32_t push_items = a.nportions * (a.N - 1), red_items = a.nportions * kReduceSplit;
  if (a.fused) {
    // one grid of <= cap workgroups split over the roles by their work
    const int32_t total = push_items + red_items + push_items;
    const int32_t budget = std::min(cap, total);
    const int32_t gp = std::max(1, int32_t(int64_t(budget) * push_items / total));
    const int32_t gr = std::max(1, int32_t(int64_t(budget) * red_items / total));
    const int32_t gq = std::max(1, budget - gp - gr);
    hipLaunchKernelGGL((ipc_fused_kernel<T, NS>), dim3(unsigned(gp + gr + gq)), dim3(unsigned(nt)), 0, s, a, gp, gr);
    return;
  }
  hipLaunchKernelGGL(ipc_push_kernel<ES>, dim3(unsigned(push_items)), dim3(unsigned(nt)), 0, s, a);
  launch_reduce<T, NS>(s, a, unsigned(std::min(red_items, cap)), unsigned(nt));
  hipLaunchKernelGGL(ipc_phase2_kernel<ES>, dim3(unsigned(std::min(push_items, cap))), dim3(unsigned(nt)), 0, s, a);
}

// Like wait_flag, but also gives up when the host marked `peer` dead.
__device__ bool wait_flag_p2p(uint32_t* f, uint32_t want, uint32_t* err, const uint32_t* dead, int32_t peer,
                              uint64_t deadline) {
  uint32_t spins = 0;
  while (true) {
    if (reached(sys_load(f), want)) return true;
    if ((++spins & 63) == 0) {
      if (__hip_atomic_load(dead + peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return false;
      if (sys_load(err) != 0) return false;
      if (wall_clock64() > deadline) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// grid = nqueues * wpg.  Workgroup (queue, w0) moves parts w0, w0 + wpg, ...
// (< wpp) of every piece of every op of its queue, pieces in order.  Every
// wait of a send is on an EARLIER piece of the peer and every wait of a
// receive on the same piece of a send, so with all workgroups resident no
// cycle of waits exists however the parts are grouped (ipc_p2p_resident_wgs
// bounds the grid).
__global__ __launch_bounds__(kThreads) void ipc_p2p_kernel(IpcP2PArgs a) {
  const int32_t wpg = a.wpg > 0 ? a.wpg : a.wpp;
  const int32_t qi = int32_t(blockIdx.x) / wpg;
  const int32_t w0 = int32_t(blockIdx.x) % wpg;
  const int32_t me = a.me;
  for (int32_t oi = a.qstart[qi]; oi < a.qstart[qi + 1]; ++oi) {
    const IpcP2POp op = a.ops[oi];
    const int32_t peer = op.peer, ch = op.ch;
    const int64_t npieces = (op.bytes + a.piece - 1) / a.piece;
    for (int64_t k = 0; k < npieces; ++k) {
      const uint32_t seq = op.seq + uint32_t(k);
      const int32_t slot = int32_t(seq % uint32_t(a.nslots));
      const int64_t pb0 = k * a.piece;
      const int64_t pbytes = min(a.piece, op.bytes - pb0);
      const int64_t part = ((pbytes + a.wpp - 1) / a.wpp + 15) / 16 * 16;
      for (int32_t w = w0; w < a.wpp; w += wpg) {
        const int64_t b0 = min(pbytes, int64_t(w) * part), b1 = min(pbytes, b0 + part);
        bool ok = true;
        if (op.send) {
          if (threadIdx.x == 0 && seq >= uint32_t(a.nslots)) {
            const uint64_t deadline = wall_clock64() + a.timeout;
            ok = wait_flag_p2p(a.flags[me] + ipc_p2p_flag_consumed(peer, ch, slot, w, a.N, a.nch, a.nslots, a.wpp),
                               seq - uint32_t(a.nslots) + 1u, a.err, a.dead, peer, deadline);
          }
          ok = acquire_all(ok);
          if (ok && b1 > b0)
            copy_bytes(a.mbox[peer] + ipc_p2p_box(me, ch, slot, a.nch, a.nslots) * a.piece + b0, op.buf + pb0 + b0,
                       b1 - b0);
          release_wg();
          if (threadIdx.x == 0)
            signal(a.flags[peer] + ipc_p2p_flag_written(me, ch, slot, w, a.nch, a.nslots, a.wpp), seq + 1u);
        } else {
          if (threadIdx.x == 0) {
            const uint64_t deadline = wall_clock64() + a.timeout;
            ok = wait_flag_p2p(a.flags[me] + ipc_p2p_flag_written(peer, ch, slot, w, a.nch, a.nslots, a.wpp),
                               seq + 1u, a.err, a.dead, peer, deadline);
          }
          ok = acquire_all(ok);
          if (ok && b1 > b0)
            copy_in(op.buf + pb0 + b0, a.mbox[me] + ipc_p2p_box(peer, ch, slot, a.nch, a.nslots) * a.piece + b0,
                    b1 - b0);
          release_wg();
          if (threadIdx.x == 0)
            signal(a.flags[peer] + ipc_p2p_flag_consumed(me, ch, slot, w, a.N, a.nch, a.nslots, a.wpp), seq + 1u);
        }
        __syncthreads();  // `ok` is rewritten by the next part
      }
    }
  }
}

}  // namespace

void launch_ipc_p2p_group(hipStream_t s, const IpcP2PArgs& a) {
  if (a.nqueues <= 0) return;
  const int32_t wpg = a.wpg > 0 ? a.wpg : a.wpp;
  hipLaunchKernelGGL(ipc_p2p_kernel, dim3(unsigned(a.nqueues * wpg)), dim3(kThreads), 0, s, a);
}

int32_t ipc_p2p_resident_wgs(int32_t device) {
  int bpm = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpm, ipc_p2p_kernel, kThreads, 0) != hipSuccess) bpm = 4;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
  return std::max(1, bpm) * std::max(1, cus);
}

__global__ void ipc_round_bump_kernel(uint32_t* p) {
  if (threadIdx.x == 0) sys_store(p, sys_load(p) + 1u);
}

void launch_ipc_round_bump(hipStream_t s, uint32_t* round_dev) {
  hipLaunchKernelGGL(ipc_round_bump_kernel, dim3(1), dim3(64), 0, s, round_dev);
}

void launch_ipc_round(hipStream_t s, const IpcArgs& a, DType dt) {
  if (a.N < 2) return;
  with_ns(a.N, [&](auto ns) {
    if (dt == DType::F32) launch_round<float, decltype(ns)::value>(s, a);
    else launch_round<uint16_t, decltype(ns)::value>(s, a);
  });
}

}  // namespace akka

namespace akka {

// Microbenchmark of the reduce role alone (one process, local fine-grained
// windows, every push flag pre-set): the in-round reduce's bandwidth, with
// system-coherent slot loads or plain ones (`plain`).  Pull mode: reads
// N x block, writes the output block and the `reduced` row.  Returns ms per
// launch over `iters` launches.
double ipc_reduce_role_bench(int32_t N, int64_t block, int64_t portion_bytes, DType dt, bool plain, int32_t iters,
                             int32_t threads, int32_t device, int32_t win_kind, bool lite, int32_t max_wgs) {
  auto ok = [](hipError_t e, const char* w) {
    if (e != hipSuccess) throw AkkaError(std::string("akka ipc bench: ") + w + ": " + hipGetErrorString(e));
  };
  ok(hipSetDevice(device), "set device");
  const int64_t es = dt == DType::F32 ? 4 : 2;
  const int64_t slot = (block + 63) / 64 * 64;
  const int64_t portion = std::max<int64_t>(1024, portion_bytes / es / 1024 * 1024);
  const int32_t np = int32_t((block + portion - 1) / portion);
  char *data = nullptr, *gdata = nullptr, *in = nullptr, *out = nullptr;
  uint32_t *flags = nullptr, *err = nullptr, *err_dev = nullptr;
  // window memory kind: 0 fine-grained (the lane's default), 1 coarse (hipMalloc), 2 uncached
  auto walloc = [&](char** p, size_t bytes, const char* what) {
    if (win_kind == 1) ok(hipMalloc(reinterpret_cast<void**>(p), bytes), what);
    else ok(hipExtMallocWithFlags(reinterpret_cast<void**>(p), bytes,
                                  win_kind == 2 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained), what);
  };
  walloc(&data, size_t(N * slot * es), "data");
  walloc(&gdata, size_t((N + 1) * slot * es), "gdata");
  ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&flags), ipc_flag_bytes(N, np), hipDeviceMallocUncached), "flags");
  ok(hipMalloc(&in, size_t(N * block * es)), "in");
  ok(hipMalloc(&out, size_t(N * block * es)), "out");
  ok(hipHostMalloc(reinterpret_cast<void**>(&err), 4, hipHostMallocMapped | hipHostMallocCoherent), "err");
  *err = 0;
  ok(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev), err, 0), "err dev");
  ok(hipMemset(data, 0x3c, size_t(N * slot * es)), "fill");
  ok(hipMemset(in, 0x3c, size_t(N * block * es)), "fill");
  ok(hipMemset(flags, 0, ipc_flag_bytes(N, np)), "flags");
  ok(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(flags), 1, size_t(N) * np * kIpcFlagStride), "push flags");
  IpcArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int32_t p = 0; p < N; ++p) {
    a.data[p] = data;
    a.gdata[p] = gdata;
    a.flags[p] = flags;
    a.bstart[p] = int64_t(p) * block;
    a.blen[p] = block;
  }
  a.slot = slot;
  a.portion = portion;
  a.nportions = np;
  a.max_wgs = std::max(64, max_wgs);
  a.N = N;
  a.me = 0;
  a.threads = threads;
  a.plain_slots = plain ? 1 : 0;
  a.lite = lite ? 1 : 0;
  a.round = 1;
  a.timeout = uint64_t(1) << 40;
  a.in = in;
  a.out = out;
  a.err = err_dev;
  const int32_t nt = (threads == 512 || threads == 1024) ? threads : kThreads;
  const int32_t cap = std::max(1, a.max_wgs * kThreads / nt);
  const unsigned grid = unsigned(std::min(np * kReduceSplit, cap));
  hipEvent_t e0, e1;
  ok(hipEventCreate(&e0), "event");
  ok(hipEventCreate(&e1), "event");
  auto launch = [&]() {
    with_ns(N, [&](auto ns) {
      if (dt == DType::F32) launch_reduce<float, decltype(ns)::value>(nullptr, a, grid, unsigned(nt));
      else launch_reduce<uint16_t, decltype(ns)::value>(nullptr, a, grid, unsigned(nt));
    });
  };
  for (int i = 0; i < 3; ++i) launch();
  ok(hipEventRecord(e0, nullptr), "record");
  for (int i = 0; i < iters; ++i) launch();
  ok(hipEventRecord(e1, nullptr), "record");
  ok(hipEventSynchronize(e1), "sync");
  float ms = 0.f;
  ok(hipEventElapsedTime(&ms, e0, e1), "elapsed");
  const uint32_t e = *err;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(data);
  (void)hipFree(gdata);
  (void)hipFree(flags);
  (void)hipFree(in);
  (void)hipFree(out);
  (void)hipHostFree(err);
  if (e != 0) throw AkkaError("akka ipc bench: a wait failed");
  return double(ms) / std::max(1, iters);
}

}  // namespace akka
