// gfx950 kernels of the one-sided threshold lane (onesided_kernels.h).
//
// The protocol decisions (tags, gates, verdicts, round selection) are the
// functions of onesided_protocol.h, shared with the CPU backend; this file
// maps them onto the roles of one launch and moves the bytes.
//
// Hand-offs are fence-free ("lite", docs/DESIGN.md section 4f rule 3):
// every byte a peer reads is stored write-through (sc0 sc1)
// or read system-coherent (sc0 sc1 loads), each storing wave drains
// (s_waitcnt vmcnt(0)) before its workgroup's flag store, and flag / local
// words live in uncached memory, accessed with system-scope atomics -- so a
// store followed by s_waitcnt vmcnt(0) is performed before any later load
// issues (the announce -> look hand-shake).  No buffer_wbl2 / buffer_inv on
// the aligned paths; unaligned spans (odd chunk sizes) fall back to plain
// stores + a system release.
//
// Args::fenced selects the conservative twin for every span: plain stores, a
// system-scope release (cache write-back) before each flag store and a
// system-scope acquire after each observed flag (xgmi_device.h release_wg /
// acquire) -- the ordering the HIP memory model guarantees across devices,
// for links where write-through + drain is not known to order data before
// the flag.  Both modes share the tags, so ranks may differ in mode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

#include "onesided_kernels.h"
#include "xgmi_device.h"

namespace akka {
namespace os {
namespace {

using namespace xgmi;

constexpr int kMaxThreads = 1024;

// Memory policy of the protocol functions on the device (flag words: own or a
// peer's, over xGMI; both uncached, system-scope atomics).
struct DevMem {
  __device__ static uint32_t ld(const uint32_t* p) { return sys_load(p); }
  __device__ static void st(uint32_t* p, uint32_t v) { sys_store(p, v); }
  // announce, then look: the store is performed before the next load issues
  __device__ static void st_sc(uint32_t* p, uint32_t v) {
    sys_store(p, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __device__ static uint32_t ld_sc(const uint32_t* p) { return sys_load(p); }
};

__device__ inline uint64_t ld64(const uint32_t* p) {
  return __hip_atomic_load(reinterpret_cast<uint64_t*>(const_cast<uint32_t*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st64(uint32_t* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline uint32_t add_loc(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline void stat_add(const Args& a, int32_t i, unsigned long long v) {
  if (v) atomicAdd(a.stats + i, v);
}

__device__ inline void set_err(const Args& a) { sys_store(a.err, 1u); }

// A work item: part j of chunk k of block p.
struct Item {
  int32_t p, k, j;
};

// Part j of chunk k of block p: element offset inside the block and length.
__device__ inline int64_t part_len_of(const Args& a, int32_t p, int32_t k, int32_t j) {
  const int64_t clen = min(a.C, a.tab->blen[p] - int64_t(k) * a.C);
  return max(int64_t(0), min(a.part_len, clen - int64_t(j) * a.part_len));
}
__device__ inline int64_t part_off(const Args& a, int32_t k, int32_t j) {
  return int64_t(k) * a.C + int64_t(j) * a.part_len;
}

// One thread: wait until no peer is still storing into gather row `row` of my
// window (writer_in_flight) -- every part of every peer block, or only part
// (k, j) of block p when p >= 0.  Bounded by the lane's timeout (a writer that
// died mid-copy): then the error is flagged and the caller goes on.
__device__ void wait_row_writers(const Args& a, const uint32_t* fl, int32_t row, int32_t p0, int32_t kj) {
  const Layout& L = a.L;
  const uint64_t deadline = wall_clock64() + a.timeout;
  for (int32_t p = p0 < 0 ? 0 : p0; p < (p0 < 0 ? L.N : p0 + 1); ++p) {
    if (p == a.me) continue;
    for (int32_t c = kj < 0 ? 0 : kj; c < (kj < 0 ? a.tab->nch[p] * L.P : kj + 1); ++c) {
      while (writer_in_flight(DevMem::ld(fl + L.gtag(row, p, c / L.P, c % L.P)), row, L.D)) {
        if (wall_clock64() > deadline) {
          set_err(a);
          return;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
}

// ---- begin (workgroup 0): round selection (catch-up), announcements --------------
__device__ void begin_role(const Args& a) {
  if (threadIdx.x != 0) return;
  const Layout& L = a.L;
  uint32_t* fl = a.tab->fl[a.me];
  uint32_t* loc = a.loc;
  const uint32_t seq = sys_load(loc + L.state(kCallSeq));
  const uint32_t next = sys_load(loc + L.state(kNext));
  const int64_t sm = seen_max<DevMem>(fl, L, a.me);
  const uint32_t r = select_round(next, sm, a.max_lag);
  stat_add(a, kSkippedRounds, r - next);
  sys_store(loc + L.state(kCur), r);
  sys_store(loc + L.state(kNext), r + 1u);
  sys_store(loc + L.state(kCtrFinish), 0u);
  sys_store(loc + L.state(kForcedChunks), 0u);
  // rounds skipped by catch-up count as completed for the senders' outdated check
  if (DevMem::ld(fl + L.done()) < r) DevMem::st(fl + L.done(), r);
  // from now on this call reads its gather row: announce before any copy
  // workgroup looks at a tag (the overwrite hand-shake)
  const int32_t row = int32_t(r % uint32_t(L.D));
  DevMem::st_sc(fl + L.gread(row), r + 1u);
  const int32_t vrow = int32_t(seq % uint32_t(L.D));
  if (a.wo && vrow != row) {
    // window output of a call that caught up: its result is row vrow (the
    // call id's), not the served round's row.  Announce that row too -- later
    // writers of its rounds drop -- and let any writer that passed its gate
    // before the announcement finish before a byte of the result is written
    DevMem::st_sc(fl + L.gread(vrow), r + 1u);
    wait_row_writers(a, fl, vrow, -1, -1);
  }
  sys_store(loc + L.state(kBegun), seq + 1u);
}

// Every other role: wait for begin, return the call's round and call id.
__device__ uint2 wait_begun(const Args& a) {
  __shared__ uint32_t r_s, seq_s;
  if (threadIdx.x == 0) {
    const uint32_t seq = sys_load(a.loc + a.L.state(kCallSeq));
    while (sys_load(a.loc + a.L.state(kBegun)) != seq + 1u) __builtin_amdgcn_s_sleep(1);
    r_s = sys_load(a.loc + a.L.state(kCur));
    seq_s = seq;
  }
  __syncthreads();
  return make_uint2(r_s, seq_s);
}

// ---- push: phase 1, fire and forget -----------------------------------------------
// The gates of a workgroup's items run first, one lane per item, so their
// remote round trips (owner's fired word, the writing marker, its read
// announcement: ~µs each over xGMI) overlap instead of preceding every copy;
// then the workgroup copies its items one by one.
constexpr int kGateBatch = 256;
// 16-B vectors per thread per batch of a push (copy_out_sys): 128 B, twice
// the default, half the waits for write-through acks per part -- for the
// xGMI acks of a node; on one card the batch size does not matter
// (profiles/r05/push_batch/; 16 puts some round kernels on scratch)
constexpr int kPushUnroll = 8;

template <int ES>
__device__ void push_role(const Args& a, uint32_t r, int32_t w0, int32_t stride) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P;
  const int32_t items = (N - 1) * L.Kmax * P;
  const int32_t row = int32_t(r % uint32_t(L.D));
  __shared__ int8_t go_s[kGateBatch];
  // chunk-major, peers rotated from me + 1: a chunk lands everywhere early
  // (its owner can reduce it while later chunks are still moving) and
  // consecutive workgroups feed different links
  auto item = [&](int32_t w) {
    const int32_t i = w % (N - 1), kj = w / (N - 1);
    return Item{(a.me + 1 + i) % N, kj / P, kj % P};
  };
  for (int32_t base = w0; base < items; base += stride * kGateBatch) {
    for (int32_t t = threadIdx.x; t < kGateBatch; t += blockDim.x) {
      const int32_t w = base + t * stride;
      int32_t g = -1;  // no such item / no such chunk
      if (w < items) {
        const auto [p, k, j] = item(w);
        if (k < a.tab->nch[p]) {
          g = kDead;
          if (!sys_load(a.dead + p)) {
            uint32_t* ofl = a.tab->fl[p];
            if (k == 0 && j == 0) DevMem::st(ofl + L.seen(a.me), r + 1u);  // implicit start at the owner
            g = scatter_gate<DevMem>(ofl, L, row, a.me, k, j, r);
          }
          stat_add(a, g == kGo ? kScatterPushed : g == kOutdated ? kScatterOutdated
                                                  : g == kConflict ? kScatterConflict : kDeadSkips, 1);
        }
      }
      go_s[t] = int8_t(g);
    }
    __syncthreads();
    for (int32_t t = 0; t < kGateBatch; ++t) {
      const int32_t w = base + t * stride;
      if (w >= items) break;
      if (go_s[t] != kGo) continue;  // uniform over the workgroup
      const auto [p, k, j] = item(w);
      const int64_t n = part_len_of(a, p, k, j);
      const int64_t off = part_off(a, k, j);
      char* dst = a.tab->sd[row][p] + (int64_t(a.me) * a.slot + off) * ES;
      const char* src = a.in + (a.tab->bstart[p] + off) * ES;
      const bool lite = !a.fenced && ((uintptr_t(dst) | uintptr_t(src) | uintptr_t(n * ES)) & 15) == 0;
      if (n > 0) {
        if (lite) copy_out_sys<kPushUnroll>(dst, src, n * ES);
        else copy_bytes(dst, src, n * ES);
      }
      if (lite) drain_wg();
      else release_wg();
      if (threadIdx.x == 0) DevMem::st(a.tab->fl[p] + L.stag(row, a.me, k, j), tag_done(r));
    }
    __syncthreads();  // go_s is rewritten by the next batch
  }
}

// ---- decide: reduce threshold of chunk k of my block, then the phase-2 gates ----
__device__ void decide_role(const Args& a, uint32_t r, int32_t k) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  __shared__ int32_t dn[kMaxRanks], lost[kMaxRanks];
  __shared__ int32_t verdict;
  __shared__ uint32_t mask_s;
  __shared__ uint32_t okq_s[kMaxParts];
  if (threadIdx.x == 0) DevMem::st_sc(fl + L.sread(row, k), r + 1u);  // announce before looking
  if (threadIdx.x < kMaxParts) okq_s[threadIdx.x] = 0u;
  __syncthreads();
  const uint64_t deadline = wall_clock64() + a.timeout;
  while (true) {
    if (threadIdx.x < kMaxRanks) {
      const int32_t s = threadIdx.x;
      dn[s] = 0;
      // read before the tags (source_past): then a non-"done" tag is final
      lost[s] = s < N && s != me && source_past<DevMem>(fl, L, s, r) ? 1 : 0;
    }
    __syncthreads();
    for (int32_t i = threadIdx.x; i < N * P; i += blockDim.x) {
      const int32_t s = i / P, j = i % P;
      if (s == me) continue;
      const int32_t st = tag_state(DevMem::ld(fl + L.stag(row, s, k, j)), r);
      if (st == kLanded) atomicAdd(&dn[s], 1);
      else if (st == kLost) atomicOr(&lost[s], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int32_t landed = 1, pending = 0;  // my own copy is always there (self-delivery, W:228-232)
      uint32_t mask = 1u << me;
      for (int32_t s = 0; s < N; ++s) {
        if (s == me) continue;
        if (dn[s] == P) {
          ++landed;
          mask |= 1u << s;
        } else if (!lost[s] && !sys_load(a.dead + s)) {
          ++pending;
        }
      }
      verdict = evaluate(landed, pending, a.need_r, r, seen_max<DevMem>(fl, L, me), a.max_lag, sys_load(a.force),
                         wall_clock64() > deadline);
      // the round completed without this chunk: like the reference, which
      // drops scatters of a completed round (W:155-156), it is never reduced
      if (verdict == kWait && sys_load(a.loc + L.state(kComp)) == r + 1u) verdict = kAbandoned;
      mask_s = verdict == kAbandoned ? 0u : mask;
    }
    __syncthreads();
    if (verdict != kWait) break;
    __builtin_amdgcn_s_sleep(8);
  }
  const uint32_t mask = mask_s;
  if (verdict == kAbandoned) {
    if (threadIdx.x == 0) {
      DevMem::st(fl + L.fired(row, k), r + 1u);
      stat_add(a, kReduceAbandoned, 1);
    }
    if (threadIdx.x < P) sys_store(a.loc + L.okq(k, threadIdx.x), 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st64(a.loc + L.dec(k), uint64_t(r + 1u));  // empty mask: the pieces skip
    return;
  }
  if (threadIdx.x == 0) {
    DevMem::st(fl + L.fired(row, k), r + 1u);  // late senders of round <= r now skip
    if (verdict == kThreshold) {
      stat_add(a, kReduceThreshold, 1);
    } else {
      stat_add(a, kReduceForced, 1);
      add_loc(a.loc + L.state(kForcedChunks), 1u);
    }
    if (verdict == kTimeout) {
      stat_add(a, kTimeouts, 1);
      set_err(a);
    }
    stat_add(a, kReduceContribs, __popc(mask));
  }
  // phase-2 gates of every (part, peer), one lane each: the remote round
  // trips overlap instead of running per reduce piece
  const uint32_t cnt = uint32_t(__popc(mask));
  for (int32_t t = threadIdx.x; t < P * (N - 1); t += blockDim.x) {
    const int32_t j = t / (N - 1), qi = t % (N - 1);
    const int32_t q = (me + 1 + qi) % N;
    if (sys_load(a.dead + q)) {
      stat_add(a, kDeadSkips, 1);
      continue;
    }
    uint32_t* qfl = a.tab->fl[q];
    if (k == 0 && j == 0) DevMem::st(qfl + L.seen(me), r + 1u);
    const int32_t g = gather_gate<DevMem>(qfl, L, row, me, k, j, r);
    if (g == kGo) {
      DevMem::st(qfl + L.gtag(row, me, k, j) + 1, cnt);  // count, performed before the "done" tag
      atomicOr(&okq_s[j], 1u << q);
      stat_add(a, kGatherPushed, 1);
    } else {
      stat_add(a, g == kOutdated ? kGatherOutdated : kGatherConflict, 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < P) sys_store(a.loc + L.okq(k, threadIdx.x), okq_s[threadIdx.x]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st64(a.loc + L.dec(k), (uint64_t(mask) << 32) | uint64_t(r + 1u));
}

// ---- reduce: masked sum of the landed set, phase-2 pushes ------------------------
// Sources in ascending rank order (the exact lanes' order): my own input
// (plain loads), peers' SD slots (system-coherent loads).  Destinations: my
// output block (nontemporal: nobody reads it in this launch) and GD[row][me]
// of every peer in `okq` (write-through).  Vector body with the rank count
// NS known at compile time: every thread issues the loads of all landed
// sources (U vectors each) before the first add; a source outside `mask`
// reads as zeros without a load (the branch is uniform).  Same ascending-
// source order as the runtime-N body, so the sums are bitwise identical.
template <typename T, int NS>
__device__ void masked_sum_n(const Args& a, const char* mine, const char* sd, char* o, int64_t goff, int32_t row,
                             uint32_t mask, uint32_t okq, int64_t off, int64_t n) {
  constexpr int ES = sizeof(T);
  constexpr int PV = Elt<T>::kPerVec;
  // <= 4 vectors per source: beyond that the mask-dependent bodies of small N
  // spill at the 1024-thread bound (128 VGPRs)
  constexpr int U = NS >= 16 ? 1 : (16 / NS > 4 ? 4 : 16 / NS);
  const int32_t me = a.me;
  const int64_t nv = n / PV;
  const int bd = int(blockDim.x);
  for (int64_t i0 = threadIdx.x; i0 < nv; i0 += int64_t(U) * bd) {
    uint4 v[NS][U];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (!((mask >> s) & 1u)) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[s][u] = make_uint4(0, 0, 0, 0);
      } else if (s == me) {
        const uint4* src = reinterpret_cast<const uint4*>(mine);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = i0 + int64_t(u) * bd;
          v[s][u] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
      } else {
        const auto rs = sys_rsrc(sd + (int64_t(s) * a.slot + off) * ES, n * ES);
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
      for (int s = 0; s < NS; ++s)
        if ((mask >> s) & 1u) Elt<T>::add(acc, v[s][u]);
      if (i < nv) {
        const uint4 w = Elt<T>::pack(acc);
        if (a.own_wt) store_sys16(sys_rsrc(o, nv * 16), i * 16, w);
        else store_nt16(reinterpret_cast<uint4*>(o) + i, w);
        if (a.fenced) {  // plain stores, released before the tags (reduce_piece)
#pragma unroll
          for (int q = 0; q < NS; ++q)
            if ((okq >> q) & 1u) reinterpret_cast<uint4*>(a.tab->gd[row][q] + goff)[i] = w;
        } else {
#pragma unroll
          for (int q = 0; q < NS; ++q)
            if ((okq >> q) & 1u) store_sys16(sys_rsrc(a.tab->gd[row][q] + goff, nv * 16), i * 16, w);
        }
      }
    }
  }
}

// NS > 0: instantiated for N == NS (one kernel per node rank count);
// NS == 0: any N.  Returns whether the window stores need a release fence
// before the tags (plain stores: runtime-N and unaligned bodies).
template <typename T, int NS>
__device__ bool masked_sum(const Args& a, char* out, int32_t row, uint32_t mask, uint32_t okq, int64_t off, int64_t n) {
  constexpr int ES = sizeof(T);
  constexpr int PV = Elt<T>::kPerVec;
  const int32_t N = a.L.N, me = a.me;
  const char* mine = a.in + (a.tab->bstart[me] + off) * ES;
  const char* sd = a.tab->sd[row][me];
  char* o = out + (a.tab->bstart[me] + off) * ES;
  const int64_t goff = (int64_t(me) * a.slot + off) * ES;  // same offset in every peer's GD row
  const uintptr_t al = uintptr_t(mine) | uintptr_t(o) | uintptr_t(n * ES) | uintptr_t(goff) | uintptr_t(off * ES) |
                       uintptr_t(a.slot * ES);
  if ((al & 15) == 0) {
    if constexpr (NS > 0) {
      masked_sum_n<T, NS>(a, mine, sd, o, goff, row, mask, okq, off, n);
      return a.fenced != 0;
    }
    const int64_t nv = n / PV;
    for (int64_t i0 = threadIdx.x; i0 < nv; i0 += kUnroll * int(blockDim.x)) {
      float acc[kUnroll][PV];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int e = 0; e < PV; ++e) acc[u][e] = 0.f;
      for (int32_t s = 0; s < N; ++s) {
        if (!((mask >> s) & 1u)) continue;
        uint4 v[kUnroll];
        if (s == me) {
          const uint4* src = reinterpret_cast<const uint4*>(mine);
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + int64_t(u) * int(blockDim.x);
            v[u] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
          }
        } else {
          const auto rs = sys_rsrc(sd + (int64_t(s) * a.slot + off) * ES, n * ES);
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) v[u] = load_sys16(rs, (i0 + int64_t(u) * int(blockDim.x)) * 16);
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
          for (int32_t q = 0; q < N; ++q)
            if ((okq >> q) & 1u) reinterpret_cast<uint4*>(a.tab->gd[row][q] + goff)[i] = w;
        }
      }
    }
  } else {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
      float acc = 0.f;
      for (int32_t s = 0; s < N; ++s) {
        if (!((mask >> s) & 1u)) continue;
        acc += s == me ? Elt<T>::load1(mine + i * ES)
                       : Elt<T>::load1_sys(sys_rsrc(sd + (int64_t(s) * a.slot + off) * ES, n * ES), i * ES);
      }
      Elt<T>::store1(o + i * ES, acc);
      for (int32_t q = 0; q < N; ++q)
        if ((okq >> q) & 1u) Elt<T>::store1(a.tab->gd[row][q] + goff + i * ES, acc);
    }
  }
  return true;
}

// Piece s of part j of my chunk k, once the chunk is decided.
template <typename T, int NS>
__device__ void reduce_piece(const Args& a, char* out, uint32_t r, int32_t k, int32_t j, int32_t s,
                             bool wait_decision) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t row = int32_t(r % uint32_t(L.D));
  __shared__ uint32_t mask_s, okq_s;
  if (threadIdx.x == 0) {
    uint64_t d = ld64(a.loc + L.dec(k));
    bool gated = true;
    if (wait_decision) {
      // the decider is a lower workgroup id and ends every wait itself; the
      // bound here only guards against a broken decider: then nothing is
      // reduced or pushed (no gate ran for this round)
      const uint64_t deadline = wall_clock64() + 2 * a.timeout + 1;
      while (uint32_t(d) != r + 1u) {
        if (wall_clock64() > deadline) {
          set_err(a);
          d = uint64_t(r + 1u);
          gated = false;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        d = ld64(a.loc + L.dec(k));
      }
    }
    mask_s = uint32_t(d >> 32);
    okq_s = gated ? sys_load(a.loc + L.okq(k, j)) : 0u;
    if (a.fenced) {  // the decision stands for the landed tags: acquire before reading their bytes
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  const int64_t n = part_len_of(a, me, k, j);
  const int64_t per = ((n + a.nsub - 1) / a.nsub + 63) / 64 * 64;
  const int64_t lo = min(n, int64_t(s) * per), hi = min(n, lo + per);
  bool fenced = false;
  if (hi > lo && mask_s != 0u) fenced = masked_sum<T, NS>(a, out, row, mask_s, okq_s, part_off(a, k, j) + lo, hi - lo);
  // (uniform: the alignment of a piece is the same for every thread)
  if (fenced) release_wg();
  else drain_wg();
  if (threadIdx.x == 0) {
    // the last piece of the part publishes it: every other piece's stores
    // were performed before its increment, which this one observed
    if ((add_loc(a.loc + L.pctr(k, j), 1u) + 1u) % uint32_t(a.nsub) == 0u) {
      const uint32_t okq = okq_s;
      for (int32_t q = 0; q < N; ++q)
        if ((okq >> q) & 1u) DevMem::st(a.tab->fl[q] + L.gtag(row, me, k, j), tag_done(r));
      sys_store(a.loc + L.pdone(k, j), r + 1u);  // my output span of this part is final
      if ((add_loc(a.loc + L.kctr(k), 1u) + 1u) % uint32_t(P) == 0u && mask_s != 0u)
        sys_store(a.loc + L.odone(k), r + 1u);  // chunk k reduced: it counts towards my completion
    }
  }
  __syncthreads();  // mask_s / okq_s are rewritten by the next piece
}

template <typename T, int NS>
__device__ void reduce_role(const Args& a, char* out, uint32_t r, int32_t w0, int32_t stride) {
  const int32_t P = a.L.P, ns = a.nsub;
  const int32_t items = a.kme * P * ns;
  for (int32_t w = w0; w < items; w += stride) {
    const int32_t k = w / (P * ns), j = (w / ns) % P, s = w % ns;
    reduce_piece<T, NS>(a, out, r, k, j, s, true);
  }
}

// State of peer chunk (p, k) of round r from its P gather tags: lost if any
// part is lost, else pending if any is, else landed.  The tags are loaded in
// batches of 8 before any is looked at (independent uncached loads in
// flight together): one thread scans a whole chunk, and a chunk of many parts
// must not cost one memory latency per part.
__device__ inline int32_t chunk_tags_state(const uint32_t* fl, const Layout& L, int32_t row, int32_t p, int32_t k,
                                           uint32_t r) {
  constexpr int kBatch = 8;
  int32_t st = kLanded;
  for (int32_t j0 = 0; j0 < L.P; j0 += kBatch) {
    uint32_t t[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) t[u] = j0 + u < L.P ? DevMem::ld(fl + L.gtag(row, p, k, j0 + u)) : tag_done(r);
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      const int32_t s = tag_state(t[u], r);
      if (s == kLost) return kLost;
      if (s == kPending) st = kPending;
    }
  }
  return st;
}

// ---- complete: the thComplete decision -------------------------------------------
__device__ void complete_role(const Args& a, uint32_t r) {
  const Layout& L = a.L;
  const int32_t N = L.N, me = a.me, K = L.Kmax;
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  __shared__ int32_t landed_s, pending_s, own_s, verdict;
  __shared__ int32_t past[kMaxRanks];
  const uint64_t deadline = wall_clock64() + a.timeout;
  const uint64_t hard = deadline + a.timeout;  // own reduces are bounded by their own waits
  while (true) {
    if (threadIdx.x == 0) {
      landed_s = 0;
      pending_s = 0;
      own_s = 0;
    }
    if (threadIdx.x < kMaxRanks) {
      const int32_t p = threadIdx.x;
      past[p] = p < N && p != me && source_past<DevMem>(fl, L, p, r) ? 1 : 0;  // before the tags
    }
    __syncthreads();
    int32_t my_l = 0, my_p = 0, my_o = 0;
    for (int32_t c = threadIdx.x; c < N * K; c += blockDim.x) {
      const int32_t p = c / K, k = c % K;
      if (k >= a.tab->nch[p]) continue;
      if (p == me) {
        my_o += sys_load(a.loc + L.odone(k)) == r + 1u;
        continue;
      }
      int32_t st = chunk_tags_state(fl, L, row, p, k, r);
      if (st == kPending && (past[p] || sys_load(a.dead + p))) st = kLost;
      my_l += st == kLanded;
      my_p += st == kPending;
    }
    if (my_l) atomicAdd(&landed_s, my_l);
    if (my_p) atomicAdd(&pending_s, my_p);
    if (my_o) atomicAdd(&own_s, my_o);
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t now = wall_clock64();
      verdict = completion_verdict(landed_s, pending_s, own_s, a.kme, a.need_c, r, seen_max<DevMem>(fl, L, me),
                                   a.max_lag, sys_load(a.force), now > deadline);
      if (verdict == kWait && now > hard) verdict = kTimeout;
    }
    __syncthreads();
    if (verdict != kWait) break;
    __builtin_amdgcn_s_sleep(8);
  }
  // The output set: every chunk whose parts all landed (peers) / that is
  // reduced (mine) -- read once more now, so chunks that landed while the
  // verdict was being reached are kept (they are final: "done r" tags under
  // this call's gather-row announcement).
  int32_t my_l = 0;
  for (int32_t c = threadIdx.x; c < N * K; c += blockDim.x) {
    const int32_t p = c / K, k = c % K;
    if (k >= a.tab->nch[p]) continue;
    bool in;
    if (p == me) {
      in = sys_load(a.loc + L.odone(k)) == r + 1u;
    } else {
      in = chunk_tags_state(fl, L, row, p, k, r) == kLanded;
    }
    sys_store(a.loc + L.cmask(p, k), in ? 1u : 0u);
    // the output's per-chunk contributor counts (0 outside the output set)
    int32_t cnt = 0;
    if (in) cnt = p == me ? __popc(uint32_t(ld64(a.loc + L.dec(k)) >> 32))
                          : int32_t(DevMem::ld(fl + L.gtag(row, p, k, 0) + 1));
    a.counts[int64_t(p) * a.kcols + k] = cnt;
    my_l += in;
  }
  if (threadIdx.x == 0) landed_s = 0;
  __syncthreads();
  if (my_l) atomicAdd(&landed_s, my_l);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    sys_store(a.loc + L.state(kCompReason), uint32_t(verdict));
    sys_store(a.loc + L.state(kCompLanded), uint32_t(landed_s));
    stat_add(a, verdict == kThreshold ? kCompleteThreshold : kCompleteForced, 1);
    if (verdict == kTimeout) {
      stat_add(a, kTimeouts, 1);
      set_err(a);
    }
    DevMem::st(fl + L.done(), r + 1u);  // senders of round <= r now skip me
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sys_store(a.loc + L.state(kComp), r + 1u);  // the copy workgroups may read cmask
  }
}

// ---- copy: a peer's part -> my output as soon as it lands ------------------------
// Then, once the output set is published, every part of this workgroup's
// items (peer parts and, past them, my own block's parts) that is outside it
// is zeroed -- a part copied early of a chunk that did not complete, a part
// that never landed, my own chunk reduced too late -- so the zeroing is
// spread over the copy workgroups instead of a pass of its own.
template <int ES>
__device__ void copy_role(const Args& a, char* out, bool in_place, uint32_t r, int32_t w0, int32_t stride) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t peer_items = (N - 1) * L.Kmax * P;
  const int32_t items = peer_items + a.kme * P;
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  __shared__ int32_t act;
  auto item = [&](int32_t w) {
    if (w < peer_items) {
      const int32_t i = w % (N - 1), kj = w / (N - 1);
      return Item{(me + 1 + i) % N, kj / P, kj % P};
    }
    return Item{me, (w - peer_items) / P, (w - peer_items) % P};
  };
  // (window output, in place: the peers' parts landed at their final offsets)
  for (int32_t w = in_place ? peer_items : w0; w < peer_items; w += stride) {
    const auto [p, k, j] = item(w);
    if (k >= a.tab->nch[p]) continue;
    if (threadIdx.x == 0) {
      const uint64_t deadline = wall_clock64() + 3 * a.timeout + 1;
      int32_t v = 0;
      while (true) {
        // landed: copy now.  Anything else waits for the output set: a tag a
        // later round's writer marked after a conflict says "lost" although
        // this round's bytes are intact, and the complete role may already
        // have counted them in
        if (tag_state(DevMem::ld(fl + L.gtag(row, p, k, j)), r) == kLanded) {
          v = 1;
          if (a.fenced) {  // acquire after the observed tag, before the bytes
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          break;
        }
        if (sys_load(a.loc + L.state(kComp)) == r + 1u) {
          v = sys_load(a.loc + L.cmask(p, k)) != 0u ? 1 : 0;
          if (v && a.fenced) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          break;
        }
        if (wall_clock64() > deadline) {
          set_err(a);
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      act = v;
    }
    __syncthreads();
    const int64_t n = part_len_of(a, p, k, j);
    if (act && n > 0) {
      const int64_t off = part_off(a, k, j);
      copy_in(out + (a.tab->bstart[p] + off) * ES, a.tab->gd[row][me] + (int64_t(p) * a.slot + off) * ES, n * ES);
    }
    __syncthreads();  // `act` is rewritten by the next item
  }
  // the output set (the complete role is a lower workgroup id)
  // (a flag of its own: lane 0 rewrites `act` for the first zeroing item
  // below while slower waves may still be reading this verdict -- with `act`
  // reused, a wave could take that item's 0 for "no output set", return, and
  // leave its share of every later item unzeroed)
  __shared__ int32_t set_ok;
  if (threadIdx.x == 0) {
    const uint64_t deadline = wall_clock64() + 3 * a.timeout + 1;
    int32_t v = 1;
    while (sys_load(a.loc + L.state(kComp)) != r + 1u) {
      if (wall_clock64() > deadline) {
        set_err(a);
        v = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    set_ok = v;
  }
  __syncthreads();
  if (!set_ok) return;
  for (int32_t w = w0; w < items; w += stride) {
    const auto [p, k, j] = item(w);
    if (k >= a.tab->nch[p]) continue;
    if (threadIdx.x == 0) {
      int32_t z = sys_load(a.loc + L.cmask(p, k)) == 0u ? 1 : 0;
      if (z && p != me && in_place) {
        // the output is the row: a writer that passed its gate before the
        // completion (gather_gate looks at `done` after its marker) finishes
        // before the zeros go in, or its bytes would land on top of them
        wait_row_writers(a, fl, row, p, k * L.P + j);
      }
      if (z && p == me) {
        // my own part: its reduce pieces may still be writing it (a chunk
        // reduced after the decision) -- zero it once they are done
        const uint64_t deadline = wall_clock64() + 3 * a.timeout + 1;
        while (sys_load(a.loc + L.pdone(k, j)) != r + 1u) {
          if (wall_clock64() > deadline) {
            set_err(a);
            break;
          }
          __builtin_amdgcn_s_sleep(4);
        }
      }
      act = z;
    }
    __syncthreads();
    const int64_t n = part_len_of(a, p, k, j);
    if (act && n > 0) {
      char* o = out + (a.tab->bstart[p] + part_off(a, k, j)) * ES;
      if (p == me && a.own_wt && ((uintptr_t(o) | uintptr_t(n * ES)) & 15) == 0) {
        // my own part: written through, after the reduce pieces' own
        // write-through stores (another XCD's): memory ends with the zeros
        const auto rs = sys_rsrc(o, n * ES);
        for (int64_t i = threadIdx.x; i < (n * ES) >> 4; i += blockDim.x) store_sys16(rs, i * 16, make_uint4(0, 0, 0, 0));
      } else {
        zero_bytes(o, n * ES);
      }
    }
    __syncthreads();  // `act` is rewritten by the next item
  }
}

// ---- finish: the last workgroup out of the launch --------------------------------
// Every workgroup's reads of the rows and writes of the output are done
// (each drained before its increment): withdraw the read announcements,
// count the round, publish the call's status, advance the call sequence.
__device__ void finish_if_last(const Args& a) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  const Layout& L = a.L;
  const uint32_t prev = add_loc(a.loc + L.state(kCtrFinish), 1u);
  if (prev != gridDim.x - 1) return;
  const int32_t N = L.N, me = a.me;
  const uint32_t r = sys_load(a.loc + L.state(kCur));
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  for (int32_t k = 0; k < a.kme; ++k) DevMem::st(fl + L.sread(row, k), 0u);
  DevMem::st(fl + L.gread(row), 0u);
  const uint32_t seq0 = sys_load(a.loc + L.state(kCallSeq));
  if (a.wo && int32_t(seq0 % uint32_t(L.D)) != row) DevMem::st(fl + L.gread(int32_t(seq0 % uint32_t(L.D))), 0u);
  const uint32_t landed = sys_load(a.loc + L.state(kCompLanded));
  int64_t total = 0;
  for (int32_t p = 0; p < N; ++p) total += a.tab->nch[p];
  stat_add(a, kRounds, 1);
  stat_add(a, kLandedChunks, landed);
  stat_add(a, kMissingChunks, uint64_t(total - int64_t(landed)));
  const uint32_t seq = sys_load(a.loc + L.state(kCallSeq));
  CallStatus* cs = a.status + (seq % uint32_t(kStatusSlots));
  __hip_atomic_store(&cs->round, int64_t(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&cs->reason, int64_t(sys_load(a.loc + L.state(kCompReason))), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&cs->landed_chunks, int64_t(landed), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&cs->forced_chunks, int64_t(sys_load(a.loc + L.state(kForcedChunks))), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the record names its call last: a reader that sees this id sees the fields above
  __hip_atomic_store(&cs->call, int64_t(seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  sys_store(a.loc + L.state(kCallSeq), seq + 1u);
}

// ---- the round launch -------------------------------------------------------------
template <typename T, int NS, int LB>
__global__ __launch_bounds__(LB) void os_round_kernel(Args a) {
  constexpr int ES = sizeof(T);
  const uint64_t t0 = a.tl ? wall_clock64() : 0;
  uint64_t t1 = t0;
  int32_t b = int32_t(blockIdx.x);
  if (b == 0) {
    begin_role(a);
  } else {
    const uint2 rs = wait_begun(a);
    const uint32_t r = rs.x;
    if (a.tl) t1 = wall_clock64();
    // Window output (exact rounds, no caller buffer): the call's output is
    // the gather row of ITS call id in my own window, where the peers'
    // reduced parts land at their final offsets (slot == block step) and my
    // reduce writes my block -- no copy.  A call that served another round
    // (catch-up) copies into that row like a caller buffer.
    char* out = a.out;
    bool in_place = false;
    if (a.wo) {
      const int32_t vrow = int32_t(rs.y % uint32_t(a.L.D));
      out = a.tab->gd[vrow][a.me];
      in_place = vrow == int32_t(r % uint32_t(a.L.D));
    }
    b -= 1;
    if (b < a.gp) {
      push_role<ES>(a, r, b, a.gp);
    } else if ((b -= a.gp) < a.kme) {
      decide_role(a, r, b);
    } else if ((b -= a.kme) < a.gr) {
      reduce_role<T, NS>(a, out, r, b, a.gr);
    } else if ((b -= a.gr) == 0) {
      complete_role(a, r);
    } else {
      copy_role<ES>(a, out, in_place, r, b - 1, a.gq);
    }
  }
  if (a.tl && threadIdx.x == 0) {  // vector stores (one lane)
    unsigned long long* t = a.tl + 3 * int64_t(blockIdx.x);
    t[0] = t0;
    t[1] = t1;
    t[2] = wall_clock64();
  }
  finish_if_last(a);
}

// retire: tell every peer that this rank serves no round >= its next one
__global__ void os_retire_kernel(Args a) {
  const int32_t q = threadIdx.x;
  if (q >= a.L.N || q == a.me || a.tab->fl[q] == nullptr) return;  // (null: a rank that never joined)
  DevMem::st(a.tab->fl[q] + a.L.fin(a.me), sys_load(a.loc + a.L.state(kNext)) + 1u);
}

// Reduce role alone (microbenchmark): every piece of my block, decisions pre-set.
template <typename T, int NS, int LB>
__global__ __launch_bounds__(LB) void os_reduce_bench_kernel(Args a, uint32_t r) {
  const int32_t P = a.L.P, ns = a.nsub;
  const int32_t items = a.kme * P * ns;
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x)
    reduce_piece<T, NS>(a, a.out, r, w / (P * ns), (w / ns) % P, w % ns, false);
}

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

template <typename T>
void launch_call(hipStream_t s, const Args& a) {
  const unsigned nt = a.threads <= 256 ? 256u : 1024u;
  const unsigned grid = unsigned(onesided_grid(a));
  with_ns(a.L.N, [&](auto ns) {
    constexpr int NS = decltype(ns)::value;
    if (nt == 256u) hipLaunchKernelGGL((os_round_kernel<T, NS, 256>), dim3(grid), dim3(nt), 0, s, a);
    else hipLaunchKernelGGL((os_round_kernel<T, NS, kMaxThreads>), dim3(grid), dim3(nt), 0, s, a);
  });
}

}  // namespace

void launch_onesided_retire(hipStream_t s, const Args& a) {
  hipLaunchKernelGGL(os_retire_kernel, dim3(1), dim3(64), 0, s, a);
}

void launch_onesided_call(hipStream_t s, const Args& a, int32_t dtype) {
  if (dtype == 0) launch_call<float>(s, a);
  else launch_call<uint16_t>(s, a);
}

double onesided_reduce_role_bench(int32_t N, int64_t block, int64_t chunk, int64_t part, int32_t nsub, int32_t dtype,
                                  int32_t threads, int32_t grid, int32_t iters, int32_t device) {
  auto ok = [](hipError_t e, const char* w) {
    if (e != hipSuccess) throw std::runtime_error(std::string("akka onesided bench: ") + w + ": " + hipGetErrorString(e));
  };
  ok(hipSetDevice(device), "set device");
  const int64_t es = dtype == 0 ? 4 : 2;
  const int64_t slot = (block + 63) / 64 * 64;
  const int32_t K = int32_t((block + chunk - 1) / chunk);
  const int32_t P = int32_t((chunk + part - 1) / part);
  Layout L;
  L.init(N, 2, K, P);
  char *sd = nullptr, *gd = nullptr, *in = nullptr, *out = nullptr;
  uint32_t *fl = nullptr, *loc = nullptr;
  unsigned long long* stats = nullptr;
  Tables* tab = nullptr;
  ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&sd), size_t(N * slot * es), hipDeviceMallocFinegrained), "sd");
  ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&gd), size_t(N * slot * es), hipDeviceMallocFinegrained), "gd");
  ok(hipMalloc(&in, size_t(N * block * es)), "in");
  ok(hipMalloc(&out, size_t(N * block * es)), "out");
  ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&fl), size_t(L.flag_words) * 4, hipDeviceMallocUncached), "fl");
  ok(hipExtMallocWithFlags(reinterpret_cast<void**>(&loc), size_t(L.local_words) * 4, hipDeviceMallocUncached),
     "loc");
  ok(hipMalloc(reinterpret_cast<void**>(&stats), kNumStats * 8), "stats");
  ok(hipMalloc(reinterpret_cast<void**>(&tab), sizeof(Tables)), "tab");
  ok(hipMemset(sd, 0x3c, size_t(N * slot * es)), "fill");
  ok(hipMemset(in, 0x3c, size_t(N * block * es)), "fill");
  ok(hipMemset(fl, 0, size_t(L.flag_words) * 4), "fl");
  ok(hipMemset(loc, 0, size_t(L.local_words) * 4), "loc");
  Tables t;
  std::memset(&t, 0, sizeof(t));
  for (int32_t q = 0; q < N; ++q) {
    t.fl[q] = fl;
    t.bstart[q] = int64_t(q) * block;
    t.blen[q] = block;
    t.nch[q] = K;
    for (int32_t d = 0; d < 2; ++d) {
      t.sd[d][q] = sd;
      t.gd[d][q] = gd;
    }
  }
  ok(hipMemcpy(tab, &t, sizeof(t), hipMemcpyHostToDevice), "tab");
  // every chunk decided with all N sources, every peer gated (bcast to N-1 rows)
  std::vector<uint32_t> hl(size_t(L.local_words), 0u);
  const uint32_t r = 0;
  for (int32_t k = 0; k < K; ++k) {
    const uint64_t d = (uint64_t((N >= 32 ? 0xffffffffu : ((1u << N) - 1u))) << 32) | uint64_t(r + 1u);
    std::memcpy(&hl[size_t(L.dec(k))], &d, 8);
    for (int32_t j = 0; j < P; ++j) hl[size_t(L.okq(k, j))] = ((1u << N) - 1u) & ~1u;  // me = 0
  }
  ok(hipMemcpy(loc, hl.data(), hl.size() * 4, hipMemcpyHostToDevice), "loc");
  Args a;
  a.tab = tab;
  a.loc = loc;
  a.stats = stats;
  a.L = L;
  a.C = chunk;
  a.slot = slot;
  a.part_len = part;
  a.me = 0;
  a.kme = K;
  a.nsub = std::max(1, nsub);
  a.threads = threads;
  a.timeout = uint64_t(1) << 40;
  a.in = in;
  a.out = out;
  const unsigned nt = threads <= 256 ? 256u : 1024u;
  const unsigned g = unsigned(std::max(1, grid));
  auto launch = [&]() {
    auto go = [&](auto tt) {
      using T = decltype(tt);
      with_ns(N, [&](auto ns) {
        constexpr int NS = decltype(ns)::value;
        if (nt == 256u) hipLaunchKernelGGL((os_reduce_bench_kernel<T, NS, 256>), dim3(g), dim3(nt), 0, nullptr, a, r);
        else hipLaunchKernelGGL((os_reduce_bench_kernel<T, NS, kMaxThreads>), dim3(g), dim3(nt), 0, nullptr, a, r);
      });
    };
    if (dtype == 0) go(float{});
    else go(uint16_t{});
  };
  hipEvent_t e0, e1;
  ok(hipEventCreate(&e0), "event");
  ok(hipEventCreate(&e1), "event");
  for (int i = 0; i < 3; ++i) launch();
  ok(hipEventRecord(e0, nullptr), "record");
  for (int i = 0; i < iters; ++i) launch();
  ok(hipEventRecord(e1, nullptr), "record");
  ok(hipEventSynchronize(e1), "sync");
  float ms = 0.f;
  ok(hipEventElapsedTime(&ms, e0, e1), "elapsed");
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  for (void* p : {static_cast<void*>(sd), static_cast<void*>(gd), static_cast<void*>(in), static_cast<void*>(out),
                  static_cast<void*>(fl), static_cast<void*>(loc), static_cast<void*>(stats),
                  static_cast<void*>(tab)})
    (void)hipFree(p);
  return double(ms) / std::max(1, iters);
}

}  // namespace os
}  // namespace akka
