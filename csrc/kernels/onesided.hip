// gfx950 kernels of the one-sided threshold lane (onesided_kernels.h).
//
// The protocol decisions (tags, gates, verdicts, round selection) are the
// functions of onesided_protocol.h, shared with the CPU backend; this file
// only maps them onto workgroups and moves the bytes.  Hand-offs follow the
// system-scope recipe of xgmi_device.h: data -> release -> "done" tag;
// observe tag -> acquire -> system-coherent (sc0 sc1) loads of the data.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "onesided_kernels.h"
#include "xgmi_device.h"

namespace akka {
namespace os {
namespace {

using namespace xgmi;

constexpr int kWaitThreads = 256;  // decide / cdecide workgroups
constexpr int kMaxThreads = 1024;

// Memory policy of the protocol functions on the device: flag words are in
// uncached fine-grained memory (own or a peer's, over xGMI) -> system scope.
struct DevMem {
  __device__ static uint32_t ld(const uint32_t* p) { return sys_load(p); }
  __device__ static void st(uint32_t* p, uint32_t v) { sys_store(p, v); }
  // announce, then look: the store must be performed before the load issues
  __device__ static void st_sc(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __device__ static uint32_t ld_sc(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
  }
};

__device__ inline void stat_add(const Args& a, int32_t i, unsigned long long v) {
  if (v) atomicAdd(a.stats + i, v);
}

// Part j of chunk k of block p: element offset inside the block and length.
__device__ inline int64_t part_len_of(const Args& a, int32_t p, int32_t k, int32_t j) {
  const int64_t clen = min(a.C, a.tab->blen[p] - int64_t(k) * a.C);
  return max(int64_t(0), min(a.part_len, clen - int64_t(j) * a.part_len));
}
__device__ inline int64_t part_off(const Args& a, int32_t k, int32_t j) {
  return int64_t(k) * a.C + int64_t(j) * a.part_len;
}

__device__ inline uint32_t cur_round(const Args& a) { return a.loc[a.L.state(kCur)]; }

// ---- begin: round selection (catch-up) ----------------------------------------
__global__ void os_begin_kernel(Args a) {
  if (threadIdx.x != 0) return;
  const Layout& L = a.L;
  uint32_t* fl = a.tab->fl[a.me];
  uint32_t* loc = a.loc;
  const uint32_t next = loc[L.state(kNext)];
  const int64_t sm = seen_max<DevMem>(fl, L, a.me);
  const uint32_t r = select_round(next, sm, a.max_lag);
  stat_add(a, kSkippedRounds, r - next);
  loc[L.state(kCur)] = r;
  loc[L.state(kNext)] = r + 1u;
  loc[L.state(kCtrReduce)] = 0;
  loc[L.state(kCtrCopy)] = 0;
  loc[L.state(kForcedChunks)] = 0;
  // rounds skipped by catch-up count as completed for the senders' outdated check
  if (DevMem::ld(fl + L.done()) < r) DevMem::st(fl + L.done(), r);
}

// ---- push: phase 1, fire and forget -----------------------------------------------
template <int ES>
__global__ __launch_bounds__(kMaxThreads) void os_push_kernel(Args a) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P;
  const int32_t items = (N - 1) * L.Kmax * P;
  const uint32_t r = cur_round(a);
  const int32_t row = int32_t(r % uint32_t(L.D));
  __shared__ int32_t go;
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) {
    // part-major, peers rotated from me + 1: consecutive workgroups feed different links
    const int32_t i = w % (N - 1), kj = w / (N - 1);
    const int32_t k = kj / P, j = kj % P;
    const int32_t p = (a.me + 1 + i) % N;
    if (k >= a.tab->nch[p]) continue;  // uniform over the workgroup
    uint32_t* ofl = a.tab->fl[p];
    if (threadIdx.x == 0) {
      int32_t g = kDead;
      if (!sys_load(a.dead + p)) {
        if (k == 0 && j == 0) DevMem::st(ofl + L.seen(a.me), r + 1u);  // implicit start at the owner
        g = scatter_gate<DevMem>(ofl, L, row, a.me, k, j, r);
      }
      go = g;
      stat_add(a, g == kGo ? kScatterPushed : g == kOutdated ? kScatterOutdated : g == kConflict ? kScatterConflict
                                                                                               : kDeadSkips, 1);
    }
    __syncthreads();
    if (go == kGo) {
      const int64_t n = part_len_of(a, p, k, j);
      const int64_t off = part_off(a, k, j);
      if (n > 0)
        copy_bytes(a.tab->sd[row][p] + (int64_t(a.me) * a.slot + off) * ES, a.in + (a.tab->bstart[p] + off) * ES,
                   n * ES);
      release_wg();
      if (threadIdx.x == 0) DevMem::st(ofl + L.stag(row, a.me, k, j), tag_done(r));
    }
    __syncthreads();  // `go` is rewritten by the next item
  }
}

// ---- decide: reduce threshold of one chunk of my block --------------------------
__global__ __launch_bounds__(kWaitThreads) void os_decide_kernel(Args a) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t k = blockIdx.x;
  const uint32_t r = cur_round(a);
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  __shared__ int32_t dn[kMaxRanks], lost[kMaxRanks];
  __shared__ int32_t verdict;
  __shared__ uint32_t mask_s;
  if (threadIdx.x == 0) DevMem::st_sc(fl + L.sread(row, k), r + 1u);  // announce before looking
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
      mask_s = mask;
    }
    __syncthreads();
    if (verdict != kWait) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (threadIdx.x == 0) {
    a.loc[L.dec(row, k)] = r + 1u;
    a.loc[L.dec(row, k) + 1] = mask_s;
    DevMem::st(fl + L.fired(row, k), r + 1u);  // late senders of round <= r now skip
    if (verdict == kThreshold) {
      stat_add(a, kReduceThreshold, 1);
    } else {
      stat_add(a, kReduceForced, 1);
      atomicAdd(a.loc + L.state(kForcedChunks), 1u);
    }
    if (verdict == kTimeout) {
      stat_add(a, kTimeouts, 1);
      sys_store(a.err, 1u);
    }
    stat_add(a, kReduceContribs, __popc(mask_s));
  }
}

// ---- reduce: masked sum of the landed set, phase 2 pushes ------------------------
// Sources in ascending rank order (the exact lanes' order): my own input
// (plain loads), peers' SD slots (system-coherent loads).  Destinations: my
// output block (local) and GD[row][me] of every peer in `okq`.
// Vector body with the rank count NS known at compile time: every thread
// issues the loads of all landed sources (U = 16 / NS vectors each) before the
// first add, as the exact lanes' reduce does; a source outside `mask` reads as
// zeros without a load (the branch is uniform).  Same ascending-source order as
// the runtime-N body, so the sums are bitwise identical.
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
        store_nt16(reinterpret_cast<uint4*>(o) + i, w);  // my output: not read again in this kernel
#pragma unroll
        for (int q = 0; q < NS; ++q)
          if ((okq >> q) & 1u) reinterpret_cast<uint4*>(a.tab->gd[row][q] + goff)[i] = w;
      }
    }
  }
}

// NS > 0: instantiated for N == NS (one reduce kernel per node rank count);
// NS == 0: any N.
template <typename T, int NS>
__device__ void masked_sum(const Args& a, int32_t row, uint32_t mask, uint32_t okq, int64_t off, int64_t n) {
  constexpr int ES = sizeof(T);
  constexpr int PV = Elt<T>::kPerVec;
  const int32_t N = a.L.N, me = a.me;
  const char* mine = a.in + (a.tab->bstart[me] + off) * ES;
  const char* sd = a.tab->sd[row][me];
  char* o = a.out + (a.tab->bstart[me] + off) * ES;
  const int64_t goff = (int64_t(me) * a.slot + off) * ES;  // same offset in every peer's GD row
  const uintptr_t al = uintptr_t(mine) | uintptr_t(o) | uintptr_t(n * ES) | uintptr_t(goff) | uintptr_t(off * ES) |
                       uintptr_t(a.slot * ES);
  if ((al & 15) == 0) {
    if constexpr (NS > 0) {
      masked_sum_n<T, NS>(a, mine, sd, o, goff, row, mask, okq, off, n);
      return;
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
}

template <typename T, int NS, int LB>
__global__ __launch_bounds__(LB) void os_reduce_kernel(Args a) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t kme = a.tab->nch[me];
  const int32_t items = kme * P;
  const uint32_t r = cur_round(a);
  const int32_t row = int32_t(r % uint32_t(L.D));
  __shared__ uint32_t okq_s, mask_s;
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const int32_t k = w / P, j = w % P;
    if (threadIdx.x == 0) {
      const uint32_t mask = a.loc[L.dec(row, k) + 1];  // decided by the previous kernel
      const uint32_t cnt = uint32_t(__popc(mask));
      uint32_t okq = 0;
      for (int32_t i = 1; i < N; ++i) {
        const int32_t q = (me + i) % N;
        if (sys_load(a.dead + q)) {
          stat_add(a, kDeadSkips, 1);
          continue;
        }
        uint32_t* qfl = a.tab->fl[q];
        if (k == 0 && j == 0) DevMem::st(qfl + L.seen(me), r + 1u);
        const int32_t g = gather_gate<DevMem>(qfl, L, row, me, k, j, r);
        if (g == kGo) {
          okq |= 1u << q;
          DevMem::st(qfl + L.gtag(row, me, k, j) + 1, cnt);  // count, ordered before the tag by the release
          stat_add(a, kGatherPushed, 1);
        } else {
          stat_add(a, g == kOutdated ? kGatherOutdated : kGatherConflict, 1);
        }
      }
      if (j == 0) a.counts[int64_t(me) * a.kcols + k] = int32_t(cnt);
      okq_s = okq;
      mask_s = mask;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the landed SD bytes (peers' tags seen by decide)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const int64_t n = part_len_of(a, me, k, j);
    if (n > 0) masked_sum<T, NS>(a, row, mask_s, okq_s, part_off(a, k, j), n);
    release_wg();
    if (threadIdx.x == 0) {
      for (int32_t q = 0; q < N; ++q)
        if ((okq_s >> q) & 1u) DevMem::st(a.tab->fl[q] + L.gtag(row, me, k, j), tag_done(r));
    }
    __syncthreads();
  }
  // the last workgroup out withdraws the row's read announcements (every
  // workgroup's SD loads completed before its increment: release_wg above)
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.loc + L.state(kCtrReduce), 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      for (int32_t k = 0; k < kme; ++k) DevMem::st(a.tab->fl[me] + L.sread(row, k), 0u);
    }
  }
}

// ---- cdecide: completion threshold -------------------------------------------------
__global__ __launch_bounds__(kWaitThreads) void os_cdecide_kernel(Args a) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me, K = L.Kmax;
  const uint32_t r = cur_round(a);
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  __shared__ int32_t landed_s, pending_s, verdict;
  __shared__ int32_t past[kMaxRanks];
  if (threadIdx.x == 0) DevMem::st_sc(fl + L.gread(row), r + 1u);  // announce before looking
  __syncthreads();
  const uint64_t deadline = wall_clock64() + a.timeout;
  int32_t landed = 0;
  while (true) {
    if (threadIdx.x == 0) {
      landed_s = 0;
      pending_s = 0;
    }
    if (threadIdx.x < kMaxRanks) {
      const int32_t p = threadIdx.x;
      past[p] = p < N && p != me && source_past<DevMem>(fl, L, p, r) ? 1 : 0;  // before the tags
    }
    __syncthreads();
    int32_t my_l = 0, my_p = 0;
    for (int32_t c = threadIdx.x; c < N * K; c += blockDim.x) {
      const int32_t p = c / K, k = c % K;
      if (p == me || k >= a.tab->nch[p]) continue;
      int32_t st = kLanded;
      for (int32_t j = 0; j < P; ++j) {
        const int32_t s = tag_state(DevMem::ld(fl + L.gtag(row, p, k, j)), r);
        if (s == kLost) {
          st = kLost;
          break;
        }
        if (s == kPending) st = kPending;
      }
      if (st == kPending && (past[p] || sys_load(a.dead + p))) st = kLost;
      a.loc[L.cmask(p, k)] = st == kLanded ? 1u : 0u;
      my_l += st == kLanded;
      my_p += st == kPending;
    }
    if (my_l) atomicAdd(&landed_s, my_l);
    if (my_p) atomicAdd(&pending_s, my_p);
    __syncthreads();
    if (threadIdx.x == 0) {
      landed = landed_s + a.tab->nch[me];  // my own reduced chunks are delivered to myself
      verdict = evaluate(landed, pending_s, a.need_c, r, seen_max<DevMem>(fl, L, me), a.max_lag, sys_load(a.force),
                         wall_clock64() > deadline);
    }
    __syncthreads();
    if (verdict != kWait) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (threadIdx.x == 0) {
    a.loc[L.state(kCompReason)] = uint32_t(verdict);
    a.loc[L.state(kCompLanded)] = uint32_t(landed);
    stat_add(a, verdict == kThreshold ? kCompleteThreshold : kCompleteForced, 1);
    if (verdict == kTimeout) {
      stat_add(a, kTimeouts, 1);
      sys_store(a.err, 1u);
    }
  }
}

// ---- copy: landed chunks -> output, completion ------------------------------------
template <int ES>
__global__ __launch_bounds__(kMaxThreads) void os_copy_kernel(Args a) {
  const Layout& L = a.L;
  const int32_t N = L.N, P = L.P, me = a.me;
  const int32_t items = (N - 1) * L.Kmax * P;
  const uint32_t r = cur_round(a);
  const int32_t row = int32_t(r % uint32_t(L.D));
  uint32_t* fl = a.tab->fl[me];
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const int32_t i = w % (N - 1), kj = w / (N - 1);
    const int32_t k = kj / P, j = kj % P;
    const int32_t p = (me + 1 + i) % N;
    if (k >= a.tab->nch[p]) continue;
    const bool landed = a.loc[L.cmask(p, k)] != 0u;
    const int64_t n = part_len_of(a, p, k, j);
    const int64_t off = part_off(a, k, j);
    char* o = a.out + (a.tab->bstart[p] + off) * ES;
    if (n > 0) {
      if (landed) copy_in(o, a.tab->gd[row][me] + (int64_t(p) * a.slot + off) * ES, n * ES);
      else zero_bytes(o, n * ES);
    }
    if (j == 0 && threadIdx.x == 0)
      a.counts[int64_t(p) * a.kcols + k] = landed ? int32_t(DevMem::ld(fl + L.gtag(row, p, k, 0) + 1)) : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my GD reads are done before the row is released
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.loc + L.state(kCtrCopy), 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      DevMem::st(fl + L.done(), r + 1u);  // senders of round <= r now skip me
      DevMem::st(fl + L.gread(row), 0u);
      const uint32_t landed = a.loc[L.state(kCompLanded)];
      int64_t total = 0;
      for (int32_t p = 0; p < N; ++p) total += a.tab->nch[p];
      stat_add(a, kRounds, 1);
      stat_add(a, kLandedChunks, landed);
      stat_add(a, kMissingChunks, uint64_t(total - int64_t(landed)));
      CallStatus* cs = a.status + a.call_slot;
      __hip_atomic_store(&cs->reason, int64_t(a.loc[L.state(kCompReason)]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&cs->landed_chunks, int64_t(landed), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&cs->forced_chunks, int64_t(a.loc[L.state(kForcedChunks)]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(&cs->round, int64_t(r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// retire: tell every peer that this rank serves no round >= its next one
__global__ void os_retire_kernel(Args a) {
  const int32_t q = threadIdx.x;
  if (q >= a.L.N || q == a.me) return;
  DevMem::st(a.tab->fl[q] + a.L.fin(a.me), a.loc[a.L.state(kNext)] + 1u);
}

int32_t grid_for(int64_t items, int32_t cap) { return int32_t(std::max<int64_t>(1, std::min<int64_t>(items, cap))); }

// The reduce kernel for this call's rank count (2..8, 16; else runtime N) and
// workgroup size (a 256-thread launch bound leaves the body all its VGPRs).
template <typename T, int NS>
void launch_reduce_ns(hipStream_t s, const Args& a, unsigned grid, unsigned nt) {
  if (nt <= 256u) hipLaunchKernelGGL((os_reduce_kernel<T, NS, 256>), dim3(grid), dim3(nt), 0, s, a);
  else hipLaunchKernelGGL((os_reduce_kernel<T, NS, kMaxThreads>), dim3(grid), dim3(nt), 0, s, a);
}

template <typename T>
void launch_reduce(hipStream_t s, const Args& a, unsigned grid, unsigned nt) {
  switch (a.L.N) {
    case 2: return launch_reduce_ns<T, 2>(s, a, grid, nt);
    case 3: return launch_reduce_ns<T, 3>(s, a, grid, nt);
    case 4: return launch_reduce_ns<T, 4>(s, a, grid, nt);
    case 5: return launch_reduce_ns<T, 5>(s, a, grid, nt);
    case 6: return launch_reduce_ns<T, 6>(s, a, grid, nt);
    case 7: return launch_reduce_ns<T, 7>(s, a, grid, nt);
    case 8: return launch_reduce_ns<T, 8>(s, a, grid, nt);
    case 16: return launch_reduce_ns<T, 16>(s, a, grid, nt);
    default: return launch_reduce_ns<T, 0>(s, a, grid, nt);
  }
}

template <typename T>
void launch_call(hipStream_t s, const Args& a) {
  constexpr int ES = sizeof(T);
  const int32_t nt = (a.threads == 512 || a.threads == 1024) ? a.threads : 256;
  const int64_t peer_items = int64_t(a.L.N - 1) * a.L.Kmax * a.L.P;
  hipLaunchKernelGGL(os_begin_kernel, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(os_push_kernel<ES>, dim3(unsigned(grid_for(peer_items, 8192))), dim3(unsigned(nt)), 0, s, a);
  if (a.kme > 0) {
    hipLaunchKernelGGL(os_decide_kernel, dim3(unsigned(a.kme)), dim3(kWaitThreads), 0, s, a);
    launch_reduce<T>(s, a, unsigned(grid_for(int64_t(a.kme) * a.L.P, 8192)), unsigned(nt));
  }
  hipLaunchKernelGGL(os_cdecide_kernel, dim3(1), dim3(kWaitThreads), 0, s, a);
  hipLaunchKernelGGL(os_copy_kernel<ES>, dim3(unsigned(grid_for(peer_items, 8192))), dim3(unsigned(nt)), 0, s, a);
}

}  // namespace

void launch_onesided_retire(hipStream_t s, const Args& a) {
  hipLaunchKernelGGL(os_retire_kernel, dim3(1), dim3(64), 0, s, a);
}

void launch_onesided_call(hipStream_t s, const Args& a, int32_t dtype) {
  if (dtype == 0) launch_call<float>(s, a);
  else launch_call<uint16_t>(s, a);
}

}  // namespace os
}  // namespace akka
