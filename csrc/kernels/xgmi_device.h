// Device-side building blocks shared by the one-sided xGMI kernels
// (ipc.hip: exact rounds and the mailbox p2p; onesided.hip: threshold rounds).
//
// Memory-model protocol (HIP / LLVM AMDGPU, system scope because producer and
// consumer sit on different devices and the bytes cross xGMI):
//   producer: its stores -> s_waitcnt vmcnt(0) in every wave -> workgroup
//             barrier -> lane 0: release fence (system) -> s_waitcnt vmcnt(0)
//             -> relaxed system-scope store of the flag word;
//   consumer: lane 0 polls the flag with relaxed system-scope loads (with
//             s_sleep) -> acquire fence (system) -> s_waitcnt vmcnt(0) ->
//             workgroup barrier -> system-coherent loads of the payload.
// The explicit s_waitcnt after the release fence is there on purpose: the
// compiler may drop its own when it proves the scoreboard empty, letting the
// flag overtake the write-back (docs/DESIGN.md section 4f rule 2).
// Only to be included by .hip translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace akka {
namespace xgmi {

constexpr int kUnroll = 4;  // 16-B vectors per thread per source in flight

__device__ inline bool reached(uint32_t v, uint32_t want) { return int32_t(v - want) >= 0; }

__device__ inline uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Whole workgroup: make this workgroup's stores visible at system scope.
// Lane 0 may then signal (flag stores).
__device__ inline void release_wg() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Whole workgroup: acquire after lane 0's successful waits.  Returns the
// shared verdict.
__device__ inline bool acquire_all(bool ok_lane0) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ok = ok_lane0 ? 1 : 0;
  }
  __syncthreads();
  return ok != 0;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streaming (nontemporal) 16-byte store of local memory nobody reads before
// the kernel ends: it does not evict the lines still to be read.
__device__ inline void store_nt16(uint4* p, const uint4& v) {
  u32x4 w;
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

// dst <- src with plain loads and stores (src is this rank's own memory).
__device__ inline void copy_bytes(char* __restrict__ dst, const char* __restrict__ src, int64_t bytes) {
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | uintptr_t(bytes)) & 15) == 0) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    const int64_t n = bytes >> 4;
    int64_t i = threadIdx.x;
    for (; i + (kUnroll - 1) * int(blockDim.x) < n; i += kUnroll * int(blockDim.x)) {
      uint4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = s[i + u * int(blockDim.x)];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) d[i + u * int(blockDim.x)] = v[u];
    }
    for (; i < n; i += int(blockDim.x)) d[i] = s[i];
  } else if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | uintptr_t(bytes)) & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = threadIdx.x; i < (bytes >> 2); i += int(blockDim.x)) d[i] = s[i];
  } else {
    for (int64_t i = threadIdx.x; i < bytes; i += int(blockDim.x)) dst[i] = src[i];
  }
}

// ---- reads of window memory another rank wrote ------------------------------
// Every byte a peer stored into a window is read with system-coherent buffer
// loads (sc0 sc1: L1 and L2 bypassed), so no line cached from an earlier round
// can be returned -- the consumer side of the hand-off is correct whatever
// caching policy the window's memory has on this or the peer GPU.  Buffer
// loads also bound every read by the span's size (out-of-range reads return 0).
constexpr int kSysAux = 17;  // sc0 | sc1

__device__ inline __amdgpu_buffer_rsrc_t sys_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, int(min(bytes, int64_t(0x7fffffff))),
                                           0x00020000);
}
__device__ inline uint4 load_sys16(__amdgpu_buffer_rsrc_t r, int64_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, int(off), 0, kSysAux);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// dst (local, streamed past the caches: the round's output, read after the
// round) <- src (window memory written by a peer).
__device__ inline void copy_in(char* __restrict__ dst, const char* __restrict__ src, int64_t bytes) {
  const auto r = sys_rsrc(src, bytes);
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | uintptr_t(bytes)) & 15) == 0) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    const int64_t n = bytes >> 4;
    int64_t i = threadIdx.x;
    for (; i + (kUnroll - 1) * int(blockDim.x) < n; i += kUnroll * int(blockDim.x)) {
      uint4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) v[u] = load_sys16(r, (i + u * int(blockDim.x)) * 16);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) store_nt16(d + i + u * int(blockDim.x), v[u]);
    }
    for (; i < n; i += int(blockDim.x)) store_nt16(d + i, load_sys16(r, i * 16));
  } else if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | uintptr_t(bytes)) & 3) == 0) {
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = threadIdx.x; i < (bytes >> 2); i += int(blockDim.x))
      d[i] = __builtin_amdgcn_raw_buffer_load_b32(r, int(i * 4), 0, kSysAux);
  } else {
    for (int64_t i = threadIdx.x; i < bytes; i += int(blockDim.x))
      dst[i] = char(__builtin_amdgcn_raw_buffer_load_b8(r, int(i), 0, kSysAux));
  }
}

// ---- fence-free hand-offs ("lite") -------------------------------------------
// Producer: every byte a consumer will read goes out as a system-coherent
// (sc0 sc1, write-through) store; each storing wave waits for its stores
// (s_waitcnt vmcnt(0)), the workgroup meets at a barrier, lane 0 stores the
// flag.  Consumer: lane(s) poll the flag(s); after the barrier every load of
// the bytes is a system-coherent load.  No buffer_wbl2 / buffer_inv at all
// (docs/DESIGN.md section 4f rule 3: write-through stores + drained flag; sc
// loads in place of the acquire), at system scope.
__device__ inline void store_sys16(__amdgpu_buffer_rsrc_t r, int64_t off, const uint4& v) {
  u32x4 w;
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
  __builtin_amdgcn_raw_buffer_store_b128(w, r, int(off), 0, kSysAux);
}

// dst (a window, read by a peer) <- src (local), 16-byte aligned.
// U vectors per thread per batch: the vmcnt counter is in order and counts
// stores too, so a batch's loads wait for the previous batch's write-through
// stores to be acknowledged (by the peer's memory, over xGMI on a node) --
// the bytes moved per such wait set the push rate of a workgroup.
template <int U = kUnroll>
__device__ inline void copy_out_sys(char* __restrict__ dst, const char* __restrict__ src, int64_t bytes) {
  const auto r = sys_rsrc(dst, bytes);
  const uint4* s = reinterpret_cast<const uint4*>(src);
  const int64_t n = bytes >> 4;
  int64_t i = threadIdx.x;
  for (; i + (U - 1) * int(blockDim.x) < n; i += U * int(blockDim.x)) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = s[i + u * int(blockDim.x)];
#pragma unroll
    for (int u = 0; u < U; ++u) store_sys16(r, (i + u * int(blockDim.x)) * 16, v[u]);
  }
  for (; i < n; i += int(blockDim.x)) store_sys16(r, i * 16, s[i]);
}

// Whole workgroup: every wave's stores performed, then lane 0 may signal.
__device__ inline void drain_wg() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ inline void zero_bytes(char* __restrict__ dst, int64_t bytes) {
  if (((reinterpret_cast<uintptr_t>(dst) | uintptr_t(bytes)) & 15) == 0) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (int64_t i = threadIdx.x; i < (bytes >> 4); i += int(blockDim.x)) d[i] = make_uint4(0, 0, 0, 0);
  } else {
    for (int64_t i = threadIdx.x; i < bytes; i += int(blockDim.x)) dst[i] = 0;
  }
}

__device__ inline float bf16_to_f32(uint16_t h) { return __uint_as_float(uint32_t(h) << 16); }
__device__ inline uint16_t f32_to_bf16(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return uint16_t((u >> 16) | 0x40);  // quiet NaN
  return uint16_t((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// Element codecs: a 16-B vector <-> fp32 accumulators (bf16 via RNE).
template <typename T>
struct Elt;
template <>
struct Elt<float> {
  static constexpr int kPerVec = 4;
  __device__ static void add(float* acc, const uint4& v) {
    acc[0] += __uint_as_float(v.x);
    acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z);
    acc[3] += __uint_as_float(v.w);
  }
  __device__ static uint4 pack(const float* acc) {
    return make_uint4(__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]),
                      __float_as_uint(acc[3]));
  }
  __device__ static float load1(const char* p) { return *reinterpret_cast<const float*>(p); }
  __device__ static float load1_sys(__amdgpu_buffer_rsrc_t r, int64_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, int(off), 0, kSysAux));
  }
  __device__ static void store1(char* p, float v) { *reinterpret_cast<float*>(p) = v; }
};
template <>
struct Elt<uint16_t> {
  static constexpr int kPerVec = 8;
  __device__ static void add(float* acc, const uint4& v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += __uint_as_float(w[i] << 16);
      acc[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static uint4 pack(const float* acc) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = uint32_t(f32_to_bf16(acc[2 * i])) | (uint32_t(f32_to_bf16(acc[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static float load1(const char* p) { return bf16_to_f32(*reinterpret_cast<const uint16_t*>(p)); }
  __device__ static float load1_sys(__amdgpu_buffer_rsrc_t r, int64_t off) {
    return bf16_to_f32(uint16_t(__builtin_amdgcn_raw_buffer_load_b16(r, int(off), 0, kSysAux)));
  }
  __device__ static void store1(char* p, float v) { *reinterpret_cast<uint16_t*>(p) = f32_to_bf16(v); }
};

}  // namespace xgmi
}  // namespace akka
