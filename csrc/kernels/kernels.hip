// gfx950 (MI355X / CDNA4) kernels for the threshold allreduce.
//
// Hot spot K1 of SURVEY §2.3: the chunk N-way sum (reference: the scalar JVM
// loop of ScatteredDataBuffer.reduce, SB:20-32), plus the count expansion of
// ReducedDataBuffer.getWithCounts (RB:41-47).
//
// The sum is pure HBM streaming (nsrc reads + 1 write per element, no reuse),
// so the design goal is bytes-in-flight, not arithmetic:
//   * Vec: every lane issues 16-B loads for ALL sources of UNROLL vectors before
//     the first add (NSRC*UNROLL independent loads per lane), grid-stride over
//     the chunk with a grid capped at 8 blocks/CU x 256 CUs.  fp32 accumulate.
//   * Lds: each wave streams its own 1-KiB-per-source tiles through LDS with
//     global_load_lds_dwordx4 (LDS-DMA, no VGPR destination), double-buffered
//     with a counted vmcnt so tile t+1 is in flight while tile t is summed.
// Both are templated on the source count so the loads unroll completely.
// 64-lane waves throughout; blocks of 256 threads = 4 waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include <cstdlib>
#include <cstring>

#include "kernels.h"
#include "xgmi_device.h"

namespace akka {

namespace {

using v4u = unsigned int __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;
constexpr int kCUs = 256;
constexpr int kMaxGrid = kCUs * 8;  // 256 CUs x 8 blocks

struct SrcTable {
  const void* p[kMaxReduceSrc];
  int32_t* fill;  // optional counts-row fill done by block 0 (saves a dispatch per round)
  int32_t fill_value;
  int32_t fill_n;
  int32_t head_n;  // elements below the aligned body (vector kernels, block 0)
};

__device__ __forceinline__ void do_fill(const SrcTable& t) {
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < t.fill_n; i += kBlock) t.fill[i] = t.fill_value;
}

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) {
  return v;
}
template <>
__device__ __forceinline__ float to_f<unsigned short>(unsigned short v) {
  return __uint_as_float(uint32_t(v) << 16);
}
template <typename T>
__device__ __forceinline__ T from_f(float v);
template <>
__device__ __forceinline__ float from_f<float>(float v) {
  return v;
}
template <>
__device__ __forceinline__ unsigned short from_f<unsigned short>(float v) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(v));
}

// Misaligned head folded into a vector launch: the head_n elements just below
// the (16-B aligned) body pointers, summed by block 0 (saves a dispatch per
// chunk when the block offset is not a multiple of 16 B).
template <typename T, int NSRC>
__device__ __forceinline__ void do_head(const SrcTable& t, void* dst) {
  if (blockIdx.x == 0 && int(threadIdx.x) < t.head_n) {
    const int i = int(threadIdx.x) - t.head_n;
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < NSRC; ++s) acc += to_f(static_cast<const T*>(t.p[s])[i]);
    static_cast<T*>(dst)[i] = from_f<T>(acc);
  }
}

__device__ __forceinline__ void add_vec(float (&acc)[4], const v4u& v, float) {
  acc[0] += __uint_as_float(v.x);
  acc[1] += __uint_as_float(v.y);
  acc[2] += __uint_as_float(v.z);
  acc[3] += __uint_as_float(v.w);
}

__device__ __forceinline__ void add_vec(float (&acc)[8], const v4u& v, unsigned short) {
  acc[0] += __uint_as_float(v.x << 16);
  acc[1] += __uint_as_float(v.x & 0xffff0000u);
  acc[2] += __uint_as_float(v.y << 16);
  acc[3] += __uint_as_float(v.y & 0xffff0000u);
  acc[4] += __uint_as_float(v.z << 16);
  acc[5] += __uint_as_float(v.z & 0xffff0000u);
  acc[6] += __uint_as_float(v.w << 16);
  acc[7] += __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  // Plain casts lower to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving).
  __bf16 a = static_cast<__bf16>(lo);
  __bf16 b = static_cast<__bf16>(hi);
  return uint32_t(__builtin_bit_cast(unsigned short, a)) | (uint32_t(__builtin_bit_cast(unsigned short, b)) << 16);
}

__device__ __forceinline__ v4u pack_vec(const float (&acc)[4]) {
  return v4u{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
}
__device__ __forceinline__ v4u pack_vec(const float (&acc)[8]) {
  return v4u{pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]), pack_bf16x2(acc[4], acc[5]),
             pack_bf16x2(acc[6], acc[7])};
}

template <typename T>
struct VecTraits;
template <>
struct VecTraits<float> {
  static constexpr int kElems = 4;
};
template <>
struct VecTraits<unsigned short> {
  static constexpr int kElems = 8;
};

// ---- Vec: loads straight to VGPRs ----------------------------------------------
// Load/store cache policy (measured by bench/stream_variants.hip, see
// profiles/README.md): nontemporal stores keep a streamed output from
// evicting the sources out of the 256 MiB Infinity Cache; nontemporal loads
// help once the sources do not fit there anyway.
enum VecPolicy : int { kNtl = 0, kNts = 1, kBoth = 2 };

template <typename T, int NSRC, int UNROLL, int POL>
__global__ __launch_bounds__(kBlock) void reduce_vec_kernel(SrcTable srcs, v4u* __restrict__ dst, int64_t nvec) {
  constexpr int E = VecTraits<T>::kElems;
  do_fill(srcs);
  do_head<T, NSRC>(srcs, dst);
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t base = int64_t(blockIdx.x) * kBlock + threadIdx.x; base < nvec; base += stride * UNROLL) {
    v4u v[UNROLL][NSRC];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * stride;
      if (i < nvec) {
#pragma unroll
        for (int s = 0; s < NSRC; ++s) {
          const v4u* src = static_cast<const v4u*>(srcs.p[s]) + i;
          v[u][s] = POL == kNts ? *src : __builtin_nontemporal_load(src);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t i = base + u * stride;
      if (i < nvec) {
        v4u o;
        if constexpr (NSRC == 1) {
          o = v[u][0];  // one contributor: the sum is the value itself, bit for bit (-0.0, NaN payloads)
        } else {
          float acc[E];
#pragma unroll
          for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
          for (int s = 0; s < NSRC; ++s) add_vec(acc, v[u][s], T{});
          o = pack_vec(acc);
        }
        if constexpr (POL == kNtl) dst[i] = o;
        else __builtin_nontemporal_store(o, dst + i);
      }
    }
  }
}

// ---- Lds: LDS-DMA staging, per-wave double buffer ----------------------------------
// Wave w of the block owns LDS [buf][src][w][64 lanes] x 16 B.  A tile is 64
// vectors (1 KiB) per source.  global_load_lds writes lane l's 16 B at
// wave_base + 16*l, i.e. exactly where lane l reads it back.
template <typename T, int NSRC>
__global__ __launch_bounds__(kBlock) void reduce_lds_kernel(SrcTable srcs, v4u* __restrict__ dst, int64_t nvec) {
  constexpr int E = VecTraits<T>::kElems;
  constexpr int kWaves = kBlock / 64;
  __shared__ v4u lds[2][NSRC][kWaves][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  do_fill(srcs);
  do_head<T, NSRC>(srcs, dst);
  const int64_t ntiles = nvec / 64;  // full wave tiles; the tail goes through VGPRs
  const int64_t wave_id = int64_t(blockIdx.x) * kWaves + wave;
  const int64_t wave_stride = int64_t(gridDim.x) * kWaves;

  auto issue = [&](int64_t tile, int buf) {
#pragma unroll
    for (int s = 0; s < NSRC; ++s) {
      const v4u* g = static_cast<const v4u*>(srcs.p[s]) + tile * 64 + lane;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                       (__attribute__((address_space(3))) void*)&lds[buf][s][wave][0], 16, 0, 0);
    }
  };

  int64_t t = wave_id;
  int buf = 0;
  if (t < ntiles) issue(t, 0);
  for (; t < ntiles; t += wave_stride) {
    const int64_t nt = t + wave_stride;
    if (nt < ntiles) {
      issue(nt, buf ^ 1);
      // NSRC loads of the next tile may stay in flight; the current tile's are retired
      // (loads retire in order; an interleaved store only makes the wait stricter).
      if constexpr (NSRC == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if constexpr (NSRC == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if constexpr (NSRC == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if constexpr (NSRC == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (NSRC == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if constexpr (NSRC == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (NSRC == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < NSRC; ++s) add_vec(acc, lds[buf][s][wave][lane], T{});
    dst[t * 64 + lane] = pack_vec(acc);
    // The reads of `buf` must land before tile t+2 re-targets it.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    buf ^= 1;
  }
  // Tail (< 64 vectors): first wave of the grid, through VGPRs.
  if (wave_id == 0) {
    const int64_t i = ntiles * 64 + lane;
    if (i < nvec) {
      float acc[E];
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < NSRC; ++s) add_vec(acc, static_cast<const v4u*>(srcs.p[s])[i], T{});
      dst[i] = pack_vec(acc);
    }
  }
}

// ---- Scalar: unaligned pointers / sub-vector tails --------------------------------

template <typename T>
__global__ __launch_bounds__(kBlock) void reduce_scalar_kernel(SrcTable srcs, int nsrc, T* __restrict__ dst,
                                                               int64_t n) {
  do_fill(srcs);
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int s = 0; s < nsrc; ++s) acc += to_f(static_cast<const T*>(srcs.p[s])[i]);
    dst[i] = from_f<T>(acc);
  }
}

// One workgroup per (block, chunk) region at a time: the count is a
// wave-uniform scalar and the region is filled with 16-B stores (scalar head /
// tail where the region is not 16-B aligned); no per-element division.
__global__ __launch_bounds__(kBlock) void count_expand_kernel(int32_t* __restrict__ out,
                                                              const int32_t* __restrict__ counts, int64_t S,
                                                              int64_t step, int32_t N, int64_t C, int32_t kmax) {
  const int64_t nregions = int64_t(N) * kmax;
  for (int64_t reg = blockIdx.x; reg < nregions; reg += gridDim.x) {
    const int32_t j = int32_t(reg / kmax);
    const int64_t k = reg - int64_t(j) * kmax;
    const int64_t bs = j * step < S ? j * step : S;
    const int64_t be = j >= N - 1 ? S : ((j + 1) * step < S ? (j + 1) * step : S);
    const int64_t s = bs + k * C;
    if (s >= be) continue;
    const int64_t e = s + C < be ? s + C : be;
    const int32_t v = counts[reg];
    int64_t a = (s + 3) & ~int64_t(3);  // first 16-B aligned element
    if (a > e) a = e;
    const int64_t nv = (e - a) >> 2;
    if (blockIdx.y == 0) {
      for (int64_t i = s + threadIdx.x; i < a; i += kBlock) out[i] = v;
      for (int64_t i = a + nv * 4 + threadIdx.x; i < e; i += kBlock) out[i] = v;
    }
    int4* o4 = reinterpret_cast<int4*>(out + a);
    const int4 vv = make_int4(v, v, v, v);
    // gridDim.y workgroups share one region when there are few regions
    for (int64_t i = int64_t(blockIdx.y) * kBlock + threadIdx.x; i < nv; i += int64_t(kBlock) * gridDim.y) o4[i] = vv;
  }
}

// dst[i] = src[i] / count(block(i), chunk(i)), 0 where the count is 0: the
// count-weighted mean of an allreduce output (AllReduceOutput.mean) in one
// pass, reading the tiny per-chunk count table instead of a per-element one.
// Same region walk as count_expand (one wave-uniform count per region).
// AXPY: dst[i] += alpha * mean[i] instead (the SGD update fused into the
// averaging: one read of the sum, one read + write of the parameters).
// SHADOW (fp32 AXPY only): the updated parameters are also stored as bf16 into
// `shadow` (same element index), so a bf16 forward reads a weight copy the
// update already wrote instead of casting 4 B/element again every step.
// dst may alias src (mean(out=data): a gradient bucket averaged in place);
// each element is read before the same thread writes it, so no __restrict__.
constexpr int kCmUnroll = 4;

template <typename T, bool AXPY, bool SHADOW>
__global__ __launch_bounds__(kBlock) void count_mean_kernel(T* dst, const T* src,
                                                            const int32_t* __restrict__ counts, int64_t S,
                                                            int64_t step, int32_t N, int64_t C, int32_t kmax,
                                                            float alpha, unsigned short* __restrict__ shadow) {
  static_assert(!SHADOW || (AXPY && std::is_same_v<T, float>), "shadow: fp32 SGD update only");
  constexpr int E = VecTraits<T>::kElems;
  const int64_t nregions = int64_t(N) * kmax;
  for (int64_t reg = blockIdx.x; reg < nregions; reg += gridDim.x) {
    const int32_t j = int32_t(reg / kmax);
    const int64_t k = reg - int64_t(j) * kmax;
    const int64_t bs = j * step < S ? j * step : S;
    const int64_t be = j >= N - 1 ? S : ((j + 1) * step < S ? (j + 1) * step : S);
    const int64_t s = bs + k * C;
    if (s >= be) continue;
    const int64_t e = s + C < be ? s + C : be;
    const int32_t v = counts[reg];
    const float fv = float(v);
    int64_t a = (s + E - 1) & ~int64_t(E - 1);  // first 16-B aligned element
    if (a > e) a = e;
    const int64_t nv = (e - a) / E;
    auto one = [&](int64_t i) {
      const float m = v > 0 ? to_f(src[i]) / fv : 0.f;
      const float r = AXPY ? to_f(dst[i]) + alpha * m : m;
      dst[i] = from_f<T>(r);
      if constexpr (SHADOW) shadow[i] = from_f<unsigned short>(r);
    };
    if (blockIdx.y == 0) {
      for (int64_t i = s + threadIdx.x; i < a; i += kBlock) one(i);
      for (int64_t i = a + nv * E + threadIdx.x; i < e; i += kBlock) one(i);
    }
    const v4u* s4 = reinterpret_cast<const v4u*>(src + a);
    v4u* d4 = reinterpret_cast<v4u*>(dst + a);
    uint2* h2 = SHADOW ? reinterpret_cast<uint2*>(shadow + a) : nullptr;  // 4 bf16 per fp32 vector
    auto mean_vec = [&](const v4u& sv, const v4u& dv, int64_t at) {
      float acc[E];
#pragma unroll
      for (int q = 0; q < E; ++q) acc[q] = 0.f;
      add_vec(acc, sv, T{});
#pragma unroll
      for (int q = 0; q < E; ++q) acc[q] = v > 0 ? acc[q] / fv : 0.f;
      if constexpr (AXPY) {
        float p[E];
#pragma unroll
        for (int q = 0; q < E; ++q) p[q] = 0.f;
        add_vec(p, dv, T{});
#pragma unroll
        for (int q = 0; q < E; ++q) acc[q] = p[q] + alpha * acc[q];
      }
      if constexpr (SHADOW) {
        if constexpr (E == 4) h2[at] = make_uint2(pack_bf16x2(acc[0], acc[1]), pack_bf16x2(acc[2], acc[3]));
      }
      return pack_vec(acc);
    };
    // kCmUnroll vectors per thread: every load of the group in flight before
    // the first store (one vector at a time left the pass latency-bound)
    constexpr int U = kCmUnroll;
    const int64_t stride = int64_t(kBlock) * gridDim.y;
    int64_t i = int64_t(blockIdx.y) * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < nv; i += U * stride) {
      v4u sv[U], dv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sv[u] = s4[i + u * stride];
#pragma unroll
      for (int u = 0; u < U; ++u) dv[u] = AXPY ? d4[i + u * stride] : sv[u];
#pragma unroll
      for (int u = 0; u < U; ++u) d4[i + u * stride] = mean_vec(sv[u], dv[u], i + u * stride);
    }
    for (; i < nv; i += stride) d4[i] = mean_vec(s4[i], AXPY ? d4[i] : s4[i], i);
  }
}

// ---- column sum (the bias gradient of a linear layer) -------------------------
// out[c] = sum_r in[r, c] for a row-major bf16 [M, Ncol] matrix, fp32
// accumulation and output: db = sum over the batch of dY.  Each lane owns 8
// adjacent columns (one 16-B load per row), a wave 512 columns, and the rows
// of a column tile are split over `gridDim.y` workgroups (x 4 waves) so a
// batch of a few hundred rows still spreads over the whole chip.  Each
// workgroup leaves its fp32 partial row in `part[blockIdx.y]`; the last to
// arrive at the tile's ticket sums the partials in row-split order
// (deterministic: no float atomics) and re-arms the ticket for the next call.
// Hand-off of the partial rows: LITE = write-through (sc0 sc1) stores, a
// drained vmcnt and system-coherent loads in the last workgroup (no cache
// write-back or invalidate); otherwise device-scope release / acquire fences.
constexpr int kCsCols = 64 * 8;  // columns per workgroup (one wave's width)
constexpr int kCsRows = 8;       // rows per lane in flight
constexpr int kCsMaxSplits = 16;

// RELU: the ReLU backward rides along -- the summed value is in[r, c] where
// act[r, c] > 0, else 0, and it is also written to gout (bf16, same layout):
// dY of the layer below the activation and its bias gradient in one pass.
__device__ __forceinline__ v4u relu_mask_bf16x8(const v4u& g, const v4u& h) {
  v4u o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t gw = g[k], hw = h[k];
    // bf16 > 0: sign bit clear and not +0 (NaN passes through as > 0 is false for NaN in fp32 too)
    const bool lo = __uint_as_float(hw << 16) > 0.f, hi = __uint_as_float(hw & 0xffff0000u) > 0.f;
    o[k] = (lo ? (gw & 0xffffu) : 0u) | (hi ? (gw & 0xffff0000u) : 0u);
  }
  return o;
}

template <bool LITE, bool RELU>
__global__ __launch_bounds__(kBlock) void colsum_bf16_kernel(float* __restrict__ out,
                                                             const unsigned short* __restrict__ in, int64_t M,
                                                             int64_t ncol, float* __restrict__ part,
                                                             uint32_t* __restrict__ tickets, int32_t vec,
                                                             const unsigned short* __restrict__ act,
                                                             unsigned short* __restrict__ gout) {
  __shared__ float red[kBlock / 64][kCsCols + kCsCols / 8];
  __shared__ uint32_t last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c0 = int64_t(blockIdx.x) * kCsCols + lane * 8;
  const int64_t rows_per = (M + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = int64_t(blockIdx.y) * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (vec && c0 + 8 <= ncol) {
    // kCsRows rows in flight per lane before the adds
    int64_t r = r0 + wave;
    for (; r + 4 * (kCsRows - 1) < r1; r += 4 * kCsRows) {
      v4u v[kCsRows];
#pragma unroll
      for (int u = 0; u < kCsRows; ++u) v[u] = *reinterpret_cast<const v4u*>(in + (r + 4 * u) * ncol + c0);
      if constexpr (RELU) {
        v4u h[kCsRows];
#pragma unroll
        for (int u = 0; u < kCsRows; ++u) h[u] = *reinterpret_cast<const v4u*>(act + (r + 4 * u) * ncol + c0);
#pragma unroll
        for (int u = 0; u < kCsRows; ++u) {
          v[u] = relu_mask_bf16x8(v[u], h[u]);
          *reinterpret_cast<v4u*>(gout + (r + 4 * u) * ncol + c0) = v[u];
        }
      }
#pragma unroll
      for (int u = 0; u < kCsRows; ++u) add_vec(acc, v[u], (unsigned short)0);
    }
    for (; r < r1; r += 4) {
      v4u v = *reinterpret_cast<const v4u*>(in + r * ncol + c0);
      if constexpr (RELU) {
        v = relu_mask_bf16x8(v, *reinterpret_cast<const v4u*>(act + r * ncol + c0));
        *reinterpret_cast<v4u*>(gout + r * ncol + c0) = v;
      }
      add_vec(acc, v, (unsigned short)0);
    }
  } else {
    for (int64_t r = r0 + wave; r < r1; r += 4)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (c0 + q < ncol) {
          float g = to_f(in[r * ncol + c0 + q]);
          if constexpr (RELU) {
            if (!(to_f(act[r * ncol + c0 + q]) > 0.f)) g = 0.f;
            gout[r * ncol + c0 + q] = from_f<unsigned short>(g);
          }
          acc[q] += g;
        }
  }
  // the workgroup's 4 waves -> one partial row (acc[q] is column c0 + q),
  // staged with one pad word per lane (slot lane * 9 + q): a wave's stores of
  // one q are 9 words apart and the combine's reads of consecutive columns
  // are consecutive but for the pads -- no bank conflicts either way
#pragma unroll
  for (int q = 0; q < 8; ++q) red[wave][lane * 9 + q] = acc[q];
  __syncthreads();
  float* prow = part + int64_t(blockIdx.y) * ncol;
  const auto prs = xgmi::sys_rsrc(part, int64_t(gridDim.y) * ncol * 4);
  for (int i = threadIdx.x; i < kCsCols; i += kBlock) {
    const int64_t c = int64_t(blockIdx.x) * kCsCols + i;
    if (c >= ncol) continue;
    const int li = i + (i >> 3);  // column i of the tile = lane i / 8, element i % 8
    const float v = red[0][li] + red[1][li] + red[2][li] + red[3][li];
    if constexpr (LITE)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), prs, int((int64_t(blockIdx.y) * ncol + c) * 4), 0,
                                            xgmi::kSysAux);
    else
      prow[c] = v;
  }
  if constexpr (LITE) {
    xgmi::drain_wg();  // every wave's write-through stores performed
  } else {
    __threadfence();  // release: this workgroup's partial row before its ticket
    __syncthreads();
  }
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&tickets[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   gridDim.y - 1
               ? 1u
               : 0u;
  __syncthreads();
  if (!last) return;
  if constexpr (!LITE) __threadfence();  // acquire: every partial row of this tile
  // every partial of a column loaded before the first add (one memory
  // latency for the combine, not one per split), summed in split order
  for (int i = threadIdx.x; i < kCsCols; i += kBlock) {
    const int64_t c = int64_t(blockIdx.x) * kCsCols + i;
    if (c >= ncol) continue;
    float v[kCsMaxSplits];
#pragma unroll
    for (int y = 0; y < kCsMaxSplits; ++y) {
      v[y] = 0.f;
      if (y < int(gridDim.y)) {
        if constexpr (LITE)
          v[y] = __uint_as_float(
              __builtin_amdgcn_raw_buffer_load_b32(prs, int((int64_t(y) * ncol + c) * 4), 0, xgmi::kSysAux));
        else
          v[y] = part[int64_t(y) * ncol + c];
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int y = 0; y < kCsMaxSplits; ++y) sum += v[y];
    out[c] = sum;
  }
  if (threadIdx.x == 0)  // re-armed for the next launch on this workspace
    __hip_atomic_store(&tickets[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- fused cross entropy (the MLP's loss) -------------------------------------
// Forward: one workgroup per row of bf16 logits [B, C]: lse = log sum exp,
// loss_r = lse - x[y_r] (0 for a label outside [0, C): torch's ignore_index),
// lse kept for the backward; the mean over the valid rows is combined by the
// last-arriving workgroup (write-through per-row words, drained vmcnt, relaxed
// ticket, system-coherent loads: the colsum hand-off) in row order.
// Backward: grad[r, c] = (exp(x - lse_r) - [c == y_r]) * go / nvalid, bf16.
// Replaces autocast's fp32 upcast + log_softmax + nll_loss (+ their
// backwards and the bf16 downcast of the gradient): two launches instead of
// six, logits read once per pass.
__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  for (int o = 32; o > 0; o >>= 1) {
    const float w = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, w) : v + w;
  }
  __syncthreads();  // red may still be read by a previous reduction
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < int(blockDim.x >> 6); ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
  return r;
}

constexpr int64_t kIgnoreIndex = -100;  // torch's default ignore_index

__global__ __launch_bounds__(kBlock) void xent_fwd_kernel(const unsigned short* __restrict__ x,
                                                          const int64_t* __restrict__ y, int64_t B, int64_t C,
                                                          float* __restrict__ lse, float* __restrict__ rowloss,
                                                          float* __restrict__ out, uint32_t* __restrict__ ticket) {
  __shared__ float red[kBlock / 64 + 1];
  const int64_t r = blockIdx.x;
  const unsigned short* row = x + r * C;
  float m = -INFINITY;
  for (int64_t c = threadIdx.x; c < C; c += kBlock) m = fmaxf(m, to_f(row[c]));
  m = block_reduce(m, red, true);
  float sum = 0.f;
  for (int64_t c = threadIdx.x; c < C; c += kBlock) sum += __expf(to_f(row[c]) - m);
  sum = block_reduce(sum, red, false);
  const auto rs = xgmi::sys_rsrc(rowloss, B * 8);
  if (threadIdx.x == 0) {
    const float l = m + __logf(sum);
    const int64_t t = y[r];
    const bool valid = t >= 0 && t < C;
    // torch ignores ignore_index (-100) only; any other label outside [0, C)
    // is an error there: here the row is flagged (-1) and the loss is NaN
    const float flag = valid ? 1.f : (t == kIgnoreIndex ? 0.f : -1.f);
    lse[r] = l;
    // [loss, flag] per row, written through for the last arriver
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(valid ? l - to_f(row[t]) : 0.f), rs, int(r * 8), 0,
                                          xgmi::kSysAux);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(flag), rs, int(r * 8 + 4), 0, xgmi::kSysAux);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    red[kBlock / 64] =
        __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == uint32_t(B - 1) ? 1.f : 0.f;
  }
  __syncthreads();
  if (red[kBlock / 64] == 0.f) return;
  // last workgroup: mean over the valid rows, in row order per thread, then
  // a fixed-order tree across threads (deterministic)
  float ls = 0.f, nv = 0.f, nb = 0.f;
  for (int64_t i = threadIdx.x; i < B; i += kBlock) {
    ls += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, int(i * 8), 0, xgmi::kSysAux));
    const float f = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, int(i * 8 + 4), 0, xgmi::kSysAux));
    nv += f > 0.f ? f : 0.f;
    nb += f < 0.f ? 1.f : 0.f;
  }
  ls = block_reduce(ls, red, false);
  nv = block_reduce(nv, red, false);
  nb = block_reduce(nb, red, false);
  if (threadIdx.x == 0) {
    // torch: NaN when every row is ignored; NaN (and the bad-label count) when a label is out of range
    out[0] = (nv > 0.f && nb == 0.f) ? ls / nv : __uint_as_float(0x7fc00000u);
    out[1] = nv;
    out[2] = nb;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(kBlock) void xent_bwd_kernel(const unsigned short* __restrict__ x,
                                                          const int64_t* __restrict__ y, int64_t C,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ stat,  // [loss, nvalid]
                                                          const float* __restrict__ go,
                                                          unsigned short* __restrict__ gx) {
  const int64_t r = blockIdx.x;
  const int64_t t = y[r];
  const float nv = stat[1];
  const float scale = (t >= 0 && t < C && nv > 0.f && stat[2] == 0.f) ? go[0] / nv : 0.f;
  const float l = lse[r];
  const unsigned short* row = x + r * C;
  unsigned short* g = gx + r * C;
  for (int64_t c = threadIdx.x; c < C; c += kBlock) {
    const float p = __expf(to_f(row[c]) - l) - (c == t ? 1.f : 0.f);
    g[c] = from_f<unsigned short>(p * scale);
  }
}

template <typename T, int NSRC, int POL, int UNROLL>
void launch_vec_u(hipStream_t s, const SrcTable& t, v4u* dst, int64_t nvec, int blocks_per_cu) {
  const int64_t cap = int64_t(kCUs) * blocks_per_cu;
  int64_t want = (nvec + int64_t(kBlock) * UNROLL - 1) / (int64_t(kBlock) * UNROLL);
  int grid = int(want < cap ? (want < 1 ? 1 : want) : cap);
  hipLaunchKernelGGL((reduce_vec_kernel<T, NSRC, UNROLL, POL>), dim3(grid), dim3(kBlock), 0, s, t, dst, nvec);
}

template <typename T, int NSRC, int POL>
void launch_vec_pol(hipStream_t s, const SrcTable& t, v4u* dst, int64_t nvec, int blocks_per_cu) {
  constexpr int U0 = NSRC <= 4 ? 4 : (NSRC <= 8 ? 2 : 1);
  // kBoth (big streams): 2 vectors per lane per source, but 4 for the
  // one-source pass (1 GiB bf16: 5.69 vs 5.53 TB/s at 2 blocks/CU, pass V)
  constexpr int UNROLL = POL == kBoth ? (NSRC == 1 ? 4 : (U0 < 2 ? U0 : 2)) : U0;
  if constexpr ((NSRC == 8 && POL == kNts && std::is_same<T, float>::value) || (NSRC == 1 && POL != kNtl)) {
    // experiments (bench/reduce_kernel_bw.py, bench/n1_bigcopy.py sweeps): loads in flight per lane
    static const int u = [] {
      const char* v = std::getenv("AKKA_VEC_UNROLL");
      return v ? std::atoi(v) : 0;
    }();
    if (u == 1) return launch_vec_u<T, NSRC, POL, 1>(s, t, dst, nvec, blocks_per_cu);
    if (u == 4) return launch_vec_u<T, NSRC, POL, 4>(s, t, dst, nvec, blocks_per_cu);
    if (u == 8) return launch_vec_u<T, NSRC, POL, 8>(s, t, dst, nvec, blocks_per_cu);
  }
  launch_vec_u<T, NSRC, POL, UNROLL>(s, t, dst, nvec, blocks_per_cu);
}

template <typename T, int NSRC>
void launch_vec_n(hipStream_t s, const SrcTable& t, v4u* dst, int64_t nvec, int pol, int blocks_per_cu) {
  if (pol == kNts) launch_vec_pol<T, NSRC, kNts>(s, t, dst, nvec, blocks_per_cu);
  else if (pol == kBoth) launch_vec_pol<T, NSRC, kBoth>(s, t, dst, nvec, blocks_per_cu);
  else launch_vec_pol<T, NSRC, kNtl>(s, t, dst, nvec, blocks_per_cu);
}

template <typename T, int NSRC>
void launch_lds_n(hipStream_t s, const SrcTable& t, v4u* dst, int64_t nvec) {
  constexpr int kWaves = kBlock / 64;
  int64_t tiles = nvec / 64;
  int64_t want = (tiles + kWaves * 2 - 1) / (kWaves * 2);  // >= 2 tiles per wave to pipeline
  int grid = int(want < kMaxGrid ? (want < 1 ? 1 : want) : kMaxGrid);
  hipLaunchKernelGGL((reduce_lds_kernel<T, NSRC>), dim3(grid), dim3(kBlock), 0, s, t, dst, nvec);
}

template <typename T>
void launch_vec(hipStream_t s, const SrcTable& t, int nsrc, v4u* dst, int64_t nvec, bool lds, int pol,
                int blocks_per_cu) {
#define AKKA_CASE(K)                                                       \
  case K:                                                                  \
    if (lds && K <= 8) launch_lds_n<T, (K <= 8 ? K : 8)>(s, t, dst, nvec); \
    else launch_vec_n<T, K>(s, t, dst, nvec, pol, blocks_per_cu);         \
    break;
  switch (nsrc) {
    AKKA_CASE(1)
    AKKA_CASE(2)
    AKKA_CASE(3)
    AKKA_CASE(4)
    AKKA_CASE(5)
    AKKA_CASE(6)
    AKKA_CASE(7)
    AKKA_CASE(8)
    AKKA_CASE(9)
    AKKA_CASE(10)
    AKKA_CASE(11)
    AKKA_CASE(12)
    AKKA_CASE(13)
    AKKA_CASE(14)
    AKKA_CASE(15)
    AKKA_CASE(16)
    default:
      throw AkkaError("reduce: unsupported source count");
  }
#undef AKKA_CASE
}

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw AkkaError(std::string("akka: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

ReduceImpl reduce_impl_from_name(const char* v) {
  if (!v) return ReduceImpl::Auto;
  if (!std::strcmp(v, "vec")) return ReduceImpl::Vec;
  if (!std::strcmp(v, "lds")) return ReduceImpl::Lds;
  if (!std::strcmp(v, "scalar")) return ReduceImpl::Scalar;
  if (!std::strcmp(v, "vec_nts")) return ReduceImpl::VecNts;
  if (!std::strcmp(v, "vec_ntl")) return ReduceImpl::VecNtl;
  if (!std::strcmp(v, "vec_both")) return ReduceImpl::VecBoth;
  return ReduceImpl::Auto;
}

ReduceImpl reduce_impl_from_env() { return reduce_impl_from_name(std::getenv("AKKA_REDUCE_IMPL")); }

const char* reduce_impl_name(ReduceImpl i) {
  switch (i) {
    case ReduceImpl::Vec:
      return "vec";
    case ReduceImpl::Lds:
      return "lds";
    case ReduceImpl::Scalar:
      return "scalar";
    case ReduceImpl::VecNts:
      return "vec_nts";
    case ReduceImpl::VecNtl:
      return "vec_ntl";
    case ReduceImpl::VecBoth:
      return "vec_both";
    default:
      return "auto";
  }
}

void launch_reduce(hipStream_t s, const ReduceSpec& spec, DType dt, ReduceImpl impl) {
  if (spec.n <= 0) return;
  AKKA_CHECK(spec.nsrc >= 1 && spec.nsrc <= kMaxReduceSrc, "reduce: bad source count");
  // Common misalignment (every pointer at the same offset mod 16 B, which the
  // data plane's layout guarantees): the body runs on 16-B vectors from the
  // first aligned element and block 0 also sums the few head elements.
  int32_t head = 0;
  ReduceSpec body = spec;
  if (impl != ReduceImpl::Scalar) {
    const uintptr_t mis = reinterpret_cast<uintptr_t>(spec.dst) & 15;
    bool same = mis != 0;
    for (int i = 0; i < spec.nsrc && same; ++i) same = (reinterpret_cast<uintptr_t>(spec.srcs[i]) & 15) == mis;
    const size_t es = dt == DType::F32 ? 4 : 2;
    const int64_t h = int64_t((16 - mis) / es);
    if (same && mis % es == 0 && spec.n > h + 64) {
      head = int32_t(h);
      body.dst = static_cast<char*>(spec.dst) + h * es;
      for (int i = 0; i < spec.nsrc; ++i) body.srcs[i] = static_cast<const char*>(spec.srcs[i]) + h * es;
      body.n = spec.n - h;
    }
  }
  const ReduceSpec& sp = body;
  SrcTable t{};
  bool aligned = (reinterpret_cast<uintptr_t>(sp.dst) & 15) == 0;
  for (int i = 0; i < sp.nsrc; ++i) {
    t.p[i] = sp.srcs[i];
    aligned &= (reinterpret_cast<uintptr_t>(sp.srcs[i]) & 15) == 0;
  }
  const int64_t per_vec = dt == DType::F32 ? 4 : 8;
  const int64_t nvec = aligned ? sp.n / per_vec : 0;
  const int64_t es_b = dt == DType::F32 ? 4 : 2;
  const int64_t rbytes = int64_t(sp.nsrc) * sp.n * es_b, wbytes = sp.n * es_b;
  if (impl == ReduceImpl::Auto) {
    // Measured (profiles/README.md): LDS-DMA staging wins while the working set
    // sits in the 256 MiB Infinity Cache (chunk-sized reduces inside a round,
    // data just landed from xGMI); direct 16-B loads win for larger streams.
    impl = (rbytes + wbytes <= (int64_t(96) << 20) && sp.nsrc <= 8) ? ReduceImpl::Lds : ReduceImpl::Vec;
  }
  // Vec load/store policy and grid (bench/stream_variants.hip sweep):
  //   sources fit the Infinity Cache      -> plain loads, NT stores, 16 blocks/CU (64 for one source)
  //   big stream with a big output        -> NT loads + NT stores, unroll 2 (4 for one source), 2 blocks/CU
  //   otherwise (many sources, <=256 MiB) -> NT loads, plain stores, 4 blocks/CU
  int pol = kNtl, bpc = 4;
  if (impl == ReduceImpl::Vec) {
    // one source (the N=1 round): a grid that covers the whole stream in one
    // pass, 76 vs 80-82 us per 256 MiB fp32 (profiles/r03/pass_ai)
    if (rbytes <= (int64_t(256) << 20)) pol = kNts, bpc = sp.nsrc == 1 ? 64 : 16;
    else if (wbytes >= (int64_t(512) << 20)) pol = kBoth, bpc = 2;  // 1 GiB bf16: 5.56 vs 5.11 TB/s at 4 (profiles/r03/pass_u, pass_v)
    else pol = kNtl, bpc = 4;
  } else if (impl == ReduceImpl::VecNts) {
    pol = kNts, bpc = 16;
  } else if (impl == ReduceImpl::VecBoth) {
    pol = kBoth, bpc = 2;
  } else if (impl == ReduceImpl::VecNtl) {
    pol = kNtl, bpc = 8;
  }
  bool filled = false;
  t.head_n = head;
  if (impl == ReduceImpl::Scalar) {
    // forced scalar path over everything
  } else if (nvec > 0) {
    const bool lds = impl == ReduceImpl::Lds;
    if (const char* g = std::getenv("AKKA_VEC_BPC")) bpc = std::max(1, std::atoi(g));  // experiments
    t.fill = sp.fill;
    t.fill_value = sp.fill_value;
    t.fill_n = sp.fill ? sp.fill_n : 0;
    filled = true;
    if (dt == DType::F32) launch_vec<float>(s, t, sp.nsrc, static_cast<v4u*>(sp.dst), nvec, lds, pol, bpc);
    else launch_vec<unsigned short>(s, t, sp.nsrc, static_cast<v4u*>(sp.dst), nvec, lds, pol, bpc);
    check_launch("reduce_vec");
  }
  const int64_t done = impl == ReduceImpl::Scalar ? 0 : nvec * per_vec;
  const int64_t rest = sp.n - done;
  if (rest > 0 || (!filled && sp.fill && sp.fill_n > 0)) {
    const size_t es = dt == DType::F32 ? 4 : 2;
    SrcTable tt{};
    if (!filled) {
      tt.fill = sp.fill;
      tt.fill_value = sp.fill_value;
      tt.fill_n = sp.fill ? sp.fill_n : 0;
    }
    for (int i = 0; i < sp.nsrc; ++i) tt.p[i] = static_cast<const char*>(sp.srcs[i]) + done * es;
    int64_t want = (rest + kBlock - 1) / kBlock;
    if (want < 1) want = 1;  // fill-only launch
    int grid = int(want < kMaxGrid ? want : kMaxGrid);
    if (dt == DType::F32) {
      hipLaunchKernelGGL(reduce_scalar_kernel<float>, dim3(grid), dim3(kBlock), 0, s, tt, sp.nsrc,
                         reinterpret_cast<float*>(static_cast<char*>(sp.dst) + done * es), rest);
    } else {
      hipLaunchKernelGGL(reduce_scalar_kernel<unsigned short>, dim3(grid), dim3(kBlock), 0, s, tt, sp.nsrc,
                         reinterpret_cast<unsigned short*>(static_cast<char*>(sp.dst) + done * es), rest);
    }
    check_launch("reduce_scalar");
  }
}

namespace {
// A failed one-sided round (ipc lane wait timed out / aborted): every count
// of the round becomes 0, so the output is never handed back as exact.
__global__ void poison_counts_kernel(const uint32_t* flag, int32_t* counts, int64_t n) {
  if (__hip_atomic_load(const_cast<uint32_t*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) return;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    counts[i] = 0;
}
}  // namespace

namespace {
// An exact round's counts table in one launch: value everywhere, or 0 when
// the lane's error word is set by the time the stream gets here.
__global__ void fill_counts_kernel(const uint32_t* flag, int32_t* counts, int64_t n, int32_t value) {
  const int32_t v =
      __hip_atomic_load(const_cast<uint32_t*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 ? value : 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    counts[i] = v;
}
}  // namespace

void launch_fill_counts(hipStream_t s, const uint32_t* flag, int32_t* counts, int32_t value, int64_t n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_counts_kernel, dim3(unsigned(std::min<int64_t>(64, (n + 255) / 256))), dim3(256), 0, s,
                     flag, counts, n, value);
}

void launch_poison_counts(hipStream_t s, const uint32_t* flag, int32_t* counts, int64_t n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(poison_counts_kernel, dim3(unsigned(std::min<int64_t>(64, (n + 255) / 256))), dim3(256), 0, s,
                     flag, counts, n);
}

void launch_count_expand(hipStream_t s, int32_t* out, const int32_t* counts, int64_t S, int64_t step, int32_t N,
                         int64_t C, int32_t kmax) {
  if (S <= 0) return;
  // out must be 16-B aligned for the vector stores (torch allocations are)
  AKKA_CHECK((reinterpret_cast<uintptr_t>(out) & 15) == 0, "count_expand: output not 16-B aligned");
  const int64_t regions = int64_t(N) * kmax;
  int grid = int(regions < kMaxGrid ? regions : kMaxGrid);
  int split = int(kMaxGrid / grid);
  const int64_t per_region_vecs = (S / regions) / 4 + 1;
  const int64_t useful = (per_region_vecs + kBlock - 1) / kBlock;
  if (split > useful) split = int(useful);
  if (split < 1) split = 1;
  hipLaunchKernelGGL(count_expand_kernel, dim3(grid, split), dim3(kBlock), 0, s, out, counts, S, step, N, C, kmax);
  check_launch("count_expand");
}

int32_t colsum_row_splits(int64_t M, int64_t ncol) {
  const int64_t tiles = (ncol + kCsCols - 1) / kCsCols;
  // one workgroup per CU over the chip at most, >= 32 rows per workgroup
  int64_t r = (kCUs + tiles - 1) / tiles;
  const int64_t cap = M / 32;
  if (r > cap) r = cap;
  if (r > kCsMaxSplits) r = kCsMaxSplits;
  return int32_t(r < 1 ? 1 : r);
}

void launch_colsum_bf16(hipStream_t s, float* out, const void* in, int64_t M, int64_t ncol, float* part,
                        uint32_t* tickets, int32_t splits, bool lite, const void* act, void* gout) {
  if (ncol <= 0) return;
  AKKA_CHECK(M > 0 && splits >= 1 && splits <= kCsMaxSplits, "colsum: bad shape or row splits (1..16)");
  const int64_t tiles = (ncol + kCsCols - 1) / kCsCols;
  AKKA_CHECK(tiles < (int64_t(1) << 31), "colsum: too many columns");
  // the partial rows are addressed through one buffer resource (32-bit offsets)
  AKKA_CHECK(int64_t(splits) * ncol * 4 < (int64_t(1) << 31), "colsum: partial rows exceed 2 GiB");
  AKKA_CHECK((act == nullptr) == (gout == nullptr), "colsum: the ReLU mask needs both act and gout");
  const bool relu = act != nullptr;
  const int vec = ((reinterpret_cast<uintptr_t>(in) | (relu ? reinterpret_cast<uintptr_t>(act) |
                                                                   reinterpret_cast<uintptr_t>(gout)
                                                             : uintptr_t(0))) &
                   15) == 0 && ncol % 8 == 0
                      ? 1
                      : 0;
  const auto* a16 = static_cast<const unsigned short*>(act);
  auto* g16 = static_cast<unsigned short*>(gout);
  const dim3 grid{uint32_t(tiles), uint32_t(splits), 1u};
#define AKKA_CS(L, R)                                                                                         \
  hipLaunchKernelGGL((colsum_bf16_kernel<L, R>), grid, dim3(kBlock), 0, s, out, static_cast<const unsigned short*>(in), \
                     M, ncol, part, tickets, vec, a16, g16)
  if (lite) {
    if (relu) AKKA_CS(true, true);
    else AKKA_CS(true, false);
  } else {
    if (relu) AKKA_CS(false, true);
    else AKKA_CS(false, false);
  }
#undef AKKA_CS
  check_launch("colsum_bf16");
}

void launch_xent_fwd(hipStream_t s, const void* x, const int64_t* y, int64_t B, int64_t C, float* lse,
                     float* rowloss, float* out, uint32_t* ticket) {
  AKKA_CHECK(B >= 1 && C >= 1 && B < (int64_t(1) << 27), "xent: bad shape");
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(uint32_t(B)), dim3(kBlock), 0, s, static_cast<const unsigned short*>(x), y,
                     B, C, lse, rowloss, out, ticket);
  check_launch("xent_fwd");
}

void launch_xent_bwd(hipStream_t s, const void* x, const int64_t* y, int64_t B, int64_t C, const float* lse,
                     const float* stat, const float* go, void* gx) {
  AKKA_CHECK(B >= 1 && C >= 1, "xent: bad shape");
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(uint32_t(B)), dim3(kBlock), 0, s, static_cast<const unsigned short*>(x), y,
                     C, lse, stat, go, static_cast<unsigned short*>(gx));
  check_launch("xent_bwd");
}

void launch_count_mean(hipStream_t s, void* dst, const void* src, const int32_t* counts, int64_t S, int64_t step,
                       int32_t N, int64_t C, int32_t kmax, DType dt, bool axpy, float alpha, void* shadow) {
  if (S <= 0) return;
  AKKA_CHECK((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0,
             "count_mean: buffers must be 16-B aligned");
  AKKA_CHECK(shadow == nullptr || (axpy && dt == DType::F32 && (reinterpret_cast<uintptr_t>(shadow) & 15) == 0),
             "count_mean: a bf16 shadow needs the fp32 SGD update and a 16-B aligned buffer");
  const int64_t regions = int64_t(N) * kmax;
  // workgroups over the whole pass (AKKA_CM_MAXGRID: measurement knob)
  static const int64_t max_grid = [] {
    const char* v = std::getenv("AKKA_CM_MAXGRID");
    return v && std::atoll(v) > 0 ? int64_t(std::atoll(v)) : int64_t(kMaxGrid);
  }();
  int grid = int(regions < max_grid ? regions : max_grid);
  int split = int(max_grid / grid);
  const int64_t per_region_vecs = (S / regions) / 4 + 1;
  const int64_t useful = (per_region_vecs + kBlock - 1) / kBlock;
  if (split > useful) split = int(useful);
  if (split < 1) split = 1;
#define AKKA_CM(T, AX, SH)                                                                                       \
  hipLaunchKernelGGL((count_mean_kernel<T, AX, SH>), dim3(grid, split), dim3(kBlock), 0, s, static_cast<T*>(dst), \
                     static_cast<const T*>(src), counts, S, step, N, C, kmax, alpha,                              \
                     static_cast<unsigned short*>(shadow))
  if (dt == DType::F32) {
    if (shadow) AKKA_CM(float, true, true);
    else if (axpy) AKKA_CM(float, true, false);
    else AKKA_CM(float, false, false);
  } else {
    if (axpy) AKKA_CM(unsigned short, true, false);
    else AKKA_CM(unsigned short, false, false);
  }
#undef AKKA_CM
  check_launch("count_mean");
}

}  // namespace akka
