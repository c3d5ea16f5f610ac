// Copy kernel of the link probe (transport/link_probe.h): moves `bytes` from
// src to dst with a wide grid of 16-byte vector copies.  With dst in a peer's
// mapped window it measures remote WRITES over xGMI (push), with src there
// remote READS (pull).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace akka {
namespace {

__global__ __launch_bounds__(256) void probe_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                         int64_t n16) {
  constexpr int U = 4;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// Every peer's copy in one launch (blockIdx.y = copy): the all-peers-at-once
// pattern without a stream (hardware queue) per peer.
constexpr int kProbeMaxCopies = 16;
struct ProbeCopies {
  uint4* dst[kProbeMaxCopies];
  const uint4* src[kProbeMaxCopies];
};

__global__ __launch_bounds__(256) void probe_copies_kernel(ProbeCopies t, int64_t n16) {
  constexpr int U = 4;
  uint4* __restrict__ dst = t.dst[blockIdx.y];
  const uint4* __restrict__ src = t.src[blockIdx.y];
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

}  // namespace

void launch_probe_copies(hipStream_t s, void* const* dst, const void* const* src, int32_t n, int64_t bytes,
                         int32_t wgs) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0 || n <= 0) return;
  ProbeCopies t{};
  for (int32_t i = 0; i < n && i < kProbeMaxCopies; ++i) {
    t.dst[i] = static_cast<uint4*>(dst[i]);
    t.src[i] = static_cast<const uint4*>(src[i]);
  }
  hipLaunchKernelGGL(probe_copies_kernel, dim3(unsigned(std::max(1, wgs)), unsigned(std::min(n, kProbeMaxCopies))),
                     dim3(256), 0, s, t, n16);
}

void launch_probe_copy(hipStream_t s, void* dst, const void* src, int64_t bytes, int32_t wgs) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0) return;
  hipLaunchKernelGGL(probe_copy_kernel, dim3(unsigned(std::max(1, wgs))), dim3(256), 0, s, static_cast<uint4*>(dst),
                     static_cast<const uint4*>(src), n16);
}

}  // namespace akka
