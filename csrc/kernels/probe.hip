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

}  // namespace

void launch_probe_copy(hipStream_t s, void* dst, const void* src, int64_t bytes, int32_t wgs) {
  const int64_t n16 = bytes / 16;
  if (n16 <= 0) return;
  hipLaunchKernelGGL(probe_copy_kernel, dim3(unsigned(std::max(1, wgs))), dim3(256), 0, s, static_cast<uint4*>(dst),
                     static_cast<const uint4*>(src), n16);
}

}  // namespace akka
