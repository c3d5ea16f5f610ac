// Streaming-kernel variant sweep for the chunk reduce on gfx950 (standalone:
// hipcc --offload-arch=gfx950 -O3 bench/stream_variants.hip -o build/stream_variants).
//
// dst = sum of NSRC sources, 16-B vectors, grid-stride.  Variants: nontemporal
// loads (NTL), nontemporal stores (NTS), unroll depth, blocks per CU.  Prints
// one JSON line per (size, nsrc, variant) with achieved (NSRC+1)*bytes/time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

struct Srcs {
  const v4u* p[8];
};

template <int NSRC, int UNROLL, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void sum_kernel(Srcs s, v4u* __restrict__ dst, long nvec) {
  const long stride = long(gridDim.x) * 256;
  for (long base = long(blockIdx.x) * 256 + threadIdx.x; base < nvec; base += stride * UNROLL) {
    v4u v[UNROLL][NSRC];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long i = base + u * stride;
      if (i < nvec) {
#pragma unroll
        for (int k = 0; k < NSRC; ++k) v[u][k] = NTL ? __builtin_nontemporal_load(s.p[k] + i) : s.p[k][i];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const long i = base + u * stride;
      if (i < nvec) {
        float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
        for (int k = 0; k < NSRC; ++k) {
          a0 += __uint_as_float(v[u][k].x);
          a1 += __uint_as_float(v[u][k].y);
          a2 += __uint_as_float(v[u][k].z);
          a3 += __uint_as_float(v[u][k].w);
        }
        v4u r = {__float_as_uint(a0), __float_as_uint(a1), __float_as_uint(a2), __float_as_uint(a3)};
        if (NTS) __builtin_nontemporal_store(r, dst + i);
        else dst[i] = r;
      }
    }
  }
}

template <int NSRC, int UNROLL, bool NTL, bool NTS>
void run(const char* name, const Srcs& s, v4u* dst, long nvec, int bpc, double mib) {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  long want = (nvec + 256L * UNROLL - 1) / (256L * UNROLL);
  int grid = int(want < long(cus) * bpc ? want : long(cus) * bpc);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((sum_kernel<NSRC, UNROLL, NTL, NTS>), dim3(grid), dim3(256), 0, 0, s, dst, nvec);
  CHECK(hipDeviceSynchronize());
  const int iters = 10;
  CHECK(hipEventRecord(a, 0));
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((sum_kernel<NSRC, UNROLL, NTL, NTS>), dim3(grid), dim3(256), 0, 0, s, dst, nvec);
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  double tbps = (NSRC + 1) * mib * 1048576.0 / (ms * 1e-3) / 1e12;
  std::printf("{\"MiB\": %.0f, \"nsrc\": %d, \"variant\": \"%s\", \"unroll\": %d, \"blocks_per_cu\": %d, \"us\": %.1f, \"TBps\": %.3f}\n",
              mib, NSRC, name, UNROLL, bpc, ms * 1e3, tbps);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

template <int NSRC>
void sweep(double mib) {
  const long n = long(mib * 1048576.0 / 4);
  const long nvec = n / 4;
  Srcs s{};
  std::vector<void*> bufs;
  for (int k = 0; k < NSRC; ++k) {
    void* p;
    CHECK(hipMalloc(&p, n * 4));
    CHECK(hipMemset(p, 0, n * 4));
    s.p[k] = static_cast<const v4u*>(p);
    bufs.push_back(p);
  }
  v4u* dst;
  CHECK(hipMalloc(&dst, n * 4));
  for (int bpc : {4, 8, 16}) {
    run<NSRC, 4, true, false>("ntl", s, dst, nvec, bpc, mib);
    run<NSRC, 4, false, false>("plain", s, dst, nvec, bpc, mib);
    run<NSRC, 4, true, true>("ntl+nts", s, dst, nvec, bpc, mib);
    run<NSRC, 4, false, true>("nts", s, dst, nvec, bpc, mib);
    run<NSRC, 8, true, true>("ntl+nts", s, dst, nvec, bpc, mib);
    run<NSRC, 2, true, true>("ntl+nts", s, dst, nvec, bpc, mib);
  }
  for (void* p : bufs) CHECK(hipFree(p));
  CHECK(hipFree(dst));
}

int main() {
  for (double mib : {64.0, 256.0, 1024.0}) {
    sweep<1>(mib);
    sweep<2>(mib);
  }
  sweep<8>(32.0);
  sweep<8>(256.0);
  return 0;
}
