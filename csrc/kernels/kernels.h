// Launchers for the gfx950 kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../engine/device.h"

namespace akka {

enum class ReduceImpl : int32_t {
  Auto = 0,     // pick per call from the working set (profiles/README.md)
  Vec = 1,      // 16-B global loads straight to VGPRs; load/store policy picked per call
  Lds = 2,      // global_load_lds (LDS-DMA) double-buffered staging, then ds_read + sum
  Scalar = 3,   // unaligned fallback
  VecNts = 4,   // vec, plain loads + nontemporal stores (inputs stay in the Infinity Cache)
  VecNtl = 5,   // vec, nontemporal loads + plain stores
  VecBoth = 6,  // vec, nontemporal loads and stores, unroll 2 (large streams)
};
ReduceImpl reduce_impl_from_name(const char* name);

// dst = sum(srcs) over n elements (fp32 accumulate).
void launch_reduce(hipStream_t s, const ReduceSpec& spec, DType dt, ReduceImpl impl);
// counts[N][kmax] (per block, per chunk) -> out[S] (per element), RB:41-47.
void launch_count_expand(hipStream_t s, int32_t* out, const int32_t* counts, int64_t S, int64_t step, int32_t N,
                         int64_t C, int32_t kmax);
// dst = src / per-chunk count (0 where the count is 0), one pass; with
// `axpy`: dst += alpha * that mean (fused SGD update).
void launch_count_mean(hipStream_t s, void* dst, const void* src, const int32_t* counts, int64_t S, int64_t step,
                       int32_t N, int64_t C, int32_t kmax, DType dt, bool axpy = false, float alpha = 0.f,
                       void* shadow = nullptr);
// out[c] = sum_r in[r, c] (bf16 [M, ncol] row-major, fp32 out): the bias
// gradient.  part: fp32 [splits, ncol] workspace; tickets: uint32
// [ceil(ncol / 512)] zeroed once (each launch leaves them zero again).
// act / gout (both or neither, bf16 [M, ncol]): ReLU backward fused in --
// gout = in where act > 0 else 0, and out sums gout.
void launch_colsum_bf16(hipStream_t s, float* out, const void* in, int64_t M, int64_t ncol, float* part,
                        uint32_t* tickets, int32_t splits, bool lite = true, const void* act = nullptr,
                        void* gout = nullptr);
int32_t colsum_row_splits(int64_t M, int64_t ncol);
// Cross entropy over bf16 logits [B, C] with int64 labels (mean over the rows
// whose label is in [0, C)).  Forward: lse [B] fp32, rowloss [2B] fp32
// workspace, out [2] = {loss, valid rows}, ticket: one uint32 zeroed once.
// Backward: gx [B, C] bf16 = d(loss)/d(x) * go[0].
void launch_xent_fwd(hipStream_t s, const void* x, const int64_t* y, int64_t B, int64_t C, float* lse,
                     float* rowloss, float* out, uint32_t* ticket);
void launch_xent_bwd(hipStream_t s, const void* x, const int64_t* y, int64_t B, int64_t C, const float* lse,
                     const float* stat, const float* go, void* gx);
// counts[0..n) = 0 if *flag != 0 (read when the kernel runs): poisons the
// counts of a one-sided round whose waits failed.
void launch_poison_counts(hipStream_t s, const uint32_t* flag, int32_t* counts, int64_t n);
// counts[0..n) = (*flag != 0 ? 0 : value): fill + poison of an exact round in one launch.
void launch_fill_counts(hipStream_t s, const uint32_t* flag, int32_t* counts, int32_t value, int64_t n);
// Standalone kernels for tests/bench: out = a (+ b ...) via a pointer table on device.
ReduceImpl reduce_impl_from_env();
const char* reduce_impl_name(ReduceImpl i);

}  // namespace akka
