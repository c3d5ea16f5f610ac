// Vector partitioning: N blocks (one per worker), each split into chunks of at
// most C elements.
//
// Reference: AllreduceWorker.scala:240-250 (initDataBlockRanges / range) and
// AllreduceWorker.scala:218-223 (chunking inside scatter).  The reference uses a
// float32 ceil(dataSize*1f/peerNum), which misrounds past 2^24 elements and
// indexes out of bounds when S < N*step leaves fewer than N range entries
// (SURVEY §5.3 quirks 3-4).  Here all arithmetic is exact int64, and trailing
// blocks that fall past S are empty (0 chunks) instead of crashing.  For every
// size the reference handles correctly the block/chunk layout is identical.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "common.h"

namespace akka {

struct Geometry {
  int64_t S = 0;   // total elements
  int32_t N = 0;   // number of blocks (= workers)
  int64_t C = 1;   // max chunk size (elements)
  int64_t step = 0;

  Geometry() = default;
  Geometry(int64_t S_, int32_t N_, int64_t C_) : S(S_), N(N_), C(C_) {
    AKKA_CHECK(N_ >= 1, "peer count must be >= 1");
    AKKA_CHECK(C_ >= 1, "maxChunkSize must be >= 1");
    AKKA_CHECK(S_ >= 0, "dataSize must be >= 0");
    step = (S + N - 1) / N;
  }

  int64_t block_start(int32_t j) const { return std::min<int64_t>(int64_t(j) * step, S); }
  int64_t block_end(int32_t j) const {
    return j >= N - 1 ? S : std::min<int64_t>(int64_t(j + 1) * step, S);
  }
  int64_t block_len(int32_t j) const { return block_end(j) - block_start(j); }
  int32_t num_chunks(int32_t j) const {
    return static_cast<int32_t>((block_len(j) + C - 1) / C);
  }
  // Chunk k of block j, relative to block start.
  int64_t chunk_start(int32_t /*j*/, int32_t k) const { return int64_t(k) * C; }
  int64_t chunk_len(int32_t j, int32_t k) const {
    return std::min<int64_t>(C, block_len(j) - int64_t(k) * C);
  }
  // Absolute offset in the full vector.
  int64_t chunk_offset(int32_t j, int32_t k) const { return block_start(j) + int64_t(k) * C; }

  int32_t max_block_len_chunks() const {
    int32_t m = 0;
    for (int32_t j = 0; j < N; ++j) m = std::max(m, num_chunks(j));
    return m;
  }
  int64_t max_block_len() const {
    int64_t m = 0;
    for (int32_t j = 0; j < N; ++j) m = std::max(m, block_len(j));
    return m;
  }
  int64_t total_chunks() const {
    int64_t t = 0;
    for (int32_t j = 0; j < N; ++j) t += num_chunks(j);
    return t;
  }
  // Block index owning absolute element i.
  int32_t block_of(int64_t i) const {
    if (step == 0) return N - 1;
    int32_t j = static_cast<int32_t>(i / step);
    return std::min(j, N - 1);
  }
};

}  // namespace akka
