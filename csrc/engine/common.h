// Shared types for the native threshold-allreduce core.
//
// The reference moves every chunk as a freshly allocated Array[Float] inside an
// Akka message (AllreduceMessage.scala:19-20).  Here a chunk is a typed view
// (pointer + element count) into memory owned by a Device (host or HIP), so the
// engine never copies payloads itself: the data plane decides whether a view is
// aliased (zero-copy self path), copied into a slot, or was written in place by
// the transport (RCCL recv straight into its final slot).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace akka {

enum class DType : int32_t { F32 = 0, BF16 = 1 };

inline size_t dtype_size(DType t) { return t == DType::F32 ? 4 : 2; }

// Where a payload lives / how it got there.
enum class PayloadKind : int32_t {
  None = 0,
  InputView = 1,    // view into this worker's own input for the round (zero-copy self scatter)
  ReducedView = 2,  // view into this worker's output row (result of its own chunk reduce)
  Landed = 3,       // transport already wrote the bytes into the destination slot
  External = 4,     // bytes owned by an inbound message (probe/TCP/gloo); must be copied
};

struct Payload {
  const void* ptr = nullptr;  // host or device pointer, per the owning Device
  int64_t len = 0;            // elements (not bytes)
  PayloadKind kind = PayloadKind::None;
  bool on_host = true;        // External payloads may be host memory even for a HIP data plane
};

class AkkaError : public std::runtime_error {
 public:
  explicit AkkaError(const std::string& m) : std::runtime_error(m) {}
};

#define AKKA_CHECK(cond, msg)                                                  \
  do {                                                                         \
    if (!(cond)) throw ::akka::AkkaError(std::string("akka: ") + (msg));       \
  } while (0)

// Reference thresholds are Scala Float and the cut-offs are computed in float32
// then truncated (ScatteredDataBuffer.scala:9, ReducedDataBuffer.scala:13-17).
// Reproduce that arithmetic bit-for-bit so th*n boundaries match the reference.
inline int32_t float_threshold(float th, int64_t n) {
  float prod = th * static_cast<float>(n);
  return static_cast<int32_t>(prod);
}

}  // namespace akka
