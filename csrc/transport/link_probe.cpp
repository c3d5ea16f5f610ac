// LinkProbe (link_probe.h).
#include "link_probe.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <random>

#include "../engine/common.h"
#include "ipc_lane.h"

namespace akka {

// probe.hip: every (dst, src) pair of the table in one launch (<= 16 pairs)
void launch_probe_copies(hipStream_t s, void* const* dst, const void* const* src, int32_t n, int64_t bytes,
                         int32_t wgs);

namespace {

#define AKKA_PROBE_HIP(call)                                                                           \
  do {                                                                                                 \
    hipError_t e_ = (call);                                                                            \
    if (e_ != hipSuccess) throw AkkaError(std::string("akka link probe: ") + #call + ": " + hipGetErrorString(e_)); \
  } while (0)

struct Blob {
  char magic[8];
  int32_t rank, kind;
  int64_t bytes;
  char shm[64];
  hipIpcMemHandle_t h;
};
constexpr char kMagic[8] = {'A', 'K', 'P', 'R', 'O', 'B', 'E', 0};

}  // namespace

LinkProbe::LinkProbe(int32_t device, int32_t rank, int32_t nranks, int64_t bytes)
    : device_(device), rank_(rank), n_(nranks), bytes_(std::max<int64_t>(16, bytes / 16 * 16)) {
  AKKA_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "link probe: bad rank");
  peer_.assign(size_t(n_), nullptr);
  if (device_ >= 0) {
    AKKA_PROBE_HIP(hipSetDevice(device_));
    buf_ = static_cast<char*>(ipc_alloc_window(size_t(bytes_), nullptr));
    AKKA_PROBE_HIP(hipMalloc(reinterpret_cast<void**>(&local_), size_t(bytes_)));
    AKKA_PROBE_HIP(hipMemset(buf_, 1, size_t(bytes_)));
    AKKA_PROBE_HIP(hipMemset(local_, 2, size_t(bytes_)));
    // ONE stream: the peers' copies share a launch (probe_copies_kernel), so the
    // probe adds one hardware queue to the process, not one per peer
    hipStream_t s;
    AKKA_PROBE_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    streams_.push_back(s);
    AKKA_PROBE_HIP(hipDeviceSynchronize());
  } else {
    std::random_device rd;
    char name[64];
    std::snprintf(name, sizeof(name), "/akka_probe_%d_%08x_r%d", int(getpid()), unsigned(rd()), int(rank));
    shm_name_ = name;
    const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    AKKA_CHECK(fd >= 0, "link probe: shm_open failed");
    if (ftruncate(fd, off_t(bytes_)) != 0) {
      close(fd);
      shm_unlink(name);
      throw AkkaError("akka: link probe: ftruncate failed");
    }
    void* m = mmap(nullptr, size_t(bytes_), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    AKKA_CHECK(m != MAP_FAILED, "link probe: mmap failed");
    buf_ = static_cast<char*>(m);
    local_ = new char[size_t(bytes_)];
    std::memset(local_, 2, size_t(bytes_));
  }
  peer_[size_t(rank_)] = buf_;
}

LinkProbe::~LinkProbe() {
  if (device_ >= 0) {
    hipSetDevice(device_);
    hipDeviceSynchronize();
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    for (void* s : streams_) hipStreamDestroy(static_cast<hipStream_t>(s));
    if (buf_) hipFree(buf_);
    if (local_) hipFree(local_);
  } else {
    for (auto& m : maps_) munmap(m.first, m.second);
    if (buf_) munmap(buf_, size_t(bytes_));
    if (!unlinked_ && !shm_name_.empty()) shm_unlink(shm_name_.c_str());
    delete[] local_;
  }
}

std::string LinkProbe::handle() const {
  Blob b;
  std::memset(&b, 0, sizeof(b));
  std::memcpy(b.magic, kMagic, sizeof(kMagic));
  b.rank = rank_;
  b.kind = device_ >= 0 ? 0 : 1;
  b.bytes = bytes_;
  if (device_ >= 0) AKKA_PROBE_HIP(hipIpcGetMemHandle(&b.h, buf_));
  else std::snprintf(b.shm, sizeof(b.shm), "%s", shm_name_.c_str());
  return std::string(reinterpret_cast<const char*>(&b), sizeof(b));
}

void LinkProbe::open(const std::vector<std::string>& handles) {
  AKKA_CHECK(int32_t(handles.size()) == n_, "link probe: need one handle per rank");
  if (device_ >= 0) AKKA_PROBE_HIP(hipSetDevice(device_));
  for (int32_t q = 0; q < n_; ++q) {
    if (q == rank_) continue;
    Blob b;
    AKKA_CHECK(handles[size_t(q)].size() == sizeof(b), "link probe: malformed handle");
    std::memcpy(&b, handles[size_t(q)].data(), sizeof(b));
    AKKA_CHECK(std::memcmp(b.magic, kMagic, sizeof(kMagic)) == 0 && b.rank == q && b.bytes == bytes_ &&
                   b.kind == (device_ >= 0 ? 0 : 1),
               "link probe: rank " + std::to_string(q) + "'s handle does not match");
    if (device_ >= 0) {
      void* p = nullptr;
      AKKA_PROBE_HIP(hipIpcOpenMemHandle(&p, b.h, hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(p);
      peer_[size_t(q)] = static_cast<char*>(p);
    } else {
      const int fd = shm_open(b.shm, O_RDWR, 0600);
      AKKA_CHECK(fd >= 0, "link probe: cannot open a peer's buffer");
      void* m = mmap(nullptr, size_t(bytes_), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      AKKA_CHECK(m != MAP_FAILED, "link probe: mmap of a peer's buffer failed");
      maps_.push_back({static_cast<char*>(m), size_t(bytes_)});
      peer_[size_t(q)] = static_cast<char*>(m);
    }
  }
}

void LinkProbe::unlink() {
  if (device_ < 0 && !unlinked_ && !shm_name_.empty()) {
    shm_unlink(shm_name_.c_str());
    unlinked_ = true;
  }
}

double LinkProbe::push(const std::vector<int32_t>& peers, int32_t iters) { return run(peers, iters, true); }
double LinkProbe::pull(const std::vector<int32_t>& peers, int32_t iters) { return run(peers, iters, false); }

double LinkProbe::run(const std::vector<int32_t>& peers, int32_t iters, bool push) {
  for (int32_t q : peers) AKKA_CHECK(q >= 0 && q < n_ && q != rank_ && peer_[size_t(q)], "link probe: bad peer");
  iters = std::max(1, iters);
  if (device_ < 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int32_t it = 0; it < iters; ++it)
      for (int32_t q : peers) {
        if (push) std::memcpy(peer_[size_t(q)], local_, size_t(bytes_));
        else std::memcpy(local_, peer_[size_t(q)], size_t(bytes_));
      }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  AKKA_PROBE_HIP(hipSetDevice(device_));
  // every peer's copy in one launch per iteration (blockIdx.y = peer); 1024
  // workgroups per copy keep plenty of 16-byte requests in flight per link
  AKKA_CHECK(peers.size() <= 16, "link probe: at most 16 peers per launch");
  const int32_t wgs = 1024;
  std::vector<void*> dst(peers.size());
  std::vector<const void*> src(peers.size());
  for (size_t i = 0; i < peers.size(); ++i) {
    const int32_t q = peers[i];
    dst[i] = push ? static_cast<void*>(peer_[size_t(q)]) : static_cast<void*>(local_);
    src[i] = push ? static_cast<const void*>(local_) : static_cast<const void*>(peer_[size_t(q)]);
  }
  hipStream_t s = static_cast<hipStream_t>(streams_[0]);
  auto enqueue = [&](int32_t reps) {
    for (int32_t it = 0; it < reps; ++it)
      launch_probe_copies(s, dst.data(), src.data(), int32_t(peers.size()), bytes_, wgs);
  };
  enqueue(1);  // warm-up (mapping, TLB)
  AKKA_PROBE_HIP(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  enqueue(iters);
  AKKA_PROBE_HIP(hipGetLastError());
  AKKA_PROBE_HIP(hipDeviceSynchronize());
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace akka
