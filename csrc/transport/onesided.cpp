// OneSidedLane host side (onesided.h): windows, handle exchange, the GPU
// launch and the CPU backend.  The CPU backend runs the kernels' roles in the
// same order, calling the same protocol functions (onesided_protocol.h) on
// POSIX shared memory; only the byte movement is written twice.
#include "onesided.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <thread>
#include <tuple>

#include "../kernels/onesided_kernels.h"
#include "ipc_lane.h"

namespace akka {

using namespace os;

#define AKKA_OS_HIP(call)                                                                      \
  do {                                                                                         \
    hipError_t e_ = (call);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      throw AkkaError(std::string("akka onesided: ") + #call + " failed: " + hipGetErrorString(e_)); \
  } while (0)

namespace {

constexpr char kMagic[8] = {'A', 'K', 'O', 'S', '0', '1', 0, 0};

struct Blob {
  char magic[8];
  int32_t rank, nranks, esize, rows, parts, kmax, kind, pad;  // kind: 0 gpu, 1 cpu
  int64_t S, C, slot, part_len, shm_bytes;
  char bus[32];
  char shm[64];
  hipIpcMemHandle_t h[1 + 2 * kMaxRows];  // flags, SD rows, GD rows
  // GPU: the creating process and its raw pointers -- lanes of ONE process
  // (the single-process spec harness) map each other without IPC, which
  // refuses a process's own allocations
  int64_t pid;
  uint64_t p_flags, p_sd[kMaxRows], p_gd[kMaxRows];
};

// Memory policy of the protocol functions for HOST code acting on DEVICE
// words (the GPU spec harness's injected peer messages): blocking copies on
// a non-blocking stream, so they run while the lane's kernels spin.
struct DevFromHost {
  static hipStream_t s;
  static uint32_t ld(const uint32_t* p) {
    uint32_t v = 0;
    AKKA_OS_HIP(hipMemcpyAsync(&v, p, sizeof(v), hipMemcpyDeviceToHost, s));
    AKKA_OS_HIP(hipStreamSynchronize(s));
    return v;
  }
  static void st(uint32_t* p, uint32_t v) {
    AKKA_OS_HIP(hipMemcpyAsync(p, &v, sizeof(v), hipMemcpyHostToDevice, s));
    AKKA_OS_HIP(hipStreamSynchronize(s));
  }
  static void st_sc(uint32_t* p, uint32_t v) { st(p, v); }
  static uint32_t ld_sc(const uint32_t* p) { return ld(p); }
};
hipStream_t DevFromHost::s = nullptr;

// ONE non-blocking stream per device for every lane's host-side copies
// (inject / peek / stats_nowait), created once for the process: streams
// share the device's hardware queues (GPU_MAX_HW_QUEUES), and a copy queued
// behind a lane's waiting round kernel on a shared queue would wait for it.
hipStream_t host_side_stream(int32_t device) {
  static hipStream_t streams[64] = {};
  AKKA_CHECK(device >= 0 && device < 64, "onesided lane: device index out of range");
  if (!streams[device]) {
    hipStream_t s = nullptr;
    AKKA_OS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    streams[device] = s;
  }
  return streams[device];
}

// The round launches' CU-masked stream of a device: `keep` of every 8 CUs,
// spread over every XCD / shader engine.  One per (device, keep) for the
// whole process, never destroyed: every such stream is a hardware queue of
// its own, and a DP job's lanes (one per bucket size) each with its own
// would oversubscribe the GPU's queues (then the scheduler time-slices
// them: 10-20 ms stalls, profiles/r05/bounded/).  Returns the stream and
// the CUs kept.
// `offset` rotates the kept CUs of every group of 8 (measurement knob
// AKKA_OS_CU_DISJOINT: ranks sharing one card each on CUs of their own).
std::pair<hipStream_t, int32_t> cu_mask_stream(int32_t device, int32_t keep, int32_t offset = 0) {
  static std::mutex mu;
  static std::map<std::tuple<int32_t, int32_t, int32_t>, std::pair<hipStream_t, int32_t>> streams;
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find({device, keep, offset});
  if (it != streams.end()) return it->second;
  hipDeviceProp_t prop;
  AKKA_OS_HIP(hipGetDeviceProperties(&prop, device));
  const int32_t ncu = std::max(1, prop.multiProcessorCount);
  std::vector<uint32_t> mask(size_t((ncu + 31) / 32), 0u);
  int32_t on = 0;
  for (int32_t cu = 0; cu < ncu; ++cu)
    if ((cu % 8 - offset + 8) % 8 < keep) {
      mask[size_t(cu / 32)] |= 1u << (cu % 32);
      ++on;
    }
  hipStream_t s = nullptr;
  AKKA_OS_HIP(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()));
  return streams[{device, keep, offset}] = {s, on};
}

// Memory policy of the protocol functions on the host (shared memory between
// processes): C++ atomics; the announce / look pair is sequentially consistent.
struct HostMem {
  static uint32_t ld(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
  static void st(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
  static void st_sc(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
  static uint32_t ld_sc(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
};

inline float bf16_f32(uint16_t h) {
  uint32_t u = uint32_t(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
inline uint16_t f32_bf16(float f) {  // RNE, quiet NaN: the kernels' conversion
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return uint16_t((u >> 16) | 0x40);
  return uint16_t((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

}  // namespace

// Role sizes of the round launch.  Defaults: 256 workgroups for push and
// copy, 512 for reduce (256 threads each) -- the whole grid (~4 per CU) is
// resident at once on a GPU of its own, so the copies of landed chunks run
// while later chunks are still crossing the links.  Fixed once open() ran (the reduce pieces'
// counters count modulo nsub_).
void OneSidedLane::size_roles(int64_t wgs, int64_t push_wgs, int64_t copy_wgs) {
  const int32_t N = g_.N;
  wgs = std::max<int64_t>(1, wgs);
  const int64_t push_items = int64_t(N - 1) * Kmax_ * P_;
  const int64_t red_parts = int64_t(g_.num_chunks(me_)) * P_;
  gp_ = int32_t(std::clamp<int64_t>(push_items, 1, push_wgs > 0 ? push_wgs : wgs));
  gq_ = int32_t(std::clamp<int64_t>(push_items, 1, copy_wgs > 0 ? copy_wgs : wgs));
  // pieces of >= 4096 elements; twice the workgroups of the other roles:
  // the reduce reads N sources per element (bench/onesided_role.py: 512
  // 256-thread workgroups reach 5.0 TB/s at N=8 where 256 reach 3.7)
  const int64_t rwgs = 2 * wgs;
  const int64_t max_sub = std::max<int64_t>(1, part_len_ / 4096);
  nsub_ = red_parts > 0 ? int32_t(std::clamp<int64_t>((rwgs + red_parts - 1) / red_parts, 1, max_sub)) : 1;
  gr_ = red_parts > 0 ? int32_t(std::clamp<int64_t>(red_parts * nsub_, 1, rwgs)) : 0;
  if (const char* v = std::getenv("AKKA_OS_REDUCE_WGS")) {  // measurement knob
    const int64_t rw = std::max<int64_t>(1, std::atoll(v));
    nsub_ = red_parts > 0 ? int32_t(std::clamp<int64_t>((rw + red_parts - 1) / red_parts, 1, max_sub)) : 1;
    gr_ = red_parts > 0 ? int32_t(std::clamp<int64_t>(red_parts * nsub_, 1, rw)) : 0;
  }
}

OneSidedLane::OneSidedLane(int32_t device, int64_t S, int32_t N, int64_t C, int32_t me, DType dt,
                           const OneSidedParams& p)
    : device_(device), g_(S, N, C), me_(me), dt_(dt), es_(dtype_size(dt)), p_(p) {
  AKKA_CHECK(N >= 2 && N <= kMaxRanks, "onesided lane: 2..16 ranks");
  AKKA_CHECK(me >= 0 && me < N, "onesided lane: rank out of range");
  AKKA_CHECK(S >= 1, "onesided lane: empty buffer");
  AKKA_CHECK(p.max_lag >= 0, "onesided lane: maxLag must be >= 0");
  if (const char* hv = std::getenv("AKKA_OS_HANDOFF")) {  // lite | fenced
    if (std::strcmp(hv, "fenced") == 0) p_.fenced = true;
    else if (std::strcmp(hv, "lite") == 0) p_.fenced = false;
  }
  D_ = p.rows > 0 ? p.rows : std::max(3, p.max_lag + 2);
  D_ = std::clamp(D_, 2, kMaxRows);
  Kmax_ = std::max(1, g_.max_block_len_chunks());
  // parts: the unit one workgroup moves under one tag (64-element multiples)
  const int64_t want = std::max<int64_t>(64, (p.part_bytes > 0 ? p.part_bytes : kAutoPartBytes) / int64_t(es_));
  part_len_ = std::min(round_up(want, 64), round_up(C, 64));
  P_ = int32_t((C + part_len_ - 1) / part_len_);
  // (Splitting a small round's chunks into more parts, for more push / copy
  // workgroups, made it slower: 42-44 vs 33-37 us at 64 Ki floats, N=2 --
  // its time is hand-off latency, and every part adds a gate and a tag to
  // scan, profiles/r06/onesided_small/.)
  if (P_ > 64) {
    part_len_ = round_up((C + 63) / 64, 64);
    P_ = int32_t((C + part_len_ - 1) / part_len_);
  }
  slot_ = std::max<int64_t>(64, round_up(g_.max_block_len(), 64));
  need_r_ = std::clamp(float_threshold(p.th_reduce, N), 1, N);
  const int64_t total = g_.total_chunks();
  need_c_ = int32_t(std::clamp<int64_t>(float_threshold(p.th_complete, total), 1, std::max<int64_t>(total, 1)));
  // window output: gather rows laid out as the output itself (slot = step,
  // block p at p * step), exact thresholds only.  Nothing is zeroed in place
  // while a writer could still be storing into the row: gather_gate looks at
  // `done` after its marker and copy_role waits for in-flight markers before
  // zeroing; a call that caught up announces its output row too (begin_role)
  wo_ = p.window_output && device >= 0 && need_r_ == N && need_c_ == total && g_.step > 0 &&
        (g_.step * int64_t(es_)) % 16 == 0;
  if (wo_) slot_ = g_.step;
  AKKA_CHECK(P_ <= kMaxParts, "onesided lane: too many parts per chunk");
  AKKA_CHECK(int64_t(D_) * N * Kmax_ * P_ <= (int64_t(1) << 22),
             "onesided lane: " + std::to_string(int64_t(D_) * N * Kmax_ * P_) +
                 " chunk parts per ring -- use a larger max_chunk_size");
  L_.init(N, D_, Kmax_, P_);
  nt_ = p.threads <= 256 ? 256 : 1024;
  if (const char* v = std::getenv("AKKA_OS_THREADS")) nt_ = std::atoi(v) >= 1024 ? 1024 : 256;  // measurement knob
  int64_t wgs = p.role_wgs > 0 ? p.role_wgs : kDefaultRoleWgs;
  if (const char* v = std::getenv("AKKA_OS_ROLE_WGS")) wgs = std::max<int64_t>(1, std::atoll(v));
  size_roles(wgs);
  flag_bytes_ = size_t(L_.flag_words) * sizeof(uint32_t);
  row_bytes_ = size_t(N) * size_t(slot_) * es_;
  win_bytes_ = flag_bytes_ + 2 * size_t(D_) * row_bytes_;
  sd_.assign(size_t(D_), nullptr);
  gd_.assign(size_t(D_), nullptr);
  pfl_.assign(size_t(N), nullptr);
  psd_.assign(size_t(D_), std::vector<char*>(size_t(N), nullptr));
  pgd_.assign(size_t(D_), std::vector<char*>(size_t(N), nullptr));

  if (device_ >= 0) {
    // every row is one IPC allocation: refuse what hipIpcOpenMemHandle would hang on
    AKKA_CHECK(row_bytes_ <= kIpcMaxWindowBytes,
               "onesided lane: a window row of " + std::to_string(row_bytes_ >> 20) + " MiB exceeds the " +
                   std::to_string(kIpcMaxWindowBytes >> 20) +
                   " MiB an IPC mapping opens (allocations of 2 GiB or more hang in hipIpcOpenMemHandle)");
    AKKA_OS_HIP(hipSetDevice(device_));
    char bus[32] = {0};
    AKKA_OS_HIP(hipDeviceGetPCIBusId(bus, int(sizeof(bus)) - 1, device_));
    my_bus_ = bus;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flag_bytes_, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      AKKA_OS_HIP(hipMalloc(reinterpret_cast<void**>(&flags_), flag_bytes_));
    }
    AKKA_OS_HIP(hipMemset(flags_, 0, flag_bytes_));
    for (int32_t d = 0; d < D_; ++d) {
      sd_[size_t(d)] = static_cast<char*>(ipc_alloc_window(row_bytes_, d == 0 ? &mem_kind_ : nullptr));
      gd_[size_t(d)] = static_cast<char*>(ipc_alloc_window(row_bytes_, nullptr));
    }
    // local words: uncached, like the flag area (system-scope atomics across XCDs, no cache maintenance)
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&loc_), size_t(L_.local_words) * sizeof(uint32_t),
                              hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      AKKA_OS_HIP(hipMalloc(reinterpret_cast<void**>(&loc_), size_t(L_.local_words) * sizeof(uint32_t)));
    }
    AKKA_OS_HIP(hipMemset(loc_, 0, size_t(L_.local_words) * sizeof(uint32_t)));
    // uncached: the counters can be read while a call runs (stats_nowait)
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&stats_dev_), kNumStats * sizeof(unsigned long long),
                              hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      AKKA_OS_HIP(hipMalloc(reinterpret_cast<void**>(&stats_dev_), kNumStats * sizeof(unsigned long long)));
    }
    AKKA_OS_HIP(hipMemset(stats_dev_, 0, kNumStats * sizeof(unsigned long long)));
    AKKA_OS_HIP(hipMalloc(&tab_dev_, sizeof(Tables)));
    AKKA_OS_HIP(hipHostMalloc(reinterpret_cast<void**>(&hw_), sizeof(HostWords),
                              hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(hw_, 0, sizeof(HostWords));
    for (auto& c : hw_->status) c.call = -1;
    AKKA_OS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&hw_dev_), hw_, 0));
    AKKA_OS_HIP(hipDeviceSynchronize());
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || khz <= 0) khz = 100000;
    clock_khz_ = khz;
    timeout_ticks_ = uint64_t(std::max<int64_t>(1, p.timeout_ms)) * uint64_t(khz);
  } else {
    // one shared-memory segment: [flags | SD rows | GD rows]
    const size_t fb = size_t(round_up(int64_t(flag_bytes_), 4096));
    const size_t rb = size_t(round_up(int64_t(row_bytes_), 4096));
    shm_bytes_ = fb + 2 * size_t(D_) * rb;
    std::random_device rd;
    char name[64];
    std::snprintf(name, sizeof(name), "/akka_os_%d_%08x_r%d", int(getpid()), unsigned(rd()), int(me));
    shm_name_ = name;
    const int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    AKKA_CHECK(fd >= 0, "onesided lane: shm_open failed for " + shm_name_);
    if (ftruncate(fd, off_t(shm_bytes_)) != 0) {
      close(fd);
      shm_unlink(name);
      throw AkkaError("akka: onesided lane: ftruncate of the shared window failed");
    }
    void* m = mmap(nullptr, shm_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
      shm_unlink(name);
      throw AkkaError("akka: onesided lane: mmap of the shared window failed");
    }
    shm_base_ = static_cast<char*>(m);  // zero-filled by ftruncate
    flags_ = reinterpret_cast<uint32_t*>(shm_base_);
    for (int32_t d = 0; d < D_; ++d) {
      sd_[size_t(d)] = shm_base_ + fb + size_t(d) * rb;
      gd_[size_t(d)] = shm_base_ + fb + size_t(D_ + d) * rb;
    }
    mem_kind_ = "shm";
    loc_host_.assign(size_t(L_.local_words), 0u);
    loc_ = loc_host_.data();
    stats_host_.assign(kNumStats, 0ull);
    hw_ = new HostWords();
    std::memset(hw_, 0, sizeof(HostWords));
    for (auto& c : hw_->status) c.call = -1;
    timeout_ticks_ = uint64_t(std::max<int64_t>(1, p.timeout_ms));  // milliseconds on the host
  }
  pfl_[size_t(me_)] = flags_;
  for (int32_t d = 0; d < D_; ++d) {
    psd_[size_t(d)][size_t(me_)] = sd_[size_t(d)];
    pgd_[size_t(d)][size_t(me_)] = gd_[size_t(d)];
  }
}

OneSidedLane::~OneSidedLane() {
  if (device_ >= 0) {
    hipSetDevice(device_);
    hipDeviceSynchronize();  // none of our kernels may still touch a window
    for (void* m : opened_) hipIpcCloseMemHandle(m);  // (same-process peers: nothing opened)
    // (cu_stream_ / side_stream_: process-wide streams, never destroyed)
    if (tl_dev_) hipFree(tl_dev_);
    if (ev_in_) hipEventDestroy(static_cast<hipEvent_t>(ev_in_));
    if (ev_out_) hipEventDestroy(static_cast<hipEvent_t>(ev_out_));
    for (char* p : sd_)
      if (p) hipFree(p);
    for (char* p : gd_)
      if (p) hipFree(p);
    if (flags_) hipFree(flags_);
    if (loc_) hipFree(loc_);
    if (stats_dev_) hipFree(stats_dev_);
    if (tab_dev_) hipFree(tab_dev_);
    if (hw_) hipHostFree(hw_);
  } else {
    for (auto& pm : peer_maps_) munmap(pm.first, pm.second);
    if (shm_base_) munmap(shm_base_, shm_bytes_);
    if (!unlinked_ && !shm_name_.empty()) shm_unlink(shm_name_.c_str());
    delete hw_;
  }
}

std::string OneSidedLane::handle() const {
  Blob b;
  std::memset(&b, 0, sizeof(b));
  std::memcpy(b.magic, kMagic, sizeof(kMagic));
  b.rank = me_;
  b.nranks = g_.N;
  b.esize = int32_t(es_);
  b.rows = D_;
  b.parts = P_;
  b.kmax = Kmax_;
  b.kind = device_ >= 0 ? 0 : 1;
  b.S = g_.S;
  b.C = g_.C;
  b.slot = slot_;
  b.part_len = part_len_;
  b.shm_bytes = int64_t(shm_bytes_);
  if (device_ >= 0) {
    std::memcpy(b.bus, my_bus_.c_str(), std::min(sizeof(b.bus) - 1, my_bus_.size()));
    b.pid = int64_t(getpid());
    b.p_flags = uint64_t(reinterpret_cast<uintptr_t>(flags_));
    for (int32_t d = 0; d < D_; ++d) {
      b.p_sd[d] = uint64_t(reinterpret_cast<uintptr_t>(sd_[size_t(d)]));
      b.p_gd[d] = uint64_t(reinterpret_cast<uintptr_t>(gd_[size_t(d)]));
    }
    AKKA_OS_HIP(hipIpcGetMemHandle(&b.h[0], flags_));
    for (int32_t d = 0; d < D_; ++d) {
      AKKA_OS_HIP(hipIpcGetMemHandle(&b.h[1 + d], sd_[size_t(d)]));
      AKKA_OS_HIP(hipIpcGetMemHandle(&b.h[1 + D_ + d], gd_[size_t(d)]));
    }
  } else {
    std::snprintf(b.shm, sizeof(b.shm), "%s", shm_name_.c_str());
  }
  return std::string(reinterpret_cast<const char*>(&b), sizeof(b));
}

// Parse and check one rank's window handle against this lane's geometry.
static Blob parse_handle(const std::string& h, int32_t q, int32_t N, size_t es, int32_t D, int32_t P, int32_t Kmax,
                         const Geometry& g, int64_t slot, int64_t part_len, bool gpu) {
  AKKA_CHECK(h.size() == sizeof(Blob), "onesided lane: malformed handle");
  Blob b;
  std::memcpy(&b, h.data(), sizeof(b));
  AKKA_CHECK(std::memcmp(b.magic, kMagic, sizeof(kMagic)) == 0, "onesided lane: not a onesided window handle");
  AKKA_CHECK(b.rank == q && b.nranks == N && b.esize == int32_t(es) && b.rows == D && b.parts == P &&
                 b.kmax == Kmax && b.S == g.S && b.C == g.C && b.slot == slot && b.part_len == part_len &&
                 b.kind == (gpu ? 0 : 1),
             "onesided lane: rank " + std::to_string(q) + "'s window was built for another geometry / ring");
  return b;
}

void OneSidedLane::map_peer(int32_t q, const std::string& h) {
  const Blob b = parse_handle(h, q, g_.N, es_, D_, P_, Kmax_, g_, slot_, part_len_, device_ >= 0);
  if (device_ >= 0 && b.pid == int64_t(getpid())) {
    // a lane of this same process: its device pointers as they are
    pfl_[size_t(q)] = reinterpret_cast<uint32_t*>(uintptr_t(b.p_flags));
    for (int32_t d = 0; d < D_; ++d) {
      psd_[size_t(d)][size_t(q)] = reinterpret_cast<char*>(uintptr_t(b.p_sd[d]));
      pgd_[size_t(d)][size_t(q)] = reinterpret_cast<char*>(uintptr_t(b.p_gd[d]));
    }
  } else if (device_ >= 0) {
    void* f = nullptr;
    AKKA_OS_HIP(hipIpcOpenMemHandle(&f, b.h[0], hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(f);
    pfl_[size_t(q)] = static_cast<uint32_t*>(f);
    for (int32_t d = 0; d < D_; ++d) {
      void* sp = nullptr;
      void* gp = nullptr;
      AKKA_OS_HIP(hipIpcOpenMemHandle(&sp, b.h[1 + d], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(sp);
      AKKA_OS_HIP(hipIpcOpenMemHandle(&gp, b.h[1 + D_ + d], hipIpcMemLazyEnablePeerAccess));
      opened_.push_back(gp);
      psd_[size_t(d)][size_t(q)] = static_cast<char*>(sp);
      pgd_[size_t(d)][size_t(q)] = static_cast<char*>(gp);
    }
  } else {
    const size_t fb = size_t(round_up(int64_t(flag_bytes_), 4096));
    const size_t rb = size_t(round_up(int64_t(row_bytes_), 4096));
    const int fd = shm_open(b.shm, O_RDWR, 0600);
    AKKA_CHECK(fd >= 0, std::string("onesided lane: cannot open rank ") + std::to_string(q) + "'s window " + b.shm);
    void* m = mmap(nullptr, size_t(b.shm_bytes), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    AKKA_CHECK(m != MAP_FAILED, "onesided lane: mmap of a peer window failed");
    char* base = static_cast<char*>(m);
    peer_maps_.push_back({base, size_t(b.shm_bytes)});
    pfl_[size_t(q)] = reinterpret_cast<uint32_t*>(base);
    for (int32_t d = 0; d < D_; ++d) {
      psd_[size_t(d)][size_t(q)] = base + fb + size_t(d) * rb;
      pgd_[size_t(d)][size_t(q)] = base + fb + size_t(D_ + d) * rb;
    }
  }
}

void OneSidedLane::write_tables(void* stream) {
  if (device_ < 0) return;
  Tables t;
  std::memset(&t, 0, sizeof(t));
  for (int32_t q = 0; q < g_.N; ++q) {
    t.fl[q] = pfl_[size_t(q)];
    t.bstart[q] = g_.block_start(q);
    t.blen[q] = g_.block_len(q);
    t.nch[q] = g_.num_chunks(q);
    for (int32_t d = 0; d < D_; ++d) {
      t.sd[d][q] = psd_[size_t(d)][size_t(q)];
      t.gd[d][q] = pgd_[size_t(d)][size_t(q)];
    }
  }
  if (stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    AKKA_OS_HIP(hipMemcpyAsync(tab_dev_, &t, sizeof(t), hipMemcpyHostToDevice, s));
    AKKA_OS_HIP(hipStreamSynchronize(s));
  } else {
    AKKA_OS_HIP(hipMemcpy(tab_dev_, &t, sizeof(t), hipMemcpyHostToDevice));
  }
}

void OneSidedLane::wait_own_calls() const {
  // Only THIS lane's calls: other lanes' round kernels on the device may be
  // waiting for this rank's next call, so a device-wide synchronize could
  // stall for their whole timeout.  The last call's status record (host
  // memory its final workgroup writes) names it once the call is done.
  if (calls_ == 0) return;
  const int64_t last = calls_ - 1;
  const auto t0 = std::chrono::steady_clock::now();
  const auto limit = std::chrono::milliseconds(3 * p_.timeout_ms + 1000);
  while (__atomic_load_n(&hw_->status[last % kStatusSlots].call, __ATOMIC_ACQUIRE) < last) {
    if (std::chrono::steady_clock::now() - t0 > limit)
      throw AkkaError("onesided lane: call " + std::to_string(last) + " did not finish");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void OneSidedLane::open(const std::vector<std::string>& handles) {
  AKKA_CHECK(!ready_, "onesided lane: windows already open");
  AKKA_CHECK(int32_t(handles.size()) == g_.N, "onesided lane: need one handle per rank");
  if (device_ >= 0) AKKA_OS_HIP(hipSetDevice(device_));
  absent_.assign(size_t(g_.N), 0);
  for (int32_t q = 0; q < g_.N; ++q) {
    const std::string& h = handles[size_t(q)];
    if (q == me_) {
      (void)parse_handle(h, q, g_.N, es_, D_, P_, Kmax_, g_, slot_, part_len_, device_ >= 0);
      continue;
    }
    if (h.empty()) {
      // not a member yet (partial peer map, W:213-216): never written to or
      // waited for -- dead until add_peer() maps its window (re-init, W:87-89)
      absent_[size_t(q)] = 1;
      __atomic_store_n(&hw_->dead[q], 1u, __ATOMIC_RELEASE);
      continue;
    }
    map_peer(q, h);
  }
  if (device_ >= 0) {
    int32_t share = 0;  // member ranks on this GPU (tests / rehearsals on a 1-GPU box)
    for (int32_t q = 0; q < g_.N; ++q) {
      if (handles[size_t(q)].empty()) continue;
      Blob b;
      std::memcpy(&b, handles[size_t(q)].data(), sizeof(b));
      share += std::strncmp(b.bus, my_bus_.c_str(), sizeof(b.bus)) == 0;
    }
    shared_ranks_ = share;
    const char* kv = std::getenv("AKKA_OS_CU_KEEP");  // CUs kept of every 8 (measurement knob)
    const int32_t keep = kv ? std::clamp(std::atoi(kv), 0, 8) : std::clamp(p_.cu_keep, 0, 8);
    // (AKKA_OS_DEDICATED=1: size as on a GPU of its own although ranks share
    // this one -- the tests' way to run that path on a 1-GPU box, with grids
    // small enough for every sharing rank's to be resident at once: small
    // buffers or AKKA_OS_ROLE_WGS, see the budget below)
    const bool dedicated = share <= 1 || (std::getenv("AKKA_OS_DEDICATED") &&
                                          std::strcmp(std::getenv("AKKA_OS_DEDICATED"), "1") == 0);
    int32_t ncu = 0;
    if (keep > 0 && keep < 8) ncu = make_cu_stream(keep);
    const bool auto_roles = p_.role_wgs <= 0 && !std::getenv("AKKA_OS_ROLE_WGS");
    if (auto_roles && !dedicated) {
      // Ranks sharing this GPU: every rank's round launch must fit on the
      // card at once, or one rank's waiting workgroups could hold the slots
      // another rank's pushers need.  Budget: 768 of the card's ~1024
      // resident 256-thread workgroups (103 VGPRs: 4 per CU) for all sharing
      // ranks' grids together (pass F sweep, profiles/r04/README.md: 512 /
      // 768 / 1024 -> 1.26 / 1.15 / 1.44 ms at 256 MiB, 4 ranks).  (Members
      // only: a rank joining later keeps the grid this one was sized for.)
      // 256-thread workgroups (AKKA_OS_THREADS=1024 to measure: the budget
      // then counts 1024-thread workgroups, a quarter as many)
      const char* tv = std::getenv("AKKA_OS_THREADS");
      nt_ = (tv && std::atoi(tv) >= 1024) ? 1024 : 256;
      const int64_t total_default = ncu > 0 ? 768 * int64_t(lane_cus_) / ncu : 768;  // same density on masked CUs
      const char* bv = std::getenv("AKKA_OS_SHARED_BUDGET");  // measurement knob (resident 256-thread WGs)
      const int64_t total = bv ? std::max(16, std::atoi(bv)) : total_default;
      const int64_t budget = total * 256 / nt_ / share - 2 - g_.num_chunks(me_);
      // shares of the budget, push / reduce / copy (AKKA_OS_SHARES="p,r,c" to measure)
      int64_t sp = 1, sr = 2, sc = 1;
      if (const char* sv = std::getenv("AKKA_OS_SHARES")) {
        long a = 0, b = 0, c2 = 0;
        if (std::sscanf(sv, "%ld,%ld,%ld", &a, &b, &c2) == 3 && a > 0 && b > 0 && c2 > 0) sp = a, sr = b, sc = c2;
      }
      const int64_t unit = std::max<int64_t>(1, budget / (sp + sr + sc));
      size_roles(std::max<int64_t>(1, unit * sr / 2), unit * sp, unit * sc);
    } else if (auto_roles && ncu > 0) {
      // A GPU of its own with a bounded footprint (comm/compute overlap):
      // the default grid's density on the kept CUs, the rest of every group
      // of 8 left to the compute kernels the round overlaps
      size_roles(std::max<int64_t>(8, kDefaultRoleWgs * lane_cus_ / ncu));
    }
  }
  write_tables();
  ready_ = true;
}

void OneSidedLane::add_peer(int32_t q, const std::string& handle) {
  AKKA_CHECK(ready_, "onesided lane: open() the peer windows first");
  AKKA_CHECK(q >= 0 && q < g_.N && q != me_, "onesided lane: bad peer");
  AKKA_CHECK(absent_[size_t(q)], "onesided lane: rank " + std::to_string(q) +
                                     " is already mapped (a rank's window is mapped once; a departed rank stays dead)");
  AKKA_CHECK(!cr_.active, "onesided lane: add_peer between rounds only");
  hipStream_t hs = nullptr;
  if (device_ >= 0) {
    AKKA_OS_HIP(hipSetDevice(device_));
    // a round boundary on the device too: no call of this lane still reads
    // the pointer tables (they are rewritten below, on the process's
    // non-blocking side stream: nothing queues behind a waiting round)
    wait_own_calls();
    hs = host_side_stream(device_);
  }
  map_peer(q, handle);
  write_tables(hs);
  // Announce my position to the newcomer: I serve no round before my next
  // one any more, so its waits for my copies of those rounds end at once
  // (source_past) and its first call catches up to my window (select_round)
  // -- without this, a newcomer serving an old round would wait for copies
  // this rank already moved past until a force or its timeout.
  uint32_t next = 0;
  if (device_ >= 0) {
    AKKA_OS_HIP(hipMemcpyAsync(&next, loc_ + L_.state(kNext), sizeof(next), hipMemcpyDeviceToHost, hs));
    AKKA_OS_HIP(hipStreamSynchronize(hs));
  } else {
    next = loc_[L_.state(kNext)];
  }
  const uint32_t seen = next + 1u;
  if (device_ >= 0) {
    AKKA_OS_HIP(hipMemcpyAsync(pfl_[size_t(q)] + L_.seen(me_), &seen, sizeof(seen), hipMemcpyHostToDevice, hs));
    AKKA_OS_HIP(hipStreamSynchronize(hs));
  } else {
    HostMem::st(pfl_[size_t(q)] + L_.seen(me_), seen);
  }
  absent_[size_t(q)] = 0;
  // from the next call on: pushed to and waited for (a fresh window: no
  // word of this rank's window was ever written by it)
  __atomic_store_n(&hw_->dead[q], 0u, __ATOMIC_RELEASE);
}

std::vector<int32_t> OneSidedLane::members() const {
  std::vector<int32_t> v;
  for (int32_t q = 0; q < g_.N; ++q)
    if (q == me_ || (size_t(q) < absent_.size() && !absent_[size_t(q)])) v.push_back(q);
  return v;
}

void OneSidedLane::unlink() {
  if (device_ < 0 && !unlinked_ && !shm_name_.empty()) {
    shm_unlink(shm_name_.c_str());
    unlinked_ = true;
  }
}


int64_t OneSidedLane::round(uintptr_t stream, const void* in, void* out, int32_t* counts, int32_t kcols) {
  AKKA_CHECK(ready_, "onesided lane: open() the peer windows first");
  AKKA_CHECK(kcols >= Kmax_, "onesided lane: counts table has too few columns");
  AKKA_CHECK(out != nullptr || wo_, "onesided lane: a call without an output buffer needs the window output");
  if (device_ >= 0) {
    // A call captured into a graph runs no kernel now: the device's call
    // sequence advances once per REPLAY (note_replays), so the host's call
    // ids must not advance here -- the captured call has no id (-1).
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    const bool capturing = hipStreamIsCapturing(reinterpret_cast<hipStream_t>(stream), &cst) == hipSuccess &&
                           cst == hipStreamCaptureStatusActive;
    const int64_t call = capturing ? -1 : calls_++;
    gpu_call(stream, static_cast<const char*>(in), static_cast<char*>(out), counts, kcols);
    return call;
  }
  const int64_t call = begin(in, out, counts, kcols);
  int us = 20;
  while (!progress()) {
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = std::min(us * 2, 200);  // (a coarser back-off adds up to its cap to a round that waited)
  }
  return call;
}

// The round launch's CU-masked stream (cu_mask_stream, shared by the
// process's lanes) plus this lane's fork / join events.  Returns the
// device's CU count (lane_cus_ = CUs kept).
int32_t OneSidedLane::make_cu_stream(int32_t keep) {
  hipDeviceProp_t prop;
  AKKA_OS_HIP(hipGetDeviceProperties(&prop, device_));
  const int32_t ncu = std::max(1, prop.multiProcessorCount);
  int32_t offset = 0;
  if (const char* dv = std::getenv("AKKA_OS_CU_DISJOINT"); dv && std::strcmp(dv, "1") == 0)
    offset = (me_ * keep) % 8;  // rank me on CUs [me * keep, me * keep + keep) of every 8
  const auto [s, on] = cu_mask_stream(device_, keep, offset);
  cu_stream_ = s;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  AKKA_OS_HIP(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
  AKKA_OS_HIP(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  ev_in_ = e0;
  ev_out_ = e1;
  lane_cus_ = on;
  return ncu;
}

void OneSidedLane::gpu_call(uintptr_t stream, const char* in, char* out, int32_t* counts, int32_t kcols) {
  Args a;
  a.tab = static_cast<const Tables*>(tab_dev_);
  a.loc = loc_;
  a.stats = stats_dev_;
  a.L = L_;
  a.C = g_.C;
  a.slot = slot_;
  a.part_len = part_len_;
  a.me = me_;
  a.kme = g_.num_chunks(me_);
  a.need_r = need_r_;
  a.need_c = need_c_;
  a.max_lag = p_.max_lag;
  a.kcols = kcols;
  a.threads = nt_;
  a.gp = gp_;
  a.gr = gr_;
  a.gq = gq_;
  a.nsub = nsub_;
  a.own_wt = need_c_ < g_.total_chunks() ? 1 : 0;
  a.fenced = p_.fenced ? 1 : 0;
  a.wo = (wo_ && out == nullptr) ? 1 : 0;
  a.timeout = timeout_ticks_;
  a.in = in;
  a.out = out;
  a.counts = counts;
  a.err = &hw_dev_->err;
  a.dead = hw_dev_->dead;
  a.force = &hw_dev_->force;
  a.status = hw_dev_->status;
  AKKA_OS_HIP(hipSetDevice(device_));
  if (const char* tv = std::getenv("AKKA_OS_TIMELINE"); tv && std::strcmp(tv, "1") == 0) {
    const int64_t words = 3 * int64_t(os::onesided_grid(a));
    if (words > tl_words_) {
      if (tl_dev_) AKKA_OS_HIP(hipFree(tl_dev_));
      AKKA_OS_HIP(hipMalloc(reinterpret_cast<void**>(&tl_dev_), size_t(words) * sizeof(unsigned long long)));
      tl_words_ = words;
    }
    a.tl = tl_dev_;
  }
  hipStream_t caller = reinterpret_cast<hipStream_t>(stream);
  if (cu_stream_ && caller != static_cast<hipStream_t>(cu_stream_)) {
    // fork/join through events (graph capture follows the same edges)
    hipStream_t ls = static_cast<hipStream_t>(cu_stream_);
    AKKA_OS_HIP(hipEventRecord(static_cast<hipEvent_t>(ev_in_), caller));
    AKKA_OS_HIP(hipStreamWaitEvent(ls, static_cast<hipEvent_t>(ev_in_), 0));
    launch_onesided_call(ls, a, dt_ == DType::F32 ? 0 : 1);
    AKKA_OS_HIP(hipGetLastError());
    AKKA_OS_HIP(hipEventRecord(static_cast<hipEvent_t>(ev_out_), ls));
    AKKA_OS_HIP(hipStreamWaitEvent(caller, static_cast<hipEvent_t>(ev_out_), 0));
    return;
  }
  launch_onesided_call(caller, a, dt_ == DType::F32 ? 0 : 1);  // (the caller's stream, or the masked one itself)
  AKKA_OS_HIP(hipGetLastError());
}

// ---- CPU backend: the kernel's roles as a progress loop -------------------------

int64_t OneSidedLane::begin(const void* in, void* out, int32_t* counts, int32_t kcols) {
  AKKA_CHECK(ready_, "onesided lane: open() the peer windows first");
  AKKA_CHECK(device_ < 0, "onesided lane: begin/progress drive the CPU backend");
  AKKA_CHECK(!cr_.active, "onesided lane: a round is already in progress");
  AKKA_CHECK(kcols >= Kmax_, "onesided lane: counts table has too few columns");
  const int32_t N = g_.N, me = me_, P = P_;
  uint32_t* fl = pfl_[size_t(me)];
  uint32_t* loc = loc_;
  // begin: round selection (catch-up), the gather row announcement
  const uint32_t next = loc[L_.state(kNext)];
  const uint32_t r = select_round(next, seen_max<HostMem>(fl, L_, me), p_.max_lag);
  stats_host_[kSkippedRounds] += r - next;
  loc[L_.state(kCur)] = r;
  loc[L_.state(kNext)] = r + 1u;
  loc[L_.state(kForcedChunks)] = 0;
  if (HostMem::ld(fl + L_.done()) < r) HostMem::st(fl + L_.done(), r);
  const int32_t row = int32_t(r % uint32_t(D_));
  HostMem::st_sc(fl + L_.gread(row), r + 1u);
  cr_ = CpuRound();
  cr_.active = true;
  cr_.r = r;
  cr_.row = row;
  cr_.call = calls_++;
  cr_.in = static_cast<const char*>(in);
  cr_.out = static_cast<char*>(out);
  cr_.counts = counts;
  cr_.kcols = kcols;
  cr_.decided.assign(size_t(g_.num_chunks(me)), 0);
  cr_.deadline_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count() + int64_t(timeout_ticks_);
  // decide announces (before any look at the scatter tags)
  for (int32_t k = 0; k < g_.num_chunks(me); ++k) HostMem::st_sc(fl + L_.sread(row, k), r + 1u);
  // push: phase 1 in the kernel's item order (chunk-major, peers from me + 1)
  const int64_t items = int64_t(N - 1) * Kmax_ * P;
  for (int64_t w = 0; w < items; ++w) {
    const int32_t i = int32_t(w % (N - 1)), kj = int32_t(w / (N - 1));
    const int32_t k = kj / P, j = kj % P;
    const int32_t p = (me + 1 + i) % N;
    if (k >= g_.num_chunks(p)) continue;
    push(0, p, k, j, r, 0, cr_.in + (g_.block_start(p) + int64_t(k) * g_.C + int64_t(j) * part_len_) * int64_t(es_));
  }
  return cr_.call;
}

// A push: performed at once, or (held) queued with a copy of its bytes.
void OneSidedLane::push(int32_t phase, int32_t dst, int32_t k, int32_t j, uint32_t r, uint32_t cnt,
                        const char* src) {
  Msg m{phase, dst, k, j, r, cnt, {}};
  if (__atomic_load_n(&hw_->dead[dst], __ATOMIC_ACQUIRE) != 0u) {  // as the kernels' push role: never queued
    stats_host_[kDeadSkips] += 1;
    return;
  }
  if (!hold_) {
    exec(m, src);
    return;
  }
  const int64_t clen = std::min(g_.C, g_.block_len(phase == 0 ? dst : me_) - int64_t(k) * g_.C);
  const int64_t n = std::max<int64_t>(0, std::min(part_len_, clen - int64_t(j) * part_len_));
  m.bytes.assign(src, src + n * int64_t(es_));
  outbox_.push_back(std::move(m));
}

void OneSidedLane::exec(const Msg& m, const char* src) {
  const int32_t me = me_, q = m.dst, k = m.k, j = m.j;
  const uint32_t r = m.r;
  const int32_t row = int32_t(r % uint32_t(D_));
  if (__atomic_load_n(&hw_->dead[q], __ATOMIC_ACQUIRE) != 0u) {
    stats_host_[kDeadSkips] += 1;
    return;
  }
  uint32_t* qfl = pfl_[size_t(q)];
  if (k == 0 && j == 0) HostMem::st(qfl + L_.seen(me), r + 1u);  // implicit start at the receiver
  const int64_t tag = m.phase == 0 ? L_.stag(row, me, k, j) : L_.gtag(row, me, k, j);
  // A held message older than what this sender already wrote to that slot
  // (a later round, delivered first) is outdated: the single writer of a slot
  // moves forward only (the reference drops it on arrival, W:155-156).
  if (HostMem::ld(qfl + tag) >= tag_writing(r + 1u)) {
    stats_host_[m.phase == 0 ? kScatterOutdated : kGatherOutdated] += 1;
    return;
  }
  const int32_t g = m.phase == 0 ? scatter_gate<HostMem>(qfl, L_, row, me, k, j, r)
                                 : gather_gate<HostMem>(qfl, L_, row, me, k, j, r);
  if (m.phase == 0) stats_host_[g == kGo ? kScatterPushed : g == kOutdated ? kScatterOutdated : kScatterConflict] += 1;
  else stats_host_[g == kGo ? kGatherPushed : g == kOutdated ? kGatherOutdated : kGatherConflict] += 1;
  if (g != kGo) return;
  const int32_t blk = m.phase == 0 ? q : me;
  const int64_t clen = std::min(g_.C, g_.block_len(blk) - int64_t(k) * g_.C);
  const int64_t n = std::max<int64_t>(0, std::min(part_len_, clen - int64_t(j) * part_len_));
  const int64_t off = int64_t(k) * g_.C + int64_t(j) * part_len_;
  if (m.phase == 1) HostMem::st(qfl + tag + 1, m.cnt);  // count before the "done" tag
  char* dst = (m.phase == 0 ? psd_ : pgd_)[size_t(row)][size_t(q)] + (int64_t(me) * slot_ + off) * int64_t(es_);
  if (n > 0) std::memcpy(dst, src ? src : m.bytes.data(), size_t(n) * es_);
  HostMem::st(qfl + tag, tag_done(r));  // release: the bytes are visible first
}

void OneSidedLane::flush() {
  if (hold_) return;
  while (!outbox_.empty()) {
    Msg m = std::move(outbox_.front());
    outbox_.pop_front();
    exec(m, nullptr);
  }
}

std::vector<std::array<int64_t, 6>> OneSidedLane::outbox() const {
  std::vector<std::array<int64_t, 6>> v;
  for (const Msg& m : outbox_) v.push_back({m.phase, m.dst, m.k, m.j, int64_t(m.r), int64_t(m.cnt)});
  return v;
}

void OneSidedLane::deliver(int64_t i) {
  AKKA_CHECK(i >= 0 && i < int64_t(outbox_.size()), "onesided lane: no such outbox entry");
  Msg m = std::move(outbox_[size_t(i)]);
  outbox_.erase(outbox_.begin() + i);
  exec(m, nullptr);
}

std::string OneSidedLane::outbox_bytes(int64_t i) const {
  AKKA_CHECK(i >= 0 && i < int64_t(outbox_.size()), "onesided lane: no such outbox entry");
  const Msg& m = outbox_[size_t(i)];
  return std::string(m.bytes.begin(), m.bytes.end());
}

void OneSidedLane::inject(int32_t phase, int32_t dst, int32_t k, int32_t j, uint32_t r, uint32_t cnt,
                          const std::string& bytes, int32_t stage) {
  AKKA_CHECK(ready_, "onesided lane: open() the peer windows first");
  AKKA_CHECK(phase == 0 || phase == 1, "onesided lane: phase 0 (scatter) or 1 (gather)");
  AKKA_CHECK(dst >= 0 && dst < g_.N && dst != me_, "onesided lane: bad destination");
  const int32_t blk = phase == 0 ? dst : me_;
  AKKA_CHECK(k >= 0 && k < g_.num_chunks(blk) && j >= 0 && j < P_, "onesided lane: no such chunk part");
  const int64_t clen = std::min(g_.C, g_.block_len(blk) - int64_t(k) * g_.C);
  const int64_t n = std::max<int64_t>(0, std::min(part_len_, clen - int64_t(j) * part_len_));
  AKKA_CHECK(int64_t(bytes.size()) == n * int64_t(es_), "onesided lane: injected part has the wrong size");
  AKKA_CHECK(stage == 0 || device_ >= 0, "onesided lane: staged pushes are injected into GPU lanes");
  Msg m{phase, dst, k, j, r, cnt, std::vector<char>(bytes.begin(), bytes.end()), stage};
  if (device_ >= 0) exec_gpu(m);
  else exec(m, nullptr);
}

// inject() on a GPU lane: this rank (played by the host) pushes into the
// receiver's device window through the same gates, while the receiver's
// round kernel runs (the GPU spec harness, tests/test_onesided_spec_gpu.py).
void OneSidedLane::exec_gpu(const Msg& m) {
  AKKA_OS_HIP(hipSetDevice(device_));
  side_stream_ = host_side_stream(device_);
  DevFromHost::s = static_cast<hipStream_t>(side_stream_);
  const int32_t me = me_, q = m.dst, k = m.k, j = m.j;
  const uint32_t r = m.r;
  const int32_t row = int32_t(r % uint32_t(D_));
  if (__atomic_load_n(&hw_->dead[q], __ATOMIC_ACQUIRE) != 0u) {
    ++inj_stats_[kDeadSkips];
    return;
  }
  uint32_t* qfl = pfl_[size_t(q)];
  const int64_t tag = m.phase == 0 ? L_.stag(row, me, k, j) : L_.gtag(row, me, k, j);
  if (m.stage != 2) {  // (stage 2: the gate passed at stage 1)
    if (k == 0 && j == 0) DevFromHost::st(qfl + L_.seen(me), r + 1u);  // implicit start at the receiver
    if (DevFromHost::ld(qfl + tag) >= tag_writing(r + 1u)) {  // the slot's single writer moved past r
      ++inj_stats_[m.phase == 0 ? kScatterOutdated : kGatherOutdated];
      return;
    }
    const int32_t g = m.phase == 0 ? scatter_gate<DevFromHost>(qfl, L_, row, me, k, j, r)
                                   : gather_gate<DevFromHost>(qfl, L_, row, me, k, j, r);
    if (m.phase == 0) ++inj_stats_[g == kGo ? kScatterPushed : g == kOutdated ? kScatterOutdated : kScatterConflict];
    else ++inj_stats_[g == kGo ? kGatherPushed : g == kOutdated ? kGatherOutdated : kGatherConflict];
    if (g != kGo || m.stage == 1) return;
  }
  const int64_t off = int64_t(k) * g_.C + int64_t(j) * part_len_;
  if (m.phase == 1) DevFromHost::st(qfl + tag + 1, m.cnt);  // count before the "done" tag
  char* dst = (m.phase == 0 ? psd_ : pgd_)[size_t(row)][size_t(q)] + (int64_t(me) * slot_ + off) * int64_t(es_);
  if (!m.bytes.empty()) {
    AKKA_OS_HIP(hipMemcpyAsync(dst, m.bytes.data(), m.bytes.size(), hipMemcpyHostToDevice, DevFromHost::s));
    AKKA_OS_HIP(hipStreamSynchronize(DevFromHost::s));
  }
  DevFromHost::st(qfl + tag, tag_done(r));  // after the bytes (the copy completed)
}

std::vector<uint32_t> OneSidedLane::peek_flags() {
  std::vector<uint32_t> v(size_t(L_.flag_words), 0u);
  if (device_ < 0) {
    for (size_t i = 0; i < v.size(); ++i) v[i] = HostMem::ld(flags_ + i);
    return v;
  }
  AKKA_OS_HIP(hipSetDevice(device_));
  side_stream_ = host_side_stream(device_);
  AKKA_OS_HIP(hipMemcpyAsync(v.data(), flags_, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                             static_cast<hipStream_t>(side_stream_)));
  AKKA_OS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(side_stream_)));
  return v;
}

std::string OneSidedLane::peek_part(int32_t phase, int32_t row, int32_t src, int32_t k, int32_t j) {
  AKKA_CHECK(row >= 0 && row < D_ && src >= 0 && src < g_.N && k >= 0 && k < Kmax_ && j >= 0 && j < P_,
             "onesided lane: no such part");
  const int32_t blk = phase == 0 ? me_ : src;  // SD holds my block's chunks, GD block src's
  const int64_t clen = std::max<int64_t>(0, std::min(g_.C, g_.block_len(blk) - int64_t(k) * g_.C));
  const int64_t n = std::max<int64_t>(0, std::min(part_len_, clen - int64_t(j) * part_len_));
  const int64_t off = int64_t(k) * g_.C + int64_t(j) * part_len_;
  const char* p = (phase == 0 ? sd_ : gd_)[size_t(row)] + (int64_t(src) * slot_ + off) * int64_t(es_);
  std::string out(size_t(n) * es_, '\0');
  if (n == 0) return out;
  if (device_ < 0) {
    std::memcpy(out.data(), p, out.size());
    return out;
  }
  AKKA_OS_HIP(hipSetDevice(device_));
  side_stream_ = host_side_stream(device_);
  AKKA_OS_HIP(hipMemcpyAsync(out.data(), p, out.size(), hipMemcpyDeviceToHost, static_cast<hipStream_t>(side_stream_)));
  AKKA_OS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(side_stream_)));
  return out;
}

std::vector<uint64_t> OneSidedLane::stats_nowait() {
  std::vector<uint64_t> v(kNumStats, 0);
  if (device_ < 0) return stats();
  AKKA_OS_HIP(hipSetDevice(device_));
  side_stream_ = host_side_stream(device_);
  std::vector<unsigned long long> h(kNumStats, 0);
  AKKA_OS_HIP(hipMemcpyAsync(h.data(), stats_dev_, kNumStats * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                             static_cast<hipStream_t>(side_stream_)));
  AKKA_OS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(side_stream_)));
  for (int i = 0; i < kNumStats; ++i) v[size_t(i)] = h[size_t(i)] + inj_stats_[size_t(i)];
  return v;
}

void OneSidedLane::drop(int64_t i) {
  AKKA_CHECK(i >= 0 && i < int64_t(outbox_.size()), "onesided lane: no such outbox entry");
  outbox_.erase(outbox_.begin() + i);
}

// decide (+ reduce + phase-2 pushes) of my chunk k, if its wait is over.
bool OneSidedLane::try_decide(int32_t k, bool timed_out) {
  const int32_t N = g_.N, me = me_, P = P_;
  const uint32_t r = cr_.r;
  const int32_t row = cr_.row;
  uint32_t* fl = pfl_[size_t(me)];
  int32_t landed = 1, pending = 0;  // my own copy is always there (W:228-232)
  uint32_t mask = 1u << me;
  for (int32_t s = 0; s < N; ++s) {
    if (s == me) continue;
    int32_t dn = 0;
    bool lost = source_past<HostMem>(fl, L_, s, r);  // before the tags
    for (int32_t j = 0; j < P; ++j) {
      const int32_t st = tag_state(HostMem::ld(fl + L_.stag(row, s, k, j)), r);
      dn += st == kLanded;
      lost |= st == kLost;
    }
    if (dn == P) {
      ++landed;
      mask |= 1u << s;
    } else if (!lost && __atomic_load_n(&hw_->dead[s], __ATOMIC_ACQUIRE) == 0u) {
      ++pending;
    }
  }
  const int32_t verdict = evaluate(landed, pending, need_r_, r, seen_max<HostMem>(fl, L_, me), p_.max_lag,
                                   __atomic_load_n(&hw_->force, __ATOMIC_ACQUIRE), timed_out);
  if (verdict == kWait) return false;
  uint32_t* loc = loc_;
  const uint64_t d = (uint64_t(mask) << 32) | uint64_t(r + 1u);
  std::memcpy(&loc[L_.dec(k)], &d, 8);
  HostMem::st(fl + L_.fired(row, k), r + 1u);  // late senders of round <= r now skip
  if (verdict == kThreshold) {
    stats_host_[kReduceThreshold] += 1;
  } else {
    stats_host_[kReduceForced] += 1;
    ++loc[L_.state(kForcedChunks)];
  }
  if (verdict == kTimeout) {
    stats_host_[kTimeouts] += 1;
    __atomic_store_n(&hw_->err, 1u, __ATOMIC_RELEASE);
    dump("decide", k);
  }
  const uint32_t cnt = uint32_t(__builtin_popcount(mask));
  stats_host_[kReduceContribs] += cnt;
  // reduce: masked sum, ascending source order, fp32 accumulation -> my output block
  const size_t es = es_;
  for (int32_t j = 0; j < P; ++j) {
    const int64_t clen = std::min(g_.C, g_.block_len(me) - int64_t(k) * g_.C);
    const int64_t n = std::max<int64_t>(0, std::min(part_len_, clen - int64_t(j) * part_len_));
    const int64_t off = int64_t(k) * g_.C + int64_t(j) * part_len_;
    char* o = cr_.out + (g_.block_start(me) + off) * int64_t(es);
    if (n > 0) {
      acc_.assign(size_t(n), 0.f);
      for (int32_t s = 0; s < N; ++s) {
        if (!((mask >> s) & 1u)) continue;
        const char* src = s == me ? cr_.in + (g_.block_start(me) + off) * int64_t(es)
                                  : sd_[size_t(row)] + (int64_t(s) * slot_ + off) * int64_t(es);
        if (dt_ == DType::F32) {
          const float* f = reinterpret_cast<const float*>(src);
          for (int64_t e = 0; e < n; ++e) acc_[size_t(e)] += f[e];
        } else {
          const uint16_t* h = reinterpret_cast<const uint16_t*>(src);
          for (int64_t e = 0; e < n; ++e) acc_[size_t(e)] += bf16_f32(h[e]);
        }
      }
      if (dt_ == DType::F32) {
        std::memcpy(o, acc_.data(), size_t(n) * 4);
      } else {
        uint16_t* h = reinterpret_cast<uint16_t*>(o);
        for (int64_t e = 0; e < n; ++e) h[e] = f32_bf16(acc_[size_t(e)]);
      }
    }
    // phase 2: broadcast to every peer, rotated from me + 1 (W:254-255)
    for (int32_t i = 1; i < N; ++i) push(1, (me + i) % N, k, j, r, cnt, o);
  }
  loc[L_.odone(k)] = r + 1u;  // reduced: counts towards my completion (self-delivery, W:260-261)
  return true;
}

// complete (+ copy + finish), if its wait is over.
bool OneSidedLane::try_complete(bool timed_out) {
  const int32_t N = g_.N, me = me_, P = P_;
  const uint32_t r = cr_.r;
  const int32_t row = cr_.row;
  uint32_t* fl = pfl_[size_t(me)];
  uint32_t* loc = loc_;
  const int32_t kme = g_.num_chunks(me);
  int32_t lp = 0, pending = 0, own = 0;
  for (int32_t k = 0; k < kme; ++k) own += loc[L_.odone(k)] == r + 1u;
  for (int32_t p = 0; p < N; ++p) {
    if (p == me) continue;
    const bool past = source_past<HostMem>(fl, L_, p, r);  // before the tags
    for (int32_t k = 0; k < g_.num_chunks(p); ++k) {
      int32_t st = kLanded;
      for (int32_t j = 0; j < P; ++j) {
        const int32_t s = tag_state(HostMem::ld(fl + L_.gtag(row, p, k, j)), r);
        if (s == kLost) {
          st = kLost;
          break;
        }
        if (s == kPending) st = kPending;
      }
      if (st == kPending && (past || __atomic_load_n(&hw_->dead[p], __ATOMIC_ACQUIRE) != 0u)) st = kLost;
      lp += st == kLanded;
      pending += st == kPending;
    }
  }
  const int32_t verdict = completion_verdict(lp, pending, own, kme, need_c_, r, seen_max<HostMem>(fl, L_, me),
                                             p_.max_lag, __atomic_load_n(&hw_->force, __ATOMIC_ACQUIRE), timed_out);
  if (verdict == kWait) return false;
  // the output set, copies, the rest 0 / count 0 (copy + finish roles)
  int32_t landed = 0;
  for (int32_t p = 0; p < N; ++p) {
    for (int32_t k = 0; k < g_.num_chunks(p); ++k) {
      bool in = true;
      if (p == me) in = loc[L_.odone(k)] == r + 1u;
      else
        for (int32_t j = 0; j < P && in; ++j) in = tag_state(HostMem::ld(fl + L_.gtag(row, p, k, j)), r) == kLanded;
      loc[L_.cmask(p, k)] = in ? 1u : 0u;
      landed += in;
      const int64_t clen = g_.chunk_len(p, k);
      char* o = cr_.out + g_.chunk_offset(p, k) * int64_t(es_);
      if (in && p != me) std::memcpy(o, gd_[size_t(row)] + (int64_t(p) * slot_ + int64_t(k) * g_.C) * int64_t(es_),
                                     size_t(clen) * es_);
      if (!in) std::memset(o, 0, size_t(clen) * es_);
      uint64_t d = 0;
      if (p == me) std::memcpy(&d, &loc[L_.dec(k)], 8);
      cr_.counts[int64_t(p) * cr_.kcols + k] =
          !in ? 0 : p == me ? __builtin_popcount(uint32_t(d >> 32)) : int32_t(HostMem::ld(fl + L_.gtag(row, p, k, 0) + 1));
    }
  }
  stats_host_[verdict == kThreshold ? kCompleteThreshold : kCompleteForced] += 1;
  if (verdict == kTimeout) {
    stats_host_[kTimeouts] += 1;
    __atomic_store_n(&hw_->err, 1u, __ATOMIC_RELEASE);
    dump("complete", -1);
  }
  HostMem::st(fl + L_.done(), r + 1u);  // senders of round <= r now skip me
  // my chunks still waiting are never reduced: the round completed first
  // (the reference drops scatters of a completed round, W:155-156)
  for (int32_t k = 0; k < kme; ++k)
    if (!cr_.decided[size_t(k)]) {
      cr_.decided[size_t(k)] = 1;
      HostMem::st(fl + L_.fired(row, k), r + 1u);
      stats_host_[kReduceAbandoned] += 1;
    }
  for (int32_t k = 0; k < kme; ++k) HostMem::st(fl + L_.sread(row, k), 0u);
  HostMem::st(fl + L_.gread(row), 0u);
  stats_host_[kRounds] += 1;
  stats_host_[kLandedChunks] += uint64_t(landed);
  stats_host_[kMissingChunks] += uint64_t(g_.total_chunks() - landed);
  CallStatus& cs = hw_->status[cr_.call % kStatusSlots];
  cs.round = r;
  cs.reason = verdict;
  cs.landed_chunks = landed;
  cs.forced_chunks = loc[L_.state(kForcedChunks)];
  __atomic_store_n(&cs.call, cr_.call, __ATOMIC_RELEASE);  // the record names its call last
  cr_.active = false;
  return true;
}

bool OneSidedLane::progress() {
  flush();
  if (!cr_.active) return false;
  const int64_t now = std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  const bool timed_out = now > cr_.deadline_ms;
  for (int32_t k = 0; k < int32_t(cr_.decided.size()); ++k)
    if (!cr_.decided[size_t(k)] && try_decide(k, timed_out)) cr_.decided[size_t(k)] = 1;
  return try_complete(timed_out);
}

void OneSidedLane::dump(const char* role, int32_t k) const {
  if (!std::getenv("AKKA_OS_DEBUG")) return;
  const int32_t N = g_.N, me = me_;
  const uint32_t* fl = pfl_[size_t(me)];
  std::fprintf(stderr, "[onesided r%d] %s timeout: round %u chunk %d next %u seen/fin:", me, role, cr_.r, k,
               loc_[L_.state(kNext)]);
  for (int32_t s = 0; s < N; ++s)
    std::fprintf(stderr, " %u/%u", HostMem::ld(fl + L_.seen(s)), HostMem::ld(fl + L_.fin(s)));
  std::fprintf(stderr, " done %u | tags:", HostMem::ld(fl + L_.done()));
  for (int32_t s = 0; s < N; ++s) {
    if (s == me) continue;
    if (k >= 0) std::fprintf(stderr, " s%d=%u", s, HostMem::ld(fl + L_.stag(cr_.row, s, k, 0)));
    else
      for (int32_t kk = 0; kk < g_.num_chunks(s); ++kk)
        std::fprintf(stderr, " b%dk%d=%u", s, kk, HostMem::ld(fl + L_.gtag(cr_.row, s, kk, 0)));
  }
  std::fprintf(stderr, "\n");
}

void OneSidedLane::retire(uintptr_t stream) {
  AKKA_CHECK(ready_, "onesided lane: open() the peer windows first");
  if (device_ >= 0) {
    Args a;
    a.tab = static_cast<const Tables*>(tab_dev_);
    a.loc = loc_;
    a.L = L_;
    a.me = me_;
    AKKA_OS_HIP(hipSetDevice(device_));
    launch_onesided_retire(reinterpret_cast<hipStream_t>(stream), a);
    AKKA_OS_HIP(hipGetLastError());
  } else {
    flush();
    for (int32_t q = 0; q < g_.N; ++q)
      if (q != me_ && pfl_[size_t(q)]) HostMem::st(pfl_[size_t(q)] + L_.fin(me_), loc_[L_.state(kNext)] + 1u);
  }
}

CallStatus OneSidedLane::status(int64_t call) const {
  AKKA_CHECK(call >= 0 && call < calls_, "onesided lane: no such call");
  const CallStatus& rec = hw_->status[call % kStatusSlots];
  CallStatus c;
  c.call = __atomic_load_n(&rec.call, __ATOMIC_ACQUIRE);
  if (c.call > call)
    throw AkkaError("onesided lane: the status record of call " + std::to_string(call) + " was reused by call " +
                    std::to_string(c.call) + " (read an output's status within 64 calls)");
  c.round = c.call == call ? rec.round : -1;
  c.reason = rec.reason;
  c.landed_chunks = rec.landed_chunks;
  c.forced_chunks = rec.forced_chunks;
  return c;
}

std::vector<uint64_t> OneSidedLane::stats() {
  std::vector<uint64_t> v(kNumStats, 0);
  if (device_ >= 0) {
    AKKA_OS_HIP(hipSetDevice(device_));
    AKKA_OS_HIP(hipDeviceSynchronize());
    std::vector<unsigned long long> h(kNumStats, 0);
    AKKA_OS_HIP(hipMemcpy(h.data(), stats_dev_, kNumStats * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int i = 0; i < kNumStats; ++i) v[size_t(i)] = h[size_t(i)] + inj_stats_[size_t(i)];
  } else {
    for (int i = 0; i < kNumStats; ++i) v[size_t(i)] = stats_host_[size_t(i)];
  }
  return v;
}

uint32_t OneSidedLane::error() const { return __atomic_load_n(&hw_->err, __ATOMIC_ACQUIRE); }
void OneSidedLane::clear_error() { __atomic_store_n(&hw_->err, 0u, __ATOMIC_RELEASE); }

void OneSidedLane::set_dead(int32_t peer, bool d) {
  AKKA_CHECK(peer >= 0 && peer < g_.N && peer != me_, "onesided lane: bad peer");
  __atomic_store_n(&hw_->dead[peer], d ? 1u : 0u, __ATOMIC_RELEASE);
}

void OneSidedLane::force_below(uint32_t v) { __atomic_store_n(&hw_->force, v, __ATOMIC_RELEASE); }

std::vector<uint64_t> OneSidedLane::timeline() {
  std::vector<uint64_t> v(size_t(tl_words_), 0);
  if (!tl_dev_ || device_ < 0) return v;
  AKKA_OS_HIP(hipSetDevice(device_));
  AKKA_OS_HIP(hipDeviceSynchronize());
  AKKA_OS_HIP(hipMemcpy(v.data(), tl_dev_, v.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return v;
}

}  // namespace akka
