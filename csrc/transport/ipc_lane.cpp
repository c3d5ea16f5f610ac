// IpcLane host side: windows, handle exchange, round launch (ipc_lane.h).
#include "ipc_lane.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "../kernels/ipc_kernels.h"

namespace akka {

#define AKKA_IPC_HIP(call)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess)                                                                    \
      throw AkkaError(std::string("akka ipc: ") + #call + " failed: " + hipGetErrorString(e_)); \
  } while (0)

namespace {

constexpr char kMagic[8] = {'A', 'K', 'I', 'P', 'C', '0', '3', 0};

struct HandleBlob {  // what handle() serialises
  char magic[8];
  int32_t rank, nranks, esize, shared;  // shared: the windows are another lane's (only flags travel)
  int64_t S, slot, portion;
  char bus[32];  // PCI bus id of the rank's GPU: ranks sharing a card (tests) share its CUs
  hipIpcMemHandle_t data, gdata, flags;
};

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoll(v) : dflt;
}

}  // namespace

void* ipc_alloc_window(size_t bytes, std::string* kind) {
  const char* want = std::getenv("AKKA_IPC_MEM");
  const std::string w = want && *want ? want : "fine";
  void* p = nullptr;
  if (w == "fine" || w == "uncached") {
    const unsigned flags = w == "fine" ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
    if (hipExtMallocWithFlags(&p, bytes, flags) == hipSuccess) {
      if (kind) *kind = w;
      return p;
    }
    (void)hipGetLastError();
  }
  AKKA_IPC_HIP(hipMalloc(&p, bytes));
  if (kind) *kind = "coarse";
  return p;
}

IpcWindows::~IpcWindows() {
  if (!dev) return;
  hipSetDevice(dev->device_index());
  hipDeviceSynchronize();  // no kernel of any lane may still touch a window
  for (void* m : opened) hipIpcCloseMemHandle(m);
  if (data) hipFree(data);
  if (gdata) hipFree(gdata);
}

IpcLane::IpcLane(Device* dev, const Geometry& g, int32_t me, DType dt, int64_t capacity, const IpcLane* share)
    : dev_(dev), g_(g), me_(me), dt_(dt), es_(dtype_size(dt)) {
  AKKA_CHECK(dev_ && !dev_->is_host(), "ipc lane needs a HIP device");
  AKKA_CHECK(g_.N >= 2 && g_.N <= kIpcMaxRanks, "ipc lane: 2..16 ranks");
  AKKA_CHECK(me_ >= 0 && me_ < g_.N, "ipc lane: rank out of range");
  AKKA_IPC_HIP(hipSetDevice(dev_->device_index()));
  int64_t maxb = 0;
  for (int32_t p = 0; p < g_.N; ++p) maxb = std::max(maxb, g_.block_len(p));
  slot_ = std::max<int64_t>(64, (maxb + 63) / 64 * 64);
  // Portion: the unit one producer workgroup hands to one consumer workgroup
  // (AKKA_IPC_PORTION_BYTES, default 512 KiB; whole 1024-element multiples).
  const int64_t pbytes = std::max<int64_t>(4096, env_i64("AKKA_IPC_PORTION_BYTES", int64_t(512) << 10));
  portion_ = std::max<int64_t>(1024, (pbytes / int64_t(es_)) / 1024 * 1024);
  nportions_ = int32_t(std::max<int64_t>(1, (maxb + portion_ - 1) / portion_));
  const size_t need_in = size_t(g_.N) * size_t(slot_) * es_;
  const size_t need_out = size_t(g_.N + 1) * size_t(slot_) * es_;
  if (share && share->win_ && share->win_->open && share->win_->N == g_.N && share->win_->me == me_ &&
      share->dev_ == dev_ && share->win_->in_bytes >= need_in && share->win_->out_bytes >= need_out) {
    win_ = share->win_;  // this geometry fits the shared windows
    shared_windows_ = true;
  } else {
    // Windows sized for `capacity` elements (>= this buffer) so that lanes of
    // engines that share this one's transport can share them too.  Every part
    // stays below the 2 GiB IPC boundary (kIpcMaxWindowBytes), every rank
    // alike (the sizes are a function of the geometry), so the job keeps its
    // other exact lanes instead of hanging in open().
    const int64_t cap = std::max<int64_t>(capacity, g_.S);
    const int64_t cap_slot = std::max<int64_t>(slot_, ((cap + g_.N - 1) / g_.N + 63) / 64 * 64);
    size_t in_bytes = size_t(g_.N) * size_t(cap_slot) * es_;
    size_t out_bytes = size_t(g_.N + 1) * size_t(cap_slot) * es_;
    if (std::max(in_bytes, out_bytes) > kIpcMaxWindowBytes) {  // capacity too ambitious: just this buffer
      in_bytes = need_in;
      out_bytes = need_out;
    }
    AKKA_CHECK(std::max(in_bytes, out_bytes) <= kIpcMaxWindowBytes,
               "ipc lane: window part of " + std::to_string(std::max(in_bytes, out_bytes) >> 20) +
                   " MiB exceeds the " + std::to_string(kIpcMaxWindowBytes >> 20) +
                   " MiB an IPC mapping opens (allocations of 2 GiB or more hang in hipIpcOpenMemHandle; buffer too "
                   "large for this N: use the p2p lanes)");
    auto w = std::make_shared<IpcWindows>();
    w->N = g_.N;
    w->me = me_;
    w->in_bytes = in_bytes;
    w->out_bytes = out_bytes;
    w->data = static_cast<char*>(ipc_alloc_window(in_bytes, &w->kind));
    w->gdata = static_cast<char*>(ipc_alloc_window(out_bytes, nullptr));
    w->dev = dev_;  // set last: a throw above leaves nothing for the destructor to free twice
    w->peer_data.assign(size_t(g_.N), nullptr);
    w->peer_gdata.assign(size_t(g_.N), nullptr);
    w->peer_data[size_t(me_)] = w->data;
    w->peer_gdata[size_t(me_)] = w->gdata;
    win_ = std::move(w);
  }
  flag_bytes_ = ipc_flag_bytes(g_.N, nportions_);
  // Flags uncached: every poll and every signal goes to memory.
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&flags_), flag_bytes_, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    AKKA_IPC_HIP(hipMalloc(reinterpret_cast<void**>(&flags_), flag_bytes_));
  }
  AKKA_IPC_HIP(hipMemset(flags_, 0, flag_bytes_));
  // the error word lives in host memory: the host reads it every round for free
  AKKA_IPC_HIP(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(uint32_t),
                             hipHostMallocMapped | hipHostMallocCoherent));
  *err_host_ = 0;
  AKKA_IPC_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0));
  AKKA_IPC_HIP(hipDeviceSynchronize());
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_->device_index()) != hipSuccess || khz <= 0)
    khz = 100000;  // 100 MHz
  timeout_ticks_ = uint64_t(std::max<int64_t>(1, env_i64("AKKA_IPC_TIMEOUT_MS", 10000))) * uint64_t(khz);
  threads_ = int32_t(env_i64("AKKA_IPC_THREADS", 256));
  if (threads_ != 512 && threads_ != 1024) threads_ = 256;
  lite_ = env_i64("AKKA_IPC_LITE", 0) != 0;
  peer_flags_.assign(size_t(g_.N), nullptr);
  peer_flags_[size_t(me_)] = flags_;
}

IpcLane::~IpcLane() {
  hipSetDevice(dev_->device_index());
  hipDeviceSynchronize();  // no kernel of ours may still touch a window
  for (void* m : opened_flags_) hipIpcCloseMemHandle(m);
  if (flags_) hipFree(flags_);
  if (err_host_) hipHostFree(err_host_);
  if (round_dev_) hipFree(round_dev_);
  if (fin_ctr_) hipFree(fin_ctr_);
  // win_: freed by its last owner (IpcWindows::~IpcWindows)
}

std::string IpcLane::handle() const {
  HandleBlob b;
  std::memset(&b, 0, sizeof(b));
  std::memcpy(b.magic, kMagic, sizeof(kMagic));
  b.rank = me_;
  b.nranks = g_.N;
  b.esize = int32_t(es_);
  b.shared = shared_windows_ ? 1 : 0;
  b.S = g_.S;
  b.slot = slot_;
  b.portion = portion_;
  AKKA_IPC_HIP(hipDeviceGetPCIBusId(b.bus, int(sizeof(b.bus)) - 1, dev_->device_index()));
  if (!shared_windows_) {
    AKKA_IPC_HIP(hipIpcGetMemHandle(&b.data, win_->data));
    AKKA_IPC_HIP(hipIpcGetMemHandle(&b.gdata, win_->gdata));
  }
  AKKA_IPC_HIP(hipIpcGetMemHandle(&b.flags, flags_));
  return std::string(reinterpret_cast<const char*>(&b), sizeof(b));
}

void IpcLane::open(const std::vector<std::string>& handles) {
  AKKA_CHECK(!ready_, "ipc lane: windows already open");
  AKKA_CHECK(int32_t(handles.size()) == g_.N, "ipc lane: need one handle per rank");
  AKKA_IPC_HIP(hipSetDevice(dev_->device_index()));
  char mybus[32] = {};
  AKKA_IPC_HIP(hipDeviceGetPCIBusId(mybus, int(sizeof(mybus)) - 1, dev_->device_index()));
  int32_t sharers = 0;
  for (int32_t p = 0; p < g_.N; ++p) {
    const std::string& h = handles[size_t(p)];
    AKKA_CHECK(h.size() == sizeof(HandleBlob), "ipc lane: malformed handle");
    HandleBlob b;
    std::memcpy(&b, h.data(), sizeof(b));
    AKKA_CHECK(std::memcmp(b.magic, kMagic, sizeof(kMagic)) == 0, "ipc lane: not an ipc window handle");
    AKKA_CHECK(b.rank == p && b.nranks == g_.N && b.esize == int32_t(es_) && b.S == g_.S && b.slot == slot_ &&
                   b.portion == portion_,
               "ipc lane: rank " + std::to_string(p) + "'s window was built for another geometry");
    AKKA_CHECK((b.shared != 0) == shared_windows_,
               "ipc lane: rank " + std::to_string(p) + " shares windows where this rank does not (or the reverse)");
    if (std::strncmp(b.bus, mybus, sizeof(mybus)) == 0) ++sharers;
    if (p == me_) continue;
    if (!shared_windows_) {
      void* d = nullptr;
      void* gd = nullptr;
      AKKA_IPC_HIP(hipIpcOpenMemHandle(&d, b.data, hipIpcMemLazyEnablePeerAccess));
      win_->opened.push_back(d);
      AKKA_IPC_HIP(hipIpcOpenMemHandle(&gd, b.gdata, hipIpcMemLazyEnablePeerAccess));
      win_->opened.push_back(gd);
      win_->peer_data[size_t(p)] = static_cast<char*>(d);
      win_->peer_gdata[size_t(p)] = static_cast<char*>(gd);
    }
    void* f = nullptr;
    AKKA_IPC_HIP(hipIpcOpenMemHandle(&f, b.flags, hipIpcMemLazyEnablePeerAccess));
    opened_flags_.push_back(f);
    peer_flags_[size_t(p)] = static_cast<uint32_t*>(f);
  }
  win_->open = true;
  // Grid cap of the waiting kernels: their parked workgroups must leave room
  // for the other ranks' push kernels when several ranks share one card.
  max_wgs_ = int32_t(std::max<int64_t>(64, env_i64("AKKA_IPC_MAX_WGS", 1024) / std::max(1, sharers)));
  sharers_ = sharers;
  ready_ = true;
}

void IpcLane::round(StreamH s, const void* in, void* out, int32_t* fail_counts, int64_t fail_n, int32_t* counts_out,
                    int64_t counts_n, int32_t counts_value) {
  AKKA_CHECK(ready_, "ipc lane: open() the peer windows first");
  IpcArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int32_t p = 0; p < g_.N; ++p) {
    a.data[p] = win_->peer_data[size_t(p)];
    a.gdata[p] = win_->peer_gdata[size_t(p)];
    a.flags[p] = peer_flags_[size_t(p)];
    a.bstart[p] = g_.block_start(p);
    a.blen[p] = g_.block_len(p);
  }
  a.slot = slot_;
  a.portion = portion_;
  a.nportions = nportions_;
  a.max_wgs = max_wgs_;
  a.threads = threads_;
  a.bcast = bcast_ ? 1 : 0;
  a.fused = fused_ ? 1 : 0;
  a.lite = lite_ ? 1 : 0;
  a.N = g_.N;
  a.me = me_;
  a.round = ++round_;
  if (round_dev_on_) {
    a.round_dev = round_dev_;
    launch_ipc_round_bump(static_cast<hipStream_t>(s), round_dev_);
  }
  a.timeout = timeout_ticks_;
  a.in = static_cast<const char*>(in);
  a.out = static_cast<char*>(out);
  a.err = err_dev_;
  a.fail_counts = fail_counts;
  a.fail_n = fail_counts ? fail_n : 0;
  if (counts_out && counts_n > 0) {
    if (!fin_ctr_) {
      if (hipExtMallocWithFlags(reinterpret_cast<void**>(&fin_ctr_), 64, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        AKKA_IPC_HIP(hipMalloc(reinterpret_cast<void**>(&fin_ctr_), 64));
      }
      AKKA_IPC_HIP(hipMemset(fin_ctr_, 0, 64));
    }
    a.counts_out = counts_out;
    a.counts_n = counts_n;
    a.counts_value = counts_value;
    a.fin_ctr = fin_ctr_;
  }
  launch_ipc_round(static_cast<hipStream_t>(s), a, dt_);
  AKKA_IPC_HIP(hipGetLastError());
  ++stats_.rounds;
  if (bcast_) ++stats_.bcast_rounds;
  stats_.bytes_pushed += (g_.S - g_.block_len(me_)) * int64_t(es_);
  stats_.bytes_pulled += (g_.S - g_.block_len(me_)) * int64_t(es_);
}

void IpcLane::set_device_rounds(bool on) {
  AKKA_CHECK(ready_, "ipc lane: open() the peer windows first");
  if (on == round_dev_on_) return;
  AKKA_IPC_HIP(hipSetDevice(dev_->device_index()));
  if (!round_dev_) {
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&round_dev_), 64, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      AKKA_IPC_HIP(hipMalloc(reinterpret_cast<void**>(&round_dev_), 64));
    }
  }
  AKKA_IPC_HIP(hipDeviceSynchronize());  // every round enqueued so far has its id
  if (on) {
    AKKA_IPC_HIP(hipMemcpy(round_dev_, &round_, sizeof(uint32_t), hipMemcpyHostToDevice));
  } else {
    AKKA_IPC_HIP(hipMemcpy(&round_, round_dev_, sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  round_dev_on_ = on;
}

uint32_t IpcLane::current_round() {
  if (!round_dev_on_) return round_;
  AKKA_IPC_HIP(hipSetDevice(dev_->device_index()));
  AKKA_IPC_HIP(hipDeviceSynchronize());
  uint32_t v = 0;
  AKKA_IPC_HIP(hipMemcpy(&v, round_dev_, sizeof(uint32_t), hipMemcpyDeviceToHost));
  return v;
}

uint32_t IpcLane::error() {
  AKKA_IPC_HIP(hipSetDevice(dev_->device_index()));
  AKKA_IPC_HIP(hipDeviceSynchronize());  // the rounds enqueued so far have drained
  return error_now();
}

uint32_t IpcLane::error_now() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE); }

}  // namespace akka
