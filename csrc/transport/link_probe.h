// LinkProbe: measured bandwidth of the links between the ranks of a node.
//
// SURVEY §5.8 prices the direct algorithm at ~153 GB/s per xGMI link (7 links
// per MI355X, algbw <= N * L / 2); this probe measures what a rank actually
// gets per ordered pair -- remote writes (push) and remote reads (pull) of a
// buffer through the same IPC mappings the one-sided lanes use -- and with
// every peer at once.  It replaces nothing in the reference (Akka remoting,
// application.conf:5-11, has no such probe); it validates the bound the
// bench compares against and explains the lanes' push-vs-pull choice.
//
// GPU: fine-grained buffers exported with IPC handles, a wide copy kernel,
// timed with events.  CPU (device < 0): POSIX shared memory + memcpy (the
// rehearsal of the flow; not a link measurement).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace akka {

class LinkProbe {
 public:
  LinkProbe(int32_t device, int32_t rank, int32_t nranks, int64_t bytes);
  ~LinkProbe();
  LinkProbe(const LinkProbe&) = delete;
  LinkProbe& operator=(const LinkProbe&) = delete;

  std::string handle() const;
  void open(const std::vector<std::string>& handles);
  void unlink();
  // Seconds for `iters` copies of the whole buffer to (push) / from (pull)
  // `peer`'s buffer; `peers` empty = one peer; several = all of them at once
  // (one stream each, all enqueued before any completes).
  double push(const std::vector<int32_t>& peers, int32_t iters);
  double pull(const std::vector<int32_t>& peers, int32_t iters);
  int64_t bytes() const { return bytes_; }

 private:
  double run(const std::vector<int32_t>& peers, int32_t iters, bool push);
  int32_t device_, rank_, n_;
  int64_t bytes_;
  char* buf_ = nullptr;    // exported (peers write / read it)
  char* local_ = nullptr;  // private source / destination
  std::vector<char*> peer_;
  std::vector<void*> opened_;
  std::vector<void*> streams_;
  std::string shm_name_;
  bool unlinked_ = false;
  std::vector<std::pair<char*, size_t>> maps_;
};

}  // namespace akka
