#include <atomic>
#include "watchdog.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>

namespace akka {

namespace {

struct State {
  std::mutex mu;
  bool armed = false;
  std::chrono::steady_clock::time_point deadline;
  double seconds = 0;
  std::string line;
  bool to_stdout = false;
  std::atomic<int> out_fd{1};  // "stdout" for failure lines (watchdog_set_out_fd)
  std::string debug_path;
  std::string beacon_path;
  int exit_code = 3;
  int tail_bytes = 4096;
  int pipe_r = -1, pipe_w = -1;
  bool started = false;
  // child processes to take down with this one (watchdog_track_child): a
  // watchdog exit skips every Python `finally`, and a child left behind (a
  // master of bench.py's cluster configs) would run on without its parent
  std::atomic<int> children[16] = {};
};

State& st() {
  static State* s = new State();  // never destroyed: the thread may outlive static teardown
  return *s;
}

void write_all(int fd, const std::string& s) {
  const char* p = s.data();
  size_t left = s.size();
  while (left > 0) {
    ssize_t n = ::write(fd, p, left);
    if (n <= 0) return;
    p += n;
    left -= size_t(n);
  }
}

std::string read_tail(const std::string& path, int bytes) {
  if (path.empty()) return "";
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return "";
  off_t end = ::lseek(fd, 0, SEEK_END);
  off_t start = end > bytes ? end - bytes : 0;
  ::lseek(fd, start, SEEK_SET);
  std::string out(size_t(end - start), '\0');
  ssize_t got = ::read(fd, out.data(), out.size());
  ::close(fd);
  out.resize(got > 0 ? size_t(got) : 0);
  return out;
}

void replace_token(std::string& s, const std::string& token, const std::string& value) {
  size_t pos = s.find(token);
  if (pos != std::string::npos) s.replace(pos, token.size(), value);
}

void kill_children() {
  for (auto& c : st().children) {
    const int pid = c.exchange(0);
    if (pid > 0) ::kill(pid, SIGKILL);
  }
}

[[noreturn]] void fire(const std::string& reason) {
  State& S = st();
  std::string line, path;
  bool to_stdout;
  int code, tail_bytes;
  {
    std::lock_guard<std::mutex> lk(S.mu);
    line = S.line;
    path = S.debug_path;
    to_stdout = S.to_stdout;
    code = S.exit_code;
    tail_bytes = S.tail_bytes;
  }
  const std::string tail = read_tail(path, tail_bytes);
  replace_token(line, "\"__AKKA_REASON__\"", "\"" + json_escape(reason) + "\"");
  replace_token(line, "\"__AKKA_TAIL__\"", "\"" + json_escape(tail) + "\"");
  if (!line.empty() && line.back() != '\n') line.push_back('\n');
  write_all(to_stdout ? st().out_fd.load() : 2, line);
  write_all(2, "akka watchdog: " + reason + "; exiting " + std::to_string(code) + "\n");
  if (!tail.empty()) write_all(2, "---- tail of " + path + " ----\n" + tail + "\n");
  ::fsync(1);
  kill_children();
  ::_exit(code);
}

void on_sigterm(int) {
  const int fd = st().pipe_w;
  if (fd >= 0) {
    char c = 'T';
    ssize_t r = ::write(fd, &c, 1);  // async-signal-safe; the thread does the rest
    (void)r;
  } else {
    ::_exit(128 + SIGTERM);
  }
}

void loop() {
  State& S = st();
  for (;;) {
    int timeout_ms = -1;
    bool armed;
    std::chrono::steady_clock::time_point dl;
    double secs;
    std::string beacon;
    {
      std::lock_guard<std::mutex> lk(S.mu);
      armed = S.armed;
      dl = S.deadline;
      secs = S.seconds;
      beacon = S.beacon_path;
    }
    if (armed && !beacon.empty() && ::access(beacon.c_str(), F_OK) == 0) {
      // another rank failed and said so: leave now instead of at the deadline
      std::string what = read_tail(beacon, 2048);
      while (!what.empty() && (what.back() == '\n' || what.back() == '\r')) what.pop_back();
      fire("failure reported by a rank: " + what);
    }
    if (armed) {
      auto left = std::chrono::duration_cast<std::chrono::milliseconds>(dl - std::chrono::steady_clock::now()).count();
      if (left <= 0) {
        char buf[64];
        std::snprintf(buf, sizeof(buf), "deadline of %.0f s exceeded", secs);
        fire(buf);
      }
      timeout_ms = int(std::min<long long>(left, 1 << 30));
      if (!beacon.empty()) timeout_ms = std::min(timeout_ms, 200);
    }
    pollfd p{S.pipe_r, POLLIN, 0};
    int n = ::poll(&p, 1, timeout_ms);
    if (n > 0 && (p.revents & POLLIN)) {
      char c = 0;
      if (::read(S.pipe_r, &c, 1) == 1 && c == 'T') {
        bool was_armed;
        std::string b;
        {
          std::lock_guard<std::mutex> lk(S.mu);
          was_armed = S.armed;
          b = S.beacon_path;
        }
        // the launcher usually sends SIGTERM because some rank already failed:
        // if that rank left word, report it rather than the signal
        if (was_armed && !b.empty() && ::access(b.c_str(), F_OK) == 0) {
          std::string what = read_tail(b, 2048);
          while (!what.empty() && (what.back() == '\n' || what.back() == '\r')) what.pop_back();
          fire("SIGTERM after a failure reported by a rank: " + what);
        }
        if (was_armed) fire("SIGTERM");
        kill_children();
        ::_exit(128 + SIGTERM);
      }
    }
  }
}

void ensure_thread() {
  State& S = st();
  if (S.started) return;
  int fds[2];
  if (::pipe(fds) != 0) return;
  ::fcntl(fds[0], F_SETFD, FD_CLOEXEC);
  ::fcntl(fds[1], F_SETFD, FD_CLOEXEC);
  S.pipe_r = fds[0];
  S.pipe_w = fds[1];
  std::thread(loop).detach();
  S.started = true;
}

void wake() {
  char c = 'A';
  ssize_t r = ::write(st().pipe_w, &c, 1);
  (void)r;
}

}  // namespace

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 16);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20 || c >= 0x7f) {  // keep the line plain ASCII whatever the log holds
          char buf[8];
          std::snprintf(buf, sizeof(buf), "\\u%04x", c);
          o += buf;
        } else {
          o.push_back(char(c));
        }
    }
  }
  return o;
}

void watchdog_set_out_fd(int fd) { st().out_fd.store(fd < 0 ? 1 : fd); }

void watchdog_arm(double seconds, const std::string& line, bool to_stdout, const std::string& debug_path,
                  int exit_code, int tail_bytes, const std::string& beacon_path) {
  State& S = st();
  {
    std::lock_guard<std::mutex> lk(S.mu);
    ensure_thread();
    S.armed = true;
    S.seconds = seconds;
    S.deadline = std::chrono::steady_clock::now() +
                 std::chrono::milliseconds(static_cast<long long>(seconds * 1000.0));
    S.line = line;
    S.to_stdout = to_stdout;
    S.debug_path = debug_path;
    S.exit_code = exit_code;
    S.tail_bytes = tail_bytes;
    S.beacon_path = beacon_path;
  }
  wake();
}

void watchdog_disarm() {
  State& S = st();
  {
    std::lock_guard<std::mutex> lk(S.mu);
    if (!S.started) return;
    S.armed = false;
  }
  wake();
}

bool watchdog_track_child(int pid) {
  for (auto& c : st().children) {
    int z = 0;
    if (c.compare_exchange_strong(z, pid)) return true;
  }
  return false;
}

void watchdog_untrack_child(int pid) {
  for (auto& c : st().children) {
    int v = pid;
    c.compare_exchange_strong(v, 0);
  }
}

void watchdog_install_sigterm() {
  {
    std::lock_guard<std::mutex> lk(st().mu);
    ensure_thread();
  }
  struct sigaction sa {};
  sa.sa_handler = on_sigterm;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART;
  ::sigaction(SIGTERM, &sa, nullptr);
}

}  // namespace akka
