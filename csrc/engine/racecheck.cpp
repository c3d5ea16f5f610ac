// Stream race checker (racecheck.h): vector clocks + a shadow interval map.
#include "racecheck.h"

#include <algorithm>
#include <sstream>

namespace akka {

int32_t RaceChecker::index(StreamH s) {
  auto it = ids_.find(s);
  if (it != ids_.end()) return it->second;
  const int32_t id = int32_t(clocks_.size());
  ids_[s] = id;
  clocks_.emplace_back();
  return id;
}

void RaceChecker::join(VC& a, const VC& b) {
  if (a.size() < b.size()) a.resize(b.size(), 0);
  for (size_t i = 0; i < b.size(); ++i) a[i] = std::max(a[i], b[i]);
}

const RaceChecker::VC& RaceChecker::tick(StreamH s) {
  const int32_t id = index(s);
  VC& c = clocks_[size_t(id)];
  join(c, host_);
  if (c.size() <= size_t(id)) c.resize(size_t(id) + 1, 0);
  ++c[size_t(id)];
  return c;
}

void RaceChecker::record(void* event, StreamH s) { events_[event] = clocks_[size_t(index(s))]; }

void RaceChecker::wait(StreamH s, void* event) {
  auto it = events_.find(event);
  if (it == events_.end()) return;  // never recorded: HIP treats the wait as satisfied
  join(clocks_[size_t(index(s))], it->second);
}

void RaceChecker::host_join_stream(StreamH s) { join(host_, clocks_[size_t(index(s))]); }

void RaceChecker::host_join_event(void* event) {
  auto it = events_.find(event);
  if (it != events_.end()) join(host_, it->second);
}

void RaceChecker::split(uintptr_t at) {
  auto it = shadow_.upper_bound(at);
  if (it == shadow_.begin()) return;
  --it;
  if (it->first == at || it->second.end <= at) return;
  Cell right = it->second;
  it->second.end = at;
  shadow_.emplace(at, std::move(right));
}

void RaceChecker::report(const Stamp& prev, bool prev_write, int32_t cur_stream, const Access& a, uintptr_t lo,
                         uintptr_t hi) {
  ++races_;
  if (reports_.size() >= 64) return;
  std::ostringstream os;
  os << (a.write ? "write" : "read") << " '" << a.tag << "' on stream " << cur_stream << " races with earlier "
     << (prev_write ? "write" : "read") << " '" << prev.tag << "' on stream " << prev.stream << " (tick " << prev.clock
     << "), bytes [0x" << std::hex << lo << ", 0x" << hi << std::dec << ")";
  reports_.push_back(os.str());
}

void RaceChecker::access(StreamH s, const std::vector<Access>& acc) {
  const int32_t sid = index(s);
  const VC now = clocks_[size_t(sid)];
  const Stamp me{sid, now.size() > size_t(sid) ? now[size_t(sid)] : 0, ""};
  for (const Access& a : acc) {
    if (!a.ptr || a.bytes == 0) continue;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(a.ptr), hi = lo + a.bytes;
    split(lo);
    split(hi);
    // fill the gaps of [lo, hi) with empty cells so every byte has one
    uintptr_t cur = lo;
    auto it = shadow_.lower_bound(lo);
    while (cur < hi) {
      if (it == shadow_.end() || it->first > cur) {
        const uintptr_t gap_end = (it == shadow_.end()) ? hi : std::min(hi, it->first);
        Cell c;
        c.end = gap_end;
        it = shadow_.emplace_hint(it, cur, std::move(c));
      }
      const uintptr_t cell_lo = it->first, cell_hi = it->second.end;
      Cell& c = it->second;
      bool reported = false;
      if (c.write.stream >= 0 && c.write.stream != sid && !before(c.write, now)) {
        report(c.write, true, sid, a, cell_lo, cell_hi);
        reported = true;
      }
      if (a.write && !reported)
        for (const Stamp& r : c.reads)
          if (r.stream != sid && !before(r, now)) {
            report(r, false, sid, a, cell_lo, cell_hi);
            break;
          }
      Stamp st = me;
      st.tag = a.tag;
      if (a.write) {
        c.write = st;
        c.reads.clear();
      } else {
        bool found = false;
        for (Stamp& r : c.reads)
          if (r.stream == sid) {
            r = st;
            found = true;
          }
        if (!found) c.reads.push_back(st);
      }
      cur = cell_hi;
      ++it;
    }
  }
}

}  // namespace akka
