// Wire frames of the CPU data plane, natively (akka_allreduce_amd/parallel/wire.py
// is the definition: [u32 big-endian length][msgpack map]).
//
// The reference's deployment is a CPU cluster exchanging tiny ScatterBlock /
// ReduceBlock messages (README demo: 2-float chunks; script config: 3-float
// chunks, 65 chunks per block, ~400 messages per worker per round), so the
// per-message cost IS the round time.  Building a Python message object, a
// torch tensor and a msgpack dict per chunk cost ~15 µs each way; here the
// engine's outbox is framed straight from the payload bytes, and an arriving
// data frame is parsed in place and handed to the engine with a pointer into
// the frame (no copy of the value).  Only the two data messages are handled;
// every other frame (and any layout this reader does not know) goes to the
// Python codec, which stays the single definition of the format.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

namespace akka {
namespace frames {

// ---- msgpack subset writer ---------------------------------------------------------
inline void put_be(std::string& s, uint64_t v, int bytes) {
  for (int i = bytes - 1; i >= 0; --i) s.push_back(char((v >> (8 * i)) & 0xff));
}
inline void put_str(std::string& s, const char* p, size_t n) {
  if (n < 32) {
    s.push_back(char(0xa0 | n));
  } else {
    s.push_back(char(0xd9));
    s.push_back(char(n));
  }
  s.append(p, n);
}
inline void put_str(std::string& s, const char* p) { put_str(s, p, std::strlen(p)); }
inline void put_bin(std::string& s, const char* p, size_t n) {
  if (n < 256) {
    s.push_back(char(0xc4));
    s.push_back(char(n));
  } else if (n < 65536) {
    s.push_back(char(0xc5));
    put_be(s, n, 2);
  } else {
    s.push_back(char(0xc6));
    put_be(s, n, 4);
  }
  s.append(p, n);
}
inline void put_int(std::string& s, int64_t v) {
  if (v >= 0 && v < 128) {
    s.push_back(char(v));
  } else if (v < 0 && v >= -32) {
    s.push_back(char(0xe0 | (v + 32)));
  } else if (v >= 0 && v < 256) {
    s.push_back(char(0xcc));
    s.push_back(char(v));
  } else if (v >= 0 && v < 65536) {
    s.push_back(char(0xcd));
    put_be(s, uint64_t(v), 2);
  } else if (v >= 0 && v <= 0xffffffffLL) {
    s.push_back(char(0xce));
    put_be(s, uint64_t(v), 4);
  } else {
    s.push_back(char(0xd3));
    put_be(s, uint64_t(v), 8);
  }
}

// One ScatterBlock (kind 1) or ReduceBlock (kind 2) frame, appended to `out`;
// the key order of wire.encode.
inline void append_data_frame(std::string& out, int32_t kind, const char* value, size_t nbytes, const char* dtype,
                              int32_t src, int32_t dest, int32_t chunk, int32_t round, int32_t count) {
  const size_t at = out.size();
  out.append(4, '\0');  // length, patched below
  out.push_back(char(0x80 | (kind == 1 ? 7 : 8)));
  put_str(out, "t");
  put_str(out, kind == 1 ? "ScatterBlock" : "ReduceBlock");
  put_str(out, "value");
  put_bin(out, value, nbytes);
  put_str(out, "dtype");
  put_str(out, dtype);
  put_str(out, "srcId");
  put_int(out, src);
  put_str(out, "destId");
  put_int(out, dest);
  put_str(out, "chunkId");
  put_int(out, chunk);
  put_str(out, "round");
  put_int(out, round);
  if (kind == 2) {
    put_str(out, "count");
    put_int(out, count);
  }
  const uint64_t n = out.size() - at - 4;
  for (int i = 0; i < 4; ++i) out[at + i] = char((n >> (8 * (3 - i))) & 0xff);
}

// ---- reader (the same subset; anything else -> not a data frame) ----------------------
struct Reader {
  const unsigned char* p;
  const unsigned char* end;
  bool ok = true;

  bool need(size_t n) {
    if (size_t(end - p) < n) ok = false;
    return ok;
  }
  uint64_t be(int bytes) {
    uint64_t v = 0;
    if (!need(size_t(bytes))) return 0;
    for (int i = 0; i < bytes; ++i) v = (v << 8) | p[i];
    p += bytes;
    return v;
  }
  // a string -> (ptr, len); false if the next value is not a string
  bool str(const char*& s, size_t& n) {
    if (!need(1)) return false;
    const unsigned char c = *p++;
    if ((c & 0xe0) == 0xa0) n = c & 0x1f;
    else if (c == 0xd9) n = size_t(be(1));
    else if (c == 0xda) n = size_t(be(2));
    else return ok = false;
    if (!need(n)) return false;
    s = reinterpret_cast<const char*>(p);
    p += n;
    return true;
  }
  bool bin(const char*& s, size_t& n) {
    if (!need(1)) return false;
    const unsigned char c = *p++;
    if (c == 0xc4) n = size_t(be(1));
    else if (c == 0xc5) n = size_t(be(2));
    else if (c == 0xc6) n = size_t(be(4));
    else return ok = false;
    if (!need(n)) return false;
    s = reinterpret_cast<const char*>(p);
    p += n;
    return true;
  }
  bool integer(int64_t& v) {
    if (!need(1)) return false;
    const unsigned char c = *p++;
    if (c < 0x80) v = c;
    else if (c >= 0xe0) v = int64_t(int8_t(c));
    else if (c == 0xcc) v = int64_t(be(1));
    else if (c == 0xcd) v = int64_t(be(2));
    else if (c == 0xce) v = int64_t(be(4));
    else if (c == 0xcf) v = int64_t(be(8));
    else if (c == 0xd0) v = int64_t(int8_t(be(1)));
    else if (c == 0xd1) v = int64_t(int16_t(be(2)));
    else if (c == 0xd2) v = int64_t(int32_t(be(4)));
    else if (c == 0xd3) v = int64_t(be(8));
    else return ok = false;
    return ok;
  }
};

struct DataFrame {
  int32_t kind = 0;  // 1 ScatterBlock, 2 ReduceBlock
  const char* value = nullptr;
  size_t nbytes = 0;
  std::string dtype;
  int64_t src = -1, dest = -1, chunk = -1, round = -1, count = 0;
};

inline bool key_is(const char* s, size_t n, const char* k) { return std::strlen(k) == n && std::memcmp(s, k, n) == 0; }

// Parse a frame BODY (no length prefix).  False: not a data frame, or a
// layout this reader does not handle -- the caller decodes it in Python.
inline bool parse_data_frame(const char* body, size_t n, DataFrame& f) {
  Reader r{reinterpret_cast<const unsigned char*>(body), reinterpret_cast<const unsigned char*>(body) + n};
  if (!r.need(1)) return false;
  const unsigned char m = *r.p++;
  if ((m & 0xf0) != 0x80) return false;  // fixmap only
  const int entries = m & 0x0f;
  bool have_value = false, have_dtype = false;
  for (int i = 0; i < entries; ++i) {
    const char* k = nullptr;
    size_t kn = 0;
    if (!r.str(k, kn)) return false;
    if (key_is(k, kn, "t")) {
      const char* t = nullptr;
      size_t tn = 0;
      if (!r.str(t, tn)) return false;
      if (key_is(t, tn, "ScatterBlock")) f.kind = 1;
      else if (key_is(t, tn, "ReduceBlock")) f.kind = 2;
      else return false;
    } else if (key_is(k, kn, "value")) {
      if (!r.bin(f.value, f.nbytes)) return false;
      have_value = true;
    } else if (key_is(k, kn, "dtype")) {
      const char* d = nullptr;
      size_t dn = 0;
      if (!r.str(d, dn)) return false;
      f.dtype.assign(d, dn);
      have_dtype = true;
    } else {
      int64_t v = 0;
      if (!r.integer(v)) return false;
      if (key_is(k, kn, "srcId")) f.src = v;
      else if (key_is(k, kn, "destId")) f.dest = v;
      else if (key_is(k, kn, "chunkId")) f.chunk = v;
      else if (key_is(k, kn, "round")) f.round = v;
      else if (key_is(k, kn, "count")) f.count = v;
      else return false;
    }
  }
  return r.ok && r.p == r.end && f.kind != 0 && have_value && have_dtype && f.src >= 0 && f.dest >= 0 &&
         f.chunk >= 0 && f.round >= 0;
}

}  // namespace frames
}  // namespace akka
