// Minimal protobuf wire-format codec (proto3: varint, length-delimited, fixed32/64 skipping)
// for the handful of ``dapr.proto.runtime.v1`` messages the native gRPC API decodes and
// encodes (field numbers: sdk/proto.py, which mirrors the public Dapr 1.14 protos).
//
// Readers never allocate: strings and sub-messages are views into the request buffer.
// Unknown fields are skipped (forward compatibility, as protobuf requires); a truncated or
// malformed buffer sets `ok = false`.
#pragma once

#include <cstdint>
#include <string>
#include <string_view>

namespace tt::pb {

enum WireType : uint32_t { VARINT = 0, I64 = 1, LEN = 2, I32 = 5 };

struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  explicit Reader(std::string_view s) : p((const uint8_t*)s.data()), e((const uint8_t*)s.data() + s.size()) {}

  bool varint(uint64_t& v) {
    v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= e) return ok = false;
      uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return true;
    }
    return ok = false;
  }
  // Next field tag; false at the end of the buffer or on a malformed tag.
  bool next(uint32_t& field, uint32_t& wt) {
    if (!ok || p >= e) return false;
    uint64_t t;
    if (!varint(t)) return false;
    field = (uint32_t)(t >> 3);
    wt = (uint32_t)(t & 7);
    if (field == 0) return ok = false;
    return true;
  }
  bool bytes(std::string_view& out) {
    uint64_t n;
    if (!varint(n)) return false;
    if (n > (uint64_t)(e - p)) return ok = false;
    out = std::string_view((const char*)p, (size_t)n);
    p += n;
    return true;
  }
  bool skip(uint32_t wt) {
    uint64_t v;
    std::string_view s;
    switch (wt) {
      case VARINT: return varint(v);
      case I64:
        if (e - p < 8) return ok = false;
        p += 8;
        return true;
      case LEN: return bytes(s);
      case I32:
        if (e - p < 4) return ok = false;
        p += 4;
        return true;
      default: return ok = false;  // groups are not used by proto3
    }
  }
};

// map<string,string> entry {key = 1, value = 2}
inline bool map_entry(std::string_view entry, std::string& k, std::string& v) {
  Reader r(entry);
  uint32_t f, wt;
  k.clear();
  v.clear();
  while (r.next(f, wt)) {
    std::string_view s;
    if ((f == 1 || f == 2) && wt == LEN) {
      if (!r.bytes(s)) break;
      (f == 1 ? k : v).assign(s);
    } else if (!r.skip(wt)) {
      break;
    }
  }
  return r.ok;
}

// Encoded sizes, for writing a sub-message's length before its fields (no temporary message).
inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) v >>= 7, ++n;
  return n;
}
// a length-delimited field of `n` bytes (written always: repeated element / sub-message)
inline size_t len_field_size(uint32_t field, size_t n) { return varint_size((uint64_t)field << 3) + varint_size(n) + n; }
// a proto3 singular string / bytes field (not written when empty)
inline size_t str_size(uint32_t field, size_t n) { return n ? len_field_size(field, n) : 0; }

struct Writer {
  std::string s;
  // the header of a length-delimited field whose `n` bytes the caller appends next
  void len_header(uint32_t field, size_t n) {
    key(field, 2);
    varint(n);
  }
  void varint(uint64_t v) {
    while (v >= 0x80) {
      s.push_back((char)(0x80 | (v & 0x7f)));
      v >>= 7;
    }
    s.push_back((char)v);
  }
  void key(uint32_t field, uint32_t wt) { varint((uint64_t)field << 3 | wt); }
  // proto3 singular string / bytes: the default (empty) is not written
  void str(uint32_t field, std::string_view v) {
    if (v.empty()) return;
    len_field(field, v);
  }
  // repeated element / sub-message: always written
  void len_field(uint32_t field, std::string_view v) {
    key(field, LEN);
    varint(v.size());
    s.append(v);
  }
  void u64(uint32_t field, uint64_t v) {
    if (!v) return;
    key(field, VARINT);
    varint(v);
  }
  void map_entry(uint32_t field, std::string_view k, std::string_view v) {
    Writer e;
    e.str(1, k);
    e.str(2, v);
    len_field(field, e.s);
  }
};

}  // namespace tt::pb
