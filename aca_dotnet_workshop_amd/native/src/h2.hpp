// HTTP/2 server connections (RFC 9113, cleartext "prior knowledge") with an HPACK codec
// (RFC 7541), carrying unary gRPC calls -- the transport of the sidecar's gRPC API
// (``dapr.proto.runtime.v1.Dapr``) in the native data plane.
//
// The reference's services reach daprd through ``Dapr.Client.DaprClient``, whose state,
// pub/sub and binding calls are gRPC (Backend.Api Services/TasksStoreManager.cs:35,50,155;
// Processor ExternalTasksProcessorController.cs:43).  No HTTP/2 or gRPC library is available to
// the native build, so this header implements the parts a unary gRPC server needs on the
// single-threaded epoll loop of evhttp.hpp:
//
// * framing     -- connection preface, SETTINGS (+ACK), HEADERS/CONTINUATION, DATA, PING,
//                  WINDOW_UPDATE, RST_STREAM, GOAWAY, PRIORITY; padding; frame-size limits.
// * HPACK       -- decoder with the static table, a bounded dynamic table, size updates,
//                  prefix integers and Huffman strings (canonical code rebuilt from the RFC's
//                  per-symbol code lengths); the encoder emits literals without indexing (no
//                  dynamic-table state on our side, always valid).
// * flow control-- both directions: our receive windows are replenished as DATA is consumed
//                  (and violations are connection errors); responses are split into frames of
//                  the peer's SETTINGS_MAX_FRAME_SIZE and queued while a stream or the
//                  connection has no send window.
// * gRPC        -- length-prefixed messages (uncompressed), ``grpc-status`` / ``grpc-message``
//                  trailers, trailers-only error responses, percent-encoded messages.
//
// A handler receives one GrpcCall per stream (``:path``, metadata, the request message) and
// completes it asynchronously through a GrpcReply holding a weak reference to the connection,
// exactly like ev::Reply for HTTP/1.1.
#pragma once

#include <array>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "evhttp.hpp"

namespace tt::h2 {

using ev::HeaderList;

// ------------------------------------------------------------------------------ HPACK Huffman
// Code length in bits of each symbol 0..256 (256 = EOS), RFC 7541 Appendix B.  The code is
// canonical (codes of equal length are consecutive in symbol order, shorter codes first), so
// the lengths alone define it.
inline constexpr uint8_t kHuffLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 30, 28, 28, 28,
    28, 28, 28, 28, 28, 28,  6, 10, 10, 12, 13,  6,  8, 11, 10, 10,  8, 11,  8,  6,  6,  6,  5,  5,  5,  6,
     6,  6,  6,  6,  6,  6,  7,  8, 15,  6, 12, 10, 13,  6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,
     7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8, 13, 19, 13, 14,  6, 15,  5,  6,  5,  6,  5,  6,  6,
     6,  5,  7,  7,  6,  6,  6,  5,  6,  7,  6,  5,  5,  6,  7,  7,  7,  7,  7, 15, 11, 14, 13, 28, 20, 22,
    20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23,
    22, 23, 23, 24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22,
    23, 23, 20, 22, 22, 22, 23, 22, 22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21, 22, 21, 21, 23, 22, 22,
    25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26, 30};

class Huffman {
 public:
  static const Huffman& get() {
    static const Huffman h;
    return h;
  }
  // Appends the decoded bytes of `in` to `out`; false on an invalid string (EOS symbol,
  // padding longer than 7 bits or not all ones).
  bool decode(std::string_view in, std::string& out) const {
    uint32_t code = 0;
    int len = 0;
    bool ones = true;  // the bits of the unfinished code so far are all 1
    for (unsigned char byte : in) {
      for (int b = 7; b >= 0; --b) {
        uint32_t bit = (byte >> b) & 1u;
        code = (code << 1) | bit;
        ones = ones && bit;
        ++len;
        if (len > 30) return false;
        if (count_[len] && code >= first_[len] && code - first_[len] < count_[len]) {
          int sym = sorted_[offset_[len] + (code - first_[len])];
          if (sym == 256) return false;  // EOS inside a string is an error (RFC 7541 5.2)
          out.push_back((char)sym);
          code = 0;
          len = 0;
          ones = true;
        }
      }
    }
    return len < 8 && ones;
  }
  // Exposed for tests: the canonical code of a symbol.
  uint32_t code_of(int sym) const { return codes_[sym]; }

 private:
  std::array<uint32_t, 32> first_{}, count_{}, offset_{};
  std::array<int, 257> sorted_{};
  std::array<uint32_t, 257> codes_{};
  Huffman() {
    for (int s = 0; s < 257; ++s) count_[kHuffLen[s]]++;
    uint32_t code = 0, off = 0;
    for (int l = 1; l < 32; ++l) {
      first_[l] = code;
      offset_[l] = off;
      code = (code + count_[l]) << 1;
      off += count_[l];
    }
    std::array<uint32_t, 32> next = first_;
    std::array<uint32_t, 32> fill = offset_;
    for (int s = 0; s < 257; ++s) {  // symbol order within a length = canonical order
      int l = kHuffLen[s];
      codes_[s] = next[l]++;
      sorted_[fill[l]++] = s;
    }
  }
};

// ------------------------------------------------------------------------------ HPACK tables
struct StaticEntry {
  const char* name;
  const char* value;
};
inline constexpr StaticEntry kStatic[62] = {
    {"", ""},  // index 0 is not used
    {":authority", ""}, {":method", "GET"}, {":method", "POST"}, {":path", "/"}, {":path", "/index.html"},
    {":scheme", "http"}, {":scheme", "https"}, {":status", "200"}, {":status", "204"}, {":status", "206"},
    {":status", "304"}, {":status", "400"}, {":status", "404"}, {":status", "500"}, {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"}, {"accept-language", ""}, {"accept-ranges", ""}, {"accept", ""},
    {"access-control-allow-origin", ""}, {"age", ""}, {"allow", ""}, {"authorization", ""},
    {"cache-control", ""}, {"content-disposition", ""}, {"content-encoding", ""}, {"content-language", ""},
    {"content-length", ""}, {"content-location", ""}, {"content-range", ""}, {"content-type", ""},
    {"cookie", ""}, {"date", ""}, {"etag", ""}, {"expect", ""}, {"expires", ""}, {"from", ""}, {"host", ""},
    {"if-match", ""}, {"if-modified-since", ""}, {"if-none-match", ""}, {"if-range", ""},
    {"if-unmodified-since", ""}, {"last-modified", ""}, {"link", ""}, {"location", ""}, {"max-forwards", ""},
    {"proxy-authenticate", ""}, {"proxy-authorization", ""}, {"range", ""}, {"referer", ""}, {"refresh", ""},
    {"retry-after", ""}, {"server", ""}, {"set-cookie", ""}, {"strict-transport-security", ""},
    {"transfer-encoding", ""}, {"user-agent", ""}, {"vary", ""}, {"via", ""}, {"www-authenticate", ""}};

// Prefix-coded integer (RFC 7541 5.1); false on truncation or overflow.
inline bool hpack_int(const uint8_t*& p, const uint8_t* e, int prefix_bits, uint64_t& out) {
  if (p >= e) return false;
  uint64_t mask = (1u << prefix_bits) - 1;
  out = *p++ & mask;
  if (out < mask) return true;
  int shift = 0;
  while (true) {
    if (p >= e || shift > 28) return false;
    uint8_t b = *p++;
    out += (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) return true;
  }
}

inline void hpack_put_int(std::string& out, uint8_t first, int prefix_bits, uint64_t v) {
  uint64_t mask = (1u << prefix_bits) - 1;
  if (v < mask) {
    out.push_back((char)(first | v));
    return;
  }
  out.push_back((char)(first | mask));
  v -= mask;
  while (v >= 128) {
    out.push_back((char)(0x80 | (v & 0x7f)));
    v >>= 7;
  }
  out.push_back((char)v);
}

class HpackDecoder {
 public:
  explicit HpackDecoder(size_t max_table = 4096) : limit_(max_table), max_(max_table) {}
  size_t table_size() const { return size_; }
  size_t table_entries() const { return dyn_.size(); }

  // Decodes one complete header block; false + `err` on a compression error (a connection
  // error: the dynamic table can no longer be trusted).  `max_list`: cap on the decoded size.
  bool decode(std::string_view block, HeaderList& out, std::string& err, size_t max_list = 65536) {
    const uint8_t* p = (const uint8_t*)block.data();
    const uint8_t* e = p + block.size();
    size_t list = 0;
    bool fields_seen = false;
    while (p < e) {
      uint8_t b = *p;
      std::string name, value;
      if (b & 0x80) {  // indexed header field
        uint64_t idx;
        if (!hpack_int(p, e, 7, idx) || !lookup(idx, name, value, err)) return fail(err, "bad indexed field");
      } else if ((b & 0xe0) == 0x20) {  // dynamic table size update: only before the first field
        uint64_t sz;
        if (!hpack_int(p, e, 5, sz)) return fail(err, "bad table size update");
        if (fields_seen) return fail(err, "table size update after a header field");
        if (sz > limit_) return fail(err, "table size update above SETTINGS_HEADER_TABLE_SIZE");
        max_ = (size_t)sz;
        evict(0);
        continue;
      } else {
        bool incremental = (b & 0xc0) == 0x40;
        int prefix = incremental ? 6 : 4;  // 0000xxxx without indexing, 0001xxxx never indexed
        uint64_t idx;
        if (!hpack_int(p, e, prefix, idx)) return fail(err, "bad literal field");
        if (idx) {
          std::string ignored;
          if (!lookup(idx, name, ignored, err)) return fail(err, "bad literal name index");
        } else if (!string(p, e, name)) {
          return fail(err, "bad literal name");
        }
        if (!string(p, e, value)) return fail(err, "bad literal value");
        if (incremental) insert(name, value);
      }
      fields_seen = true;
      list += name.size() + value.size() + 32;
      if (list > max_list) return fail(err, "header list too large");
      out.emplace_back(std::move(name), std::move(value));
    }
    return true;
  }

 private:
  std::deque<std::pair<std::string, std::string>> dyn_;  // front = most recent (index 62)
  size_t size_ = 0, limit_, max_;

  static bool fail(std::string& err, const char* what) {
    if (err.empty()) err = what;
    return false;
  }
  bool lookup(uint64_t idx, std::string& name, std::string& value, std::string& err) const {
    if (idx == 0) return fail(err, "index 0");
    if (idx < 62) {
      name = kStatic[idx].name;
      value = kStatic[idx].value;
      return true;
    }
    size_t d = (size_t)(idx - 62);
    if (d >= dyn_.size()) return fail(err, "index beyond the dynamic table");
    name = dyn_[d].first;
    value = dyn_[d].second;
    return true;
  }
  static bool string(const uint8_t*& p, const uint8_t* e, std::string& out) {
    if (p >= e) return false;
    bool huff = *p & 0x80;
    uint64_t n;
    if (!hpack_int(p, e, 7, n) || n > (uint64_t)(e - p)) return false;
    std::string_view raw((const char*)p, (size_t)n);
    p += n;
    if (!huff) {
      out.assign(raw);
      return true;
    }
    out.reserve(raw.size() * 8 / 5);
    return Huffman::get().decode(raw, out);
  }
  void evict(size_t incoming) {
    while (!dyn_.empty() && size_ + incoming > max_) {
      size_ -= dyn_.back().first.size() + dyn_.back().second.size() + 32;
      dyn_.pop_back();
    }
  }
  void insert(const std::string& n, const std::string& v) {
    size_t sz = n.size() + v.size() + 32;
    evict(sz);
    if (sz > max_) return;  // larger than the table: the table is just emptied (RFC 7541 4.4)
    dyn_.emplace_front(n, v);
    size_ += sz;
  }
};

// Literal header field without indexing (new name or static name index); never Huffman.
inline void hpack_literal(std::string& out, std::string_view name, std::string_view value) {
  int idx = 0;
  for (int i = 1; i < 62; ++i)
    if (name == kStatic[i].name) {
      idx = i;
      break;
    }
  if (idx) {
    hpack_put_int(out, 0x00, 4, (uint64_t)idx);
  } else {
    out.push_back(0x00);
    hpack_put_int(out, 0x00, 7, name.size());
    out.append(name);
  }
  hpack_put_int(out, 0x00, 7, value.size());
  out.append(value);
}

// grpc-message: percent-encode bytes outside printable ASCII and '%' (gRPC HTTP/2 protocol spec).
inline std::string grpc_percent_encode(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  o.reserve(s.size());
  for (unsigned char c : s) {
    if (c < 0x20 || c > 0x7e || c == '%') {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    } else {
      o.push_back((char)c);
    }
  }
  return o;
}

// ------------------------------------------------------------------------------ frames
enum FrameType : uint8_t {
  DATA = 0, HEADERS = 1, PRIORITY = 2, RST_STREAM = 3, SETTINGS = 4, PUSH_PROMISE = 5, PING = 6,
  GOAWAY = 7, WINDOW_UPDATE = 8, CONTINUATION = 9
};
enum Flags : uint8_t { END_STREAM = 0x1, ACK = 0x1, END_HEADERS = 0x4, PADDED = 0x8, PRIORITY_FLAG = 0x20 };
enum ErrorCode : uint32_t {
  NO_ERROR = 0, PROTOCOL_ERROR = 1, INTERNAL_ERROR = 2, FLOW_CONTROL_ERROR = 3, SETTINGS_TIMEOUT = 4,
  STREAM_CLOSED = 5, FRAME_SIZE_ERROR = 6, REFUSED_STREAM = 7, CANCEL = 8, COMPRESSION_ERROR = 9
};

inline void put_frame_header(std::string& out, uint32_t len, uint8_t type, uint8_t flags, uint32_t stream) {
  char h[9] = {(char)(len >> 16), (char)(len >> 8), (char)len, (char)type, (char)flags,
               (char)((stream >> 24) & 0x7f), (char)(stream >> 16), (char)(stream >> 8), (char)stream};
  out.append(h, 9);
}
inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
inline void put_be32(std::string& out, uint32_t v) {
  char b[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
  out.append(b, 4);
}

inline constexpr std::string_view kPreface = "PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n";

// ------------------------------------------------------------------------------ gRPC server
struct GrpcCall {
  std::string path;      // "/package.Service/Method"
  HeaderList metadata;   // non-pseudo request headers (lower-case names)
  std::string message;   // the request message (gRPC length prefix removed)
  uint32_t stream = 0;
};

class H2Conn;

// Completes one call; safe to use after the connection or the stream went away.
class GrpcReply {
 public:
  GrpcReply() = default;
  GrpcReply(std::weak_ptr<H2Conn> c, uint32_t stream) : conn_(std::move(c)), stream_(stream) {}
  // status 0 (OK) sends `message` as the response; otherwise a trailers-only error response.
  void send(int status, std::string_view status_message, std::string_view message,
            const HeaderList& trailers = {}) const;
  void ok(std::string_view message) const { send(0, {}, message); }
  void error(int status, std::string_view msg, const HeaderList& trailers = {}) const { send(status, msg, {}, trailers); }

 private:
  std::weak_ptr<H2Conn> conn_;
  uint32_t stream_ = 0;
};

using GrpcHandler = std::function<void(GrpcCall&&, GrpcReply)>;

class H2Conn : public ev::IoObj {
 public:
  static constexpr uint32_t kMaxFrame = 16384;             // our SETTINGS_MAX_FRAME_SIZE (default)
  static constexpr uint32_t kStreamWindow = 4u << 20;      // our SETTINGS_INITIAL_WINDOW_SIZE
  static constexpr int64_t kConnWindow = 16 << 20;         // our connection receive window
  static constexpr uint32_t kMaxStreams = 1024;            // SETTINGS_MAX_CONCURRENT_STREAMS
  static constexpr size_t kMaxMessage = 64ull << 20;       // request message cap

  H2Conn(ev::Loop& loop, int fd, GrpcHandler& h) : loop_(loop), handler_(h) {
    this->fd = fd;
    // server preface: SETTINGS, then open the connection window beyond the initial 65535
    std::string s;
    put_frame_header(s, 18, SETTINGS, 0, 0);
    auto setting = [&](uint16_t id, uint32_t v) {
      s.push_back((char)(id >> 8));
      s.push_back((char)id);
      put_be32(s, v);
    };
    setting(0x3, kMaxStreams);
    setting(0x4, kStreamWindow);
    setting(0x6, 65536);  // SETTINGS_MAX_HEADER_LIST_SIZE
    put_frame_header(s, 4, WINDOW_UPDATE, 0, 0);
    put_be32(s, (uint32_t)(kConnWindow - 65535));
    out_ += s;
    recv_conn_window_ = kConnWindow;
  }

  void on_event(uint32_t ev) override {
    if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
      char buf[65536];
      while (true) {
        ssize_t n = ::recv(fd, buf, sizeof buf, 0);
        if (n > 0) {
          in_.append(buf, (size_t)n);
          if ((size_t)n < sizeof buf) break;
          continue;
        }
        if (n == 0) {
          peer_closed_ = true;
          break;
        }
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        if (errno == EINTR) continue;
        close_now();
        return;
      }
      process();
      if (dead) return;
      if (peer_closed_) {
        close_now();  // a half-closed HTTP/2 connection has no one to answer
        return;
      }
    }
    flush();
  }

  // Called through GrpcReply.
  void respond(uint32_t sid, int status, std::string_view status_msg, std::string_view message,
               const HeaderList& trailers) {
    if (dead) return;
    auto it = streams_.find(sid);
    if (it == streams_.end() || it->second.responded) return;
    Stream& st = it->second;
    st.responded = true;
    if (status == 0) {
      std::string hb;
      hb.push_back((char)0x88);  // :status 200 (static index 8)
      hpack_literal(hb, "content-type", "application/grpc");
      put_headers(sid, hb, false);
      st.pending.reserve(message.size() + 5);
      st.pending.push_back(0);  // uncompressed
      uint32_t n = (uint32_t)message.size();
      char len[4] = {(char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
      st.pending.append(len, 4);
      st.pending.append(message);
      st.trailers.clear();
      hpack_literal(st.trailers, "grpc-status", "0");
      for (auto& kv : trailers) hpack_literal(st.trailers, kv.first, kv.second);
      pump_stream(sid);
    } else {  // trailers-only response
      std::string hb;
      hb.push_back((char)0x88);
      hpack_literal(hb, "content-type", "application/grpc");
      hpack_literal(hb, "grpc-status", std::to_string(status));
      if (!status_msg.empty()) hpack_literal(hb, "grpc-message", grpc_percent_encode(status_msg.substr(0, 4096)));
      for (auto& kv : trailers) hpack_literal(hb, kv.first, kv.second);
      put_headers(sid, hb, true);
      streams_.erase(it);
    }
    flush();
  }

  size_t open_streams() const { return streams_.size(); }

 private:
  struct Stream {
    HeaderList headers;
    std::string body;
    int64_t send_window = 65535;
    int64_t recv_window = kStreamWindow;
    bool remote_closed = false, dispatched = false, responded = false;
    std::string pending;   // response DATA bytes not yet sent (flow control)
    std::string trailers;  // trailer header block, sent after `pending` drains
  };
  ev::Loop& loop_;
  GrpcHandler& handler_;
  HpackDecoder hpack_;
  std::string in_;
  size_t in_off_ = 0;
  std::string out_;
  size_t out_off_ = 0;
  bool preface_ok_ = false, peer_closed_ = false, goaway_sent_ = false, closing_ = false;
  uint32_t interest_ = EPOLLIN | EPOLLOUT;  // registered so by H2Listener: the preface is queued
  std::unordered_map<uint32_t, Stream> streams_;
  uint32_t last_stream_ = 0;
  // header block being assembled (HEADERS + CONTINUATION)
  uint32_t hb_stream_ = 0;
  bool hb_end_stream_ = false;
  std::string hb_;
  // flow control
  int64_t send_conn_window_ = 65535;
  int64_t peer_initial_window_ = 65535;
  uint32_t peer_max_frame_ = 16384;
  int64_t recv_conn_window_ = 65535;
  int64_t recv_conn_consumed_ = 0;

  void put_headers(uint32_t sid, const std::string& block, bool end_stream) {
    // one HEADERS frame, then CONTINUATION frames if the block exceeds the peer's frame size
    size_t off = 0;
    bool first = true;
    do {
      size_t n = std::min<size_t>(block.size() - off, peer_max_frame_);
      bool last = off + n == block.size();
      uint8_t flags = (last ? END_HEADERS : 0) | (first && end_stream ? END_STREAM : 0);
      put_frame_header(out_, (uint32_t)n, first ? HEADERS : CONTINUATION, flags, sid);
      out_.append(block, off, n);
      off += n;
      first = false;
    } while (off < block.size());
  }

  // Sends as much of a stream's pending DATA as the windows allow; trailers once drained.
  void pump_stream(uint32_t sid) {
    auto it = streams_.find(sid);
    if (it == streams_.end()) return;
    Stream& st = it->second;
    while (!st.pending.empty()) {
      int64_t room = std::min<int64_t>({send_conn_window_, st.send_window, (int64_t)peer_max_frame_});
      if (room <= 0) return;
      size_t n = std::min<size_t>(st.pending.size(), (size_t)room);
      put_frame_header(out_, (uint32_t)n, DATA, 0, sid);
      out_.append(st.pending, 0, n);
      st.pending.erase(0, n);
      send_conn_window_ -= (int64_t)n;
      st.send_window -= (int64_t)n;
    }
    if (st.responded && !st.trailers.empty()) {
      put_headers(sid, st.trailers, true);
      streams_.erase(it);
    }
  }
  void pump_all() {
    std::vector<uint32_t> ids;
    for (auto& kv : streams_)
      if (kv.second.responded && !kv.second.trailers.empty()) ids.push_back(kv.first);
    for (uint32_t id : ids) pump_stream(id);
  }

  void goaway(ErrorCode code, std::string_view debug) {
    if (goaway_sent_) return;
    goaway_sent_ = true;
    closing_ = true;
    put_frame_header(out_, 8 + (uint32_t)debug.size(), GOAWAY, 0, 0);
    put_be32(out_, last_stream_);
    put_be32(out_, code);
    out_.append(debug);
  }
  void rst(uint32_t sid, ErrorCode code) {
    put_frame_header(out_, 4, RST_STREAM, 0, sid);
    put_be32(out_, code);
    streams_.erase(sid);
  }

  void process() {
    if (!preface_ok_) {
      if (in_.size() < kPreface.size()) {
        if (kPreface.compare(0, in_.size(), in_) != 0) close_now();
        return;
      }
      if (std::string_view(in_).substr(0, kPreface.size()) != kPreface) {
        close_now();  // not an HTTP/2 prior-knowledge client
        return;
      }
      preface_ok_ = true;
      in_off_ = kPreface.size();
    }
    while (!dead && !closing_ && in_.size() - in_off_ >= 9) {
      const uint8_t* h = (const uint8_t*)in_.data() + in_off_;
      uint32_t len = (uint32_t)h[0] << 16 | (uint32_t)h[1] << 8 | h[2];
      uint8_t type = h[3], flags = h[4];
      uint32_t sid = be32(h + 5) & 0x7fffffffu;
      if (len > kMaxFrame) {
        goaway(FRAME_SIZE_ERROR, "frame larger than SETTINGS_MAX_FRAME_SIZE");
        break;
      }
      if (in_.size() - in_off_ < 9 + (size_t)len) break;
      std::string_view payload(in_.data() + in_off_ + 9, len);
      in_off_ += 9 + len;
      frame(type, flags, sid, payload);
    }
    if (in_off_ > 0 && (in_off_ == in_.size() || in_off_ > 65536)) {
      in_.erase(0, in_off_);
      in_off_ = 0;
    }
    if (recv_conn_consumed_ >= kConnWindow / 4 && !closing_) {  // replenish the connection window
      put_frame_header(out_, 4, WINDOW_UPDATE, 0, 0);
      put_be32(out_, (uint32_t)recv_conn_consumed_);
      recv_conn_window_ += recv_conn_consumed_;
      recv_conn_consumed_ = 0;
    }
  }

  static bool strip_padding(uint8_t flags, std::string_view& p) {
    if (!(flags & PADDED)) return true;
    if (p.empty()) return false;
    size_t pad = (uint8_t)p[0];
    if (pad >= p.size()) return false;
    p = p.substr(1, p.size() - 1 - pad);
    return true;
  }

  void frame(uint8_t type, uint8_t flags, uint32_t sid, std::string_view p) {
    if (hb_stream_ && type != CONTINUATION) {
      goaway(PROTOCOL_ERROR, "header block interrupted");
      return;
    }
    switch (type) {
      case SETTINGS: {
        if (sid) return goaway(PROTOCOL_ERROR, "SETTINGS on a stream");
        if (flags & ACK) return;
        if (p.size() % 6) return goaway(FRAME_SIZE_ERROR, "SETTINGS length");
        for (size_t i = 0; i < p.size(); i += 6) {
          uint16_t id = (uint16_t)((uint8_t)p[i] << 8 | (uint8_t)p[i + 1]);
          uint32_t v = be32((const uint8_t*)p.data() + i + 2);
          if (id == 0x4) {  // SETTINGS_INITIAL_WINDOW_SIZE: adjust every open stream (RFC 9113 6.9.2)
            if (v > 0x7fffffffu) return goaway(FLOW_CONTROL_ERROR, "initial window too large");
            int64_t delta = (int64_t)v - peer_initial_window_;
            peer_initial_window_ = v;
            for (auto& kv : streams_) kv.second.send_window += delta;
          } else if (id == 0x5) {
            if (v < 16384 || v > 16777215) return goaway(PROTOCOL_ERROR, "max frame size");
            peer_max_frame_ = v;
          } else if (id == 0x2 && v > 1) {
            return goaway(PROTOCOL_ERROR, "ENABLE_PUSH");
          }
        }
        put_frame_header(out_, 0, SETTINGS, ACK, 0);
        pump_all();
        return;
      }
      case PING:
        if (sid || p.size() != 8) return goaway(PROTOCOL_ERROR, "PING");
        if (!(flags & ACK)) {
          put_frame_header(out_, 8, PING, ACK, 0);
          out_.append(p);
        }
        return;
      case WINDOW_UPDATE: {
        if (p.size() != 4) return goaway(FRAME_SIZE_ERROR, "WINDOW_UPDATE length");
        uint32_t inc = be32((const uint8_t*)p.data()) & 0x7fffffffu;
        if (!sid) {
          if (!inc) return goaway(PROTOCOL_ERROR, "zero window increment");
          send_conn_window_ += inc;
          if (send_conn_window_ > 0x7fffffff) return goaway(FLOW_CONTROL_ERROR, "window overflow");
          pump_all();
        } else {
          auto it = streams_.find(sid);
          if (it == streams_.end()) return;
          if (!inc) return rst(sid, PROTOCOL_ERROR);
          it->second.send_window += inc;
          if (it->second.responded) pump_stream(sid);
        }
        return;
      }
      case GOAWAY:
        closing_ = streams_.empty();  // finish the calls in flight, then close
        peer_goaway_ = true;
        return;
      case RST_STREAM:
        if (!sid || p.size() != 4) return goaway(PROTOCOL_ERROR, "RST_STREAM");
        streams_.erase(sid);
        return;
      case PRIORITY:
        if (!sid || p.size() != 5) return goaway(PROTOCOL_ERROR, "PRIORITY");
        return;
      case PUSH_PROMISE:
        return goaway(PROTOCOL_ERROR, "PUSH_PROMISE from a client");
      case HEADERS: {
        if (!sid || !(sid & 1)) return goaway(PROTOCOL_ERROR, "HEADERS stream id");
        if (!strip_padding(flags, p)) return goaway(PROTOCOL_ERROR, "padding");
        if (flags & PRIORITY_FLAG) {
          if (p.size() < 5) return goaway(PROTOCOL_ERROR, "priority fields");
          p.remove_prefix(5);
        }
        auto it = streams_.find(sid);
        if (it == streams_.end() && sid <= last_stream_) return goaway(PROTOCOL_ERROR, "stream id reused");
        hb_.assign(p);
        hb_end_stream_ = flags & END_STREAM;
        if (flags & END_HEADERS) return header_block_done(sid);
        hb_stream_ = sid;
        return;
      }
      case CONTINUATION: {
        if (!hb_stream_ || sid != hb_stream_) return goaway(PROTOCOL_ERROR, "unexpected CONTINUATION");
        hb_.append(p);
        if (hb_.size() > 256 * 1024) return goaway(PROTOCOL_ERROR, "header block too large");
        if (flags & END_HEADERS) {
          hb_stream_ = 0;
          header_block_done(sid);
        }
        return;
      }
      case DATA: {
        if (!sid) return goaway(PROTOCOL_ERROR, "DATA on stream 0");
        int64_t flen = (int64_t)p.size();  // padding counts against flow control
        recv_conn_window_ -= flen;
        recv_conn_consumed_ += flen;
        if (recv_conn_window_ < 0) return goaway(FLOW_CONTROL_ERROR, "connection window exceeded");
        if (!strip_padding(flags, p)) return goaway(PROTOCOL_ERROR, "padding");
        auto it = streams_.find(sid);
        if (it == streams_.end()) {
          if (sid > last_stream_) return goaway(PROTOCOL_ERROR, "DATA on an idle stream");
          return;  // a stream we already answered or reset
        }
        Stream& st = it->second;
        if (st.remote_closed) return rst(sid, STREAM_CLOSED);
        st.recv_window -= flen;
        if (st.recv_window < 0) return rst(sid, FLOW_CONTROL_ERROR);
        if (st.body.size() + p.size() > kMaxMessage + 5) {
          GrpcReply(self(), sid).error(8, "request message larger than the server's limit");  // RESOURCE_EXHAUSTED
          return rst(sid, CANCEL);
        }
        st.body.append(p);
        if (flags & END_STREAM) {
          st.remote_closed = true;
          dispatch(sid);
        } else if (st.recv_window < (int64_t)kStreamWindow / 2) {
          int64_t inc = (int64_t)kStreamWindow - st.recv_window;
          put_frame_header(out_, 4, WINDOW_UPDATE, 0, sid);
          put_be32(out_, (uint32_t)inc);
          st.recv_window += inc;
        }
        return;
      }
      default:
        return;  // unknown frame types are ignored (RFC 9113 4.1)
    }
  }
  bool peer_goaway_ = false;

  std::shared_ptr<H2Conn> self() { return std::static_pointer_cast<H2Conn>(shared_from_this()); }

  void header_block_done(uint32_t sid) {
    HeaderList hl;
    std::string err;
    if (!hpack_.decode(hb_, hl, err)) return goaway(COMPRESSION_ERROR, err);
    hb_.clear();
    auto it = streams_.find(sid);
    if (it != streams_.end()) {  // trailers of a request: only END_STREAM matters for unary calls
      if (!hb_end_stream_) return rst(sid, PROTOCOL_ERROR);
      it->second.remote_closed = true;
      dispatch(sid);
      return;
    }
    if (peer_goaway_) return;
    last_stream_ = sid;
    if (streams_.size() >= kMaxStreams) return rst(sid, REFUSED_STREAM);
    Stream& st = streams_[sid];
    st.headers = std::move(hl);
    st.send_window = peer_initial_window_;
    if (hb_end_stream_) {
      st.remote_closed = true;
      dispatch(sid);
    }
  }

  void dispatch(uint32_t sid) {
    auto it = streams_.find(sid);
    if (it == streams_.end() || it->second.dispatched) return;
    Stream& st = it->second;
    st.dispatched = true;
    GrpcCall c;
    c.stream = sid;
    std::string method, ctype;
    for (auto& kv : st.headers) {
      if (kv.first == ":path") c.path = kv.second;
      else if (kv.first == ":method") method = kv.second;
      else if (kv.first == "content-type") ctype = kv.second;
      else if (!kv.first.empty() && kv.first[0] != ':') c.metadata.push_back(kv);
    }
    GrpcReply reply(self(), sid);
    if (method != "POST" || c.path.empty()) return reply.error(13, "gRPC requires POST with a :path");  // INTERNAL
    if (ctype.rfind("application/grpc", 0) != 0) return reply.error(13, "content-type is not application/grpc");
    const std::string& b = st.body;
    if (b.size() < 5) return reply.error(13, "missing gRPC message");
    if (b[0] != 0) return reply.error(12, "compressed messages are not supported");  // UNIMPLEMENTED
    uint32_t n = be32((const uint8_t*)b.data() + 1);
    if ((size_t)n + 5 != b.size()) return reply.error(12, "unary calls carry exactly one message");
    c.message.assign(b, 5, n);
    st.body.clear();
    st.body.shrink_to_fit();
    handler_(std::move(c), std::move(reply));
  }

  void update_interest() {
    uint32_t want = (peer_closed_ ? 0u : (uint32_t)EPOLLIN) | (out_off_ < out_.size() ? (uint32_t)EPOLLOUT : 0u);
    if (want != interest_) {
      interest_ = want;
      loop_.mod(this, want);
    }
  }
  void flush() {
    while (out_off_ < out_.size()) {
      ssize_t n = ::send(fd, out_.data() + out_off_, out_.size() - out_off_, MSG_NOSIGNAL);
      if (n > 0) {
        out_off_ += (size_t)n;
        continue;
      }
      if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      if (n < 0 && errno == EINTR) continue;
      close_now();
      return;
    }
    if (out_off_ == out_.size()) {
      out_.clear();
      out_off_ = 0;
      if (goaway_sent_ || (peer_goaway_ && streams_.empty())) {
        close_now();
        return;
      }
    }
    update_interest();
  }
  void close_now() { loop_.remove(this); }
};

inline void GrpcReply::send(int status, std::string_view status_message, std::string_view message,
                            const HeaderList& trailers) const {
  if (auto c = conn_.lock()) c->respond(stream_, status, status_message, message, trailers);
}

class H2Listener : public ev::IoObj {
 public:
  H2Listener(ev::Loop& loop, int fd, GrpcHandler& h) : loop_(loop), handler_(h) { this->fd = fd; }
  void on_event(uint32_t) override {
    while (true) {
      int c = ::accept4(fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (c < 0) {
        if (errno == EINTR) continue;
        return;
      }
      int one = 1;
      setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto conn = std::make_shared<H2Conn>(loop_, c, handler_);
      loop_.add(conn, EPOLLIN | EPOLLOUT);  // EPOLLOUT: the server preface is already queued
    }
  }

 private:
  ev::Loop& loop_;
  GrpcHandler& handler_;
};

// ------------------------------------------------------------------------------ gRPC client
// Unary gRPC calls over multiplexed HTTP/2 connections (one per endpoint): the transport of
// the SDK's DaprClient in the native app host (apphost.hpp), the counterpart of grpcio's
// channel.  Handles the full HPACK of the peer (the Python plane's grpcio server Huffman-codes
// and indexes), both flow-control directions, SETTINGS_MAX_CONCURRENT_STREAMS (calls queue),
// GOAWAY (calls the server never saw fail as UNAVAILABLE), RST_STREAM, per-call deadlines.
struct GrpcResult {
  int err = 0;          // transport failure (errno-like); 0: the call ended with a gRPC status
  int status = 2;       // grpc-status (UNKNOWN until the server says otherwise)
  std::string message;  // grpc-message, percent-decoded
  HeaderList metadata;  // response headers + trailers (without pseudo-headers)
  std::string payload;  // response message (length prefix removed)
};
using GrpcCallback = std::function<void(GrpcResult&&)>;

inline std::string grpc_percent_decode(std::string_view s) {
  std::string o;
  o.reserve(s.size());
  auto hv = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && hv(s[i + 1]) >= 0 && hv(s[i + 2]) >= 0) {
      o.push_back((char)(hv(s[i + 1]) << 4 | hv(s[i + 2])));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

class GrpcClient;

class H2ClientConn : public ev::IoObj {
 public:
  static constexpr uint32_t kStreamWindow = 4u << 20;
  static constexpr int64_t kConnWindow = 16 << 20;
  static constexpr size_t kMaxMessage = 256ull << 20;

  H2ClientConn(ev::Loop& loop, GrpcClient& owner, std::string key, std::string authority)
      : loop_(loop), owner_(owner), key_(std::move(key)), authority_(std::move(authority)) {
    out_.append(kPreface);
    put_frame_header(out_, 12, SETTINGS, 0, 0);
    auto setting = [&](uint16_t id, uint32_t v) {
      out_.push_back((char)(id >> 8));
      out_.push_back((char)id);
      put_be32(out_, v);
    };
    setting(0x2, 0);  // ENABLE_PUSH off
    setting(0x4, kStreamWindow);
    put_frame_header(out_, 4, WINDOW_UPDATE, 0, 0);
    put_be32(out_, (uint32_t)(kConnWindow - 65535));
  }
  bool connecting = false;
  bool usable() const { return !dead && !draining_; }
  const std::string& key() const { return key_; }

  void call(std::string path, const HeaderList& md, std::string_view msg, double deadline, GrpcCallback cb) {
    Pending p;
    p.path = std::move(path);
    p.md = md;
    p.body.reserve(msg.size() + 5);
    p.body.push_back(0);
    uint32_t n = (uint32_t)msg.size();
    char len[4] = {(char)(n >> 24), (char)(n >> 16), (char)(n >> 8), (char)n};
    p.body.append(len, 4);
    p.body.append(msg);
    p.deadline = deadline;
    p.cb = std::move(cb);
    waiting_.push_back(std::move(p));
    start_waiting();
    flush();
  }

  void on_event(uint32_t ev) override;
  void on_tick(double now) override {
    std::vector<uint32_t> expired;
    for (auto& kv : streams_)
      if (kv.second.deadline > 0 && now > kv.second.deadline) expired.push_back(kv.first);
    for (uint32_t id : expired) {
      put_frame_header(out_, 4, RST_STREAM, 0, id);
      put_be32(out_, CANCEL);
      finish_status(id, 4, "Deadline Exceeded");  // DEADLINE_EXCEEDED
    }
    for (auto it = waiting_.begin(); it != waiting_.end();) {
      if (it->deadline > 0 && now > it->deadline) {
        GrpcResult r;
        r.status = 4;
        r.message = "Deadline Exceeded";
        auto cb = std::move(it->cb);
        it = waiting_.erase(it);
        cb(std::move(r));
      } else {
        ++it;
      }
    }
    if (!expired.empty()) flush();
  }
  void fail_all(int err);

 private:
  struct Pending {
    std::string path;
    HeaderList md;
    std::string body;  // length-prefixed request message
    double deadline = 0;
    GrpcCallback cb;
  };
  struct Stream {
    GrpcCallback cb;
    std::string pending;  // request DATA not yet sent (flow control)
    int64_t send_window = 65535;
    int64_t recv_window = kStreamWindow;
    double deadline = 0;
    bool got_headers = false;
    int http_status = 0;
    HeaderList md;
    std::string data;
  };
  ev::Loop& loop_;
  GrpcClient& owner_;
  std::string key_, authority_;
  HpackDecoder hpack_;
  std::string in_, out_;
  size_t in_off_ = 0, out_off_ = 0;
  bool draining_ = false;
  uint32_t interest_ = 0;
  uint32_t next_id_ = 1;
  std::unordered_map<uint32_t, Stream> streams_;
  std::deque<Pending> waiting_;
  uint32_t peer_max_streams_ = 1000;  // until the peer's SETTINGS say otherwise
  uint32_t peer_max_frame_ = 16384;
  int64_t peer_initial_window_ = 65535;
  int64_t send_conn_window_ = 65535;
  int64_t recv_conn_window_ = kConnWindow, recv_conn_consumed_ = 0;
  uint32_t hb_stream_ = 0;
  bool hb_end_stream_ = false;
  std::string hb_;

  void start_waiting() {
    while (!waiting_.empty() && !draining_ && streams_.size() < peer_max_streams_) {
      if (next_id_ > 0x7ffffffdu) {  // stream ids exhausted: this connection takes no more calls
        draining_ = true;
        break;
      }
      Pending p = std::move(waiting_.front());
      waiting_.pop_front();
      uint32_t id = next_id_;
      next_id_ += 2;
      std::string hb;
      hb.push_back((char)0x83);  // :method POST
      hb.push_back((char)0x86);  // :scheme http
      hpack_literal(hb, ":path", p.path);
      hpack_literal(hb, ":authority", authority_);
      hpack_literal(hb, "content-type", "application/grpc");
      hpack_literal(hb, "te", "trailers");
      if (p.deadline > 0) {
        long long ms = (long long)((p.deadline - ev::now_s()) * 1000) + 1;
        hpack_literal(hb, "grpc-timeout", std::to_string(ms < 1 ? 1 : ms) + "m");
      }
      for (auto& kv : p.md) hpack_literal(hb, kv.first, kv.second);
      size_t off = 0;
      bool first = true;
      do {  // HEADERS (+ CONTINUATION) -- END_STREAM travels on the last DATA frame
        size_t n = std::min<size_t>(hb.size() - off, peer_max_frame_);
        bool last = off + n == hb.size();
        put_frame_header(out_, (uint32_t)n, first ? HEADERS : CONTINUATION, last ? END_HEADERS : 0, id);
        out_.append(hb, off, n);
        off += n;
        first = false;
      } while (off < hb.size());
      Stream& st = streams_[id];
      st.cb = std::move(p.cb);
      st.pending = std::move(p.body);
      st.send_window = peer_initial_window_;
      st.deadline = p.deadline;
      pump(id);
    }
  }
  void pump(uint32_t id) {
    auto it = streams_.find(id);
    if (it == streams_.end()) return;
    Stream& st = it->second;
    while (!st.pending.empty()) {
      int64_t room = std::min<int64_t>({send_conn_window_, st.send_window, (int64_t)peer_max_frame_});
      if (room <= 0) return;
      size_t n = std::min<size_t>(st.pending.size(), (size_t)room);
      bool last = n == st.pending.size();
      put_frame_header(out_, (uint32_t)n, DATA, last ? END_STREAM : 0, id);
      out_.append(st.pending, 0, n);
      st.pending.erase(0, n);
      send_conn_window_ -= (int64_t)n;
      st.send_window -= (int64_t)n;
    }
  }
  void pump_all() {
    std::vector<uint32_t> ids;
    for (auto& kv : streams_)
      if (!kv.second.pending.empty()) ids.push_back(kv.first);
    for (uint32_t id : ids) pump(id);
  }

  void finish_status(uint32_t id, int status, std::string msg) {
    auto it = streams_.find(id);
    if (it == streams_.end()) return;
    GrpcResult r;
    r.status = status;
    r.message = std::move(msg);
    r.metadata = std::move(it->second.md);
    auto cb = std::move(it->second.cb);
    streams_.erase(it);
    cb(std::move(r));
    start_waiting();
  }
  void finish(uint32_t id) {
    auto it = streams_.find(id);
    if (it == streams_.end()) return;
    Stream& st = it->second;
    GrpcResult r;
    const std::string* gs = nullptr;
    for (auto& kv : st.md) {
      if (kv.first == "grpc-status") gs = &kv.second;
      else if (kv.first == "grpc-message") r.message = grpc_percent_decode(kv.second);
    }
    if (st.http_status != 200) {  // gRPC over HTTP/2: map the HTTP status (gRPC spec)
      r.status = st.http_status == 400 ? 13 : st.http_status == 401 ? 16 : st.http_status == 403 ? 7
               : st.http_status == 404 ? 12 : (st.http_status >= 502 && st.http_status <= 504) ? 14 : 2;
      if (r.message.empty()) r.message = "HTTP status " + std::to_string(st.http_status);
    } else if (!gs) {
      r.status = 2;
      if (r.message.empty()) r.message = "missing grpc-status";
    } else {
      r.status = std::atoi(gs->c_str());
    }
    if (r.status == 0) {  // unary: exactly one uncompressed message
      const std::string& d = st.data;
      if (d.size() >= 5 && d[0] == 0 && be32((const uint8_t*)d.data() + 1) + (size_t)5 == d.size()) {
        r.payload.assign(d, 5, std::string::npos);
      } else {
        r.status = 13;  // INTERNAL
        r.message = !d.empty() && d[0] != 0 ? "compressed response not supported" : "malformed response message";
      }
    }
    r.metadata = std::move(st.md);
    auto cb = std::move(st.cb);
    streams_.erase(it);
    cb(std::move(r));
    start_waiting();
  }

  void conn_error(ErrorCode code, std::string_view why) {
    put_frame_header(out_, 8 + (uint32_t)why.size(), GOAWAY, 0, 0);
    put_be32(out_, 0);
    put_be32(out_, code);
    out_.append(why);
    draining_ = true;
    fail_all(EPROTO);
    flush();  // sends the GOAWAY, then closes (draining, nothing left)
  }

  void process();
  void frame(uint8_t type, uint8_t flags, uint32_t sid, std::string_view p);
  void header_block_done(uint32_t sid);
  void update_interest() {
    uint32_t want = EPOLLIN | ((connecting || out_off_ < out_.size()) ? (uint32_t)EPOLLOUT : 0u);
    if (want != interest_) {
      interest_ = want;
      loop_.mod(this, want);
    }
  }

 public:
  void registered(uint32_t ev) { interest_ = ev; }
  void flush();
};

class GrpcClient {
 public:
  explicit GrpcClient(ev::Loop& loop) : loop_(loop) {}
  void call(const ev::Endpoint& ep, std::string path, const HeaderList& md, std::string_view msg, double timeout_s,
            GrpcCallback cb) {
    std::string key = ep.key();
    auto it = conns_.find(key);
    std::shared_ptr<H2ClientConn> c;
    if (it != conns_.end() && it->second->usable()) c = it->second;
    if (!c) {
      int err = 0;
      c = connect(ep, key, err);
      if (!c) {
        loop_.defer([cb = std::move(cb), err]() mutable {
          GrpcResult r;
          r.err = err;
          cb(std::move(r));
        });
        return;
      }
      conns_[key] = c;
    }
    c->call(std::move(path), md, msg, timeout_s > 0 ? ev::now_s() + timeout_s : 0, std::move(cb));
  }
  void forget(H2ClientConn* c) {
    auto it = conns_.find(c->key());
    if (it != conns_.end() && it->second.get() == c) conns_.erase(it);
  }

 private:
  ev::Loop& loop_;
  std::unordered_map<std::string, std::shared_ptr<H2ClientConn>> conns_;

  std::shared_ptr<H2ClientConn> connect(const ev::Endpoint& ep, const std::string& key, int& err) {
    int fd;
    bool in_progress = false;
    if (ep.unix_socket) {
      fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      sockaddr_un a{};
      a.sun_family = AF_UNIX;
      std::strncpy(a.sun_path, ep.path.c_str(), sizeof a.sun_path - 1);
      if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        err = errno;
        ::close(fd);
        return nullptr;
      }
    } else {
      fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)ep.port);
      inet_pton(AF_INET, ep.host.c_str(), &a.sin_addr);
      if (::connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        if (errno != EINPROGRESS) {
          err = errno;
          ::close(fd);
          return nullptr;
        }
        in_progress = true;
      }
    }
    auto c = std::make_shared<H2ClientConn>(loop_, *this, key,
                                            ep.unix_socket ? std::string("localhost") : ep.host + ":" + std::to_string(ep.port));
    c->fd = fd;
    c->connecting = in_progress;
    uint32_t ev = EPOLLIN | EPOLLOUT;  // the preface is queued either way
    loop_.add(c, ev);
    c->registered(ev);
    return c;
  }
};

inline void H2ClientConn::fail_all(int err) {
  owner_.forget(this);
  std::vector<GrpcCallback> cbs;
  for (auto& kv : streams_) cbs.push_back(std::move(kv.second.cb));
  for (auto& p : waiting_) cbs.push_back(std::move(p.cb));
  streams_.clear();
  waiting_.clear();
  for (auto& cb : cbs) {
    GrpcResult r;
    r.err = err;
    cb(std::move(r));
  }
}

inline void H2ClientConn::flush() {
  if (dead || connecting) return;
  while (out_off_ < out_.size()) {
    ssize_t n = ::send(fd, out_.data() + out_off_, out_.size() - out_off_, MSG_NOSIGNAL);
    if (n > 0) {
      out_off_ += (size_t)n;
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    if (n < 0 && errno == EINTR) continue;
    loop_.remove(this);
    fail_all(ECONNRESET);
    return;
  }
  if (out_off_ == out_.size()) {
    out_.clear();
    out_off_ = 0;
  }
  if (draining_ && streams_.empty() && waiting_.empty() && out_.empty()) {
    loop_.remove(this);
    owner_.forget(this);
    return;
  }
  update_interest();
}

inline void H2ClientConn::on_event(uint32_t ev) {
  if (connecting) {
    if (!(ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) return;
    int e = 0;
    socklen_t l = sizeof e;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &l);
    if (e) {
      loop_.remove(this);
      fail_all(e);
      return;
    }
    connecting = false;
  }
  if (ev & (EPOLLIN | EPOLLHUP | EPOLLERR)) {
    char buf[65536];
    bool closed = false;
    while (true) {
      ssize_t n = ::recv(fd, buf, sizeof buf, 0);
      if (n > 0) {
        in_.append(buf, (size_t)n);
        if ((size_t)n < sizeof buf) break;
        continue;
      }
      if (n == 0) {
        closed = true;
        break;
      }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      closed = true;
      break;
    }
    process();
    if (dead) return;
    if (closed) {
      loop_.remove(this);
      fail_all(ECONNRESET);
      return;
    }
  }
  flush();
}

inline void H2ClientConn::process() {
  while (!dead && in_.size() - in_off_ >= 9) {
    const uint8_t* h = (const uint8_t*)in_.data() + in_off_;
    uint32_t len = (uint32_t)h[0] << 16 | (uint32_t)h[1] << 8 | h[2];
    if (len > 16384) return conn_error(FRAME_SIZE_ERROR, "frame larger than SETTINGS_MAX_FRAME_SIZE");
    if (in_.size() - in_off_ < 9 + (size_t)len) break;
    uint8_t type = h[3], flags = h[4];
    uint32_t sid = be32(h + 5) & 0x7fffffffu;
    std::string_view payload(in_.data() + in_off_ + 9, len);
    in_off_ += 9 + len;
    frame(type, flags, sid, payload);
  }
  if (dead) return;
  if (in_off_ > 0 && (in_off_ == in_.size() || in_off_ > 65536)) {
    in_.erase(0, in_off_);
    in_off_ = 0;
  }
  if (recv_conn_consumed_ >= kConnWindow / 4) {
    put_frame_header(out_, 4, WINDOW_UPDATE, 0, 0);
    put_be32(out_, (uint32_t)recv_conn_consumed_);
    recv_conn_window_ += recv_conn_consumed_;
    recv_conn_consumed_ = 0;
  }
}

inline void H2ClientConn::frame(uint8_t type, uint8_t flags, uint32_t sid, std::string_view p) {
  if (hb_stream_ && type != CONTINUATION) return conn_error(PROTOCOL_ERROR, "header block interrupted");
  auto strip = [&](std::string_view& v) {
    if (!(flags & PADDED)) return true;
    if (v.empty()) return false;
    size_t pad = (uint8_t)v[0];
    if (pad >= v.size()) return false;
    v = v.substr(1, v.size() - 1 - pad);
    return true;
  };
  switch (type) {
    case SETTINGS: {
      if (flags & ACK) return;
      if (p.size() % 6) return conn_error(FRAME_SIZE_ERROR, "SETTINGS length");
      for (size_t i = 0; i < p.size(); i += 6) {
        uint16_t id = (uint16_t)((uint8_t)p[i] << 8 | (uint8_t)p[i + 1]);
        uint32_t v = be32((const uint8_t*)p.data() + i + 2);
        if (id == 0x3) peer_max_streams_ = v;
        else if (id == 0x4) {
          if (v > 0x7fffffffu) return conn_error(FLOW_CONTROL_ERROR, "initial window");
          int64_t delta = (int64_t)v - peer_initial_window_;
          peer_initial_window_ = v;
          for (auto& kv : streams_) kv.second.send_window += delta;
        } else if (id == 0x5) {
          if (v < 16384 || v > 16777215) return conn_error(PROTOCOL_ERROR, "max frame size");
          peer_max_frame_ = v;
        }
      }
      put_frame_header(out_, 0, SETTINGS, ACK, 0);
      pump_all();
      start_waiting();
      return;
    }
    case PING:
      if (p.size() != 8) return conn_error(FRAME_SIZE_ERROR, "PING length");
      if (!(flags & ACK)) {
        put_frame_header(out_, 8, PING, ACK, 0);
        out_.append(p);
      }
      return;
    case WINDOW_UPDATE: {
      if (p.size() != 4) return conn_error(FRAME_SIZE_ERROR, "WINDOW_UPDATE length");
      uint32_t inc = be32((const uint8_t*)p.data()) & 0x7fffffffu;
      if (!sid) {
        send_conn_window_ += inc;
        pump_all();
      } else if (auto it = streams_.find(sid); it != streams_.end()) {
        it->second.send_window += inc;
        pump(sid);
      }
      return;
    }
    case GOAWAY: {
      if (p.size() < 8) return conn_error(FRAME_SIZE_ERROR, "GOAWAY length");
      uint32_t last = be32((const uint8_t*)p.data()) & 0x7fffffffu;
      draining_ = true;
      owner_.forget(this);
      std::vector<uint32_t> unseen;
      for (auto& kv : streams_)
        if (kv.first > last) unseen.push_back(kv.first);
      for (uint32_t id : unseen) finish_status(id, 14, "connection going away");  // UNAVAILABLE
      while (!waiting_.empty()) {  // never started on this connection
        GrpcResult r;
        r.status = 14;
        r.message = "connection going away";
        auto cb = std::move(waiting_.front().cb);
        waiting_.pop_front();
        cb(std::move(r));
      }
      return;
    }
    case RST_STREAM: {
      if (p.size() != 4) return conn_error(FRAME_SIZE_ERROR, "RST_STREAM length");
      uint32_t code = be32((const uint8_t*)p.data());
      return finish_status(sid, code == REFUSED_STREAM ? 14 : code == CANCEL ? 1 : 13,
                           "stream reset by the server (HTTP/2 error " + std::to_string(code) + ")");
    }
    case PUSH_PROMISE:
      return conn_error(PROTOCOL_ERROR, "push disabled");
    case HEADERS: {
      if (!strip(p)) return conn_error(PROTOCOL_ERROR, "padding");
      if (flags & PRIORITY_FLAG) {
        if (p.size() < 5) return conn_error(PROTOCOL_ERROR, "priority");
        p.remove_prefix(5);
      }
      hb_.assign(p);
      hb_end_stream_ = flags & END_STREAM;
      if (flags & END_HEADERS) return header_block_done(sid);
      hb_stream_ = sid;
      return;
    }
    case CONTINUATION:
      if (!hb_stream_ || sid != hb_stream_) return conn_error(PROTOCOL_ERROR, "unexpected CONTINUATION");
      hb_.append(p);
      if (hb_.size() > 256 * 1024) return conn_error(PROTOCOL_ERROR, "header block too large");
      if (flags & END_HEADERS) {
        hb_stream_ = 0;
        header_block_done(sid);
      }
      return;
    case DATA: {
      int64_t flen = (int64_t)p.size();
      recv_conn_window_ -= flen;
      recv_conn_consumed_ += flen;
      if (recv_conn_window_ < 0) return conn_error(FLOW_CONTROL_ERROR, "connection window exceeded");
      if (!strip(p)) return conn_error(PROTOCOL_ERROR, "padding");
      auto it = streams_.find(sid);
      if (it == streams_.end()) return;
      Stream& st = it->second;
      st.recv_window -= flen;
      if (st.data.size() + p.size() > kMaxMessage + 5) {
        put_frame_header(out_, 4, RST_STREAM, 0, sid);
        put_be32(out_, CANCEL);
        return finish_status(sid, 8, "response message larger than the client's limit");
      }
      st.data.append(p);
      if (flags & END_STREAM) return finish(sid);
      if (st.recv_window < (int64_t)kStreamWindow / 2) {
        int64_t inc = (int64_t)kStreamWindow - st.recv_window;
        put_frame_header(out_, 4, WINDOW_UPDATE, 0, sid);
        put_be32(out_, (uint32_t)inc);
        st.recv_window += inc;
      }
      return;
    }
    default:
      return;
  }
}

inline void H2ClientConn::header_block_done(uint32_t sid) {
  HeaderList hl;
  std::string err;
  if (!hpack_.decode(hb_, hl, err)) return conn_error(COMPRESSION_ERROR, err);  // table state is lost
  hb_.clear();
  auto it = streams_.find(sid);
  if (it == streams_.end()) return;  // a stream we already finished (e.g. deadline)
  Stream& st = it->second;
  for (auto& kv : hl) {
    if (kv.first == ":status") st.http_status = std::atoi(kv.second.c_str());
    else if (!kv.first.empty() && kv.first[0] != ':') st.md.push_back(std::move(kv));
  }
  if (!st.got_headers) {
    st.got_headers = true;
    if (!st.http_status) st.http_status = 200;
  }
  if (hb_end_stream_) finish(sid);
}

// Listen for HTTP/2 gRPC clients; returns the bound TCP port (0 for a unix socket).
inline int listen_grpc(ev::Loop& loop, const ev::Endpoint& ep, GrpcHandler& h) {
  int port = 0;
  int fd = ev::bind_listen(ep, false, port);
  loop.add(std::make_shared<H2Listener>(loop, fd, h), EPOLLIN);
  return port;
}

}  // namespace tt::h2
