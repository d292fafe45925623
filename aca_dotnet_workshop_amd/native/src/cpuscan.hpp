// Multi-threaded CPU executor of the columnar query program (ops/columnar.py Program) over the
// SAME narrow encodings the gfx950 kernels read (ops/hip/query_scan.hip): dictionary codes of
// 1/2/4 bytes per row (all-ones = path missing), rank-encoded copies for range leaves, 1-bit
// liveness.  It is the fair host baseline for the GPU scan (same bytes per row, every core of the
// process's CPU share, SIMD compares) and the state store's columnar executor on hosts without a
// GPU.  Semantics are tt_scan_eval's: leaves produce row masks, AND/OR/NOT combine them, the
// result is ANDed with liveness and compacted to ascending row ids.
//
// Rows are processed 64 at a time: each leaf yields one 64-bit mask (AVX-512BW compare-to-mask
// when the CPU has it, a scalar loop otherwise), the program's stack holds 64-bit masks.  Pass 1
// (threads over contiguous row ranges) writes the masks and per-thread counts; pass 2 writes each
// thread's row ids at its exclusive-prefix offset.
#pragma once

#include <immintrin.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <thread>
#include <vector>

namespace cpuscan {

enum Op : int32_t { OP_LEAF = 1, OP_AND = 2, OP_OR = 3, OP_NOT = 4, OP_TRUE = 5, OP_EQ = 6, OP_RANGE = 7 };
constexpr int kMaxDepth = 8;

struct Col {
  const uint8_t* p = nullptr;
  int width = 1;  // bytes per row; 0 = 2 bits per row (4 rows per byte, row r in bits 2(r mod 4))
};

inline uint32_t raw_at(const Col& c, int64_t row) {
  if (c.width == 0) return (c.p[row >> 2] >> ((row & 3) * 2)) & 3u;
  if (c.width == 1) return c.p[row];
  if (c.width == 2) return reinterpret_cast<const uint16_t*>(c.p)[row];
  return reinterpret_cast<const uint32_t*>(c.p)[row];
}

inline int32_t id_of(uint32_t raw, int width) {
  if (width == 0) return raw == 3u ? -1 : (int32_t)raw;
  if (width == 1) return raw == 0xFFu ? -1 : (int32_t)raw;
  if (width == 2) return raw == 0xFFFFu ? -1 : (int32_t)raw;
  return (int32_t)raw;
}

// ---- 64-row leaf masks -------------------------------------------------------------------
inline uint64_t eq_scalar(const Col& c, int64_t r0, int32_t b) {
  uint64_t m = 0;
  for (int i = 0; i < 64; ++i) m |= (uint64_t)(id_of(raw_at(c, r0 + i), c.width) == b) << i;
  return m;
}

inline uint64_t range_scalar(const Col& c, int64_t r0, uint32_t b, uint32_t span) {
  uint64_t m = 0;
  for (int i = 0; i < 64; ++i) m |= (uint64_t)((raw_at(c, r0 + i) - b) < span) << i;
  return m;
}

inline uint64_t bitmap_scalar(const Col& c, int64_t r0, const uint32_t* bm, int32_t nbits) {
  uint64_t m = 0;
  for (int i = 0; i < 64; ++i) {
    const int32_t id = id_of(raw_at(c, r0 + i), c.width);
    m |= (uint64_t)((id >= 0 && id < nbits) ? ((bm[id >> 5] >> (id & 31)) & 1u) : 0u) << i;
  }
  return m;
}

// 2-bit codes of 64 rows (16 bytes) equal to `b`: XOR with the replicated code leaves a zero
// pair exactly where they match; the even bits of (pair == 0) gathered with PEXT.
__attribute__((target("bmi2"))) inline uint64_t eq_2bit(const Col& c, int64_t r0, int32_t b) {
  if (b < 0 || b > 2) return 0;
  uint64_t w[2];
  std::memcpy(w, c.p + (r0 >> 2), 16);
  const uint64_t pat = 0x5555555555555555ull * (uint64_t)b;
  uint64_t m = 0;
  for (int h = 0; h < 2; ++h) {
    const uint64_t x = w[h] ^ pat;
    const uint64_t zero = ~(x | (x >> 1)) & 0x5555555555555555ull;
    m |= (uint64_t)_pext_u64(zero, 0x5555555555555555ull) << (32 * h);
  }
  return m;
}

// AVX-512BW: one compare instruction per 64 (1-byte) / 32 (2-byte) / 16 (4-byte) rows.
__attribute__((target("avx512f,avx512bw,bmi2"))) inline uint64_t eq_avx512(const Col& c, int64_t r0, int32_t b) {
  if (c.width == 0) return eq_2bit(c, r0, b);
  if (c.width == 1) {
    if (b < 0 || b >= 0xFF) return 0;  // ids of a 1-byte column are < 255; -1/-2 never stored
    return _mm512_cmpeq_epi8_mask(_mm512_loadu_si512(c.p + r0), _mm512_set1_epi8((char)b));
  }
  if (c.width == 2) {
    if (b < 0 || b >= 0xFFFF) return 0;
    const uint16_t* p = reinterpret_cast<const uint16_t*>(c.p) + r0;
    const __m512i v = _mm512_set1_epi16((short)b);
    return (uint64_t)_mm512_cmpeq_epi16_mask(_mm512_loadu_si512(p), v) |
           ((uint64_t)_mm512_cmpeq_epi16_mask(_mm512_loadu_si512(p + 32), v) << 32);
  }
  const uint32_t* p = reinterpret_cast<const uint32_t*>(c.p) + r0;
  const __m512i v = _mm512_set1_epi32(b);
  uint64_t m = 0;
  for (int q = 0; q < 4; ++q) m |= (uint64_t)_mm512_cmpeq_epi32_mask(_mm512_loadu_si512(p + 16 * q), v) << (16 * q);
  return m;
}

__attribute__((target("avx512f,avx512bw"))) inline uint64_t range_avx512(const Col& c, int64_t r0, uint32_t b,
                                                                        uint32_t span) {
  // (raw - b) < span, unsigned, in the column's own width (spans never exceed the width's codes)
  // in the narrow width the subtraction wraps mod 2^8 / 2^16, which equals the 32-bit test
  // while b + span (the leaf's upper rank) fits the width: range_ok() checks that
  if (c.width == 1) {
    const __m512i d = _mm512_sub_epi8(_mm512_loadu_si512(c.p + r0), _mm512_set1_epi8((char)b));
    return _mm512_cmplt_epu8_mask(d, _mm512_set1_epi8((char)span));
  }
  if (c.width == 2) {
    const uint16_t* p = reinterpret_cast<const uint16_t*>(c.p) + r0;
    const __m512i vb = _mm512_set1_epi16((short)b), vs = _mm512_set1_epi16((short)span);
    const __m512i d0 = _mm512_sub_epi16(_mm512_loadu_si512(p), vb), d1 = _mm512_sub_epi16(_mm512_loadu_si512(p + 32), vb);
    return (uint64_t)_mm512_cmplt_epu16_mask(d0, vs) | ((uint64_t)_mm512_cmplt_epu16_mask(d1, vs) << 32);
  }
  const uint32_t* p = reinterpret_cast<const uint32_t*>(c.p) + r0;
  const __m512i vb = _mm512_set1_epi32((int)b), vs = _mm512_set1_epi32((int)span);
  uint64_t m = 0;
  for (int q = 0; q < 4; ++q)
    m |= (uint64_t)_mm512_cmplt_epu32_mask(_mm512_sub_epi32(_mm512_loadu_si512(p + 16 * q), vb), vs) << (16 * q);
  return m;
}

inline bool range_ok(const Col& c, int32_t b, int32_t hi) {
  if (b < 0 || hi < b || c.width == 0) return false;
  return c.width == 4 || (c.width == 1 ? hi <= 0xFF : hi <= 0xFFFF);
}

struct Program {
  std::vector<int32_t> code;      // [L x 4]
  std::vector<uint32_t> bitmaps;
};

inline bool has_avx512() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                         __builtin_cpu_supports("bmi2");
  return ok;
}

// Masks of rows [r0, r0 + 64) (r0 a multiple of 64, the columns padded to the capacity).  Two
// copies: one compiled for AVX-512BW (its leaf tests inline into it), one portable.
#define TT_CPUSCAN_EVAL64(NAME, ATTR, EQ, RANGE)                                                         \
  ATTR inline uint64_t NAME(const std::vector<Col>& cols, const Program& pg, int64_t r0) {              \
    uint64_t st[kMaxDepth + 1];                                                                         \
    int sp = 0;                                                                                         \
    const size_t L = pg.code.size() / 4;                                                                \
    const int32_t* code = pg.code.data();                                                               \
    for (size_t pc = 0; pc < L; ++pc) {                                                                 \
      const int32_t op = code[pc * 4], a = code[pc * 4 + 1], b = code[pc * 4 + 2], c = code[pc * 4 + 3]; \
      switch (op) {                                                                                     \
        case OP_EQ:                                                                                     \
          st[sp++] = EQ(cols[a], r0, b);                                                                \
          break;                                                                                        \
        case OP_RANGE:                                                                                  \
          st[sp++] = RANGE(cols[a], r0, b, c);                                                          \
          break;                                                                                        \
        case OP_LEAF:                                                                                   \
          st[sp++] = bitmap_scalar(cols[a], r0, pg.bitmaps.data() + b, c);                              \
          break;                                                                                        \
        case OP_AND:                                                                                    \
        case OP_OR: {                                                                                   \
          uint64_t r = op == OP_AND ? ~0ull : 0ull;                                                     \
          for (int k = 0; k < a; ++k) r = op == OP_AND ? (r & st[--sp]) : (r | st[--sp]);              \
          st[sp++] = r;                                                                                 \
          break;                                                                                        \
        }                                                                                               \
        case OP_NOT:                                                                                    \
          st[sp - 1] = ~st[sp - 1];                                                                     \
          break;                                                                                        \
        default:                                                                                        \
          st[sp++] = ~0ull;                                                                             \
      }                                                                                                 \
    }                                                                                                   \
    return st[sp - 1];                                                                                  \
  }

inline uint64_t range_leaf_scalar(const Col& c, int64_t r0, int32_t b, int32_t hi) {
  return range_scalar(c, r0, (uint32_t)b, (uint32_t)(hi - b));
}
__attribute__((target("avx512f,avx512bw,bmi2"))) inline uint64_t range_leaf_avx512(const Col& c, int64_t r0, int32_t b,
                                                                             int32_t hi) {
  return range_ok(c, b, hi) ? range_avx512(c, r0, (uint32_t)b, (uint32_t)(hi - b))
                            : range_scalar(c, r0, (uint32_t)b, (uint32_t)(hi - b));
}

TT_CPUSCAN_EVAL64(eval64_avx512, __attribute__((target("avx512f,avx512bw,bmi2"))), eq_avx512, range_leaf_avx512)
TT_CPUSCAN_EVAL64(eval64_scalar, , eq_scalar, range_leaf_scalar)
#undef TT_CPUSCAN_EVAL64

// Pass 1 over blocks [b0, b1): masks (ANDed with liveness, the tail cut at nrows) and their count.
#define TT_CPUSCAN_PASS1(NAME, ATTR, EVAL)                                                                \
  ATTR inline int64_t NAME(const std::vector<Col>& cols, const Program& pg, const uint16_t* live,         \
                           int64_t nrows, int64_t b0, int64_t b1, uint64_t* masks) {                     \
    int64_t cnt = 0;                                                                                      \
    const int64_t last = (nrows + 63) / 64 - 1;                                                           \
    for (int64_t blk = b0; blk < b1; ++blk) {                                                             \
      uint64_t m = EVAL(cols, pg, blk * 64);                                                              \
      uint64_t lv;                                                                                        \
      std::memcpy(&lv, live + blk * 4, 8);                                                                \
      m &= lv;                                                                                            \
      if (blk == last && (nrows & 63)) m &= (1ull << (nrows & 63)) - 1;                                   \
      masks[blk] = m;                                                                                     \
      cnt += __builtin_popcountll(m);                                                                     \
    }                                                                                                     \
    return cnt;                                                                                           \
  }
TT_CPUSCAN_PASS1(pass1_avx512, __attribute__((target("avx512f,avx512bw,bmi2,popcnt"))), eval64_avx512)
TT_CPUSCAN_PASS1(pass1_scalar, , eval64_scalar)
#undef TT_CPUSCAN_PASS1

// Large scratch / result buffers on 2 MiB pages when the kernel allows it: the scan's threads
// first-touch them concurrently, and 4 KiB page faults serialise on the process's mm lock.
struct HugeFree {
  void operator()(void* p) const { std::free(p); }
};
inline void* huge_alloc(size_t bytes) {
  constexpr size_t kHuge = 2u << 20;
  const size_t n = std::max<size_t>(kHuge, (bytes + kHuge - 1) / kHuge * kHuge);
  void* p = std::aligned_alloc(kHuge, n);
  if (p == nullptr) throw std::bad_alloc();
  ::madvise(p, n, MADV_HUGEPAGE);  // advisory: 4 KiB pages if THP is off
  return p;
}

// Program check: leaf columns / bitmaps in range, well-formed stack (throws invalid_argument).
inline void validate(const std::vector<Col>& cols, const Program& pg) {
  const size_t L = pg.code.size() / 4;
  if (L == 0) throw std::invalid_argument("empty program");
  int depth = 0, maxd = 0;
  for (size_t pc = 0; pc < L; ++pc) {
    const int32_t op = pg.code[pc * 4], a = pg.code[pc * 4 + 1];
    if (op == OP_EQ || op == OP_RANGE || op == OP_LEAF || op == OP_TRUE) {
      if (op != OP_TRUE && (a < 0 || (size_t)a >= cols.size())) throw std::invalid_argument("leaf column out of range");
      if (op == OP_LEAF && (pg.code[pc * 4 + 2] < 0 || pg.code[pc * 4 + 3] < 0 ||
                            (int64_t)pg.code[pc * 4 + 2] + ((int64_t)pg.code[pc * 4 + 3] + 31) / 32 > (int64_t)pg.bitmaps.size()))
        throw std::invalid_argument("leaf bitmap out of range");
      ++depth;
    } else if (op == OP_AND || op == OP_OR) {
      if (a < 1 || a > depth) throw std::invalid_argument("malformed program");
      depth -= a - 1;
    } else if (op == OP_NOT) {
      if (depth < 1) throw std::invalid_argument("malformed program");
    } else {
      throw std::invalid_argument("unknown opcode");
    }
    maxd = std::max(maxd, depth);
  }
  if (depth != 1 || maxd > kMaxDepth) throw std::invalid_argument("malformed program");
}

// Two-pass selection of rows [0, nrows): `live` holds 1 bit per row (little-endian 16-bit words,
// the device layout); columns must be readable up to nrows rounded up to 64.  count() evaluates
// the masks (threads over contiguous row ranges) and returns the total; write() stores the
// ascending row ids into a caller-provided buffer of that size (each thread at its prefix).
class Selection {
 public:
  Selection(const std::vector<Col>& cols, const uint16_t* live, int64_t nrows, const Program& pg, int nthreads,
            bool allow_simd)
      : cols_(cols), live_(live), nrows_(nrows), pg_(pg) {
    validate(cols, pg);
    blocks_ = (nrows + 63) / 64;
    nthreads_ = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, (blocks_ + 255) / 256));
    simd_ = allow_simd && has_avx512();
  }

  int64_t count() {
    masks_.reset(static_cast<uint64_t*>(huge_alloc((size_t)blocks_ * sizeof(uint64_t))));
    offs_.assign((size_t)nthreads_ + 1, 0);
    run([this](int t) {
      auto [b0, b1] = range(t);
      offs_[(size_t)t + 1] = simd_ ? pass1_avx512(cols_, pg_, live_, nrows_, b0, b1, masks_.get())
                                   : pass1_scalar(cols_, pg_, live_, nrows_, b0, b1, masks_.get());
    });
    for (int t = 0; t < nthreads_; ++t) offs_[(size_t)t + 1] += offs_[(size_t)t];
    return offs_[(size_t)nthreads_];
  }

  void write(int32_t* out) {
    run([this, out](int t) {
      auto [b0, b1] = range(t);
      int32_t* o = out + offs_[(size_t)t];
      for (int64_t blk = b0; blk < b1; ++blk) {
        uint64_t m = masks_.get()[blk];
        const int32_t base = (int32_t)(blk * 64);
        while (m) {
          *o++ = base + __builtin_ctzll(m);
          m &= m - 1;
        }
      }
    });
  }

 private:
  const std::vector<Col>& cols_;
  const uint16_t* live_;
  int64_t nrows_, blocks_ = 0;
  const Program& pg_;
  int nthreads_ = 1;
  bool simd_ = false;
  std::unique_ptr<uint64_t, HugeFree> masks_;
  std::vector<int64_t> offs_;

  std::pair<int64_t, int64_t> range(int t) const {
    const int64_t per = (blocks_ + nthreads_ - 1) / nthreads_;
    return {std::min(blocks_, t * per), std::min(blocks_, (t + 1) * per)};
  }
  template <class F>
  void run(F f) {
    std::vector<std::thread> th;
    th.reserve((size_t)nthreads_);
    for (int t = 1; t < nthreads_; ++t) th.emplace_back(f, t);
    f(0);
    for (auto& x : th) x.join();
  }
};

inline std::vector<int32_t> select(const std::vector<Col>& cols, const uint16_t* live, int64_t nrows,
                                   const Program& pg, int nthreads, bool allow_simd = true) {
  Selection s(cols, live, nrows, pg, nthreads, allow_simd);
  std::vector<int32_t> out((size_t)s.count());
  s.write(out.data());
  return out;
}

}  // namespace cpuscan
