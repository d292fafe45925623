// Shared device code of the gfx950 query kernels (query_scan.hip, page_topk.hip): the column
// descriptor table, the narrow-code loads and the postfix filter interpreter over 16-row groups.
// See query_scan.hip for the data model.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kBlock = 256;                    // 4 waves (compaction, group count)
constexpr int kRowsPerLane = 16;
constexpr int kTileRows = 8192;               // rows per scan / compaction block
static_assert(kTileRows == kBlock * 32, "compaction takes 32 mask bits per thread per tile");
constexpr int kMaxDepth = 8;                   // 8 x 16-bit masks in a 128-bit stack
constexpr int kMaxLdsBitmapWords = 8192;       // stage up to 32 KiB of leaf bitmaps in LDS

enum Op : int32_t { OP_LEAF = 1, OP_AND = 2, OP_OR = 3, OP_NOT = 4, OP_TRUE = 5, OP_EQ = 6, OP_RANGE = 7 };

struct ColumnDesc {     // 16 bytes, host-built table
  uint64_t ptr;         // device address of the column (row 0)
  int32_t width;        // 1, 2 or 4 bytes per row; 0 = 2 bits per row
  int32_t pad;
};

using u128 = unsigned __int128;

__device__ __forceinline__ int32_t id_of(uint32_t raw, int width) {
  if (width == 0) return raw == 3u ? -1 : (int32_t)raw;
  if (width == 1) return raw == 0xFFu ? -1 : (int32_t)raw;
  if (width == 2) return raw == 0xFFFFu ? -1 : (int32_t)raw;
  return (int32_t)raw;
}

// Load the 16 ids of rows [row0, row0+16) of one column.
__device__ __forceinline__ void load16(const ColumnDesc& cd, int64_t row0, int32_t (&ids)[16]) {
  if (cd.width == 0) {  // one dword: 16 two-bit codes (row0 is a multiple of 16)
    const uint32_t w = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(cd.ptr) + (row0 >> 2));
#pragma unroll
    for (int i = 0; i < 16; ++i) ids[i] = id_of((w >> (2 * i)) & 3u, 0);
  } else if (cd.width == 1) {
    const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(cd.ptr) + row0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) ids[i] = id_of((w[i >> 2] >> ((i & 3) * 8)) & 0xFFu, 1);
  } else if (cd.width == 2) {
    const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(cd.ptr) + row0);
    const uint4 a = p[0], b = p[1];
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) ids[i] = id_of((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu, 2);
  } else {
    const int4* p = reinterpret_cast<const int4*>(reinterpret_cast<const int32_t*>(cd.ptr) + row0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 v = p[q];
      ids[q * 4 + 0] = v.x; ids[q * 4 + 1] = v.y; ids[q * 4 + 2] = v.z; ids[q * 4 + 3] = v.w;
    }
  }
}

}  // namespace

// Raw code words of one 16-row group: 2-bit columns one dword, 1/2/4-byte columns 4/8/16.
template <int W>
struct GroupWords {
  static constexpr int n = W == 0 ? 1 : 4 * W;
};

template <int W>
__device__ __forceinline__ void load_words(const ColumnDesc& cd, int64_t row0, uint32_t (&w)[GroupWords<W>::n]) {
  const uint8_t* base = reinterpret_cast<const uint8_t*>(cd.ptr);
  if constexpr (W == 0) {
    w[0] = *reinterpret_cast<const uint32_t*>(base + (row0 >> 2));
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(base + row0 * W);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint4 v = p[q];
      w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
  }
}

template <int W, int N>
__device__ __forceinline__ uint32_t code_at(const uint32_t (&w)[N], int i) {
  if constexpr (W == 0) return (w[0] >> (2 * i)) & 3u;
  if constexpr (W == 1) return (w[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
  if constexpr (W == 2) return (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
  return w[i];
}

// 16-row mask of one leaf straight from the raw codes (no translation to ids: the all-ones
// missing code of a width is never a dictionary id, a bitmap bit or inside a rank range).
// EQ on 2-bit codes is SWAR over the whole dword: XOR with the replicated code, a zero pair
// marks a match, and the even bits are compacted to 16 bits.
template <int W, typename BitmapPtr>
__device__ __forceinline__ uint32_t leaf_bits(int32_t op, int32_t b, int32_t c, const uint32_t (&w)[GroupWords<W>::n],
                                              BitmapPtr bitmaps) {
  uint32_t m = 0;
  if (op == OP_EQ) {
    if constexpr (W == 0) {
      if ((uint32_t)b > 2u) return 0;
      const uint32_t x = w[0] ^ (0x55555555u * (uint32_t)b);
      uint32_t z = ~(x | (x >> 1)) & 0x55555555u;
      z = (z | (z >> 1)) & 0x33333333u;
      z = (z | (z >> 2)) & 0x0F0F0F0Fu;
      z = (z | (z >> 4)) & 0x00FF00FFu;
      return (z | (z >> 8)) & 0x0000FFFFu;
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) m |= (uint32_t)(code_at<W>(w, i) == (uint32_t)b) << i;
    }
  } else if (op == OP_RANGE) {  // b <= rank < c on a rank-encoded column
    const uint32_t span = (uint32_t)(c - b);
#pragma unroll
    for (int i = 0; i < 16; ++i) m |= (uint32_t)(code_at<W>(w, i) - (uint32_t)b < span) << i;
  } else {  // OP_LEAF: dictionary-id bitmap (register copy for <= 64 ids, else LDS / global words)
    const BitmapPtr bm = bitmaps + b;
    const uint32_t nbits = (uint32_t)c;
    if (nbits <= 64) {
      const uint64_t b64 = (uint64_t)bm[0] | ((nbits > 32) ? ((uint64_t)bm[1] << 32) : 0ull);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t r = code_at<W>(w, i);
        m |= (uint32_t)(r < nbits && ((b64 >> (r & 63u)) & 1ull)) << i;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t r = code_at<W>(w, i);
        m |= (uint32_t)(r < nbits && ((bm[r >> 5] >> (r & 31u)) & 1u)) << i;
      }
    }
  }
  return m;
}

// One leaf over the lane's U groups: all U loads first (U loads in flight), then the tests.
template <int W, int U, typename BitmapPtr>
__device__ __forceinline__ void leaf_groups(const ColumnDesc& cd, const int64_t (&row0)[U], int32_t op, int32_t b,
                                            int32_t c, BitmapPtr bitmaps, uint32_t (&m)[U]) {
  uint32_t w[U][GroupWords<W>::n];
#pragma unroll
  for (int u = 0; u < U; ++u) load_words<W>(cd, row0[u], w[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) m[u] = leaf_bits<W>(op, b, c, w[u], bitmaps);
}

// Evaluate the program for U independent 16-row groups at once: every leaf issues its U vector
// loads back to back, so each lane keeps U column loads in flight instead of one (the
// interpreted program otherwise serialises load -> test -> next leaf).
template <int U, typename BitmapPtr>
__device__ __forceinline__ void run_program(const ColumnDesc* __restrict__ cols, const int32_t* __restrict__ prog,
                                            int32_t prog_len, BitmapPtr bitmaps, const int64_t (&row0)[U],
                                            uint32_t (&out)[U]) {
  u128 st[U];
#pragma unroll
  for (int u = 0; u < U; ++u) st[u] = 0;
#pragma unroll 1
  for (int pc = 0; pc < prog_len; ++pc) {
    const int32_t op = prog[pc * 4 + 0];
    const int32_t a = prog[pc * 4 + 1];
    const int32_t b = prog[pc * 4 + 2];
    const int32_t c = prog[pc * 4 + 3];
    if (op == OP_RANGE || op == OP_LEAF || op == OP_EQ) {
      const ColumnDesc cd = cols[a];
      uint32_t m[U];
      switch (cd.width) {  // uniform per leaf: one code path per wave
        case 0: leaf_groups<0, U>(cd, row0, op, b, c, bitmaps, m); break;
        case 1: leaf_groups<1, U>(cd, row0, op, b, c, bitmaps, m); break;
        case 2: leaf_groups<2, U>(cd, row0, op, b, c, bitmaps, m); break;
        default: leaf_groups<4, U>(cd, row0, op, b, c, bitmaps, m); break;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st[u] = (st[u] << 16) | (u128)m[u];
    } else if (op == OP_AND || op == OP_OR) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint32_t r = (op == OP_AND) ? 0xFFFFu : 0u;
        for (int k = 0; k < a; ++k) {
          const uint32_t top = (uint32_t)(st[u] & (u128)0xFFFFu);
          r = (op == OP_AND) ? (r & top) : (r | top);
          st[u] >>= 16;
        }
        st[u] = (st[u] << 16) | (u128)r;
      }
    } else if (op == OP_NOT) {
#pragma unroll
      for (int u = 0; u < U; ++u) st[u] ^= (u128)0xFFFFu;
    } else {  // OP_TRUE
#pragma unroll
      for (int u = 0; u < U; ++u) st[u] = (st[u] << 16) | (u128)0xFFFFu;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) out[u] = (uint32_t)(st[u] & (u128)0xFFFFu);
}

