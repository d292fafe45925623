// Columnar predicate scan + order-preserving compaction for the state-store query engine
// (gfx950 / CDNA4, wave64).  Version 2: narrow columns, bit-sliced evaluation.
//
// Data model (built by ops/columnar.py): every queryable JSON path of a collection is a
// dictionary-encoded column of 2 bits (width code 0: dictionaries of <= 3 values -- booleans),
// 1, 2 or 4 bytes per row (width chosen from the dictionary size; the all-ones value of the
// width means "path missing"), plus a 1-bit liveness mask.  A 2-bit column packs 16 rows per
// 32-bit word, row r in bits 2(r mod 16) of word r / 16.
// A query filter (EQ/NEQ/IN/GT/GTE/LT/LTE/AND/OR of the Dapr state-query API) is compiled on
// the host into a postfix program whose leaves are "id of column c == v" or "id in bitmap
// S"; ordering/type semantics are resolved against the dictionary on the host, so the
// device only compares ids and tests bits.
//
// tt_scan_eval: each lane owns U groups of 16 consecutive rows (default 2; loads for all U in
// flight).  For every leaf it loads the 16 ids with
// one 16/32/64-byte vector load (width 1/2/4) and produces a 16-bit row mask; the program's
// stack holds 16-bit masks packed in a 128-bit register (depth <= 8), so AND/OR/NOT are
// plain bitwise ops on all 16 rows at once.  The lane ANDs the liveness bits and stores its
// 16-bit slice straight into the row-order selection mask (64 lanes x 2 B = one coalesced
// 128-B store); the block writes its selected count.  Traffic per row: sum of column
// widths + 1/8 B liveness + 1/8 B mask.
// tt_scan_compact: per 8192-row tile, 256 threads each take 32 mask bits, block-scan their
// popcounts (wave shuffles + LDS), stage the selected row indices in LDS and write them out
// contiguously (coalesced), at the tile's offset from the exclusive scan of block counts.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kBlock = 256;                    // 4 waves (compaction, group count)
constexpr int kRowsPerLane = 16;
constexpr int kTileRows = 8192;               // rows per scan / compaction block
constexpr int kChunkShift = 6;                // 64 tiles per chunk: per-chunk selected counts let a
                                              // compaction block find its offset with one wave
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

// NT: non-temporal loads (the columns are streamed once per query; A/B).
template <int W, bool NT = false>
__device__ __forceinline__ void load_words(const ColumnDesc& cd, int64_t row0, uint32_t (&w)[GroupWords<W>::n]) {
  const uint8_t* base = reinterpret_cast<const uint8_t*>(cd.ptr);
  if constexpr (W == 0) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (row0 >> 2));
    w[0] = NT ? __builtin_nontemporal_load(p) : *p;
  } else if constexpr (NT) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + row0 * W);
#pragma unroll
    for (int i = 0; i < 4 * W; ++i) w[i] = __builtin_nontemporal_load(p + i);
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
template <int W, int U, bool NT, typename BitmapPtr>
__device__ __forceinline__ void leaf_groups(const ColumnDesc& cd, const int64_t (&row0)[U], int32_t op, int32_t b,
                                            int32_t c, BitmapPtr bitmaps, uint32_t (&m)[U]) {
  uint32_t w[U][GroupWords<W>::n];
#pragma unroll
  for (int u = 0; u < U; ++u) load_words<W, NT>(cd, row0[u], w[u]);
#pragma unroll
  for (int u = 0; u < U; ++u) m[u] = leaf_bits<W>(op, b, c, w[u], bitmaps);
}

// Evaluate the program for U independent 16-row groups at once: every leaf issues its U vector
// loads back to back, so each lane keeps U column loads in flight instead of one (the
// interpreted program otherwise serialises load -> test -> next leaf).
template <int U, bool NT, typename BitmapPtr>
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
        case 0: leaf_groups<0, U, NT>(cd, row0, op, b, c, bitmaps, m); break;
        case 1: leaf_groups<1, U, NT>(cd, row0, op, b, c, bitmaps, m); break;
        case 2: leaf_groups<2, U, NT>(cd, row0, op, b, c, bitmaps, m); break;
        default: leaf_groups<4, U, NT>(cd, row0, op, b, c, bitmaps, m); break;
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

// One block per 8192-row tile; U = row groups per lane evaluated together (U x 16 rows per
// lane, 8192 / (16 U) threads per block).  U trades registers (occupancy) for loads in flight.
template <int U, bool NT>
__global__ void __launch_bounds__(kTileRows / (kRowsPerLane * U))
tt_scan_eval_t(const ColumnDesc* __restrict__ cols,
             int64_t nrows,
             const uint16_t* __restrict__ live,      // 1 bit per row, row order
             const int32_t* __restrict__ prog, int32_t prog_len,
             const uint32_t* __restrict__ bitmaps, int32_t bitmap_words,
             uint16_t* __restrict__ mask,            // 1 bit per row, row order
             int32_t* __restrict__ block_counts) {
  extern __shared__ uint32_t lds_bitmaps[];  // sized by the launcher: bitmap_words if they fit, else 0
  const bool in_lds = bitmap_words <= kMaxLdsBitmapWords;
  if (in_lds) {
    for (int i = threadIdx.x; i < bitmap_words; i += (kTileRows / (kRowsPerLane * U))) lds_bitmaps[i] = bitmaps[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  int64_t row0[U];
  uint16_t lv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    // group u covers rows [tile*8192 + u*2048, +2048): 16 per lane, lanes contiguous -> the
    // per-group mask stores of a wave form one 128-byte segment
    row0[u] = tile * kTileRows + (int64_t)u * ((kTileRows / (kRowsPerLane * U)) * kRowsPerLane) + (int64_t)threadIdx.x * kRowsPerLane;
    lv[u] = live[row0[u] >> 4];  // issued early, consumed after the program
  }
  uint32_t m[U];
  if (in_lds) run_program<U, NT>(cols, prog, prog_len, lds_bitmaps, row0, m);
  else run_program<U, NT>(cols, prog, prog_len, bitmaps, row0, m);
  int32_t local = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t sel = row0[u] < nrows ? (m[u] & (uint32_t)lv[u]) : 0u;
    mask[row0[u] >> 4] = (uint16_t)sel;  // the launched tiles are inside the buffers' capacity
    local += __popc(sel);
  }
  // block reduction of the per-lane counts
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  __shared__ int32_t wave_counts[(kTileRows / (kRowsPerLane * U)) / 64];
  if (lane == 0) wave_counts[wave] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int w = 0; w < (kTileRows / (kRowsPerLane * U)) / 64; ++w) s += wave_counts[w];
    block_counts[tile] = s;
  }
}

// ---------------------------------------------------------------------------------------
// tt_scan_flat: tt_scan_eval for FLAT programs -- one AND or OR over leaves, each optionally
// negated (the creator page, the overdue sweep, a single EQ: nearly every query the services
// issue) -- evaluated wave-wide instead of lane by lane.  Lane l owns rows 16l..16l+15 of a
// 1024-row chunk (one 16/32/64-byte load per lane per leaf); the test of row position p is
// ONE vector compare over the wave whose 64-bit result (bit l = row 16l+p) stays in scalar
// registers, where the leaves are combined with scalar logic.  Only the chunk's final result
// is turned back into per-lane bits (lane l: bit l of the 16 masks) -- the row-order 16-bit
// selection word of rows 16l..16l+15, i.e. exactly tt_scan_eval's mask layout, so compaction
// and grouped counts are shared.  Per row and leaf this is ~1/64 of a wave instruction (EQ)
// instead of the interpreter's per-lane extract / translate / compare / assemble sequence.
// Per chunk the column loads of up to four leaves are issued back to back before any compare,
// so a wave keeps all of them in flight.
//
// Leaf rows (host-built, int32 x4): {op | flip << 8, column, b, c} with op OP_EQ (code == b),
// OP_RANGE (b <= rank < c on a rank-encoded column) or OP_LEAF (bitmap words at b, c bits).
// Everything is evaluated as an AND: the host folds NOT and OR (De Morgan: flip every leaf,
// flip the result) into the flip bits and `flip_result`.
// Raw column codes are compared unsigned: the all-ones missing code of each width is never a
// dictionary id or rank (ColumnarIndex.width_for keeps dictionaries below it), so "missing"
// fails every leaf test without translating it to -1 first.
namespace {
constexpr int kFlatRows = 16;                 // rows per lane per chunk
constexpr int kFlatChunk = 64 * kFlatRows;    // 1024 rows per wave step
constexpr int kFlatChunksPerWave = kTileRows / kFlatChunk / (kBlock / 64);
constexpr int kMaxFlatLeaves = 8;
static_assert(kFlatChunksPerWave == 2, "a tile is 4 waves x 2 chunks");

// The lane's 16 rows of one column through a global (not flat) address (the column pointers
// arrive as integers; flat loads would also wait on the LDS counter).  N = 4 x the widest
// column of the program: always N/4 16-byte loads per leaf, a narrower column re-reading its
// first piece (an L2 hit, never past the column's end), so every leaf step issues the same
// number of loads and the compiler's wait counts stay exact across the pipelined loop.
// A 2-bit column needs one dword per lane (16 rows) and is read with the same 16-byte loads as
// the others (its device buffer carries 16 bytes of padding, ColumnarIndex.to_device); only
// w[0] is used.
template <int N>
__device__ __forceinline__ void issue_leaf_load(const ColumnDesc& cd, int64_t row0, uint32_t (&w)[N]) {
  const __attribute__((address_space(1))) uint32_t* p = reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(
      cd.ptr + (cd.width == 0 ? (uint64_t)row0 / 4 : (uint64_t)row0 * cd.width));
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const int qq = q < cd.width ? q : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[4 * q + i] = p[4 * qq + i];
  }
}

template <int W, int N>
__device__ __forceinline__ uint32_t raw_at(const uint32_t (&w)[N], int i) {
  if (W == 0) return (w[0] >> (2 * i)) & 3u;
  if (W == 1) return (w[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
  if (W == 2) return (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
  return w[i];
}

// acc[p] &= ballot(test(row 16 lane + p)) ^ flip, for one leaf over one chunk
template <int W, int N, typename BitmapPtr>
__device__ __forceinline__ void apply_leaf(int32_t op, uint32_t b, uint32_t c, uint64_t flip,
                                           const uint32_t (&w)[N], BitmapPtr bitmaps, uint64_t (&acc)[16]) {
  if (op == OP_EQ) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] &= __ballot(raw_at<W>(w, i) == b) ^ flip;
  } else if (op == OP_RANGE) {
    const uint32_t span = c - b;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] &= __ballot(raw_at<W>(w, i) - b < span) ^ flip;
  } else if (c <= 64) {  // bitmap leaf, dictionary of <= 64 ids: register-resident bitmap
    const BitmapPtr bm = bitmaps + b;
    const uint64_t b64 = (uint64_t)bm[0] | ((c > 32) ? ((uint64_t)bm[1] << 32) : 0ull);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t r = raw_at<W>(w, i);
      acc[i] &= __ballot(r < c && ((b64 >> (r & 63u)) & 1ull)) ^ flip;
    }
  } else {
    const BitmapPtr bm = bitmaps + b;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t r = raw_at<W>(w, i);
      acc[i] &= __ballot(r < c && ((bm[r >> 5] >> (r & 31u)) & 1u)) ^ flip;
    }
  }
}

template <int N, typename BitmapPtr>
__device__ __forceinline__ void flat_step(const int32_t* __restrict__ leaf, int width, const uint32_t (&w)[N],
                                          BitmapPtr bitmaps, uint64_t (&acc)[16]) {
  const int32_t op = leaf[0] & 0xFF;
  const uint64_t flip = (leaf[0] >> 8) ? ~0ull : 0ull;
  const uint32_t b = (uint32_t)leaf[2], c = (uint32_t)leaf[3];
  if (width == 0) apply_leaf<0>(op, b, c, flip, w, bitmaps, acc);
  else if (N == 4 || width == 1) apply_leaf<1>(op, b, c, flip, w, bitmaps, acc);
  else if (N == 8 || width == 2) apply_leaf<2>(op, b, c, flip, w, bitmaps, acc);
  else apply_leaf<4>(op, b, c, flip, w, bitmaps, acc);
}

// One wave's two chunks as a pipeline of (chunk, leaf) steps, chunk-major, with the column
// loads of the next two steps in flight while a step's compares run (three register buffers
// in rotation).  The liveness words are read up front and the two selection words stored at
// the end, so the loop body issues nothing but the leaf loads.
template <int N, typename BitmapPtr>
__device__ __forceinline__ void scan_flat_wave(const ColumnDesc* __restrict__ cols, int64_t nrows,
                                               const uint16_t* __restrict__ live, const int32_t* __restrict__ leaves,
                                               int32_t nleaves, uint32_t res_flip, BitmapPtr bitmaps,
                                               uint16_t* __restrict__ mask, int64_t wave_row0, int lane,
                                               int32_t& local) {
  static_assert(kFlatChunksPerWave == 2, "two selection words per lane");
  const int64_t r0 = wave_row0 + (int64_t)lane * kFlatRows, r1 = r0 + kFlatChunk;
  const uint32_t lv0 = live[r0 >> 4], lv1 = live[r1 >> 4];
  uint32_t sel0 = 0xFFFFu, sel1 = 0xFFFFu;
  uint64_t acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = ~0ull;
  const int steps = kFlatChunksPerWave * nleaves;
  auto issue = [&](int s, uint32_t (&w)[N]) {
    s = s < steps ? s : steps - 1;  // past the end: re-read the last step (keeps wait counts exact)
    const int j = s >= nleaves ? 1 : 0, k = s - j * nleaves;
    issue_leaf_load(cols[leaves[4 * k + 1]], j ? r1 : r0, w);
  };
  auto consume = [&](int s, const uint32_t (&w)[N]) {
    const int j = s >= nleaves ? 1 : 0, k = s - j * nleaves;
    flat_step(leaves + 4 * k, cols[leaves[4 * k + 1]].width, w, bitmaps, acc);
    if (k == nleaves - 1) {  // chunk done: back to per-lane bits (bit p = bit lane of acc[p])
      uint32_t bits = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) bits |= (uint32_t)((acc[i] >> lane) & 1ull) << i;
      if (j) sel1 = bits;
      else sel0 = bits;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = ~0ull;
    }
  };
  if (steps > 0) {
    uint32_t wa[N], wb[N], wc[N];
    issue(0, wa);
    issue(1, wb);
#pragma unroll 1
    for (int s = 0; s < steps; s += 3) {
      issue(s + 2, wc);
      consume(s, wa);
      if (s + 1 >= steps) break;
      issue(s + 3, wa);
      consume(s + 1, wb);
      if (s + 2 >= steps) break;
      issue(s + 4, wb);
      consume(s + 2, wc);
    }
  }
  const uint32_t m0 = r0 < nrows ? ((sel0 ^ res_flip) & lv0) : 0u;
  const uint32_t m1 = r1 < nrows ? ((sel1 ^ res_flip) & lv1) : 0u;
  mask[r0 >> 4] = (uint16_t)m0;
  mask[r1 >> 4] = (uint16_t)m1;
  local += __popc(m0) + __popc(m1);
}
}  // namespace

// N = 4 x the widest column the program reads (the launcher picks the instantiation)
template <int N>
__global__ void __launch_bounds__(kBlock)
tt_scan_flat_t(const ColumnDesc* __restrict__ cols, int64_t nrows, const uint16_t* __restrict__ live,
               const int32_t* __restrict__ leaves, int32_t nleaves, int32_t flip_result,
               const uint32_t* __restrict__ bitmaps, int32_t bitmap_words,
               uint16_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  extern __shared__ uint32_t lds_flat_bitmaps[];
  const bool in_lds = bitmap_words <= kMaxLdsBitmapWords;
  if (in_lds) {
    for (int i = threadIdx.x; i < bitmap_words; i += kBlock) lds_flat_bitmaps[i] = bitmaps[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint32_t res_flip = flip_result ? 0xFFFFu : 0u;
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  __shared__ int32_t wave_counts[2][kBlock / 64];
  // a bounded grid walks the tiles (grid-stride): fewer, longer-lived workgroups keep the
  // streams going instead of paying a dispatch and a ramp per 8192-row tile
  int parity = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, parity ^= 1) {
    const int64_t wave_row0 = tile * kTileRows + (int64_t)wave * kFlatChunksPerWave * kFlatChunk;
    int32_t local = 0;
    if (in_lds)
      scan_flat_wave<N>(cols, nrows, live, leaves, nleaves, res_flip, (const uint32_t*)lds_flat_bitmaps, mask,
                        wave_row0, lane, local);
    else
      scan_flat_wave<N>(cols, nrows, live, leaves, nleaves, res_flip, bitmaps, mask, wave_row0, lane, local);
    for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
    if (lane == 0) wave_counts[parity][wave] = local;  // double-buffered: one barrier per tile
    __syncthreads();
    if (threadIdx.x == 0)
      block_counts[tile] = wave_counts[parity][0] + wave_counts[parity][1] + wave_counts[parity][2] +
                           wave_counts[parity][3];
  }
}

// tt_chunk_sums: selected rows per 64-tile chunk -- one wave per chunk, one coalesced load per
// lane, a shuffle reduction; ~190 waves for 1e8 rows.  (Accumulating these with atomics in the
// scan kernel instead cost it 10-15 us at 1e8 rows; a "last block" ticket to reset them cost the
// compaction 35 -> 460 us: single-address atomics serialize across the 8 XCDs.)
extern "C" __global__ void __launch_bounds__(kBlock)
tt_chunk_sums(const int32_t* __restrict__ block_counts, int64_t tiles, int32_t* __restrict__ chunk_sums) {
  const int lane = threadIdx.x & 63;
  const int64_t chunk = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int64_t nchunks = (tiles + (1 << kChunkShift) - 1) >> kChunkShift;
  if (chunk >= nchunks) return;
  const int64_t j = (chunk << kChunkShift) + lane;
  int32_t v = j < tiles ? block_counts[j] : 0;
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if (lane == 0) chunk_sums[chunk] = v;
}

// Each compaction block finds its tile's output offset itself -- one wave sums the selected
// counts of the preceding chunks plus the preceding tiles of its own chunk -- so neither a
// full scan of the tile counts nor a host round trip sits between the scan and the
// compaction.  Block 0 also publishes the grand total: to `total` (device) and, when given,
// straight into pinned host memory (`total_host`, system-scope store), which the host reads
// after one event wait.
// NT: the row ids are written with non-temporal stores (streamed past the caches; A/B).
template <bool NT>
__global__ void __launch_bounds__(kBlock)
tt_scan_compact_t(const uint32_t* __restrict__ mask32,      // selection mask viewed as 32-bit words
                  const int32_t* __restrict__ block_counts,  // selected rows per tile
                  const int32_t* __restrict__ chunk_sums,    // selected rows per 64-tile chunk
                  int64_t tiles, int32_t* __restrict__ out, int64_t* __restrict__ total, int64_t* total_host) {
  __shared__ int32_t staged[kTileRows];
  __shared__ int32_t wave_sums[kBlock / 64];
  __shared__ int64_t tile_base;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int64_t tile = blockIdx.x;
  const uint32_t bits = mask32[tile * kBlock + t];     // rows [tile*8192 + 32t, +32)
  if (wave == 0) {
    const int64_t chunk = tile >> kChunkShift;
    int64_t s = 0;
    for (int64_t i = lane; i < chunk; i += 64) s += chunk_sums[i];
    const int64_t j = (chunk << kChunkShift) + lane;   // 64 tiles per chunk = one per lane
    if (j < tile) s += block_counts[j];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0) tile_base = s;
    if (tile == 0) {
      const int64_t nchunks = (tiles + (1 << kChunkShift) - 1) >> kChunkShift;
      int64_t g = 0;
      for (int64_t i = lane; i < nchunks; i += 64) g += chunk_sums[i];
      for (int off = 32; off > 0; off >>= 1) g += __shfl_down(g, off, 64);
      if (lane == 0) {
        *total = g;
        if (total_host) {
          __hip_atomic_store(total_host, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __threadfence_system();
        }
      }
    }
  }
  const int32_t cnt = __popc(bits);
  int32_t incl = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wave_sums[wave] = incl;
  __syncthreads();
  int32_t base = 0;
  for (int w = 0; w < wave; ++w) base += wave_sums[w];
  int32_t pos = base + incl - cnt;
  const int32_t count = wave_sums[0] + wave_sums[1] + wave_sums[2] + wave_sums[3];
  const int32_t row_base = (int32_t)(tile * kTileRows) + t * 32;
  uint32_t b = bits;
  while (b) {
    const int k = __ffs(b) - 1;
    staged[pos++] = row_base + k;
    b &= b - 1;
  }
  __syncthreads();
  int32_t* dst = out + tile_base;
  if constexpr (NT) {
    // 16-byte stores: a scalar head up to the first 16-byte aligned output slot, then each
    // thread writes 4 consecutive ids per store (4x fewer store instructions), a scalar tail
    const int head = (int)((4 - (tile_base & 3)) & 3) < count ? (int)((4 - (tile_base & 3)) & 3) : count;
    if (t < head) __builtin_nontemporal_store(staged[t], dst + t);
    const int body = (count - head) >> 2;
    typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
    i32x4* dst4 = reinterpret_cast<i32x4*>(dst + head);
    for (int q = t; q < body; q += kBlock) {
      const int i = head + 4 * q;
      i32x4 v = {staged[i], staged[i + 1], staged[i + 2], staged[i + 3]};
      __builtin_nontemporal_store(v, dst4 + q);
    }
    for (int i = head + 4 * body + t; i < count; i += kBlock) __builtin_nontemporal_store(staged[i], dst + i);
  } else {
    for (int i = t; i < count; i += kBlock) dst[i] = staged[i];
  }
}

// ---------------------------------------------------------------------------------------
// Wave-independent compaction (default).  tt_tile_offsets turns the per-tile counts into
// exclusive output offsets in ONE block (1024 threads x 16 tiles per pass with 16-byte loads and
// stores: 1e8 rows = 12.2k tiles is one pass) and publishes the total; tt_scan_compact_w then
// needs no block-level step: each wave of a tile owns 2048 rows, finds its base as
// tile_off[tile] + the popcounts of the preceding waves' mask words (L1 hits: the sibling waves
// load the same words), stages its ids in its own LDS slice and writes its segment with 16-byte
// stores.  No __syncthreads and no dependent chain through wave 0 (tt_scan_compact_t: one wave
// sums up to ~190 chunk counts while the other three wait at a barrier).
constexpr int kOffBlock = 1024;
constexpr int kOffPer = 16;

extern "C" __global__ void __launch_bounds__(kOffBlock)
tt_tile_offsets(const int32_t* __restrict__ block_counts, int64_t tiles, int32_t* __restrict__ tile_off,
                int64_t* __restrict__ total, int64_t* total_host) {
  typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
  __shared__ int32_t wsum[kOffBlock / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int64_t carry = 0;
  for (int64_t base = 0; base < tiles; base += (int64_t)kOffBlock * kOffPer) {
    const int64_t i0 = base + (int64_t)t * kOffPer;
    const bool full = i0 + kOffPer <= tiles;  // i0 is a multiple of 16: 64-byte aligned
    int32_t v[kOffPer];
    if (full) {
#pragma unroll
      for (int q = 0; q < kOffPer / 4; ++q) {
        const i32x4 x = reinterpret_cast<const i32x4*>(block_counts + i0)[q];
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kOffPer; ++k) v[k] = i0 + k < tiles ? block_counts[i0 + k] : 0;
    }
    int32_t s = 0;
#pragma unroll
    for (int k = 0; k < kOffPer; ++k) s += v[k];
    int32_t incl = s;
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kOffBlock / 64; ++w) {
      const int32_t x = wsum[w];
      before += w < wave ? x : 0;
      all += x;
    }
    int32_t o[kOffPer];
    int32_t run = (int32_t)carry + before + incl - s;  // ids are int32: every offset < 2^31
#pragma unroll
    for (int k = 0; k < kOffPer; ++k) {
      o[k] = run;
      run += v[k];
    }
    if (full) {
#pragma unroll
      for (int q = 0; q < kOffPer / 4; ++q)
        reinterpret_cast<i32x4*>(tile_off + i0)[q] = i32x4{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    } else {
#pragma unroll
      for (int k = 0; k < kOffPer; ++k)
        if (i0 + k < tiles) tile_off[i0 + k] = o[k];
    }
    carry += all;
    __syncthreads();  // wsum is rewritten by the next pass
  }
  if (t == 0) {
    *total = carry;
    if (total_host) {
      __hip_atomic_store(total_host, carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
    }
  }
}

template <bool NT>
__global__ void __launch_bounds__(kBlock)
tt_scan_compact_w(const uint32_t* __restrict__ mask32, const int32_t* __restrict__ tile_off,
                  int32_t* __restrict__ out) {
  __shared__ uint16_t staged[kBlock / 64][64 * 32];  // one slice per wave: row - wave_base (11 bits)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t tile = blockIdx.x;
  const uint32_t* m = mask32 + tile * kBlock;
  const int32_t tbase = tile_off[tile];
  const uint32_t bits = m[t];
  int32_t before = 0;  // selected rows of the tile's preceding waves
  for (int w = 0; w < wave; ++w) before += __popc(m[w * 64 + lane]);
  for (int off = 32; off > 0; off >>= 1) before += __shfl_xor(before, off, 64);
  const int32_t cnt = __popc(bits);
  int32_t incl = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  const int32_t count = __shfl(incl, 63, 64);
  uint16_t* st = staged[wave];
  int32_t pos = incl - cnt;
  const int32_t wave_base = (int32_t)(tile * kTileRows) + wave * 2048;
  const int lane_base = lane * 32;
  uint32_t b = bits;
  while (b) {
    const int k = __ffs(b) - 1;
    st[pos++] = (uint16_t)(lane_base + k);
    b &= b - 1;
  }
  // the slice is read back by other lanes of the same wave only
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int64_t a = (int64_t)tbase + before;
  int32_t* dst = out + a;
  int head = (int)((4 - (a & 3)) & 3);
  if (head > count) head = count;
  const int body = (count - head) >> 2;
  if constexpr (NT) {
    if (lane < head) __builtin_nontemporal_store(wave_base + st[lane], dst + lane);
    typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
    i32x4* dst4 = reinterpret_cast<i32x4*>(dst + head);
    for (int q = lane; q < body; q += 64) {
      const int i = head + 4 * q;
      i32x4 v = {wave_base + st[i], wave_base + st[i + 1], wave_base + st[i + 2], wave_base + st[i + 3]};
      __builtin_nontemporal_store(v, dst4 + q);
    }
    for (int i = head + 4 * body + lane; i < count; i += 64) __builtin_nontemporal_store(wave_base + st[i], dst + i);
  } else {
    for (int i = lane; i < count; i += 64) dst[i] = wave_base + st[i];
  }
}

// ---------------------------------------------------------------------------------------
// tt_scan_select: filter evaluation + order-preserving compaction in ONE pass (no selection
// mask round trip through HBM, no separate scan of tile counts, no host sync in between).
// Tiles are claimed through an atomic ticket, so every tile's predecessors have already
// started; each tile publishes its count (flag 1) and then its inclusive prefix (flag 2) in
// `status`, and finds its own offset by decoupled look-back over the predecessors' words
// (one wave reads 64 of them at a time).  The selection bits of the tile stay in LDS and are
// compacted exactly like tt_scan_compact.  The last tile writes the total.
namespace {
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagPrefix = 2ull << 62, kValueMask = (1ull << 62) - 1;
constexpr int kSelectBlock = 256;   // 4 waves: 2 row groups of 16 rows per lane for the scan,
                                    // 32 selection bits per thread for the compaction
static_assert(kSelectBlock * kRowsPerLane * 2 == kTileRows, "tile = 256 lanes x 2 groups x 16 rows");
static_assert(kSelectBlock * 32 == kTileRows, "compaction takes 32 bits per thread");

__device__ __forceinline__ uint64_t load_status(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_status(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

extern "C" __global__ void __launch_bounds__(kSelectBlock)
tt_scan_select(const ColumnDesc* __restrict__ cols, int64_t nrows, int64_t ntiles,
               const uint16_t* __restrict__ live, const int32_t* __restrict__ prog, int32_t prog_len,
               const uint32_t* __restrict__ bitmaps, int32_t bitmap_words,
               uint64_t* __restrict__ status,      // ntiles words, zeroed
               uint32_t* __restrict__ ticket,      // zeroed
               int32_t* __restrict__ out, int64_t* __restrict__ total) {
  extern __shared__ uint32_t lds_bitmaps[];
  __shared__ uint16_t sel_bits[kTileRows / 16];       // 1 KiB: the tile's selection
  __shared__ int32_t staged[kTileRows];               // 32 KiB: selected row ids, tile order
  __shared__ int32_t wave_sums[kSelectBlock / 64];
  __shared__ int64_t tile_s, offset_s;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) tile_s = (int64_t)atomicAdd(ticket, 1u);
  const bool in_lds = bitmap_words <= kMaxLdsBitmapWords;
  if (in_lds)
    for (int i = t; i < bitmap_words; i += kSelectBlock) lds_bitmaps[i] = bitmaps[i];
  __syncthreads();
  const int64_t tile = tile_s;
  // ---- evaluate: 2 groups of 16 rows per lane, all leaf loads of both groups in flight
  int64_t row0[2];
  uint16_t lv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    row0[u] = tile * kTileRows + (int64_t)u * (kSelectBlock * kRowsPerLane) + (int64_t)t * kRowsPerLane;
    lv[u] = live[row0[u] >> 4];
  }
  uint32_t m[2];
  if (in_lds) run_program<2, false>(cols, prog, prog_len, lds_bitmaps, row0, m);
  else run_program<2, false>(cols, prog, prog_len, bitmaps, row0, m);
  int32_t local = 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t sel = row0[u] < nrows ? (m[u] & (uint32_t)lv[u]) : 0u;
    sel_bits[u * kSelectBlock + t] = (uint16_t)sel;
    local += __popc(sel);
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if (lane == 0) wave_sums[wave] = local;
  __syncthreads();
  const int32_t count = wave_sums[0] + wave_sums[1] + wave_sums[2] + wave_sums[3];
  // ---- publish the aggregate, then look back for the exclusive prefix (wave 0)
  if (wave == 0) {
    if (lane == 0) store_status(&status[tile], (tile == 0 ? kFlagPrefix : kFlagAgg) | (uint64_t)count);
    int64_t exclusive = 0;
    int64_t j = tile - 1;
    while (j >= 0) {
      // lane l inspects predecessor j - l; spin until every inspected word carries a flag
      const int64_t idx = j - lane;
      uint64_t w = idx >= 0 ? load_status(&status[idx]) : kFlagPrefix;
      while (__any(w >> 62 == 0)) {
        if (w >> 62 == 0) w = load_status(&status[idx]);
      }
      // nearest lane (lowest l) holding an inclusive prefix ends the walk
      const uint64_t have_prefix = __ballot(w >> 62 == 2);
      const int stop = have_prefix ? __ffsll((unsigned long long)have_prefix) - 1 : 64;
      int64_t v = lane <= stop && lane < 64 ? (int64_t)(w & kValueMask) : 0;
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      exclusive += __shfl(v, 0, 64);
      if (have_prefix) break;
      j -= 64;
    }
    if (lane == 0) {
      if (tile != 0) store_status(&status[tile], kFlagPrefix | (uint64_t)(exclusive + count));
      offset_s = exclusive;
      if (tile == ntiles - 1) *total = exclusive + count;
    }
  }
  __syncthreads();
  // ---- compaction from the LDS selection bits (as tt_scan_compact)
  const uint32_t bits = (uint32_t)sel_bits[2 * t] | ((uint32_t)sel_bits[2 * t + 1] << 16);
  const int32_t cnt = __popc(bits);
  int32_t incl = cnt;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  __syncthreads();  // wave_sums reuse
  if (lane == 63) wave_sums[wave] = incl;
  __syncthreads();
  int32_t base = 0;
  for (int w = 0; w < wave; ++w) base += wave_sums[w];
  int32_t pos = base + incl - cnt;
  const int32_t row_base = (int32_t)(tile * kTileRows) + t * 32;
  uint32_t b = bits;
  while (b) {
    const int k = __ffs(b) - 1;
    staged[pos++] = row_base + k;
    b &= b - 1;
  }
  __syncthreads();
  int32_t* dst = out + offset_s;
  for (int i = t; i < count; i += kSelectBlock) dst[i] = staged[i];
}

// Rank encoding of one column for range leaves: dst[row] = rank_table[id] (sort rank of the
// dictionary value, 1-based), the all-ones missing code where the path is missing.  Rank
// table staged in LDS when it fits.  Rows [lo, hi): the 16-aligned body is done 16 rows per
// thread with one 16/32/64-byte load and store per thread (a full re-encode of 1e8 rows is a
// streaming pass), the unaligned head and tail row by row.
namespace {
__device__ __forceinline__ int32_t rank_of(int32_t id, const int32_t* lds_rank, const int32_t* rank_table,
                                           int32_t nranks, bool staged) {
  return (id >= 0 && id < nranks) ? (staged ? lds_rank[id] : rank_table[id]) : -1;
}

__device__ __forceinline__ void store_rank(uint64_t dst_ptr, int32_t dst_width, int64_t row, int32_t r) {
  if (dst_width == 1) reinterpret_cast<uint8_t*>(dst_ptr)[row] = (uint8_t)(r < 0 ? 0xFF : r);
  else if (dst_width == 2) reinterpret_cast<uint16_t*>(dst_ptr)[row] = (uint16_t)(r < 0 ? 0xFFFF : r);
  else reinterpret_cast<int32_t*>(dst_ptr)[row] = r;
}
}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock)
tt_rank_encode(const ColumnDesc* __restrict__ src, const int32_t* __restrict__ rank_table, int32_t nranks,
               int64_t lo, int64_t hi, uint64_t dst_ptr, int32_t dst_width) {
  extern __shared__ int32_t lds_rank[];
  const bool staged = nranks <= 8192;
  if (staged)
    for (int i = threadIdx.x; i < nranks; i += kBlock) lds_rank[i] = rank_table[i];
  __syncthreads();
  const ColumnDesc cd = *src;
  const int64_t a = (lo + 15) & ~(int64_t)15, b = hi & ~(int64_t)15;  // aligned body [a, b)
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  auto one = [&](int64_t row) {
    uint32_t raw;
    if (cd.width == 0) raw = (reinterpret_cast<const uint8_t*>(cd.ptr)[row >> 2] >> ((row & 3) * 2)) & 3u;
    else if (cd.width == 1) raw = reinterpret_cast<const uint8_t*>(cd.ptr)[row];
    else if (cd.width == 2) raw = reinterpret_cast<const uint16_t*>(cd.ptr)[row];
    else raw = reinterpret_cast<const uint32_t*>(cd.ptr)[row];
    store_rank(dst_ptr, dst_width, row, rank_of(id_of(raw, cd.width), lds_rank, rank_table, nranks, staged));
  };
  if (a >= b) {  // short range: row by row
    for (int64_t row = lo + tid; row < hi; row += stride) one(row);
    return;
  }
  for (int64_t row = lo + tid; row < a; row += stride) one(row);
  for (int64_t row = b + tid; row < hi; row += stride) one(row);
  for (int64_t g = a / 16 + tid; g < b / 16; g += stride) {
    int32_t ids[16];
    load16(cd, g * 16, ids);
    int32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = rank_of(ids[i], lds_rank, rank_table, nranks, staged);
    if (dst_width == 1) {
      uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i >> 2] |= (uint32_t)(r[i] < 0 ? 0xFF : r[i] & 0xFF) << ((i & 3) * 8);
      reinterpret_cast<uint4*>(dst_ptr)[g] = make_uint4(w[0], w[1], w[2], w[3]);
    } else if (dst_width == 2) {
      uint32_t w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        w[i] = (uint32_t)(r[2 * i] < 0 ? 0xFFFF : r[2 * i] & 0xFFFF) |
               ((uint32_t)(r[2 * i + 1] < 0 ? 0xFFFF : r[2 * i + 1] & 0xFFFF) << 16);
      uint4* d = reinterpret_cast<uint4*>(dst_ptr) + g * 2;
      d[0] = make_uint4(w[0], w[1], w[2], w[3]);
      d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
      int4* d = reinterpret_cast<int4*>(dst_ptr) + g * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = make_int4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    }
  }
}

// Grouped count: histogram of column `g` dictionary ids over the selected rows (the
// "open tasks per assignee" dashboard aggregate).  LDS-privatised counters for dictionaries
// up to 8192 entries, global atomics otherwise.
extern "C" __global__ void __launch_bounds__(kBlock)
tt_group_count(const ColumnDesc* __restrict__ cols, int32_t g, const uint16_t* __restrict__ mask, int64_t nrows,
               int32_t ngroups, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t hist[];
  const bool use_lds = ngroups <= 8192;
  if (use_lds)
    for (int i = threadIdx.x; i < ngroups; i += kBlock) hist[i] = 0;
  __syncthreads();
  const ColumnDesc cd = cols[g];
  const int64_t nslices = (nrows + 15) / 16;
  for (int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x; s < nslices; s += (int64_t)gridDim.x * kBlock) {
    uint32_t m = mask[s];
    if (!m) continue;
    int32_t ids[16];
    load16(cd, s * 16, ids);
    while (m) {
      const int k = __ffs(m) - 1;
      m &= m - 1;
      const int32_t id = ids[k];
      if (id >= 0 && id < ngroups) {
        if (use_lds) atomicAdd(&hist[id], 1u);
        else atomicAdd(&counts[id], 1u);
      }
    }
  }
  __syncthreads();
  if (use_lds)
    for (int i = threadIdx.x; i < ngroups; i += kBlock)
      if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

// ------------------------------------------------------------------ host launchers
// Non-temporal column loads in the scan (A/B; default off).
static int g_eval_nt = 0;
extern "C" int tt_set_eval_nt(int on) {
  g_eval_nt = on ? 1 : 0;
  return 0;
}

// Row groups per lane of the scan kernel (1, 2, 4 or 8); tunable for A/B measurements.
static int g_eval_groups = 2;  // measured on MI355X: 1 -> 0.183 ms, 2 -> 0.175 ms, 4 -> 0.194 ms per 1e8-row query
extern "C" int tt_set_eval_groups(int u) {
  if (u != 1 && u != 2 && u != 4 && u != 8) return -1;
  g_eval_groups = u;
  return 0;
}

// Preconditions (checked by the Python wrapper): every column and the live/mask buffers are
// allocated for a capacity that is a multiple of kTileRows rows, nrows <= capacity.
extern "C" int tt_launch_scan_eval(const void* cols, int64_t nrows, const uint16_t* live, const int32_t* prog,
                                   int32_t prog_len, const uint32_t* bitmaps, int32_t bitmap_words, uint16_t* mask,
                                   int32_t* block_counts, hipStream_t stream) {
  if (prog_len <= 0 || nrows < 0 || bitmap_words <= 0) return -1;
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  const size_t lds = bitmap_words <= kMaxLdsBitmapWords ? (size_t)bitmap_words * sizeof(uint32_t) : 0;
  const ColumnDesc* cd = reinterpret_cast<const ColumnDesc*>(cols);
  if (g_eval_nt) {
    switch (g_eval_groups) {
#define TT_EVAL_CASE(UU)                                                                                    \
  case UU:                                                                                                   \
    hipLaunchKernelGGL((tt_scan_eval_t<UU, true>), dim3((unsigned)tiles), dim3(kTileRows / (kRowsPerLane * UU)), \
                       lds, stream, cd, nrows, live, prog, prog_len, bitmaps, bitmap_words, mask, block_counts);    \
    break;
      TT_EVAL_CASE(1) TT_EVAL_CASE(4) TT_EVAL_CASE(8)
      default: TT_EVAL_CASE(2)
#undef TT_EVAL_CASE
    }
  } else {
    switch (g_eval_groups) {
#define TT_EVAL_CASE(UU)                                                                                     \
  case UU:                                                                                                    \
    hipLaunchKernelGGL((tt_scan_eval_t<UU, false>), dim3((unsigned)tiles), dim3(kTileRows / (kRowsPerLane * UU)), \
                       lds, stream, cd, nrows, live, prog, prog_len, bitmaps, bitmap_words, mask, block_counts);     \
    break;
      TT_EVAL_CASE(1) TT_EVAL_CASE(4) TT_EVAL_CASE(8)
      default: TT_EVAL_CASE(2)
#undef TT_EVAL_CASE
    }
  }
  return (int)hipGetLastError();
}

// Workgroups of the flat scan (grid-stride over tiles); 0 = one per tile.  Tunable for A/B.
static int64_t g_flat_grid = (int64_t)1 << 40;  // measured: one per tile 0.164 ms, 2048 0.171 ms
extern "C" int tt_set_flat_grid(int64_t g) {
  if (g < 0) return -1;
  g_flat_grid = g == 0 ? (int64_t)1 << 40 : g;
  return 0;
}

// Flat programs (see tt_scan_flat_t): `leaves` is int32 [nleaves, 4] on the device and
// `max_width` the widest column (1, 2 or 4 bytes) any leaf reads.
extern "C" int tt_launch_scan_flat(const void* cols, int64_t nrows, const uint16_t* live, const int32_t* leaves,
                                   int32_t nleaves, int32_t flip_result, int32_t max_width, const uint32_t* bitmaps,
                                   int32_t bitmap_words, uint16_t* mask, int32_t* block_counts, hipStream_t stream) {
  if (nleaves < 0 || nleaves > kMaxFlatLeaves || nrows < 0 || bitmap_words <= 0) return -1;
  if (max_width != 1 && max_width != 2 && max_width != 4) return -1;
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  const size_t lds = bitmap_words <= kMaxLdsBitmapWords ? (size_t)bitmap_words * sizeof(uint32_t) : 0;
  const ColumnDesc* cd = reinterpret_cast<const ColumnDesc*>(cols);
  const unsigned grid = (unsigned)(tiles < g_flat_grid ? tiles : g_flat_grid);
  if (max_width == 1)
    hipLaunchKernelGGL(tt_scan_flat_t<4>, dim3(grid), dim3(kBlock), lds, stream, cd, nrows, live, leaves,
                       nleaves, flip_result, bitmaps, bitmap_words, mask, block_counts);
  else if (max_width == 2)
    hipLaunchKernelGGL(tt_scan_flat_t<8>, dim3(grid), dim3(kBlock), lds, stream, cd, nrows, live, leaves,
                       nleaves, flip_result, bitmaps, bitmap_words, mask, block_counts);
  else
    hipLaunchKernelGGL(tt_scan_flat_t<16>, dim3(grid), dim3(kBlock), lds, stream, cd, nrows, live, leaves,
                       nleaves, flip_result, bitmaps, bitmap_words, mask, block_counts);
  return (int)hipGetLastError();
}

extern "C" int tt_max_flat_leaves() { return kMaxFlatLeaves; }

// Non-temporal stores for the compacted row ids: measured on MI355X (1e8 rows, 31.5M selected)
// 0.1215 -> 0.111 ms per query -- the ids stream past L2, and the next scan keeps its cache.
static int g_compact_nt = 1;
extern "C" int tt_set_compact_nt(int on) {
  g_compact_nt = on ? 1 : 0;
  return 0;
}

// Compaction variant (A/B): 1 = tt_tile_offsets + tt_scan_compact_w (default), 0 = chunk sums +
// tt_scan_compact_t (wave 0 of each block finds the block's offset).
static int g_compact_mode = 1;
extern "C" int tt_set_compact_mode(int mode) {
  if (mode != 0 && mode != 1) return 1;
  g_compact_mode = mode;
  return 0;
}

// `chunk_sums`: 16-byte aligned scratch for `tiles` int32 (mode 1: the tiles' output offsets;
// mode 0: the ceil(tiles / 64) chunk counts); `out` holds up to nrows ids; the selected count
// lands in `total` (device) and `total_host` (pinned host memory, optional).
extern "C" int tt_launch_scan_compact(const uint16_t* mask, const int32_t* block_counts, int32_t* chunk_sums,
                                      int64_t nrows, int32_t* out, int64_t* total, int64_t* total_host,
                                      hipStream_t stream) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  if (g_compact_mode == 1) {  // tile offsets in one block, then wave-independent compaction
    hipLaunchKernelGGL(tt_tile_offsets, dim3(1), dim3(kOffBlock), 0, stream, block_counts, tiles, chunk_sums, total,
                       total_host);
    if (g_compact_nt)
      hipLaunchKernelGGL(tt_scan_compact_w<true>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                         reinterpret_cast<const uint32_t*>(mask), chunk_sums, out);
    else
      hipLaunchKernelGGL(tt_scan_compact_w<false>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                         reinterpret_cast<const uint32_t*>(mask), chunk_sums, out);
    return (int)hipGetLastError();
  }
  const int64_t nchunks = (tiles + (1 << kChunkShift) - 1) >> kChunkShift;
  hipLaunchKernelGGL(tt_chunk_sums, dim3((unsigned)((nchunks + kBlock / 64 - 1) / (kBlock / 64))), dim3(kBlock), 0,
                     stream, block_counts, tiles, chunk_sums);
  if (g_compact_nt)
    hipLaunchKernelGGL(tt_scan_compact_t<true>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                       reinterpret_cast<const uint32_t*>(mask), block_counts, chunk_sums, tiles, out, total, total_host);
  else
    hipLaunchKernelGGL(tt_scan_compact_t<false>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                       reinterpret_cast<const uint32_t*>(mask), block_counts, chunk_sums, tiles, out, total, total_host);
  return (int)hipGetLastError();
}
extern "C" int tt_chunk_tiles() { return 1 << kChunkShift; }

// `status` (ntiles uint64) and `ticket` must be zeroed; `out` holds up to nrows ids; the
// selected count lands in `total` (device int64).
extern "C" int tt_launch_scan_select(const void* cols, int64_t nrows, const uint16_t* live, const int32_t* prog,
                                     int32_t prog_len, const uint32_t* bitmaps, int32_t bitmap_words, uint64_t* status,
                                     uint32_t* ticket, int32_t* out, int64_t* total, hipStream_t stream) {
  if (prog_len <= 0 || nrows < 0 || bitmap_words <= 0) return -1;
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  const size_t lds = bitmap_words <= kMaxLdsBitmapWords ? (size_t)bitmap_words * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(tt_scan_select, dim3((unsigned)tiles), dim3(kSelectBlock), lds, stream,
                     reinterpret_cast<const ColumnDesc*>(cols), nrows, tiles, live, prog, prog_len, bitmaps,
                     bitmap_words, status, ticket, out, total);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_group_count(const void* cols, int32_t g, const uint16_t* mask, int64_t nrows, int32_t ngroups,
                                     uint32_t* counts, hipStream_t stream) {
  if (ngroups <= 0) return -1;
  const int64_t nslices = (nrows + 15) / 16;
  int64_t blocks = (nslices + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  if (blocks == 0) return 0;
  const size_t lds = ngroups <= 8192 ? (size_t)ngroups * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(tt_group_count, dim3((unsigned)blocks), dim3(kBlock), lds, stream,
                     reinterpret_cast<const ColumnDesc*>(cols), g, mask, nrows, ngroups, counts);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_rank_encode(const void* src, const int32_t* rank_table, int32_t nranks, int64_t lo, int64_t hi,
                                     void* dst, int32_t dst_width, hipStream_t stream) {
  if (hi <= lo) return 0;
  if (nranks < 0 || (dst_width != 1 && dst_width != 2 && dst_width != 4)) return -1;
  int64_t blocks = ((hi - lo + 15) / 16 + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  const size_t lds = nranks <= 8192 ? (size_t)nranks * sizeof(int32_t) : 0;
  hipLaunchKernelGGL(tt_rank_encode, dim3((unsigned)blocks), dim3(kBlock), lds, stream,
                     reinterpret_cast<const ColumnDesc*>(src), rank_table, nranks, lo, hi, (uint64_t)dst, dst_width);
  return (int)hipGetLastError();
}

extern "C" int tt_tile_rows() { return kTileRows; }
extern "C" int tt_max_depth() { return kMaxDepth; }
