// Columnar predicate scan + order-preserving compaction for the state-store query engine
// (gfx950 / CDNA4, wave64).
//
// Data model (built by ops/columnar.py): every queryable JSON path of a collection is a
// dictionary-encoded int32 column (one id per document row); row liveness is column 0
// semantics-free: tombstoned rows carry id -1 in the `live` column.  A query filter
// (EQ/NEQ/IN/GT/GTE/LT/LTE/AND/OR of the Dapr state-query API) is compiled on the host into
// a tiny postfix program whose leaves are "id of column c is in dictionary-id set S"; S is
// a bitmap over the column's dictionary, so every comparison semantics (typed equality,
// range order) is resolved exactly on the host against the dictionary and the device only
// does bit tests.
//
// Kernel 1 (tt_scan_eval): each lane evaluates the program for 4 consecutive rows loaded
// as one int4 per referenced column (16 B/lane, 1 KiB per wave-instruction), the wave
// forms 4 ballots and re-interleaves them into four 64-bit row-order mask words
// (bit r of word w = row 64w + r), and the block writes its popcount.  Memory-bound: one
// read of each referenced column + N/8 bytes of mask.
// Kernel 2 (tt_scan_compact): per 4096-row tile, exclusive-scan the 64 word popcounts in
// LDS, add the tile's global offset (exclusive scan of block counts), and each lane writes
// its row index if its bit is set -- output is in row (= insertion) order, deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kBlock = 256;              // 4 waves
constexpr int kRowsPerLane = 4;          // one int4 load per column
constexpr int kIters = 4;                // 256 lanes * 4 rows * 4 iters = 4096 rows per block
constexpr int kTileRows = kBlock * kRowsPerLane * kIters;
constexpr int kWordsPerTile = kTileRows / 64;

enum Op : int32_t { OP_LEAF = 1, OP_AND = 2, OP_OR = 3, OP_NOT = 4, OP_TRUE = 5, OP_EQ = 6 };

// Program layout (int32): [op, a, b, c] quads.
//   OP_LEAF col bitmap_word_offset nbits : push(id in [0,nbits) && bitmap[id])
//   OP_EQ   col id            -          : push(colval == id)
//   OP_AND  n                            : pop n, push AND
//   OP_OR   n                            : pop n, push OR
//   OP_NOT                               : invert top
//   OP_TRUE                              : push 1
// The stack is a uint32 per row (depth <= 32, enforced by the compiler on the host).

__device__ __forceinline__ uint64_t spread4(uint64_t x) {
  x &= 0xFFFFull;
  x = (x | (x << 24)) & 0x000000FF000000FFull;
  x = (x | (x << 12)) & 0x000F000F000F000Full;
  x = (x | (x << 6)) & 0x0303030303030303ull;
  x = (x | (x << 3)) & 0x1111111111111111ull;
  return x;
}

__device__ __forceinline__ uint32_t bit_of(const uint32_t* __restrict__ bm, int32_t id, int32_t nbits) {
  return (id >= 0 && id < nbits) ? ((bm[id >> 5] >> (id & 31)) & 1u) : 0u;
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock)
tt_scan_eval(const int32_t* __restrict__ cols,      // [ncols, stride] dictionary ids, -1 = missing
             int64_t stride,                         // row capacity per column (multiple of 4096)
             int64_t nrows,
             const int32_t* __restrict__ live,       // [stride] 1 = live row, 0 = tombstone / padding
             const int32_t* __restrict__ prog, int32_t prog_len,
             const uint32_t* __restrict__ bitmaps,
             uint64_t* __restrict__ mask,            // [stride/64]
             int32_t* __restrict__ block_counts) {   // [stride/4096]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  int32_t local = 0;
  for (int it = 0; it < kIters; ++it) {
    // rows handled by this lane: 4 consecutive rows
    const int64_t wave_base = tile * kTileRows + (int64_t)it * (kBlock * kRowsPerLane) + wave * 256;
    const int64_t row0 = wave_base + lane * 4;
    uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;  // per-row bool stacks
    if (row0 < nrows) {
      const int4 lv = *reinterpret_cast<const int4*>(live + row0);
      for (int pc = 0; pc < prog_len; ++pc) {
        const int32_t op = prog[pc * 4 + 0];
        const int32_t a = prog[pc * 4 + 1];
        const int32_t b = prog[pc * 4 + 2];
        const int32_t c = prog[pc * 4 + 3];
        if (op == OP_LEAF || op == OP_EQ) {
          const int4 v = *reinterpret_cast<const int4*>(cols + (int64_t)a * stride + row0);
          uint32_t r0, r1, r2, r3;
          if (op == OP_EQ) {
            r0 = v.x == b; r1 = v.y == b; r2 = v.z == b; r3 = v.w == b;
          } else {
            const uint32_t* bm = bitmaps + b;
            r0 = bit_of(bm, v.x, c); r1 = bit_of(bm, v.y, c); r2 = bit_of(bm, v.z, c); r3 = bit_of(bm, v.w, c);
          }
          st0 = (st0 << 1) | r0; st1 = (st1 << 1) | r1; st2 = (st2 << 1) | r2; st3 = (st3 << 1) | r3;
        } else if (op == OP_AND || op == OP_OR) {
          const uint32_t m = (a >= 32) ? 0xFFFFFFFFu : ((1u << a) - 1u);
          if (op == OP_AND) {
            st0 = (st0 >> a << 1) | ((st0 & m) == m); st1 = (st1 >> a << 1) | ((st1 & m) == m);
            st2 = (st2 >> a << 1) | ((st2 & m) == m); st3 = (st3 >> a << 1) | ((st3 & m) == m);
          } else {
            st0 = (st0 >> a << 1) | ((st0 & m) != 0); st1 = (st1 >> a << 1) | ((st1 & m) != 0);
            st2 = (st2 >> a << 1) | ((st2 & m) != 0); st3 = (st3 >> a << 1) | ((st3 & m) != 0);
          }
        } else if (op == OP_NOT) {
          st0 ^= 1u; st1 ^= 1u; st2 ^= 1u; st3 ^= 1u;
        } else {  // OP_TRUE
          st0 = (st0 << 1) | 1u; st1 = (st1 << 1) | 1u; st2 = (st2 << 1) | 1u; st3 = (st3 << 1) | 1u;
        }
      }
      st0 &= (lv.x != 0); st1 &= (lv.y != 0); st2 &= (lv.z != 0); st3 &= (lv.w != 0);
      // rows past nrows inside the last int4 are padding with live == 0
    }
    const uint64_t b0 = __ballot(st0 & 1u);
    const uint64_t b1 = __ballot(st1 & 1u);
    const uint64_t b2 = __ballot(st2 & 1u);
    const uint64_t b3 = __ballot(st3 & 1u);
    if (lane < 4) {
      const int sh = lane * 16;
      const uint64_t w = spread4(b0 >> sh) | (spread4(b1 >> sh) << 1) | (spread4(b2 >> sh) << 2) | (spread4(b3 >> sh) << 3);
      mask[wave_base / 64 + lane] = w;
    }
    if (lane == 0) local += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
  }
  __shared__ int32_t wave_counts[kBlock / 64];
  if (lane == 0) wave_counts[wave] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += wave_counts[w];
    block_counts[tile] = s;
  }
}

extern "C" __global__ void __launch_bounds__(kBlock)
tt_scan_compact(const uint64_t* __restrict__ mask,
                const int64_t* __restrict__ block_offsets,  // exclusive scan of block_counts
                int32_t* __restrict__ out) {
  __shared__ int32_t word_prefix[kWordsPerTile];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  const uint64_t* m = mask + tile * kWordsPerTile;
  if (wave == 0) {
    // inclusive scan of the 64 word popcounts across the wave, then make it exclusive
    const int32_t pc = __popcll(m[lane]);
    int32_t v = pc;
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t y = __shfl_up(v, off, 64);
      if (lane >= off) v += y;
    }
    word_prefix[lane] = v - pc;
  }
  __syncthreads();
  const int64_t base_out = block_offsets[tile];
  for (int i = 0; i < kWordsPerTile / (kBlock / 64); ++i) {
    const int w = wave * (kWordsPerTile / (kBlock / 64)) + i;
    const uint64_t word = m[w];
    if ((word >> lane) & 1ull) {
      const uint64_t below = lane ? (word & ((1ull << lane) - 1ull)) : 0ull;
      out[base_out + word_prefix[w] + __popcll(below)] = (int32_t)(tile * kTileRows + (int64_t)w * 64 + lane);
    }
  }
}

// Grouped count: histogram of column `gcol` dictionary ids over the rows selected in
// `mask` (the "tasks per assignee / per creator" dashboard aggregate).  LDS-privatised
// counters for small dictionaries, global atomics otherwise.
extern "C" __global__ void __launch_bounds__(kBlock)
tt_group_count(const int32_t* __restrict__ gcol, const uint64_t* __restrict__ mask, int64_t nwords,
               int32_t ngroups, uint32_t* __restrict__ counts) {
  extern __shared__ uint32_t hist[];
  const bool use_lds = ngroups <= 8192;
  if (use_lds)
    for (int i = threadIdx.x; i < ngroups; i += kBlock) hist[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (int64_t w = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); w < nwords;
       w += (int64_t)gridDim.x * (kBlock / 64)) {
    const uint64_t word = mask[w];
    if ((word >> lane) & 1ull) {
      const int32_t g = gcol[w * 64 + lane];
      if (g >= 0 && g < ngroups) {
        if (use_lds) atomicAdd(&hist[g], 1u);
        else atomicAdd(&counts[g], 1u);
      }
    }
  }
  __syncthreads();
  if (use_lds)
    for (int i = threadIdx.x; i < ngroups; i += kBlock)
      if (hist[i]) atomicAdd(&counts[i], hist[i]);
}

// ------------------------------------------------------------------ host launchers
extern "C" int tt_launch_scan_eval(const int32_t* cols, int64_t stride, int64_t nrows, const int32_t* live,
                                   const int32_t* prog, int32_t prog_len, const uint32_t* bitmaps, uint64_t* mask,
                                   int32_t* block_counts, hipStream_t stream) {
  if (stride % kTileRows != 0 || nrows > stride || prog_len <= 0) return -1;
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(tt_scan_eval, dim3((unsigned)tiles), dim3(kBlock), 0, stream, cols, stride, nrows, live, prog,
                     prog_len, bitmaps, mask, block_counts);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_scan_compact(const uint64_t* mask, const int64_t* block_offsets, int64_t nrows,
                                      int32_t* out, hipStream_t stream) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(tt_scan_compact, dim3((unsigned)tiles), dim3(kBlock), 0, stream, mask, block_offsets, out);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_group_count(const int32_t* gcol, const uint64_t* mask, int64_t nrows, int32_t ngroups,
                                     uint32_t* counts, hipStream_t stream) {
  if (ngroups <= 0) return -1;
  const int64_t nwords = (nrows + 63) / 64;
  int64_t blocks = (nwords + (kBlock / 64) - 1) / (kBlock / 64);
  if (blocks > 2048) blocks = 2048;
  const size_t lds = ngroups <= 8192 ? (size_t)ngroups * sizeof(uint32_t) : 0;
  hipLaunchKernelGGL(tt_group_count, dim3((unsigned)blocks), dim3(kBlock), lds, stream, gcol, mask, nwords, ngroups,
                     counts);
  return (int)hipGetLastError();
}

extern "C" int tt_tile_rows() { return kTileRows; }
