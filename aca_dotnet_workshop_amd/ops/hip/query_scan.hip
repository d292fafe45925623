// Columnar predicate scan + order-preserving compaction for the state-store query engine
// (gfx950 / CDNA4, wave64).  Narrow columns, bit-sliced evaluation.
//
// Data model (built by ops/columnar.py): every queryable JSON path of a collection is a
// dictionary-encoded column of 2 bits (width code 0: dictionaries of <= 3 values -- booleans),
// 1, 2 or 4 bytes per row (width chosen from the dictionary size; the all-ones value of the
// width means "path missing"), plus a 1-bit liveness mask.  A 2-bit column packs 16 rows per
// 32-bit word, row r in bits 2(r mod 16) of word r / 16.
// A query filter (EQ/NEQ/IN/GT/GTE/LT/LTE/AND/OR of the Dapr state-query API) is compiled on
// the host into a postfix program whose leaves are "id of column c == v" or "id in bitmap
// S"; ordering/type semantics are resolved against the dictionary on the host, so the
// device only compares ids and tests bits (scan_common.h).
//
// tt_scan_eval: each lane owns U groups of 16 consecutive rows (default 2; loads for all U in
// flight).  For every leaf it loads the 16 ids with one 16/32/64-byte vector load (width
// 1/2/4) and produces a 16-bit row mask; the program's stack holds 16-bit masks packed in a
// 128-bit register (depth <= 8), so AND/OR/NOT are plain bitwise ops on all 16 rows at once.
// The lane ANDs the liveness bits and stores its 16-bit slice straight into the row-order
// selection mask (64 lanes x 2 B = one coalesced 128-B store); the block writes its selected
// count.  Traffic per row: sum of column widths + 1/8 B liveness + 1/8 B mask.
// tt_tile_offsets + tt_scan_compact_w: the tiles' output offsets in one block, then a
// wave-independent compaction of the selected row ids (non-temporal 16-byte stores).
//
// Paged queries do not come through here: page_topk.hip evaluates only the tiles that can hold
// the page.  Variants that lost their A/B measurements (single-pass decoupled look-back select,
// wave-wide flat evaluator, chunk-sum compaction, non-temporal column loads) were removed in
// round 3; their records stay in profiles/r1_query_scan_*.md.
#include "scan_common.h"

// One block per 8192-row tile; U = row groups per lane evaluated together (U x 16 rows per
// lane, 8192 / (16 U) threads per block).  U trades registers (occupancy) for loads in flight.
template <int U>
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
  if (in_lds) run_program<U>(cols, prog, prog_len, lds_bitmaps, row0, m);
  else run_program<U>(cols, prog, prog_len, bitmaps, row0, m);
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

__global__ void __launch_bounds__(kBlock)
tt_scan_compact_w(const uint32_t* __restrict__ mask32, const int32_t* __restrict__ tile_off,
                  int32_t* __restrict__ out, int64_t cap) {
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
  if (a + count > cap) return;  // the output was sized from an estimate: the host re-runs this
  int32_t* dst = out + a;
  int head = (int)((4 - (a & 3)) & 3);
  if (head > count) head = count;
  const int body = (count - head) >> 2;
  if (lane < head) __builtin_nontemporal_store(wave_base + st[lane], dst + lane);
  typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
  i32x4* dst4 = reinterpret_cast<i32x4*>(dst + head);
  for (int q = lane; q < body; q += 64) {
    const int i = head + 4 * q;
    i32x4 v = {wave_base + st[i], wave_base + st[i + 1], wave_base + st[i + 2], wave_base + st[i + 3]};
    __builtin_nontemporal_store(v, dst4 + q);
  }
  for (int i = head + 4 * body + lane; i < count; i += 64) __builtin_nontemporal_store(wave_base + st[i], dst + i);

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
// Row groups per lane of the scan kernel: 2, measured on MI355X over a 1e8-row query --
// 1 -> 0.183 ms, 2 -> 0.175 ms, 4 -> 0.194 ms (profiles/r1_query_scan_kernels_v3.md).
constexpr int kEvalGroups = 2;

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
  hipLaunchKernelGGL((tt_scan_eval_t<kEvalGroups>), dim3((unsigned)tiles), dim3(kTileRows / (kRowsPerLane * kEvalGroups)),
                     lds, stream, cd, nrows, live, prog, prog_len, bitmaps, bitmap_words, mask, block_counts);
  return (int)hipGetLastError();
}

// `tile_off`: 16-byte aligned scratch for `tiles` int32 (the tiles' output offsets); `out`
// holds up to nrows ids; the selected count lands in `total` (device) and `total_host` (pinned
// host memory, optional).  Non-temporal id stores: measured on MI355X (1e8 rows, 31.5M
// selected) 0.1215 -> 0.111 ms per query -- the ids stream past L2, the next scan keeps its cache.
// `out` holds `cap` ids: a wave whose segment would end past it writes nothing (the host sized
// `out` from the previous selection's count, sees the total and re-runs the compaction alone
// into an exact buffer when it did not fit: tt_launch_compact).
extern "C" int tt_launch_scan_compact(const uint16_t* mask, const int32_t* block_counts, int32_t* tile_off,
                                      int64_t nrows, int32_t* out, int64_t cap, int64_t* total, int64_t* total_host,
                                      hipStream_t stream) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(tt_tile_offsets, dim3(1), dim3(kOffBlock), 0, stream, block_counts, tiles, tile_off, total,
                     total_host);
  hipLaunchKernelGGL(tt_scan_compact_w, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                     reinterpret_cast<const uint32_t*>(mask), tile_off, out, cap);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_compact(const uint16_t* mask, const int32_t* tile_off, int64_t nrows, int32_t* out,
                                 int64_t cap, hipStream_t stream) {
  const int64_t tiles = (nrows + kTileRows - 1) / kTileRows;
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(tt_scan_compact_w, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                     reinterpret_cast<const uint32_t*>(mask), tile_off, out, cap);
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
