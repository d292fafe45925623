// Ordering keys for state-store query results (gfx950).
//
// The query API orders results by up to a few document paths (ASC/DESC) with ties broken by
// insertion order (backing/accel.py, ops/columnar.py ColumnarIndex.order -- the native
// engine's semantics).  For a selection produced by tt_scan_compact this kernel packs, per
// selected row, one 63-bit unsigned key
//
//     [rank(key0) | rank(key1) | ... | seq]          (most significant first)
//
// where rank(k) is the value's position in the column dictionary's sort order (missing paths
// rank like null; DESC keys store max_rank - rank), and seq is the document's insertion
// sequence.  Sorting the keys (radix sort / top-k) then yields exactly the host ordering.
// Rank lookups go through a small per-key rank table (dictionary id -> rank) staged in LDS
// when it fits (it is gathered once per row and per key, so LDS keeps those random reads
// off HBM).
//
// Layout: one thread per selected row, 256-thread blocks; rows are ascending row ids, so the
// id / seq gathers of neighbouring lanes hit neighbouring addresses.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kBlock = 256;
constexpr int kMaxKeys = 4;
constexpr int kLdsRankWords = 8192;  // 32 KiB of rank tables in LDS (all keys together)
constexpr int kHistBins = 4096;      // 12-bit radix-select histogram (top-k)

struct SortColumn {   // 16 bytes, same layout as the scan kernel's ColumnDesc
  uint64_t ptr;
  int32_t width;      // 1, 2 or 4 bytes per row; 0 = 2 bits per row
  int32_t pad;
};

struct SortSpec {     // host-built, one per sort key (primary first)
  int32_t col;        // column index into the column table
  int32_t rank_off;   // offset of this key's rank table in `ranks`
  int32_t nranks;     // entries in this key's rank table (dictionary size)
  int32_t bits;       // key field width
  int32_t desc;       // 1 = descending
  int32_t missing;    // rank of a missing path
  int32_t max_rank;   // for DESC: stored value = max_rank - rank
  int32_t pad;
};

__device__ __forceinline__ int32_t load_id(const SortColumn& c, int64_t row) {
  if (c.width == 0) {  // 2-bit codes, 3 = missing
    const uint32_t v = (reinterpret_cast<const uint8_t*>(c.ptr)[row >> 2] >> ((row & 3) * 2)) & 3u;
    return v == 3u ? -1 : (int32_t)v;
  }
  if (c.width == 1) {
    const uint32_t v = reinterpret_cast<const uint8_t*>(c.ptr)[row];
    return v == 0xFFu ? -1 : (int32_t)v;
  }
  if (c.width == 2) {
    const uint32_t v = reinterpret_cast<const uint16_t*>(c.ptr)[row];
    return v == 0xFFFFu ? -1 : (int32_t)v;
  }
  return reinterpret_cast<const int32_t*>(c.ptr)[row];
}

}  // namespace


// One thread per selected row in a grid-stride loop (a few rows per thread amortise the LDS
// staging of the rank tables); `seq` is the 32-bit device copy of the insertion sequence.
// With `hist != nullptr` the 12-bit radix-select histogram of the keys (bits [shift, shift+12))
// is accumulated in the same pass (LDS-privatised, one global atomic per non-empty bin).
extern "C" __global__ void __launch_bounds__(kBlock)
tt_sort_keys(const SortColumn* __restrict__ cols, const int32_t* __restrict__ rows, int64_t n,
             const SortSpec* __restrict__ specs, int32_t nkeys, const int32_t* __restrict__ ranks,
             int32_t rank_words, const uint32_t* __restrict__ seq, int32_t seq_bits, uint64_t* __restrict__ keys,
             uint32_t* __restrict__ hist, int32_t shift) {
  // dynamic LDS: [hist (kHistBins words, only with `hist`)] [rank tables (rank_words, when they fit)]
  extern __shared__ uint32_t lds_dyn[];
  uint32_t* lds_hist = lds_dyn;
  int32_t* lds_ranks = reinterpret_cast<int32_t*>(lds_dyn + (hist ? kHistBins : 0));
  __shared__ SortSpec lds_specs[kMaxKeys];
  __shared__ SortColumn lds_cols[kMaxKeys];
  const bool staged = rank_words <= kLdsRankWords;
  if (staged)
    for (int i = threadIdx.x; i < rank_words; i += kBlock) lds_ranks[i] = ranks[i];
  if (hist)
    for (int i = threadIdx.x; i < kHistBins; i += kBlock) lds_hist[i] = 0;
  if (threadIdx.x < nkeys) {
    lds_specs[threadIdx.x] = specs[threadIdx.x];
    lds_cols[threadIdx.x] = cols[specs[threadIdx.x].col];
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int64_t row = rows[i];
    uint64_t k = 0;
    for (int j = 0; j < nkeys; ++j) {
      const SortSpec s = lds_specs[j];
      const int32_t id = load_id(lds_cols[j], row);
      int32_t r = s.missing;
      if (id >= 0 && id < s.nranks) r = staged ? lds_ranks[s.rank_off + id] : ranks[s.rank_off + id];
      if (s.desc) r = s.max_rank - r;
      k = (k << s.bits) | (uint64_t)(uint32_t)r;
    }
    k = (k << seq_bits) | (uint64_t)seq[row];
    keys[i] = k;
    if (hist) atomicAdd(&lds_hist[(uint32_t)(k >> shift) & (kHistBins - 1)], 1u);
  }
  if (hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < kHistBins; i += kBlock)
      if (lds_hist[i]) atomicAdd(&hist[i], lds_hist[i]);
  }
}

extern "C" int tt_launch_sort_keys(const void* cols, const int32_t* rows, int64_t n, const void* specs, int32_t nkeys,
                                   const int32_t* ranks, int32_t rank_words, const uint32_t* seq, int32_t seq_bits,
                                   uint64_t* keys, uint32_t* hist, int32_t shift, hipStream_t stream) {
  if (n <= 0) return 0;
  if (nkeys < 0 || nkeys > kMaxKeys || seq_bits < 0 || seq_bits > 32 || shift < 0 || shift > 63) return -1;
  // a bounded grid (8 blocks per CU on 256 CUs): each thread loops over many rows, so the LDS
  // staging and the histogram flush (<= 4096 global atomics per block) are amortised
  int64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  const size_t lds = ((hist ? kHistBins : 0) + (rank_words <= kLdsRankWords ? rank_words : 0)) * sizeof(uint32_t);
  hipLaunchKernelGGL(tt_sort_keys, dim3((unsigned)blocks), dim3(kBlock), lds, stream,
                     reinterpret_cast<const SortColumn*>(cols), rows, n, reinterpret_cast<const SortSpec*>(specs), nkeys,
                     ranks, rank_words, seq, seq_bits, keys, hist, shift);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int tt_sort_max_keys() { return kMaxKeys; }

// ---------------------------------------------------------------------------------------
// Top-k by radix select: a paged, ordered query needs only the first `k` keys of the
// selection, so instead of sorting all of them (radix sort of tens of millions of 64-bit
// keys) we (1) histogram the 12 most significant *used* key bits (fused into tt_sort_keys),
// (2) find on the host the
// bin where the running count reaches k, (3) compact the (key, row) pairs at or below that bin
// and (4) sort only those candidates.
namespace {
constexpr int kSelItems = 16;       // keys per thread per block-iteration
}  // namespace

// Keep pairs whose bin <= `last_bin`; one global atomic per block reserves the block's range.
extern "C" __global__ void __launch_bounds__(kBlock)
tt_select_le_bin(const uint64_t* __restrict__ keys, const int32_t* __restrict__ rows, int64_t n, int32_t shift,
                 uint32_t last_bin, uint64_t* __restrict__ out_keys, int32_t* __restrict__ out_rows,
                 uint32_t* __restrict__ counter, uint32_t capacity) {
  __shared__ uint32_t warp_counts[kBlock / 64];
  __shared__ uint32_t block_base;
  const int64_t base = (int64_t)blockIdx.x * kBlock * kSelItems;
  // pass 1: count this thread's matches (no dynamically indexed register arrays -> no scratch).
  // Item j of a thread is key base + (j / 2) * 2 * kBlock + 2 * thread + (j & 1): pairs of keys
  // come in one 16-byte load (8 per thread, 1 KiB per wave-instruction); a pair that straddles
  // n (odd n, last pair) is read key by key.
  uint32_t matchbits = 0, cnt = 0;
#pragma unroll
  for (int j2 = 0; j2 < kSelItems / 2; ++j2) {
    const int64_t i = base + (int64_t)j2 * 2 * kBlock + 2 * (int64_t)threadIdx.x;
    uint64_t k0 = 0, k1 = 0;
    if (i + 1 < n) {
      const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(keys + i);
      k0 = v.x;
      k1 = v.y;
    } else if (i < n) {
      k0 = keys[i];
    }
    if (i < n && ((uint32_t)(k0 >> shift) & (kHistBins - 1)) <= last_bin) {
      matchbits |= 1u << (2 * j2);
      ++cnt;
    }
    if (i + 1 < n && ((uint32_t)(k1 >> shift) & (kHistBins - 1)) <= last_bin) {
      matchbits |= 1u << (2 * j2 + 1);
      ++cnt;
    }
  }
  // block-wide exclusive scan of per-thread counts (wave prefix via shuffles, then wave sums)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) warp_counts[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      const uint32_t c = warp_counts[w];
      warp_counts[w] = s;
      s += c;
    }
    block_base = s ? atomicAdd(counter, s) : 0;
  }
  __syncthreads();
  // pass 2: write the matches (the keys were just read: this re-read hits the cache)
  uint32_t pos = block_base + warp_counts[wave] + incl - cnt;
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    if (!(matchbits & (1u << j))) continue;
    const int64_t i = base + (int64_t)(j >> 1) * 2 * kBlock + 2 * (int64_t)threadIdx.x + (j & 1);
    if (pos < capacity) {
      out_keys[pos] = keys[i];
      out_rows[pos] = rows[i];
    }
    ++pos;
  }
}

extern "C" int tt_launch_select_le_bin(const uint64_t* keys, const int32_t* rows, int64_t n, int32_t shift,
                                       uint32_t last_bin, uint64_t* out_keys, int32_t* out_rows, uint32_t* counter,
                                       uint32_t capacity, hipStream_t stream) {
  if (n <= 0) return 0;
  if (shift < 0 || shift > 63) return -1;
  const int64_t blocks = (n + (int64_t)kBlock * kSelItems - 1) / ((int64_t)kBlock * kSelItems);
  hipLaunchKernelGGL(tt_select_le_bin, dim3((unsigned)blocks), dim3(kBlock), 0, stream, keys, rows, n, shift, last_bin,
                     out_keys, out_rows, counter, capacity);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int tt_hist_bins() { return kHistBins; }
