// Paged, ordered state queries without a collection scan (gfx950 / CDNA4, wave64).
//
// A page of an ordered query -- the overdue sweep's `ORDER BY taskCreatedOn ASC LIMIT 1000`, a
// Dapr client's `page.limit` -- needs the first k = offset + limit rows in the order of the
// packed key [rank(sort key 0) | ... | seq] (sort_keys.hip).  Scanning every tile, compacting
// every match and radix-sorting them (the unpaged path) costs O(collection).  Here:
//
// * zone maps: per 8192-row tile, the row holding the smallest key among its live rows
//   (tt_zone_argmin).  The row -- not its key -- is kept: inserting new dictionary values shifts
//   ranks but never reorders existing values, so a tile's argmin stays its argmin until the
//   tile gets new rows or loses rows (the host re-runs those tiles only).  The host turns the
//   argmins into keys with the current rank tables and picks the B tiles with the smallest
//   ones; `bound` = the smallest key among the tiles left out (no row outside the chosen tiles
//   can order before it).
// * tt_page_gather: the filter program (scan_common.h) over the chosen tiles only; every match
//   whose key orders before `bound` appends its (key, row) pair to a candidate buffer (one
//   atomic per tile).  Matches at or after `bound` cannot be on the page unless fewer than k
//   orders before it, and then the host takes more tiles anyway.
// * tt_page_topk: ONE workgroup sorts the candidates in LDS (bitonic, <= 8192 pairs) and writes
//   the page's rows plus [candidates, complete, written].  complete = at least k candidates
//   (all of them order before every unread row), or every tile was read.  Otherwise the host
//   widens B and repeats; with more candidates than the LDS sort holds it narrows B.  It also
//   resets the candidate counter for the next query, so the page path launches no fill kernel.
//
// At 1e8 rows the page costs a handful of tiles instead of 12,207 (profiles/r3_page_topk.md).
#include "scan_common.h"

namespace {

constexpr int kPageCap = 8192;       // candidate pairs one workgroup sorts in LDS (96 KiB)
constexpr int kTopkBlock = 1024;
constexpr int kGatherBlock = kTileRows / kRowsPerLane;  // 512 lanes x 16 rows = one tile
constexpr int kZoneBlock = 256;      // 32 rows per lane
constexpr int kMaxSortKeys = 4;

struct SortSpec {     // host-built, one per sort key (primary first); layout of sort_keys.hip's
  int32_t col;        // column index into the column table
  int32_t rank_off;   // offset of this key's rank table in `ranks`
  int32_t nranks;     // entries in this key's rank table (dictionary size)
  int32_t bits;       // key field width
  int32_t desc;       // 1 = descending
  int32_t missing;    // rank of a missing path
  int32_t max_rank;   // for DESC: stored value = max_rank - rank
  int32_t pad;
};

// The packed ordering keys (identical to tt_sort_keys and ColumnarIndex.sort_keys_numpy) of the
// 16 rows [row0, row0 + 16) (row0 a multiple of 16), for the rows set in
// `sel` (others are left 0): per sort key one vector load of the 16 codes, then the rank lookups
// of all selected rows issued back to back, then one 64-byte load of the sequences -- three
// dependent memory rounds per group instead of three per row.
__device__ __forceinline__ void keys16(const ColumnDesc* cols, const SortSpec* specs, int nkeys,
                                       const int32_t* __restrict__ ranks, const uint32_t* __restrict__ seq,
                                       int seq_bits, int64_t row0, uint32_t sel, uint64_t (&k)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) k[i] = 0;
  for (int j = 0; j < nkeys; ++j) {
    const SortSpec s = specs[j];
    int32_t ids[16];
    load16(cols[s.col], row0, ids);
    int32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      r[i] = s.missing;
      if (((sel >> i) & 1u) && ids[i] >= 0 && ids[i] < s.nranks) r[i] = ranks[s.rank_off + ids[i]];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int32_t v = s.desc ? s.max_rank - r[i] : r[i];
      k[i] = (k[i] << s.bits) | (uint64_t)(uint32_t)v;
    }
  }
  const uint4* sp = reinterpret_cast<const uint4*>(seq + row0);
  uint32_t q[16];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const uint4 x = sp[v];
    q[4 * v] = x.x; q[4 * v + 1] = x.y; q[4 * v + 2] = x.z; q[4 * v + 3] = x.w;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) k[i] = (k[i] << seq_bits) | (uint64_t)q[i];
}

__device__ __forceinline__ void min_pair(uint64_t& k, int32_t& r, uint64_t k2, int32_t r2) {
  if (k2 < k || (k2 == k && (uint32_t)r2 < (uint32_t)r)) {
    k = k2;
    r = r2;
  }
}

}  // namespace

// One workgroup per listed tile: zarg[i] = the live row of tiles[i] with the smallest key, -1 if
// the tile has no live row.
extern "C" __global__ void __launch_bounds__(kZoneBlock)
tt_zone_argmin(const ColumnDesc* __restrict__ cols, int64_t nrows, const uint16_t* __restrict__ live,
               const SortSpec* __restrict__ specs, int32_t nkeys, const int32_t* __restrict__ ranks,
               const uint32_t* __restrict__ seq, int32_t seq_bits, const int32_t* __restrict__ tiles,
               int32_t* __restrict__ zarg) {
  __shared__ SortSpec s_specs[kMaxSortKeys];
  __shared__ ColumnDesc s_cols[kMaxSortKeys];
  __shared__ uint64_t w_key[kZoneBlock / 64];
  __shared__ int32_t w_row[kZoneBlock / 64];
  if (threadIdx.x < nkeys) {
    SortSpec s = specs[threadIdx.x];
    s_cols[threadIdx.x] = cols[s.col];
    s.col = threadIdx.x;  // the key's column now sits at s_cols[j]
    s_specs[threadIdx.x] = s;
  }
  __syncthreads();
  const int64_t tile = tiles[blockIdx.x];
  const int64_t r0 = tile * kTileRows + (int64_t)threadIdx.x * 32;
  uint64_t best = ~0ull;
  int32_t arg = -1;
  if (r0 < nrows) {
    uint32_t lv = (uint32_t)live[r0 >> 4] | ((uint32_t)live[(r0 >> 4) + 1] << 16);
    if (r0 + 32 > nrows) lv &= (nrows - r0 >= 32) ? ~0u : ((1u << (uint32_t)(nrows - r0)) - 1u);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const uint32_t sel = (lv >> (16 * g)) & 0xFFFFu;
      if (!sel) continue;
      uint64_t k[16];
      keys16(s_cols, s_specs, nkeys, ranks, seq, seq_bits, r0 + 16 * g, sel, k);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if ((sel >> i) & 1u) min_pair(best, arg, k[i], (int32_t)(r0 + 16 * g + i));
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t k2 = __shfl_down(best, off, 64);
    const int32_t r2 = __shfl_down(arg, off, 64);
    if (r2 >= 0 && (arg < 0 || k2 < best || (k2 == best && r2 < arg))) {
      best = k2;
      arg = r2;
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    w_key[wave] = best;
    w_row[wave] = arg;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t k = ~0ull;
    int32_t r = -1;
    for (int w = 0; w < kZoneBlock / 64; ++w)
      if (w_row[w] >= 0 && (r < 0 || w_key[w] < k || (w_key[w] == k && w_row[w] < r))) {
        k = w_key[w];
        r = w_row[w];
      }
    zarg[blockIdx.x] = r;
  }
}

// One workgroup per candidate tile: evaluate the filter on the tile's 8192 rows (16 per lane),
// append (key, row) of every live match.  Pairs beyond `cap` are counted, not written.
extern "C" __global__ void __launch_bounds__(kGatherBlock)
tt_page_gather(const ColumnDesc* __restrict__ cols, int64_t nrows, const uint16_t* __restrict__ live,
               const int32_t* __restrict__ prog, int32_t prog_len, const uint32_t* __restrict__ bitmaps,
               int32_t bitmap_words, const SortSpec* __restrict__ specs, int32_t nkeys,
               const int32_t* __restrict__ ranks, const uint32_t* __restrict__ seq, int32_t seq_bits,
               const int32_t* __restrict__ tiles, uint64_t bound, uint64_t* __restrict__ cand_keys,
               int32_t* __restrict__ cand_rows, uint32_t* __restrict__ counter, uint32_t cap) {
  extern __shared__ uint32_t lds_bitmaps[];
  __shared__ SortSpec s_specs[kMaxSortKeys];
  __shared__ ColumnDesc s_cols[kMaxSortKeys];
  __shared__ uint32_t wave_counts[kGatherBlock / 64];
  __shared__ uint32_t block_base;
  const bool in_lds = bitmap_words <= kMaxLdsBitmapWords;
  if (in_lds)
    for (int i = threadIdx.x; i < bitmap_words; i += kGatherBlock) lds_bitmaps[i] = bitmaps[i];
  if (threadIdx.x < nkeys) {
    SortSpec s = specs[threadIdx.x];
    s_cols[threadIdx.x] = cols[s.col];
    s.col = threadIdx.x;
    s_specs[threadIdx.x] = s;
  }
  __syncthreads();
  const int64_t tile = tiles[blockIdx.x];
  const int64_t row0[1] = {tile * kTileRows + (int64_t)threadIdx.x * kRowsPerLane};
  uint32_t m[1];
  if (in_lds) run_program<1>(cols, prog, prog_len, (const uint32_t*)lds_bitmaps, row0, m);
  else run_program<1>(cols, prog, prog_len, bitmaps, row0, m);
  uint32_t sel = row0[0] < nrows ? (m[0] & (uint32_t)live[row0[0] >> 4]) : 0u;
  if (row0[0] < nrows && row0[0] + 16 > nrows) sel &= (1u << (uint32_t)(nrows - row0[0])) - 1u;
  uint64_t key[16];
  keys16(s_cols, s_specs, nkeys, ranks, seq, seq_bits, row0[0], sel, key);
  if (bound != ~0ull) {  // keep the matches that order before every unread tile
    uint32_t keep = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) keep |= (uint32_t)(((sel >> i) & 1u) && key[i] < bound) << i;
    sel = keep;
  }
  const uint32_t cnt = __popc(sel);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = cnt;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wave_counts[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int w = 0; w < kGatherBlock / 64; ++w) {
      const uint32_t c = wave_counts[w];
      wave_counts[w] = s;
      s += c;
    }
    block_base = s ? atomicAdd(counter, s) : 0u;
  }
  __syncthreads();
  uint32_t pos = block_base + wave_counts[wave] + incl - cnt;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (!((sel >> i) & 1u)) continue;
    if (pos < cap) {
      cand_keys[pos] = key[i];
      cand_rows[pos] = (int32_t)(row0[0] + i);
    }
    ++pos;
  }
}

// Bitonic network over keys/rows[0, p) in LDS (p a power of two, the pad is ~0).  Each wave owns
// a contiguous chunk of C = p / 16 elements (the whole array in wave 0 when p < 32): every pass
// whose stride is below C only pairs elements inside one chunk, so it runs under a wave barrier;
// only the strides >= C (cross-chunk, ~10 passes at p = 4096) need the workgroup barrier --
// instead of one per pass (78).  Entered and left with the workgroup synchronised.
// (A register-resident variant -- E elements per thread, cross-lane exchanges by ds_bpermute
// inside a wave, LDS only for cross-wave strides -- measured 56 us against this network's 39 us
// for 4,096 elements: the bpermute chains are latency bound with 16 waves on one CU.)
__device__ __forceinline__ void lds_bitonic(uint64_t* keys, int32_t* rows, int p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk = p >= 32 ? p / (kTopkBlock / 64) : p;
  const bool owner = p >= 32 || wave == 0;
  const int base = p >= 32 ? wave * chunk : 0;
  auto cmpx = [&](int lo, int stride, int size) {
    const int hi = lo | stride;
    const bool up = (lo & size) == 0;
    const uint64_t a = keys[lo], b = keys[hi];
    if ((a > b) == up) {
      keys[lo] = b;
      keys[hi] = a;
      const int32_t t = rows[lo];
      rows[lo] = rows[hi];
      rows[hi] = t;
    }
  };
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto local_passes = [&](int size, int from_stride) {  // strides from_stride .. 1 inside the chunk
    if (!owner) return;
    for (int stride = from_stride; stride > 0; stride >>= 1) {
      for (int i = lane; i < (chunk >> 1); i += 64) {
        const int li = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
        cmpx(base + li, stride, size);
      }
      wave_sync();
    }
  };
  for (int size = 2; size <= p; size <<= 1) {
    int stride = size >> 1;
    if (stride >= chunk) __syncthreads();  // the chunks' wave-local passes are done
    for (; stride >= chunk && stride > 0; stride >>= 1) {  // cross-chunk: the whole workgroup
      for (int i = threadIdx.x; i < (p >> 1); i += kTopkBlock) {
        const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1));
        cmpx(lo, stride, size);
      }
      __syncthreads();
    }
    local_passes(size, stride);
  }
  __syncthreads();
}

// Lane exchange of x with lane ^ J: ds_swizzle (bitmask mode, within 32 lanes) for J < 32, a
// bpermute for 32.  No LDS memory is touched.
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t x) {
  if constexpr (J < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (J << 10));
  else return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x & 63) ^ 32) << 2, (int)x);
}

template <int J>
__device__ __forceinline__ void cmpx_lanes(uint64_t& key, int32_t& row, int lane, int size) {
  const uint64_t ok = ((uint64_t)xor_lane<J>((uint32_t)(key >> 32)) << 32) | xor_lane<J>((uint32_t)key);
  const int32_t orow = (int32_t)xor_lane<J>((uint32_t)row);
  // branch-free: keep the partner's pair if it is the min (max) this lane keeps; equal keys:
  // both lanes keep their own
  const uint32_t keep_min = (uint32_t)(((lane & J) == 0) == ((lane & size) == 0));
  const uint32_t take = ((uint32_t)(ok < key) & keep_min) | ((uint32_t)(key < ok) & (keep_min ^ 1u));
  key = take ? ok : key;
  row = take ? orow : row;
}

// Bitonic sort of the wave's 64 (key, row) pairs, one per lane, ascending by lane: 21
// compare-exchange steps, each three lane exchanges -- no LDS traffic, no barriers.
__device__ __forceinline__ void wave_sort64(uint64_t& key, int32_t& row) {
  const int lane = threadIdx.x & 63;
  cmpx_lanes<1>(key, row, lane, 2);
  cmpx_lanes<2>(key, row, lane, 4); cmpx_lanes<1>(key, row, lane, 4);
  cmpx_lanes<4>(key, row, lane, 8); cmpx_lanes<2>(key, row, lane, 8); cmpx_lanes<1>(key, row, lane, 8);
  cmpx_lanes<8>(key, row, lane, 16); cmpx_lanes<4>(key, row, lane, 16); cmpx_lanes<2>(key, row, lane, 16);
  cmpx_lanes<1>(key, row, lane, 16);
  cmpx_lanes<16>(key, row, lane, 32); cmpx_lanes<8>(key, row, lane, 32); cmpx_lanes<4>(key, row, lane, 32);
  cmpx_lanes<2>(key, row, lane, 32); cmpx_lanes<1>(key, row, lane, 32);
  cmpx_lanes<32>(key, row, lane, 64); cmpx_lanes<16>(key, row, lane, 64); cmpx_lanes<8>(key, row, lane, 64);
  cmpx_lanes<4>(key, row, lane, 64); cmpx_lanes<2>(key, row, lane, 64); cmpx_lanes<1>(key, row, lane, 64);
}

// Sort of p <= 1024 pairs (p a power of two, pad keys ~0), writing only the page's rows:
// wave w sorts elements [64w, 64w + 64) in registers (wave_sort64), then the sorted runs merge
// pairwise, log2(p / 64) levels: every element finds its place in the merged run as its index
// in its own run plus the number of the partner run's keys before it (a branchless binary
// search; equal keys order by run).  An element stays in its thread's registers throughout; only
// its key is published in LDS at each level (two ping-pong areas above the first 1,024 keys, so
// the caller's unsorted pairs there are not overwritten).  At the end the element goes straight
// to out_rows if its position is in [offset, upto).  log2(p / 64) barriers, against ~15 for the
// LDS network at p = 1024 (profiles/r3_page_topk.md: 37 k of the kernel's 61 k shader clocks
// were that network).  `key`/`row`: this thread's element (threads >= max(p, 64) are idle but
// reach the barriers).
__device__ __forceinline__ void rank_sort_1024(uint64_t key, int32_t row, int p, uint64_t* keys, int offset,
                                               int upto, int32_t* __restrict__ out_rows) {
  const int tid = threadIdx.x, wave = tid >> 6;
  const int runs = p > 64 ? p >> 6 : 1;
  const bool active = wave < runs;
  if (active) wave_sort64(key, row);
  uint64_t* cur = keys + kTopkBlock;
  uint64_t* nxt = keys + 2 * kTopkBlock;
  int pos = tid;
  if (active) cur[pos] = key;
  for (int lg = 6; (1 << lg) < 64 * runs; ++lg) {
    __syncthreads();  // this level's run keys are published
    if (active) {
      const int len = 1 << lg;
      const int r = pos >> lg, i = pos & (len - 1), q = r ^ 1;
      const uint64_t* run = cur + q * len;
      const uint32_t lower = (uint32_t)(q < r);
      uint32_t at = 0;
      for (int s = len >> 1; s > 0; s >>= 1) {
        const uint64_t a = run[at + s - 1];
        at += ((uint32_t)(a < key) | (lower & (uint32_t)(a == key))) * (uint32_t)s;
      }
      const uint64_t a = run[at];
      at += (uint32_t)(a < key) | (lower & (uint32_t)(a == key));
      pos = ((r >> 1) << (lg + 1)) + i + (int)at;
      nxt[pos] = key;
    }
    uint64_t* t = cur;
    cur = nxt;
    nxt = t;
  }
  if (active && pos >= offset && pos < upto) out_rows[pos - offset] = row;
}

// Inclusive prefix sum across the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d);
    if (lane >= d) v += o;
  }
  return v;
}

// ONE workgroup: the page [offset, k) of the candidates' key order.
// info = [candidates, complete, written, 0]; out_rows = the page's rows.
//
// n <= k: a sort of all n (padded to a power of two): up to 1,024 in registers plus a merge tree
// (rank_sort_1024), more by the LDS network.  n > k (a bound that let more candidates through than
// the page holds -- 2,600 for a 1,000-row page at 1e8 rows): the k-th smallest key is found first
// by a most-significant-digit radix select over the LDS copy (8-bit digits, starting at the
// highest bit in which the candidates differ; it stops at the first digit whose keys end exactly
// at the k-th -- usually the second), then only the k keys at or below it are compacted (one LDS
// atomic per wave) and sorted.  Keys are unique (the insertion sequence is their low bits), so
// exactly k keys are at or below the k-th.  `stamps` (kernel tests only, else null): thread 0's
// shader clock at the phase boundaries (scripts/topk_phases.py).
extern "C" __global__ void __launch_bounds__(kTopkBlock)
tt_page_topk(const uint64_t* __restrict__ cand_keys, const int32_t* __restrict__ cand_rows,
             uint32_t* __restrict__ counter, uint32_t cap, int32_t k, int32_t offset, uint64_t bound,
             int32_t* __restrict__ info, int32_t* __restrict__ out_rows, int64_t* __restrict__ stamps) {
  auto stamp = [&](int i) {
    if (stamps && threadIdx.x == 0) stamps[i] = clock64();
  };
  stamp(0);
  __shared__ uint64_t keys[kPageCap];
  __shared__ int32_t rows[kPageCap];
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_lo, s_hi, s_prefix;
  __shared__ uint32_t s_need, s_count, s_done;
  const uint32_t total = *counter;
  const int n = (int)(total < cap ? total : cap);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int p = 1;
  const int upto = n < k ? n : k;
  const int written = upto > offset ? upto - offset : 0;
  if (n <= k && n <= kTopkBlock) {  // the common page: one element per thread, straight from memory
    while (p < n) p <<= 1;
    stamp(3);
    rank_sort_1024(tid < n ? cand_keys[tid] : ~0ull, tid < n ? cand_rows[tid] : -1, p, keys, offset, upto,
                   out_rows);
    stamp(4);
  } else if (n <= k) {
    while (p < n) p <<= 1;
    for (int i = tid; i < p; i += kTopkBlock) {
      keys[i] = i < n ? cand_keys[i] : ~0ull;
      rows[i] = i < n ? cand_rows[i] : -1;
    }
    __syncthreads();
  } else {
    // the candidates' range: min and max key (wave reductions, then wave 0 over the waves)
    uint64_t lo = ~0ull, hi = 0;
    for (int i = tid; i < n; i += kTopkBlock) {
      const uint64_t x = cand_keys[i];
      keys[i] = x;
      rows[i] = cand_rows[i];
      lo = x < lo ? x : lo;
      hi = x > hi ? x : hi;
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const uint64_t ol = __shfl_xor(lo, d), oh = __shfl_xor(hi, d);
      lo = ol < lo ? ol : lo;
      hi = oh > hi ? oh : hi;
    }
    if (tid == 0) {
      s_lo = ~0ull;
      s_hi = 0;
    }
    __syncthreads();
    if (lane == 0) {
      atomicMin(reinterpret_cast<unsigned long long*>(&s_lo), (unsigned long long)lo);
      atomicMax(reinterpret_cast<unsigned long long*>(&s_hi), (unsigned long long)hi);
    }
    __syncthreads();
    stamp(1);
    const uint64_t diff = s_lo ^ s_hi;
    const int top = diff ? 63 - __clzll((long long)diff) : 0;  // highest bit in which keys differ
    int shift = (top / 8) * 8;                                  // its 8-bit digit
    if (tid == 0) {
      s_prefix = shift + 8 >= 64 ? 0 : (s_lo >> (shift + 8)) << (shift + 8);  // the common high bits
      s_need = (uint32_t)k;
      s_done = 0;
    }
    __syncthreads();
    for (; shift >= 0 && !s_done; shift -= 8) {
      for (int i = tid; i < 256; i += kTopkBlock) hist[i] = 0;
      __syncthreads();
      const uint64_t prefix = s_prefix;
      const uint64_t above = shift + 8 >= 64 ? 0 : ~0ull << (shift + 8);
      for (int i = tid; i < n; i += kTopkBlock) {
        const uint64_t x = keys[i];
        if ((x & above) == prefix) atomicAdd(&hist[(x >> shift) & 255], 1u);
      }
      __syncthreads();
      if (wave == 0) {  // the digit holding the need-th key of the remaining range
        uint32_t c[4];
        uint32_t own = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          c[j] = hist[lane * 4 + j];
          own += c[j];
        }
        const uint32_t incl = wave_inclusive_sum(own);
        const uint32_t need = s_need;
        uint32_t before = incl - own;
        if (before < need && need <= incl) {  // exactly one lane holds the digit
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (need <= before + c[j]) {
              // the k-th key is the last of its digit's keys: every key up to the digit's end
              // is on the page -- the threshold is found without the lower digits' passes
              const bool last = need == before + c[j];
              s_prefix = prefix | ((uint64_t)(lane * 4 + j) << shift) | (last ? (1ull << shift) - 1 : 0);
              s_need = need - before;
              s_done = last;
              break;
            }
            before += c[j];
          }
        }
      }
      __syncthreads();
    }
    // keys <= the k-th key: exactly k of them, compacted to the front (read, barrier, write)
    stamp(2);
    const uint64_t kth = s_prefix;
    constexpr int kPer = kPageCap / kTopkBlock;  // candidates per thread (8), held in registers
    uint64_t xk[kPer];
    int32_t xr[kPer];
    bool sel[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int i = tid + r * kTopkBlock;
      sel[r] = false;
      xk[r] = 0;
      xr[r] = -1;
      if (i < n) {
        xk[r] = keys[i];
        xr[r] = rows[i];
        sel[r] = xk[r] <= kth;
      }
    }
    if (tid == 0) s_count = 0;
    __syncthreads();
    while (p < k) p <<= 1;
#pragma unroll
    for (int r = 0; r < kPer; ++r) {  // one LDS atomic per wave and round: ballot + lane offsets
      const uint64_t m = __ballot(sel[r]);
      if (!m) continue;
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&s_count, (uint32_t)__popcll(m));
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl(base, 0));
      const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (sel[r] && (int)slot < p) {
        keys[slot] = xk[r];
        rows[slot] = xr[r];
      }
    }
    __syncthreads();
    const int got = (int)(s_count < (uint32_t)p ? s_count : (uint32_t)p);
    if (p <= kTopkBlock) {  // k <= 1024: the selected k straight from the compaction
      stamp(3);
      rank_sort_1024(tid < got ? keys[tid] : ~0ull, tid < got ? rows[tid] : -1, p, keys, offset, upto, out_rows);
      stamp(4);
    } else {
      for (int i = got + tid; i < p; i += kTopkBlock) {
        keys[i] = ~0ull;
        rows[i] = -1;
      }
      __syncthreads();
    }
  }
  if (p > kTopkBlock || (n <= k && n > kTopkBlock)) {
    stamp(3);
    lds_bitonic(keys, rows, p);
    stamp(4);
    for (int i = tid; i < written; i += kTopkBlock) out_rows[i] = rows[offset + i];
  }
  if (tid == 0) {
    int complete;
    if (total > cap) complete = 0;                     // overflow: the host takes fewer tiles
    else if (n >= k) complete = 1;                     // k candidates, all before every unread row
    else complete = bound == ~0ull;                    // every tile was read
    info[0] = (int32_t)total;
    info[1] = complete;
    info[2] = written;
    info[3] = 0;
    *counter = 0;  // ready for the next query's gather (stream order)
  }
  stamp(5);
}

extern "C" __global__ void tt_page_reset(uint32_t* __restrict__ counter) {
  if (threadIdx.x == 0) *counter = 0;
}

extern "C" int tt_page_cap() { return kPageCap; }

// The candidate counter's first zeroing (tt_page_topk resets it after every query).
extern "C" int tt_launch_page_reset(uint32_t* counter, hipStream_t stream) {
  hipLaunchKernelGGL(tt_page_reset, dim3(1), dim3(64), 0, stream, counter);
  return (int)hipGetLastError();
}

extern "C" int tt_launch_zone_argmin(const void* cols, int64_t nrows, const uint16_t* live, const void* specs,
                                     int32_t nkeys, const int32_t* ranks, const uint32_t* seq, int32_t seq_bits,
                                     const int32_t* tiles, int32_t ntiles, int32_t* zarg, hipStream_t stream) {
  if (ntiles <= 0) return 0;
  if (nkeys < 0 || nkeys > kMaxSortKeys || seq_bits < 0 || seq_bits > 32) return -1;
  hipLaunchKernelGGL(tt_zone_argmin, dim3((unsigned)ntiles), dim3(kZoneBlock), 0, stream,
                     reinterpret_cast<const ColumnDesc*>(cols), nrows, live, reinterpret_cast<const SortSpec*>(specs),
                     nkeys, ranks, seq, seq_bits, tiles, zarg);
  return (int)hipGetLastError();
}

// The top-k alone over a caller-filled candidate buffer (`counter` holds their number): the
// kernel tests drive it with every candidate count from 0 to kPageCap.
extern "C" int tt_launch_page_topk(const uint64_t* cand_keys, const int32_t* cand_rows, uint32_t* counter, int32_t k,
                                   int32_t offset, uint64_t bound, int32_t* info, int32_t* out_rows,
                                   int64_t* stamps, hipStream_t stream) {
  if (k <= 0 || k > kPageCap || offset < 0 || offset > k) return -1;
  hipLaunchKernelGGL(tt_page_topk, dim3(1), dim3(kTopkBlock), 0, stream, cand_keys, cand_rows, counter,
                     (uint32_t)kPageCap, k, offset, bound, info, out_rows, stamps);
  return (int)hipGetLastError();
}

// `counter` must be 0 before the first query (tt_page_topk resets it after each).
extern "C" int tt_launch_page(const void* cols, int64_t nrows, const uint16_t* live, const int32_t* prog, int32_t prog_len,
                              const uint32_t* bitmaps, int32_t bitmap_words, const void* specs, int32_t nkeys,
                              const int32_t* ranks, const uint32_t* seq, int32_t seq_bits, const int32_t* tiles,
                              int32_t ntiles, uint64_t* cand_keys, int32_t* cand_rows, uint32_t* counter, int32_t k,
                              int32_t offset, uint64_t bound, int32_t* info, int32_t* out_rows, hipStream_t stream) {
  if (prog_len <= 0 || bitmap_words <= 0 || ntiles < 0) return -1;
  if (nkeys < 0 || nkeys > kMaxSortKeys || seq_bits < 0 || seq_bits > 32) return -1;
  if (k <= 0 || k > kPageCap || offset < 0 || offset > k) return -1;
  if (ntiles > 0) {
    const size_t lds = bitmap_words <= kMaxLdsBitmapWords ? (size_t)bitmap_words * sizeof(uint32_t) : 0;
    hipLaunchKernelGGL(tt_page_gather, dim3((unsigned)ntiles), dim3(kGatherBlock), lds, stream,
                       reinterpret_cast<const ColumnDesc*>(cols), nrows, live, prog, prog_len, bitmaps, bitmap_words,
                       reinterpret_cast<const SortSpec*>(specs), nkeys, ranks, seq, seq_bits, tiles, bound, cand_keys,
                       cand_rows, counter, (uint32_t)kPageCap);
  }
  hipLaunchKernelGGL(tt_page_topk, dim3(1), dim3(kTopkBlock), 0, stream, cand_keys, cand_rows, counter,
                     (uint32_t)kPageCap, k, offset, bound, info, out_rows, (int64_t*)nullptr);
  return (int)hipGetLastError();
}

// Host-mapped mailboxes for the page path: its inputs (tile ids) and outputs (info + rows) live
// in pinned, coherent host memory that the kernels read and write directly, so a page query is
// two kernel launches and one stream synchronise -- no copy kernels, no DMA, no allocation.
extern "C" void* tt_host_alloc(int64_t bytes) {
  void* p = nullptr;
  if (bytes <= 0 || hipHostMalloc(&p, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return nullptr;
  return p;
}

extern "C" void* tt_host_device_ptr(void* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
  return d;
}

extern "C" int tt_host_free(void* p) { return p ? (int)hipHostFree(p) : 0; }

extern "C" int tt_stream_sync(hipStream_t stream) { return (int)hipStreamSynchronize(stream); }
