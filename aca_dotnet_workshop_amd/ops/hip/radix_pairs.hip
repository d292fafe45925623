// Final ordering of query results: a stable LSD radix sort of (packed ordering key, row id)
// pairs over only the key bits that can be set (ops/gpu.py GpuKernels._sorted_rows).
//
// tt_sort_keys packs [ranks | seq] into key_bits <= 63 bits (e.g. a 10-bit date rank + a
// 27-bit insertion sequence = 37 bits), so the sort needs ceil(key_bits / 8) digit passes
// instead of the 8 an int64 argsort makes, and it moves the row ids with the keys -- no argsort
// index plus gather of the rows afterwards.
//
// Up to 8192 pairs: one launch, every pass inside one workgroup with the pairs in LDS
// (tt_radix_small).  Beyond that, one launch for the first digit's totals plus ONE launch per
// 8-bit pass (profiles/r4_radix_sort.md):
//   tt_radix_totals   the first pass's 256 digit totals (each pass counts the next pass's digits
//                     from the keys it already holds: the totals are complete at the launch
//                     boundary);
//   tt_radix_onesweep per tile (8192 pairs from kBigTileMin pairs up, 2048 below), taken in
//                     order from an atomic tile counter: the tile's digit counts are published
//                     first, each wave ranks its own contiguous keys among equal digits (the
//                     ballot match + popcount of the lanes below, a wave-private running count
//                     per digit in LDS), the tile finds where its run of each digit starts by
//                     decoupled look-back over the earlier tiles' status words, and its keys and
//                     then its rows pass through one LDS exchange buffer, digit-sorted, to be
//                     written in tile order (consecutive threads, consecutive addresses within
//                     each digit's run).
// Look-back hand-off: the status word IS the data -- {2-bit flag, 30-bit count} in one 4-byte word,
// stored and polled with agent-scope relaxed atomics (sc1: the per-XCD L2s are not coherent, and a
// plain poll could be served from L1 or a register forever).  No other bytes cross between
// workgroups inside a launch.  Forward progress: a tile waits only on tiles with smaller indices,
// which were dequeued by workgroups already running, and every tile publishes its counts
// before it waits; the spin is bounded anyway (kSpinLimit), a timeout is counted in `fault` and
// the host raises (ops/gpu.py) -- no wave can spin forever.
// Wave64 throughout (64-bit ballots).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kBins = 256;                      // 8-bit digits
constexpr int kSortBlock = 256;                 // the totals kernel's workgroup
constexpr int kSortItems = 16;                  // pairs per thread in tt_radix_small
constexpr int kWaveKeys = 64 * kSortItems;      // contiguous keys ranked by one wave there

// Lanes of this wave whose (valid) digit equals this lane's: one ballot per digit bit.  Per
// bit, x is all ones where the bit is set (one signed bit-field extract), the ballot of x, and
// each 32-bit half of the match keeps the lanes whose ballot bit agrees with x: m &= ~(on ^ x),
// one 3-input logic op per half (no per-lane select of a scalar mask, which gfx950's single
// scalar operand per VALU instruction would turn into extra moves).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int bits = 8) {
  const uint64_t act = __ballot(valid);
  uint32_t lo = (uint32_t)act, hi = (uint32_t)(act >> 32);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    if (b >= bits) break;  // uniform: a narrower last digit skips the rest
    const uint32_t x = (uint32_t)((int32_t)(d << (31 - b)) >> 31);
    const uint64_t on = __ballot(x != 0u);
    lo &= ~((uint32_t)on ^ x);
    hi &= ~((uint32_t)(on >> 32) ^ x);
  }
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// The wave-private running counts: relaxed atomics keep every step's LDS read and write real and
// in program order, and (unlike a volatile pointer, which the compiler leaves generic: flat_
// accesses that also wait on the vector-memory counter) they stay ds_ operations.
__device__ __forceinline__ uint32_t run_get(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void run_set(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int kMaxPasses = 8;
constexpr int kTotalsBlocks = 1024;
constexpr int kTotalsItems = 16;
constexpr uint32_t kFlagAgg = 1u << 30;   // the tile's own count
constexpr uint32_t kFlagIncl = 2u << 30;  // the count of this tile and every earlier one
constexpr uint32_t kCountMask = (1u << 30) - 1u;
constexpr uint32_t kSpinLimit = 1u << 24;
constexpr int kLookback = 8;  // predecessor status words polled per look-back round

__device__ __forceinline__ uint32_t poll_status(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_status(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Adds this lane's digit to an LDS histogram; a wave whose valid digits are all equal adds once
// (skewed high digits: no 64-way same-address LDS atomics).
__device__ __forceinline__ void count_digit(uint32_t* h, uint32_t d, bool valid, int lane) {
  const uint64_t act = __ballot(valid);
  if (act == 0) return;
  // valid lanes are a prefix of the wave (indices rise with the lane): lane 0 is one of them
  const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)d);
  if (__ballot(valid && d != d0) == 0) {
    if (lane == 0) atomicAdd(&h[d0], (uint32_t)__popcll(act));
  } else if (valid) {
    atomicAdd(&h[d], 1u);
  }
}

// totals[d]: keys whose first digit is d (each later pass's totals come from the pass before it).
__global__ __launch_bounds__(kSortBlock) void tt_radix_totals(const uint64_t* __restrict__ keys, int64_t n,
                                                              uint32_t mask, uint32_t* __restrict__ totals) {
  __shared__ uint32_t h[kBins];
  const int t = threadIdx.x, lane = t & 63;
  h[t] = 0;
  __syncthreads();
  const int64_t step = (int64_t)gridDim.x * kSortBlock * kTotalsItems;
  for (int64_t c0 = (int64_t)blockIdx.x * kSortBlock * kTotalsItems; c0 < n; c0 += step) {
    uint64_t k[kTotalsItems];
#pragma unroll
    for (int i = 0; i < kTotalsItems; ++i) {
      const int64_t idx = c0 + (int64_t)i * kSortBlock + t;
      k[i] = idx < n ? keys[idx] : 0ull;
    }
#pragma unroll
    for (int i = 0; i < kTotalsItems; ++i)
      count_digit(h, (uint32_t)k[i] & mask, c0 + (int64_t)i * kSortBlock + t < n, lane);
  }
  __syncthreads();
  if (h[t]) atomicAdd(&totals[t], h[t]);
}

// 512 threads x kOsItems pairs per tile.  Large sorts take 16 (8192-pair tiles: each digit's
// run in the output averages 32 pairs, 256-B key and 128-B row segments; the LDS holds one
// 64 KiB exchange buffer that takes the tile's keys and then its rows, two workgroups per CU);
// below kBigTileMin pairs 4 (2048-pair tiles), so that a mid-size sort (a top-k's candidates)
// still spreads over the CUs.
constexpr int kOsBlock = 512;
constexpr int kOsWaves = kOsBlock / 64;
constexpr int64_t kBigTileMin = 1 << 21;

template <int kOsItems>
__global__ __launch_bounds__(kOsBlock) void tt_radix_onesweep(const uint64_t* __restrict__ kin,
                                                              const int32_t* __restrict__ vin,
                                                              uint64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                              int64_t n, int shift, uint32_t mask,
                                                              const uint32_t* __restrict__ totals,
                                                              uint32_t* __restrict__ next_totals, int next_shift,
                                                              uint32_t next_mask, uint32_t* __restrict__ status,
                                                              uint32_t* __restrict__ tile_counter,
                                                              uint32_t* __restrict__ fault) {
  constexpr int kOsTile = kOsBlock * kOsItems;
  constexpr int kOsWaveKeys = 64 * kOsItems;  // contiguous keys ranked by one wave
  __shared__ uint64_t xbuf[kOsTile];          // the tile's keys, digit-sorted; then its rows
  __shared__ uint32_t start[kBins];           // tile-local start of each digit's run
  __shared__ uint32_t gbase[kBins];           // where the tile's run of each digit starts in the output
  __shared__ uint32_t wrun[kOsWaves][kBins];  // per wave: keys of each digit ranked so far, then prefixes
  __shared__ uint32_t nh[kBins];              // the tile's counts of the NEXT pass's digits
  __shared__ uint32_t cnt[kBins];             // the tile's counts of this pass's digits
  __shared__ uint32_t tile_s;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int bits = __popc(mask);
  const bool digit_lane = t < kBins;          // threads 0..255 each own one digit
  if (t == 0) tile_s = atomicAdd(tile_counter, 1u);
  for (int j = t; j < kOsWaves * kBins; j += kOsBlock) (&wrun[0][0])[j] = 0;
  if (digit_lane) {
    nh[t] = 0;
    cnt[t] = 0;
  }
  __syncthreads();
  const uint32_t tile = tile_s;
  const int64_t tile0 = (int64_t)tile * kOsTile;
  const int64_t base = tile0 + (int64_t)wave * kOsWaveKeys + lane;
  uint64_t k[kOsItems];
  int32_t v[kOsItems];
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int64_t idx = base + (int64_t)i * 64;
    const bool valid = idx < n;
    k[i] = valid ? kin[idx] : 0ull;
    v[i] = valid ? vin[idx] : 0;
  }
  const uint32_t total = digit_lane ? totals[t] : 0u;
  // 1. the tile's digit counts, published before the ranking: the later tiles' look-back waits
  //    only for this, not for the whole tile
#pragma unroll
  for (int i = 0; i < kOsItems; ++i)
    count_digit(cnt, (uint32_t)(k[i] >> shift) & mask, base + (int64_t)i * 64 < n, lane);
  __syncthreads();
  uint32_t* my = status + (int64_t)tile * kBins + t;
  const uint32_t c = digit_lane ? cnt[t] : 0u;
  if (digit_lane) publish_status(my, (tile == 0 ? kFlagIncl : kFlagAgg) | c);
  // 2. each wave ranks its own keys, in input order: earlier steps through the wave's running
  //    count of the digit, the same step through the lanes below with the same digit.  Only a
  //    digit's first lane writes its count, and LDS operations of one wave complete in program
  //    order; run_get/run_set keep every step's read of the counters a real LDS read.
  uint32_t* run = wrun[wave];
  uint32_t r[kOsItems];
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const bool valid = base + (int64_t)i * 64 < n;
    const uint32_t d = (uint32_t)(k[i] >> shift) & mask;
    const uint64_t eq = match_digit(d, valid, bits);
    const uint64_t below = eq & lanes_below(lane);
    r[i] = run_get(&run[d]) + (uint32_t)__popcll(below);
    __builtin_amdgcn_wave_barrier();
    if (valid && below == 0) run_set(&run[d], r[i] + (uint32_t)__popcll(eq));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // 3. per digit: the earlier waves' counts (wave order = input order)
  if (digit_lane) {
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < kOsWaves; ++w) {
      const uint32_t x = wrun[w][t];
      wrun[w][t] = acc;
      acc += x;
    }
    start[t] = c;
    gbase[t] = total;
  }
  if (next_totals != nullptr) {  // the next pass's digit totals, while the keys are in registers
#pragma unroll
    for (int i = 0; i < kOsItems; ++i)
      count_digit(nh, (uint32_t)(k[i] >> next_shift) & next_mask, base + (int64_t)i * 64 < n, lane);
  }
  __syncthreads();
  if (next_totals != nullptr && digit_lane && nh[t]) atomicAdd(&next_totals[t], nh[t]);
  for (int off = 1; off < kBins; off <<= 1) {  // inclusive scans: the tile's counts, the digit totals
    uint32_t x = 0, y = 0;
    if (digit_lane && t >= off) {
      x = start[t - off];
      y = gbase[t - off];
    }
    __syncthreads();
    if (digit_lane) {
      start[t] += x;
      gbase[t] += y;
    }
    __syncthreads();
  }
  // 4. decoupled look-back: this tile's keys of digit t go after every earlier tile's.  Each
  //    round polls the next kLookback predecessors at once (independent loads in flight, not one
  //    dependent hop per tile) and consumes them nearest first: aggregates add up, an inclusive
  //    count ends the walk, an unpublished word ends the round (polled again next round).
  if (digit_lane) {
    uint32_t before = 0;
    if (tile > 0) {
      int64_t j = (int64_t)tile - 1;  // the nearest predecessor not yet accounted for
      uint32_t spins = 0;
      for (;;) {
        uint32_t st[kLookback];
#pragma unroll
        for (int m = 0; m < kLookback; ++m)  // below tile 0: an empty inclusive count
          st[m] = j - m >= 0 ? poll_status(status + (j - m) * kBins + t) : kFlagIncl;
        bool live = true, done = false;
        int used = 0;
#pragma unroll
        for (int m = 0; m < kLookback; ++m) {  // predicated, so st[] stays in registers
          const uint32_t f = st[m] & ~kCountMask;
          const bool take = live && f != 0;    // f == 0: not published yet
          before += take ? (st[m] & kCountMask) : 0u;
          used = take ? m + 1 : used;
          done = done || (take && f == kFlagIncl);
          live = take && f != kFlagIncl;
        }
        if (done) break;
        if (used == 0) {  // no progress: back off, bounded
          if (++spins >= kSpinLimit) {
            atomicAdd(fault, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        j -= used;
      }
      publish_status(my, kFlagIncl | (before + c));
    }
    const uint32_t run_start = start[t] - c;
    const uint32_t out_start = gbase[t] - total + before;
    start[t] = run_start;  // only thread t reads or writes slot t in this phase
    gbase[t] = out_start;
  }
  __syncthreads();
  // 5. keys through LDS: digit-sorted into the exchange buffer, then out in tile order
  //    (consecutive positions of a digit's run go to consecutive addresses)
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const uint32_t d = (uint32_t)(k[i] >> shift) & mask;
    r[i] += start[d] + wrun[wave][d];  // r[i] is now the pair's slot in the digit-sorted tile
    if (base + (int64_t)i * 64 < n) xbuf[r[i]] = k[i];
  }
  __syncthreads();
  const int64_t left = n - tile0;
  const int here = left < kOsTile ? (int)left : kOsTile;
  uint32_t g[kOsItems];
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int p = i * kOsBlock + t;
    if (p < here) {
      const uint64_t key = xbuf[p];
      const uint32_t d = (uint32_t)(key >> shift) & mask;
      g[i] = gbase[d] + (uint32_t)p - start[d];
      kout[g[i]] = key;
    }
  }
  __syncthreads();
  // 6. rows the same way, through the same buffer
  int32_t* xv = reinterpret_cast<int32_t*>(xbuf);
#pragma unroll
  for (int i = 0; i < kOsItems; ++i)
    if (base + (int64_t)i * 64 < n) xv[r[i]] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kOsItems; ++i) {
    const int p = i * kOsBlock + t;
    if (p < here) vout[g[i]] = xv[p];
  }
}

// Up to kSmallKeys pairs (the top-k candidates of a radix select, small selections): every pass
// inside ONE workgroup, the pairs resident in LDS -- one launch instead of four per pass.  Per
// pass each thread takes its 16 pairs from LDS into registers, the waves rank them (as in
// tt_radix_scatter), and after a barrier every pair is written back to its digit-sorted slot.
constexpr int kSmallBlock = 512;                     // 8 waves
constexpr int kSmallWaves = kSmallBlock / 64;
constexpr int kSmallKeys = kSmallBlock * kSortItems;  // 8192

__global__ __launch_bounds__(kSmallBlock) void tt_radix_small(const uint64_t* __restrict__ kin,
                                                              const int32_t* __restrict__ vin,
                                                              uint64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                              int32_t n, int32_t end_bit) {
  __shared__ uint64_t sk[kSmallKeys];            // 64 KiB
  __shared__ int32_t sv[kSmallKeys];             // 32 KiB
  __shared__ uint32_t wrun[kSmallWaves][kBins];  // 8 KiB
  __shared__ uint32_t start[kBins];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  for (int i = t; i < n; i += kSmallBlock) {
    sk[i] = kin[i];
    sv[i] = vin[i];
  }
  const int base = wave * kWaveKeys + lane;  // this thread's pairs: base + 64 i
  for (int shift = 0; shift < end_bit; shift += 8) {
    const int bits = end_bit - shift < 8 ? end_bit - shift : 8;
    const uint32_t mask = (1u << bits) - 1u;
    for (int j = t; j < kSmallWaves * kBins; j += kSmallBlock) (&wrun[0][0])[j] = 0;
    __syncthreads();
    uint64_t k[kSortItems];
    int32_t v[kSortItems];
    uint32_t r[kSortItems];
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
      const int idx = base + i * 64;
      k[i] = idx < n ? sk[idx] : 0ull;
      v[i] = idx < n ? sv[idx] : 0;
    }
    uint32_t* run = wrun[wave];
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
      const bool valid = base + i * 64 < n;
      const uint32_t d = (uint32_t)(k[i] >> shift) & mask;
      const uint64_t eq = match_digit(d, valid, bits);
      const uint64_t below = eq & lanes_below(lane);
      r[i] = run_get(&run[d]) + (uint32_t)__popcll(below);
      __builtin_amdgcn_wave_barrier();
      if (valid && below == 0) run_set(&run[d], r[i] + (uint32_t)__popcll(eq));
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();  // every pair is in registers and ranked: LDS may be overwritten from here
    if (t < kBins) {  // per digit: the earlier waves' counts, and the digit's total
      uint32_t acc = 0;
#pragma unroll
      for (int w = 0; w < kSmallWaves; ++w) {
        const uint32_t x = wrun[w][t];
        wrun[w][t] = acc;
        acc += x;
      }
      start[t] = acc;
    }
    __syncthreads();
    for (int off = 1; off < kBins; off <<= 1) {  // inclusive scan of the digit totals
      uint32_t x = 0;
      if (t < kBins && t >= off) x = start[t - off];
      __syncthreads();
      if (t < kBins) start[t] += x;
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < kSortItems; ++i) {
      if (base + i * 64 < n) {
        const uint32_t d = (uint32_t)(k[i] >> shift) & mask;
        const uint32_t before = d ? start[d - 1] : 0u;  // inclusive scan -> the digit's start
        const uint32_t pos = before + wrun[wave][d] + r[i];
        sk[pos] = k[i];
        sv[pos] = v[i];
      }
    }
    __syncthreads();
  }
  for (int i = t; i < n; i += kSmallBlock) {
    kout[i] = sk[i];
    vout[i] = sv[i];
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
  int64_t tiles = 0;
  int passes = 0;
  size_t keys = 0, vals = 0, totals = 0, counters = 0, status = 0, zero_bytes = 0, total = 0;
};

inline int tile_items(int64_t n) { return n >= kBigTileMin ? 16 : 4; }

// The counts travel in 30 bits of a status word: n < 2^30.
inline bool layout(int64_t n, int32_t end_bit, Layout& L) {
  if (n <= 0 || n >= (int64_t)kCountMask || end_bit < 1 || end_bit > 64) return false;
  const int64_t tile = (int64_t)kOsBlock * tile_items(n);
  L.tiles = (n + tile - 1) / tile;
  L.passes = (end_bit + 7) / 8;
  L.keys = 0;
  L.vals = align256((size_t)n * sizeof(uint64_t));
  L.totals = L.vals + align256((size_t)n * sizeof(int32_t));  // zeroed per sort from here on
  L.counters = L.totals + align256((size_t)kMaxPasses * kBins * sizeof(uint32_t));
  L.status = L.counters + 256;
  L.total = L.status + align256((size_t)L.passes * L.tiles * kBins * sizeof(uint32_t));
  L.zero_bytes = L.total - L.totals;
  return true;
}

}  // namespace

extern "C" int64_t tt_sort_pairs_temp_bytes(int64_t n, int32_t end_bit) {
  Layout L;
  if (!layout(n, end_bit, L)) return -1;
  return (int64_t)L.total;
}

// keys/vals in -> out (distinct buffers), ascending by key bits [0, end_bit); stable.  `temp`
// (tt_sort_pairs_temp_bytes) holds the ping-pong copy, the digit totals, the tile counters and the
// look-back status words.  `fault` (device uint32) counts look-back spins that hit kSpinLimit:
// nonzero means the output is not to be trusted.
extern "C" int tt_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in, int32_t* vals_out,
                             int64_t n, int32_t end_bit, void* temp, int64_t temp_bytes, uint32_t* fault,
                             hipStream_t stream) {
  if (n <= 0) return 0;
  Layout L;
  if (temp == nullptr || fault == nullptr || !layout(n, end_bit, L) || temp_bytes < (int64_t)L.total) return -1;
  if (n <= kSmallKeys) {  // one workgroup, every pass in LDS
    hipLaunchKernelGGL(tt_radix_small, dim3(1), dim3(kSmallBlock), 0, stream, keys_in, vals_in, keys_out, vals_out,
                       (int32_t)n, end_bit);
    return (int)hipGetLastError();
  }
  uint8_t* tb = static_cast<uint8_t*>(temp);
  uint64_t* tk = reinterpret_cast<uint64_t*>(tb + L.keys);
  int32_t* tv = reinterpret_cast<int32_t*>(tb + L.vals);
  uint32_t* totals = reinterpret_cast<uint32_t*>(tb + L.totals);
  uint32_t* counters = reinterpret_cast<uint32_t*>(tb + L.counters);
  uint32_t* status = reinterpret_cast<uint32_t*>(tb + L.status);
  hipError_t e = hipMemsetAsync(tb + L.totals, 0, L.zero_bytes, stream);
  if (e != hipSuccess) return (int)e;
  const int64_t want = (n + kSortBlock * kTotalsItems - 1) / (kSortBlock * kTotalsItems);
  const unsigned tblocks = (unsigned)(want < kTotalsBlocks ? want : kTotalsBlocks);
  auto digit_mask = [end_bit](int shift) {
    const int bits = end_bit - shift < 8 ? end_bit - shift : 8;
    return (1u << bits) - 1u;
  };
  hipLaunchKernelGGL(tt_radix_totals, dim3(tblocks), dim3(kSortBlock), 0, stream, keys_in, n, digit_mask(0), totals);
  const uint64_t* src_k = keys_in;
  const int32_t* src_v = vals_in;
  for (int p = 0; p < L.passes; ++p) {
    const int shift = 8 * p;
    const uint32_t mask = digit_mask(shift);
    const bool last = p + 1 == L.passes;
    // the last pass writes the caller's output: alternate so that it does
    const bool to_out = ((L.passes - 1 - p) & 1) == 0;
    uint64_t* dk = to_out ? keys_out : tk;
    int32_t* dv = to_out ? vals_out : tv;
    auto kernel = tile_items(n) == 16 ? tt_radix_onesweep<16> : tt_radix_onesweep<4>;
    hipLaunchKernelGGL(kernel, dim3((unsigned)L.tiles), dim3(kOsBlock), 0, stream, src_k, src_v, dk, dv, n, shift,
                       mask, totals + p * kBins, last ? nullptr : totals + (p + 1) * kBins, shift + 8,
                       last ? 0u : digit_mask(shift + 8), status + (int64_t)p * L.tiles * kBins, counters + p, fault);
    src_k = dk;
    src_v = dv;
  }
  return (int)hipGetLastError();
}
