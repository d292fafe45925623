// Final ordering of query results: a stable LSD radix sort of (packed ordering key, row id)
// pairs over only the key bits that can be set (ops/gpu.py GpuKernels._sorted_rows).
//
// tt_sort_keys packs [ranks | seq] into key_bits <= 63 bits (e.g. a 10-bit date rank + a
// 27-bit insertion sequence = 37 bits), so the sort needs ceil(key_bits / 8) digit passes
// instead of the 8 an int64 argsort makes, and it moves the row ids with the keys -- no argsort
// index plus gather of the rows afterwards.
//
// One pass = three launches, no inter-workgroup waiting (nothing spins on another workgroup's
// flag, so every wave of every launch runs to completion on its own):
//   tt_radix_hist     per tile of 2048 keys, the count of each 8-bit digit (wave-aggregated:
//                     a 64-lane digit match from 8 ballots, one LDS add per distinct digit per
//                     wave), stored digit-major: counts[d * tiles + t];
//   tt_radix_scan     exclusive scan of the digit-major counts (4096 per workgroup, the chunk
//                     totals scanned by a second, single-workgroup launch): offs[d * tiles + t]
//                     is where tile t's keys of digit d start in the output;
//   tt_radix_scatter  stable scatter: per 256-key step, each wave ranks its keys among equal
//                     digits with the same ballot match (popcount of the lanes below), the waves'
//                     counts are combined in LDS in wave order, and the keys land digit-sorted in
//                     an LDS tile; then they are written out tile-order, so consecutive threads
//                     write consecutive addresses within each digit's run.
// Wave64 throughout (64-bit ballots, __launch_bounds__(256) = 4 waves per workgroup).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kBins = 256;                      // 8-bit digits
constexpr int kSortBlock = 256;                 // 4 waves of 64
constexpr int kSortItems = 8;                   // keys per thread per tile
constexpr int kSortTile = kSortBlock * kSortItems;  // 2048 keys per workgroup
constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanChunk = kScanBlock * kScanItems;  // 4096 counts per scan workgroup
constexpr int kPartialBlock = 1024;
constexpr int kMaxPartials = kPartialBlock * kScanItems;  // chunks the one-workgroup scan covers

// Lanes of this wave whose (valid) digit equals this lane's: 8 ballots, one per digit bit.
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t on = __ballot(bit);
    m &= bit ? on : ~on;
  }
  return m;
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__global__ __launch_bounds__(kSortBlock) void tt_radix_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                            uint32_t mask, uint32_t* __restrict__ counts,
                                                            int64_t tiles) {
  __shared__ uint32_t h[kBins];
  const int t = threadIdx.x, lane = t & 63;
  h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int64_t idx = base + (int64_t)i * kSortBlock + t;
    const bool valid = idx < n;
    const uint32_t d = valid ? (uint32_t)(keys[idx] >> shift) & mask : 0u;
    const uint64_t eq = match_digit(d, valid);
    if (valid && (eq & lanes_below(lane)) == 0) atomicAdd(&h[d], (uint32_t)__popcll(eq));  // the digit's first lane
  }
  __syncthreads();
  counts[(int64_t)t * tiles + blockIdx.x] = h[t];
}

// Exclusive scan of one 4096-count chunk (in -> out); the chunk total goes to partial[chunk].
__global__ __launch_bounds__(kScanBlock) void tt_radix_scan_chunks(const uint32_t* __restrict__ in,
                                                                   uint32_t* __restrict__ out, int64_t m,
                                                                   uint32_t* __restrict__ partial) {
  __shared__ uint32_t s[kScanBlock];
  const int t = threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.x * kScanChunk + (int64_t)t * kScanItems;
  uint32_t v[kScanItems], sum = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = c0 + i < m ? in[c0 + i] : 0u;
    sum += v[i];
  }
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < kScanBlock; off <<= 1) {  // Hillis-Steele inclusive scan of the thread sums
    const uint32_t x = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (c0 + i < m) out[c0 + i] = run;
    run += v[i];
  }
  if (t == kScanBlock - 1) partial[blockIdx.x] = s[t];
}

// Exclusive scan of the chunk totals in place (one workgroup, up to kMaxPartials of them).
__global__ __launch_bounds__(kPartialBlock) void tt_radix_scan_partials(uint32_t* __restrict__ partial, int32_t p) {
  __shared__ uint32_t s[kPartialBlock];
  const int t = threadIdx.x;
  const int c0 = t * kScanItems;
  uint32_t v[kScanItems], sum = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = c0 + i < p ? partial[c0 + i] : 0u;
    sum += v[i];
  }
  s[t] = sum;
  __syncthreads();
  for (int off = 1; off < kPartialBlock; off <<= 1) {
    const uint32_t x = t >= off ? s[t - off] : 0u;
    __syncthreads();
    s[t] += x;
    __syncthreads();
  }
  uint32_t run = s[t] - sum;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (c0 + i < p) partial[c0 + i] = run;
    run += v[i];
  }
}

__global__ __launch_bounds__(kSortBlock) void tt_radix_scatter(const uint64_t* __restrict__ kin,
                                                               const int32_t* __restrict__ vin,
                                                               uint64_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                               int64_t n, int shift, uint32_t mask,
                                                               const uint32_t* __restrict__ counts,
                                                               const uint32_t* __restrict__ offs,
                                                               const uint32_t* __restrict__ partial, int64_t tiles) {
  __shared__ uint64_t sk[kSortTile];       // the tile, digit-sorted (16 KiB)
  __shared__ int32_t sv[kSortTile];        // 8 KiB
  __shared__ uint32_t start[kBins];        // tile-local start of each digit's run
  __shared__ uint32_t run[kBins];          // keys of each digit placed so far
  __shared__ uint32_t gbase[kBins];        // where the tile's run of each digit starts in the output
  __shared__ uint32_t wc[kSortBlock / 64][kBins];  // this step's count per (wave, digit)
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  const int64_t cell = (int64_t)t * tiles + blockIdx.x;
  const uint32_t c = counts[cell];
  gbase[t] = offs[cell] + partial[cell / kScanChunk];
  run[t] = 0;
#pragma unroll
  for (int w = 0; w < kSortBlock / 64; ++w) wc[w][t] = 0;
  start[t] = c;
  __syncthreads();
  for (int off = 1; off < kBins; off <<= 1) {  // exclusive scan of the tile's digit counts
    const uint32_t x = t >= off ? start[t - off] : 0u;
    __syncthreads();
    start[t] += x;
    __syncthreads();
  }
  start[t] -= c;
  __syncthreads();
  for (int i = 0; i < kSortItems; ++i) {
    const int64_t idx = base + (int64_t)i * kSortBlock + t;
    const bool valid = idx < n;
    const uint64_t k = valid ? kin[idx] : 0ull;
    const int32_t v = valid ? vin[idx] : 0;
    const uint32_t d = (uint32_t)(k >> shift) & mask;
    const uint64_t eq = match_digit(d, valid);
    const uint64_t below = eq & lanes_below(lane);
    if (valid && below == 0) wc[wave][d] = (uint32_t)__popcll(eq);
    __syncthreads();
    if (valid) {
      uint32_t pos = start[d] + run[d] + (uint32_t)__popcll(below);
      for (int w = 0; w < wave; ++w) pos += wc[w][d];  // earlier waves' keys of this digit (input order)
      sk[pos] = k;
      sv[pos] = v;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < kSortBlock / 64; ++w) {
      add += wc[w][t];
      wc[w][t] = 0;
    }
    run[t] += add;
    __syncthreads();
  }
  const int64_t left = n - base;
  const int here = left < kSortTile ? (int)left : kSortTile;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int p = i * kSortBlock + t;
    if (p < here) {
      const uint64_t k = sk[p];
      const uint32_t d = (uint32_t)(k >> shift) & mask;
      const uint32_t g = gbase[d] + (uint32_t)p - start[d];
      kout[g] = k;
      vout[g] = sv[p];
    }
  }
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
  int64_t tiles = 0, m = 0;
  int32_t chunks = 0;
  size_t keys = 0, vals = 0, counts = 0, offs = 0, partial = 0, total = 0;
};

inline bool layout(int64_t n, Layout& L) {
  if (n <= 0 || n > INT32_MAX) return false;
  L.tiles = (n + kSortTile - 1) / kSortTile;
  L.m = L.tiles * kBins;
  const int64_t chunks = (L.m + kScanChunk - 1) / kScanChunk;
  if (chunks > kMaxPartials) return false;
  L.chunks = (int32_t)chunks;
  L.keys = 0;
  L.vals = align256((size_t)n * sizeof(uint64_t));
  L.counts = L.vals + align256((size_t)n * sizeof(int32_t));
  L.offs = L.counts + align256((size_t)L.m * sizeof(uint32_t));
  L.partial = L.offs + align256((size_t)L.m * sizeof(uint32_t));
  L.total = L.partial + align256((size_t)L.chunks * sizeof(uint32_t));
  return true;
}

}  // namespace

extern "C" int64_t tt_sort_pairs_temp_bytes(int64_t n, int32_t end_bit) {
  Layout L;
  if (end_bit < 1 || end_bit > 64 || !layout(n, L)) return -1;
  return (int64_t)L.total;
}

// keys/vals in -> out (distinct buffers), ascending by key bits [0, end_bit); stable.  `temp`
// (tt_sort_pairs_temp_bytes) holds the ping-pong copy and the digit counts.
extern "C" int tt_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in, int32_t* vals_out,
                             int64_t n, int32_t end_bit, void* temp, int64_t temp_bytes, hipStream_t stream) {
  if (n <= 0) return 0;
  Layout L;
  if (end_bit < 1 || end_bit > 64 || temp == nullptr || !layout(n, L) || temp_bytes < (int64_t)L.total) return -1;
  uint8_t* tb = static_cast<uint8_t*>(temp);
  uint64_t* tk = reinterpret_cast<uint64_t*>(tb + L.keys);
  int32_t* tv = reinterpret_cast<int32_t*>(tb + L.vals);
  uint32_t* counts = reinterpret_cast<uint32_t*>(tb + L.counts);
  uint32_t* offs = reinterpret_cast<uint32_t*>(tb + L.offs);
  uint32_t* partial = reinterpret_cast<uint32_t*>(tb + L.partial);
  const int passes = (end_bit + 7) / 8;
  const uint64_t* src_k = keys_in;
  const int32_t* src_v = vals_in;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    const int bits = end_bit - shift < 8 ? end_bit - shift : 8;
    const uint32_t mask = (1u << bits) - 1u;
    // the last pass writes the caller's output: alternate so that it does
    const bool to_out = ((passes - 1 - p) & 1) == 0;
    uint64_t* dk = to_out ? keys_out : tk;
    int32_t* dv = to_out ? vals_out : tv;
    hipLaunchKernelGGL(tt_radix_hist, dim3((unsigned)L.tiles), dim3(kSortBlock), 0, stream, src_k, n, shift, mask,
                       counts, L.tiles);
    hipLaunchKernelGGL(tt_radix_scan_chunks, dim3((unsigned)L.chunks), dim3(kScanBlock), 0, stream, counts, offs, L.m,
                       partial);
    hipLaunchKernelGGL(tt_radix_scan_partials, dim3(1), dim3(kPartialBlock), 0, stream, partial, L.chunks);
    hipLaunchKernelGGL(tt_radix_scatter, dim3((unsigned)L.tiles), dim3(kSortBlock), 0, stream, src_k, src_v, dk, dv, n,
                       shift, mask, counts, offs, partial, L.tiles);
    src_k = dk;
    src_v = dv;
  }
  return (int)hipGetLastError();
}
