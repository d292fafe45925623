// Final ordering of query results: LSD radix sort of (packed ordering key, row id) pairs over
// only the key bits that can be set.
//
// tt_sort_keys packs [ranks | seq] into key_bits <= 63 bits (e.g. a 10-bit date rank + a
// 27-bit insertion sequence = 37 bits), so a pair sort over bits [0, key_bits) needs
// ceil(key_bits / 8) digit passes instead of the 8 an int64 argsort makes, and it moves the
// row ids with the keys -- no argsort index plus gather of the rows afterwards.  rocPRIM's
// onesweep radix sort (through hipCUB) is the engine; this file only fixes the bit range and
// the key/value types for the query path.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <hipcub/device/device_radix_sort.hpp>

extern "C" int64_t tt_sort_pairs_temp_bytes(int64_t n, int32_t end_bit) {
  if (n <= 0 || n > INT32_MAX || end_bit < 1 || end_bit > 64) return -1;
  size_t bytes = 0;
  const hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const uint64_t*>(nullptr),
                                                          static_cast<uint64_t*>(nullptr),
                                                          static_cast<const int32_t*>(nullptr),
                                                          static_cast<int32_t*>(nullptr), (int)n, 0, end_bit);
  return e == hipSuccess ? (int64_t)bytes : -1;
}

// keys/vals in -> out (distinct buffers), ascending by key bits [0, end_bit); stable.
extern "C" int tt_sort_pairs(const uint64_t* keys_in, uint64_t* keys_out, const int32_t* vals_in, int32_t* vals_out,
                             int64_t n, int32_t end_bit, void* temp, int64_t temp_bytes, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > INT32_MAX || end_bit < 1 || end_bit > 64 || temp == nullptr || temp_bytes <= 0) return -1;
  size_t bytes = (size_t)temp_bytes;
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                                 end_bit, stream);
}
