// One launch per mirror sync (ops/columnar.py ColumnarIndex.to_device, backing/accel.py's
// background sync): the rows appended to the column mirror since the last sync -- every
// column's codes, the insertion sequence, the liveness words, the sort plan's rank tails -- are
// staged by the host in ONE pinned, coherent, device-mapped buffer (the same mailbox memory the
// page path uses) together with a segment table, and this kernel writes each segment to its
// device buffer.  No copy kernels and no DMA setups per segment: before this, a sync issued
// ~8 hipMemcpyAsync (copyBuffer) calls, and the headline's kernel trace held more copy time than
// query-kernel time (profiles/r4_headline_kernels.md).
//
// Staging layout (all offsets in bytes from the buffer's start, every segment's source 16-byte
// aligned by the host): the segment table, then the payloads.  Reads cross the host link once
// per 16-byte unit (global_load_dwordx4 from mapped memory); writes go to HBM with the widest
// store the destination's alignment allows.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

struct Segment {
  int64_t src;    // payload offset in the staging buffer (multiple of 16)
  uint64_t dst;   // device address
  int64_t bytes;
};

constexpr int kBlock = 256;              // 4 wave64 per workgroup
constexpr int64_t kChunk = kBlock * 16;  // bytes per workgroup per segment: one 16-byte unit a lane

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock)
tt_scatter_segments(const uint8_t* __restrict__ staging, const Segment* __restrict__ segs, int32_t nsegs) {
  const int32_t s = (int32_t)blockIdx.y;
  if (s >= nsegs) return;
  const Segment g = segs[s];
  const int64_t at = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * 16;
  if (at >= g.bytes) return;
  const uint8_t* src = staging + g.src + at;
  uint8_t* dst = reinterpret_cast<uint8_t*>(g.dst) + at;
  const int64_t n = g.bytes - at < 16 ? g.bytes - at : 16;
  if (n == 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(src);  // the source is 16-byte aligned
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    if ((a & 15) == 0) {
      *reinterpret_cast<uint4*>(dst) = v;
    } else if ((a & 3) == 0) {
      uint32_t* d = reinterpret_cast<uint32_t*>(dst);
      d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      for (int i = 0; i < 16; ++i) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
    return;
  }
  for (int64_t i = 0; i < n; ++i) dst[i] = src[i];  // the segment's last partial unit
}

// `staging_dev`: the device view of the pinned buffer; `table_off`: where the segment table
// starts in it; `max_bytes`: the largest segment (sizes the grid).  Returns hipError_t.
extern "C" int tt_launch_scatter_segments(const void* staging_dev, int64_t table_off, int32_t nsegs, int64_t max_bytes,
                                          hipStream_t stream) {
  if (nsegs <= 0 || max_bytes <= 0) return 0;
  if (nsegs > 65535 || table_off < 0 || (table_off & 15)) return -1;
  const int64_t chunks = (max_bytes + kChunk - 1) / kChunk;
  if (chunks > 0x7fffffff) return -1;
  const uint8_t* base = static_cast<const uint8_t*>(staging_dev);
  hipLaunchKernelGGL(tt_scatter_segments, dim3((unsigned)chunks, (unsigned)nsegs), dim3(kBlock), 0, stream, base,
                     reinterpret_cast<const Segment*>(base + table_off), nsegs);
  return (int)hipGetLastError();
}
