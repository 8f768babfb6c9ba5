// Decode-step input staging on the compute queue.
//
// Each decode step uploads a packed pinned host buffer (token ids, positions,
// KV slots, sampling params, block tables) into the device twin the captured
// decode graphs read.  A hipMemcpyAsync H2D of pinned memory is handed to an
// SDMA engine; the compute queue then waits on the SDMA completion signal,
// and the profile of the serving bench showed 190-330 us of GPU idle between
// the previous step's sampler and the next graph's first kernel on every step
// (profiles/r3/gaps_ws_bench.md).  This kernel instead reads the mapped
// pinned buffer directly over the host link from the compute queue, and only
// the bytes the step's graph bucket reads: the scalar sections plus rows
// [0, rows) x columns [0, row_bytes) of the block table -- ~80 KB instead of
// the whole 530 KB staging buffer.
//
// Layout contract (checked on the host): every offset/size is a multiple of
// 16 B; `src` is a device-visible pointer of a pinned (hipHostMalloc'd) buffer.
#include "common.h"

using namespace omnia;

namespace {

// grid-stride copy of 16-B items: [0, head) then `rows` strided row segments
__global__ __launch_bounds__(256) void stage_copy_kernel(uint4v* __restrict__ dst,
                                                         const uint4v* __restrict__ src,
                                                         int head, int bt_off, int stride,
                                                         int rows, int row_items) {
  const int total = head + rows * row_items;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int o = i;
    if (i >= head) {
      const int j = i - head;
      const int r = j / row_items;
      o = bt_off + r * stride + (j - r * row_items);
    }
    dst[o] = __builtin_nontemporal_load(src + o);
  }
}

}  // namespace

extern "C" {

// all sizes in bytes; returns a hipError_t
int omnia_stage_copy(void* dst, const void* src, int64_t head_bytes, int64_t bt_off,
                     int64_t row_stride, int rows, int64_t row_bytes, hipStream_t s) {
  if ((head_bytes | bt_off | row_stride | row_bytes) & 15) return (int)hipErrorInvalidValue;
  if (rows < 0 || head_bytes < 0 || row_bytes < 0 || head_bytes > bt_off ||
      (rows > 0 && row_bytes > row_stride))
    return (int)hipErrorInvalidValue;
  const int64_t items = head_bytes / 16 + (int64_t)rows * (row_bytes / 16);
  if (items == 0) return 0;
  if (bt_off / 16 + (int64_t)rows * (row_stride / 16) > (int64_t)1 << 30)
    return (int)hipErrorInvalidValue;
  // enough 16-B loads in flight to cover host-link latency, never more blocks
  // than items
  const int blocks = (int)std::min<int64_t>((items + 255) / 256, 128);
  hipLaunchKernelGGL(stage_copy_kernel, dim3(blocks), dim3(256), 0, s,
                     reinterpret_cast<uint4v*>(dst), reinterpret_cast<const uint4v*>(src),
                     (int)(head_bytes / 16), (int)(bt_off / 16), (int)(row_stride / 16), rows,
                     (int)(row_bytes / 16));
  return (int)hipGetLastError();
}

// device-visible address of a pinned host allocation (0 if it is not mapped)
int64_t omnia_host_device_ptr(void* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return reinterpret_cast<int64_t>(d);
}

}  // extern "C"
