// Batched segment copy for the HBM trajectory ring: assembles a padded learner batch
// from trajectory blobs already resident in HBM.  Each segment copies `nbytes` from
// arena + src_off to out + dst_off (destination pre-filled with the padding value), so one launch
// gathers every leaf of every step of every trajectory in the batch (tens of thousands of rows).
// One workgroup per segment (grid-stride); 16 B vector copies when both ends and the length are
// 16-B aligned, 4 B when 4-B aligned, bytes otherwise.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

__global__ __launch_bounds__(256) void segment_copy_kernel(const uint8_t* __restrict__ arena, uint8_t* __restrict__ out,
                                                           const int64_t* __restrict__ seg, long nseg) {
  for (long s = blockIdx.x; s < nseg; s += gridDim.x) {
    const int64_t src = seg[3 * s], dst = seg[3 * s + 1], n = seg[3 * s + 2];
#ifdef AS_DEBUG
    assert(src >= 0 && dst >= 0 && n >= 0);
#endif
    const uint8_t* a = arena + src;
    uint8_t* o = out + dst;
    if (((src | dst | n) & 15) == 0) {
      const uint4* a4 = reinterpret_cast<const uint4*>(a);
      uint4* o4 = reinterpret_cast<uint4*>(o);
      for (long i = threadIdx.x; i < n / 16; i += blockDim.x) o4[i] = a4[i];
    } else if (((src | dst | n) & 3) == 0) {
      const uint32_t* a1 = reinterpret_cast<const uint32_t*>(a);
      uint32_t* o1 = reinterpret_cast<uint32_t*>(o);
      for (long i = threadIdx.x; i < n / 4; i += blockDim.x) o1[i] = a1[i];
    } else {
      for (long i = threadIdx.x; i < n; i += blockDim.x) o[i] = a[i];
    }
  }
}

}  // namespace

void segment_copy(const uint8_t* arena, uint8_t* out, const int64_t* seg, long nseg, hipStream_t s) {
  if (nseg <= 0) return;
  const long grid = nseg < 65536 ? nseg : 65536;
  hipLaunchKernelGGL(segment_copy_kernel, dim3(grid), dim3(256), 0, s, arena, out, seg, nseg);
}

}  // namespace as
