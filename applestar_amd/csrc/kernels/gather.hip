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

// Input-gradient weight of a 3x3 conv: out[ci][ky][kx][co] = w[co][ci][2-ky][2-kx] (bf16), read through
// w's strides so contiguous and channels_last weights both work.  Replaces flip + permute + contiguous
// (two launches) with one; each thread writes one output element, consecutive threads consecutive co.
namespace as {
namespace {
__global__ __launch_bounds__(256) void conv_wt_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ out,
                                                      int cout, int cin, long s0, long s1, long s2, long s3) {
  const long n = (long)cout * cin * 9;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % cout);
    const long r = i / cout;              // (ci*3 + ky)*3 + kx
    const int kx = (int)(r % 3), ky = (int)((r / 3) % 3), ci = (int)(r / 9);
    out[i] = w[co * s0 + ci * s1 + (2 - ky) * s2 + (2 - kx) * s3];
  }
}
}  // namespace

void conv_wt(const uint16_t* w, uint16_t* out, int cout, int cin, long s0, long s1, long s2, long s3,
             hipStream_t s) {
  const long n = (long)cout * cin * 9;
  if (n <= 0) return;
  long grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(conv_wt_kernel, dim3(grid), dim3(256), 0, s, w, out, cout, cin, s0, s1, s2, s3);
}
}  // namespace as
