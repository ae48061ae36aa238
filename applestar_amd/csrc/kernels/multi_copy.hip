// Multi-tensor copy with dtype conversion: a few launches move every parameter gradient into its slot of
// a flat (bucket / fp32 master) buffer.  The gradient list of an RL step has ~470 tensors; copied one by
// one that is ~470 hipMemcpy / elementwise launches (rocprof r1_v13: 770 copyBuffer calls, 1.9 ms).
// Up to kCopyMaxT tensors travel BY VALUE in the kernel arguments (no host->device table upload, which
// would put a synchronising copy in the middle of the step); workgroup b finds its tensor by scanning
// the chunk prefix sums and copies one chunk of <= kCopyChunk elements.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

// element i of a converting copy's source: fp32, bf16, or an integer feature column (uint8 / int16, exact in fp32)
__device__ __forceinline__ float copy_src(const void* src, long i, unsigned char dts) {
  if (dts & 8) return static_cast<float>(static_cast<const unsigned char*>(src)[i]);
  if (dts & 16) return static_cast<float>(static_cast<const short*>(src)[i]);
  return (dts & 1) ? static_cast<const float*>(src)[i] : bf2f(static_cast<const bf16_t*>(src)[i]);
}

__global__ __launch_bounds__(256) void multi_copy_kernel(const CopyArgs a) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < a.ntensors && a.chunk_start[t + 1] <= b) ++t;
  const void* src = a.src[t];
  void* dst = a.dst[t];
  if (a.dts[t] & 4) {
    // raw bytes (any dtype, n in bytes): 16-byte words when both ends and the length are 16-aligned
    const long i0 = static_cast<long>(b - a.chunk_start[t]) * kCopyRawChunk;
    const long i1 = i0 + kCopyRawChunk < a.n[t] ? i0 + kCopyRawChunk : a.n[t];
    const auto* s8 = static_cast<const unsigned char*>(src);
    auto* d8 = static_cast<unsigned char*>(dst);
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | a.n[t]) & 15) == 0) {
      // a full chunk: each thread's 16-B words all loaded before any is stored (one memory latency per chunk; the
      // dependent load -> store loop over 64-KB chunks moved the step's 126 MB of gradients at ~0.5 TB/s)
      constexpr int U = static_cast<int>(kCopyRawChunk / (16 * 256));
      if (i1 - i0 == kCopyRawChunk) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(s8 + i0 + 16 * (threadIdx.x + 256 * u));
#pragma unroll
        for (int u = 0; u < U; ++u) *reinterpret_cast<uint4*>(d8 + i0 + 16 * (threadIdx.x + 256 * u)) = v[u];
        return;
      }
      for (long i = i0 + 16 * threadIdx.x; i < i1; i += 16 * 256)
        *reinterpret_cast<uint4*>(d8 + i) = *reinterpret_cast<const uint4*>(s8 + i);
    } else {
      for (long i = i0 + threadIdx.x; i < i1; i += 256) d8[i] = s8[i];
    }
    return;
  }
  const long i0 = static_cast<long>(b - a.chunk_start[t]) * kCopyChunk;
  const long i1 = i0 + kCopyChunk < a.n[t] ? i0 + kCopyChunk : a.n[t];
  const bool df = (a.dts[t] & 2) != 0;
  const unsigned char dts = a.dts[t];
  if (i1 - i0 == kCopyChunk) {
    // a full chunk: the thread's 32 elements loaded before any is stored (see the raw path)
    constexpr int U = static_cast<int>(kCopyChunk / 256);
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = copy_src(src, i0 + threadIdx.x + 256 * u, dts);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + threadIdx.x + 256 * u;
      if (df) static_cast<float*>(dst)[i] = v[u];
      else static_cast<bf16_t*>(dst)[i] = f2bf(v[u]);
    }
    return;
  }
  for (long i = i0 + threadIdx.x; i < i1; i += 256) {
    const float v = copy_src(src, i, dts);
    if (df) static_cast<float*>(dst)[i] = v;
    else static_cast<bf16_t*>(dst)[i] = f2bf(v);
  }
}


__global__ __launch_bounds__(256) void strided_copy_kernel(const StridedCopyArgs a) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < a.ntensors && a.chunk_start[t + 1] <= b) ++t;
  const int i0 = (b - a.chunk_start[t]) * static_cast<int>(kCopyChunk);
  const int i1 = i0 + static_cast<int>(kCopyChunk) < a.n[t] ? i0 + static_cast<int>(kCopyChunk) : a.n[t];
  const bool sf = (a.dts[t] & 1) != 0, df = (a.dts[t] & 2) != 0;
  if (a.dts[t] & 4) {
    // transpose form (dst [R, Cc] from src element (r, c) at base + r + c * S): a 64 x 128 tile through LDS,
    // read along r and written along c, both coalesced (the per-element path reads one row per lane)
    __shared__ float tile[128][65];
    const int R = a.size[t][2], Cc = a.size[t][3];
    const long S = a.stride[t][3];
    const int tiles_c = (Cc + 127) / 128, tb = b - a.chunk_start[t];
    const int r0 = (tb / tiles_c) * 64, c0 = (tb % tiles_c) * 128;
    for (int i = threadIdx.x; i < 128 * 64; i += 256) {
      const int cc = i >> 6, rr = i & 63, r = r0 + rr, c = c0 + cc;
      float v = 0.f;
      if (r < R && c < Cc) {
        const long off = a.base[t] + r + c * S;
        v = sf ? static_cast<const float*>(a.src[t])[off] : bf2f(static_cast<const bf16_t*>(a.src[t])[off]);
      }
      tile[cc][rr] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 128; i += 256) {
      const int rr = i >> 7, cc = i & 127, r = r0 + rr, c = c0 + cc;
      if (r < R && c < Cc) {
        const long o = static_cast<long>(r) * Cc + c;
        if (df) static_cast<float*>(a.dst[t])[o] = tile[cc][rr];
        else static_cast<bf16_t*>(a.dst[t])[o] = f2bf(tile[cc][rr]);
      }
    }
    return;
  }
  const int s1 = a.size[t][1], s2 = a.size[t][2], s3 = a.size[t][3];
  const long st0 = a.stride[t][0], st1 = a.stride[t][1], st2 = a.stride[t][2], st3 = a.stride[t][3];
  const void* src = a.src[t];
  void* dst = a.dst[t];
  constexpr int U = 8;   // loads of a pass issued before its stores
  for (int i = i0 + threadIdx.x; i < i1; i += 256 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + 256 * u;
      if (j < i1) {
        int r = j;
        const int c3 = r % s3;
        r /= s3;
        const int c2 = r % s2;
        r /= s2;
        const int c1 = r % s1;
        const int c0 = r / s1;
        const long off = a.base[t] + c0 * st0 + c1 * st1 + c2 * st2 + c3 * st3;
        v[u] = sf ? static_cast<const float*>(src)[off] : bf2f(static_cast<const bf16_t*>(src)[off]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + 256 * u;
      if (j < i1) {
        if (df) static_cast<float*>(dst)[j] = v[u];
        else static_cast<bf16_t*>(dst)[j] = f2bf(v[u]);
      }
    }
  }
}

}  // namespace

void multi_copy(const CopyArgs& a, hipStream_t s) {
  const int nblk = a.chunk_start[a.ntensors];
  if (nblk > 0) hipLaunchKernelGGL(multi_copy_kernel, dim3(nblk), dim3(256), 0, s, a);
}

__global__ __launch_bounds__(256) void col_sum_kernel(const ColSumArgs a) {
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < a.npieces && a.block_start[p + 1] <= b) ++p;
  const long n = a.rows * a.width[p];
  const int w = a.width[p], ns = a.nsrc[p];
  for (long i = static_cast<long>(b - a.block_start[p]) * 256 + threadIdx.x; i < n;
       i += static_cast<long>(a.block_start[p + 1] - a.block_start[p]) * 256) {
    const long r = i / w;
    const int c = static_cast<int>(i - r * w);
    float v = a.src[p][0][r * a.sld[p][0] + a.soff[p][0] + c];
    if (ns > 1) v += a.src[p][1][r * a.sld[p][1] + a.soff[p][1] + c];
    if (ns > 2) v += a.src[p][2][r * a.sld[p][2] + a.soff[p][2] + c];
    a.dst[p][r * a.dld[p] + a.doff[p] + c] = v;
  }
}

void col_sum(const ColSumArgs& a, hipStream_t s) {
  const int nblk = a.block_start[a.npieces];
  if (nblk > 0) hipLaunchKernelGGL(col_sum_kernel, dim3(nblk), dim3(256), 0, s, a);
}

void multi_strided_copy(const StridedCopyArgs& a, hipStream_t s) {
  const int nblk = a.chunk_start[a.ntensors];
  if (nblk > 0) hipLaunchKernelGGL(strided_copy_kernel, dim3(nblk), dim3(256), 0, s, a);
}

}  // namespace as
