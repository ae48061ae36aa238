// Conv-epilogue backward: dpre = dout * (out > 0) (ReLU) or dpre = dout, as contiguous NHWC bf16 - the
// A operand of the dX implicit-GEMM conv and of the split-R weight-gradient kernel.
//
// The incoming gradient arrives either NHWC-contiguous (from another NHWC kernel) or NCHW-contiguous (from
// a torch op on the [B,C,H,W] view), in fp32 or bf16.  Previously this was compare + mul + cast +
// contiguous: four torch passes, two of them strided (rocprof r1_v11: ~3 ms/step).  One pass here:
//   * NHWC input: 8 channels per thread, 16-B loads of out, one 16-B store;
//   * NCHW input: 64-pixel x 32-channel tiles transposed through LDS (coalesced reads along the pixel
//     axis, coalesced 16-B writes along the channel axis).
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <typename T>
__device__ __forceinline__ void load8f(const T* p, float* v);
template <>
__device__ __forceinline__ void load8f<float>(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <>
__device__ __forceinline__ void load8f<bf16_t>(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* v) {
  uint4 u;
  u.x = f2bf2(v[0], v[1]);
  u.y = f2bf2(v[2], v[3]);
  u.z = f2bf2(v[4], v[5]);
  u.w = f2bf2(v[6], v[7]);
  return u;
}

template <typename T>
__global__ __launch_bounds__(256) void act_grad_nhwc_kernel(const T* __restrict__ dout, const bf16_t* __restrict__ out,
                                                            bf16_t* __restrict__ dpre, long n8, int relu) {
  const long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n8) return;
  float v[8];
  load8f<T>(dout + 8 * i, v);
  if (relu) {
    float o[8];
    load8f<bf16_t>(out + 8 * i, o);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = o[e] > 0.f ? v[e] : 0.f;
  }
  *reinterpret_cast<uint4*>(dpre + 8 * i) = pack8(v);
}

// grid (ceil(HW / 64), C / 32, B); dout NCHW [B, C, HW], out / dpre NHWC [B, HW, C]
template <typename T>
__global__ __launch_bounds__(256) void act_grad_nchw_kernel(const T* __restrict__ dout, const bf16_t* __restrict__ out,
                                                            bf16_t* __restrict__ dpre, int C, int HW, int relu) {
  __shared__ float tile[32][65];
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 32;
  const long b = blockIdx.z;
  const int tid = threadIdx.x;
  // read: 32 channel rows x 64 pixels, 8 rows per pass (64 lanes along pixels)
  {
    const int px = tid & 63, cr = tid >> 6;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cr + 4 * k;
      const int p = p0 + px;
      tile[c][px] = p < HW ? Cvt<T>::load(dout, (b * C + c0 + c) * HW + p) : 0.f;
    }
  }
  __syncthreads();
  // write: 64 pixels x 4 chunks of 8 channels = 256 threads, one 16-B store each
  const int p = p0 + (tid >> 2), ch = (tid & 3) * 8;
  if (p >= HW) return;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = tile[ch + e][tid >> 2];
  const long o = (b * HW + p) * C + c0 + ch;
  if (relu) {
    float m[8];
    load8f<bf16_t>(out + o, m);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
  }
  *reinterpret_cast<uint4*>(dpre + o) = pack8(v);
}

}  // namespace

void act_grad_nhwc(const void* dout, int dt, bool dout_nchw, const void* out, void* dpre, int B, int C, int HW, int relu,
                   hipStream_t s) {
  const bf16_t* o = static_cast<const bf16_t*>(out);
  bf16_t* d = static_cast<bf16_t*>(dpre);
  if (!dout_nchw) {
    const long n8 = static_cast<long>(B) * HW * C / 8;
    const unsigned g = static_cast<unsigned>((n8 + 255) / 256);
    if (dt == DT_F32)
      hipLaunchKernelGGL(act_grad_nhwc_kernel<float>, dim3(g), dim3(256), 0, s, static_cast<const float*>(dout), o, d, n8,
                         relu);
    else
      hipLaunchKernelGGL(act_grad_nhwc_kernel<bf16_t>, dim3(g), dim3(256), 0, s, static_cast<const bf16_t*>(dout), o, d,
                         n8, relu);
    return;
  }
  const dim3 grid((HW + 63) / 64, C / 32, B);
  if (dt == DT_F32)
    hipLaunchKernelGGL(act_grad_nchw_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(dout), o, d, C, HW,
                       relu);
  else
    hipLaunchKernelGGL(act_grad_nchw_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(dout), o, d, C,
                       HW, relu);
}

}  // namespace as
