// Fused elementwise tails.
//
// gated_residual: the location head's GatedResBlock output  relu(tanh(y * sigmoid(g)) * sp + x)
// (module_utils.py:224-231) — 5 torch kernels + 4 temporaries per block in the reference, one pass
// here; the backward recomputes sigmoid/tanh from y, g and writes dy, dg, dx plus per-block partial
// sums for d(sp) in one pass.  ``post``: a tensor added to the block output in the same pass (the location head
// adds the next encoder skip map to every block's output); the backward then takes the ReLU mask from the
// recomputed pre-activation (``xin`` = the block input) instead of the saved output.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void gated_residual_fwd_kernel(const T* __restrict__ y, const T* __restrict__ g,
                                                                 const float* __restrict__ sp, const T* __restrict__ x,
                                                                 const T* __restrict__ post, T* __restrict__ out,
                                                                 long n) {
  const float s = sp[0];
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float yv = Cvt<T>::load(y, i), gv = Cvt<T>::load(g, i), xv = Cvt<T>::load(x, i);
    const float v = fmaxf(fmaf(tanhf(yv * sigmoidf_(gv)), s, xv), 0.f);
    Cvt<T>::store(out, i, post != nullptr ? v + Cvt<T>::load(post, i) : v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gated_residual_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                                 const T* __restrict__ g, const float* __restrict__ sp,
                                                                 const T* __restrict__ out, const T* __restrict__ xin,
                                                                 T* __restrict__ dy, T* __restrict__ dg,
                                                                 T* __restrict__ dx, float* __restrict__ dsp_part,
                                                                 long n) {
  __shared__ float red[4];
  const float s = sp[0];
  float acc = 0.f;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float yv = Cvt<T>::load(y, i), gv = Cvt<T>::load(g, i);
    const float sg = sigmoidf_(gv);
    const float th = tanhf(yv * sg);
    // the ReLU mask: from the saved output, or (xin: the output carried a post-add) from the recomputed
    // pre-activation, the forward's exact expression
    const bool on = xin != nullptr ? fmaf(th, s, Cvt<T>::load(xin, i)) > 0.f : Cvt<T>::load(out, i) > 0.f;
    const float d = on ? Cvt<T>::load(dout, i) : 0.f;
    acc += d * th;
    const float dpre = d * s * (1.f - th * th);  // d/d(y*sg)
    Cvt<T>::store(dy, i, dpre * sg);
    Cvt<T>::store(dg, i, dpre * yv * sg * (1.f - sg));
    Cvt<T>::store(dx, i, d);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) dsp_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// bf16, n % 8 == 0: 8 elements (16-B vectors) per lane and iteration; the scalar form above moved 2-byte
// elements (0.077 ms per location-head block backward, r2cp)
__device__ __forceinline__ void gr_unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 gr_pack8(const float* f) {
  return make_uint4(f2bf2(f[0], f[1]), f2bf2(f[2], f[3]), f2bf2(f[4], f[5]), f2bf2(f[6], f[7]));
}

__global__ __launch_bounds__(256) void gated_residual_fwd_v8_kernel(const bf16_t* __restrict__ y,
                                                                    const bf16_t* __restrict__ g,
                                                                    const float* __restrict__ sp,
                                                                    const bf16_t* __restrict__ x,
                                                                    const bf16_t* __restrict__ post,
                                                                    bf16_t* __restrict__ out, long n8) {
  const float s = sp[0];
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    float yv[8], gv[8], xv[8], o[8];
    gr_unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
    gr_unpack8(reinterpret_cast<const uint4*>(g)[i], gv);
    gr_unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaxf(fmaf(tanhf(yv[e] * sigmoidf_(gv[e])), s, xv[e]), 0.f);
    if (post != nullptr) {
      // the block output stays in fp32 until the post-add: one bf16 rounding where the separate add rounded twice
      float pv[8];
      gr_unpack8(reinterpret_cast<const uint4*>(post)[i], pv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += pv[e];
    }
    reinterpret_cast<uint4*>(out)[i] = gr_pack8(o);
  }
}

__global__ __launch_bounds__(256) void gated_residual_bwd_v8_kernel(const bf16_t* __restrict__ dout,
                                                                    const bf16_t* __restrict__ y,
                                                                    const bf16_t* __restrict__ g,
                                                                    const float* __restrict__ sp,
                                                                    const bf16_t* __restrict__ out,
                                                                    const bf16_t* __restrict__ xin,
                                                                    bf16_t* __restrict__ dy, bf16_t* __restrict__ dg,
                                                                    bf16_t* __restrict__ dx,
                                                                    float* __restrict__ dsp_part, long n8) {
  __shared__ float red[4];
  const float s = sp[0];
  float acc = 0.f;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n8;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    float ov[8], dv[8], yv[8], gv[8], ody[8], odg[8], odx[8];
    gr_unpack8(reinterpret_cast<const uint4*>(xin != nullptr ? xin : out)[i], ov);
    gr_unpack8(reinterpret_cast<const uint4*>(dout)[i], dv);
    gr_unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
    gr_unpack8(reinterpret_cast<const uint4*>(g)[i], gv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = sigmoidf_(gv[e]);
      const float th = tanhf(yv[e] * sg);
      const bool on = xin != nullptr ? fmaf(th, s, ov[e]) > 0.f : ov[e] > 0.f;
      const float d = on ? dv[e] : 0.f;
      acc += d * th;
      const float dpre = d * s * (1.f - th * th);
      ody[e] = dpre * sg;
      odg[e] = dpre * yv[e] * sg * (1.f - sg);
      odx[e] = d;
    }
    reinterpret_cast<uint4*>(dy)[i] = gr_pack8(ody);
    reinterpret_cast<uint4*>(dg)[i] = gr_pack8(odg);
    reinterpret_cast<uint4*>(dx)[i] = gr_pack8(odx);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) dsp_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace

int elementwise_blocks(long n) {
  long b = (n + 255) / 256;
  return static_cast<int>(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

void gated_residual_fwd(const void* y, const void* g, const float* sp, const void* x, const void* post, void* out,
                        int dt, long n, hipStream_t s) {
  if (dt == DT_BF16 && n % 8 == 0) {
    hipLaunchKernelGGL(gated_residual_fwd_v8_kernel, dim3(elementwise_blocks(n / 8)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(g), sp, static_cast<const bf16_t*>(x),
                       static_cast<const bf16_t*>(post), static_cast<bf16_t*>(out), n / 8);
    return;
  }
  dim3 grid(elementwise_blocks(n)), block(256);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gated_residual_fwd_kernel<bf16_t>, grid, block, 0, s, static_cast<const bf16_t*>(y),
                       static_cast<const bf16_t*>(g), sp, static_cast<const bf16_t*>(x),
                       static_cast<const bf16_t*>(post), static_cast<bf16_t*>(out), n);
  else
    hipLaunchKernelGGL(gated_residual_fwd_kernel<float>, grid, block, 0, s, static_cast<const float*>(y),
                       static_cast<const float*>(g), sp, static_cast<const float*>(x), static_cast<const float*>(post),
                       static_cast<float*>(out), n);
}

void gated_residual_bwd(const void* dout, const void* y, const void* g, const float* sp, const void* out,
                        const void* xin, int dt, void* dy, void* dg, void* dx, float* dsp_part, long n, int nblk,
                        hipStream_t s) {
  dim3 grid(nblk), block(256);
  if (dt == DT_BF16 && n % 8 == 0) {   // nblk (from elementwise_blocks(n)) >= the blocks the 8-wide loop needs
    hipLaunchKernelGGL(gated_residual_bwd_v8_kernel, grid, block, 0, s, static_cast<const bf16_t*>(dout),
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(g), sp,
                       static_cast<const bf16_t*>(out), static_cast<const bf16_t*>(xin), static_cast<bf16_t*>(dy),
                       static_cast<bf16_t*>(dg), static_cast<bf16_t*>(dx), dsp_part, n / 8);
    return;
  }
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gated_residual_bwd_kernel<bf16_t>, grid, block, 0, s, static_cast<const bf16_t*>(dout),
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(g), sp,
                       static_cast<const bf16_t*>(out), static_cast<const bf16_t*>(xin), static_cast<bf16_t*>(dy),
                       static_cast<bf16_t*>(dg), static_cast<bf16_t*>(dx), dsp_part, n);
  else
    hipLaunchKernelGGL(gated_residual_bwd_kernel<float>, grid, block, 0, s, static_cast<const float*>(dout),
                       static_cast<const float*>(y), static_cast<const float*>(g), sp, static_cast<const float*>(out),
                       static_cast<const float*>(xin), static_cast<float*>(dy), static_cast<float*>(dg),
                       static_cast<float*>(dx), dsp_part, n);
}

}  // namespace as
