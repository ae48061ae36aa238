// Fused elementwise tails.
//
// gated_residual: the location head's GatedResBlock output  relu(tanh(y * sigmoid(g)) * sp + x)
// (module_utils.py:224-231) — 5 torch kernels + 4 temporaries per block in the reference, one pass
// here; the backward recomputes sigmoid/tanh from y, g and writes dy, dg, dx plus per-block partial
// sums for d(sp) in one pass.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void gated_residual_fwd_kernel(const T* __restrict__ y, const T* __restrict__ g,
                                                                 const float* __restrict__ sp, const T* __restrict__ x,
                                                                 T* __restrict__ out, long n) {
  const float s = sp[0];
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float yv = Cvt<T>::load(y, i), gv = Cvt<T>::load(g, i), xv = Cvt<T>::load(x, i);
    const float v = tanhf(yv * sigmoidf_(gv)) * s + xv;
    Cvt<T>::store(out, i, fmaxf(v, 0.f));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gated_residual_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                                 const T* __restrict__ g, const float* __restrict__ sp,
                                                                 const T* __restrict__ out, T* __restrict__ dy,
                                                                 T* __restrict__ dg, T* __restrict__ dx,
                                                                 float* __restrict__ dsp_part, long n) {
  __shared__ float red[4];
  const float s = sp[0];
  float acc = 0.f;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float o = Cvt<T>::load(out, i);
    const float d = o > 0.f ? Cvt<T>::load(dout, i) : 0.f;
    const float yv = Cvt<T>::load(y, i), gv = Cvt<T>::load(g, i);
    const float sg = sigmoidf_(gv);
    const float th = tanhf(yv * sg);
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

}  // namespace

int elementwise_blocks(long n) {
  long b = (n + 255) / 256;
  return static_cast<int>(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

void gated_residual_fwd(const void* y, const void* g, const float* sp, const void* x, void* out, int dt, long n,
                        hipStream_t s) {
  dim3 grid(elementwise_blocks(n)), block(256);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gated_residual_fwd_kernel<bf16_t>, grid, block, 0, s, static_cast<const bf16_t*>(y),
                       static_cast<const bf16_t*>(g), sp, static_cast<const bf16_t*>(x), static_cast<bf16_t*>(out), n);
  else
    hipLaunchKernelGGL(gated_residual_fwd_kernel<float>, grid, block, 0, s, static_cast<const float*>(y),
                       static_cast<const float*>(g), sp, static_cast<const float*>(x), static_cast<float*>(out), n);
}

void gated_residual_bwd(const void* dout, const void* y, const void* g, const float* sp, const void* out, int dt,
                        void* dy, void* dg, void* dx, float* dsp_part, long n, int nblk, hipStream_t s) {
  dim3 grid(nblk), block(256);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gated_residual_bwd_kernel<bf16_t>, grid, block, 0, s, static_cast<const bf16_t*>(dout),
                       static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(g), sp,
                       static_cast<const bf16_t*>(out), static_cast<bf16_t*>(dy), static_cast<bf16_t*>(dg),
                       static_cast<bf16_t*>(dx), dsp_part, n);
  else
    hipLaunchKernelGGL(gated_residual_bwd_kernel<float>, grid, block, 0, s, static_cast<const float*>(dout),
                       static_cast<const float*>(y), static_cast<const float*>(g), sp, static_cast<const float*>(out),
                       static_cast<float*>(dy), static_cast<float*>(dg), static_cast<float*>(dx), dsp_part, n);
}

}  // namespace as
