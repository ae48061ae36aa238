// Narrow 1x1 convolution on NHWC bf16 pixels: y[p, :] = act(W x[p, :] + b) for Cin, Cout <= 32.
//
// The value encoder's full-resolution 1x1 projection (value_encoder.py: 10 -> 16 channels over
// B x 152 x 160 = 9.5M pixels) is a GEMM with N = K = 16 and M = 9.5M, a shape the library GEMM
// handles with 16 x 256 tiles at ~0.85 ms per call (rocprof r1_v16) for what is a 600 MB streaming pass.
// Here one thread owns one pixel: 16-B loads of its Cin channels, Cout x Cin FMAs against the weight held
// in LDS (fp32), bias + ReLU, 16-B stores.  The input gradient is the same kernel with W^T and no bias /
// activation; the weight gradient goes through the split-R MFMA kernel (wgrad.hip).
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <int CIN, int COUT>
__global__ __launch_bounds__(256) void pointwise_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                        long P, int act) {
  __shared__ float ws[COUT * CIN];
  __shared__ float bs[COUT];
  for (int i = threadIdx.x; i < COUT * CIN; i += 256) ws[i] = w[i];
  if (threadIdx.x < COUT) bs[threadIdx.x] = bias ? bias[threadIdx.x] : 0.f;
  __syncthreads();
  const long p = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= P) return;
  float xin[CIN];
#pragma unroll
  for (int c = 0; c < CIN; c += 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(x + p * CIN + c);
    const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xin[c + 2 * e] = __uint_as_float(q[e] << 16);
      xin[c + 2 * e + 1] = __uint_as_float(q[e] & 0xffff0000u);
    }
  }
#pragma unroll
  for (int o = 0; o < COUT; o += 8) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float a = bs[o + e];
#pragma unroll
      for (int c = 0; c < CIN; ++c) a = fmaf(ws[(o + e) * CIN + c], xin[c], a);
      v[e] = act == ACT_RELU ? fmaxf(a, 0.f) : a;
    }
    uint4 u;
    u.x = f2bf2(v[0], v[1]);
    u.y = f2bf2(v[2], v[3]);
    u.z = f2bf2(v[4], v[5]);
    u.w = f2bf2(v[6], v[7]);
    *reinterpret_cast<uint4*>(y + p * COUT + o) = u;
  }
}

template <int CIN, int COUT>
void launch(const bf16_t* x, const float* w, const float* b, bf16_t* y, long P, int act, hipStream_t s) {
  hipLaunchKernelGGL((pointwise_kernel<CIN, COUT>), dim3(static_cast<unsigned>((P + 255) / 256)), dim3(256), 0, s,
                     x, w, b, y, P, act);
}

}  // namespace

bool pointwise_supported(int cin, int cout) {
  auto ok = [](int c) { return c == 8 || c == 16 || c == 32; };
  return ok(cin) && ok(cout);
}

void pointwise_conv(const void* x, const float* w, const float* bias, void* y, long P, int cin, int cout, int act,
                    hipStream_t s) {
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  bf16_t* yp = static_cast<bf16_t*>(y);
#define AS_PW(CI, CO) \
  if (cin == CI && cout == CO) return launch<CI, CO>(xp, w, bias, yp, P, act, s);
  AS_PW(8, 8) AS_PW(8, 16) AS_PW(8, 32) AS_PW(16, 8) AS_PW(16, 16) AS_PW(16, 32) AS_PW(32, 8) AS_PW(32, 16)
  AS_PW(32, 32)
#undef AS_PW
}

}  // namespace as
