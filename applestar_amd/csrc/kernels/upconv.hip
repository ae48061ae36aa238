// Fused bilinear x2 upsample + 3x3 conv to ONE output channel: the last stage of the location head
// (action_arg_head.py:417-450).  Unfused, this stage writes and re-reads the 32-channel
// 152x160 upsampled map (~600 MB for a 384-observation batch) and runs a Cout=1 convolution that
// GEMM-based solvers map poorly.  Here the upsampled values are produced in LDS tile by tile and
// consumed immediately:
//   y[b, Y, X] = bias + sum_{c,ky,kx} w[c,ky,kx] * up[b, c, Y+ky-1, X+kx-1]      (zero padding)
//   up = bilinear x2, align_corners=False (source index clamped at 0, PyTorch semantics)
// Backward: dW / db as per-tile partials (column-reduced after), dX through the conv adjoint and
// the bilinear adjoint computed as a gather per low-res pixel (deterministic, no atomics).
// Layouts: x NHWC [B, Hl, Wl, C] (channels_last storage), y / dy [B, 2Hl, 2Wl] fp32.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kC = 32;        // input channels (location head: 32 -> 1)
constexpr int TH = 16, TW = 32;  // high-res output tile
constexpr int UH = TH + 2, UW = TW + 2;

// bilinear source for a high-res coordinate (align_corners=False, scale 2)
__device__ __forceinline__ void src_index(int d, int n_in, int& i0, int& i1, float& l0, float& l1) {
  float s = (d + 0.5f) * 0.5f - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = static_cast<int>(s);
  i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
  l1 = s - static_cast<float>(i0);
  l0 = 1.f - l1;
}

// fills up_s[c][r][cc] (cc fastest) for high-res rows Y0-1.., cols X0-1.. of image b
template <typename T>
__device__ void stage_up(const T* __restrict__ x, float* up_s, int b, int Y0, int X0, int Hl, int Wl) {
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  for (int e = threadIdx.x; e < UH * UW * kC; e += blockDim.x) {
    const int c = e % kC;            // consecutive threads -> consecutive channels (coalesced NHWC reads)
    const int rc = e / kC;
    const int r = rc / UW, cc = rc % UW;
    const int yy = Y0 - 1 + r, xx = X0 - 1 + cc;
    float v = 0.f;
    if (yy >= 0 && yy < H2 && xx >= 0 && xx < W2) {
      int y0, y1, x0, x1;
      float ly0, ly1, lx0, lx1;
      src_index(yy, Hl, y0, y1, ly0, ly1);
      src_index(xx, Wl, x0, x1, lx0, lx1);
      const long base = static_cast<long>(b) * Hl * Wl * kC + c;
      const float a = Cvt<T>::load(x, base + (static_cast<long>(y0) * Wl + x0) * kC);
      const float bb = Cvt<T>::load(x, base + (static_cast<long>(y0) * Wl + x1) * kC);
      const float cc2 = Cvt<T>::load(x, base + (static_cast<long>(y1) * Wl + x0) * kC);
      const float d = Cvt<T>::load(x, base + (static_cast<long>(y1) * Wl + x1) * kC);
      v = ly0 * (lx0 * a + lx1 * bb) + ly1 * (lx0 * cc2 + lx1 * d);
    }
    up_s[(c * UH + r) * UW + cc] = v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void upconv1_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias_p, float* __restrict__ y,
                                                          int Hl, int Wl) {
  const float bias = bias_p[0];
  __shared__ float up_s[kC * UH * UW];
  const int b = blockIdx.z, Y0 = blockIdx.y * TH, X0 = blockIdx.x * TW;
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  stage_up<T>(x, up_s, b, Y0, X0, Hl, Wl);
  __syncthreads();
  for (int o = threadIdx.x; o < TH * TW; o += blockDim.x) {
    const int ty = o / TW, tx = o % TW;
    const int Y = Y0 + ty, X = X0 + tx;
    if (Y >= H2 || X >= W2) continue;
    float acc = bias;
    for (int c = 0; c < kC; ++c) {
      const float* u = up_s + (c * UH + ty) * UW + tx;
      const float* wc = w + c * 9;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(wc[ky * 3 + kx], u[ky * UW + kx], acc);
    }
    y[(static_cast<long>(b) * H2 + Y) * W2 + X] = acc;
  }
}

// per-tile partial dW (288) and db (1) -> part[tile][289]
template <typename T>
__global__ __launch_bounds__(256) void upconv1_bwd_w_kernel(const T* __restrict__ x, const float* __restrict__ dy,
                                                            float* __restrict__ part, int Hl, int Wl) {
  __shared__ float up_s[kC * UH * UW];
  __shared__ float dy_s[TH * TW];
  const int b = blockIdx.z, Y0 = blockIdx.y * TH, X0 = blockIdx.x * TW;
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  stage_up<T>(x, up_s, b, Y0, X0, Hl, Wl);
  for (int o = threadIdx.x; o < TH * TW; o += blockDim.x) {
    const int Y = Y0 + o / TW, X = X0 + o % TW;
    dy_s[o] = (Y < H2 && X < W2) ? dy[(static_cast<long>(b) * H2 + Y) * W2 + X] : 0.f;
  }
  __syncthreads();
  const long tile = (static_cast<long>(blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  for (int p = threadIdx.x; p < kC * 9 + 1; p += blockDim.x) {
    float acc = 0.f;
    if (p == kC * 9) {
      for (int o = 0; o < TH * TW; ++o) acc += dy_s[o];
    } else {
      const int c = p / 9, k = p % 9, ky = k / 3, kx = k % 3;
      const float* u = up_s + c * UH * UW;
      for (int ty = 0; ty < TH; ++ty)
        for (int tx = 0; tx < TW; ++tx) acc = fmaf(dy_s[ty * TW + tx], u[(ty + ky) * UW + tx + kx], acc);
    }
    part[tile * (kC * 9 + 1) + p] = acc;
  }
}

// dX for a low-res tile of LH x LW pixels (all channels)
constexpr int LH = 8, LW = 16;
constexpr int DH = 2 * LH + 2, DW = 2 * LW + 2;   // hi-res rows/cols that touch the tile
template <typename T>
__global__ __launch_bounds__(256) void upconv1_bwd_x_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                            T* __restrict__ dx, int Hl, int Wl) {
  __shared__ float dy_s[(DH + 2) * (DW + 2)];
  __shared__ float dup_s[kC * DH * DW];
  const int b = blockIdx.z, yl0 = blockIdx.y * LH, xl0 = blockIdx.x * LW;
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  const int hy0 = 2 * yl0 - 1, hx0 = 2 * xl0 - 1;  // hi-res origin of the dup region
  for (int e = threadIdx.x; e < (DH + 2) * (DW + 2); e += blockDim.x) {
    const int r = e / (DW + 2), cc = e % (DW + 2);
    const int Y = hy0 - 1 + r, X = hx0 - 1 + cc;
    dy_s[e] = (Y >= 0 && Y < H2 && X >= 0 && X < W2) ? dy[(static_cast<long>(b) * H2 + Y) * W2 + X] : 0.f;
  }
  __syncthreads();
  // dup(c, yy, xx) = sum_k w[c,k] dy(yy - ky + 1, xx - kx + 1); zero outside the hi-res image
  for (int e = threadIdx.x; e < kC * DH * DW; e += blockDim.x) {
    const int c = e / (DH * DW), rc = e % (DH * DW), r = rc / DW, cc = rc % DW;
    const int yy = hy0 + r, xx = hx0 + cc;
    float v = 0.f;
    if (yy >= 0 && yy < H2 && xx >= 0 && xx < W2) {
      const float* wc = w + c * 9;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) v = fmaf(wc[ky * 3 + kx], dy_s[(r + 2 - ky) * (DW + 2) + (cc + 2 - kx)], v);
    }
    dup_s[e] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < LH * LW * kC; e += blockDim.x) {
    const int c = e % kC, p = e / kC, ly = p / LW, lx = p % LW;
    const int yl = yl0 + ly, xl = xl0 + lx;
    if (yl >= Hl || xl >= Wl) continue;
    float acc = 0.f;
    for (int yy = 2 * yl - 1; yy <= 2 * yl + 2; ++yy) {
      if (yy < 0 || yy >= H2) continue;
      int y0, y1;
      float a0, a1;
      src_index(yy, Hl, y0, y1, a0, a1);
      const float wy = (y0 == yl ? a0 : 0.f) + (y1 == yl ? a1 : 0.f);
      if (wy == 0.f) continue;
      for (int xx = 2 * xl - 1; xx <= 2 * xl + 2; ++xx) {
        if (xx < 0 || xx >= W2) continue;
        int x0, x1;
        float b0, b1;
        src_index(xx, Wl, x0, x1, b0, b1);
        const float wx = (x0 == xl ? b0 : 0.f) + (x1 == xl ? b1 : 0.f);
        if (wx == 0.f) continue;
        acc = fmaf(wy * wx, dup_s[(c * DH + (yy - hy0)) * DW + (xx - hx0)], acc);
      }
    }
    Cvt<T>::store(dx, ((static_cast<long>(b) * Hl + yl) * Wl + xl) * kC + c, acc);
  }
}

}  // namespace

int upconv1_channels() { return kC; }

long upconv1_tiles(int B, int Hl, int Wl) {
  return static_cast<long>(B) * ((2 * Hl + TH - 1) / TH) * ((2 * Wl + TW - 1) / TW);
}

void upconv1_fwd(const void* x, int x_dt, const float* w, const float* bias, float* y, int B, int Hl, int Wl,
                 hipStream_t s) {
  const dim3 grid((2 * Wl + TW - 1) / TW, (2 * Hl + TH - 1) / TH, B);
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(upconv1_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(x), w, bias, y, Hl, Wl);
  else
    hipLaunchKernelGGL(upconv1_fwd_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(x), w, bias, y, Hl, Wl);
}

void upconv1_bwd(const void* x, int x_dt, const float* w, const float* dy, void* dx, float* part, float* dwb, int B,
                 int Hl, int Wl, hipStream_t s) {
  const dim3 grid((2 * Wl + TW - 1) / TW, (2 * Hl + TH - 1) / TH, B);
  const dim3 gx((Wl + LW - 1) / LW, (Hl + LH - 1) / LH, B);
  const long tiles = upconv1_tiles(B, Hl, Wl);
  if (x_dt == DT_BF16) {
    hipLaunchKernelGGL(upconv1_bwd_w_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(x), dy, part, Hl, Wl);
    hipLaunchKernelGGL(upconv1_bwd_x_kernel<bf16_t>, gx, dim3(256), 0, s, dy, w, static_cast<bf16_t*>(dx), Hl, Wl);
  } else {
    hipLaunchKernelGGL(upconv1_bwd_w_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(x), dy, part, Hl, Wl);
    hipLaunchKernelGGL(upconv1_bwd_x_kernel<float>, gx, dim3(256), 0, s, dy, w, static_cast<float*>(dx), Hl, Wl);
  }
  column_reduce(part, dwb, static_cast<int>(tiles), kC * 9 + 1, s);
}

}  // namespace as
