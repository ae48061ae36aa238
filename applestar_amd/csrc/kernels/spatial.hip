// Spatial-path kernels for the encoder and the location head (NHWC / channels_last, bf16 or fp32).
//
// upsample2x: bilinear x2, align_corners=False (F.interpolate(scale_factor=2, mode='bilinear')),
//   the location head's 3 upsampling stages (action_arg_head.py:440-446).  torch runs this in fp32
//   under autocast with a generic NCHW kernel (21.6 % of the first learner profile); here it is a
//   bf16 NHWC gather with the fixed 0.25/0.75 stencil, channels contiguous per lane.  The backward is
//   a deterministic gather (each input pixel pulls its <= 4x4 outputs), no atomics.
// spatial_embed: the spatial encoder input planes + 1x1 projection (spatial_encoder.py:51-72) in
//   one pass: one thread per pixel reads height/6 categorical planes/effect bits and writes the 32
//   pre-activation channels; entity contributions (the scatter connection pre-multiplied by the
//   scatter columns of the 1x1 conv) are added by scatter_add_rows; relu_cast finishes.
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"

#include <cstdlib>

namespace as {
namespace {

// 1-D source taps of output index o (align_corners=False, scale 2)
__device__ __forceinline__ void taps(int o, int n_in, int& i0, int& i1, float& l) {
  float src = (o + 0.5f) * 0.5f - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = static_cast<int>(src);
  if (i0 > n_in - 1) i0 = n_in - 1;
  i1 = i0 + 1 < n_in ? i0 + 1 : n_in - 1;
  l = src - static_cast<float>(i0);
}

__device__ __forceinline__ float tap_weight(int o, int k, int n_in) {
  int i0, i1;
  float l;
  taps(o, n_in, i0, i1, l);
  return (k == i0 ? 1.f - l : 0.f) + (k == i1 ? l : 0.f);
}

// x [B][H][W][C] -> y [B][2H][2W][C]; thread handles 4 channels
template <typename T>
__global__ __launch_bounds__(256) void upsample2x_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H,
                                                             int W, int C) {
  const int C4 = C / 4;
  const long total = static_cast<long>(B) * 2 * H * 2 * W * C4;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c4 = static_cast<int>(i % C4);
    long r = i / C4;
    const int ox = static_cast<int>(r % (2 * W));
    r /= 2 * W;
    const int oy = static_cast<int>(r % (2 * H));
    const int b = static_cast<int>(r / (2 * H));
    int y0, y1, x0, x1;
    float ly, lx;
    taps(oy, H, y0, y1, ly);
    taps(ox, W, x0, x1, lx);
    const long base = static_cast<long>(b) * H * W;
    const long p00 = ((base + static_cast<long>(y0) * W + x0) * C) + c4 * 4;
    const long p01 = ((base + static_cast<long>(y0) * W + x1) * C) + c4 * 4;
    const long p10 = ((base + static_cast<long>(y1) * W + x0) * C) + c4 * 4;
    const long p11 = ((base + static_cast<long>(y1) * W + x1) * C) + c4 * 4;
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
    const long o = ((static_cast<long>(b) * 2 * H + oy) * 2 * W + ox) * C + c4 * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = w00 * Cvt<T>::load(x, p00 + k) + w01 * Cvt<T>::load(x, p01 + k) +
                      w10 * Cvt<T>::load(x, p10 + k) + w11 * Cvt<T>::load(x, p11 + k);
      Cvt<T>::store(y, o + k, v);
    }
  }
}

// dy [B][2H][2W][C] -> dx [B][H][W][C]
// mask (optional): the upsample's input x when it is a ReLU output - dx is also multiplied by [x > 0] (the
// producer's ReLU backward folded in, ops/native.py _premasked); the bf16 vector path below takes none
template <typename T>
__global__ __launch_bounds__(256) void upsample2x_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int B, int H,
                                                             int W, int C, const T* __restrict__ mask) {
  const int C4 = C / 4;
  const long total = static_cast<long>(B) * H * W * C4;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c4 = static_cast<int>(i % C4);
    long r = i / C4;
    const int kx = static_cast<int>(r % W);
    r /= W;
    const int ky = static_cast<int>(r % H);
    const int b = static_cast<int>(r / H);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int oy = 2 * ky - 1; oy <= 2 * ky + 2; ++oy) {
      if (oy < 0 || oy >= 2 * H) continue;
      const float wy = tap_weight(oy, ky, H);
      if (wy == 0.f) continue;
      for (int ox = 2 * kx - 1; ox <= 2 * kx + 2; ++ox) {
        if (ox < 0 || ox >= 2 * W) continue;
        const float w = wy * tap_weight(ox, kx, W);
        if (w == 0.f) continue;
        const long o = ((static_cast<long>(b) * 2 * H + oy) * 2 * W + ox) * C + c4 * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = fmaf(w, Cvt<T>::load(dy, o + k), acc[k]);
      }
    }
    const long d = ((static_cast<long>(b) * H + ky) * W + kx) * C + c4 * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float v = mask && !(Cvt<T>::load(mask, d + k) > 0.f) ? 0.f : acc[k];
      Cvt<T>::store(dx, d + k, v);
    }
  }
}

// bf16, C % 8 == 0: one thread per INPUT pixel and 8 channels (16-B vectors, 32-bit index math).
// Forward: the 3x3 neighbourhood (clamped) gives the 2x2 outputs of the fixed 0.25 / 0.75 stencil; border
// clamping reproduces align_corners=False exactly (a clamped neighbour is the pixel itself).  The per-output
// form above did 64-bit divisions and 16 scalar 2-byte loads per 4 channels (0.14 ms per location-head
// upsample).  Backward: the input pixel pulls its 4 x 4 output neighbourhood with the 1-D weights
// 0.25 | 0.75 (+0.25 at the first / last index) | 0.75 (+0.25) | 0.25.
__device__ __forceinline__ void up_unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 up_pack8(const float* f) {
  uint4 v;
  v.x = f2bf2(f[0], f[1]);
  v.y = f2bf2(f[2], f[3]);
  v.z = f2bf2(f[4], f[5]);
  v.w = f2bf2(f[6], f[7]);
  return v;
}

__global__ __launch_bounds__(256) void upsample2x_fwd_v8_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                int B, int H, int W, int C) {
  const int C8 = C >> 3;
  const int total = B * H * W * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    int p = i / C8;
    const int xx = p % W;
    p /= W;
    const int yy = p % H;
    const int b = p / H;
    const int ys[3] = {yy > 0 ? yy - 1 : 0, yy, yy + 1 < H ? yy + 1 : H - 1};
    const int xs[3] = {xx > 0 ? xx - 1 : 0, xx, xx + 1 < W ? xx + 1 : W - 1};
    float r0[3][8], r1[3][8];                      // rows 2yy / 2yy+1 interpolated, per source column
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float a[8], m[8], z[8];
      const long col = static_cast<long>(xs[c]) * C + 8 * c8;
      up_unpack8(*reinterpret_cast<const uint4*>(x + (static_cast<long>(b * H + ys[0]) * W) * C + col), a);
      up_unpack8(*reinterpret_cast<const uint4*>(x + (static_cast<long>(b * H + ys[1]) * W) * C + col), m);
      up_unpack8(*reinterpret_cast<const uint4*>(x + (static_cast<long>(b * H + ys[2]) * W) * C + col), z);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        r0[c][e] = 0.25f * a[e] + 0.75f * m[e];
        r1[c][e] = 0.75f * m[e] + 0.25f * z[e];
      }
    }
    float o[8];
    const long W2 = 2L * W;
    const long base = ((static_cast<long>(b) * 2 * H + 2 * yy) * W2 + 2 * xx) * C + 8 * c8;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.25f * r0[0][e] + 0.75f * r0[1][e];
    *reinterpret_cast<uint4*>(y + base) = up_pack8(o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.75f * r0[1][e] + 0.25f * r0[2][e];
    *reinterpret_cast<uint4*>(y + base + C) = up_pack8(o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.25f * r1[0][e] + 0.75f * r1[1][e];
    *reinterpret_cast<uint4*>(y + base + W2 * C) = up_pack8(o);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.75f * r1[1][e] + 0.25f * r1[2][e];
    *reinterpret_cast<uint4*>(y + base + W2 * C + C) = up_pack8(o);
  }
}

__device__ __forceinline__ float up_w(int t, int k, int n) {   // weight of output 2k-1+t on input k
  if (t == 0) return k > 0 ? 0.25f : 0.f;
  if (t == 1) return k == 0 ? 1.f : 0.75f;
  if (t == 2) return k == n - 1 ? 1.f : 0.75f;
  return k < n - 1 ? 0.25f : 0.f;
}

__global__ __launch_bounds__(256) void upsample2x_bwd_v8_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                                int B, int H, int W, int C) {
  const int C8 = C >> 3;
  const int total = B * H * W * C8;
  const long W2 = 2L * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    int p = i / C8;
    const int xx = p % W;
    p /= W;
    const int yy = p % H;
    const int b = p / H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ty = 0; ty < 4; ++ty) {
      const float wy = up_w(ty, yy, H);
      if (wy == 0.f) continue;
      const int oy = 2 * yy - 1 + ty;
#pragma unroll
      for (int tx = 0; tx < 4; ++tx) {
        const float w = wy * up_w(tx, xx, W);
        if (w == 0.f) continue;
        const int ox = 2 * xx - 1 + tx;
        float v[8];
        up_unpack8(*reinterpret_cast<const uint4*>(dy + ((static_cast<long>(b) * 2 * H + oy) * W2 + ox) * C + 8 * c8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(w, v[e], acc[e]);
      }
    }
    *reinterpret_cast<uint4*>(dx + ((static_cast<long>(b) * H + yy) * W + xx) * C + 8 * c8) = up_pack8(acc);
  }
}

// fp32, C % 4 == 0: the same per-input-pixel stencils with 16-B float4 vectors and 32-bit index math (the generic
// per-output kernels above did 64-bit divisions and scalar loads: ~180 / 200 us per location-head upsample
// forward / backward in the fp32 step).  mask (backward, optional): dx *= [mask > 0] (the producer's ReLU).
__device__ __forceinline__ void f4a(const float4 v, float* f) { f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w; }

__global__ __launch_bounds__(256) void upsample2x_fwd_v4f_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                 int B, int H, int W, int C) {
  const int C4 = C >> 2;
  const int total = B * H * W * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    int p = i / C4;
    const int xx = p % W;
    p /= W;
    const int yy = p % H;
    const int b = p / H;
    const int ys[3] = {yy > 0 ? yy - 1 : 0, yy, yy + 1 < H ? yy + 1 : H - 1};
    const int xs[3] = {xx > 0 ? xx - 1 : 0, xx, xx + 1 < W ? xx + 1 : W - 1};
    float r0[3][4], r1[3][4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float a[4], m[4], z[4];
      const long col = static_cast<long>(xs[c]) * C + 4 * c4;
      f4a(*reinterpret_cast<const float4*>(x + (static_cast<long>(b * H + ys[0]) * W) * C + col), a);
      f4a(*reinterpret_cast<const float4*>(x + (static_cast<long>(b * H + ys[1]) * W) * C + col), m);
      f4a(*reinterpret_cast<const float4*>(x + (static_cast<long>(b * H + ys[2]) * W) * C + col), z);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r0[c][e] = 0.25f * a[e] + 0.75f * m[e];
        r1[c][e] = 0.75f * m[e] + 0.25f * z[e];
      }
    }
    const long W2 = 2L * W;
    const long base = ((static_cast<long>(b) * 2 * H + 2 * yy) * W2 + 2 * xx) * C + 4 * c4;
    auto st = [&](long off, const float (&r)[3][4], bool right) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = right ? 0.75f * r[1][e] + 0.25f * r[2][e] : 0.25f * r[0][e] + 0.75f * r[1][e];
      *reinterpret_cast<float4*>(y + off) = make_float4(o[0], o[1], o[2], o[3]);
    };
    st(base, r0, false);
    st(base + C, r0, true);
    st(base + W2 * C, r1, false);
    st(base + W2 * C + C, r1, true);
  }
}

__global__ __launch_bounds__(256) void upsample2x_bwd_v4f_kernel(const float* __restrict__ dy, float* __restrict__ dx,
                                                                 int B, int H, int W, int C, const float* __restrict__ mask) {
  const int C4 = C >> 2;
  const int total = B * H * W * C4;
  const long W2 = 2L * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c4 = i % C4;
    int p = i / C4;
    const int xx = p % W;
    p /= W;
    const int yy = p % H;
    const int b = p / H;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ty = 0; ty < 4; ++ty) {
      const float wy = up_w(ty, yy, H);
      if (wy == 0.f) continue;
      const int oy = 2 * yy - 1 + ty;
#pragma unroll
      for (int tx = 0; tx < 4; ++tx) {
        const float w = wy * up_w(tx, xx, W);
        if (w == 0.f) continue;
        const int ox = 2 * xx - 1 + tx;
        float v[4];
        f4a(*reinterpret_cast<const float4*>(dy + ((static_cast<long>(b) * 2 * H + oy) * W2 + ox) * C + 4 * c4), v);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = fmaf(w, v[e], acc[e]);
      }
    }
    const long d = ((static_cast<long>(b) * H + yy) * W + xx) * C + 4 * c4;
    if (mask) {
      const float4 mk = *reinterpret_cast<const float4*>(mask + d);
      acc[0] = mk.x > 0.f ? acc[0] : 0.f;
      acc[1] = mk.y > 0.f ? acc[1] : 0.f;
      acc[2] = mk.z > 0.f ? acc[2] : 0.f;
      acc[3] = mk.w > 0.f ? acc[3] : 0.f;
    }
    *reinterpret_cast<float4*>(dx + d) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// pre [B][H*W][32] fp32 = bias + W_dense . dense_input(pixel)
// dense columns: 0 height/256 | 1..4 visibility | 5..6 creep | 7..11 player_relative | 12..13 alerts |
//                14..15 pathable | 16..17 buildable | 18..23 effects
__global__ __launch_bounds__(256) void spatial_dense_kernel(SpatialPlanes sp, const uint8_t* __restrict__ effect_bits,
                                                            const float* __restrict__ wd, const float* __restrict__ bias,
                                                            float* __restrict__ pre, long npix) {
  __shared__ float w_s[24][32];
  __shared__ float b_s[32];
  for (int i = threadIdx.x; i < 24 * 32; i += blockDim.x) w_s[i % 24][i / 24] = wd[(i / 24) * 24 + (i % 24)];
  if (threadIdx.x < 32) b_s[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  const int widths[6] = {4, 2, 5, 2, 2, 2};
  for (long p = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; p < npix;
       p += static_cast<long>(gridDim.x) * blockDim.x) {
    float acc[32];
    const float h = static_cast<float>(sp.height[p]) * (1.f / 256.f);
#pragma unroll
    for (int c = 0; c < 32; ++c) acc[c] = b_s[c] + w_s[0][c] * h;
    int off = 1;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      int v = sp.plane[k][p];
      v = v < widths[k] ? v : widths[k] - 1;
      const int col = off + v;
#pragma unroll
      for (int c = 0; c < 32; ++c) acc[c] += w_s[col][c];
      off += widths[k];
    }
    const uint8_t eb = effect_bits[p];
#pragma unroll
    for (int e = 0; e < 6; ++e)
      if ((eb >> e) & 1) {
#pragma unroll
        for (int c = 0; c < 32; ++c) acc[c] += w_s[18 + e][c];
      }
    float4* dst = reinterpret_cast<float4*>(pre + p * 32);
#pragma unroll
    for (int c = 0; c < 8; ++c) dst[c] = make_float4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]);
  }
}

// effect_bits[b][pix] |= 1 << e for each effect point (int16 flat index, zero padded -> pixel 0)
__global__ void effect_bits_kernel(SpatialPlanes sp, uint32_t* __restrict__ bits_words, int B, int L, int HW) {
  const long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<long>(B) * 6 * L) return;
  const int e = static_cast<int>((i / L) % 6);
  const int b = static_cast<int>(i / (6L * L));
  const int j = static_cast<int>(i % L);
  int p = sp.effect[e][static_cast<long>(b) * L + j];
  p = p < 0 ? 0 : (p >= HW ? HW - 1 : p);
  const long byte = static_cast<long>(b) * HW + p;
  atomicOr(bits_words + (byte >> 2), 1u << (8 * (byte & 3) + e));
}

// pre[b, y*W+x, c] += rows[b, n, c] for n < entity_num[b]
template <typename T>
__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const T* __restrict__ rows, const uint8_t* __restrict__ ex,
                                                               const uint8_t* __restrict__ ey,
                                                               const int64_t* __restrict__ entity_num,
                                                               float* __restrict__ pre, int B, int N, int H, int W) {
  const long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<long>(B) * N * 32) return;
  const int c = static_cast<int>(i & 31);
  const long bn = i >> 5;
  const int b = static_cast<int>(bn / N);
  const int n = static_cast<int>(bn % N);
  if (n >= entity_num[b]) return;
  int x = ex[bn], y = ey[bn];
  x = x < W ? x : W - 1;
  y = y < H ? y : H - 1;
  atomicAdd(pre + (static_cast<long>(b) * H * W + static_cast<long>(y) * W + x) * 32 + c, Cvt<T>::load(rows, i));
}

// gate (nullable): the embedding's ReLU output - dpre is then dout * [gate > 0]
template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(const T* __restrict__ dpre, const T* __restrict__ gate,
                                                          const uint8_t* __restrict__ ex,
                                                          const uint8_t* __restrict__ ey,
                                                          const int64_t* __restrict__ entity_num, T* __restrict__ drows,
                                                          int B, int N, int H, int W) {
  const long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<long>(B) * N * 32) return;
  const int c = static_cast<int>(i & 31);
  const long bn = i >> 5;
  const int b = static_cast<int>(bn / N);
  const int n = static_cast<int>(bn % N);
  float v = 0.f;
  if (n < entity_num[b]) {
    int x = ex[bn], y = ey[bn];
    x = x < W ? x : W - 1;
    y = y < H ? y : H - 1;
    const long o = (static_cast<long>(b) * H * W + static_cast<long>(y) * W + x) * 32 + c;
    v = Cvt<T>::load(dpre, o);
    if (gate != nullptr && !(Cvt<T>::load(gate, o) > 0.f)) v = 0.f;
  }
  Cvt<T>::store(drows, i, v);
}

template <typename TO>
__global__ __launch_bounds__(256) void relu_cast_kernel(const float* __restrict__ x, TO* __restrict__ y, long n) {
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x)
    Cvt<TO>::store(y, i, fmaxf(x[i], 0.f));
}

// dense input materialised for the 1x1 conv weight gradient: X [npix][24]
template <typename TX>
__global__ __launch_bounds__(256) void spatial_dense_input_kernel(SpatialPlanes sp, const uint8_t* __restrict__ effect_bits,
                                                                  TX* __restrict__ X, long npix) {
  const int widths[6] = {4, 2, 5, 2, 2, 2};
  for (long p = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; p < npix;
       p += static_cast<long>(gridDim.x) * blockDim.x) {
    float v[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) v[i] = 0.f;
    v[0] = static_cast<float>(sp.height[p]) * (1.f / 256.f);
    int off = 1;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      int c = sp.plane[k][p];
      c = c < widths[k] ? c : widths[k] - 1;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (j < widths[k] && j == c) v[off + j] = 1.f;
      off += widths[k];
    }
    const uint8_t eb = effect_bits[p];
#pragma unroll
    for (int e = 0; e < 6; ++e) v[18 + e] = static_cast<float>((eb >> e) & 1);
#pragma unroll
    for (int i = 0; i < 24; ++i) Cvt<TX>::store(X, p * 24 + i, v[i]);
  }
}


// ------------------------------------------------------------------------------------------------
// Fused spatial input (forward): one workgroup owns a tile of 256 consecutive pixels of ONE
// observation.  It marks the tile's effect points in LDS, computes every pixel's 24 dense columns
// (height, 6 one-hot planes, effect bits) against the 1x1 weight into an fp32 LDS tile, adds the
// pre-projected rows of the observation's entities that fall inside the tile (LDS float atomics), and
// writes relu(tile) once in the output dtype with 16-B stores.  Replaces effect_bits + spatial_dense
// (one fp32 [npix, 32] round trip, 128-B strided stores per thread) + scatter_add_rows + relu_cast.
constexpr int kSpTile = 256;

template <typename TR, typename TO>
__global__ __launch_bounds__(256) void spatial_embed_fused_kernel(SpatialPlanes sp, const float* __restrict__ wd,
                                                                  const float* __restrict__ bias,
                                                                  const TR* __restrict__ rows,
                                                                  const uint8_t* __restrict__ ex,
                                                                  const uint8_t* __restrict__ ey,
                                                                  const int64_t* __restrict__ entity_num,
                                                                  TO* __restrict__ out, int N, int H, int W, int L,
                                                                  int tiles) {
  __shared__ float acc[kSpTile][33];
  __shared__ float w_s[24][32];
  __shared__ float b_s[32];
  __shared__ uint32_t eb[kSpTile];
  __shared__ int2 ent_list[kSpTile];
  __shared__ int ent_cnt;
  const int HW = H * W;
  const int b = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int p0 = tile * kSpTile, tid = threadIdx.x;
  const int np = HW - p0 < kSpTile ? HW - p0 : kSpTile;
  for (int i = tid; i < 24 * 32; i += 256) w_s[i % 24][i / 24] = wd[(i / 24) * 24 + (i % 24)];
  if (tid < 32) b_s[tid] = bias[tid];
  eb[tid] = 0;
  if (tid == 0) ent_cnt = 0;
  __syncthreads();
  for (int i = tid; i < 6 * L; i += 256) {
    const int e = i / L, j = i - e * L;
    int p = sp.effect[e][static_cast<long>(b) * L + j];
    p = p < 0 ? 0 : (p >= HW ? HW - 1 : p);
    if (p >= p0 && p < p0 + np) atomicOr(&eb[p - p0], 1u << e);
  }
  __syncthreads();
  if (tid < np) {
    const long pix = static_cast<long>(b) * HW + p0 + tid;
    const int widths[6] = {4, 2, 5, 2, 2, 2};
    float a[32];
    const float h = static_cast<float>(sp.height[pix]) * (1.f / 256.f);
#pragma unroll
    for (int c = 0; c < 32; ++c) a[c] = b_s[c] + w_s[0][c] * h;
    int off = 1;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      int v = sp.plane[k][pix];
      v = v < widths[k] ? v : widths[k] - 1;
#pragma unroll
      for (int c = 0; c < 32; ++c) a[c] += w_s[off + v][c];
      off += widths[k];
    }
    const uint32_t bits = eb[tid];
#pragma unroll
    for (int e = 0; e < 6; ++e)
      if ((bits >> e) & 1) {
#pragma unroll
        for (int c = 0; c < 32; ++c) a[c] += w_s[18 + e][c];
      }
#pragma unroll
    for (int c = 0; c < 32; ++c) acc[tid][c] = a[c];
  }
  __syncthreads();
  // entities of this observation inside the tile: add their 32 pre-projected channels
  // entities of this observation inside the tile: one position test per entity (a compacted LDS list),
  // then the listed rows' 32 channels in parallel
  const int ne = static_cast<int>(entity_num[b] < N ? entity_num[b] : N);
  for (int n = tid; n < ne; n += 256) {
    const long bn = static_cast<long>(b) * N + n;
    int x = ex[bn], y = ey[bn];
    x = x < W ? x : W - 1;
    y = y < H ? y : H - 1;
    const int p = y * W + x - p0;
    if (p >= 0 && p < np) {
      const int slot = atomicAdd(&ent_cnt, 1);
      if (slot < kSpTile) {
        ent_list[slot] = make_int2(n, p);
      } else {   // list full (> 256 entities in one tile): add this row directly
        for (int c = 0; c < 32; ++c) atomicAdd(&acc[p][c], Cvt<TR>::load(rows, bn * 32 + c));
      }
    }
  }
  __syncthreads();
  const int nl = ent_cnt < kSpTile ? ent_cnt : kSpTile;
  for (int i = tid; i < nl * 32; i += 256) {
    const int c = i & 31;
    const int2 e = ent_list[i >> 5];
    const long bn = static_cast<long>(b) * N + e.x;
    atomicAdd(&acc[e.y][c], Cvt<TR>::load(rows, bn * 32 + c));
  }
  __syncthreads();
  const long o0 = (static_cast<long>(b) * HW + p0) * 32;
  for (int i = tid; i < np * 32; i += 256) {
    const int p = i >> 5, c = i & 31;
    Cvt<TO>::store(out, o0 + i, fmaxf(acc[p][c], 0.f));
  }
}

// dW_dense [32][24] and db [32] of the spatial 1x1 projection without materialising the dense input:
// thread (slot = tid / 32, channel n = tid % 32) accumulates dpre[p][n] * X[p][k] over its pixels in
// registers (X is height + one-hot + effect bits, so every column update is a select-add); the 8 slots
// are summed in LDS and each workgroup writes one partial row [32 * 24 + 32] (reduced afterwards).
template <typename TD>
__global__ __launch_bounds__(256) void spatial_dense_wgrad_kernel(SpatialPlanes sp, const TD* __restrict__ dpre,
                                                                  const TD* __restrict__ gate,
                                                                  float* __restrict__ part, int H, int W, int L,
                                                                  int tiles, int wg_per_obs) {
  __shared__ uint32_t eb[kSpTile];
  __shared__ float red[8][32][25];
  const int HW = H * W;
  const int b = blockIdx.x / wg_per_obs, q = blockIdx.x % wg_per_obs;
  const int tid = threadIdx.x, n = tid & 31, slot = tid >> 5;
  float acc[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) acc[k] = 0.f;
  for (int tile = q; tile < tiles; tile += wg_per_obs) {
    const int p0 = tile * kSpTile;
    const int np = HW - p0 < kSpTile ? HW - p0 : kSpTile;
    __syncthreads();
    eb[tid] = 0;
    __syncthreads();
    for (int i = tid; i < 6 * L; i += 256) {
      const int e = i / L, j = i - e * L;
      int p = sp.effect[e][static_cast<long>(b) * L + j];
      p = p < 0 ? 0 : (p >= HW ? HW - 1 : p);
      if (p >= p0 && p < p0 + np) atomicOr(&eb[p - p0], 1u << e);
    }
    __syncthreads();
    // four pixels per pass: their dpre / gate / plane loads are all issued before the first update (one
    // memory latency per four pixels instead of one per pixel)
    constexpr int U = 4;
    for (int pb = slot; pb < np; pb += 8 * U) {
      float d[U];
      int pv[U][6], hv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int pl = pb + 8 * u;
        const long pix = static_cast<long>(b) * HW + p0 + (pl < np ? pl : pb);
        const float g = gate == nullptr ? 1.f : Cvt<TD>::load(gate, pix * 32 + n);
        d[u] = (pl < np && g > 0.f) ? Cvt<TD>::load(dpre, pix * 32 + n) : 0.f;
        hv[u] = sp.height[pix];
#pragma unroll
        for (int k = 0; k < 6; ++k) pv[u][k] = sp.plane[k][pix];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float du = d[u];
        acc[24] += du;
        acc[0] += du * (static_cast<float>(hv[u]) * (1.f / 256.f));
        const int widths[6] = {4, 2, 5, 2, 2, 2};
        int off = 1;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          int v = pv[u][k];
          v = v < widths[k] ? v : widths[k] - 1;
#pragma unroll
          for (int j = 0; j < 5; ++j)
            if (j < widths[k]) acc[off + j] += (v == j) ? du : 0.f;
          off += widths[k];
        }
        const int pl = pb + 8 * u;
        const uint32_t bits = pl < np ? eb[pl] : 0u;
#pragma unroll
        for (int e = 0; e < 6; ++e) acc[18 + e] += ((bits >> e) & 1) ? du : 0.f;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 25; ++k) red[slot][n][k] = acc[k];
  __syncthreads();
  float* row = part + static_cast<long>(blockIdx.x) * (32 * 24 + 32);
  for (int i = tid; i < 32 * 25; i += 256) {
    const int nn = i / 25, k = i % 25;
    float s = 0.f;
#pragma unroll
    for (int sl = 0; sl < 8; ++sl) s += red[sl][nn][k];
    if (k < 24) row[nn * 24 + k] = s;
    else row[32 * 24 + nn] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// MFMA forms (bf16 activations).  Every dense column except height is 0 or 1 and height/256 has 8
// significant bits, so the dense input is EXACT in bf16: a pixel is described by one 25-bit column
// mask (bit c set <=> X[p][c] = 1; bit 24 is the bias / db column) plus its height as bf16 bits.
//   forward  pre[p][n] = sum_c X[p][c] Wd'[n][c]  — K = 32 columns = ONE 16x16x32 MFMA step per
//            16 pixels x 16 channels; Wd' (bias in column 24) is split hi + lo bf16 so the product
//            keeps ~fp32 accuracy (X exact, hi + lo carries 16 mantissa bits).
//   backward dWd'[n][c] = sum_p dpre[p][n] X[p][c] — K = pixels: dpre^T is staged in LDS per tile,
//            the X fragments are expanded from the LDS masks on the fly.
__device__ __forceinline__ uint32_t pixel_mask(const SpatialPlanes& sp, long pix, uint32_t ebits) {
  const uint32_t v0 = min(static_cast<uint32_t>(sp.plane[0][pix]), 3u), v1 = min(static_cast<uint32_t>(sp.plane[1][pix]), 1u);
  const uint32_t v2 = min(static_cast<uint32_t>(sp.plane[2][pix]), 4u), v3 = min(static_cast<uint32_t>(sp.plane[3][pix]), 1u);
  const uint32_t v4 = min(static_cast<uint32_t>(sp.plane[4][pix]), 1u), v5 = min(static_cast<uint32_t>(sp.plane[5][pix]), 1u);
  return (2u << v0) | (32u << v1) | (128u << v2) | (4096u << v3) | (16384u << v4) | (65536u << v5) |
         ((ebits & 63u) << 18) | (1u << 24);
}

// two bf16 words for columns j, j + 1 of the mask byte m (1.0 = 0x3F80)
__device__ __forceinline__ uint32_t bit_pair(uint32_t m, int j) {
  return (((m >> j) & 1u) ? 0x3F80u : 0u) | (((m >> (j + 1)) & 1u) ? 0x3F800000u : 0u);
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ bf8v as_frag(uint4 u) {
  bf8v r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// effect points of observation b that fall into [p0, p0 + np) -> eb (LDS, zeroed)
__device__ __forceinline__ void mark_effects(const SpatialPlanes& sp, uint32_t* eb, int b, int L, int HW, int p0,
                                             int np) {
  for (int i = threadIdx.x; i < 6 * L; i += blockDim.x) {
    const int e = i / L, j = i - e * L;
    int p = sp.effect[e][static_cast<long>(b) * L + j];
    p = p < 0 ? 0 : (p >= HW ? HW - 1 : p);
    if (p >= p0 && p < p0 + np) atomicOr(&eb[p - p0], 1u << e);
  }
}

__global__ __launch_bounds__(256) void spatial_embed_mfma_kernel(SpatialPlanes sp, const float* __restrict__ wd,
                                                                 const float* __restrict__ bias,
                                                                 const bf16_t* __restrict__ rows,
                                                                 const uint8_t* __restrict__ ex,
                                                                 const uint8_t* __restrict__ ey,
                                                                 const int64_t* __restrict__ entity_num,
                                                                 bf16_t* __restrict__ out, int N, int H, int W, int L,
                                                                 int tiles) {
  __shared__ float acc_s[kSpTile][33];
  __shared__ uint32_t eb[kSpTile];
  __shared__ uint32_t msk[kSpTile];
  __shared__ uint32_t hgt[kSpTile];
  __shared__ int2 ent_list[kSpTile];
  __shared__ int ent_cnt;
  const int HW = H * W;
  const int b = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int p0 = tile * kSpTile, tid = threadIdx.x, l = tid & 63, w = tid >> 6, g = l >> 4, lr = l & 15;
  const int np = HW - p0 < kSpTile ? HW - p0 : kSpTile;
  eb[tid] = 0;
  if (tid == 0) ent_cnt = 0;
  // B fragments: B[c = 8 g + j][n = 16 nt + lr] = Wd'[n][c], hi and lo halves
  bf8v bhi[2], blo[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = 16 * nt + lr;
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t h2 = 0, l2 = 0;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int c = 8 * g + j + t;
        const float v = c < 24 ? wd[n * 24 + c] : (c == 24 ? bias[n] : 0.f);
        const bf16_t hi = f2bf(v);
        const bf16_t lo = f2bf(v - bf2f(hi));
        h2 |= static_cast<uint32_t>(hi) << (16 * t);
        l2 |= static_cast<uint32_t>(lo) << (16 * t);
      }
      hw[j / 2] = h2;
      lw[j / 2] = l2;
    }
    bhi[nt] = as_frag(make_uint4(hw[0], hw[1], hw[2], hw[3]));
    blo[nt] = as_frag(make_uint4(lw[0], lw[1], lw[2], lw[3]));
  }
  __syncthreads();
  mark_effects(sp, eb, b, L, HW, p0, np);
  __syncthreads();
  if (tid < np) {
    const long pix = static_cast<long>(b) * HW + p0 + tid;
    msk[tid] = pixel_mask(sp, pix, eb[tid]);
    hgt[tid] = f2bf(static_cast<float>(sp.height[pix]) * (1.f / 256.f));
  } else {
    msk[tid] = 0;
    hgt[tid] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int pr = 64 * w + 16 * m + lr;  // A row (pixel) of this lane
    const uint32_t mb = (msk[pr] >> (8 * g)) & 0xFFu;
    uint32_t q0 = bit_pair(mb, 0);
    if (g == 0) q0 = (q0 & 0xFFFF0000u) | hgt[pr];
    const bf8v a = as_frag(make_uint4(q0, bit_pair(mb, 2), bit_pair(mb, 4), bit_pair(mb, 6)));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      f4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bhi[nt], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, blo[nt], c, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc_s[64 * w + 16 * m + 4 * g + i][16 * nt + lr] = c[i];
    }
  }
  __syncthreads();
  // entities of this observation inside the tile: one position test per entity (a compacted LDS list),
  // then the listed rows' 32 channels in parallel
  const int ne = static_cast<int>(entity_num[b] < N ? entity_num[b] : N);
  for (int n = tid; n < ne; n += 256) {
    const long bn = static_cast<long>(b) * N + n;
    int x = ex[bn], y = ey[bn];
    x = x < W ? x : W - 1;
    y = y < H ? y : H - 1;
    const int p = y * W + x - p0;
    if (p >= 0 && p < np) {
      const int slot = atomicAdd(&ent_cnt, 1);
      if (slot < kSpTile) {
        ent_list[slot] = make_int2(n, p);
      } else {   // list full (> 256 entities in one tile): add this row directly
        for (int c = 0; c < 32; ++c) atomicAdd(&acc_s[p][c], bf2f(rows[bn * 32 + c]));
      }
    }
  }
  __syncthreads();
  const int nl = ent_cnt < kSpTile ? ent_cnt : kSpTile;
  for (int i = tid; i < nl * 32; i += 256) {
    const int c = i & 31;
    const int2 e = ent_list[i >> 5];
    const long bn = static_cast<long>(b) * N + e.x;
    atomicAdd(&acc_s[e.y][c], bf2f(rows[bn * 32 + c]));
  }
  __syncthreads();
  // relu + bf16, 8 channels (16 B) per store
  uint4* o = reinterpret_cast<uint4*>(out + (static_cast<long>(b) * HW + p0) * 32);
  for (int i = tid; i < np * 4; i += 256) {
    const int p = i >> 2, c8 = 8 * (i & 3);
    uint32_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      q[j] = f2bf2(fmaxf(acc_s[p][c8 + 2 * j], 0.f), fmaxf(acc_s[p][c8 + 2 * j + 1], 0.f));
    o[i] = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

// Pooled form: the encoder's first stage is relu(embed) -> max_pool2x2 -> conv, and the full-resolution
// embed map (B x 152 x 160 x 32 bf16 = 607 MB at the learner batch) feeds only that pool.  A tile here is one
// pair of image rows (2W <= kPoolTile pixels), so the 2x2 windows are tile-local: the kernel writes the pooled
// map and the argmax byte per channel (maxpool2's format, for its backward) and never the full map.
constexpr int kPoolTile = 320;
constexpr int kPoolMF = kPoolTile / 64;   // 16-pixel MFMA row fragments per wave

// T = bf16_t: the mixed-precision step (W as hi + lo bf16, values compared as the bf16 map would hold them);
// T = float: the fp32 step (W as three bf16 parts, ~fp32-exact products against the exact-in-bf16 planes; fp32
// entity rows, fp32 pooled output)
template <typename T>
__global__ __launch_bounds__(256) void spatial_embed_pool_kernel(SpatialPlanes sp, const float* __restrict__ wd,
                                                                 const float* __restrict__ bias,
                                                                 const T* __restrict__ rows,
                                                                 const uint8_t* __restrict__ ex,
                                                                 const uint8_t* __restrict__ ey,
                                                                 const int64_t* __restrict__ entity_num,
                                                                 T* __restrict__ pooled, uint8_t* __restrict__ pos,
                                                                 int N, int H, int W, int L) {
  constexpr bool F32 = sizeof(T) == 4;
  __shared__ float acc_s[kPoolTile][33];
  __shared__ uint32_t eb[kPoolTile];
  __shared__ uint32_t msk[kPoolTile];
  __shared__ uint32_t hgt[kPoolTile];
  __shared__ int2 ent_list[kSpTile];
  __shared__ int ent_cnt;
  const int HW = H * W, Ho = H >> 1, Wo = W >> 1;
  const int b = blockIdx.x / Ho, rp = blockIdx.x % Ho;
  const int np = 2 * W, p0 = rp * np;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, g = l >> 4, lr = l & 15;
  for (int i = tid; i < kPoolTile; i += 256) eb[i] = 0;
  if (tid == 0) ent_cnt = 0;
  bf8v bhi[2], blo[2], bl2[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int n = 16 * nt + lr;
    uint32_t hw[4], lw[4], l2w[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t h2 = 0, l2 = 0, m2 = 0;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int c = 8 * g + j + t;
        const float v = c < 24 ? wd[n * 24 + c] : (c == 24 ? bias[n] : 0.f);
        const bf16_t hi = f2bf(v);
        const float r1 = v - bf2f(hi);
        const bf16_t lo = f2bf(r1);
        const bf16_t lo2 = f2bf(r1 - bf2f(lo));
        h2 |= static_cast<uint32_t>(hi) << (16 * t);
        l2 |= static_cast<uint32_t>(lo) << (16 * t);
        m2 |= static_cast<uint32_t>(lo2) << (16 * t);
      }
      hw[j / 2] = h2;
      lw[j / 2] = l2;
      l2w[j / 2] = m2;
    }
    bhi[nt] = as_frag(make_uint4(hw[0], hw[1], hw[2], hw[3]));
    blo[nt] = as_frag(make_uint4(lw[0], lw[1], lw[2], lw[3]));
    bl2[nt] = as_frag(make_uint4(l2w[0], l2w[1], l2w[2], l2w[3]));
  }
  __syncthreads();
  mark_effects(sp, eb, b, L, HW, p0, np);
  __syncthreads();
  for (int i = tid; i < kPoolTile; i += 256) {
    if (i < np) {
      const long pix = static_cast<long>(b) * HW + p0 + i;
      msk[i] = pixel_mask(sp, pix, eb[i]);
      hgt[i] = f2bf(static_cast<float>(sp.height[pix]) * (1.f / 256.f));
    } else {
      msk[i] = 0;
      hgt[i] = 0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < kPoolMF; ++m) {
    const int pr = kPoolMF * 16 * w + 16 * m + lr;  // A row (pixel) of this lane
    const uint32_t mb = (msk[pr] >> (8 * g)) & 0xFFu;
    uint32_t q0 = bit_pair(mb, 0);
    if (g == 0) q0 = (q0 & 0xFFFF0000u) | hgt[pr];
    const bf8v a = as_frag(make_uint4(q0, bit_pair(mb, 2), bit_pair(mb, 4), bit_pair(mb, 6)));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      f4 c = f4{0.f, 0.f, 0.f, 0.f};
      if constexpr (F32) {   // smallest part first
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl2[nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, blo[nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bhi[nt], c, 0, 0, 0);
      } else {
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bhi[nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, blo[nt], c, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) acc_s[kPoolMF * 16 * w + 16 * m + 4 * g + i][16 * nt + lr] = c[i];
    }
  }
  __syncthreads();
  const int ne = static_cast<int>(entity_num[b] < N ? entity_num[b] : N);
  for (int n = tid; n < ne; n += 256) {
    const long bn = static_cast<long>(b) * N + n;
    int x = ex[bn], y = ey[bn];
    x = x < W ? x : W - 1;
    y = y < H ? y : H - 1;
    const int p = y * W + x - p0;
    if (p >= 0 && p < np) {
      const int slot = atomicAdd(&ent_cnt, 1);
      if (slot < kSpTile) {
        ent_list[slot] = make_int2(n, p);
      } else {
        for (int c = 0; c < 32; ++c) atomicAdd(&acc_s[p][c], Cvt<T>::load(rows, bn * 32 + c));
      }
    }
  }
  __syncthreads();
  const int nl = ent_cnt < kSpTile ? ent_cnt : kSpTile;
  for (int i = tid; i < nl * 32; i += 256) {
    const int c = i & 31;
    const int2 e = ent_list[i >> 5];
    const long bn = static_cast<long>(b) * N + e.x;
    atomicAdd(&acc_s[e.y][c], Cvt<T>::load(rows, bn * 32 + c));
  }
  __syncthreads();
  // relu + 2x2 max (first maximum in window order wins, NaN propagates: maxpool2_fwd's rule) -> 8 channels
  // of one pooled pixel per thread: 16-B value store + 8 argmax bytes
  const long obase = (static_cast<long>(b) * Ho + rp) * Wo;
  for (int i = tid; i < Wo * 4; i += 256) {
    const int ox = i >> 2, c8 = 8 * (i & 3);
    const int q[4] = {2 * ox, 2 * ox + 1, W + 2 * ox, W + 2 * ox + 1};
    float mv[8];
    uint32_t lo = 0, hi = 0;
    // compared as the values the unfused map would hold (bf16-rounded in the bf16 step), so ties resolve as
    // max_pool2x2 on that map
    auto held = [](float v) { return F32 ? fmaxf(v, 0.f) : bf2f(f2bf(fmaxf(v, 0.f))); };
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float m = held(acc_s[q[0]][c8 + k]);
      uint32_t pp = 0;
#pragma unroll
      for (int t = 1; t < 4; ++t) {
        const float v = held(acc_s[q[t]][c8 + k]);
        if (v > m || isnan(v)) { m = v; pp = t; }
      }
      mv[k] = m;
      if (k < 4) lo |= pp << (8 * k);
      else hi |= pp << (8 * (k - 4));
    }
    const long o = (obase + ox) * 32 + c8;
    if constexpr (F32) {
      *reinterpret_cast<float4*>(pooled + o) = make_float4(mv[0], mv[1], mv[2], mv[3]);
      *reinterpret_cast<float4*>(pooled + o + 4) = make_float4(mv[4], mv[5], mv[6], mv[7]);
    } else {
      uint32_t o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = f2bf2(mv[2 * j], mv[2 * j + 1]);
      *reinterpret_cast<uint4*>(pooled + o) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
    *reinterpret_cast<uint2*>(pos + o) = make_uint2(lo, hi);
  }
}

constexpr int kSpP = kSpTile + 8;  // padded bf16 LDS row of the dpre^T image

// 8 bf16 of v kept where the matching bf16 of g is > 0 (sign clear, not +0), zeroed elsewhere
__device__ __forceinline__ uint4 relu_gate8(uint4 v, uint4 g) {
  uint32_t a[4] = {v.x, v.y, v.z, v.w};
  const uint32_t b[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t lo = b[e] & 0xffffu, hi = b[e] >> 16;
    const uint32_t mlo = (!(lo & 0x8000u) && (lo & 0x7fffu)) ? 0xffffu : 0u;
    const uint32_t mhi = (!(hi & 0x8000u) && (hi & 0x7fffu)) ? 0xffff0000u : 0u;
    a[e] &= mlo | mhi;
  }
  return make_uint4(a[0], a[1], a[2], a[3]);
}

__global__ __launch_bounds__(256) void spatial_dense_wgrad_mfma_kernel(SpatialPlanes sp, const bf16_t* __restrict__ dpre,
                                                                       const bf16_t* __restrict__ gate,
                                                                       float* __restrict__ part, int H, int W, int L,
                                                                       int tiles, int wg_per_obs) {
  __shared__ __attribute__((aligned(16))) bf16_t dT[32 * kSpP];
  __shared__ __attribute__((aligned(16))) uint32_t msk[kSpTile];
  __shared__ __attribute__((aligned(16))) uint16_t hgt[kSpTile];
  __shared__ uint32_t eb[kSpTile];
  static_assert(sizeof(bf16_t) * 32 * kSpP >= sizeof(float) * 4 * 32 * 33, "reduction image aliases dT");
  const int HW = H * W;
  const int b = blockIdx.x / wg_per_obs, q = blockIdx.x % wg_per_obs;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, g = l >> 4, lr = l & 15;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  eb[tid] = 0;
  for (int tile = q; tile < tiles; tile += wg_per_obs) {
    const int p0 = tile * kSpTile;
    const int np = HW - p0 < kSpTile ? HW - p0 : kSpTile;
    __syncthreads();  // previous tile consumed, eb zeroed
    mark_effects(sp, eb, b, L, HW, p0, np);
    __syncthreads();
    const long base = static_cast<long>(b) * HW + p0;
    if (tid < np) {
      msk[tid] = pixel_mask(sp, base + tid, eb[tid]);
      hgt[tid] = f2bf(static_cast<float>(sp.height[base + tid]) * (1.f / 256.f));
    } else {
      msk[tid] = 0;
      hgt[tid] = 0;
    }
    {  // dpre^T: thread = (pixel pair, 16-channel half); tail pixels are zero
      const int pp = 2 * (tid & 127), h16 = 16 * (tid >> 7);
      uint4 r0[2], r1[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        r0[k] = pp < np ? *reinterpret_cast<const uint4*>(dpre + (base + pp) * 32 + h16 + 8 * k) : make_uint4(0, 0, 0, 0);
        r1[k] = pp + 1 < np ? *reinterpret_cast<const uint4*>(dpre + (base + pp + 1) * 32 + h16 + 8 * k)
                            : make_uint4(0, 0, 0, 0);
        if (gate != nullptr) {
          if (pp < np) r0[k] = relu_gate8(r0[k], *reinterpret_cast<const uint4*>(gate + (base + pp) * 32 + h16 + 8 * k));
          if (pp + 1 < np)
            r1[k] = relu_gate8(r1[k], *reinterpret_cast<const uint4*>(gate + (base + pp + 1) * 32 + h16 + 8 * k));
        }
      }
      uint32_t* d32 = reinterpret_cast<uint32_t*>(dT);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint32_t a[4] = {r0[k].x, r0[k].y, r0[k].z, r0[k].w}, c[4] = {r1[k].x, r1[k].y, r1[k].z, r1[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = h16 + 8 * k + 2 * j;
          d32[(n * kSpP + pp) >> 1] = (a[j] & 0xFFFFu) | (c[j] << 16);
          d32[((n + 1) * kSpP + pp) >> 1] = (a[j] >> 16) | (c[j] & 0xFFFF0000u);
        }
      }
    }
    __syncthreads();
    eb[tid] = 0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p = 64 * w + 32 * ks + 8 * g;
      const bf8v a0 = as_frag(*reinterpret_cast<const uint4*>(dT + lr * kSpP + p));
      const bf8v a1 = as_frag(*reinterpret_cast<const uint4*>(dT + (16 + lr) * kSpP + p));
      const uint4 m0 = *reinterpret_cast<const uint4*>(msk + p), m1 = *reinterpret_cast<const uint4*>(msk + p + 4);
      const uint4 hh = *reinterpret_cast<const uint4*>(hgt + p);
      const uint32_t mm[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
      const uint32_t hw[4] = {hh.x, hh.y, hh.z, hh.w};
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int c = 16 * ct + lr;
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = (((mm[2 * j] >> c) & 1u) ? 0x3F80u : 0u) | (((mm[2 * j + 1] >> c) & 1u) ? 0x3F800000u : 0u);
        if (c == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = hw[j];
        }
        const bf8v bx = as_frag(make_uint4(v[0], v[1], v[2], v[3]));
        acc[0][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bx, acc[0][ct], 0, 0, 0);
        acc[1][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bx, acc[1][ct], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(dT);  // [4 waves][32 n][33]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(w * 32 + 16 * nt + 4 * g + i) * 33 + 16 * ct + lr] = acc[nt][ct][i];
  __syncthreads();
  float* row = part + static_cast<long>(blockIdx.x) * (32 * 24 + 32);
  for (int i = tid; i < 32 * 25; i += 256) {
    const int nn = i / 25, k = i % 25;
    const float s = red[nn * 33 + k] + red[(32 + nn) * 33 + k] + red[(64 + nn) * 33 + k] + red[(96 + nn) * 33 + k];
    if (k < 24) row[nn * 24 + k] = s;
    else row[32 * 24 + nn] = s;
  }
}

// fp32 form of the MFMA weight gradient (the fp32 step): the dense input X is exact in bf16, so splitting only the
// fp32 dpre (gated by the projection's ReLU) exactly into three bf16 planes (split_mfma.h truncation split:
// dpre = d0 + d1 + d2) makes dW = sum_p (d0 + d1 + d2)[p][n] X[p][c] three bf16 MFMAs per step, each product exact,
// accumulated in fp32.  The scalar fp32 kernel above streams the same 2.4 GB of dpre / gate at ~1 ms per step with a
// select-add per column; the planes are staged transposed (channel-major) in LDS like the bf16 image.
// POOLED (the fused embed + max-pool stage's backward): dpre is not materialised - each pixel's value is the pooled
// gradient dpre = pdy[window] where the window's per-channel argmax (ppos) is this pixel and the pooled ReLU output
// (py) is positive, else 0 (pdy / py / ppos [B, H/2, W/2, 32]); it replaces a maxpool2_bwd_relu pass that wrote the
// 1.2 GB full-resolution dpre this kernel and the row gather then read back.
template <bool POOLED>
__global__ __launch_bounds__(256) void spatial_dense_wgrad_mfma_f32_kernel(SpatialPlanes sp, const float* __restrict__ dpre,
                                                                           const float* __restrict__ gate,
                                                                           float* __restrict__ part, int H, int W, int L,
                                                                           int tiles, int wg_per_obs,
                                                                           const float* __restrict__ py,
                                                                           const uint8_t* __restrict__ ppos) {
  __shared__ __attribute__((aligned(16))) bf16_t dT[3][32 * kSpP];
  __shared__ __attribute__((aligned(16))) uint32_t msk[kSpTile];
  __shared__ __attribute__((aligned(16))) uint16_t hgt[kSpTile];
  __shared__ uint32_t eb[kSpTile];
  static_assert(sizeof(bf16_t) * 3 * 32 * kSpP >= sizeof(float) * 4 * 32 * 33, "reduction image aliases dT");
  const int HW = H * W;
  const int b = blockIdx.x / wg_per_obs, q = blockIdx.x % wg_per_obs;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, g = l >> 4, lr = l & 15;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  eb[tid] = 0;
  for (int tile = q; tile < tiles; tile += wg_per_obs) {
    const int p0 = tile * kSpTile;
    const int np = HW - p0 < kSpTile ? HW - p0 : kSpTile;
    __syncthreads();  // previous tile consumed, eb zeroed
    mark_effects(sp, eb, b, L, HW, p0, np);
    __syncthreads();
    const long base = static_cast<long>(b) * HW + p0;
    if (tid < np) {
      msk[tid] = pixel_mask(sp, base + tid, eb[tid]);
      hgt[tid] = f2bf(static_cast<float>(sp.height[base + tid]) * (1.f / 256.f));
    } else {
      msk[tid] = 0;
      hgt[tid] = 0;
    }
    {  // split dpre^T planes: thread = (pixel pair, 16-channel half); tail pixels are zero (clamped loads + select)
      const int pp = 2 * (tid & 127), h16 = 16 * (tid >> 7);
      const bool ok0 = pp < np, ok1 = pp + 1 < np;
      long r0 = (base + (ok0 ? pp : 0)) * 32 + h16, r1 = (base + (ok1 ? pp + 1 : 0)) * 32 + h16;
      uint32_t t0 = 0, t1 = 0;
      if constexpr (POOLED) {   // the pooled pixel of each of the two pixels, and its position in the 2x2 window
        const int q0 = p0 + (ok0 ? pp : 0), q1 = p0 + (ok1 ? pp + 1 : 0);
        const int y0 = q0 / W, x0 = q0 - y0 * W, y1 = q1 / W, x1 = q1 - y1 * W;
        const long ob = static_cast<long>(b) * (H >> 1);
        r0 = ((ob + (y0 >> 1)) * (W >> 1) + (x0 >> 1)) * 32 + h16;
        r1 = ((ob + (y1 >> 1)) * (W >> 1) + (x1 >> 1)) * 32 + h16;
        t0 = static_cast<uint32_t>((y0 & 1) * 2 + (x0 & 1));
        t1 = static_cast<uint32_t>((y1 & 1) * 2 + (x1 & 1));
      }
      uint32_t* d0 = reinterpret_cast<uint32_t*>(dT[0]);
      uint32_t* d1 = reinterpret_cast<uint32_t*>(dT[1]);
      uint32_t* d2 = reinterpret_cast<uint32_t*>(dT[2]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float4 a = *reinterpret_cast<const float4*>(dpre + r0 + 4 * k);
        float4 c = *reinterpret_cast<const float4*>(dpre + r1 + 4 * k);
        float4 ga = make_float4(1.f, 1.f, 1.f, 1.f), gc = ga;
        if constexpr (POOLED) {
          // gate > 0 <=> this pixel is the channel's argmax in its window and the pooled ReLU output is positive
          const float4 ya = *reinterpret_cast<const float4*>(py + r0 + 4 * k);
          const float4 yc = *reinterpret_cast<const float4*>(py + r1 + 4 * k);
          const uint32_t pa = *reinterpret_cast<const uint32_t*>(ppos + r0 + 4 * k);
          const uint32_t pc = *reinterpret_cast<const uint32_t*>(ppos + r1 + 4 * k);
          const float yav[4] = {ya.x, ya.y, ya.z, ya.w}, ycv[4] = {yc.x, yc.y, yc.z, yc.w};
          float gav[4], gcv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            gav[j] = (((pa >> (8 * j)) & 0xffu) == t0 && yav[j] > 0.f) ? 1.f : 0.f;
            gcv[j] = (((pc >> (8 * j)) & 0xffu) == t1 && ycv[j] > 0.f) ? 1.f : 0.f;
          }
          ga = make_float4(gav[0], gav[1], gav[2], gav[3]);
          gc = make_float4(gcv[0], gcv[1], gcv[2], gcv[3]);
        } else if (gate != nullptr) {
          ga = *reinterpret_cast<const float4*>(gate + r0 + 4 * k);
          gc = *reinterpret_cast<const float4*>(gate + r1 + 4 * k);
        }
        const float av[4] = {ok0 && ga.x > 0.f ? a.x : 0.f, ok0 && ga.y > 0.f ? a.y : 0.f,
                             ok0 && ga.z > 0.f ? a.z : 0.f, ok0 && ga.w > 0.f ? a.w : 0.f};
        const float cv[4] = {ok1 && gc.x > 0.f ? c.x : 0.f, ok1 && gc.y > 0.f ? c.y : 0.f,
                             ok1 && gc.z > 0.f ? c.z : 0.f, ok1 && gc.w > 0.f ? c.w : 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = h16 + 4 * k + j;
          unsigned s0, s1, s2;
          split_pair(av[j], cv[j], s0, s1, s2);      // (pixel pp, pixel pp + 1) of channel n, per part
          const int o = (n * kSpP + pp) >> 1;
          d0[o] = s0;
          d1[o] = s1;
          d2[o] = s2;
        }
      }
    }
    __syncthreads();
    eb[tid] = 0;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p = 64 * w + 32 * ks + 8 * g;
      bf8v a0[3], a1[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        a0[pl] = as_frag(*reinterpret_cast<const uint4*>(dT[pl] + lr * kSpP + p));
        a1[pl] = as_frag(*reinterpret_cast<const uint4*>(dT[pl] + (16 + lr) * kSpP + p));
      }
      const uint4 m0 = *reinterpret_cast<const uint4*>(msk + p), m1 = *reinterpret_cast<const uint4*>(msk + p + 4);
      const uint4 hh = *reinterpret_cast<const uint4*>(hgt + p);
      const uint32_t mm[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
      const uint32_t hw[4] = {hh.x, hh.y, hh.z, hh.w};
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int c = 16 * ct + lr;
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = (((mm[2 * j] >> c) & 1u) ? 0x3F80u : 0u) | (((mm[2 * j + 1] >> c) & 1u) ? 0x3F800000u : 0u);
        if (c == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = hw[j];
        }
        const bf8v bx = as_frag(make_uint4(v[0], v[1], v[2], v[3]));
#pragma unroll
        for (int pl = 2; pl >= 0; --pl) {   // smallest part first
          acc[0][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[pl], bx, acc[0][ct], 0, 0, 0);
          acc[1][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[pl], bx, acc[1][ct], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(dT[0]);  // [4 waves][32 n][33]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(w * 32 + 16 * nt + 4 * g + i) * 33 + 16 * ct + lr] = acc[nt][ct][i];
  __syncthreads();
  float* row = part + static_cast<long>(blockIdx.x) * (32 * 24 + 32);
  for (int i = tid; i < 32 * 25; i += 256) {
    const int nn = i / 25, k = i % 25;
    const float s = red[nn * 33 + k] + red[(32 + nn) * 33 + k] + red[(64 + nn) * 33 + k] + red[(96 + nn) * 33 + k];
    if (k < 24) row[nn * 24 + k] = s;
    else row[32 * 24 + nn] = s;
  }
}

// APPLESTAR_SPATIAL_MFMA=0 selects the scalar fp32 kernels (A/B measurements)
bool spatial_mfma() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_SPATIAL_MFMA");
    return !(e && e[0] == '0');
  }();
  return on;
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return static_cast<int>(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

// APPLESTAR_UPSAMPLE_V4F=0: the generic per-output fp32 kernels (A/B switch)
bool upsample_v4f() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_UPSAMPLE_V4F");
    return !(e && e[0] == '0');
  }();
  return on;
}

void upsample2x_fwd(const void* x, void* y, int dt, int B, int H, int W, int C, hipStream_t s) {
  const long n8 = static_cast<long>(B) * H * W * (C / 8);
  if (dt == DT_BF16 && C % 8 == 0 && n8 < (1L << 31) - (1L << 24)) {
    hipLaunchKernelGGL(upsample2x_fwd_v8_kernel, dim3(grid_for(n8)), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<bf16_t*>(y), B, H, W, C);
    return;
  }
  const long n4 = static_cast<long>(B) * H * W * (C / 4);
  if (dt != DT_BF16 && C % 4 == 0 && n4 < (1L << 31) - (1L << 24) && upsample_v4f()) {
    hipLaunchKernelGGL(upsample2x_fwd_v4f_kernel, dim3(grid_for(n4)), dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), B, H, W, C);
    return;
  }
  const long n = static_cast<long>(B) * 4 * H * W * (C / 4);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(upsample2x_fwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<bf16_t*>(y), B, H, W, C);
  else
    hipLaunchKernelGGL(upsample2x_fwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), B, H, W, C);
}

void upsample2x_bwd(const void* dy, void* dx, int dt, int B, int H, int W, int C, hipStream_t s, const void* mask) {
  const long n8 = static_cast<long>(B) * H * W * (C / 8);
  if (dt == DT_BF16 && C % 8 == 0 && n8 < (1L << 31) - (1L << 24) && mask == nullptr) {
    hipLaunchKernelGGL(upsample2x_bwd_v8_kernel, dim3(grid_for(n8)), dim3(256), 0, s, static_cast<const bf16_t*>(dy),
                       static_cast<bf16_t*>(dx), B, H, W, C);
    return;
  }
  const long n = static_cast<long>(B) * H * W * (C / 4);
  if (dt != DT_BF16 && C % 4 == 0 && n < (1L << 31) - (1L << 24) && upsample_v4f()) {
    hipLaunchKernelGGL(upsample2x_bwd_v4f_kernel, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(dy),
                       static_cast<float*>(dx), B, H, W, C, static_cast<const float*>(mask));
    return;
  }
  if (dt == DT_BF16)
    hipLaunchKernelGGL(upsample2x_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(dy), static_cast<bf16_t*>(dx), B, H, W, C,
                       static_cast<const bf16_t*>(mask));
  else
    hipLaunchKernelGGL(upsample2x_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(dy),
                       static_cast<float*>(dx), B, H, W, C, static_cast<const float*>(mask));
}

bool spatial_pool_supported(int H, int W) { return H % 2 == 0 && W % 2 == 0 && 2 * W <= kPoolTile && W >= 2; }

void spatial_embed_pool(const SpatialPlanes& sp, const float* wd, const float* bias, const void* rows, const uint8_t* ex,
                        const uint8_t* ey, const int64_t* entity_num, void* pooled, uint8_t* pos, int B, int N, int H,
                        int W, int L, hipStream_t s, bool f32) {
  if (f32)
    hipLaunchKernelGGL(spatial_embed_pool_kernel<float>, dim3(B * (H / 2)), dim3(256), 0, s, sp, wd, bias,
                       static_cast<const float*>(rows), ex, ey, entity_num, static_cast<float*>(pooled), pos, N, H, W, L);
  else
    hipLaunchKernelGGL(spatial_embed_pool_kernel<bf16_t>, dim3(B * (H / 2)), dim3(256), 0, s, sp, wd, bias,
                       static_cast<const bf16_t*>(rows), ex, ey, entity_num, static_cast<bf16_t*>(pooled), pos, N, H, W,
                       L);
}

void spatial_effect_bits(const SpatialPlanes& sp, uint8_t* bits, int B, int L, int HW, hipStream_t s) {
  const long n = static_cast<long>(B) * 6 * L;
  hipLaunchKernelGGL(effect_bits_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, sp,
                     reinterpret_cast<uint32_t*>(bits), B, L, HW);
}

void spatial_dense(const SpatialPlanes& sp, const uint8_t* bits, const float* wd, const float* bias, float* pre, long npix,
                   hipStream_t s) {
  hipLaunchKernelGGL(spatial_dense_kernel, dim3(grid_for(npix)), dim3(256), 0, s, sp, bits, wd, bias, pre, npix);
}

void spatial_dense_input(const SpatialPlanes& sp, const uint8_t* bits, void* X, int x_dt, long npix, hipStream_t s) {
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(spatial_dense_input_kernel<bf16_t>, dim3(grid_for(npix)), dim3(256), 0, s, sp, bits,
                       static_cast<bf16_t*>(X), npix);
  else
    hipLaunchKernelGGL(spatial_dense_input_kernel<float>, dim3(grid_for(npix)), dim3(256), 0, s, sp, bits,
                       static_cast<float*>(X), npix);
}

void scatter_add_rows(const void* rows, int dt, const uint8_t* ex, const uint8_t* ey, const int64_t* entity_num,
                      float* pre, int B, int N, int H, int W, hipStream_t s) {
  const long n = static_cast<long>(B) * N * 32;
  if (n == 0) return;
  dim3 grid(static_cast<unsigned>((n + 255) / 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(scatter_add_rows_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(rows), ex,
                       ey, entity_num, pre, B, N, H, W);
  else
    hipLaunchKernelGGL(scatter_add_rows_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(rows), ex, ey,
                       entity_num, pre, B, N, H, W);
}

void gather_rows(const void* dpre, const void* gate, int dt, const uint8_t* ex, const uint8_t* ey,
                 const int64_t* entity_num, void* drows, int B, int N, int H, int W, hipStream_t s) {
  const long n = static_cast<long>(B) * N * 32;
  if (n == 0) return;
  dim3 grid(static_cast<unsigned>((n + 255) / 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(gather_rows_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(dpre),
                       static_cast<const bf16_t*>(gate), ex, ey, entity_num, static_cast<bf16_t*>(drows), B, N, H, W);
  else
    hipLaunchKernelGGL(gather_rows_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(dpre),
                       static_cast<const float*>(gate), ex, ey, entity_num, static_cast<float*>(drows), B, N, H, W);
}

void spatial_embed_fused(const SpatialPlanes& sp, const float* wd, const float* bias, const void* rows, int rows_dt,
                         const uint8_t* ex, const uint8_t* ey, const int64_t* entity_num, void* out, int out_dt, int B,
                         int N, int H, int W, int L, hipStream_t s) {
  const int tiles = (H * W + kSpTile - 1) / kSpTile;
  const dim3 grid(static_cast<unsigned>(B) * tiles);
  if (B == 0) return;
#define AS_SP(TR, TO)                                                                                              \
  hipLaunchKernelGGL((spatial_embed_fused_kernel<TR, TO>), grid, dim3(256), 0, s, sp, wd, bias,                    \
                     static_cast<const TR*>(rows), ex, ey, entity_num, static_cast<TO*>(out), N, H, W, L, tiles)
  if (rows_dt == DT_BF16 && out_dt == DT_BF16 && spatial_mfma())
    hipLaunchKernelGGL(spatial_embed_mfma_kernel, grid, dim3(256), 0, s, sp, wd, bias, static_cast<const bf16_t*>(rows), ex,
                       ey, entity_num, static_cast<bf16_t*>(out), N, H, W, L, tiles);
  else if (rows_dt == DT_BF16 && out_dt == DT_BF16) AS_SP(bf16_t, bf16_t);
  else if (rows_dt == DT_BF16) AS_SP(bf16_t, float);
  else if (out_dt == DT_BF16) AS_SP(float, bf16_t);
  else AS_SP(float, float);
#undef AS_SP
}

// workgroups per observation of the spatial dense wgrad: 16 (was 4: 6 waves per SIMD in one round, too few
// loads in flight for the 2.4 GB of dpre / gate the fp32 step streams)
constexpr int kSpWgPerObs = 16;
int spatial_wgrad_blocks(int B) { return B * kSpWgPerObs; }

void spatial_dense_wgrad(const SpatialPlanes& sp, const void* dpre, const void* gate, int dt, float* part, int B, int H,
                         int W, int L, hipStream_t s) {
  const int tiles = (H * W + kSpTile - 1) / kSpTile;
  if (B == 0) return;
  if (dt == DT_BF16 && spatial_mfma())
    hipLaunchKernelGGL(spatial_dense_wgrad_mfma_kernel, dim3(static_cast<unsigned>(B) * kSpWgPerObs), dim3(256), 0, s, sp,
                       static_cast<const bf16_t*>(dpre), static_cast<const bf16_t*>(gate), part, H, W, L, tiles, kSpWgPerObs);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL(spatial_dense_wgrad_kernel<bf16_t>, dim3(static_cast<unsigned>(B) * kSpWgPerObs), dim3(256), 0, s, sp,
                       static_cast<const bf16_t*>(dpre), static_cast<const bf16_t*>(gate), part, H, W, L, tiles, kSpWgPerObs);
  else if (spatial_mfma())
    hipLaunchKernelGGL(spatial_dense_wgrad_mfma_f32_kernel<false>, dim3(static_cast<unsigned>(B) * kSpWgPerObs), dim3(256),
                       0, s, sp, static_cast<const float*>(dpre), static_cast<const float*>(gate), part, H, W, L, tiles,
                       kSpWgPerObs, nullptr, nullptr);
  else
    hipLaunchKernelGGL(spatial_dense_wgrad_kernel<float>, dim3(static_cast<unsigned>(B) * kSpWgPerObs), dim3(256), 0, s, sp,
                       static_cast<const float*>(dpre), static_cast<const float*>(gate), part, H, W, L, tiles, kSpWgPerObs);
}

void spatial_dense_wgrad_pooled(const SpatialPlanes& sp, const float* dy, const float* y, const uint8_t* pos,
                                float* part, int B, int H, int W, int L, hipStream_t s) {
  const int tiles = (H * W + kSpTile - 1) / kSpTile;
  if (B == 0) return;
  hipLaunchKernelGGL(spatial_dense_wgrad_mfma_f32_kernel<true>, dim3(static_cast<unsigned>(B) * kSpWgPerObs), dim3(256),
                     0, s, sp, dy, nullptr, part, H, W, L, tiles, kSpWgPerObs, y, pos);
}

namespace {
// rows gather of the pooled form (see spatial_dense_wgrad_mfma_f32_kernel<true>): an entity at full-resolution (x, y)
// takes the pooled gradient of its window where that channel's argmax is its pixel and the pooled output is positive
__global__ __launch_bounds__(256) void gather_rows_pooled_kernel(const float* __restrict__ dy, const float* __restrict__ yp,
                                                                 const uint8_t* __restrict__ pos,
                                                                 const uint8_t* __restrict__ ex,
                                                                 const uint8_t* __restrict__ ey,
                                                                 const int64_t* __restrict__ entity_num,
                                                                 float* __restrict__ drows, int B, int N, int H, int W) {
  const long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<long>(B) * N * 32) return;
  const int c = static_cast<int>(i & 31);
  const long bn = i >> 5;
  const int b = static_cast<int>(bn / N);
  const int n = static_cast<int>(bn % N);
  float v = 0.f;
  if (n < entity_num[b]) {
    int x = ex[bn], y = ey[bn];
    x = x < W ? x : W - 1;
    y = y < H ? y : H - 1;
    const long o = ((static_cast<long>(b) * (H >> 1) + (y >> 1)) * (W >> 1) + (x >> 1)) * 32 + c;
    if (pos[o] == static_cast<uint8_t>((y & 1) * 2 + (x & 1)) && yp[o] > 0.f) v = dy[o];
  }
  drows[i] = v;
}
}  // namespace

void gather_rows_pooled(const float* dy, const float* y, const uint8_t* pos, const uint8_t* ex, const uint8_t* ey,
                        const int64_t* entity_num, float* drows, int B, int N, int H, int W, hipStream_t s) {
  const long n = static_cast<long>(B) * N * 32;
  if (n == 0) return;
  hipLaunchKernelGGL(gather_rows_pooled_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, dy, y, pos,
                     ex, ey, entity_num, drows, B, N, H, W);
}

void relu_cast(const float* x, void* y, int dt, long n, hipStream_t s) {
  if (dt == DT_BF16)
    hipLaunchKernelGGL(relu_cast_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, x, static_cast<bf16_t*>(y), n);
  else
    hipLaunchKernelGGL(relu_cast_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, x, static_cast<float*>(y), n);
}

}  // namespace as
