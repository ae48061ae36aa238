// Fused bilinear x2 upsample + 3x3 conv to ONE output channel: the last stage of the location head
// (action_arg_head.py:417-450).  Unfused, this stage writes and re-reads the 32-channel
// 152x160 upsampled map (~600 MB for a 384-observation batch) and runs a Cout=1 convolution that
// GEMM-based solvers map poorly.
//
// Both operators are linear, so the channel contraction is moved BEFORE the upsample:
//   y(P) = bias + sum_k sum_c w[c,k] up_c(P + k - 1) = bias + sum_k U[z_k](P + k - 1),
//   z_k(q) = sum_c w[c,k] x_c(q)                              (a 32 -> 9 1x1 conv at LOW resolution)
// where U is the bilinear x2 interpolation (align_corners=False, source clamped at 0, PyTorch semantics)
// and terms with P+k-1 outside the image vanish (zero padding of the up-sampled map).  The 288-term
// contraction runs once per low-res pixel instead of once per high-res pixel (4x fewer FMAs) and the
// per-output work is 9 bilinear taps of an LDS-resident 9-channel tile.
// Backward uses the same factorisation:
//   dz_k(q) = sum_P a(P + k - 1, q) dy(P)      (bilinear adjoint, a 6x6 dy window per low-res pixel)
//   dx_c(q) = sum_k w[c,k] dz_k(q),  dW[c,k] = sum_q x_c(q) dz_k(q),  db = sum_P dy(P)
// in ONE kernel per low-res tile: dx is written directly, dW/db as per-tile partials that a column
// reduction sums afterwards (deterministic, no atomics).
// Layouts: x / dx NHWC [B, Hl, Wl, 32] (channels_last storage), y / dy [B, 2Hl, 2Wl] fp32.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kC = 32;  // input channels (location head: 32 -> 1)
constexpr int kK = 9;   // 3x3 taps
constexpr int kThreads = 256;

// bilinear source for a high-res coordinate (align_corners=False, scale 2)
__device__ __forceinline__ void src_index(int d, int n_in, int& i0, int& i1, float& l0, float& l1) {
  float s = (d + 0.5f) * 0.5f - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = static_cast<int>(s);
  i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
  l1 = s - static_cast<float>(i0);
  l0 = 1.f - l1;
}

// 32 channels of one NHWC pixel, 16-byte loads
__device__ __forceinline__ void load_px(const bf16_t* __restrict__ p, float v[kC]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < kC / 8; ++i) {
    const uint4 u = q[i];
    const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[i * 8 + 2 * j] = __uint_as_float(w4[j] << 16);
      v[i * 8 + 2 * j + 1] = __uint_as_float(w4[j] & 0xffff0000u);
    }
  }
}
__device__ __forceinline__ void load_px(const float* __restrict__ p, float v[kC]) {
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < kC / 4; ++i) {
    const float4 u = q[i];
    v[4 * i] = u.x; v[4 * i + 1] = u.y; v[4 * i + 2] = u.z; v[4 * i + 3] = u.w;
  }
}
__device__ __forceinline__ void store_px(bf16_t* __restrict__ p, const float v[kC]) {
  uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
  for (int i = 0; i < kC / 8; ++i) {
    uint32_t w4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w4[j] = f2bf2(v[i * 8 + 2 * j], v[i * 8 + 2 * j + 1]);
    q[i] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}
__device__ __forceinline__ void store_px(float* __restrict__ p, const float v[kC]) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < kC / 4; ++i) q[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

// ------------------------------------------------------------------------------------------ forward
// block = TH x TW high-res outputs; needs low-res rows Y0/2-1 .. Y0/2+TH/2 (TH/2+2) and likewise cols
constexpr int TH = 32, TW = 80;
constexpr int ZR = TH / 2 + 2, ZC = TW / 2 + 2, ZCP = ZC + 1;  // +1: odd row pitch

template <typename T>
__global__ __launch_bounds__(kThreads) void upconv1_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ bias_p, float* __restrict__ y,
                                                              int Hl, int Wl) {
  __shared__ float z_s[kK][ZR][ZCP];
  const int b = blockIdx.z, Y0 = blockIdx.y * TH, X0 = blockIdx.x * TW;
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  const int r0 = Y0 / 2 - 1, c0 = X0 / 2 - 1;  // low-res origin of the z tile (may be -1)
  // phase 1: z_k = w_k . x  for every low-res pixel the tile's bilinear taps can touch
  for (int e = threadIdx.x; e < ZR * ZC; e += kThreads) {
    const int r = e / ZC, cc = e % ZC;
    const int yl = r0 + r, xl = c0 + cc;
    float z[kK];
#pragma unroll
    for (int k = 0; k < kK; ++k) z[k] = 0.f;
    if (yl >= 0 && yl < Hl && xl >= 0 && xl < Wl) {
      float v[kC];
      load_px(x + ((static_cast<long>(b) * Hl + yl) * Wl + xl) * kC, v);
#pragma unroll
      for (int c = 0; c < kC; ++c)
#pragma unroll
        for (int k = 0; k < kK; ++k) z[k] = fmaf(w[c * kK + k], v[c], z[k]);
    }
#pragma unroll
    for (int k = 0; k < kK; ++k) z_s[k][r][cc] = z[k];
  }
  __syncthreads();
  const float bias = bias_p[0];
  // phase 2: y(P) = bias + sum_k U[z_k](P + k - 1)
  for (int o = threadIdx.x; o < TH * TW; o += kThreads) {
    const int Y = Y0 + o / TW, X = X0 + o % TW;
    if (Y >= H2 || X >= W2) continue;
    float acc = bias;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = Y + ky - 1;
      if (yy < 0 || yy >= H2) continue;
      int ya, yb;
      float wa, wb;
      src_index(yy, Hl, ya, yb, wa, wb);
      ya -= r0;
      yb -= r0;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = X + kx - 1;
        if (xx < 0 || xx >= W2) continue;
        int xa, xb;
        float va, vb;
        src_index(xx, Wl, xa, xb, va, vb);
        xa -= c0;
        xb -= c0;
        const int k = ky * 3 + kx;
        acc += wa * (va * z_s[k][ya][xa] + vb * z_s[k][ya][xb]) + wb * (va * z_s[k][yb][xa] + vb * z_s[k][yb][xb]);
      }
    }
    y[(static_cast<long>(b) * H2 + Y) * W2 + X] = acc;
  }
}

// ------------------------------------------------------------------------------------------ backward
// block = LH x LW low-res pixels (one per thread).  High-res pixels touching them through a tap
// (p = 2q-1 .. 2q+2) and a conv shift (P = p - k + 1): rows 2*yl0-2 .. 2*(yl0+LH-1)+3.
constexpr int LH = 16, LW = 16;
constexpr int DR = 2 * LH + 4, DC = 2 * LW + 4, DCP = DC + 1;
static_assert(LH * LW == kThreads, "one low-res pixel per thread");

// bilinear weight of low-res index q in high-res coordinate p (0 if p is outside the image)
__device__ __forceinline__ float tap_weight(int p, int q, int n_in) {
  if (p < 0 || p >= 2 * n_in) return 0.f;
  int i0, i1;
  float l0, l1;
  src_index(p, n_in, i0, i1, l0, l1);
  return (i0 == q ? l0 : 0.f) + (i1 == q ? l1 : 0.f);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void upconv1_bwd_kernel(const T* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ dy, T* __restrict__ dx,
                                                              float* __restrict__ part, int Hl, int Wl,
                                                              int relu_mask) {
  __shared__ float dy_s[DR][DCP];
  __shared__ float dz_s[kK][kThreads];
  __shared__ float x_s[kC][kThreads + 1];
  __shared__ float red_s[kThreads / kWave];
  const int b = blockIdx.z, yl0 = blockIdx.y * LH, xl0 = blockIdx.x * LW;
  const int H2 = 2 * Hl, W2 = 2 * Wl;
  const int hy0 = 2 * yl0 - 2, hx0 = 2 * xl0 - 2;
  const int t = threadIdx.x;
  float dbs = 0.f;  // db partial: high-res pixels [2*yl0, 2*(yl0+LH)) x [2*xl0, 2*(xl0+LW)) of this tile
  for (int e = t; e < DR * DC; e += kThreads) {
    const int r = e / DC, cc = e % DC;
    const int Y = hy0 + r, X = hx0 + cc;
    const float v = (Y >= 0 && Y < H2 && X >= 0 && X < W2) ? dy[(static_cast<long>(b) * H2 + Y) * W2 + X] : 0.f;
    dy_s[r][cc] = v;
    if (r >= 2 && r < 2 + 2 * LH && cc >= 2 && cc < 2 + 2 * LW) dbs += v;
  }
  __syncthreads();
  const int ly = t / LW, lx = t % LW;
  const int yl = yl0 + ly, xl = xl0 + lx;
  const bool valid = yl < Hl && xl < Wl;
  float dz[kK];
#pragma unroll
  for (int k = 0; k < kK; ++k) dz[k] = 0.f;
  if (valid) {
    // taps: high-res p = 2q - 1 + i (i = 0..3); window rows/cols of P = p - k + 1 start at 2q - 2
    float wy[4], wx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wy[i] = tap_weight(2 * yl - 1 + i, yl, Hl);
      wx[i] = tap_weight(2 * xl - 1 + i, xl, Wl);
    }
    float D[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) D[i][j] = dy_s[2 * ly + i][2 * lx + j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float row = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) row = fmaf(wx[j], D[i + 2 - ky][j + 2 - kx], row);
          acc = fmaf(wy[i], row, acc);
        }
        dz[ky * 3 + kx] = acc;
      }
  }
  float v[kC];
#pragma unroll
  for (int c = 0; c < kC; ++c) v[c] = 0.f;
  if (valid) {
    const long px = ((static_cast<long>(b) * Hl + yl) * Wl + xl) * kC;
    load_px(x + px, v);
    float g[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kK; ++k) s = fmaf(w[c * kK + k], dz[k], s);
      // x is a ReLU output: its mask (x > 0) = relu'(pre) is applied here, the producer skips its threshold pass
      g[c] = (relu_mask && !(v[c] > 0.f)) ? 0.f : s;
    }
    store_px(dx + px, g);
  }
#pragma unroll
  for (int k = 0; k < kK; ++k) dz_s[k][t] = dz[k];
#pragma unroll
  for (int c = 0; c < kC; ++c) x_s[c][t] = v[c];
  dbs = wave_sum(dbs);
  if ((t & (kWave - 1)) == 0) red_s[t / kWave] = dbs;
  __syncthreads();
  // per-tile dW[c,k] = sum_q x_c(q) dz_k(q); thread p owns one (c,k)
  const long tile = (static_cast<long>(blockIdx.z) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  float* out = part + tile * (kC * kK + 1);
  for (int p = t; p < kC * kK; p += kThreads) {
    const int c = p / kK, k = p % kK;
    float acc = 0.f;
    for (int q = 0; q < kThreads; ++q) acc = fmaf(x_s[c][q], dz_s[k][q], acc);
    out[p] = acc;
  }
  if (t == 0) {
    float s = 0.f;
    for (int i = 0; i < kThreads / kWave; ++i) s += red_s[i];
    out[kC * kK] = s;
  }
}

}  // namespace

int upconv1_channels() { return kC; }

long upconv1_tiles(int B, int Hl, int Wl) {
  return static_cast<long>(B) * ((Hl + LH - 1) / LH) * ((Wl + LW - 1) / LW);
}

void upconv1_fwd(const void* x, int x_dt, const float* w, const float* bias, float* y, int B, int Hl, int Wl,
                 hipStream_t s) {
  const dim3 grid((2 * Wl + TW - 1) / TW, (2 * Hl + TH - 1) / TH, B);
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(upconv1_fwd_kernel<bf16_t>, grid, dim3(kThreads), 0, s, static_cast<const bf16_t*>(x), w, bias,
                       y, Hl, Wl);
  else
    hipLaunchKernelGGL(upconv1_fwd_kernel<float>, grid, dim3(kThreads), 0, s, static_cast<const float*>(x), w, bias, y,
                       Hl, Wl);
}

void upconv1_bwd(const void* x, int x_dt, const float* w, const float* dy, void* dx, float* part, float* dwb, int B,
                 int Hl, int Wl, hipStream_t s, bool relu_mask) {
  const dim3 grid((Wl + LW - 1) / LW, (Hl + LH - 1) / LH, B);
  const long tiles = upconv1_tiles(B, Hl, Wl);
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(upconv1_bwd_kernel<bf16_t>, grid, dim3(kThreads), 0, s, static_cast<const bf16_t*>(x), w, dy,
                       static_cast<bf16_t*>(dx), part, Hl, Wl, relu_mask ? 1 : 0);
  else
    hipLaunchKernelGGL(upconv1_bwd_kernel<float>, grid, dim3(kThreads), 0, s, static_cast<const float*>(x), w, dy,
                       static_cast<float*>(dx), part, Hl, Wl, relu_mask ? 1 : 0);
  column_reduce(part, dwb, static_cast<int>(tiles), kC * kK + 1, s);
}

}  // namespace as
