// Value-encoder spatial input (value_encoder.py:52-60 in the reference):
//
//     sp = relu(conv1x1(cat([scatter(units -> 8 ch), own_units_spatial, enemy_units_spatial]), 10 -> 16))
//
// over B x 152 x 160 = 9.5 M pixels per learner batch.  Here the 10-channel input is never built: each
// pixel reads its 8 scattered channels (one 16-byte vector of the NHWC scatter map) and the two bool
// planes and writes the 16 ReLU'd outputs (two lanes per pixel, 8 channels / 16 bytes each).  The cat
// path wrote a 16-channel zero-padded NHWC copy (303 MB, 0.45 ms, r2bm) and ran the projection as a
// separate pass.
//
// Backward, one pass over dOut: dPre = dOut * (out > 0); dSc = W_sc^T dPre (8 channels per pixel, the
// scatter's gradient); dW (16 x 10) and db accumulated in registers per lane, reduced across the wave by
// shuffles and across the block in LDS into one partial row per block.  The unfused chain was act_grad,
// a pointwise dX pass and a 9.5M-row weight-gradient pass over 16-channel maps.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kVsSc = 8;               // scattered unit channels
constexpr int kVsIn = kVsSc + 2;       // + own / enemy planes
constexpr int kVsOut = 16;             // output channels; two lanes per pixel, 8 each
constexpr int kVsAcc = 8 * (kVsIn + 1);  // per-lane dW / db accumulators

__device__ __forceinline__ void vs_unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f(static_cast<bf16_t>(w[i] & 0xffffu));
    f[2 * i + 1] = bf2f(static_cast<bf16_t>(w[i] >> 16));
  }
}

__device__ __forceinline__ uint4 vs_pack8(const float* f) {
  uint4 v;
  v.x = f2bf2(f[0], f[1]);
  v.y = f2bf2(f[2], f[3]);
  v.z = f2bf2(f[4], f[5]);
  v.w = f2bf2(f[6], f[7]);
  return v;
}

// 8 consecutive elements <-> fp32 registers for both I/O types (the fp32 learner step: fp32 maps end to end,
// the same fp32 FMA math as the bf16 form)
template <typename T> __device__ __forceinline__ void vs_load8(const T* p, float* f);
template <> __device__ __forceinline__ void vs_load8<bf16_t>(const bf16_t* p, float* f) {
  vs_unpack8(*reinterpret_cast<const uint4*>(p), f);
}
template <> __device__ __forceinline__ void vs_load8<float>(const float* p, float* f) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <typename T> __device__ __forceinline__ void vs_store8(T* p, const float* f);
template <> __device__ __forceinline__ void vs_store8<bf16_t>(bf16_t* p, const float* f) {
  *reinterpret_cast<uint4*>(p) = vs_pack8(f);
}
template <> __device__ __forceinline__ void vs_store8<float>(float* p, const float* f) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}
// the value the materialised map of type T would hold
template <typename T> __device__ __forceinline__ float vs_round(float v) { return v; }
template <> __device__ __forceinline__ float vs_round<bf16_t>(float v) { return bf2f(f2bf(v)); }

template <typename T>
__global__ __launch_bounds__(256) void vsp_fwd_kernel(const T* __restrict__ sc, const uint8_t* __restrict__ own,
                                                      const uint8_t* __restrict__ enemy, const float* __restrict__ w,
                                                      const float* __restrict__ b, T* __restrict__ out, long P) {
  const int h = threadIdx.x & 1;
  float wr[8][kVsIn], br[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    br[c] = b[8 * h + c];
#pragma unroll
    for (int k = 0; k < kVsIn; ++k) wr[c][k] = w[(8 * h + c) * kVsIn + k];
  }
  const long step = static_cast<long>(gridDim.x) * (blockDim.x >> 1);
  for (long pix = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 1; pix < P; pix += step) {
    float s[kVsSc];
    vs_load8<T>(sc + pix * kVsSc, s);
    const float fo = own[pix] ? 1.f : 0.f, fe = enemy[pix] ? 1.f : 0.f;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float a = fmaf(wr[c][kVsSc], fo, fmaf(wr[c][kVsSc + 1], fe, br[c]));
#pragma unroll
      for (int k = 0; k < kVsSc; ++k) a = fmaf(wr[c][k], s[k], a);
      v[c] = fmaxf(a, 0.f);
    }
    vs_store8<T>(out + pix * kVsOut + 8 * h, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void vsp_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                                      const T* __restrict__ sc, const uint8_t* __restrict__ own,
                                                      const uint8_t* __restrict__ enemy, const float* __restrict__ w,
                                                      T* __restrict__ dsc, float* __restrict__ part, long P) {
  __shared__ float red[4][2][kVsAcc];
  const int h = threadIdx.x & 1;
  float wr[8][kVsSc], acc[8][kVsIn + 1];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
#pragma unroll
    for (int k = 0; k < kVsSc; ++k) wr[c][k] = w[(8 * h + c) * kVsIn + k];
#pragma unroll
    for (int k = 0; k <= kVsIn; ++k) acc[c][k] = 0.f;
  }
  const long step = static_cast<long>(gridDim.x) * (blockDim.x >> 1);
  // both lanes of a pixel pair run the same trip count, so the pair shuffle always sees its partner
  for (long pix = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 1; pix < P; pix += step) {
    float d[8], o[8], s[kVsSc];
    vs_load8<T>(dout + pix * kVsOut + 8 * h, d);
    vs_load8<T>(out + pix * kVsOut + 8 * h, o);
    vs_load8<T>(sc + pix * kVsSc, s);
    const float fo = own[pix] ? 1.f : 0.f, fe = enemy[pix] ? 1.f : 0.f;
    float ds[kVsSc];
#pragma unroll
    for (int k = 0; k < kVsSc; ++k) ds[k] = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float g = o[c] > 0.f ? d[c] : 0.f;
#pragma unroll
      for (int k = 0; k < kVsSc; ++k) {
        acc[c][k] = fmaf(g, s[k], acc[c][k]);
        ds[k] = fmaf(wr[c][k], g, ds[k]);
      }
      acc[c][kVsSc] = fmaf(g, fo, acc[c][kVsSc]);
      acc[c][kVsSc + 1] = fmaf(g, fe, acc[c][kVsSc + 1]);
      acc[c][kVsIn] += g;
    }
#pragma unroll
    for (int k = 0; k < kVsSc; ++k) ds[k] += __shfl_xor(ds[k], 1, 64);
    if (h == 0) vs_store8<T>(dsc + pix * kVsSc, ds);
  }
  // lanes of equal parity hold partial sums of the same 88 entries: fold the 32 of each wave
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int k = 0; k <= kVsIn; ++k) {
      float v = acc[c][k];
#pragma unroll
      for (int off = 2; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
      acc[c][k] = v;
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 2) {
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int k = 0; k <= kVsIn; ++k) red[wv][lane][c * (kVsIn + 1) + k] = acc[c][k];
  }
  __syncthreads();
  // part[block][ch * 11 + k] with ch = 8 * h + c  (== h * 88 + c * 11 + k)
  for (int e = threadIdx.x; e < 2 * kVsAcc; e += blockDim.x) {
    const int hh = e / kVsAcc, j = e % kVsAcc;
    part[static_cast<long>(blockIdx.x) * 2 * kVsAcc + e] = red[0][hh][j] + red[1][hh][j] + red[2][hh][j] + red[3][hh][j];
  }
}

// Pooled forms: the value encoder applies max_pool2x2 right after this projection, so (even H, W) one lane pair
// per POOLED pixel evaluates its 2x2 window and writes the pooled map + maxpool2's argmax bytes; the 303 MB
// full-resolution map is never written or re-read.  Backward: the gradient reaches only the argmax pixel of
// each channel, and only where the pooled (ReLU) value is positive.
template <typename T>
__global__ __launch_bounds__(256) void vsp_pool_fwd_kernel(const T* __restrict__ sc, const uint8_t* __restrict__ own,
                                                           const uint8_t* __restrict__ enemy, const float* __restrict__ w,
                                                           const float* __restrict__ b, T* __restrict__ pooled,
                                                           uint8_t* __restrict__ pos, int B, int H, int W) {
  const int h = threadIdx.x & 1;
  float wr[8][kVsIn], br[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    br[c] = b[8 * h + c];
#pragma unroll
    for (int k = 0; k < kVsIn; ++k) wr[c][k] = w[(8 * h + c) * kVsIn + k];
  }
  const int Ho = H >> 1, Wo = W >> 1;
  const long Po = static_cast<long>(B) * Ho * Wo;
  const long step = static_cast<long>(gridDim.x) * (blockDim.x >> 1);
  for (long q = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 1; q < Po; q += step) {
    const int ox = static_cast<int>(q % Wo);
    const long t = q / Wo;
    const int oy = static_cast<int>(t % Ho);
    const long bb = t / Ho;
    const long p00 = (bb * H + 2 * oy) * W + 2 * ox;
    const long pix[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    float m[8];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      float s[kVsSc];
      vs_load8<T>(sc + pix[t4] * kVsSc, s);
      const float fo = own[pix[t4]] ? 1.f : 0.f, fe = enemy[pix[t4]] ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = fmaf(wr[c][kVsSc], fo, fmaf(wr[c][kVsSc + 1], fe, br[c]));
#pragma unroll
        for (int k = 0; k < kVsSc; ++k) a = fmaf(wr[c][k], s[k], a);
        const float v = vs_round<T>(fmaxf(a, 0.f));     // the value the unfused map would hold
        if (t4 == 0) {
          m[c] = v;
        } else if (v > m[c]) {
          m[c] = v;
          if (c < 4) lo = (lo & ~(0xffu << (8 * c))) | (static_cast<uint32_t>(t4) << (8 * c));
          else hi = (hi & ~(0xffu << (8 * (c - 4)))) | (static_cast<uint32_t>(t4) << (8 * (c - 4)));
        }
      }
    }
    vs_store8<T>(pooled + q * kVsOut + 8 * h, m);
    *reinterpret_cast<uint2*>(pos + q * kVsOut + 8 * h) = make_uint2(lo, hi);
  }
}

// four lanes per pooled pixel, four output channels each (acc 4 x 11 + weights 4 x 8 per lane: < 128 VGPRs, so
// the window's inputs can all be loaded before the first update without dropping below 4 waves per SIMD)
template <typename T>
__global__ __launch_bounds__(256) void vsp_pool_bwd_kernel(const T* __restrict__ dpooled,
                                                           const uint8_t* __restrict__ pos,
                                                           const T* __restrict__ pooled,
                                                           const T* __restrict__ sc, const uint8_t* __restrict__ own,
                                                           const uint8_t* __restrict__ enemy, const float* __restrict__ w,
                                                           T* __restrict__ dsc, float* __restrict__ part, int B,
                                                           int H, int W) {
  constexpr int CL = 4;                        // channels per lane
  constexpr int NA = CL * (kVsIn + 1);         // accumulators per lane
  __shared__ float red[4][4][NA];
  const int h = threadIdx.x & 3;
  float wr[CL][kVsSc], acc[CL][kVsIn + 1];
#pragma unroll
  for (int c = 0; c < CL; ++c) {
#pragma unroll
    for (int k = 0; k < kVsSc; ++k) wr[c][k] = w[(CL * h + c) * kVsIn + k];
#pragma unroll
    for (int k = 0; k <= kVsIn; ++k) acc[c][k] = 0.f;
  }
  const int Ho = H >> 1, Wo = W >> 1;
  const long Po = static_cast<long>(B) * Ho * Wo;
  const long step = static_cast<long>(gridDim.x) * (blockDim.x >> 2);
  for (long q = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2; q < Po; q += step) {
    const int ox = static_cast<int>(q % Wo);
    const long t = q / Wo;
    const int oy = static_cast<int>(t % Ho);
    const long bb = t / Ho;
    const long p00 = (bb * H + 2 * oy) * W + 2 * ox;
    // every load of the pooled pixel and its 2x2 window is issued before the first update
    float d[CL], y[CL];
    if constexpr (sizeof(T) == 4) {
      const float4 dv = *reinterpret_cast<const float4*>(dpooled + q * kVsOut + CL * h);
      const float4 yv = *reinterpret_cast<const float4*>(pooled + q * kVsOut + CL * h);
      d[0] = dv.x; d[1] = dv.y; d[2] = dv.z; d[3] = dv.w;
      y[0] = yv.x; y[1] = yv.y; y[2] = yv.z; y[3] = yv.w;
    } else {
      const uint2 dv = *reinterpret_cast<const uint2*>(dpooled + q * kVsOut + CL * h);
      const uint2 yv = *reinterpret_cast<const uint2*>(pooled + q * kVsOut + CL * h);
      const uint32_t dw[2] = {dv.x, dv.y}, yw[2] = {yv.x, yv.y};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        d[2 * i] = bf2f(static_cast<bf16_t>(dw[i] & 0xffffu));
        d[2 * i + 1] = bf2f(static_cast<bf16_t>(dw[i] >> 16));
        y[2 * i] = bf2f(static_cast<bf16_t>(yw[i] & 0xffffu));
        y[2 * i + 1] = bf2f(static_cast<bf16_t>(yw[i] >> 16));
      }
    }
    const uint32_t pp = *reinterpret_cast<const uint32_t*>(pos + q * kVsOut + CL * h);
    float s4[4][kVsSc], fo4[4], fe4[4];
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      const long px = p00 + (t4 >> 1) * W + (t4 & 1);
      vs_load8<T>(sc + px * kVsSc, s4[t4]);
      fo4[t4] = own[px] ? 1.f : 0.f;
      fe4[t4] = enemy[px] ? 1.f : 0.f;
    }
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      float g[CL];
#pragma unroll
      for (int c = 0; c < CL; ++c) {
        const uint32_t pc = (pp >> (8 * c)) & 0xffu;
        g[c] = (pc == static_cast<uint32_t>(t4) && y[c] > 0.f) ? d[c] : 0.f;
      }
      float ds[kVsSc];
#pragma unroll
      for (int k = 0; k < kVsSc; ++k) ds[k] = 0.f;
#pragma unroll
      for (int c = 0; c < CL; ++c) {
#pragma unroll
        for (int k = 0; k < kVsSc; ++k) {
          acc[c][k] = fmaf(g[c], s4[t4][k], acc[c][k]);
          ds[k] = fmaf(wr[c][k], g[c], ds[k]);
        }
        acc[c][kVsSc] = fmaf(g[c], fo4[t4], acc[c][kVsSc]);
        acc[c][kVsSc + 1] = fmaf(g[c], fe4[t4], acc[c][kVsSc + 1]);
        acc[c][kVsIn] += g[c];
      }
#pragma unroll
      for (int k = 0; k < kVsSc; ++k) {
        ds[k] += __shfl_xor(ds[k], 1, 64);
        ds[k] += __shfl_xor(ds[k], 2, 64);
      }
      if (h == 0) vs_store8<T>(dsc + (p00 + (t4 >> 1) * W + (t4 & 1)) * kVsSc, ds);
    }
  }
#pragma unroll
  for (int c = 0; c < CL; ++c)
#pragma unroll
    for (int k = 0; k <= kVsIn; ++k) {
      float v = acc[c][k];
#pragma unroll
      for (int off = 4; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
      acc[c][k] = v;
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 4) {
#pragma unroll
    for (int c = 0; c < CL; ++c)
#pragma unroll
      for (int k = 0; k <= kVsIn; ++k) red[wv][lane][c * (kVsIn + 1) + k] = acc[c][k];
  }
  __syncthreads();
  // part[block][ch * 11 + j] with ch = 4 * h + c  (== h * 44 + c * 11 + k): the layout of the other backward
  for (int e = threadIdx.x; e < 4 * NA; e += blockDim.x) {
    const int hh = e / NA, j = e % NA;
    part[static_cast<long>(blockIdx.x) * 4 * NA + e] = red[0][hh][j] + red[1][hh][j] + red[2][hh][j] + red[3][hh][j];
  }
}

}  // namespace

int vsp_in_channels() { return kVsIn; }
int vsp_out_channels() { return kVsOut; }

#define AS_VSP_T(dt, ...) \
  if (dt == DT_BF16) { using T = bf16_t; __VA_ARGS__; } else { using T = float; __VA_ARGS__; }

void vsp_fwd(const void* sc, const void* own, const void* enemy, const float* w, const float* b, void* out, long P,
             hipStream_t s, int dt) {
  long blocks = (P * 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  AS_VSP_T(dt, hipLaunchKernelGGL(vsp_fwd_kernel<T>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                                  static_cast<const T*>(sc), static_cast<const uint8_t*>(own),
                                  static_cast<const uint8_t*>(enemy), w, b, static_cast<T*>(out), P))
}

int vsp_bwd_blocks(long P) {
  long blocks = (P * 2 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  return static_cast<int>(blocks < 1 ? 1 : blocks);
}

void vsp_pool_fwd(const void* sc, const void* own, const void* enemy, const float* w, const float* b, void* pooled,
                  uint8_t* pos, int B, int H, int W, hipStream_t s, int dt) {
  const long Po = static_cast<long>(B) * (H / 2) * (W / 2);
  long blocks = (Po * 2 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  AS_VSP_T(dt, hipLaunchKernelGGL(vsp_pool_fwd_kernel<T>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                                  static_cast<const T*>(sc), static_cast<const uint8_t*>(own),
                                  static_cast<const uint8_t*>(enemy), w, b, static_cast<T*>(pooled), pos, B, H, W))
}

void vsp_pool_bwd(const void* dpooled, const uint8_t* pos, const void* pooled, const void* sc, const void* own,
                  const void* enemy, const float* w, void* dsc, float* part, int B, int H, int W, int nblk,
                  hipStream_t s, int dt) {
  AS_VSP_T(dt, hipLaunchKernelGGL(vsp_pool_bwd_kernel<T>, dim3(nblk), dim3(256), 0, s, static_cast<const T*>(dpooled),
                                  pos, static_cast<const T*>(pooled), static_cast<const T*>(sc),
                                  static_cast<const uint8_t*>(own), static_cast<const uint8_t*>(enemy), w,
                                  static_cast<T*>(dsc), part, B, H, W))
}

void vsp_bwd(const void* dout, const void* out, const void* sc, const void* own, const void* enemy, const float* w,
             void* dsc, float* part, long P, int nblk, hipStream_t s, int dt) {
  AS_VSP_T(dt, hipLaunchKernelGGL(vsp_bwd_kernel<T>, dim3(nblk), dim3(256), 0, s, static_cast<const T*>(dout),
                                  static_cast<const T*>(out), static_cast<const T*>(sc),
                                  static_cast<const uint8_t*>(own), static_cast<const uint8_t*>(enemy), w,
                                  static_cast<T*>(dsc), part, P))
}

#undef AS_VSP_T

}  // namespace as
