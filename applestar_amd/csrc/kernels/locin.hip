// Location-head input stage (action_arg_head.py:431-435 in the reference):
//
//     x = relu(conv1x1(relu(cat([reshape(fc(embedding)) -> [B,4,H,W], map_skip[-1]], 1))))
//
// As one [B*H*W, 4+128] x [4+128, 128] GEMM this has a reduction dim of 132 (not a multiple of 8; the
// library picks slow tiles) and needs the 38 MB channel concat written first (CatArrayBatchedCopy on
// channels_last ran at 0.25 ms per call, r2bk).  Split instead:
//
//     y0 = skip W_s^T + b               plain K = 128 library GEMM (host side)
//     y  = relu(y0 + W_p relu(p))       this kernel: a rank-4 update per pixel, reading p straight from
//                                       the fc output's [B, 4*H*W] layout (no reshape copy)
//
// Backward (one pass over dY): dY_m = dY * (y > 0) (feeds the dX GEMM and the native dW_s / db wgrad),
// dP[b, k, pix] = (p > 0) * sum_c dY_m[c] W_p[c, k] written in the fc output's layout, and per-block
// partial sums of dW_p = dY_m^T relu(p) (128 x 4).  The skip map needs no ReLU here: it is a ResBlock
// output (itself a ReLU), so relu(skip) == skip and its ReLU gradient is applied upstream.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kLocC = 128;              // output channels (= map_skip channels)
constexpr int kLocG = kLocC / 8;        // threads per pixel (8 channels each, one 16-byte vector)
constexpr int kLocP = 4;                // reshape channels

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f(static_cast<bf16_t>(w[i] & 0xffffu));
    f[2 * i + 1] = bf2f(static_cast<bf16_t>(w[i] >> 16));
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = f2bf2(f[0], f[1]);
  v.y = f2bf2(f[2], f[3]);
  v.z = f2bf2(f[4], f[5]);
  v.w = f2bf2(f[6], f[7]);
  return v;
}

__global__ __launch_bounds__(256) void loc_in_fwd_kernel(const bf16_t* __restrict__ y0, const bf16_t* __restrict__ p,
                                                         const float* __restrict__ wp, bf16_t* __restrict__ out,
                                                         long npix, int HW) {
  const int g = threadIdx.x % kLocG;
  float wr[8][kLocP];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int k = 0; k < kLocP; ++k) wr[c][k] = wp[(g * 8 + c) * kLocP + k];
  const long step = static_cast<long>(gridDim.x) * (blockDim.x / kLocG);
  for (long pix = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) / kLocG; pix < npix; pix += step) {
    const long b = pix / HW;
    const int q = static_cast<int>(pix - b * HW);
    const bf16_t* pb = p + b * kLocP * HW + q;
    float pv[kLocP];
#pragma unroll
    for (int k = 0; k < kLocP; ++k) pv[k] = fmaxf(bf2f(pb[static_cast<long>(k) * HW]), 0.f);
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(y0 + pix * kLocC + g * 8), v);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float a = v[c];
#pragma unroll
      for (int k = 0; k < kLocP; ++k) a = fmaf(wr[c][k], pv[k], a);
      v[c] = fmaxf(a, 0.f);
    }
    *reinterpret_cast<uint4*>(out + pix * kLocC + g * 8) = pack8(v);
  }
}

__global__ __launch_bounds__(256) void loc_in_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ p, const float* __restrict__ wp,
                                                         bf16_t* __restrict__ dym, bf16_t* __restrict__ dp,
                                                         float* __restrict__ part, long npix, int HW) {
  __shared__ float red[256][8 * kLocP + 1];
  const int g = threadIdx.x % kLocG;
  float wr[8][kLocP], acc[8][kLocP];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int k = 0; k < kLocP; ++k) {
      wr[c][k] = wp[(g * 8 + c) * kLocP + k];
      acc[c][k] = 0.f;
    }
  const long step = static_cast<long>(gridDim.x) * (blockDim.x / kLocG);
  // every lane of a pixel group runs the same trip count (the group is 16 consecutive lanes of one wave),
  // so the shuffles below always see their partners
  for (long pix = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) / kLocG; pix < npix; pix += step) {
    const long b = pix / HW;
    const int q = static_cast<int>(pix - b * HW);
    const bf16_t* pb = p + b * kLocP * HW + q;
    float pr[kLocP], pv[kLocP];
#pragma unroll
    for (int k = 0; k < kLocP; ++k) {
      pr[k] = bf2f(pb[static_cast<long>(k) * HW]);
      pv[k] = fmaxf(pr[k], 0.f);
    }
    float d[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + pix * kLocC + g * 8), d);
    unpack8(*reinterpret_cast<const uint4*>(y + pix * kLocC + g * 8), o);
    float s[kLocP] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      d[c] = o[c] > 0.f ? d[c] : 0.f;
#pragma unroll
      for (int k = 0; k < kLocP; ++k) {
        s[k] = fmaf(d[c], wr[c][k], s[k]);
        acc[c][k] = fmaf(d[c], pv[k], acc[c][k]);
      }
    }
    *reinterpret_cast<uint4*>(dym + pix * kLocC + g * 8) = pack8(d);
#pragma unroll
    for (int k = 0; k < kLocP; ++k) {
#pragma unroll
      for (int off = kLocG / 2; off > 0; off >>= 1) s[k] += __shfl_xor(s[k], off, 64);
    }
    if (g < kLocP) {
      // lane g of the group stores channel g of dP (all four sums are present in every lane)
      float sv = s[0], pg = pr[0];
#pragma unroll
      for (int k = 1; k < kLocP; ++k) {
        sv = g == k ? s[k] : sv;
        pg = g == k ? pr[k] : pg;
      }
      dp[b * kLocP * HW + static_cast<long>(g) * HW + q] = f2bf(pg > 0.f ? sv : 0.f);
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int k = 0; k < kLocP; ++k) red[threadIdx.x][c * kLocP + k] = acc[c][k];
  __syncthreads();
  // part[block][ch * 4 + k]: thread t sums the 256 / kLocG rows of channel group t / 32 for entry t % 32
  for (int e = threadIdx.x; e < kLocC * kLocP; e += blockDim.x) {
    const int grp = e / (8 * kLocP), j = e % (8 * kLocP);
    float t = 0.f;
    for (int r = grp; r < 256; r += kLocG) t += red[r][j];
    part[static_cast<long>(blockIdx.x) * kLocC * kLocP + e] = t;
  }
}

}  // namespace

bool loc_in_supported(int C, int P) { return C == kLocC && P == kLocP; }

void loc_in_fwd(const void* y0, const void* p, const float* wp, void* out, long npix, int HW, hipStream_t s) {
  long blocks = (npix * kLocG + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(loc_in_fwd_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(y0), static_cast<const bf16_t*>(p), wp, static_cast<bf16_t*>(out),
                     npix, HW);
}

int loc_in_bwd_blocks(long npix) {
  long blocks = (npix * kLocG + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  return static_cast<int>(blocks < 1 ? 1 : blocks);
}

void loc_in_bwd(const void* dy, const void* y, const void* p, const float* wp, void* dym, void* dp, float* part,
                long npix, int HW, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(loc_in_bwd_kernel, dim3(nblk), dim3(256), 0, s, static_cast<const bf16_t*>(dy),
                     static_cast<const bf16_t*>(y), static_cast<const bf16_t*>(p), wp, static_cast<bf16_t*>(dym),
                     static_cast<bf16_t*>(dp), part, npix, HW);
}

}  // namespace as
