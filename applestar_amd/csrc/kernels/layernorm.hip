// Fused (residual +) LayerNorm (+ activation) forward/backward for gfx950.
//
// One 64-lane wave owns one row; each lane holds VPT = cols/64 values in registers, loaded as
// CH-element vectors (8-16 B per lane) so a wave-instruction moves 512 B-1 KiB contiguous.  Row
// statistics are 64-wide __shfl_xor reductions; nothing touches LDS in the forward.  The backward
// accumulates dgamma/dbeta per wave in registers across a grid-stride loop, combines the block's
// 4 waves through LDS and writes one partial row per block; column_reduce() finishes the sum.
// Replaces torch's (x + r) -> layer_norm -> relu chains in the entity transformer (3 layers x 2),
// the ResFC/ResFC2 blocks of the heads and the 16-block value networks.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <int CH> struct VecIO;
template <> struct VecIO<4> {
  __device__ static void load(const float* p, long i, float* v) {
    float4 t = *reinterpret_cast<const float4*>(p + i);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static void load(const bf16_t* p, long i, float* v) {
    uint2 t = *reinterpret_cast<const uint2*>(p + i);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  }
  __device__ static void store(float* p, long i, const float* v) {
    *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ static void store(bf16_t* p, long i, const float* v) {
    uint2 t;
    t.x = f2bf2(v[0], v[1]);
    t.y = f2bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p + i) = t;
  }
};
template <> struct VecIO<2> {
  __device__ static void load(const float* p, long i, float* v) {
    float2 t = *reinterpret_cast<const float2*>(p + i);
    v[0] = t.x; v[1] = t.y;
  }
  __device__ static void load(const bf16_t* p, long i, float* v) {
    uint32_t t = *reinterpret_cast<const uint32_t*>(p + i);
    v[0] = __uint_as_float(t << 16); v[1] = __uint_as_float(t & 0xffff0000u);
  }
  __device__ static void store(float* p, long i, const float* v) {
    *reinterpret_cast<float2*>(p + i) = make_float2(v[0], v[1]);
  }
  __device__ static void store(bf16_t* p, long i, const float* v) {
    *reinterpret_cast<uint32_t*>(p + i) =
        f2bf2(v[0], v[1]);
  }
};
template <> struct VecIO<1> {
  template <typename T> __device__ static void load(const T* p, long i, float* v) { v[0] = Cvt<T>::load(p, i); }
  template <typename T> __device__ static void store(T* p, long i, const float* v) { Cvt<T>::store(p, i, v[0]); }
};

template <int VPT> struct Layout {
  static constexpr int CH = (VPT % 4 == 0) ? 4 : (VPT % 2 == 0 ? 2 : 1);
  static constexpr int NIT = VPT / CH;
  // element index of (iteration k, component c) for lane l
  __device__ static int col(int k, int lane, int c) { return (k * kWave + lane) * CH + c; }
};

template <int VPT, typename T>
__device__ __forceinline__ void load_row(const T* p, long base, int lane, float* v) {
  using L = Layout<VPT>;
#pragma unroll
  for (int k = 0; k < L::NIT; ++k) VecIO<L::CH>::load(p, base + L::col(k, lane, 0), v + k * L::CH);
}

template <int VPT, typename T>
__device__ __forceinline__ void store_row(T* p, long base, int lane, const float* v) {
  using L = Layout<VPT>;
#pragma unroll
  for (int k = 0; k < L::NIT; ++k) VecIO<L::CH>::store(p, base + L::col(k, lane, 0), v + k * L::CH);
}

template <int VPT, typename TX, typename TR, typename TY>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const TX* __restrict__ x, const TR* __restrict__ res,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     TY* __restrict__ y, float* __restrict__ xsum,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     long rows, float eps, int act) {
  constexpr int C = VPT * kWave;
  using L = Layout<VPT>;
  const int lane = threadIdx.x & 63;
  const long wave_id = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = (static_cast<long>(gridDim.x) * blockDim.x) >> 6;
  float wv[VPT], bv[VPT];
  load_row<VPT>(w, 0, lane, wv);
  load_row<VPT>(b, 0, lane, bv);
  for (long r = wave_id; r < rows; r += nwaves) {
    const long base = r * C;
    float v[VPT];
    load_row<VPT>(x, base, lane, v);
    if (res != nullptr) {
      float rv[VPT];
      load_row<VPT>(res, base, lane, rv);
#pragma unroll
      for (int i = 0; i < VPT; ++i) v[i] += rv[i];
      if (xsum != nullptr) store_row<VPT>(xsum, base, lane, v);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) s += v[i];
    const float mu = wave_sum(s) * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) { const float d = v[i] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) * (1.f / C) + eps);
#pragma unroll
    for (int i = 0; i < VPT; ++i) v[i] = apply_act((v[i] - mu) * rs * wv[i] + bv[i], act);
    store_row<VPT>(y, base, lane, v);
    if (lane == 0) { mean_out[r] = mu; rstd_out[r] = rs; }
  }
  (void)L::NIT;
}

template <int VPT, typename TD, typename TX, typename TY, typename TO>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TD* __restrict__ dy, const TX* __restrict__ xin,
                                                     const TY* __restrict__ y, const float* __restrict__ w,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     TO* __restrict__ dx, float* __restrict__ dw_part,
                                                     float* __restrict__ db_part, long rows, int act,
                                                     const float* __restrict__ msrc, float* __restrict__ dxm) {
  constexpr int C = VPT * kWave;
  __shared__ float red[4][2][C];
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const long wave_id = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = (static_cast<long>(gridDim.x) * blockDim.x) >> 6;
  float wv[VPT], dwa[VPT], dba[VPT];
  load_row<VPT>(w, 0, lane, wv);
#pragma unroll
  for (int i = 0; i < VPT; ++i) { dwa[i] = 0.f; dba[i] = 0.f; }
  for (long r = wave_id; r < rows; r += nwaves) {
    const long base = r * C;
    float g[VPT], xh[VPT];
    load_row<VPT>(dy, base, lane, g);
    if (act != ACT_NONE) {
      float yv[VPT];
      load_row<VPT>(y, base, lane, yv);
#pragma unroll
      for (int i = 0; i < VPT; ++i) g[i] *= act_grad_from_out(yv[i], act);
    }
    load_row<VPT>(xin, base, lane, xh);
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      xh[i] = (xh[i] - mu) * rs;
      const float gd = g[i] * wv[i];
      s1 += gd;
      s2 += gd * xh[i];
      dwa[i] += g[i] * xh[i];
      dba[i] += g[i];
    }
    s1 = wave_sum(s1) * (1.f / C);
    s2 = wave_sum(s2) * (1.f / C);
    float o[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) o[i] = rs * (g[i] * wv[i] - s1 - xh[i] * s2);
    store_row<VPT>(dx, base, lane, o);
    if (dxm) {
      // x is an fp32 ReLU output: its masked gradient as a second output (the residual branch keeps dx unmasked)
      float m[VPT];
      load_row<VPT>(msrc, base, lane, m);
#pragma unroll
      for (int i = 0; i < VPT; ++i) o[i] = m[i] > 0.f ? o[i] : 0.f;
      store_row<VPT>(dxm, base, lane, o);
    }
  }
  store_row<VPT>(&red[wib][0][0], 0, lane, dwa);
  store_row<VPT>(&red[wib][1][0], 0, lane, dba);
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float sw = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    const float sb = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    // [nblk][2C] layout (db_part = dw_part + C): both affine gradients reduce in ONE column pass
    dw_part[static_cast<long>(blockIdx.x) * 2 * C + c] = sw;
    db_part[static_cast<long>(blockIdx.x) * 2 * C + c] = sb;
  }
}

int fwd_blocks(long rows) {
  long b = (rows + 3) / 4;
  return static_cast<int>(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

template <int VPT>
void fwd_dispatch(const void* x, int x_dt, const void* res, int res_dt, const float* w, const float* b, void* y,
                  int y_dt, float* xsum, float* mean, float* rstd, long rows, float eps, int act, hipStream_t s) {
  dim3 grid(fwd_blocks(rows)), block(256);
#define LN_FWD(TX, TR, TY)                                                                              \
  hipLaunchKernelGGL((ln_fwd_kernel<VPT, TX, TR, TY>), grid, block, 0, s, static_cast<const TX*>(x),      \
                     static_cast<const TR*>(res), w, b, static_cast<TY*>(y), xsum, mean, rstd, rows, eps, act)
  // residual dtype: when res == nullptr any instantiation works; use the x type
  const int rdt = res ? res_dt : x_dt;
  if (x_dt == DT_F32 && rdt == DT_F32 && y_dt == DT_F32) LN_FWD(float, float, float);
  else if (x_dt == DT_BF16 && rdt == DT_F32 && y_dt == DT_F32) LN_FWD(bf16_t, float, float);
  else if (x_dt == DT_BF16 && rdt == DT_BF16 && y_dt == DT_F32) LN_FWD(bf16_t, bf16_t, float);
  else if (x_dt == DT_BF16 && rdt == DT_BF16 && y_dt == DT_BF16) LN_FWD(bf16_t, bf16_t, bf16_t);
  else if (x_dt == DT_F32 && rdt == DT_BF16 && y_dt == DT_F32) LN_FWD(float, bf16_t, float);
  else if (x_dt == DT_BF16 && rdt == DT_F32 && y_dt == DT_BF16) LN_FWD(bf16_t, float, bf16_t);
  else if (x_dt == DT_F32 && rdt == DT_F32 && y_dt == DT_BF16) LN_FWD(float, float, bf16_t);
  else LN_FWD(float, bf16_t, bf16_t);
#undef LN_FWD
}

template <int VPT>
void bwd_dispatch(const void* dy, int dy_dt, const void* xin, int xin_dt, const void* y, int y_dt, const float* w,
                  const float* mean, const float* rstd, void* dx, int dx_dt, float* dwp, float* dbp, long rows,
                  int act, int nblk, hipStream_t s, const float* msrc, float* dxm) {
  dim3 grid(nblk), block(256);
#define LN_BWD(TD, TX, TY, TO)                                                                           \
  hipLaunchKernelGGL((ln_bwd_kernel<VPT, TD, TX, TY, TO>), grid, block, 0, s, static_cast<const TD*>(dy), \
                     static_cast<const TX*>(xin), static_cast<const TY*>(y), w, mean, rstd, static_cast<TO*>(dx), \
                     dwp, dbp, rows, act, msrc, dxm)
  // y dtype == dy dtype in every use (y is the forward output, dy its gradient)
  if (dy_dt == DT_F32 && xin_dt == DT_F32 && dx_dt == DT_F32) LN_BWD(float, float, float, float);
  else if (dy_dt == DT_F32 && xin_dt == DT_BF16 && dx_dt == DT_BF16) LN_BWD(float, bf16_t, float, bf16_t);
  else if (dy_dt == DT_F32 && xin_dt == DT_BF16 && dx_dt == DT_F32) LN_BWD(float, bf16_t, float, float);
  else if (dy_dt == DT_BF16 && xin_dt == DT_BF16 && dx_dt == DT_BF16) LN_BWD(bf16_t, bf16_t, bf16_t, bf16_t);
  else if (dy_dt == DT_BF16 && xin_dt == DT_F32 && dx_dt == DT_F32) LN_BWD(bf16_t, float, bf16_t, float);
  else if (dy_dt == DT_F32 && xin_dt == DT_F32 && dx_dt == DT_BF16) LN_BWD(float, float, float, bf16_t);
  else if (dy_dt == DT_BF16 && xin_dt == DT_F32 && dx_dt == DT_BF16) LN_BWD(bf16_t, float, bf16_t, bf16_t);
  else LN_BWD(bf16_t, bf16_t, bf16_t, float);
#undef LN_BWD
  (void)y_dt;
}

}  // namespace

int layer_norm_bwd_blocks(long rows) {
  long b = (rows + 31) / 32;  // >= 8 rows per wave to amortise the dgamma/dbeta partials
  return static_cast<int>(b < 512 ? (b < 1 ? 1 : b) : 512);
}

#define VPT_SWITCH(cols, F, ...)                      \
  switch ((cols) / kWave) {                           \
    case 1: F<1>(__VA_ARGS__); break;                 \
    case 2: F<2>(__VA_ARGS__); break;                 \
    case 4: F<4>(__VA_ARGS__); break;                 \
    case 6: F<6>(__VA_ARGS__); break;                 \
    case 8: F<8>(__VA_ARGS__); break;                 \
    case 16: F<16>(__VA_ARGS__); break;               \
    case 24: F<24>(__VA_ARGS__); break;               \
    default: break;                                   \
  }

void layer_norm_fwd(const void* x, int x_dt, const void* res, int res_dt, const float* w, const float* b, void* y,
                    int y_dt, float* xsum, float* mean, float* rstd, long rows, int cols, float eps, int act,
                    hipStream_t s) {
  VPT_SWITCH(cols, fwd_dispatch, x, x_dt, res, res_dt, w, b, y, y_dt, xsum, mean, rstd, rows, eps, act, s);
}

void layer_norm_bwd(const void* dy, int dy_dt, const void* xin, int xin_dt, const void* y, int y_dt, const float* w,
                    const float* mean, const float* rstd, void* dx, int dx_dt, float* dw_part, float* db_part,
                    long rows, int cols, int act, int nblk, hipStream_t s, const float* msrc, float* dxm) {
  VPT_SWITCH(cols, bwd_dispatch, dy, dy_dt, xin, xin_dt, y, y_dt, w, mean, rstd, dx, dx_dt, dw_part, db_part, rows,
             act, nblk, s, msrc, dxm);
}

}  // namespace as
