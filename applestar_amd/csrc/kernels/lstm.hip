// Persistent LayerNorm-LSTM recurrence (forward + BPTT) for gfx950.
//
// Cell (lstm.py:138-153): gates = xp[t] + LN_h(h W_hh^T); i,f,g,o = chunk(gates)
//                         c' = LN_c(sig(f) c + sig(i) tanh(g));  h' = sig(o) tanh(c')
// xp[t] = LN_i(x[t] W_ih^T) has no recurrence and is computed for all T by one GEMM outside.
//
// One workgroup owns one batch row for the whole sequence (rows are independent), so a launch
// replaces T x ~12 torch kernels per layer.  Thread t computes COLS contiguous columns of the
// recurrent GEMV (8-byte bf16 / 16-byte fp32 loads of W^T rows, coalesced across the workgroup),
// LN statistics are two-pass block reductions (wave shuffles + LDS), the hidden state lives in LDS.
// Core LSTM: H=384 -> 384 threads x 4 columns; selected-units LSTM: H=32 -> 64 threads x 2.
// The backward walks t = T-1..0 and emits d(xp), d(h_{t-1} W^T) (for one dW GEMM afterwards) and
// the LN_c output gradient (for the affine-parameter reductions).
#include <cstdlib>

#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  constexpr int NW = NT / kWave;
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // scratch reuse guard
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += scratch[i];
  return s;
}

// two block sums with one barrier pair (wave shuffles + a float2 LDS slot per wave)
template <int NT>
__device__ __forceinline__ float2 block_sum2(float a, float b, float* scratch) {
  constexpr int NW = NT / kWave;
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // scratch reuse guard
  if ((threadIdx.x & 63) == 0) { scratch[2 * w] = a; scratch[2 * w + 1] = b; }
  __syncthreads();
  float2 r = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NW; ++i) { r.x += scratch[2 * i]; r.y += scratch[2 * i + 1]; }
  return r;
}

// register-resident weight slice of N values; bf16 weights stay packed two per VGPR (halves the
// split kernels' weight registers: 96 -> 48, which removed the backward's scratch spill)
template <typename TW, int N> struct RegW;
template <int N> struct RegW<float, N> {
  float v[N];
  __device__ __forceinline__ void load(int i, const float* p, long off) { v[i] = p[off]; }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
};
template <int N> struct RegW<bf16_t, N> {
  static_assert(N % 2 == 0, "pairs");
  uint32_t v[N / 2];
  __device__ __forceinline__ void load(int i, const bf16_t* p, long off) {
    const uint32_t x = p[off];
    if (i & 1) v[i >> 1] |= x << 16;
    else v[i >> 1] = x;
  }
  __device__ __forceinline__ float get(int i) const {
    return (i & 1) ? __uint_as_float(v[i >> 1] & 0xffff0000u) : __uint_as_float(v[i >> 1] << 16);
  }
};

template <typename TW, int COLS> struct WLoad;
template <> struct WLoad<bf16_t, 4> {
  __device__ static void load(const bf16_t* p, float* v) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  }
};
template <> struct WLoad<bf16_t, 2> {
  __device__ static void load(const bf16_t* p, float* v) {
    const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
    v[0] = __uint_as_float(t << 16); v[1] = __uint_as_float(t & 0xffff0000u);
  }
};
template <> struct WLoad<float, 4> {
  __device__ static void load(const float* p, float* v) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
};
template <> struct WLoad<float, 2> {
  __device__ static void load(const float* p, float* v) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  }
};

// one 16-byte load: 8 bf16 or 4 fp32 values
template <typename TW> struct WLoad16;
template <> struct WLoad16<bf16_t> {
  __device__ static void load(const bf16_t* p, float* v) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
    v[4] = __uint_as_float(t.z << 16); v[5] = __uint_as_float(t.z & 0xffff0000u);
    v[6] = __uint_as_float(t.w << 16); v[7] = __uint_as_float(t.w & 0xffff0000u);
  }
};
template <> struct WLoad16<float> {
  __device__ static void load(const float* p, float* v) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
};

// Forward for the wide (H = 384) core LSTM: the h W^T GEMV is split over SPLIT groups of rows with
// 16-byte loads (8 bf16 columns per thread), so ~4x more bytes are in flight than the one-thread-per-
// 4-columns layout; the per-row recurrence is unchanged (one workgroup per batch row).
template <int H, int NT, typename TW>
__global__ __launch_bounds__(NT) void lnlstm_fwd_wide_kernel(
    const float* __restrict__ xp, const float* __restrict__ h0, const float* __restrict__ c0,
    const TW* __restrict__ wT, const float* __restrict__ lnh_w, const float* __restrict__ lnh_b,
    const float* __restrict__ lnc_w, const float* __restrict__ lnc_b, int T, int B, float eps,
    float* __restrict__ out, float* __restrict__ c_all, float* __restrict__ xhat_h, float* __restrict__ rstd_h,
    float* __restrict__ gates_out, float* __restrict__ xhat_c, float* __restrict__ rstd_c, float* __restrict__ hT,
    float* __restrict__ cT) {
  constexpr int G = 4 * H;
  constexpr int VW = sizeof(TW) == 2 ? 8 : 4;   // columns per 16-byte load
  constexpr int CG = G / VW;                    // column groups
  constexpr int SPLIT = NT / CG;                // row splits of the reduction
  constexpr int COLS = G / NT;                  // columns per thread in the LN / gate phase
  static_assert(NT % CG == 0 && H % SPLIT == 0 && G % NT == 0 && NT >= H, "wide tiling");
  constexpr int RS = H / SPLIT;
  __shared__ float h_s[H];
  __shared__ float g_s[G];
  __shared__ float part[SPLIT][G];
  __shared__ float red[2 * (NT / kWave)];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const int cg = tid % CG, sp = tid / CG;
  float c = 0.f, lcw = 0.f, lcb = 0.f;
  if (unit) {
    h_s[tid] = h0[static_cast<long>(b) * H + tid];
    c = c0[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
    lcb = lnc_b[tid];
    c_all[static_cast<long>(b) * H + tid] = c;
  }
  float lw[COLS], lb[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) { lw[k] = lnh_w[tid * COLS + k]; lb[k] = lnh_b[tid * COLS + k]; }
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float acc[VW];
#pragma unroll
    for (int v = 0; v < VW; ++v) acc[v] = 0.f;
    const TW* wp = wT + cg * VW;
#pragma unroll 16
    for (int i = sp * RS; i < sp * RS + RS; ++i) {
      float wv[VW];
      WLoad16<TW>::load(wp + static_cast<long>(i) * G, wv);
      const float hv = h_s[i];
#pragma unroll
      for (int v = 0; v < VW; ++v) acc[v] = fmaf(hv, wv[v], acc[v]);
    }
#pragma unroll
    for (int v = 0; v < VW; ++v) part[sp][cg * VW + v] = acc[v];
    __syncthreads();
    float a[COLS];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < SPLIT; ++q) v += part[q][tid * COLS + k];
      a[k] = v;
      s += v;
    }
    float q2 = 0.f;   // LN_h statistics in one reduction (sum, sum of squares)
#pragma unroll
    for (int k = 0; k < COLS; ++k) q2 += a[k] * a[k];
    const float2 sq = block_sum2<NT>(s, q2, red);
    const float mu = sq.x * (1.f / G);
    const float rs = rsqrtf(fmaxf(sq.y * (1.f / G) - mu * mu, 0.f) + eps);
    const long row = static_cast<long>(t) * B + b;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float xh = (a[k] - mu) * rs;
      const float gv = xp[row * G + j] + xh * lw[k] + lb[k];
      xhat_h[row * G + j] = xh;
      gates_out[row * G + j] = gv;
      g_s[j] = gv;
    }
    if (tid == 0) rstd_h[row] = rs;
    __syncthreads();
    float cpre = 0.f, og = 0.f;
    if (unit) {
      const float ig = sigmoidf_(g_s[tid]);
      const float fg = sigmoidf_(g_s[H + tid]);
      const float gg = tanhf(g_s[2 * H + tid]);
      og = sigmoidf_(g_s[3 * H + tid]);
      cpre = fg * c + ig * gg;
    }
    // LN_c statistics in one reduction (sum, sum of squares)
    const float2 sc2 = block_sum2<NT>(unit ? cpre : 0.f, unit ? cpre * cpre : 0.f, red);
    const float muc = sc2.x * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(fmaxf(sc2.y * (1.f / H) - muc * muc, 0.f) + eps);
    if (unit) {
      const float xc = dc * rsc;
      c = xc * lcw + lcb;
      const float hv = og * tanhf(c);
      out[row * H + tid] = hv;
      c_all[(row + B) * H + tid] = c;
      xhat_c[row * H + tid] = xc;
      h_s[tid] = hv;
      if (t == T - 1) { hT[static_cast<long>(b) * H + tid] = hv; cT[static_cast<long>(b) * H + tid] = c; }
    }
    if (tid == 0) rstd_c[row] = rsc;
    __syncthreads();
  }
  if (T == 0 && unit) { hT[static_cast<long>(b) * H + tid] = h_s[tid]; cT[static_cast<long>(b) * H + tid] = c; }
}

// wT: W_hh transposed, [H][4H] row-major
template <int H, int NT, int COLS, typename TW>
__global__ __launch_bounds__(NT) void lnlstm_fwd_kernel(
    const float* __restrict__ xp, const float* __restrict__ h0, const float* __restrict__ c0,
    const TW* __restrict__ wT, const float* __restrict__ lnh_w, const float* __restrict__ lnh_b,
    const float* __restrict__ lnc_w, const float* __restrict__ lnc_b, int T, int B, float eps,
    float* __restrict__ out, float* __restrict__ c_all, float* __restrict__ xhat_h, float* __restrict__ rstd_h,
    float* __restrict__ gates_out, float* __restrict__ xhat_c, float* __restrict__ rstd_c, float* __restrict__ hT,
    float* __restrict__ cT) {
  static_assert(NT * COLS == 4 * H, "tiling");
  static_assert(NT >= H, "one thread per hidden unit");
  constexpr int G = 4 * H;
  __shared__ float h_s[H];
  __shared__ float g_s[G];
  __shared__ float red[2 * (NT / kWave)];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  float c = 0.f, lcw = 0.f, lcb = 0.f;
  if (unit) {
    h_s[tid] = h0[static_cast<long>(b) * H + tid];
    c = c0[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
    lcb = lnc_b[tid];
    c_all[static_cast<long>(b) * H + tid] = c;  // c_all[0] = c0
  }
  float lw[COLS], lb[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) { lw[k] = lnh_w[tid * COLS + k]; lb[k] = lnh_b[tid * COLS + k]; }
  // the whole W^T column slice of this thread in registers (H x COLS: 64 values at H = 32), loaded once - the
  // per-step L2 stream of W was the recurrence's critical path (one dependent load round trip per step)
  RegW<TW, H * COLS> wreg;
#pragma unroll
  for (int i = 0; i < H; ++i)
#pragma unroll
    for (int k = 0; k < COLS; ++k) wreg.load(i * COLS + k, wT, static_cast<long>(i) * G + tid * COLS + k);
  // the input projection of the next step is fetched during this one
  float xpc[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) xpc[k] = T > 0 ? xp[static_cast<long>(b) * G + tid * COLS + k] : 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float xpn[COLS];
    {
      const long nrow = static_cast<long>(t + 1 < T ? t + 1 : t) * B + b;
#pragma unroll
      for (int k = 0; k < COLS; ++k) xpn[k] = xp[nrow * G + tid * COLS + k];
    }
    float acc[COLS];
#pragma unroll
    for (int k = 0; k < COLS; ++k) acc[k] = 0.f;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float hv = h_s[i];
#pragma unroll
      for (int k = 0; k < COLS; ++k) acc[k] = fmaf(hv, wreg.get(i * COLS + k), acc[k]);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) s += acc[k];
    float q = 0.f;   // LN_h statistics in one reduction (sum, sum of squares)
#pragma unroll
    for (int k = 0; k < COLS; ++k) q += acc[k] * acc[k];
    const float2 sq = block_sum2<NT>(s, q, red);
    const float mu = sq.x * (1.f / G);
    const float rs = rsqrtf(fmaxf(sq.y * (1.f / G) - mu * mu, 0.f) + eps);
    const long row = static_cast<long>(t) * B + b;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float xh = (acc[k] - mu) * rs;
      const float gv = xpc[k] + xh * lw[k] + lb[k];
      xhat_h[row * G + j] = xh;
      gates_out[row * G + j] = gv;
      g_s[j] = gv;
    }
    if (tid == 0) rstd_h[row] = rs;
#pragma unroll
    for (int k = 0; k < COLS; ++k) xpc[k] = xpn[k];
    __syncthreads();
    float cpre = 0.f, og = 0.f;
    if (unit) {
      const float ig = sigmoidf_(g_s[tid]);
      const float fg = sigmoidf_(g_s[H + tid]);
      const float gg = tanhf(g_s[2 * H + tid]);
      og = sigmoidf_(g_s[3 * H + tid]);
      cpre = fg * c + ig * gg;
    }
    // LN_c statistics in one reduction (sum, sum of squares)
    const float2 sc2 = block_sum2<NT>(unit ? cpre : 0.f, unit ? cpre * cpre : 0.f, red);
    const float muc = sc2.x * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(fmaxf(sc2.y * (1.f / H) - muc * muc, 0.f) + eps);
    if (unit) {
      const float xc = dc * rsc;
      c = xc * lcw + lcb;
      const float hv = og * tanhf(c);
      out[row * H + tid] = hv;
      c_all[(row + B) * H + tid] = c;
      xhat_c[row * H + tid] = xc;
      h_s[tid] = hv;
      if (t == T - 1) { hT[static_cast<long>(b) * H + tid] = hv; cT[static_cast<long>(b) * H + tid] = c; }
    }
    if (tid == 0) rstd_c[row] = rsc;
    __syncthreads();
  }
  if (T == 0 && unit) { hT[static_cast<long>(b) * H + tid] = h_s[tid]; cT[static_cast<long>(b) * H + tid] = c; }
}

// w: W_hh [4H][H] row-major (dh_{t-1} = dhg @ W)
template <int H, int NT, int COLS, typename TW>
__global__ __launch_bounds__(NT) void lnlstm_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ dhT, const float* __restrict__ dcT,
    const float* __restrict__ gates, const float* __restrict__ c_all, const float* __restrict__ xhat_c,
    const float* __restrict__ rstd_c, const float* __restrict__ xhat_h, const float* __restrict__ rstd_h,
    const TW* __restrict__ w, const float* __restrict__ lnh_w, const float* __restrict__ lnc_w, int T, int B,
    float* __restrict__ dgates, float* __restrict__ dhg, float* __restrict__ dc_ln, float* __restrict__ dh0,
    float* __restrict__ dc0) {
  constexpr int G = 4 * H;
  // dh_{t-1} = dhg @ W  (W [G][H]): 2-D split, each thread owns KV consecutive outputs and 1/JG of the
  // reduction (partials combined through LDS); its (G / JG) x KV weight block lives in registers for the
  // whole sequence (64 values at H = 32)
  constexpr int KV = sizeof(TW) == 2 ? 8 : 4;
  constexpr int KT = H / KV;              // threads along k
  constexpr int JG = NT / KT;             // reduction groups
  constexpr int JR = G / JG;              // rows per group
  static_assert(H % KV == 0 && JG >= 1 && G % JG == 0 && KT * JG == NT, "dh tiling");
  __shared__ float dh_s[H];
  __shared__ float dg_s[G];
  __shared__ float part[JG][H];
  __shared__ float red[2 * (NT / kWave)];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const int kq = tid % KT, jg = tid / KT;
  // register-resident weight block when it is small (H = 32); the wide fallback (H = 384 unsplit) streams W
  constexpr bool kRegW = JR * KV <= 128;
  RegW<TW, kRegW ? JR * KV : 2> wreg;
  if constexpr (kRegW) {
#pragma unroll
    for (int m = 0; m < JR; ++m)
#pragma unroll
      for (int v = 0; v < KV; ++v) wreg.load(m * KV + v, w, static_cast<long>(jg * JR + m) * H + kq * KV + v);
  }
  float dc = 0.f, lcw = 0.f;
  if (unit) {
    dh_s[tid] = dhT[static_cast<long>(b) * H + tid];
    dc = dcT[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
  }
  float lw[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) lw[k] = lnh_w[tid * COLS + k];
  // the step's saved activations, fetched one step ahead (their latency hides under the previous step)
  struct StepIn { float dout, cc, go, xc, gi, gf, gg, cprev, rc, xh[COLS], rh; };
  const int ut = unit ? tid : 0;
  auto load_in = [&](int t, StepIn& v) {
    const long row = static_cast<long>(t) * B + b;
    v.dout = dout[row * H + ut];
    v.cc = c_all[(row + B) * H + ut];
    v.go = gates[row * G + 3 * H + ut];
    v.xc = xhat_c[row * H + ut];
    v.gi = gates[row * G + ut];
    v.gf = gates[row * G + H + ut];
    v.gg = gates[row * G + 2 * H + ut];
    v.cprev = c_all[row * H + ut];
    v.rc = rstd_c[row];
#pragma unroll
    for (int k = 0; k < COLS; ++k) v.xh[k] = xhat_h[row * G + tid * COLS + k];
    v.rh = rstd_h[row];
  };
  StepIn cur;
  if (T > 0) load_in(T - 1, cur);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    const long row = static_cast<long>(t) * B + b;
    StepIn nxt;
    load_in(t > 0 ? t - 1 : 0, nxt);
    // ---- cell: h = o tanh(c), c = LN_c(cpre)
    float dxh = 0.f, xc = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, cprev = 0.f;
    if (unit) {
      const float dh = cur.dout + dh_s[tid];
      const float cc = cur.cc;
      const float tc = tanhf(cc);
      const float og = sigmoidf_(cur.go);
      const float do_pre = dh * tc * og * (1.f - og);
      const float dct = dc + dh * og * (1.f - tc * tc);
      dc_ln[row * H + tid] = dct;
      dxh = dct * lcw;
      xc = cur.xc;
      ig = sigmoidf_(cur.gi);
      fg = sigmoidf_(cur.gf);
      gg = tanhf(cur.gg);
      cprev = cur.cprev;
      dg_s[3 * H + tid] = do_pre;
    }
    const float2 mm = block_sum2<NT>(dxh, dxh * xc, red);
    const float m1 = mm.x * (1.f / H), m2 = mm.y * (1.f / H);
    if (unit) {
      const float dcpre = cur.rc * (dxh - m1 - xc * m2);
      dg_s[tid] = dcpre * gg * ig * (1.f - ig);
      dg_s[H + tid] = dcpre * cprev * fg * (1.f - fg);
      dg_s[2 * H + tid] = dcpre * ig * (1.f - gg * gg);
      dc = dcpre * fg;
    }
    __syncthreads();
    // ---- LN_h backward over the 4H gate pre-activations
    float dx[COLS], xh[COLS];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float dgv = dg_s[j];
      dgates[row * G + j] = dgv;
      xh[k] = cur.xh[k];
      dx[k] = dgv * lw[k];
      s1 += dx[k];
      s2 += dx[k] * xh[k];
    }
    {
      const float2 ss = block_sum2<NT>(s1, s2, red);
      s1 = ss.x * (1.f / G);
      s2 = ss.y * (1.f / G);
    }
    const float rs = cur.rh;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float v = rs * (dx[k] - s1 - xh[k] * s2);
      dhg[row * G + j] = v;
      dg_s[j] = v;  // each thread overwrites only its own columns
    }
    __syncthreads();
    {
      float acc[KV];
#pragma unroll
      for (int v = 0; v < KV; ++v) acc[v] = 0.f;
      if constexpr (kRegW) {
#pragma unroll
        for (int m = 0; m < JR; ++m) {
          const float d = dg_s[jg * JR + m];
#pragma unroll
          for (int v = 0; v < KV; ++v) acc[v] = fmaf(d, wreg.get(m * KV + v), acc[v]);
        }
      } else {
#pragma unroll 16
        for (int m = 0; m < JR; ++m) {
          const int j = jg * JR + m;
          const float d = dg_s[j];
          float wv[KV];
          WLoad16<TW>::load(w + static_cast<long>(j) * H + kq * KV, wv);
#pragma unroll
          for (int v = 0; v < KV; ++v) acc[v] = fmaf(d, wv[v], acc[v]);
        }
      }
#pragma unroll
      for (int v = 0; v < KV; ++v) part[jg][kq * KV + v] = acc[v];
      __syncthreads();
      if (unit) {
        float sacc = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < JG; ++g2) sacc += part[g2][tid];
        dh_s[tid] = sacc;
      }
    }
    cur = nxt;
    __syncthreads();
  }
  if (unit) {
    dh0[static_cast<long>(b) * H + tid] = dh_s[tid];
    dc0[static_cast<long>(b) * H + tid] = dc;
  }
}

// ------------------------------------------------------------------------------------------------
// Split recurrence for the wide core LSTM (H = 384): the per-row kernels above stream the whole
// 1.2 MB W_hh through ONE CU per step (rocprof r1_v14: ~15 us/step, 3 ms per pass).  Here each batch row
// is served by KS = 8 workgroups; workgroup ks keeps its 1/8 slice of W_hh resident in REGISTERS for the
// whole sequence (96 fp32 weights per thread) and computes a partial product; one all-reduce per step
// gives every workgroup the full vector, after which the LN /
// gate / cell math runs redundantly (bit-identical) in all KS workgroups, so no further exchange is
// needed.  Block ids are laid out so the KS workgroups of a row share an XCD (its L2 carries the slabs).
// Forward: slice = rows of h (W_hh^T rows), partial = 4H gate pre-activations.
// Backward: slice = gate rows of W_hh, partial = dh_{t-1}.
// The exchange is the data-is-the-flag hand-off (cdna_hip_programming.md Guideline 16, R2): every
// partial value travels as an 8-byte {epoch, value} granule written by an agent-scope (write-through)
// atomic store; each consumer thread re-reads the granules IT needs with agent-scope loads until all
// carry this step's epoch (epoch = step + 1; the slab is zeroed before every launch and double-buffered
// by step parity - a producer can run at most one step ahead).  No counter, no fences, no workgroup
// barrier: the previous counter form (stores -> release -> fetch_add; poll -> acquire -> loads) cost
// several dependent L2 round trips per step.
// The poll is bounded: after kSplitPollLimit passes it sets *err and continues (garbage, but the grid drains).
constexpr int kSplitKS = 8;

// workgroups per batch row (APPLESTAR_LSTM_KS = 8 | 16): 16 halves each workgroup's W_hh slice (48 weights per thread)
// and the per-step GEMV, at twice the partials exchanged per step.  Measured slower: fp32 50.55 / 50.52 vs 50.28 / 50.20
// ms (profiles/r10za_bench_lstm_ks.txt) - the exchange, not the GEMV, sets the step; 8 stays the default
int lstm_ks() {
  static const int v = [] {
    const char* e = std::getenv("APPLESTAR_LSTM_KS");
    return (e != nullptr && std::atoi(e) == 16) ? 16 : 8;
  }();
  return v;
}

// poll budget of the cross-workgroup exchange (each pass sleeps ~64 clocks plus one L2 round trip: ~2^20
// passes is ~1 s).  Running out sets the sticky device flag (bindings: lstm_split_flag), which the trainers
// read with the step's logged scalars: the optimizer update of that step is gated to zero and the learner
// raises.  The budget is generous on purpose: side-stream kernels can delay the residency of a row's 8
// workgroups for milliseconds, and a false timeout costs a whole run.
#ifndef AS_SPLIT_POLL_LIMIT
#define AS_SPLIT_POLL_LIMIT (1u << 20)     // the 'shortpoll' build variant (csrc/build.py) restores 2^16
#endif
constexpr unsigned kSplitPollLimit = AS_SPLIT_POLL_LIMIT;

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// one wave: lanes < N poll flag[lane] (agent-scope loads) until every flag reaches `epoch`
template <int N>
__device__ __forceinline__ void wait_flags(unsigned* flags, unsigned epoch, int* err) {
  const int l = threadIdx.x & 63;
  for (unsigned spins = 0;; ++spins) {
    const unsigned f = l < N ? __hip_atomic_load((gu32*)(flags + l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : epoch;
    if (__all(f >= epoch)) return;
    if (spins > kSplitPollLimit) {
      if (l == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned epoch, float v) {
  __hip_atomic_store((gu64*)(g), (static_cast<unsigned long long>(epoch) << 32) | __float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// v[q][k] = granule (base + q * qstride + k) once all N carry `epoch` (wave-uniform loop)
template <int NQ, int NK>
__device__ __forceinline__ void get_granules(const unsigned long long* base, long qstride, unsigned epoch,
                                             float (&v)[NQ][NK], int* err) {
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const unsigned long long x = __hip_atomic_load(
            (gu64*)(const_cast<unsigned long long*>(base + q * qstride + k)), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        v[q][k] = __uint_as_float(static_cast<unsigned>(x));
        ok &= static_cast<unsigned>(x >> 32) == epoch;
      }
    if (__all(ok)) return;
    if (spins > kSplitPollLimit) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// GRAN: the partial exchange as {epoch, value} granules (as the backward): every thread writes its partials and
// polls the 8 x COLS granules it needs - one L2 round trip after the slowest producer, where the flag hand-off
// (data stores, drain, barrier, flag store, flag poll, barrier, data loads) takes three
template <int H, int NT, typename TW, bool GRAN, int KS_ = kSplitKS>
__global__ __launch_bounds__(NT) void lnlstm_fwd_split_kernel(
    const float* __restrict__ xp, const float* __restrict__ h0, const float* __restrict__ c0,
    const TW* __restrict__ wT, const float* __restrict__ lnh_w, const float* __restrict__ lnh_b,
    const float* __restrict__ lnc_w, const float* __restrict__ lnc_b, int T, int B, int Bp, float eps,
    float* __restrict__ out, float* __restrict__ c_all, float* __restrict__ xhat_h, float* __restrict__ rstd_h,
    float* __restrict__ gates_out, float* __restrict__ xhat_c, float* __restrict__ rstd_c, float* __restrict__ hT,
    float* __restrict__ cT, unsigned long long* __restrict__ slab, int* __restrict__ err,
    bf16_t* __restrict__ out_bf) {
  constexpr int KS = KS_;
  constexpr int G = 4 * H, RS = H / KS, COLS = G / NT, GS = G / KS;
  static_assert(G % NT == 0 && H % KS == 0 && NT >= H, "split tiling");
  __shared__ float h_s[H];
  __shared__ float g_s[G];
  __shared__ float red[2 * (NT / kWave)];
  const int b = blockIdx.x % Bp, ks = blockIdx.x / Bp;   // Bp % 8 == 0: a row's slices share an XCD
  if (b >= B) return;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const bool own_unit = unit && tid / RS == ks;
  RegW<TW, RS * COLS> wv;
#pragma unroll
  for (int r = 0; r < RS; ++r)
#pragma unroll
    for (int k = 0; k < COLS; ++k) wv.load(r * COLS + k, wT, static_cast<long>(ks * RS + r) * G + tid * COLS + k);
  float c = 0.f, lcw = 0.f, lcb = 0.f;
  if (unit) {
    h_s[tid] = h0[static_cast<long>(b) * H + tid];
    c = c0[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
    lcb = lnc_b[tid];
    if (own_unit) c_all[static_cast<long>(b) * H + tid] = c;
  }
  float lw[COLS], lb[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) { lw[k] = lnh_w[tid * COLS + k]; lb[k] = lnh_b[tid * COLS + k]; }
  // the input projection of step t + 1 is fetched during step t
  float xpc[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) xpc[k] = T > 0 ? xp[static_cast<long>(b) * G + tid * COLS + k] : 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float xpn[COLS];
    {
      const long nrow = static_cast<long>(t + 1 < T ? t + 1 : t) * B + b;
#pragma unroll
      for (int k = 0; k < COLS; ++k) xpn[k] = xp[nrow * G + tid * COLS + k];
    }
    float acc[COLS];
#pragma unroll
    for (int k = 0; k < COLS; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const float hv = h_s[ks * RS + r];
#pragma unroll
      for (int k = 0; k < COLS; ++k) acc[k] = fmaf(hv, wv.get(r * COLS + k), acc[k]);
    }
    const int par = t & 1;
    const unsigned epoch = static_cast<unsigned>(t + 1);
    float pv[KS][COLS];
    if constexpr (GRAN) {
      // data-is-the-flag: a producer can be at most one step ahead (its next partials need this step's h from
      // every workgroup of the row), so the parity double buffer is never overwritten while still read
      unsigned long long* gb = slab + (static_cast<long>(par) * Bp + b) * KS * G;
#pragma unroll
      for (int k = 0; k < COLS; ++k) put_granule(gb + ks * G + tid * COLS + k, epoch, acc[k]);
      // poll in two halves of the producers with a scheduling fence between them: all 16 granules in flight at
      // once (32 VGPRs) pushed the 96 register-resident weights into scratch at 3 waves per SIMD
      // (summed as they arrive, in producer order - the same order as the flag path's sum)
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < COLS; ++k) pv[0][k] = 0.f;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int q = half * (KS / 2); q < (half + 1) * (KS / 2); ++q)
#pragma unroll
            for (int k = 0; k < COLS; ++k) {
              const unsigned long long x = __hip_atomic_load((gu64*)(gb + q * G + tid * COLS + k), __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
              pv[0][k] += __uint_as_float(static_cast<unsigned>(x));
              ok &= static_cast<unsigned>(x >> 32) == epoch;
            }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (__all(ok)) break;
        if (spins > kSplitPollLimit) {
          if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    } else {
      // R1 hand-off: write-through data stores, drain, one flag per producer workgroup; one wave polls the
      // row's 8 flags, then every thread reads its 16 values with write-through (L1-bypassing) loads
      unsigned* data = reinterpret_cast<unsigned*>(slab) + (static_cast<long>(par) * Bp + b) * KS * G;
      unsigned* flags = reinterpret_cast<unsigned*>(slab) + 2L * Bp * KS * G + static_cast<long>(b) * KS;
#pragma unroll
      for (int k = 0; k < COLS; ++k)
        __hip_atomic_store((gu32*)(data + ks * G + tid * COLS + k), __float_as_uint(acc[k]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store((gu32*)(flags + ks), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid < 64) wait_flags<KS>(flags, epoch, err);
      __syncthreads();
#pragma unroll
      for (int q = 0; q < KS; ++q)
#pragma unroll
        for (int k = 0; k < COLS; ++k)
          pv[q][k] = __uint_as_float(__hip_atomic_load((gu32*)(data + q * G + tid * COLS + k), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT));
    }
    float a[COLS];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      float v = 0.f;
      if constexpr (GRAN) {
        v = pv[0][k];
      } else {
#pragma unroll
        for (int q = 0; q < KS; ++q) v += pv[q][k];
      }
      a[k] = v;
      sum += v;
    }
    float q2 = 0.f;   // LN_h statistics in one reduction (sum, sum of squares)
#pragma unroll
    for (int k = 0; k < COLS; ++k) q2 += a[k] * a[k];
    const float2 sq = block_sum2<NT>(sum, q2, red);
    const float mu = sq.x * (1.f / G);
    const float rs = rsqrtf(fmaxf(sq.y * (1.f / G) - mu * mu, 0.f) + eps);
    const long row = static_cast<long>(t) * B + b;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float xh = (a[k] - mu) * rs;
      const float gv = xpc[k] + xh * lw[k] + lb[k];
      if (j / GS == ks) {
        xhat_h[row * G + j] = xh;
        gates_out[row * G + j] = gv;
      }
      g_s[j] = gv;
    }
    if (tid == 0 && ks == 0) rstd_h[row] = rs;
    __syncthreads();
    float cpre = 0.f, og = 0.f;
    if (unit) {
      const float ig = sigmoidf_(g_s[tid]);
      const float fg = sigmoidf_(g_s[H + tid]);
      const float gg = tanhf(g_s[2 * H + tid]);
      og = sigmoidf_(g_s[3 * H + tid]);
      cpre = fg * c + ig * gg;
    }
    // LN_c statistics in one reduction (sum, sum of squares)
    const float2 sc2 = block_sum2<NT>(unit ? cpre : 0.f, unit ? cpre * cpre : 0.f, red);
    const float muc = sc2.x * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(fmaxf(sc2.y * (1.f / H) - muc * muc, 0.f) + eps);
    if (unit) {
      const float xc = dc * rsc;
      c = xc * lcw + lcb;
      const float hv = og * tanhf(c);
      h_s[tid] = hv;
      if (own_unit) {
        out[row * H + tid] = hv;
        if (out_bf) out_bf[row * H + tid] = f2bf(hv);   // the next layer's / heads' bf16 operand (inference)
        c_all[(row + B) * H + tid] = c;
        xhat_c[row * H + tid] = xc;
        if (t == T - 1) { hT[static_cast<long>(b) * H + tid] = hv; cT[static_cast<long>(b) * H + tid] = c; }
      }
    }
    if (tid == 0 && ks == 0) rstd_c[row] = rsc;
#pragma unroll
    for (int k = 0; k < COLS; ++k) xpc[k] = xpn[k];
    __syncthreads();
  }
  if (T == 0 && own_unit) { hT[static_cast<long>(b) * H + tid] = h_s[tid]; cT[static_cast<long>(b) * H + tid] = c; }
}

// w: W_hh [4H][H] row-major
template <int H, int NT, typename TW, int KS_ = kSplitKS>
__global__ __launch_bounds__(NT) void lnlstm_bwd_split_kernel(
    const float* __restrict__ dout, const float* __restrict__ dhT, const float* __restrict__ dcT,
    const float* __restrict__ gates, const float* __restrict__ c_all, const float* __restrict__ xhat_c,
    const float* __restrict__ rstd_c, const float* __restrict__ xhat_h, const float* __restrict__ rstd_h,
    const TW* __restrict__ w, const float* __restrict__ lnh_w, const float* __restrict__ lnc_w, int T, int B, int Bp,
    float* __restrict__ dgates, float* __restrict__ dhg, float* __restrict__ dc_ln, float* __restrict__ dh0,
    float* __restrict__ dc0, unsigned long long* __restrict__ slab, int* __restrict__ err) {
  constexpr int KS = KS_;
  constexpr int G = 4 * H, COLS = G / NT, JS = G / KS, RH = NT / H, JR = JS / RH, RS = H / KS;
  static_assert(NT % H == 0 && JS % RH == 0 && G % NT == 0, "split tiling");
  __shared__ float dh_s[H];
  __shared__ float dg_s[G];
  __shared__ float part[RH][H];
  __shared__ float red[2 * (NT / kWave)];
  const int b = blockIdx.x % Bp, ks = blockIdx.x / Bp;
  if (b >= B) return;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const bool own_unit = unit && tid / RS == ks;
  const int kcol = tid % H, rh = tid / H;
  const int j0 = ks * JS + rh * JR;
  RegW<TW, JR> wv;
#pragma unroll
  for (int m = 0; m < JR; ++m) wv.load(m, w, static_cast<long>(j0 + m) * H + kcol);
  float dc = 0.f, lcw = 0.f;
  if (unit) {
    dh_s[tid] = dhT[static_cast<long>(b) * H + tid];
    dc = dcT[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
  }
  float lw[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) lw[k] = lnh_w[tid * COLS + k];
  // the step's saved activations, fetched one step ahead (their latency hides under the previous
  // step's exchange instead of opening every step); unit lanes only for the H-wide ones
  struct StepIn { float dout, cc, go, xc, gi, gf, gg, cprev, rc, xh[COLS], rh; };
  const int ut = unit ? tid : 0;
  auto load_in = [&](int t, StepIn& v) {
    const long row = static_cast<long>(t) * B + b;
    v.dout = dout[row * H + ut];
    v.cc = c_all[(row + B) * H + ut];
    v.go = gates[row * G + 3 * H + ut];
    v.xc = xhat_c[row * H + ut];
    v.gi = gates[row * G + ut];
    v.gf = gates[row * G + H + ut];
    v.gg = gates[row * G + 2 * H + ut];
    v.cprev = c_all[row * H + ut];
    v.rc = rstd_c[row];
#pragma unroll
    for (int k = 0; k < COLS; ++k) v.xh[k] = xhat_h[row * G + tid * COLS + k];
    v.rh = rstd_h[row];
  };
  StepIn cur;
  if (T > 0) load_in(T - 1, cur);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    const long row = static_cast<long>(t) * B + b;
    StepIn nxt;
    load_in(t > 0 ? t - 1 : 0, nxt);
    float dxh = 0.f, xc = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, cprev = 0.f;
    if (unit) {
      const float dh = cur.dout + dh_s[tid];
      const float cc = cur.cc;
      const float tc = tanhf(cc);
      const float og = sigmoidf_(cur.go);
      const float do_pre = dh * tc * og * (1.f - og);
      const float dct = dc + dh * og * (1.f - tc * tc);
      if (own_unit) dc_ln[row * H + tid] = dct;
      dxh = dct * lcw;
      xc = cur.xc;
      ig = sigmoidf_(cur.gi);
      fg = sigmoidf_(cur.gf);
      gg = tanhf(cur.gg);
      cprev = cur.cprev;
      dg_s[3 * H + tid] = do_pre;
    }
    const float2 mm = block_sum2<NT>(dxh, dxh * xc, red);
    const float m1 = mm.x * (1.f / H), m2 = mm.y * (1.f / H);
    if (unit) {
      const float dcpre = cur.rc * (dxh - m1 - xc * m2);
      dg_s[tid] = dcpre * gg * ig * (1.f - ig);
      dg_s[H + tid] = dcpre * cprev * fg * (1.f - fg);
      dg_s[2 * H + tid] = dcpre * ig * (1.f - gg * gg);
      dc = dcpre * fg;
    }
    __syncthreads();
    float dx[COLS], xh[COLS];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float dgv = dg_s[j];
      if (j / JS == ks) dgates[row * G + j] = dgv;
      xh[k] = cur.xh[k];
      dx[k] = dgv * lw[k];
      s1 += dx[k];
      s2 += dx[k] * xh[k];
    }
    {
      const float2 ss = block_sum2<NT>(s1, s2, red);
      s1 = ss.x * (1.f / G);
      s2 = ss.y * (1.f / G);
    }
    const float rs = cur.rh;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float v = rs * (dx[k] - s1 - xh[k] * s2);
      if (j / JS == ks) dhg[row * G + j] = v;
      dg_s[j] = v;
    }
    __syncthreads();
    // partial dh_{t-1}[k] over this workgroup's JS gate rows (two row halves per column, combined in LDS)
    float acc = 0.f;
#pragma unroll
    for (int m = 0; m < JR; ++m) acc = fmaf(dg_s[j0 + m], wv.get(m), acc);
    part[rh][kcol] = acc;
    __syncthreads();
    const int par = t & 1;
    const unsigned epoch = static_cast<unsigned>(T - t);
    unsigned long long* row_slab = slab + (static_cast<long>(par) * Bp + b) * KS * H;
    if (unit) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < RH; ++q) v += part[q][tid];
      put_granule(row_slab + ks * H + tid, epoch, v);
    }
    if (tid < 64 * ((H + 63) / 64)) {   // whole waves: the poll loop is wave-uniform
      float pv[KS][1];
      get_granules<KS, 1>(row_slab + (tid < H ? tid : 0), H, epoch, pv, err);
      if (unit) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < KS; ++q) v += pv[q][0];
        dh_s[tid] = v;
      }
    }
    cur = nxt;
    __syncthreads();
  }
  if (own_unit) {
    dh0[static_cast<long>(b) * H + tid] = dh_s[tid];
    dc0[static_cast<long>(b) * H + tid] = dc;
  }
}

template <int H, int NT, int COLS>
void fwd_launch(const float* xp, const float* h0, const float* c0, const void* wT, int w_dt, const float* lnh_w,
                const float* lnh_b, const float* lnc_w, const float* lnc_b, int T, int B, float eps, float* out,
                float* c_all, float* xhat_h, float* rstd_h, float* gates, float* xhat_c, float* rstd_c, float* hT,
                float* cT, hipStream_t s) {
  if (w_dt == DT_BF16)
    hipLaunchKernelGGL((lnlstm_fwd_kernel<H, NT, COLS, bf16_t>), dim3(B), dim3(NT), 0, s, xp, h0, c0,
                       static_cast<const bf16_t*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, eps, out, c_all, xhat_h,
                       rstd_h, gates, xhat_c, rstd_c, hT, cT);
  else
    hipLaunchKernelGGL((lnlstm_fwd_kernel<H, NT, COLS, float>), dim3(B), dim3(NT), 0, s, xp, h0, c0,
                       static_cast<const float*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, eps, out, c_all, xhat_h,
                       rstd_h, gates, xhat_c, rstd_c, hT, cT);
}

template <int H, int NT, int COLS>
void bwd_launch(const float* dout, const float* dhT, const float* dcT, const float* gates, const float* c_all,
                const float* xhat_c, const float* rstd_c, const float* xhat_h, const float* rstd_h, const void* w,
                int w_dt, const float* lnh_w, const float* lnc_w, int T, int B, float* dgates, float* dhg,
                float* dc_ln, float* dh0, float* dc0, hipStream_t s) {
  if (w_dt == DT_BF16)
    hipLaunchKernelGGL((lnlstm_bwd_kernel<H, NT, COLS, bf16_t>), dim3(B), dim3(NT), 0, s, dout, dhT, dcT, gates,
                       c_all, xhat_c, rstd_c, xhat_h, rstd_h, static_cast<const bf16_t*>(w), lnh_w, lnc_w, T, B,
                       dgates, dhg, dc_ln, dh0, dc0);
  else
    hipLaunchKernelGGL((lnlstm_bwd_kernel<H, NT, COLS, float>), dim3(B), dim3(NT), 0, s, dout, dhT, dcT, gates,
                       c_all, xhat_c, rstd_c, xhat_h, rstd_h, static_cast<const float*>(w), lnh_w, lnc_w, T, B,
                       dgates, dhg, dc_ln, dh0, dc0);
}

}  // namespace

bool lnlstm_supported(int H) { return H == 384 || H == 32; }

void lnlstm_fwd(const float* xp, const float* h0, const float* c0, const void* wT, int w_dt, const float* lnh_w,
                const float* lnh_b, const float* lnc_w, const float* lnc_b, int T, int B, int H, float eps, float* out,
                float* c_all, float* xhat_h, float* rstd_h, float* gates, float* xhat_c, float* rstd_c, float* hT,
                float* cT, hipStream_t s, const LstmSplit* split, unsigned short* out_bf16) {
  if (H == 384 && split != nullptr) {
    const int Bp = (B + 7) / 8 * 8;
    const int ks = lstm_ks();
    const dim3 grid(Bp * ks);
    static const bool gran = [] {
      const char* e = std::getenv("APPLESTAR_LSTM_FWD_GRANULE");   // A/B switch, off by default
      return e != nullptr && e[0] == '1';
    }();
#define AS_FWD_SPLIT(TWv, GR, KSv)                                                                               \
    hipLaunchKernelGGL((lnlstm_fwd_split_kernel<384, 768, TWv, GR, KSv>), grid, dim3(768), 0, s, xp, h0, c0,     \
                       static_cast<const TWv*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, Bp, eps, out, c_all, xhat_h,  \
                       rstd_h, gates, xhat_c, rstd_c, hT, cT, split->slab, split->err, out_bf16)
    if (ks == 16) {
      if (w_dt == DT_BF16) AS_FWD_SPLIT(bf16_t, false, 16); else AS_FWD_SPLIT(float, false, 16);
    } else if (w_dt == DT_BF16) {
      if (gran) AS_FWD_SPLIT(bf16_t, true, 8); else AS_FWD_SPLIT(bf16_t, false, 8);
    } else {
      if (gran) AS_FWD_SPLIT(float, true, 8); else AS_FWD_SPLIT(float, false, 8);
    }
#undef AS_FWD_SPLIT
  } else if (H == 384) {
    if (w_dt == DT_BF16)
      hipLaunchKernelGGL((lnlstm_fwd_wide_kernel<384, 768, bf16_t>), dim3(B), dim3(768), 0, s, xp, h0, c0,
                         static_cast<const bf16_t*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, eps, out, c_all, xhat_h,
                         rstd_h, gates, xhat_c, rstd_c, hT, cT);
    else
      hipLaunchKernelGGL((lnlstm_fwd_wide_kernel<384, 768, float>), dim3(B), dim3(768), 0, s, xp, h0, c0,
                         static_cast<const float*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, eps, out, c_all, xhat_h,
                         rstd_h, gates, xhat_c, rstd_c, hT, cT);
  }
  else if (H == 32)
    fwd_launch<32, 64, 2>(xp, h0, c0, wT, w_dt, lnh_w, lnh_b, lnc_w, lnc_b, T, B, eps, out, c_all, xhat_h, rstd_h,
                          gates, xhat_c, rstd_c, hT, cT, s);
}

void lnlstm_bwd(const float* dout, const float* dhT, const float* dcT, const float* gates, const float* c_all,
                const float* xhat_c, const float* rstd_c, const float* xhat_h, const float* rstd_h, const void* w,
                int w_dt, const float* lnh_w, const float* lnc_w, int T, int B, int H, float* dgates, float* dhg,
                float* dc_ln, float* dh0, float* dc0, hipStream_t s, const LstmSplit* split) {
  if (H == 384 && split != nullptr) {
    const int Bp = (B + 7) / 8 * 8;
    const int ks = lstm_ks();
    const dim3 grid(Bp * ks);
#define AS_BWD_SPLIT(TWv, KSv)                                                                                   \
    hipLaunchKernelGGL((lnlstm_bwd_split_kernel<384, 768, TWv, KSv>), grid, dim3(768), 0, s, dout, dhT, dcT, gates,  \
                       c_all, xhat_c, rstd_c, xhat_h, rstd_h, static_cast<const TWv*>(w), lnh_w, lnc_w, T, B, Bp,    \
                       dgates, dhg, dc_ln, dh0, dc0, split->slab, split->err)
    if (ks == 16) {
      if (w_dt == DT_BF16) AS_BWD_SPLIT(bf16_t, 16); else AS_BWD_SPLIT(float, 16);
    } else {
      if (w_dt == DT_BF16) AS_BWD_SPLIT(bf16_t, 8); else AS_BWD_SPLIT(float, 8);
    }
#undef AS_BWD_SPLIT
  } else if (H == 384)
    bwd_launch<384, 768, 2>(dout, dhT, dcT, gates, c_all, xhat_c, rstd_c, xhat_h, rstd_h, w, w_dt, lnh_w, lnc_w, T, B,
                            dgates, dhg, dc_ln, dh0, dc0, s);
  else if (H == 32)
    bwd_launch<32, 64, 2>(dout, dhT, dcT, gates, c_all, xhat_c, rstd_c, xhat_h, rstd_h, w, w_dt, lnh_w, lnc_w, T, B,
                          dgates, dhg, dc_ln, dh0, dc0, s);
}

}  // namespace as
