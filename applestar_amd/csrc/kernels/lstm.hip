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
  __shared__ float red[NT / kWave];
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
    const float mu = block_sum<NT>(s, red) * (1.f / G);
    float q2 = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) { const float d = a[k] - mu; q2 += d * d; }
    const float rs = rsqrtf(block_sum<NT>(q2, red) * (1.f / G) + eps);
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
    const float muc = block_sum<NT>(unit ? cpre : 0.f, red) * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(block_sum<NT>(dc * dc, red) * (1.f / H) + eps);
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
  __shared__ float red[NT / kWave];
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
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float acc[COLS];
#pragma unroll
    for (int k = 0; k < COLS; ++k) acc[k] = 0.f;
    const TW* wp = wT + tid * COLS;
    // deep unroll: the W^T stream is L2-latency bound at B=6, keep many 8-16 B loads in flight
#pragma unroll 32
    for (int i = 0; i < H; ++i) {
      float wv[COLS];
      WLoad<TW, COLS>::load(wp + static_cast<long>(i) * G, wv);
      const float hv = h_s[i];
#pragma unroll
      for (int k = 0; k < COLS; ++k) acc[k] = fmaf(hv, wv[k], acc[k]);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) s += acc[k];
    const float mu = block_sum<NT>(s, red) * (1.f / G);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) { const float d = acc[k] - mu; q += d * d; }
    const float rs = rsqrtf(block_sum<NT>(q, red) * (1.f / G) + eps);
    const long row = static_cast<long>(t) * B + b;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float xh = (acc[k] - mu) * rs;
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
    const float muc = block_sum<NT>(unit ? cpre : 0.f, red) * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(block_sum<NT>(dc * dc, red) * (1.f / H) + eps);
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
  __shared__ float dh_s[H];
  __shared__ float dg_s[G];
  __shared__ float red[NT / kWave];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  float dc = 0.f, lcw = 0.f;
  if (unit) {
    dh_s[tid] = dhT[static_cast<long>(b) * H + tid];
    dc = dcT[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
  }
  float lw[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) lw[k] = lnh_w[tid * COLS + k];
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    const long row = static_cast<long>(t) * B + b;
    // ---- cell: h = o tanh(c), c = LN_c(cpre)
    float dxh = 0.f, xc = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, cprev = 0.f;
    if (unit) {
      const float dh = dout[row * H + tid] + dh_s[tid];
      const float cc = c_all[(row + B) * H + tid];
      const float tc = tanhf(cc);
      const float og = sigmoidf_(gates[row * G + 3 * H + tid]);
      const float do_pre = dh * tc * og * (1.f - og);
      const float dct = dc + dh * og * (1.f - tc * tc);
      dc_ln[row * H + tid] = dct;
      dxh = dct * lcw;
      xc = xhat_c[row * H + tid];
      ig = sigmoidf_(gates[row * G + tid]);
      fg = sigmoidf_(gates[row * G + H + tid]);
      gg = tanhf(gates[row * G + 2 * H + tid]);
      cprev = c_all[row * H + tid];
      dg_s[3 * H + tid] = do_pre;
    }
    const float m1 = block_sum<NT>(dxh, red) * (1.f / H);
    const float m2 = block_sum<NT>(dxh * xc, red) * (1.f / H);
    if (unit) {
      const float dcpre = rstd_c[row] * (dxh - m1 - xc * m2);
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
      xh[k] = xhat_h[row * G + j];
      dx[k] = dgv * lw[k];
      s1 += dx[k];
      s2 += dx[k] * xh[k];
    }
    s1 = block_sum<NT>(s1, red) * (1.f / G);
    s2 = block_sum<NT>(s2, red) * (1.f / G);
    const float rs = rstd_h[row];
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float v = rs * (dx[k] - s1 - xh[k] * s2);
      dhg[row * G + j] = v;
      dg_s[j] = v;  // each thread overwrites only its own columns
    }
    __syncthreads();
    // ---- dh_{t-1} = dhg @ W  (W [G][H]): 2-D split, each thread owns KV consecutive outputs (one
    // 16-byte load per j) and 1/JG of the reduction; partials combined through LDS
    {
      constexpr int KV = sizeof(TW) == 2 ? 8 : 4;
      constexpr int KT = H / KV;              // threads along k
      constexpr int JG = NT / KT;             // reduction groups
      static_assert(H % KV == 0 && JG >= 1 && G % JG == 0, "dh tiling");
      const int kq = tid % KT, jg = tid / KT;
      float acc[KV];
#pragma unroll
      for (int v = 0; v < KV; ++v) acc[v] = 0.f;
      if (jg < JG) {
        const int j0 = jg * (G / JG), j1 = j0 + G / JG;
#pragma unroll 16
        for (int j = j0; j < j1; ++j) {
          const float d = dg_s[j];
          float wv[KV];
          WLoad16<TW>::load(w + static_cast<long>(j) * H + kq * KV, wv);
#pragma unroll
          for (int v = 0; v < KV; ++v) acc[v] = fmaf(d, wv[v], acc[v]);
        }
      }
      __shared__ float part[JG][H];
      if (jg < JG) {
#pragma unroll
        for (int v = 0; v < KV; ++v) part[jg][kq * KV + v] = acc[v];
      }
      __syncthreads();
      if (unit) {
        float sacc = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < JG; ++g2) sacc += part[g2][tid];
        dh_s[tid] = sacc;
      }
    }
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
// (plain fp32 stores -> agent release -> counter add; relaxed poll -> agent acquire -> plain loads: the
// cdna_hip_programming.md split-K hand-off) gives every workgroup the full vector, after which the LN /
// gate / cell math runs redundantly (bit-identical) in all KS workgroups, so no further exchange is
// needed.  Block ids are laid out so the KS workgroups of a row share an XCD (its L2 carries the slabs).
// Forward: slice = rows of h (W_hh^T rows), partial = 4H gate pre-activations.
// Backward: slice = gate rows of W_hh, partial = dh_{t-1}.
// The poll is bounded: after ~0.5 s it sets *err and continues (garbage, but the grid drains).
constexpr int kSplitKS = 8;

__device__ __forceinline__ void split_exchange(unsigned* cnt, unsigned target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <int H, int NT, typename TW>
__global__ __launch_bounds__(NT) void lnlstm_fwd_split_kernel(
    const float* __restrict__ xp, const float* __restrict__ h0, const float* __restrict__ c0,
    const TW* __restrict__ wT, const float* __restrict__ lnh_w, const float* __restrict__ lnh_b,
    const float* __restrict__ lnc_w, const float* __restrict__ lnc_b, int T, int B, int Bp, float eps,
    float* __restrict__ out, float* __restrict__ c_all, float* __restrict__ xhat_h, float* __restrict__ rstd_h,
    float* __restrict__ gates_out, float* __restrict__ xhat_c, float* __restrict__ rstd_c, float* __restrict__ hT,
    float* __restrict__ cT, float* __restrict__ slab, unsigned* __restrict__ cnt, int* __restrict__ err) {
  constexpr int KS = kSplitKS;
  constexpr int G = 4 * H, RS = H / KS, COLS = G / NT, GS = G / KS;
  static_assert(G % NT == 0 && H % KS == 0 && NT >= H, "split tiling");
  __shared__ float h_s[H];
  __shared__ float g_s[G];
  __shared__ float red[NT / kWave];
  const int b = blockIdx.x % Bp, ks = blockIdx.x / Bp;   // Bp % 8 == 0: a row's slices share an XCD
  if (b >= B) return;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const bool own_unit = unit && tid / RS == ks;
  float wv[RS][COLS];
#pragma unroll
  for (int r = 0; r < RS; ++r)
#pragma unroll
    for (int k = 0; k < COLS; ++k) wv[r][k] = Cvt<TW>::load(wT, static_cast<long>(ks * RS + r) * G + tid * COLS + k);
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
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    float acc[COLS];
#pragma unroll
    for (int k = 0; k < COLS; ++k) acc[k] = 0.f;
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const float hv = h_s[ks * RS + r];
#pragma unroll
      for (int k = 0; k < COLS; ++k) acc[k] = fmaf(hv, wv[r][k], acc[k]);
    }
    const int par = t & 1;
    float* my = slab + ((static_cast<long>(par) * Bp + b) * KS + ks) * G;
#pragma unroll
    for (int k = 0; k < COLS; ++k) my[tid * COLS + k] = acc[k];
    split_exchange(cnt + b, static_cast<unsigned>(KS * (t + 1)), err);
    const float* all = slab + (static_cast<long>(par) * Bp + b) * KS * G;
    float a[COLS];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < KS; ++q) v += all[q * G + tid * COLS + k];
      a[k] = v;
      sum += v;
    }
    const float mu = block_sum<NT>(sum, red) * (1.f / G);
    float q2 = 0.f;
#pragma unroll
    for (int k = 0; k < COLS; ++k) { const float d = a[k] - mu; q2 += d * d; }
    const float rs = rsqrtf(block_sum<NT>(q2, red) * (1.f / G) + eps);
    const long row = static_cast<long>(t) * B + b;
#pragma unroll
    for (int k = 0; k < COLS; ++k) {
      const int j = tid * COLS + k;
      const float xh = (a[k] - mu) * rs;
      const float gv = xp[row * G + j] + xh * lw[k] + lb[k];
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
    const float muc = block_sum<NT>(unit ? cpre : 0.f, red) * (1.f / H);
    const float dc = unit ? cpre - muc : 0.f;
    const float rsc = rsqrtf(block_sum<NT>(dc * dc, red) * (1.f / H) + eps);
    if (unit) {
      const float xc = dc * rsc;
      c = xc * lcw + lcb;
      const float hv = og * tanhf(c);
      h_s[tid] = hv;
      if (own_unit) {
        out[row * H + tid] = hv;
        c_all[(row + B) * H + tid] = c;
        xhat_c[row * H + tid] = xc;
        if (t == T - 1) { hT[static_cast<long>(b) * H + tid] = hv; cT[static_cast<long>(b) * H + tid] = c; }
      }
    }
    if (tid == 0 && ks == 0) rstd_c[row] = rsc;
    __syncthreads();
  }
  if (T == 0 && own_unit) { hT[static_cast<long>(b) * H + tid] = h_s[tid]; cT[static_cast<long>(b) * H + tid] = c; }
}

// w: W_hh [4H][H] row-major
template <int H, int NT, typename TW>
__global__ __launch_bounds__(NT) void lnlstm_bwd_split_kernel(
    const float* __restrict__ dout, const float* __restrict__ dhT, const float* __restrict__ dcT,
    const float* __restrict__ gates, const float* __restrict__ c_all, const float* __restrict__ xhat_c,
    const float* __restrict__ rstd_c, const float* __restrict__ xhat_h, const float* __restrict__ rstd_h,
    const TW* __restrict__ w, const float* __restrict__ lnh_w, const float* __restrict__ lnc_w, int T, int B, int Bp,
    float* __restrict__ dgates, float* __restrict__ dhg, float* __restrict__ dc_ln, float* __restrict__ dh0,
    float* __restrict__ dc0, float* __restrict__ slab, unsigned* __restrict__ cnt, int* __restrict__ err) {
  constexpr int KS = kSplitKS;
  constexpr int G = 4 * H, COLS = G / NT, JS = G / KS, RH = NT / H, JR = JS / RH, RS = H / KS;
  static_assert(NT % H == 0 && JS % RH == 0 && G % NT == 0, "split tiling");
  __shared__ float dh_s[H];
  __shared__ float dg_s[G];
  __shared__ float part[RH][H];
  __shared__ float red[NT / kWave];
  const int b = blockIdx.x % Bp, ks = blockIdx.x / Bp;
  if (b >= B) return;
  const int tid = threadIdx.x;
  const bool unit = tid < H;
  const bool own_unit = unit && tid / RS == ks;
  const int kcol = tid % H, rh = tid / H;
  const int j0 = ks * JS + rh * JR;
  float wv[JR];
#pragma unroll
  for (int m = 0; m < JR; ++m) wv[m] = Cvt<TW>::load(w, static_cast<long>(j0 + m) * H + kcol);
  float dc = 0.f, lcw = 0.f;
  if (unit) {
    dh_s[tid] = dhT[static_cast<long>(b) * H + tid];
    dc = dcT[static_cast<long>(b) * H + tid];
    lcw = lnc_w[tid];
  }
  float lw[COLS];
#pragma unroll
  for (int k = 0; k < COLS; ++k) lw[k] = lnh_w[tid * COLS + k];
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    const long row = static_cast<long>(t) * B + b;
    float dxh = 0.f, xc = 0.f, ig = 0.f, fg = 0.f, gg = 0.f, cprev = 0.f;
    if (unit) {
      const float dh = dout[row * H + tid] + dh_s[tid];
      const float cc = c_all[(row + B) * H + tid];
      const float tc = tanhf(cc);
      const float og = sigmoidf_(gates[row * G + 3 * H + tid]);
      const float do_pre = dh * tc * og * (1.f - og);
      const float dct = dc + dh * og * (1.f - tc * tc);
      if (own_unit) dc_ln[row * H + tid] = dct;
      dxh = dct * lcw;
      xc = xhat_c[row * H + tid];
      ig = sigmoidf_(gates[row * G + tid]);
      fg = sigmoidf_(gates[row * G + H + tid]);
      gg = tanhf(gates[row * G + 2 * H + tid]);
      cprev = c_all[row * H + tid];
      dg_s[3 * H + tid] = do_pre;
    }
    const float m1 = block_sum<NT>(dxh, red) * (1.f / H);
    const float m2 = block_sum<NT>(dxh * xc, red) * (1.f / H);
    if (unit) {
      const float dcpre = rstd_c[row] * (dxh - m1 - xc * m2);
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
      xh[k] = xhat_h[row * G + j];
      dx[k] = dgv * lw[k];
      s1 += dx[k];
      s2 += dx[k] * xh[k];
    }
    s1 = block_sum<NT>(s1, red) * (1.f / G);
    s2 = block_sum<NT>(s2, red) * (1.f / G);
    const float rs = rstd_h[row];
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
    for (int m = 0; m < JR; ++m) acc = fmaf(dg_s[j0 + m], wv[m], acc);
    part[rh][kcol] = acc;
    __syncthreads();
    const int par = t & 1;
    if (unit) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < RH; ++q) v += part[q][tid];
      slab[((static_cast<long>(par) * Bp + b) * KS + ks) * H + tid] = v;
    }
    split_exchange(cnt + b, static_cast<unsigned>(KS * (T - t)), err);
    if (unit) {
      const float* all = slab + (static_cast<long>(par) * Bp + b) * KS * H;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < KS; ++q) v += all[q * H + tid];
      dh_s[tid] = v;
    }
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
                float* cT, hipStream_t s, const LstmSplit* split) {
  if (H == 384 && split != nullptr) {
    const int Bp = (B + 7) / 8 * 8;
    const dim3 grid(Bp * kSplitKS);
    if (w_dt == DT_BF16)
      hipLaunchKernelGGL((lnlstm_fwd_split_kernel<384, 768, bf16_t>), grid, dim3(768), 0, s, xp, h0, c0,
                         static_cast<const bf16_t*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, Bp, eps, out, c_all,
                         xhat_h, rstd_h, gates, xhat_c, rstd_c, hT, cT, split->slab, split->cnt, split->err);
    else
      hipLaunchKernelGGL((lnlstm_fwd_split_kernel<384, 768, float>), grid, dim3(768), 0, s, xp, h0, c0,
                         static_cast<const float*>(wT), lnh_w, lnh_b, lnc_w, lnc_b, T, B, Bp, eps, out, c_all,
                         xhat_h, rstd_h, gates, xhat_c, rstd_c, hT, cT, split->slab, split->cnt, split->err);
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
    const dim3 grid(Bp * kSplitKS);
    if (w_dt == DT_BF16)
      hipLaunchKernelGGL((lnlstm_bwd_split_kernel<384, 768, bf16_t>), grid, dim3(768), 0, s, dout, dhT, dcT, gates,
                         c_all, xhat_c, rstd_c, xhat_h, rstd_h, static_cast<const bf16_t*>(w), lnh_w, lnc_w, T, B, Bp,
                         dgates, dhg, dc_ln, dh0, dc0, split->slab, split->cnt, split->err);
    else
      hipLaunchKernelGGL((lnlstm_bwd_split_kernel<384, 768, float>), grid, dim3(768), 0, s, dout, dhT, dcT, gates,
                         c_all, xhat_c, rstd_c, xhat_h, rstd_h, static_cast<const float*>(w), lnh_w, lnc_w, T, B, Bp,
                         dgates, dhg, dc_ln, dh0, dc0, split->slab, split->cnt, split->err);
  } else if (H == 384)
    bwd_launch<384, 768, 2>(dout, dhT, dcT, gates, c_all, xhat_c, rstd_c, xhat_h, rstd_h, w, w_dt, lnh_w, lnc_w, T, B,
                            dgates, dhg, dc_ln, dh0, dc0, s);
  else if (H == 32)
    bwd_launch<32, 64, 2>(dout, dhT, dcT, gates, c_all, xhat_c, rstd_c, xhat_h, rstd_h, w, w_dt, lnh_w, lnc_w, T, B,
                          dgates, dhg, dc_ln, dh0, dc0, s);
}

}  // namespace as
