// Fused per-row categorical statistics of the RL / SL losses, forward and backward.
//
// For every row r of logits l [R, C] (one policy-head distribution per agent step) with teacher logits
// t [R, C] (optional) and the behaviour action a[r]:
//
//   logp_a = l[a] - lse(l)                       (V-trace / UPGO / SL cross-entropy term)
//   H      = -sum_i p_i lp_i                     (entropy, p = softmax(l), lp = log p)
//   KL     = sum_i tp_i (tlp_i - lp_i)           (teacher KL, tp = softmax(t))
//
// The reference computes log_softmax of both logit tensors, exp, gather, products and row sums as
// separate ops for each of the six heads (rl_loss.py:63-90, as_rl_utils.py:52-127): ~15 forward and
// ~15 backward kernels per head, each streaming the [R, C] tensors (C up to 24,320 for the location
// head).  Here one kernel reads l and t twice (max pass, sum pass; the second from L2) and writes three
// floats per row; the backward is one pass that writes
//
//   dl_i = g_a ([i == a] - p_i) - g_H p_i (lp_i + H) + g_KL (p_i - tp_i)
//
// All sums are taken on max-shifted values (x - m), so rows that are entirely masked with -1e9 (padded
// selected-units steps) keep exact lp = -log C like log_softmax instead of cancelling at 1e9.
// Rows of C <= 4096 use one wave each (4 rows per 256-thread workgroup); longer rows a whole workgroup.
#include <math.h>

#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

template <int TPR>
__device__ __forceinline__ float group_max(float v, float* red) {
  v = wave_max(v);
  if constexpr (TPR == 64) {
    return v;
  } else {
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  }
}

template <int TPR>
__device__ __forceinline__ float group_sum(float v, float* red) {
  v = wave_sum(v);
  if constexpr (TPR == 64) {
    return v;
  } else {
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// stats [R, 6]: m, log s, H, mt, log st, (unused)
template <typename LT, typename TT, int TPR>
__global__ __launch_bounds__(256) void head_stats_fwd_kernel(const LT* __restrict__ l, const TT* __restrict__ t,
                                                             const long* __restrict__ act, float* __restrict__ out,
                                                             float* __restrict__ stats, long R, int C) {
  constexpr int RPB = 256 / TPR;
  __shared__ float red[4];
  const int sub = threadIdx.x / TPR, lt = threadIdx.x % TPR;
  const long row = static_cast<long>(blockIdx.x) * RPB + sub;
  const bool ok = row < R;
  const long base = (ok ? row : 0) * static_cast<long>(C);
  const bool has_t = t != nullptr;
  float m = -INFINITY, mt = -INFINITY;
  if (ok) {
    for (int i = lt; i < C; i += TPR) {
      m = fmaxf(m, Cvt<LT>::load(l, base + i));
      if (has_t) mt = fmaxf(mt, Cvt<TT>::load(t, base + i));
    }
  }
  m = group_max<TPR>(m, red);
  mt = group_max<TPR>(mt, red);
  float s = 0.f, sl = 0.f, st = 0.f, stt = 0.f, stl = 0.f;
  if (ok) {
    for (int i = lt; i < C; i += TPR) {
      const float x = Cvt<LT>::load(l, base + i) - m;
      const float e = __expf(x);
      s += e;
      sl += e * x;
      if (has_t) {
        const float y = Cvt<TT>::load(t, base + i) - mt;
        const float et = __expf(y);
        st += et;
        stt += et * y;
        stl += et * x;
      }
    }
  }
  s = group_sum<TPR>(s, red);
  sl = group_sum<TPR>(sl, red);
  if (has_t) {
    st = group_sum<TPR>(st, red);
    stt = group_sum<TPR>(stt, red);
    stl = group_sum<TPR>(stl, red);
  }
  if (ok && lt == 0) {
    const float logs = logf(s);
    const float H = logs - sl / s;
    long a = act[row];
    a = a < 0 ? 0 : (a >= C ? C - 1 : a);
    out[row] = (Cvt<LT>::load(l, base + a) - m) - logs;
    out[R + row] = H;
    float* st_row = stats + row * 6;
    st_row[0] = m;
    st_row[1] = logs;
    st_row[2] = H;
    if (has_t) {
      const float logst = logf(st);
      out[2 * R + row] = (stt / st - logst) - (stl / st - logs);
      st_row[3] = mt;
      st_row[4] = logst;
    } else {
      out[2 * R + row] = 0.f;
      st_row[3] = 0.f;
      st_row[4] = 0.f;
    }
    st_row[5] = 0.f;
  }
}

template <typename LT, typename TT, int TPR>
__global__ __launch_bounds__(256) void head_stats_bwd_kernel(const LT* __restrict__ l, const TT* __restrict__ t,
                                                             const long* __restrict__ act,
                                                             const float* __restrict__ stats,
                                                             const float* __restrict__ g, LT* __restrict__ dl, long R,
                                                             int C) {
  constexpr int RPB = 256 / TPR;
  const int sub = threadIdx.x / TPR, lt = threadIdx.x % TPR;
  const long row = static_cast<long>(blockIdx.x) * RPB + sub;
  if (row >= R) return;
  const long base = row * static_cast<long>(C);
  const float* st_row = stats + row * 6;
  const float m = st_row[0], logs = st_row[1], H = st_row[2], mt = st_row[3], logst = st_row[4];
  const float ga = g[row], gh = g[R + row], gk = g[2 * R + row];
  long a = act[row];
  a = a < 0 ? 0 : (a >= C ? C - 1 : a);
  const bool has_t = t != nullptr;
  for (int i = lt; i < C; i += TPR) {
    const float lp = (Cvt<LT>::load(l, base + i) - m) - logs;
    const float p = __expf(lp);
    float d = ga * ((i == a ? 1.f : 0.f) - p) - gh * p * (lp + H);
    if (has_t) {
      const float tp = __expf((Cvt<TT>::load(t, base + i) - mt) - logst);
      d += gk * (p - tp);
    }
    Cvt<LT>::store(dl, base + i, d);
  }
}

template <typename LT, typename TT>
void fwd_dispatch(const void* l, const void* t, const long* act, float* out, float* stats, long R, int C,
                  hipStream_t s) {
  if (R == 0) return;
  if (C <= 4096) {
    const long nb = (R + 3) / 4;
    hipLaunchKernelGGL((head_stats_fwd_kernel<LT, TT, 64>), dim3(static_cast<unsigned>(nb)), dim3(256), 0, s,
                       static_cast<const LT*>(l), static_cast<const TT*>(t), act, out, stats, R, C);
  } else {
    hipLaunchKernelGGL((head_stats_fwd_kernel<LT, TT, 256>), dim3(static_cast<unsigned>(R)), dim3(256), 0, s,
                       static_cast<const LT*>(l), static_cast<const TT*>(t), act, out, stats, R, C);
  }
}

template <typename LT, typename TT>
void bwd_dispatch(const void* l, const void* t, const long* act, const float* stats, const float* g, void* dl, long R,
                  int C, hipStream_t s) {
  if (R == 0) return;
  if (C <= 4096) {
    const long nb = (R + 3) / 4;
    hipLaunchKernelGGL((head_stats_bwd_kernel<LT, TT, 64>), dim3(static_cast<unsigned>(nb)), dim3(256), 0, s,
                       static_cast<const LT*>(l), static_cast<const TT*>(t), act, stats, g, static_cast<LT*>(dl), R,
                       C);
  } else {
    hipLaunchKernelGGL((head_stats_bwd_kernel<LT, TT, 256>), dim3(static_cast<unsigned>(R)), dim3(256), 0, s,
                       static_cast<const LT*>(l), static_cast<const TT*>(t), act, stats, g, static_cast<LT*>(dl), R,
                       C);
  }
}

}  // namespace

void head_stats_fwd(const void* l, int l_dt, const void* t, int t_dt, const long* act, float* out, float* stats, long R,
                    int C, hipStream_t s) {
  const bool lb = l_dt == DT_BF16, tb = t_dt == DT_BF16;
  if (lb && tb) fwd_dispatch<bf16_t, bf16_t>(l, t, act, out, stats, R, C, s);
  else if (lb) fwd_dispatch<bf16_t, float>(l, t, act, out, stats, R, C, s);
  else if (tb) fwd_dispatch<float, bf16_t>(l, t, act, out, stats, R, C, s);
  else fwd_dispatch<float, float>(l, t, act, out, stats, R, C, s);
}

void head_stats_bwd(const void* l, int l_dt, const void* t, int t_dt, const long* act, const float* stats,
                    const float* g, void* dl, long R, int C, hipStream_t s) {
  const bool lb = l_dt == DT_BF16, tb = t_dt == DT_BF16;
  if (lb && tb) bwd_dispatch<bf16_t, bf16_t>(l, t, act, stats, g, dl, R, C, s);
  else if (lb) bwd_dispatch<bf16_t, float>(l, t, act, stats, g, dl, R, C, s);
  else if (tb) bwd_dispatch<float, bf16_t>(l, t, act, stats, g, dl, R, C, s);
  else bwd_dispatch<float, float>(l, t, act, stats, g, dl, R, C, s);
}

}  // namespace as
