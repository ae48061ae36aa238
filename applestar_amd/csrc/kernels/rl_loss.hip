// RL learner loss tail in ONE workgroup: everything of rl/loss.py after the per-head logit statistics
// (ops.head_stats) — V-trace policy gradient per baseline field, UPGO, TD(lambda) critic, normalised
// entropy and teacher KL (+ the extra action-type KL) — for [T, B] slices, together with the closed-form
// gradients of the total loss with respect to the stacked per-head log-probabilities, entropies, KLs and the
// baseline values (every return / advantage is a detached target, so the gradients are elementwise).
// The torch form issued ~150 tiny kernels forward and ~100 autograd nodes backward for 384 elements.
//
// Inputs (fp32, contiguous): alp / blp / hm / ent / kl [6, T, B] (per-head learner log-prob, behaviour
// log-prob, head mask, normalised entropy, KL — the selected-units head already reduced over its 64 steps);
// v [F, T+1, B] (bootstrap already zeroed for finished episodes), r / wm [F, T, B] (rewards, field weight
// masks); atflag [T, B] (action-type KL gate); sc: per-field / per-head scalars (layout in the kernel; built
// by ReinforcementLoss._scalars).
// Outputs: dalp / dent / dkl [6, T, B], dv [F, T+1, B], info [rl_loss_info_size(F)] (total loss last).
// Formulas: rl_utils.py (vtrace_advantages, upgo_returns, lambda_returns, td_lambda_loss), loss.py.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kH = 6;
constexpr int kMaxF = 6;
constexpr int kLossT = 256;
constexpr int kMaxTB = 2048;   // G_upgo staging in LDS

__device__ __forceinline__ void lds_add(float* p, float v) { atomicAdd(p, v); }

__global__ __launch_bounds__(kLossT) void rl_loss_kernel(const float* __restrict__ alp, const float* __restrict__ blp,
                                                         const float* __restrict__ hm, const float* __restrict__ ent,
                                                         const float* __restrict__ kl, const float* __restrict__ v,
                                                         const float* __restrict__ r, const float* __restrict__ wm,
                                                         const float* __restrict__ atflag,
                                                         const float* __restrict__ sc, int F, int T, int B, int upgo_f,
                                                         int only_value, float* __restrict__ dalp,
                                                         float* __restrict__ dent, float* __restrict__ dkl,
                                                         float* __restrict__ dv, float* __restrict__ info) {
  // scalars: per field f: [w_pg, w_baseline, gamma_pg, gamma_baseline]; then pg_w[6], upgo_w[6], ent_w[6],
  // kl_w[6], w_upgo, w_entropy, w_kl, w_action_type_kl
  const float* fsc = sc;
  const float* pg_w = sc + 4 * F;
  const float* upgo_w = pg_w + kH;
  const float* ent_w = upgo_w + kH;
  const float* kl_w = ent_w + kH;
  const float w_upgo = kl_w[kH], w_ent = kl_w[kH + 1], w_kl = kl_w[kH + 2], w_atkl = kl_w[kH + 3];
  const int TB = T * B;
  const float inv = 1.f / static_cast<float>(TB);

  __shared__ float g_up[kMaxTB];
  // accumulators: pg[f][h], td[f], rew[f], val[f], upgo[h], ent[h], kl[h], atkl
  __shared__ float s_pg[kMaxF][kH], s_td[kMaxF], s_rew[kMaxF], s_val[kMaxF], s_up[kH], s_ent[kH], s_kl[kH], s_at;
  const int tid = threadIdx.x;
  if (tid < kMaxF * kH) s_pg[tid / kH][tid % kH] = 0.f;
  if (tid < kMaxF) { s_td[tid] = 0.f; s_rew[tid] = 0.f; s_val[tid] = 0.f; }
  if (tid < kH) { s_up[tid] = 0.f; s_ent[tid] = 0.f; s_kl[tid] = 0.f; }
  if (tid == 0) s_at = 0.f;
  __syncthreads();

  // ---- phase A: one lane per (field, column): TD(lambda = 0.8) critic returns, loss and dV; UPGO returns
  for (int i = tid; i < F * B; i += kLossT) {
    const int f = i / B, b = i % B;
    const float* vf = v + static_cast<long>(f) * (T + 1) * B;
    const float* rf = r + static_cast<long>(f) * TB;
    const float* wf = wm + static_cast<long>(f) * TB;
    float* dvf = dv + static_cast<long>(f) * (T + 1) * B;
    const float gb = fsc[4 * f + 3], wbase = fsc[4 * f + 1];
    float g = 0.f, td = 0.f, rs = 0.f, vs = vf[T * B + b];
    dvf[T * B + b] = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const float lam = t == T - 1 ? 0.f : 0.8f;
      const float rr = rf[t * B + b], vn = vf[(t + 1) * B + b], vc = vf[t * B + b], w = wf[t * B + b];
      g = rr + gb * lam * g + gb * (1.f - lam) * vn;
      const float e = g - vc;
      td += 0.5f * e * e * w;
      dvf[t * B + b] = -wbase * e * w * inv;
      rs += rr;
      vs += vc;
    }
    lds_add(&s_td[f], td);
    lds_add(&s_rew[f], rs);
    lds_add(&s_val[f], vs);
    if (f == upgo_f) {
      // upgo lambda[t] = [r[t+1] + V[t+2] >= V[t+1]] (1 at the last step, then forced 0 there), gamma 1
      float gu = 0.f;
      for (int t = T - 1; t >= 0; --t) {
        float lam = 1.f;
        if (t + 1 < T) lam = (rf[(t + 1) * B + b] + vf[(t + 2) * B + b] >= vf[(t + 1) * B + b]) ? 1.f : 0.f;
        if (t == T - 1) lam = 0.f;
        gu = rf[t * B + b] + lam * gu + (1.f - lam) * vf[(t + 1) * B + b];
        g_up[t * B + b] = gu;
      }
    }
  }
  __syncthreads();

  // ---- phase B: one lane per (head, column): V-trace advantage scan per field + UPGO -> pg sums and dALP
  // (value pre-training: the sums still feed the info vector, the policy gradients are zero)
  const float gs = only_value ? 0.f : 1.f;
  {
    for (int i = tid; i < kH * B; i += kLossT) {
      const int h = i / B, b = i % B;
      const long hb = static_cast<long>(h) * TB;
      float up = 0.f;
      for (int t = 0; t < T; ++t) dalp[hb + t * B + b] = 0.f;
      for (int f = 0; f < F; ++f) {
        // every field's V-trace sum is logged (pg/<field>), also at pg weight 0 (the reference config trains
        // the policy on winloss only); the weight gates the gradient alone
        const float wpg = fsc[4 * f];
        const float gp = fsc[4 * f + 2];
        const float* vf = v + static_cast<long>(f) * (T + 1) * B;
        const float* rf = r + static_cast<long>(f) * TB;
        const float* wf = wm + static_cast<long>(f) * TB;
        float acc = 0.f, pg = 0.f;
        for (int t = T - 1; t >= 0; --t) {
          const int o = t * B + b;
          const float rho = fminf(__expf(alp[hb + o] - blp[hb + o]), 1.f);
          const float vn = vf[(t + 1) * B + b], vc = vf[o], rr = rf[o];
          // vs_next = acc[t+1] + V[t+1] (t < T-1), V[T] at the last step
          const float vs_next = (t == T - 1 ? 0.f : acc) + vn;
          const float adv = rho * (rr + gp * vs_next - vc);
          const float delta = rho * (rr + gp * vn - vc);
          acc = gp * rho * acc + delta;
          const float c = adv * hm[hb + o] * wf[o];
          pg += -c * alp[hb + o];
          dalp[hb + o] += -gs * wpg * pg_w[h] * c * inv;
        }
        lds_add(&s_pg[f][h], pg);
      }
      if (upgo_f >= 0) {
        const float* vf = v + static_cast<long>(upgo_f) * (T + 1) * B;
        for (int t = 0; t < T; ++t) {
          const int o = t * B + b;
          const float rho = fminf(__expf(alp[hb + o] - blp[hb + o]), 1.f);
          const float ua = rho * (g_up[o] - vf[o]) * hm[hb + o];
          up += -ua * alp[hb + o];
          dalp[hb + o] += -gs * w_upgo * upgo_w[h] * ua * inv;
        }
        lds_add(&s_up[h], up);
      }
    }
  }

  // ---- phase C: entropy and KL, elementwise over [6, T, B]
  float pe[kH], pk[kH], pa = 0.f;
#pragma unroll
  for (int h = 0; h < kH; ++h) { pe[h] = 0.f; pk[h] = 0.f; }
  for (int i = tid; i < kH * TB; i += kLossT) {
    const int h = i / TB, o = i % TB;
    const float m = hm[i];
    const float e = ent[i] * m, k = kl[i] * m;
#pragma unroll
    for (int q = 0; q < kH; ++q) {
      pe[q] += q == h ? e : 0.f;
      pk[q] += q == h ? k : 0.f;
    }
    float dk = only_value ? 0.f : w_kl * kl_w[h] * m * inv;
    if (h == 0) {
      pa += kl[i] * atflag[o];
      if (!only_value) dk += w_atkl * atflag[o] * inv;
    }
    dent[i] = only_value ? 0.f : -w_ent * ent_w[h] * m * inv;
    dkl[i] = dk;
  }
#pragma unroll
  for (int h = 0; h < kH; ++h) {
    const float se = wave_sum(pe[h]), sk = wave_sum(pk[h]);
    if ((tid & 63) == 0) { lds_add(&s_ent[h], se); lds_add(&s_kl[h], sk); }
  }
  {
    const float sa = wave_sum(pa);
    if ((tid & 63) == 0) lds_add(&s_at, sa);
  }
  __syncthreads();

  // ---- phase D: info + total (layout: rl_loss_info_size)
  if (tid == 0) {
    float total = 0.f, critic = 0.f;
    int o = 0;
    for (int f = 0; f < F; ++f) {
      float ft = 0.f;
      for (int h = 0; h < kH; ++h) ft += s_pg[f][h] * inv * pg_w[h];
      info[o++] = ft;
      for (int h = 0; h < kH; ++h) info[o++] = s_pg[f][h] * inv;
      const float td = s_td[f] * inv;
      info[o++] = td;
      info[o++] = s_rew[f] * inv;
      info[o++] = s_val[f] / static_cast<float>((T + 1) * B);
      total += fsc[4 * f] * ft;
      critic += fsc[4 * f + 1] * td;
    }
    float ut = 0.f;
    for (int h = 0; h < kH; ++h) {
      info[o++] = s_up[h] * inv;
      ut += s_up[h] * inv * upgo_w[h];
    }
    info[o++] = ut;
    float et = 0.f;
    for (int h = 0; h < kH; ++h) {
      info[o++] = s_ent[h] * inv;
      et -= s_ent[h] * inv * ent_w[h];
    }
    info[o++] = et;
    float kt = 0.f;
    for (int h = 0; h < kH; ++h) {
      info[o++] = s_kl[h] * inv;
      kt += s_kl[h] * inv * kl_w[h];
    }
    info[o++] = kt;
    const float at = s_at * inv;
    info[o++] = at;
    info[o++] = critic;
    if (upgo_f < 0) ut = 0.f;
    info[o] = only_value ? critic : total + ut * w_upgo + critic + et * w_ent + kt * w_kl + at * w_atkl;
  }
}

}  // namespace

int rl_loss_info_size(int F) { return 10 * F + 7 + 7 + 8 + 1 + 1; }
int rl_loss_max_tb() { return kMaxTB; }

void rl_loss(const float* alp, const float* blp, const float* hm, const float* ent, const float* kl, const float* v,
             const float* r, const float* wm, const float* atflag, const float* sc, int F, int T, int B, int upgo_f,
             int only_value, float* dalp, float* dent, float* dkl, float* dv, float* info, hipStream_t s) {
  hipLaunchKernelGGL(rl_loss_kernel, dim3(1), dim3(kLossT), 0, s, alp, blp, hm, ent, kl, v, r, wm, atflag, sc, F, T, B,
                     upgo_f, only_value, dalp, dent, dkl, dv, info);
}

}  // namespace as
