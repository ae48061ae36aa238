// Persistent selected-units pointer network for actor inference.
//
// The reference unrolls up to 64 dependent steps on the host (action_arg_head.py:262-313), ~15
// launches + host syncs per step.  Here ONE workgroup per batch row runs all steps on-chip:
//
//   x_t   = relu(c0 + bf + Wf . he_{t-1})       (t = 0: relu(c0))   Wf = Wq1 . We2 folded (256x256)
//   qin_t = Wq2 . x_t + bq2                                             (256 -> 32)
//   (h,c) = LN-LSTM32(qin_t; h, c)                                      gates i,f,g,o; LN_i, LN_h, LN_c
//   l_t[n] = (mask ? q . key[n] : -1e9) / T                             n <= entity_num (end token)
//   r_t   = inverse-CDF sample of softmax(l_t) with the given uniform u[b,t]
//   emb   = mean of the keys selected so far;  he_t = relu(We1 . emb + be1)
//
// The fold is exact algebra: query_fc1(ae0 + We2 he + be2) = (Wq1 ae0 + bq1) + Wq1 We2 he + Wq1 be2,
// so the per-step 1024-d autoregressive embedding never materialises (c0 = Wq1 ae0 + bq1 is one
// batched GEMM before the launch).  Weights live in registers for all steps (thread i owns row i
// of Wf / We1, a 32-slice of Wq2, and LSTM gate row i); keys [N+1,32] are staged once in LDS.
// Semantics match the reference loop: end token masked at step 0, sampled units masked afterwards,
// su_num = step+1 when the end token is drawn, extra_units = logits > end logit at the last step for
// rows that never drew the end token.  Rows end independently (a row's later steps are unused).
#include "common.h"
#include "kernels.h"

namespace as {
namespace {

constexpr int kThreads = 256;
constexpr int kQ = 32;       // key / query / LSTM hidden size
constexpr int kF = 256;      // func dim
constexpr int kMaxN1 = 513;  // 512 entities + end token
constexpr int kChunk = 3;    // ceil(513 / 256)
constexpr float kNeg = -1e9f;

__device__ __forceinline__ float block_sum(float v, float* red, int tid) {
  v = wave_sum(v);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float r = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_max(float v, float* red, int tid) {
  v = wave_max(v);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return r;
}

// sum over the 128 threads of waves 0-1 (waves 2-3 pass 0)
__device__ __forceinline__ float sum128(float v, float* red, int tid) {
  v = wave_sum(v);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  float r = red[0] + red[1];
  __syncthreads();
  return r;
}

template <typename KT>
__global__ __launch_bounds__(kThreads, 1) void su_sample_kernel(
    const KT* __restrict__ key, long key_bstride, const float* __restrict__ c0, const float* __restrict__ u,
    const int64_t* __restrict__ entity_num, const uint8_t* __restrict__ su_mask,
    const bf16_t* __restrict__ wf, const float* __restrict__ bf, const float* __restrict__ wq2,
    const float* __restrict__ bq2, const float* __restrict__ wih, const float* __restrict__ whh,
    const float* __restrict__ lni_w, const float* __restrict__ lni_b, const float* __restrict__ lnh_w,
    const float* __restrict__ lnh_b, const float* __restrict__ lnc_w, const float* __restrict__ lnc_b,
    const float* __restrict__ we1, const float* __restrict__ be1, float inv_temp, float eps, int n1_stride,
    int max_steps, int extra_units,
    float* __restrict__ logits_out, int64_t* __restrict__ results, float* __restrict__ logp_out,
    int64_t* __restrict__ su_num_out, float* __restrict__ emb_out, float* __restrict__ extra_out) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  // entity_num is clamped into the key tensor (no host-side check / sync needed)
  const int n1 = min(max(static_cast<int>(entity_num[b]), 0) + 1, n1_stride);
  const int en = n1 - 1;

  __shared__ float s_key[kMaxN1 * kQ];
  __shared__ uint8_t s_sel[kMaxN1 + 3];
  __shared__ float s_he[kF];
  __shared__ float s_x[kF];
  __shared__ float s_qin[kQ];
  __shared__ float s_h[kQ];
  __shared__ float s_q[kQ];
  __shared__ float s_gates[4 * kQ];
  __shared__ float s_emb[kQ];
  __shared__ float s_red[16];
  __shared__ float s_scan[4];
  __shared__ int s_result;

  const long kb = static_cast<long>(b) * key_bstride;
  for (int i = tid; i < n1 * kQ; i += kThreads) s_key[i] = Cvt<KT>::load(key, kb + i);
  for (int i = tid; i < n1; i += kThreads) s_sel[i] = 0;

  // ---- register-resident weights
  uint32_t wf_row[kF / 2];  // bf16 pairs of Wf[tid, :]
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(wf + static_cast<long>(tid) * kF);
#pragma unroll
    for (int j = 0; j < kF / 2; ++j) wf_row[j] = src[j];
  }
  const float c0_i = c0[static_cast<long>(b) * kF + tid] ;
  const float bf_i = bf[tid];
  float we1_row[kQ];
#pragma unroll
  for (int k = 0; k < kQ; ++k) we1_row[k] = we1[tid * kQ + k];
  const float be1_i = be1[tid];
  // qin: thread (o = tid>>3, p = tid&7) owns Wq2[o, p*32 : p*32+32]
  const int qo = tid >> 3, qp = tid & 7;
  float wq2_s[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) wq2_s[k] = wq2[qo * kF + qp * 32 + k];
  const float bq2_o = bq2[qo];
  // LSTM gate row tid (< 128)
  const int gr = tid < 4 * kQ ? tid : 0;
  float wih_r[kQ], whh_r[kQ];
#pragma unroll
  for (int k = 0; k < kQ; ++k) {
    wih_r[k] = wih[gr * kQ + k];
    whh_r[k] = whh[gr * kQ + k];
  }
  const float lniw = lni_w[gr], lnib = lni_b[gr], lnhw = lnh_w[gr], lnhb = lnh_b[gr];
  const float lncw = lnc_w[tid & 31], lncb = lnc_b[tid & 31];

  float h_state = 0.f, c_state = 0.f;  // lanes 0..31 of wave 0
  float emb_sum = 0.f;                 // lanes 0..31: running sum of selected keys (dim = lane)
  int cnt = 0;
  bool ended = su_mask[b] == 0;
  int su_num = ended ? 0 : max_steps;
  if (tid < kQ) s_h[tid] = 0.f;
  __syncthreads();

  float lv[kChunk];
  int step = 0;
  for (; step < max_steps && !ended; ++step) {
    // (a) x = relu(c0 + [bf + Wf he])
    float acc = c0_i;
    if (step > 0) {
      acc += bf_i;
#pragma unroll
      for (int j = 0; j < kF / 2; ++j) {
        const uint32_t w2 = wf_row[j];
        acc += __uint_as_float(w2 << 16) * s_he[2 * j] + __uint_as_float(w2 & 0xffff0000u) * s_he[2 * j + 1];
      }
    }
    s_x[tid] = fmaxf(acc, 0.f);
    __syncthreads();
    // (b) qin = Wq2 x + bq2
    float part = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) part += wq2_s[k] * s_x[qp * 32 + k];
    part += __shfl_xor(part, 1, kWave);
    part += __shfl_xor(part, 2, kWave);
    part += __shfl_xor(part, 4, kWave);
    if (qp == 0) s_qin[qo] = part + bq2_o;
    __syncthreads();
    // (c) gates = LN_i(Wih qin) + LN_h(Whh h)
    float gi = 0.f, gh = 0.f;
    if (tid < 4 * kQ) {
#pragma unroll
      for (int k = 0; k < kQ; ++k) {
        gi += wih_r[k] * s_qin[k];
        gh += whh_r[k] * s_h[k];
      }
    }
    const bool gact = tid < 4 * kQ;
    const float mi = sum128(gact ? gi : 0.f, s_red, tid) * (1.f / (4 * kQ));
    const float mh = sum128(gact ? gh : 0.f, s_red + 2, tid) * (1.f / (4 * kQ));
    const float di = gi - mi, dh = gh - mh;
    const float vi = sum128(gact ? di * di : 0.f, s_red + 4, tid) * (1.f / (4 * kQ));
    const float vh = sum128(gact ? dh * dh : 0.f, s_red + 6, tid) * (1.f / (4 * kQ));
    if (gact) s_gates[tid] = di * rsqrtf(vi + eps) * lniw + lnib + dh * rsqrtf(vh + eps) * lnhw + lnhb;
    __syncthreads();
    // (d) cell: lanes 0..31
    if (tid < kQ) {
      const float ig = sigmoidf_(s_gates[tid]), fg = sigmoidf_(s_gates[kQ + tid]);
      const float gg = tanhf(s_gates[2 * kQ + tid]), og = sigmoidf_(s_gates[3 * kQ + tid]);
      const float cp = fg * c_state + ig * gg;
      float m = cp;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) m += __shfl_xor(m, o, kWave);
      m *= (1.f / kQ);
      const float d = cp - m;
      float v = d * d;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
      v *= (1.f / kQ);
      c_state = d * rsqrtf(v + eps) * lncw + lncb;
      h_state = og * tanhf(c_state);
      s_h[tid] = h_state;
      s_q[tid] = h_state;
    }
    __syncthreads();
    // (e) logits over this thread's contiguous chunk
    const int n_base = tid * kChunk;
    float lmax = -3.0e38f;
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      const int n = n_base + k;
      float val = kNeg;
      if (n < n1) {
        const bool ok = !s_sel[n] && !(step == 0 && n == en);
        if (ok) {
          float d = 0.f;
#pragma unroll
          for (int c = 0; c < kQ; ++c) d += s_q[c] * s_key[n * kQ + c];
          val = d;
        }
        val *= inv_temp;
        logits_out[(static_cast<long>(b) * max_steps + step) * n1_stride + n] = val;
        lmax = fmaxf(lmax, val);
      }
      lv[k] = val;
    }
    const float m = block_max(lmax, s_red, tid);
    float es[kChunk];
    float local = 0.f;
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      es[k] = (n_base + k < n1) ? __expf(lv[k] - m) : 0.f;
      local += es[k];
    }
    // (f) inclusive block scan of chunk sums -> inverse-CDF pick
    float incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(incl, o, kWave);
      if ((tid & 63) >= o) incl += y;
    }
    if ((tid & 63) == 63) s_scan[tid >> 6] = incl;
    __syncthreads();
    float wave_off = 0.f;
    for (int w = 0; w < (tid >> 6); ++w) wave_off += s_scan[w];
    const float total = s_scan[0] + s_scan[1] + s_scan[2] + s_scan[3];
    const float target = u[static_cast<long>(b) * max_steps + step] * total;
    float run = wave_off + incl - local;  // exclusive prefix of this thread's chunk
    // the owner is the LAST thread whose exclusive prefix is <= target (exactly one, despite rounding)
    const float cand = (n_base < n1 && run <= target) ? static_cast<float>(tid) : -1.f;
    const int owner = static_cast<int>(block_max(cand, s_red, tid));
    if (tid == owner) {
      int pick = -1;
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        if (n_base + k < n1 && pick < 0) {
          run += es[k];
          if (run > target) pick = n_base + k;
        }
      }
      if (pick < 0) pick = min(n_base + kChunk, n1) - 1;
      s_result = pick;
    }
    __syncthreads();
    int r = s_result;
    if (r < 0) r = n1 - 1;
    // logp of the sample: l[r] - m - log(total)
    if (tid == r / kChunk) {
      const int k = r - (r / kChunk) * kChunk;
      float lr = lv[0];
      if (k == 1) lr = lv[1];
      if (k == 2) lr = lv[2];
      logp_out[static_cast<long>(b) * max_steps + step] = lr - m - __logf(total);
      results[static_cast<long>(b) * max_steps + step] = r;
    }
    // (g) bookkeeping (uniform across the block)
    if (tid == 0) s_sel[r] = 1;
    if (r == en) {
      ended = true;
      su_num = step + 1;
    } else {
      ++cnt;
      if (tid < kQ) emb_sum += s_key[r * kQ + tid];
    }
    if (tid < kQ) s_emb[tid] = cnt > 0 ? emb_sum / static_cast<float>(cnt) : 0.f;
    __syncthreads();
    // he = relu(We1 emb + be1)
    float he = be1_i;
#pragma unroll
    for (int k = 0; k < kQ; ++k) he += we1_row[k] * s_emb[k];
    s_he[tid] = fmaxf(he, 0.f);
    __syncthreads();
  }
  if (tid == 0) su_num_out[b] = su_num;
  if (tid < kQ) emb_out[static_cast<long>(b) * kQ + tid] = cnt > 0 ? emb_sum / static_cast<float>(cnt) : 0.f;
  if (extra_units) {
    // rows that never drew the end token: units whose last-step logit beats the end token's
    const bool never_ended = su_mask[b] != 0 && !ended;
    float end_logit = 0.f;
    if (never_ended) end_logit = logits_out[(static_cast<long>(b) * max_steps + (max_steps - 1)) * n1_stride + en];
    for (int n = tid; n < n1_stride; n += kThreads) {
      float e = 0.f;
      if (never_ended && n < n1)
        e = logits_out[(static_cast<long>(b) * max_steps + (max_steps - 1)) * n1_stride + n] > end_logit ? 1.f : 0.f;
      extra_out[static_cast<long>(b) * n1_stride + n] = e;
    }
  }
}

}  // namespace

void su_sample(const void* key, int key_dt, long key_bstride, const float* c0, const float* u, const int64_t* entity_num,
               const uint8_t* su_mask, const bf16_t* wf, const float* bf, const float* wq2, const float* bq2,
               const float* wih, const float* whh, const float* lni_w, const float* lni_b, const float* lnh_w,
               const float* lnh_b, const float* lnc_w, const float* lnc_b, const float* we1, const float* be1,
               float inv_temp, float eps, int B, int n1_stride, int max_steps, int extra_units, float* logits,
               int64_t* results, float* logp, int64_t* su_num, float* emb, float* extra, hipStream_t s) {
  if (B == 0) return;
  if (key_dt == DT_BF16) {
    hipLaunchKernelGGL(su_sample_kernel<bf16_t>, dim3(B), dim3(kThreads), 0, s, static_cast<const bf16_t*>(key),
                       key_bstride, c0, u, entity_num, su_mask, wf, bf, wq2, bq2, wih, whh, lni_w, lni_b, lnh_w, lnh_b,
                       lnc_w, lnc_b, we1, be1, inv_temp, eps, n1_stride, max_steps, extra_units, logits, results, logp,
                       su_num, emb, extra);
  } else {
    hipLaunchKernelGGL(su_sample_kernel<float>, dim3(B), dim3(kThreads), 0, s, static_cast<const float*>(key),
                       key_bstride, c0, u, entity_num, su_mask, wf, bf, wq2, bq2, wih, whh, lni_w, lni_b, lnh_w, lnh_b,
                       lnc_w, lnc_b, we1, be1, inv_temp, eps, n1_stride, max_steps, extra_units, logits, results, logp,
                       su_num, emb, extra);
  }
}

}  // namespace as
