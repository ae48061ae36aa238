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
// batched GEMM before the launch).  Weights stay on-chip for all steps: thread i owns row i of Wf / We1 in
// registers; keys [N+1,32], the Wq2 slices and the LSTM gate weights (wave 0's lane l: rows l and l + 64) are
// staged once in LDS.  A step has 7 block barriers (was 19): the LSTM cell runs in wave 0 alone on wave
// reductions, the sampling max / scan exchange wave totals through parity-alternating LDS slots, the owner
// of the inverse-CDF pick is found by one wave ballot, and every thread keeps the running key sum itself.
// Semantics match the reference loop: end token masked at step 0, sampled units masked afterwards,
// su_num = step+1 when the end token is drawn, extra_units = logits > end logit at the last step for
// rows that never drew the end token.  Rows end independently (a row's later steps are unused).
#include <cstdlib>

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
  __shared__ float s_wih[kQ * 4 * kQ];   // [k][gate row]
  __shared__ float s_whh[kQ * 4 * kQ];
  __shared__ float s_wq2[32 * kThreads];
  __shared__ uint8_t s_sel[kMaxN1 + 3];
  __shared__ __align__(16) float s_he[kF];
  __shared__ float s_x[kF];
  __shared__ float s_u[64];               // the row's uniforms, staged once (a global load per step sat on the
                                          // critical path of every pointer step)
  __shared__ float s_qin[kQ];
  __shared__ float s_h[kQ];
  __shared__ float s_q[kQ];
  __shared__ float s_red[16];   // two parity halves: 4 wave maxima + 4 wave scan totals each
  __shared__ int s_result;

  const long kb = static_cast<long>(b) * key_bstride;
  for (int i = tid; i < n1 * kQ; i += kThreads) s_key[i] = Cvt<KT>::load(key, kb + i);
  for (int i = tid; i < n1; i += kThreads) s_sel[i] = 0;
  for (int i = tid; i < max_steps && i < 64; i += kThreads) s_u[i] = u[static_cast<long>(b) * max_steps + i];

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
  // (in LDS as [k][thread]: conflict-free, and the registers stay below the 256 architectural VGPRs)
#pragma unroll 4
  for (int k = 0; k < 32; ++k) s_wq2[k * kThreads + tid] = wq2[qo * kF + qp * 32 + k];
  const float bq2_o = bq2[qo];
  // LSTM: wave 0 runs the whole cell (no block barriers); lane l owns gate rows l and l + 64 (i / f rows in
  // the first, g / o rows in the second), so LN_i / LN_h statistics are wave reductions and the cell's f / o
  // inputs arrive from lane l + 32 by a cross-lane read
  // (the gate weights sit in LDS, k-major so a wave's row reads are conflict-free: the registers are full)
  const int gr = tid & 63;
  for (int i = tid; i < 4 * kQ * kQ; i += kThreads) {
    const int row = i / kQ, k = i % kQ;
    s_wih[k * 4 * kQ + row] = wih[i];
    s_whh[k * 4 * kQ + row] = whh[i];
  }
  const float lniw0 = lni_w[gr], lnib0 = lni_b[gr], lnhw0 = lnh_w[gr], lnhb0 = lnh_b[gr];
  const float lniw1 = lni_w[gr + 64], lnib1 = lni_b[gr + 64], lnhw1 = lnh_w[gr + 64], lnhb1 = lnh_b[gr + 64];
  const float lncw = lnc_w[tid & 31], lncb = lnc_b[tid & 31];
  const int nwaves_valid = min((n1 + 64 * kChunk - 1) / (64 * kChunk), kThreads / 64);

  float h_state = 0.f, c_state = 0.f;  // lanes 0..31 of wave 0
  float emb_sum = 0.f;                 // lanes 0..31: running sum of the selected keys (dim = lane)
  float he_sum = 0.f;                  // every thread: We1[tid] . (running key sum), so he needs no exchange
  int cnt = 0;
  bool ended = su_mask[b] == 0;
  int su_num = ended ? 0 : max_steps;
  if (tid < kQ) s_h[tid] = 0.f;
  // the outputs of the steps this row will not run (and the padding columns of those it does): -1e9 logits, zero
  // results / log-probabilities - the host allocates them uninitialised (four fill launches per forward before);
  // the barrier below orders these stores before the step loop's
  {
    const long lbase = static_cast<long>(b) * max_steps * n1_stride;
    for (long i = tid; i < static_cast<long>(max_steps) * n1_stride; i += kThreads) logits_out[lbase + i] = kNeg;
    for (int i = tid; i < max_steps; i += kThreads) {
      results[static_cast<long>(b) * max_steps + i] = 0;
      logp_out[static_cast<long>(b) * max_steps + i] = 0.f;
    }
  }
  __syncthreads();

  float lv[kChunk];
  int step = 0;
  for (; step < max_steps && !ended; ++step) {
    // (a) x = relu(c0 + [bf + Wf he])
    float acc = c0_i;
    if (step > 0) {
      // he read 32 floats (8 LDS reads in flight) per fenced chunk into 4 independent FMA chains: unfenced, the
      // compiler hoists all 64 reads ahead of the FMAs and the live values push the weights out to AGPRs; one
      // fence per 8 floats serialised the LDS latency 32 times per step
      float a4[4] = {bf_i, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < kF / 2; j += 16) {
        float hv[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float4 h = *reinterpret_cast<const float4*>(s_he + 2 * j + 4 * q);
          hv[4 * q] = h.x;
          hv[4 * q + 1] = h.y;
          hv[4 * q + 2] = h.z;
          hv[4 * q + 3] = h.w;
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const uint32_t w2 = wf_row[j + e];
          a4[e & 3] = fmaf(__uint_as_float(w2 << 16), hv[2 * e], a4[e & 3]);
          a4[e & 3] = fmaf(__uint_as_float(w2 & 0xffff0000u), hv[2 * e + 1], a4[e & 3]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      acc += (a4[0] + a4[1]) + (a4[2] + a4[3]);
    }
    s_x[tid] = fmaxf(acc, 0.f);
    __syncthreads();
    // (b) qin = Wq2 x + bq2
    float part = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) part += s_wq2[k * kThreads + tid] * s_x[qp * 32 + k];
    part += __shfl_xor(part, 1, kWave);
    part += __shfl_xor(part, 2, kWave);
    part += __shfl_xor(part, 4, kWave);
    if (qp == 0) s_qin[qo] = part + bq2_o;
    __syncthreads();
    // (c) + (d) gates = LN_i(Wih qin) + LN_h(Whh h), then the cell: wave 0 alone
    if (tid < 64) {
      float gi0 = 0.f, gh0 = 0.f, gi1 = 0.f, gh1 = 0.f;
#pragma unroll
      for (int k = 0; k < kQ; ++k) {
        const float q = s_qin[k], hk = s_h[k];
        gi0 += s_wih[k * 4 * kQ + gr] * q;
        gh0 += s_whh[k * 4 * kQ + gr] * hk;
        gi1 += s_wih[k * 4 * kQ + gr + 64] * q;
        gh1 += s_whh[k * 4 * kQ + gr + 64] * hk;
      }
      const float mi = wave_sum(gi0 + gi1) * (1.f / (4 * kQ));
      const float mh = wave_sum(gh0 + gh1) * (1.f / (4 * kQ));
      const float di0 = gi0 - mi, di1 = gi1 - mi, dh0 = gh0 - mh, dh1 = gh1 - mh;
      const float ri = rsqrtf(wave_sum(di0 * di0 + di1 * di1) * (1.f / (4 * kQ)) + eps);
      const float rh = rsqrtf(wave_sum(dh0 * dh0 + dh1 * dh1) * (1.f / (4 * kQ)) + eps);
      const float g0 = di0 * ri * lniw0 + lnib0 + dh0 * rh * lnhw0 + lnhb0;   // row l:      i (l < 32) / f
      const float g1 = di1 * ri * lniw1 + lnib1 + dh1 * rh * lnhw1 + lnhb1;   // row l + 64: g (l < 32) / o
      const float gf = __shfl(g0, (tid & 31) + 32, kWave);
      const float go = __shfl(g1, (tid & 31) + 32, kWave);
      if (tid < kQ) {
        const float ig = sigmoidf_(g0), fg = sigmoidf_(gf), gg = tanhf(g1), og = sigmoidf_(go);
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
        s_h[tid] = h_state;   // read next step by this wave only (after the block barriers in between)
        s_q[tid] = h_state;
      }
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
    // block max: one barrier (the slots alternate by step parity, so no second barrier guards their reuse)
    float* red = s_red + 8 * (step & 1);
    lmax = wave_max(lmax);
    if ((tid & 63) == 0) red[tid >> 6] = lmax;
    __syncthreads();
    const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float es[kChunk];
    float local = 0.f;
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      es[k] = (n_base + k < n1) ? __expf(lv[k] - m) : 0.f;
      local += es[k];
    }
    // (f) inclusive wave scan of chunk sums, wave totals through LDS -> inverse-CDF pick
    float incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(incl, o, kWave);
      if ((tid & 63) >= o) incl += y;
    }
    float* scan = red + 4;
    if ((tid & 63) == 63) scan[tid >> 6] = incl;
    __syncthreads();
    const int wv = tid >> 6;
    float wave_off = 0.f;
    const float total = scan[0] + scan[1] + scan[2] + scan[3];
    const float target = s_u[step] * total;
    // the owner wave: the last wave with entities whose offset is <= target (every thread computes the same
    // offsets in the same order); the owner lane: the last lane of that wave whose exclusive prefix is <= target
    int owner_wave = 0;
    {
      float off = 0.f;
      for (int w = 0; w < nwaves_valid; ++w) {
        if (w == wv) wave_off = off;
        if (off <= target) owner_wave = w;
        off += scan[w];
      }
      if (wv >= nwaves_valid) wave_off = off;
    }
    if (wv == owner_wave) {
      float run = wave_off + incl - local;  // exclusive prefix of this thread's chunk
      const bool cand = n_base < n1 && run <= target;
      const unsigned long long bal = __ballot(cand);
      const int owner = 63 - __builtin_clzll(bal | 1ull);
      if ((tid & 63) == owner) {
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
    // (g) bookkeeping (uniform across the block); every thread keeps the running key sum itself
    if (tid == 0) s_sel[r] = 1;
    if (r == en) {
      ended = true;
      su_num = step + 1;
    } else {
      ++cnt;
      if (tid < kQ) emb_sum += s_key[r * kQ + tid];
      float d = 0.f;
#pragma unroll
      for (int k = 0; k < kQ; ++k) d += we1_row[k] * s_key[r * kQ + k];
      he_sum += d;
    }
    // he = relu(We1 emb + be1), emb = key sum / cnt
    const float he = be1_i + (cnt > 0 ? he_sum / static_cast<float>(cnt) : 0.f);
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
    // written at the padded width kMaxN1 (the model's [B, 513] extra-units map; zeros past this row's entities)
    for (int n = tid; n < kMaxN1; n += kThreads) {
      float e = 0.f;
      if (never_ended && n < n1)
        e = logits_out[(static_cast<long>(b) * max_steps + (max_steps - 1)) * n1_stride + n] > end_logit ? 1.f : 0.f;
      extra_out[static_cast<long>(b) * kMaxN1 + n] = e;
    }
  }
}


// ---------------------------------------------------------------------------------------------------------------
// Wide form: 1024 threads (16 waves, 4 per SIMD) per row.  The 256-thread kernel above measured 6.7 us per pointer
// step at ~12.7 cycles per instruction (PMC: one wave per SIMD, so every dependent VALU / LDS latency sits on the
// critical path).  Here every phase is split over the whole workgroup and the per-thread chains are short:
//   (a) x = relu(c0 + bf + Wf he): thread = (row t >> 2, quarter t & 3), 64 products, 2 shuffles
//   (b) qin = Wq2 x + bq2:         thread = (output t >> 5, slice t & 31), 8 products, 5 shuffles
//   (c) gates:                     thread = (gate row t >> 3, part t & 7: Wih / Whh, 8 inputs each), 2 shuffles;
//                                  LN statistics + the cell in wave 0 (as above)
//   (e) logits:                    thread = entity (n = t), 32 products off a conflict-free swizzled key row
//   (f) max + scan:                one barrier - each wave exchanges its max and its scan total in its own scale
// Wf (64 bf16), Wq2 (8) and the gate weights (8) of a thread live in its registers (128 VGPRs at 4 waves per SIMD);
// We1 is staged in LDS with the keys' swizzle (row j read by thread j).
// Same semantics and outputs as su_sample_kernel (the inverse-CDF pick over a 1-entity chunk per thread).
constexpr int kWThreads = 1024;
constexpr int kWWaves = kWThreads / 64;
constexpr int kHeQ = 64 + 8;     // a he quarter (64 bf16) padded by 16 bytes: the 4 quarters read 4 distinct slots

__device__ __forceinline__ float dot2bf(uint32_t a, uint32_t b, float c) {   // a.lo*b.lo + a.hi*b.hi + c
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, a), __builtin_bit_cast(bf2, b), c, false);
}
__device__ __forceinline__ float fast_tanh(float x) {     // 1 - 2 / (1 + e^2x): v_exp + v_rcp, saturates cleanly
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}

// Cross-lane arithmetic on DPP and v_readlane instead of ds_bpermute (__shfl_*): a bpermute is an LDS round trip,
// and a step's ~55 of them in serial reduction / scan chains were most of its latency.
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {      // lanes without a source (row_shr) read 0
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float lanef(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
constexpr int kXor1 = 0xB1, kXor2 = 0x4E, kHalfMirror = 0x141, kMirror = 0x140;   // quad_perm / row mirrors
__device__ __forceinline__ float row_sum16(float v) {  // every lane: the sum of its 16-lane row
  v += dppf<kXor1>(v);
  v += dppf<kXor2>(v);
  v += dppf<kHalfMirror>(v);
  return v + dppf<kMirror>(v);
}
__device__ __forceinline__ float dpp_wave_sum(float v) {
  const float r = row_sum16(v);
  return (lanef(r, 0) + lanef(r, 16)) + (lanef(r, 32) + lanef(r, 48));
}
__device__ __forceinline__ float dpp_wave_max(float v) {
  v = fmaxf(v, dppf<kXor1>(v));
  v = fmaxf(v, dppf<kXor2>(v));
  v = fmaxf(v, dppf<kHalfMirror>(v));
  v = fmaxf(v, dppf<kMirror>(v));
  return fmaxf(fmaxf(lanef(v, 0), lanef(v, 16)), fmaxf(lanef(v, 32), lanef(v, 48)));
}
__device__ __forceinline__ float dpp_wave_scan(float v, int lane) {   // inclusive prefix sum over the wave
  v += dppf<0x111>(v);   // row_shr:1
  v += dppf<0x112>(v);   // row_shr:2
  v += dppf<0x114>(v);   // row_shr:4
  v += dppf<0x118>(v);   // row_shr:8
  const float t0 = lanef(v, 15), t1 = lanef(v, 31), t2 = lanef(v, 47);
  const int row = lane >> 4;
  return v + (row >= 1 ? t0 : 0.f) + (row >= 2 ? t1 : 0.f) + (row >= 3 ? t2 : 0.f);
}

// keys and We1 as [dim / 4][row] float4 planes: a thread reading its own row touches consecutive 16-byte slots
// across the lanes (conflict-free) at immediate offsets; a broadcast row read is one address per plane
__device__ __forceinline__ int kslot(int n, int c) { return ((c >> 2) * kMaxN1 + n) * 4 + (c & 3); }
__device__ __forceinline__ int wslot(int j, int c) { return ((c >> 2) * kF + j) * 4 + (c & 3); }

template <typename KT>
__global__ __launch_bounds__(kWThreads, 1) void su_sample_wide_kernel(
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
  const int lane = tid & 63, wv = tid >> 6;
  const int n1 = min(max(static_cast<int>(entity_num[b]), 0) + 1, n1_stride);
  const int en = n1 - 1;

  __shared__ __align__(16) float s_key[kMaxN1 * kQ];
  __shared__ uint8_t s_sel[kMaxN1 + 3];
  __shared__ __align__(16) uint16_t s_hehi[4 * kHeQ];   // he split into bf16 hi + lo, 4 padded quarters
  __shared__ __align__(16) uint16_t s_helo[4 * kHeQ];
  __shared__ __align__(16) float s_x[kF];
  __shared__ float s_u[64];
  __shared__ __align__(16) float s_qin[kQ];
  __shared__ __align__(16) float s_h[kQ];
  __shared__ __align__(16) float s_q[kQ];
  __shared__ float s_gi[4 * kQ];
  __shared__ float s_gh[4 * kQ];
  __shared__ float s_red[4 * kWWaves];   // two parity halves: 16 wave maxima + 16 wave scan totals each
  __shared__ int s_result;
  __shared__ __align__(16) float s_we1[kF * kQ];

  const long kb = static_cast<long>(b) * key_bstride;
  for (int i = tid; i < n1 * kQ; i += kWThreads) s_key[kslot(i >> 5, i & 31)] = Cvt<KT>::load(key, kb + i);
  for (int i = tid; i < kF * kQ; i += kWThreads) s_we1[wslot(i >> 5, i & 31)] = we1[i];
  for (int i = tid; i < n1; i += kWThreads) s_sel[i] = 0;
  if (tid < max_steps && tid < 64) s_u[tid] = u[static_cast<long>(b) * max_steps + tid];

  // ---- register-resident weights
  const int ar = tid >> 2, aq = tid & 3;                 // (a): row, quarter of the 256 inputs
  uint32_t wf_q[32];                                     // bf16 pairs of Wf[ar, aq*64 : aq*64+64]
  {
    const uint4* src = reinterpret_cast<const uint4*>(wf + static_cast<long>(ar) * kF + aq * 64);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 v = src[j];
      wf_q[4 * j] = v.x;
      wf_q[4 * j + 1] = v.y;
      wf_q[4 * j + 2] = v.z;
      wf_q[4 * j + 3] = v.w;
    }
  }
  const float c0_r = c0[static_cast<long>(b) * kF + ar], bf_r = bf[ar];   // x_0 = relu(c0): no bf term at step 0
  const int qo = tid >> 5, qp = tid & 31;                // (b): output, slice of 8 inputs
  float wq[8];
  {
    const float4* src = reinterpret_cast<const float4*>(wq2 + qo * kF + qp * 8);
    const float4 v0 = src[0], v1 = src[1];
    wq[0] = v0.x; wq[1] = v0.y; wq[2] = v0.z; wq[3] = v0.w;
    wq[4] = v1.x; wq[5] = v1.y; wq[6] = v1.z; wq[7] = v1.w;
  }
  const float bq2_o = bq2[qo];
  const int gr = tid >> 3, gp = tid & 7;                 // (c): gate row, part (0-3: Wih, 4-7: Whh; 8 inputs each)
  float wg[8];
  {
    const float* wsrc = (gp < 4 ? wih : whh) + gr * kQ + (gp & 3) * 8;
    const float4 v0 = reinterpret_cast<const float4*>(wsrc)[0], v1 = reinterpret_cast<const float4*>(wsrc)[1];
    wg[0] = v0.x; wg[1] = v0.y; wg[2] = v0.z; wg[3] = v0.w;
    wg[4] = v1.x; wg[5] = v1.y; wg[6] = v1.z; wg[7] = v1.w;
  }
  // LN-LSTM cell in wave 0: lane l owns gate rows l and l + 64 (as in su_sample_kernel)
  float lniw0 = 0.f, lnib0 = 0.f, lnhw0 = 0.f, lnhb0 = 0.f, lniw1 = 0.f, lnib1 = 0.f, lnhw1 = 0.f, lnhb1 = 0.f;
  float lncw = 0.f, lncb = 0.f;
  if (wv == 0) {
    lniw0 = lni_w[lane]; lnib0 = lni_b[lane]; lnhw0 = lnh_w[lane]; lnhb0 = lnh_b[lane];
    lniw1 = lni_w[lane + 64]; lnib1 = lni_b[lane + 64]; lnhw1 = lnh_w[lane + 64]; lnhb1 = lnh_b[lane + 64];
    lncw = lnc_w[lane & 31]; lncb = lnc_b[lane & 31];
  }
  const float be1_j = tid < kF ? be1[tid] : 0.f;        // (g): thread j < 256 owns row j of We1
  const int nwaves_valid = min((n1 + 63) / 64, kWWaves);

  float h_state = 0.f, c_state = 0.f;   // lanes 0..31 of wave 0
  float emb_sum = 0.f;                  // threads 0..31: running sum of the selected keys (dim = tid)
  float he_sum = 0.f;                   // threads 0..255: We1[tid] . (running key sum)
  int cnt = 0;
  bool ended = su_mask[b] == 0;
  int su_num = ended ? 0 : max_steps;
  if (tid < kQ) s_h[tid] = 0.f;
  {
    const long lbase = static_cast<long>(b) * max_steps * n1_stride;
    for (long i = tid; i < static_cast<long>(max_steps) * n1_stride; i += kWThreads) logits_out[lbase + i] = kNeg;
    if (tid < max_steps) {
      results[static_cast<long>(b) * max_steps + tid] = 0;
      logp_out[static_cast<long>(b) * max_steps + tid] = 0.f;
    }
  }
  __syncthreads();

  int step = 0;
  for (; step < max_steps && !ended; ++step) {
    // (a) x = relu(c0 + bf + Wf he)
    {
      float acc = 0.f;
      if (step > 0) {
        // he = hi + lo (bf16 pairs, split by the writer): two bf16 dot2 per weight pair, products exact in fp32
        float a4[4] = {0.f, 0.f, 0.f, 0.f};
        const uint4* hh = reinterpret_cast<const uint4*>(s_hehi + aq * kHeQ);
        const uint4* hl = reinterpret_cast<const uint4*>(s_helo + aq * kHeQ);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint4 h = hh[j], l = hl[j];
          a4[0] = dot2bf(wf_q[4 * j], h.x, a4[0]);
          a4[1] = dot2bf(wf_q[4 * j + 1], h.y, a4[1]);
          a4[2] = dot2bf(wf_q[4 * j + 2], h.z, a4[2]);
          a4[3] = dot2bf(wf_q[4 * j + 3], h.w, a4[3]);
          a4[0] = dot2bf(wf_q[4 * j], l.x, a4[0]);
          a4[1] = dot2bf(wf_q[4 * j + 1], l.y, a4[1]);
          a4[2] = dot2bf(wf_q[4 * j + 2], l.z, a4[2]);
          a4[3] = dot2bf(wf_q[4 * j + 3], l.w, a4[3]);
        }
        acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        acc += dppf<kXor1>(acc);
        acc += dppf<kXor2>(acc);
        acc += bf_r;
      }
      if (aq == 0) s_x[ar] = fmaxf(c0_r + acc, 0.f);
    }
    __syncthreads();
    // (b) qin = Wq2 x + bq2
    {
      const float4 x0 = *reinterpret_cast<const float4*>(s_x + qp * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(s_x + qp * 8 + 4);
      float part = wq[0] * x0.x + wq[1] * x0.y + wq[2] * x0.z + wq[3] * x0.w;
      part += wq[4] * x1.x + wq[5] * x1.y + wq[6] * x1.z + wq[7] * x1.w;
      part = row_sum16(part);
      const float lo = lanef(part, 0) + lanef(part, 16), hi = lanef(part, 32) + lanef(part, 48);
      if (qp == 0) s_qin[qo] = (lane < 32 ? lo : hi) + bq2_o;
    }
    __syncthreads();
    // (c) gate rows: Wih qin (parts 0-3) and Whh h (parts 4-7)
    {
      const float* in = (gp < 4 ? s_qin : s_h) + (gp & 3) * 8;
      const float4 i0 = *reinterpret_cast<const float4*>(in);
      const float4 i1 = *reinterpret_cast<const float4*>(in + 4);
      float g = wg[0] * i0.x + wg[1] * i0.y + wg[2] * i0.z + wg[3] * i0.w;
      g += wg[4] * i1.x + wg[5] * i1.y + wg[6] * i1.z + wg[7] * i1.w;
      g += dppf<kXor1>(g);
      g += dppf<kXor2>(g);
      if (gp == 0) s_gi[gr] = g;
      if (gp == 4) s_gh[gr] = g;
    }
    __syncthreads();
    if (wv == 0) {
      const float gi0 = s_gi[lane], gi1 = s_gi[lane + 64], gh0 = s_gh[lane], gh1 = s_gh[lane + 64];
      const float mi = dpp_wave_sum(gi0 + gi1) * (1.f / (4 * kQ));
      const float mh = dpp_wave_sum(gh0 + gh1) * (1.f / (4 * kQ));
      const float di0 = gi0 - mi, di1 = gi1 - mi, dh0 = gh0 - mh, dh1 = gh1 - mh;
      const float ri = rsqrtf(dpp_wave_sum(di0 * di0 + di1 * di1) * (1.f / (4 * kQ)) + eps);
      const float rh = rsqrtf(dpp_wave_sum(dh0 * dh0 + dh1 * dh1) * (1.f / (4 * kQ)) + eps);
      const float g0 = di0 * ri * lniw0 + lnib0 + dh0 * rh * lnhw0 + lnhb0;   // row l:      i (l < 32) / f
      const float g1 = di1 * ri * lniw1 + lnib1 + dh1 * rh * lnhw1 + lnhb1;   // row l + 64: g (l < 32) / o
      const float gf = __shfl(g0, (lane & 31) + 32, kWave);
      const float go = __shfl(g1, (lane & 31) + 32, kWave);
      {   // the cell in lanes 0..31 (the reductions run over the whole wave: lanes 32..63 contribute nothing)
        const bool cl = lane < kQ;
        const float ig = sigmoidf_(g0), fg = sigmoidf_(gf), gg = fast_tanh(g1), og = sigmoidf_(go);
        const float cp = cl ? fg * c_state + ig * gg : 0.f;
        const float m = dpp_wave_sum(cp) * (1.f / kQ);
        const float d = cl ? cp - m : 0.f;
        const float v = dpp_wave_sum(d * d) * (1.f / kQ);
        if (cl) {
          c_state = d * rsqrtf(v + eps) * lncw + lncb;
          h_state = og * fast_tanh(c_state);
          s_h[lane] = h_state;
          s_q[lane] = h_state;
        }
      }
    }
    __syncthreads();
    // (e) this thread's entity logit
    const int n = tid;
    float lv = kNeg;
    if (n < n1) {
      if (!s_sel[n] && !(step == 0 && n == en)) {
        float d0 = 0.f, d1 = 0.f;
#pragma unroll
        for (int c4 = 0; c4 < kQ / 4; ++c4) {
          const float4 kv = *reinterpret_cast<const float4*>(s_key + kslot(n, 4 * c4));
          const float4 qv = *reinterpret_cast<const float4*>(s_q + 4 * c4);
          d0 = fmaf(qv.x, kv.x, d0);
          d1 = fmaf(qv.y, kv.y, d1);
          d0 = fmaf(qv.z, kv.z, d0);
          d1 = fmaf(qv.w, kv.w, d1);
        }
        lv = d0 + d1;
      }
      lv *= inv_temp;
      logits_out[(static_cast<long>(b) * max_steps + step) * n1_stride + n] = lv;
    }
    // (f) max + scan with one barrier
    float* red = s_red + 2 * kWWaves * (step & 1);
    const float mw = dpp_wave_max(n < n1 ? lv : -3.0e38f);
    const float es = n < n1 ? __expf(lv - mw) : 0.f;
    const float incl = dpp_wave_scan(es, lane);
    if (lane == 63) {
      red[wv] = mw;
      red[kWWaves + wv] = incl;
    }
    __syncthreads();
    float m = red[0];
    for (int w = 1; w < nwaves_valid; ++w) m = fmaxf(m, red[w]);
    // the wave totals in the common scale: every thread computes the same values in the same order
    float total = 0.f, wave_off = 0.f;
    int owner_wave = 0;
    for (int w = 0; w < nwaves_valid; ++w) total += red[kWWaves + w] * __expf(red[w] - m);
    const float target = s_u[step] * total;
    {
      float off = 0.f;
      for (int w = 0; w < nwaves_valid; ++w) {
        if (w == wv) wave_off = off;
        if (off <= target) owner_wave = w;
        off += red[kWWaves + w] * __expf(red[w] - m);
      }
    }
    if (wv == owner_wave) {
      const float scale = __expf(mw - m);
      const float run = wave_off + (incl - es) * scale;     // exclusive prefix of this entity
      const unsigned long long bal = __ballot(n < n1 && run <= target);
      const int owner = 63 - __builtin_clzll(bal | 1ull);
      if (lane == owner) s_result = n;
    }
    __syncthreads();
    const int r = s_result;
    if (tid == r) {
      logp_out[static_cast<long>(b) * max_steps + step] = lv - m - __logf(total);
      results[static_cast<long>(b) * max_steps + step] = r;
    }
    // (g) bookkeeping (uniform across the block)
    if (tid == 0) s_sel[r] = 1;
    if (r == en) {
      ended = true;
      su_num = step + 1;
    } else {
      ++cnt;
      if (tid < kQ) emb_sum += s_key[kslot(r, tid)];
      if (tid < kF) {
        float d0 = 0.f, d1 = 0.f;
#pragma unroll
        for (int c4 = 0; c4 < kQ / 4; ++c4) {
          const float4 kv = *reinterpret_cast<const float4*>(s_key + kslot(r, 4 * c4));
          const float4 wv4 = *reinterpret_cast<const float4*>(s_we1 + wslot(tid, 4 * c4));
          d0 = fmaf(wv4.x, kv.x, d0);
          d1 = fmaf(wv4.y, kv.y, d1);
          d0 = fmaf(wv4.z, kv.z, d0);
          d1 = fmaf(wv4.w, kv.w, d1);
        }
        he_sum += d0 + d1;
      }
    }
    if (tid < kF) {
      const float he = be1_j + (cnt > 0 ? he_sum / static_cast<float>(cnt) : 0.f);
      const float hv = fmaxf(he, 0.f);
      const uint32_t hb = __float_as_uint(hv) & 0xffff0000u;               // hi: truncated (exact remainder)
      const int at = (tid >> 6) * kHeQ + (tid & 63);
      s_hehi[at] = static_cast<uint16_t>(hb >> 16);
      s_helo[at] = f2bf(hv - __uint_as_float(hb));
    }
    __syncthreads();
  }
  if (tid == 0) su_num_out[b] = su_num;
  if (tid < kQ) emb_out[static_cast<long>(b) * kQ + tid] = cnt > 0 ? emb_sum / static_cast<float>(cnt) : 0.f;
  if (extra_units) {
    const bool never_ended = su_mask[b] != 0 && !ended;
    float end_logit = 0.f;
    if (never_ended) end_logit = logits_out[(static_cast<long>(b) * max_steps + (max_steps - 1)) * n1_stride + en];
    for (int n = tid; n < kMaxN1; n += kWThreads) {
      float e = 0.f;
      if (never_ended && n < n1)
        e = logits_out[(static_cast<long>(b) * max_steps + (max_steps - 1)) * n1_stride + n] > end_logit ? 1.f : 0.f;
      extra_out[static_cast<long>(b) * kMaxN1 + n] = e;
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
  // APPLESTAR_SU_WIDE=0: the 256-thread kernel (A/B; read per call)
  const char* e = std::getenv("APPLESTAR_SU_WIDE");
  const bool wide = e == nullptr || e[0] != '0';
#define AS_SU(K, KT, NT)                                                                                             \
  hipLaunchKernelGGL((K<KT>), dim3(B), dim3(NT), 0, s, static_cast<const KT*>(key), key_bstride, c0, u, entity_num,  \
                     su_mask, wf, bf, wq2, bq2, wih, whh, lni_w, lni_b, lnh_w, lnh_b, lnc_w, lnc_b, we1, be1, inv_temp, \
                     eps, n1_stride, max_steps, extra_units, logits, results, logp, su_num, emb, extra)
  if (key_dt == DT_BF16) {
    if (wide) AS_SU(su_sample_wide_kernel, bf16_t, kWThreads);
    else AS_SU(su_sample_kernel, bf16_t, kThreads);
  } else {
    if (wide) AS_SU(su_sample_wide_kernel, float, kWThreads);
    else AS_SU(su_sample_kernel, float, kThreads);
  }
#undef AS_SU
}

}  // namespace as
