// Fused sampling tails of the autoregressive action heads for actor inference:
//
//   head_sample : per row, scale the logits by 1/T, apply the head's mask (a shared [C] mask such as the
//                 action-type race mask, or a per-row length such as entity_num), draw the action by inverse CDF
//                 of softmax with the given uniform u, and gather its embedding relu(W^T[a] + b) (the
//                 "one-hot @ fc1" of action_type_head.py:61-64 / action_arg_head.py:55-60, 84-86 as a row
//                 gather).  Replaces softmax + cumsum + searchsorted + clamp + index_select + add + relu.
//   target_unit : TargetUnitHead (action_arg_head.py:343-363) in one kernel per row: query MLP 1024 -> 32
//                 (ReLU) -> 32, dot with the entity keys, length mask, 1/T, inverse-CDF sample.
//
// One 256-thread workgroup per batch row.  Sampling: m = max, p_i = exp(l_i - m), every thread sums a
// contiguous segment of p, a block-wide exclusive scan of the segment sums locates the segment holding
// u * sum p, and that thread walks its segment for the first index whose running sum exceeds the target
// (torch.searchsorted(cumsum(softmax), u * total, right=True) up to summation order).  Fully masked rows
// (impossible for valid observations) return the last index, like the clamped reference.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kHT = 256;
constexpr float kNeg = -1e9f;

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i) { return Cvt<T>::load(p, i); }

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return v;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return v;
}

// inverse-CDF draw over row[0..C) (already scaled / masked, fp32 in `row`: LDS when it fits): returns the index on
// every thread.  Segment sums are scanned per wave (shuffles) and across the 4 waves through LDS - one barrier where
// the Hillis-Steele LDS scan took 16.
__device__ __forceinline__ int sample_row(const float* __restrict__ row, int C, float u, float* red, float* scan) {
  float mx = kNeg * 2.f;
  for (int i = threadIdx.x; i < C; i += kHT) mx = fmaxf(mx, row[i]);
  mx = block_max(mx, red);
  const int seg = (C + kHT - 1) / kHT;
  const int s0 = threadIdx.x * seg, s1 = min(C, s0 + seg);
  float part = 0.f;
  for (int i = s0; i < s1; ++i) part += __expf(row[i] - mx);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float incl = part;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += y;
  }
  float excl = __shfl_up(incl, 1, kWave);   // the neighbour's inclusive value exactly: no gap / overlap by rounding
  if (lane == 0) excl = 0.f;
  if (lane == 63) scan[wv] = incl;
  __shared__ int pick;
  if (threadIdx.x == 0) pick = C - 1;
  __syncthreads();
  float woff = 0.f;
  for (int w = 0; w < wv; ++w) woff += scan[w];
  const float total = scan[0] + scan[1] + scan[2] + scan[3];
  const float target = u * total;
  incl += woff;
  const float before = excl + woff;
  if (s0 < s1 && incl > target && before <= target) {
    float run = before;
    int idx = s1 - 1;
    for (int i = s0; i < s1; ++i) {
      run += __expf(row[i] - mx);
      if (run > target) { idx = i; break; }
    }
    atomicMin(&pick, idx);
  }
  __syncthreads();
  const int r = pick;
  __syncthreads();
  return r;
}

constexpr int kRowLds = 24576;   // rows up to this many logits are staged in LDS (the location head's 24,320)

template <typename TL, typename TW>
__global__ __launch_bounds__(kHT) void head_sample_kernel(const TL* __restrict__ logits, long ld_logits, int C,
                                                          float inv_t, const uint8_t* __restrict__ mask, long mask_ld,
                                                          const int64_t* __restrict__ lens, const float* __restrict__ u,
                                                          const TW* __restrict__ table, const float* __restrict__ tbias,
                                                          int D, float* __restrict__ out_logits,
                                                          int64_t* __restrict__ action, float* __restrict__ emb) {
  __shared__ float red[4];
  __shared__ float scan[4];
  __shared__ float srow[kRowLds];
  const int b = blockIdx.x;
  const long len = lens ? lens[b] : C;
  float* row = out_logits + static_cast<long>(b) * C;
  const bool lds = C <= kRowLds;
  // 8 independent loads in flight per thread before any store (the 24,320-wide location row is 95 loads per thread:
  // one at a time, the workgroup waited on memory 75 % of its cycles, profiles/r7c_pmc_inf_b1_a_summary.txt)
  constexpr int kU = 8;
  for (int i0 = threadIdx.x; i0 < C; i0 += kHT * kU) {
    float v[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const int i = i0 + j * kHT;
      v[j] = i < C ? ld(logits, static_cast<long>(b) * ld_logits + i) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const int i = i0 + j * kHT;
      if (i < C) {
        float x = v[j] * inv_t;
        if ((mask && !mask[static_cast<long>(b) * mask_ld + i]) || i >= len) x = kNeg;
        row[i] = x;
        if (lds) srow[i] = x;
      }
    }
  }
  __syncthreads();
  const int a = lds ? sample_row(srow, C, u[b], red, scan) : sample_row(row, C, u[b], red, scan);
  if (threadIdx.x == 0) action[b] = a;
  if (table) {
    for (int d = threadIdx.x; d < D; d += kHT)
      emb[static_cast<long>(b) * D + d] = fmaxf(ld(table, static_cast<long>(a) * D + d) + tbias[d], 0.f);
  }
}

template <typename TE, typename TK>
__global__ __launch_bounds__(kHT) void target_unit_kernel(const TE* __restrict__ e, const float* __restrict__ w1,
                                                          const float* __restrict__ b1, const float* __restrict__ w2,
                                                          const float* __restrict__ b2, const TK* __restrict__ key,
                                                          int N, const int64_t* __restrict__ lens, float inv_t,
                                                          const float* __restrict__ u, float* __restrict__ out_logits,
                                                          int64_t* __restrict__ action, bool w1_vec) {
  constexpr int IN = 1024, KD = 32;
  __shared__ float red[4];
  __shared__ float scan[kHT];
  __shared__ float q1[KD], q[KD];
  const int b = blockIdx.x;
  // q1 = relu(W1 e + b1): 8 threads per output, 128 inputs each
  {
    const int o = threadIdx.x >> 3, part = threadIdx.x & 7;
    float s = 0.f;
    const TE* er = e + static_cast<long>(b) * IN;
    if (w1_vec) {
      // 16-B rows: the 8 lanes of an output read 128 contiguous bytes per load, 32 loads per thread (the scalar loop
      // below is 128 loads whose wave-wide footprint is 8 scattered 32-B pieces each)
      const float4* w4 = reinterpret_cast<const float4*>(w1 + o * IN);
#pragma unroll 4
      for (int k = part; k < IN / 4; k += 8) {
        const float4 w = w4[k];
        s += w.x * ld(er, 4 * k) + w.y * ld(er, 4 * k + 1) + w.z * ld(er, 4 * k + 2) + w.w * ld(er, 4 * k + 3);
      }
    } else {
      for (int i = part; i < IN; i += 8) s += w1[o * IN + i] * ld(er, i);
    }
    s += __shfl_xor(s, 1, kWave);
    s += __shfl_xor(s, 2, kWave);
    s += __shfl_xor(s, 4, kWave);
    if (part == 0) q1[o] = fmaxf(s + b1[o], 0.f);
  }
  __syncthreads();
  if (threadIdx.x < KD) {
    float s = b2[threadIdx.x];
    for (int i = 0; i < KD; ++i) s += w2[threadIdx.x * KD + i] * q1[i];
    q[threadIdx.x] = s;
  }
  __syncthreads();
  const long len = lens[b];
  float* row = out_logits + static_cast<long>(b) * N;
  for (int n = threadIdx.x; n < N; n += kHT) {
    float s = 0.f;
    const TK* kr = key + (static_cast<long>(b) * N + n) * KD;
#pragma unroll
    for (int c = 0; c < KD; ++c) s += q[c] * ld(kr, c);
    row[n] = n < len ? s * inv_t : kNeg;
  }
  __syncthreads();
  const int a = sample_row(row, N, u[b], red, scan);
  if (threadIdx.x == 0) action[b] = a;
}

}  // namespace

void head_sample(const void* logits, int logits_dt, long ld_logits, int B, int C, float inv_t, const uint8_t* mask,
                 long mask_ld, const int64_t* lens, const float* u, const void* table, int table_dt,
                 const float* tbias, int D, float* out_logits, int64_t* action, float* emb, hipStream_t s) {
  if (B <= 0) return;
#define AS_HS(TL, TW)                                                                                            \
  hipLaunchKernelGGL((head_sample_kernel<TL, TW>), dim3(B), dim3(kHT), 0, s, static_cast<const TL*>(logits),      \
                     ld_logits, C, inv_t, mask, mask_ld, lens, u, static_cast<const TW*>(table), tbias, D,        \
                     out_logits, action, emb)
  if (logits_dt == DT_BF16) {
    if (table_dt == DT_BF16) AS_HS(bf16_t, bf16_t); else AS_HS(bf16_t, float);
  } else {
    if (table_dt == DT_BF16) AS_HS(float, bf16_t); else AS_HS(float, float);
  }
#undef AS_HS
}

void target_unit_sample(const void* e, int e_dt, const float* w1, const float* b1, const float* w2, const float* b2,
                        const void* key, int key_dt, int B, int N, const int64_t* lens, float inv_t, const float* u,
                        float* out_logits, int64_t* action, hipStream_t s) {
  if (B <= 0) return;
#define AS_TU(TE, TK)                                                                                             \
  hipLaunchKernelGGL((target_unit_kernel<TE, TK>), dim3(B), dim3(kHT), 0, s, static_cast<const TE*>(e), w1, b1, w2, \
                     b2, static_cast<const TK*>(key), N, lens, inv_t, u, out_logits, action, w1_vec)
  const bool w1_vec = (reinterpret_cast<uintptr_t>(w1) & 15) == 0;
  if (e_dt == DT_BF16) {
    if (key_dt == DT_BF16) AS_TU(bf16_t, bf16_t); else AS_TU(bf16_t, float);
  } else {
    if (key_dt == DT_BF16) AS_TU(float, bf16_t); else AS_TU(float, float);
  }
#undef AS_TU
}


namespace {
// one wave per row of any head: row max, sum of exp, the taken action's logit
// (m, s) pairs of an online log-sum-exp: s = sum exp(x - m)
__device__ __forceinline__ void lse_merge(float& m, float& s, float om, float os) {
  const float nm = fmaxf(m, om);
  if (nm == -INFINITY) return;
  s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
  m = nm;
}

// Narrow heads: one wave per row, 4 rows per workgroup.  Wide heads (the location head's 24,320 logits per row):
// a whole workgroup per row - one wave per row walked 380 dependent-latency loads per lane twice (~0.4 ms at B = 1).
// Single pass: an online log-sum-exp per thread, 4 loads in flight, then wave and workgroup merges.
__global__ __launch_bounds__(256) void multi_logp_kernel(const LogpArgs a) {
  __shared__ float red_m[4], red_s[4];
  const long blk = blockIdx.x;
  if (blk >= a.blk_start[a.nheads]) return;
  int h = 0;
  while (h + 1 < a.nheads && a.blk_start[h + 1] <= blk) ++h;
  const long rows_h = a.row_start[h + 1] - a.row_start[h];
  const bool big = a.big[h] != 0;
  const long r = big ? blk - a.blk_start[h] : (blk - a.blk_start[h]) * 4 + (threadIdx.x >> 6);
  if (!big && r >= rows_h) return;          // whole waves (the wide path below keeps every wave)
  const int C = a.cols[h], lane = threadIdx.x & 63;
  const int t = big ? static_cast<int>(threadIdx.x) : lane, nt = big ? 256 : 64;
  const bool b16 = a.bf16[h] != 0;
  auto ld = [&](long i) {
    return b16 ? bf2f(static_cast<const bf16_t*>(a.logits[h])[i]) : static_cast<const float*>(a.logits[h])[i];
  };
  const long base = r * C;
  float m = -INFINITY, s = 0.f;
  int c = t;
  for (; c + 3 * nt < C; c += 4 * nt) {
    const float x0 = ld(base + c), x1 = ld(base + c + nt), x2 = ld(base + c + 2 * nt), x3 = ld(base + c + 3 * nt);
    const float xm = fmaxf(fmaxf(x0, x1), fmaxf(x2, x3));
    const float nm = fmaxf(m, xm);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + __expf(x0 - nm) + __expf(x1 - nm) + __expf(x2 - nm) +
        __expf(x3 - nm);
    m = nm;
  }
  for (; c < C; c += nt) lse_merge(m, s, ld(base + c), 1.f);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, kWave), __shfl_xor(s, o, kWave));
  if (big) {
    if (lane == 0) { red_m[threadIdx.x >> 6] = m; red_s[threadIdx.x >> 6] = s; }
    __syncthreads();
    if (threadIdx.x != 0) return;
    m = red_m[0];
    s = red_s[0];
    for (int w = 1; w < 4; ++w) lse_merge(m, s, red_m[w], red_s[w]);
  } else if (lane != 0) {
    return;
  }
  long act = a.action[h][r];
  act = act < 0 ? 0 : (act >= C ? C - 1 : act);
  a.out[h][r] = ld(base + act) - m - __logf(s);
}
}  // namespace

void multi_logp(const LogpArgs& args, hipStream_t s) {
  LogpArgs a = args;
  a.blk_start[0] = 0;
  for (int h = 0; h < a.nheads; ++h) {
    const long rows = a.row_start[h + 1] - a.row_start[h];
    a.big[h] = a.cols[h] >= 4096 ? 1 : 0;
    a.blk_start[h + 1] = a.blk_start[h] + (a.big[h] ? rows : (rows + 3) / 4);
  }
  if (a.blk_start[a.nheads] > 0)
    hipLaunchKernelGGL(multi_logp_kernel, dim3(static_cast<unsigned>(a.blk_start[a.nheads])), dim3(256), 0, s, a);
}

}  // namespace as
