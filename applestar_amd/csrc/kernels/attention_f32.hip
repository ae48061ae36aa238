// Variable-length (packed) multi-head self-attention, fp32 operands end to end: the like-for-like path of
// the fp32 learner step (the reference computes the entity transformer's attention in fp32:
// distar/agent/default/model/module_utils.py:88-111).  gfx950 has no xf32/TF32 mode; the products run on
// the exact-f32 MFMA v_mfma_f32_16x16x4_f32 (A[l&15][k=l>>4], B[k=l>>4][l&15], C col = l&15,
// row = 4 (l>>4) + i), 1/16 of the bf16 rate, i.e. the f32 VALU peak with the VALU left free for softmax.
//
// Same decomposition as the bf16 kernels (attention.hip): one workgroup = (observation, head, 64-row
// block), four waves of 16 rows, online softmax in registers, LSE in the log2 domain, backward as two
// recomputing kernels (dQ + delta; dK/dV) with no atomics.  Products are computed transposed so the
// softmax row (or the key) sits on the lane: S^T = K Q^T leaves lane (lg, lr) holding row lr and keys
// 16 n + 4 lg + i; the k-slot -> key assignment of the next product is free, so k-step (n, i) takes
// keys {16 n + 4 lg + i} and P^T / dS^T feed the B operand from the lane's own registers.  For the
// products that reduce over the head dim, lane group lg owns dims 32 lg .. 32 lg + 31 (k-step j = dim
// 32 lg + j): the query / dO fragments are 32 registers loaded once, the K / V / Q / dO row fragments
// are contiguous float4 LDS reads.  LDS rows are padded to 132 floats and the two 32-float halves of
// every row with bit 3 set are swapped (dim d of row r at r * 132 + (d ^ 32 ((r >> 3) & 1))): with the pitch
// alone the float4 row reads of lane groups lg and lg ^ 1 collide 2-way (rows lr and lr + 8 land 32 banks
// apart), with the swap both the float4 row reads and the transposed one-float-per-lane reads are
// conflict-free (exhaustive check over the ds_read_b128 / b32 lane groups).  (A register prefetch of the next
// key block measured slower in the learner step: 64 more live VGPRs for sequences of 1-8 blocks, r3i.)
#include <cstdlib>
#include <string>

#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int D = 128;      // head dim
constexpr int BR = 64;      // rows / keys per block
constexpr int P = D + 4;    // LDS row pitch (floats)

__device__ __forceinline__ f4 mfma4(float a, float b, const f4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float xor_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float xor_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// swizzled LDS float offset of (row r, dim d); d a multiple of 4 keeps float4 groups intact
__device__ __forceinline__ int swz(int r, int d) { return r * P + (d ^ (((r >> 3) & 1) << 5)); }

// [64 x 128] fp32 tile rows r0.. (rows >= nvalid zero) from a row-strided global matrix into LDS T[64][P]
// (swizzled)
__device__ __forceinline__ void stage_tile(float* T, const float* __restrict__ base, long ld, int r0, int nvalid) {
  // the 8 contiguous lanes of a ds_write_b128 bank group take 8 rows of one 32-float column (row r at
  // 4 r mod 32: disjoint windows); four columns of two rows per group were 4-way conflicts
  const int t = threadIdx.x, r = (t & 7) + 8 * (t >> 5), c = (t >> 3) & 3;
  const bool ok = r0 + r < nvalid;
  const float4* src = reinterpret_cast<const float4*>(base + static_cast<long>(ok ? r0 + r : 0) * ld + 32 * c);
  float4 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 x = src[q];   // clamped row, unconditional load (a guarded one branches), zeroed by select
    v[q] = make_float4(ok ? x.x : 0.f, ok ? x.y : 0.f, ok ? x.z : 0.f, ok ? x.w : 0.f);
  }
  float* row = T + swz(r, 32 * c);
#pragma unroll
  for (int q = 0; q < 8; ++q) *reinterpret_cast<float4*>(row + 4 * q) = v[q];
}

// 32 consecutive floats of one row (this lane group's dims) -> registers
// (p must be a valid address even when !ok: callers clamp the row; the load is unconditional, the select zeroes)
__device__ __forceinline__ void load_row32(float (&f)[32], const float* __restrict__ p, bool ok) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = reinterpret_cast<const float4*>(p)[q];
    f[4 * q] = ok ? v.x : 0.f; f[4 * q + 1] = ok ? v.y : 0.f; f[4 * q + 2] = ok ? v.z : 0.f; f[4 * q + 3] = ok ? v.w : 0.f;
  }
}

// acc += (rows 16 n + lr of LDS tile T) . frag over the head dim (lane group lg: dims 32 lg + j)
__device__ __forceinline__ f4 row_dot(const float* T, int n, const float (&frag)[32], f4 acc) {
  const int l = threadIdx.x & 63;
  const float* row = T + swz(16 * n + (l & 15), 32 * (l >> 4));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 a = *reinterpret_cast<const float4*>(row + 4 * q);
    acc = mfma4(a.x, frag[4 * q], acc);
    acc = mfma4(a.y, frag[4 * q + 1], acc);
    acc = mfma4(a.z, frag[4 * q + 2], acc);
    acc = mfma4(a.w, frag[4 * q + 3], acc);
  }
  return acc;
}

// acc[nd] += T^T[16 nd + lr][keys of tile n] . regs (k-step i <-> key 16 n + 4 lg + i, B = this lane's C
// registers of tile n)
__device__ __forceinline__ void tr_accumulate(const float* T, int n, const f4& b, f4 (&acc)[8]) {
  const int l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
  // rows 16 n + 4 lg + i have bit 3 = lg >> 1: dim 16 nd + lr sits at 16 nd + lr +- 32 (swapped halves),
  // i.e. +32 for nd in {0, 1, 4, 5} and -32 for {2, 3, 6, 7}: two bases with compile-time offsets
  const int sw = (lg >> 1) << 5;
  const float* lo = T + (16 * n + 4 * lg) * P + lr + sw;
  const float* hi = T + (16 * n + 4 * lg) * P + lr - sw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int nd = 0; nd < 8; ++nd)
      acc[nd] = mfma4((nd & 2) ? hi[i * P + 16 * nd] : lo[i * P + 16 * nd], b[i], acc[nd]);
}

// ---- bf16x6 split-MFMA forms (split_mfma.h) on v_mfma_f32_16x16x32_bf16: A[l&15][k = 8 (l>>4) + t],
// B[k][l&15], the same C layout as the 16x16x4 f32 MFMA.  Fragments are split in registers.
__device__ __forceinline__ f4 mfma16_bf16(u32v4 a, u32v4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(a), as_bf(b), c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma16_x6(const Split3& a, const Split3& b, f4 c) {
  c = mfma16_bf16(a.p[1], b.p[1], c);
  c = mfma16_bf16(a.p[0], b.p[2], c);
  c = mfma16_bf16(a.p[2], b.p[0], c);
  c = mfma16_bf16(a.p[0], b.p[1], c);
  c = mfma16_bf16(a.p[1], b.p[0], c);
  return mfma16_bf16(a.p[0], b.p[0], c);
}

// the 32-float register fragment (dims 32 lg + j) as four split 8-float groups: group c = dims 32 lg + 8 c + t
__device__ __forceinline__ void split_frag(const float (&f)[32], Split3 (&fs)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) fs[c] = split8(*reinterpret_cast<const float(*)[8]>(&f[8 * c]));
}

// row_dot with split products: instruction c takes dims 32 lg + 8 c + t (k-slot t of lane group lg)
__device__ __forceinline__ f4 row_dot_x6(const float* T, int n, const Split3 (&fs)[4], f4 acc) {
  const int l = threadIdx.x & 63;
  const float* row = T + swz(16 * n + (l & 15), 32 * (l >> 4));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 a0 = *reinterpret_cast<const float4*>(row + 8 * c);
    const float4 a1 = *reinterpret_cast<const float4*>(row + 8 * c + 4);
    const float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    acc = mfma16_x6(split8(v), fs[c], acc);
  }
  return acc;
}

// row_dot_x6 with the register fragment split on the fly (fewer live VGPRs than a pre-split fragment)
__device__ __forceinline__ f4 row_dot_x6_raw(const float* T, int n, const float (&f)[32], f4 acc) {
  const int l = threadIdx.x & 63;
  const float* row = T + swz(16 * n + (l & 15), 32 * (l >> 4));
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float4 a0 = *reinterpret_cast<const float4*>(row + 8 * c);
    const float4 a1 = *reinterpret_cast<const float4*>(row + 8 * c + 4);
    const float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    acc = mfma16_x6(split8(v), split8(*reinterpret_cast<const float(*)[8]>(&f[8 * c])), acc);
  }
  return acc;
}

// tr_accumulate over the key tile pair (2 p, 2 p + 1) with split products: k-slot t of lane group lg is key
// 16 (2 p + (t >> 2)) + 4 lg + (t & 3); B = this lane's C registers of the two tiles
__device__ __forceinline__ void tr_accumulate_x6(const float* T, int p, const f4& b0, const f4& b1, f4 (&acc)[8]) {
  const int l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
  const int sw = (lg >> 1) << 5;
  const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  const Split3 sb = split8(bv);
#pragma unroll
  for (int nd = 0; nd < 8; ++nd) {
    float av[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int n = 2 * p + (t >> 2), i = t & 3;
      const float* lo = T + (16 * n + 4 * lg) * P + lr + sw;
      const float* hi = T + (16 * n + 4 * lg) * P + lr - sw;
      av[t] = (nd & 2) ? hi[i * P + 16 * nd] : lo[i * P + 16 * nd];
    }
    acc[nd] = mfma16_x6(split8(av), sb, acc[nd]);
  }
}

__device__ __forceinline__ bool attn_item(int QB, int S, int H, int& blk, int& s, int& h) {
  const int per = gridDim.x >> 3;
  const int u = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (u >= QB * S * H) return false;
  blk = u % QB;
  const int sh = u / QB;
  s = sh / H;
  h = sh - s * H;
  return true;
}

template <bool SPLIT>
__global__ __launch_bounds__(256) void attn_f32_fwd_kernel(const float* __restrict__ qkv, const int* __restrict__ cu,
                                                            float* __restrict__ out, float* __restrict__ lse2, int H,
                                                            long Ttot, float scale_log2, int QB, int S) {
  __shared__ __attribute__((aligned(16))) float K_s[BR * P];
  __shared__ __attribute__((aligned(16))) float V_s[BR * P];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const int qrow = qb * BR + w * 16 + lr;
  float qf[32];
  load_row32(qf, seq + static_cast<long>(qrow < len ? qrow : 0) * ROW + h * D + 32 * lg, qrow < len);
  Split3 qs[4];
  if constexpr (SPLIT) split_frag(qf, qs);
  f4 o[8];   // O^T: o[nd][i] = O[qrow][16 nd + 4 lg + i]
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, lsum = 0.f;
  const int nkb = (len + BR - 1) / BR;
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    stage_tile(K_s, seq + HD + h * D, ROW, kb * BR, len);
    stage_tile(V_s, seq + 2 * HD + h * D, ROW, kb * BR, len);
    __syncthreads();
    f4 st[4];   // S^T: st[n][i] = S[qrow][key kb*64 + 16 n + 4 lg + i]
#pragma unroll
    for (int n = 0; n < 4; ++n)
      st[n] = SPLIT ? row_dot_x6(K_s, n, qs, f4{0.f, 0.f, 0.f, 0.f}) : row_dot(K_s, n, qf, f4{0.f, 0.f, 0.f, 0.f});
    float mx = -1e30f;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = kb * BR + 16 * n + 4 * lg + i < len ? st[n][i] * scale_log2 : -1e30f;
        st[n][i] = v;
        mx = fmaxf(mx, v);
      }
    const float mn = fmaxf(m, xor_max(mx));
    const float alpha = ex2(m - mn);
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = ex2(st[n][i] - mn);
        st[n][i] = p;
        rs += p;
      }
    lsum = lsum * alpha + xor_sum(rs);
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha;
    if constexpr (SPLIT) {
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) tr_accumulate_x6(V_s, p2, st[2 * p2], st[2 * p2 + 1], o);
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) tr_accumulate(V_s, n, st[n], o);
    }
  }
  if (qrow < len) {
    const float inv = 1.f / lsum;
    float* dst = out + (static_cast<long>(start) + qrow) * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd)
      *reinterpret_cast<float4*>(dst + 16 * nd) = make_float4(o[nd][0] * inv, o[nd][1] * inv, o[nd][2] * inv,
                                                              o[nd][3] * inv);
    if (lg == 0) lse2[static_cast<long>(h) * Ttot + start + qrow] = m + log2f(lsum);
  }
}

// dQ (and delta = rowsum(dO * O)) for 64 rows; loops key blocks: S^T, dP^T, dS^T, dQ^T += K^T dS^T
template <bool SPLIT>
__global__ __launch_bounds__(256) void attn_f32_bwd_dq_kernel(const float* __restrict__ qkv, const float* __restrict__ o,
                                                               const float* __restrict__ dout,
                                                               const float* __restrict__ lse2, float* __restrict__ delta,
                                                               const int* __restrict__ cu, float* __restrict__ dqkv,
                                                               int H, long Ttot, float scale_log2, float scale, int QB,
                                                               int S) {
  __shared__ __attribute__((aligned(16))) float K_s[BR * P];
  __shared__ __attribute__((aligned(16))) float V_s[BR * P];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const float* dseq = dout + static_cast<long>(start) * HD;
  const int qrow = qb * BR + w * 16 + lr;
  const bool rval = qrow < len;
  const int qr = rval ? qrow : 0;
  float qf[32], df[32];
  load_row32(qf, seq + static_cast<long>(qr) * ROW + h * D + 32 * lg, rval);
  load_row32(df, dseq + static_cast<long>(qr) * HD + h * D + 32 * lg, rval);
  Split3 qs[4], ds[4];
  if constexpr (SPLIT) {
    split_frag(qf, qs);
    split_frag(df, ds);
  }
  const float ls = rval ? lse2[static_cast<long>(h) * Ttot + start + qrow] : 1e30f;
  float dl = 0.f;
  {
    const float4* orow = reinterpret_cast<const float4*>(o + (static_cast<long>(start) + qr) * HD + h * D + 32 * lg);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = orow[q];   // clamped row; df is zero when !rval
      dl += v.x * df[4 * q] + v.y * df[4 * q + 1] + v.z * df[4 * q + 2] + v.w * df[4 * q + 3];
    }
    dl = xor_sum(dl);
  }
  if (rval && lg == 0) delta[static_cast<long>(h) * Ttot + start + qrow] = dl;
  f4 dq[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) dq[n] = f4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (len + BR - 1) / BR;
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    stage_tile(K_s, seq + HD + h * D, ROW, kb * BR, len);
    stage_tile(V_s, seq + 2 * HD + h * D, ROW, kb * BR, len);
    __syncthreads();
    if constexpr (SPLIT) {
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        f4 dpp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int n = 2 * p2 + u;
          const f4 st = row_dot_x6(K_s, n, qs, f4{0.f, 0.f, 0.f, 0.f});
          f4 dpt = row_dot_x6(V_s, n, ds, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool kv = kb * BR + 16 * n + 4 * lg + i < len;
            const float p = kv ? ex2(st[i] * scale_log2 - ls) : 0.f;
            dpt[i] = p * (dpt[i] - dl);
          }
          dpp[u] = dpt;
        }
        tr_accumulate_x6(K_s, p2, dpp[0], dpp[1], dq);
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const f4 st = row_dot(K_s, n, qf, f4{0.f, 0.f, 0.f, 0.f});
        f4 dpt = row_dot(V_s, n, df, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool kv = kb * BR + 16 * n + 4 * lg + i < len;
          const float p = kv ? ex2(st[i] * scale_log2 - ls) : 0.f;
          dpt[i] = p * (dpt[i] - dl);
        }
        tr_accumulate(K_s, n, dpt, dq);
      }
    }
  }
  if (rval) {
    float* dqp = dqkv + (static_cast<long>(start) + qrow) * 3 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd)
      *reinterpret_cast<float4*>(dqp + 16 * nd) = make_float4(dq[nd][0] * scale, dq[nd][1] * scale,
                                                              dq[nd][2] * scale, dq[nd][3] * scale);
  }
}

// dK, dV for 64 keys; loops row blocks: S = Q K^T and dP = dO V^T leave lane (lg, lr) holding key lr and
// rows 16 n + 4 lg + i; dV^T += dO^T P, dK^T += Q^T dS take P / dS from registers
template <bool SPLIT>
__global__ __launch_bounds__(256, 2) void attn_f32_bwd_dkdv_kernel(const float* __restrict__ qkv,
                                                                 const float* __restrict__ dout,
                                                                 const float* __restrict__ lse2,
                                                                 const float* __restrict__ delta,
                                                                 const int* __restrict__ cu, float* __restrict__ dqkv,
                                                                 int H, long Ttot, float scale_log2, float scale,
                                                                 int QB, int S) {
  __shared__ __attribute__((aligned(16))) float Q_s[BR * P];
  __shared__ __attribute__((aligned(16))) float dO_s[BR * P];
  __shared__ float lse_s[BR], del_s[BR];
  int kb, s, h;
  if (!attn_item(QB, S, H, kb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (kb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const float* dseq = dout + static_cast<long>(start) * HD;
  const int key = kb * BR + w * 16 + lr;
  const bool kval = key < len;
  const int kr = kval ? key : 0;
  float kf[32], vf[32];
  load_row32(kf, seq + static_cast<long>(kr) * ROW + HD + h * D + 32 * lg, kval);
  load_row32(vf, seq + static_cast<long>(kr) * ROW + 2 * HD + h * D + 32 * lg, kval);
  f4 dk[8], dv[8];   // dK^T / dV^T: [nd][i] = d(key)[16 nd + 4 lg + i]
#pragma unroll
  for (int n = 0; n < 8; ++n) { dk[n] = f4{0.f, 0.f, 0.f, 0.f}; dv[n] = f4{0.f, 0.f, 0.f, 0.f}; }
  const int nrb = (len + BR - 1) / BR;
  for (int rb = 0; rb < nrb; ++rb) {
    if (rb) __syncthreads();
    stage_tile(Q_s, seq + h * D, ROW, rb * BR, len);
    stage_tile(dO_s, dseq + h * D, HD, rb * BR, len);
    if (tid < BR) {
      const int r = rb * BR + tid;
      lse_s[tid] = r < len ? lse2[static_cast<long>(h) * Ttot + start + r] : 1e30f;
      del_s[tid] = r < len ? delta[static_cast<long>(h) * Ttot + start + r] : 0.f;
    }
    __syncthreads();
    if constexpr (SPLIT) {
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        f4 scp[2], dpp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int n = 2 * p2 + u;
          f4 sc = row_dot_x6_raw(Q_s, n, kf, f4{0.f, 0.f, 0.f, 0.f});
          f4 dp = row_dot_x6_raw(dO_s, n, vf, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int rl = 16 * n + 4 * lg + i;
            const float p = kval ? ex2(sc[i] * scale_log2 - lse_s[rl]) : 0.f;
            sc[i] = p;
            dp[i] = p * (dp[i] - del_s[rl]);
          }
          scp[u] = sc;
          dpp[u] = dp;
        }
        tr_accumulate_x6(dO_s, p2, scp[0], scp[1], dv);
        tr_accumulate_x6(Q_s, p2, dpp[0], dpp[1], dk);
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        f4 sc = row_dot(Q_s, n, kf, f4{0.f, 0.f, 0.f, 0.f});     // [i]: row 16 n + 4 lg + i, key lr
        f4 dp = row_dot(dO_s, n, vf, f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = 16 * n + 4 * lg + i;
          const float p = kval ? ex2(sc[i] * scale_log2 - lse_s[rl]) : 0.f;   // padded rows: lse = +inf
          sc[i] = p;
          dp[i] = p * (dp[i] - del_s[rl]);
        }
        tr_accumulate(dO_s, n, sc, dv);
        tr_accumulate(Q_s, n, dp, dk);
      }
    }
  }
  if (kval) {
    const long tok = static_cast<long>(start) + key;
    float* dkp = dqkv + tok * 3 * HD + HD + h * D + 4 * lg;
    float* dvp = dqkv + tok * 3 * HD + 2 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      *reinterpret_cast<float4*>(dkp + 16 * nd) = make_float4(dk[nd][0] * scale, dk[nd][1] * scale,
                                                              dk[nd][2] * scale, dk[nd][3] * scale);
      *reinterpret_cast<float4*>(dvp + 16 * nd) = make_float4(dv[nd][0], dv[nd][1], dv[nd][2], dv[nd][3]);
    }
  }
}

// ---- pre-split LDS images (the default split path).  The kernels above split every operand they read from LDS
// in each of the four waves: a split8 is ~44 VALU instructions (~88 issue cycles) per six-MFMA group (96 cycles),
// so those loops are VALU-bound and the four waves redo the same work.  Here each 32-row block of K / V (or Q / dO)
// is split ONCE while it is staged: three bf16 planes of [32 rows][128 dims], 256-B rows with the 16-B chunk
// index XORed by f(row) = 2 (row & 7) | ((row >> 3) & 1).  The one image serves both operand forms:
//   row read   (A = rows 16 n + lr, k = dims 32 lg + 8 c + t): one ds_read_b128 per plane;
//   transposed (A = dims 16 nd + lr, k = rows 4 lg + t (t < 4) / 16 + 4 lg + t - 4): two ds_read_b64_tr_b16
//   per plane (CDNA4's transposing LDS read: lane 4 q + p of a 16-lane group addresses row q, columns 4 p ..
//   4 p + 3; lane i receives column i of the 4 rows).
// Bank check (tools/lds_bank_check.py model of the lane groups): row reads 1 LDS cycle per 16-lane group,
// transposed reads 1 per 32-lane half, the staging ds_write_b128 1 per 8-lane group - all conflict-free.
// 48 KB of images per workgroup (vs 66 KB of fp32 tiles), 32 keys / rows per block.
constexpr int IR = 32;               // rows per image block
constexpr int PLANE = IR * 256;      // bytes per bf16 plane
constexpr int IMG = 3 * PLANE;       // bytes per split image

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ int img_off(int r, int ch) { return 256 * r + 16 * (ch ^ ((2 * (r & 7)) | ((r >> 3) & 1))); }

// rows r0 .. r0 + 31 (>= nvalid: zero) of a row-strided fp32 matrix -> registers: thread t takes row t >> 3,
// chunks (t & 7) and (t & 7) + 8 (8 floats each)
__device__ __forceinline__ void img_load(float4 (&v)[4], const float* __restrict__ base, long ld, int r0, int nvalid) {
  // unconditional loads from a clamped row, zeroed by select: a guarded load compiles to an exec-masked branch
  // around four dword loads per float4
  const int t = threadIdx.x & 255, row = t >> 3, j = t & 7;
  const bool ok = r0 + row < nvalid;
  const float4* src = reinterpret_cast<const float4*>(base + static_cast<long>(ok ? r0 + row : 0) * ld + 8 * j);
  const int o[4] = {0, 1, 16, 17};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 x = src[o[i]];
    v[i] = make_float4(ok ? x.x : 0.f, ok ? x.y : 0.f, ok ? x.z : 0.f, ok ? x.w : 0.f);
  }
}

__device__ __forceinline__ void img_store(char* img, const float4 (&v)[4]) {
  const int t = threadIdx.x & 255, row = t >> 3, j = t & 7;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 a = v[2 * h], b = v[2 * h + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const Split3 s = split8(f);
    const int o = img_off(row, j + 8 * h);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32v4*>(img + pl * PLANE + o) = s.p[pl];
  }
}

// row operand: row r, dims 8 ch .. 8 ch + 7
__device__ __forceinline__ Split3 img_row(const char* img, int r, int ch) {
  const int o = img_off(r, ch);
  Split3 s;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) s.p[pl] = *reinterpret_cast<const u32v4*>(img + pl * PLANE + o);
  return s;
}

// transposed operand: A[dim 16 nd + lr][k = 8 lg + t] = image[row 4 lg + t (t < 4), 16 + 4 lg + t - 4][dim]
__device__ __forceinline__ Split3 img_tr(const char* img, int nd) {
  const int l = threadIdx.x & 63, lg = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const int ch = 2 * nd + (p >> 1), sub = 8 * (p & 1);
  const int o1 = img_off(4 * lg + q, ch) + sub, o2 = img_off(16 + 4 * lg + q, ch) + sub;
  Split3 s;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + pl * PLANE + o1));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + pl * PLANE + o2));
    const uint2 a = __builtin_bit_cast(uint2, lo), b = __builtin_bit_cast(uint2, hi);
    s.p[pl] = u32v4{a.x, a.y, b.x, b.y};
  }
  return s;
}

// C registers of two 16-row tiles (rows 4 lg + i and 16 + 4 lg + i of the block) -> split B operand whose k-slot
// t matches img_tr's row order
__device__ __forceinline__ Split3 split_pair_regs(const f4& b0, const f4& b1) {
  const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  return split8(bv);
}

// (16-row tile n of the image) . (split register fragment) over the head dim
__device__ __forceinline__ f4 img_row_dot(const char* img, int n, const Split3 (&fs)[4]) {
  const int l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) acc = mfma16_x6(img_row(img, 16 * n + lr, 4 * lg + c), fs[c], acc);
  return acc;
}

// img_row_dot with the register fragment split on the fly (32 live VGPRs instead of 48)
__device__ __forceinline__ f4 img_row_dot_raw(const char* img, int n, const float (&f)[32]) {
  const int l = threadIdx.x & 63, lr = l & 15, lg = l >> 4;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c)
    acc = mfma16_x6(img_row(img, 16 * n + lr, 4 * lg + c), split8(*reinterpret_cast<const float(*)[8]>(&f[8 * c])), acc);
  return acc;
}

template <bool PF, int OCC>
__global__ __launch_bounds__(256, OCC) void attn_f32_fwd_img_kernel(const float* __restrict__ qkv, const int* __restrict__ cu,
                                                                float* __restrict__ out, float* __restrict__ lse2,
                                                                int H, long Ttot, float scale_log2, int QB, int S) {
  __shared__ __attribute__((aligned(16))) char K_i[IMG];
  __shared__ __attribute__((aligned(16))) char V_i[IMG];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const int qrow = qb * BR + w * 16 + lr;
  Split3 qs[4];
  {
    float qf[32];
    load_row32(qf, seq + static_cast<long>(qrow < len ? qrow : 0) * ROW + h * D + 32 * lg, qrow < len);
    split_frag(qf, qs);
  }
  f4 o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, lsum = 0.f;
  const int nkb = (len + IR - 1) / IR;
  float4 kr[4], vr[4];
  img_load(kr, seq + HD + h * D, ROW, 0, len);
  img_load(vr, seq + 2 * HD + h * D, ROW, 0, len);
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    if (!PF && kb) {
      img_load(kr, seq + HD + h * D, ROW, kb * IR, len);
      img_load(vr, seq + 2 * HD + h * D, ROW, kb * IR, len);
    }
    img_store(K_i, kr);
    img_store(V_i, vr);
    __syncthreads();
    if (PF && kb + 1 < nkb) {
      img_load(kr, seq + HD + h * D, ROW, (kb + 1) * IR, len);
      img_load(vr, seq + 2 * HD + h * D, ROW, (kb + 1) * IR, len);
    }
    f4 st[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) st[n] = img_row_dot(K_i, n, qs);
    float mx = -1e30f;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = kb * IR + 16 * n + 4 * lg + i < len ? st[n][i] * scale_log2 : -1e30f;
        st[n][i] = v;
        mx = fmaxf(mx, v);
      }
    const float mn = fmaxf(m, xor_max(mx));
    const float alpha = ex2(m - mn);
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = ex2(st[n][i] - mn);
        st[n][i] = p;
        rs += p;
      }
    lsum = lsum * alpha + xor_sum(rs);
    const Split3 sp = split_pair_regs(st[0], st[1]);
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[nd][i] *= alpha;
      o[nd] = mfma16_x6(img_tr(V_i, nd), sp, o[nd]);
    }
  }
  if (qrow < len) {
    const float inv = 1.f / lsum;
    float* dst = out + (static_cast<long>(start) + qrow) * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd)
      *reinterpret_cast<float4*>(dst + 16 * nd) = make_float4(o[nd][0] * inv, o[nd][1] * inv, o[nd][2] * inv,
                                                              o[nd][3] * inv);
    if (lg == 0) lse2[static_cast<long>(h) * Ttot + start + qrow] = m + log2f(lsum);
  }
}

template <bool PF>
__global__ __launch_bounds__(256, 2) void attn_f32_bwd_dq_img_kernel(
    const float* __restrict__ qkv, const float* __restrict__ o, const float* __restrict__ dout,
    const float* __restrict__ lse2, float* __restrict__ delta, const int* __restrict__ cu, float* __restrict__ dqkv,
    int H, long Ttot, float scale_log2, float scale, int QB, int S) {
  __shared__ __attribute__((aligned(16))) char K_i[IMG];
  __shared__ __attribute__((aligned(16))) char V_i[IMG];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const float* dseq = dout + static_cast<long>(start) * HD;
  const int qrow = qb * BR + w * 16 + lr;
  const bool rval = qrow < len;
  const int qr = rval ? qrow : 0;
  Split3 qs[4], ds[4];
  float dl = 0.f;
  {
    float qf[32], df[32];
    load_row32(qf, seq + static_cast<long>(qr) * ROW + h * D + 32 * lg, rval);
    load_row32(df, dseq + static_cast<long>(qr) * HD + h * D + 32 * lg, rval);
    const float4* orow = reinterpret_cast<const float4*>(o + (static_cast<long>(start) + qr) * HD + h * D + 32 * lg);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = orow[q];   // clamped row; df is zero when !rval
      dl += v.x * df[4 * q] + v.y * df[4 * q + 1] + v.z * df[4 * q + 2] + v.w * df[4 * q + 3];
    }
    dl = xor_sum(dl);
    split_frag(qf, qs);
    split_frag(df, ds);
  }
  const float ls = rval ? lse2[static_cast<long>(h) * Ttot + start + qrow] : 1e30f;
  if (rval && lg == 0) delta[static_cast<long>(h) * Ttot + start + qrow] = dl;
  f4 dq[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) dq[n] = f4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (len + IR - 1) / IR;
  float4 kr[4], vr[4];
  img_load(kr, seq + HD + h * D, ROW, 0, len);
  img_load(vr, seq + 2 * HD + h * D, ROW, 0, len);
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    if (!PF && kb) {
      img_load(kr, seq + HD + h * D, ROW, kb * IR, len);
      img_load(vr, seq + 2 * HD + h * D, ROW, kb * IR, len);
    }
    img_store(K_i, kr);
    img_store(V_i, vr);
    __syncthreads();
    if (PF && kb + 1 < nkb) {
      img_load(kr, seq + HD + h * D, ROW, (kb + 1) * IR, len);
      img_load(vr, seq + 2 * HD + h * D, ROW, (kb + 1) * IR, len);
    }
    f4 dpp[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const f4 st = img_row_dot(K_i, n, qs);
      f4 dpt = img_row_dot(V_i, n, ds);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool kv = kb * IR + 16 * n + 4 * lg + i < len;
        const float p = kv ? ex2(st[i] * scale_log2 - ls) : 0.f;
        dpt[i] = p * (dpt[i] - dl);
      }
      dpp[n] = dpt;
    }
    const Split3 sd = split_pair_regs(dpp[0], dpp[1]);
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) dq[nd] = mfma16_x6(img_tr(K_i, nd), sd, dq[nd]);
  }
  if (rval) {
    float* dqp = dqkv + (static_cast<long>(start) + qrow) * 3 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd)
      *reinterpret_cast<float4*>(dqp + 16 * nd) = make_float4(dq[nd][0] * scale, dq[nd][1] * scale,
                                                              dq[nd][2] * scale, dq[nd][3] * scale);
  }
}

template <bool PF, bool RAWV>
__global__ __launch_bounds__(256, 2) void attn_f32_bwd_dkdv_img_kernel(
    const float* __restrict__ qkv, const float* __restrict__ dout, const float* __restrict__ lse2,
    const float* __restrict__ delta, const int* __restrict__ cu, float* __restrict__ dqkv, int H, long Ttot,
    float scale_log2, float scale, int QB, int S) {
  __shared__ __attribute__((aligned(16))) char Q_i[IMG];
  __shared__ __attribute__((aligned(16))) char O_i[IMG];
  __shared__ float lse_s[IR], del_s[IR];
  int kb, s, h;
  if (!attn_item(QB, S, H, kb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (kb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const float* seq = qkv + static_cast<long>(start) * ROW;
  const float* dseq = dout + static_cast<long>(start) * HD;
  const int key = kb * BR + w * 16 + lr;
  const bool kval = key < len;
  const int kr0 = kval ? key : 0;
  // K fragment pre-split; V pre-split too when registers allow (RAWV: split on the fly, 16 fewer VGPRs)
  Split3 ks[4], vs[RAWV ? 1 : 4];
  float vf[32];
  {
    float kf[32];
    load_row32(kf, seq + static_cast<long>(kr0) * ROW + HD + h * D + 32 * lg, kval);
    load_row32(vf, seq + static_cast<long>(kr0) * ROW + 2 * HD + h * D + 32 * lg, kval);
    split_frag(kf, ks);
    if constexpr (!RAWV) split_frag(vf, *reinterpret_cast<Split3(*)[4]>(vs));
  }
  f4 dk[8], dv[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) { dk[n] = f4{0.f, 0.f, 0.f, 0.f}; dv[n] = f4{0.f, 0.f, 0.f, 0.f}; }
  const int nrb = (len + IR - 1) / IR;
  float4 qr[4], orr[4];
  float lse_r = 1e30f, del_r = 0.f;
  auto load_block = [&](int rb) {
    img_load(qr, seq + h * D, ROW, rb * IR, len);
    img_load(orr, dseq + h * D, HD, rb * IR, len);
    if (tid < IR) {
      const int r = rb * IR + tid;
      lse_r = r < len ? lse2[static_cast<long>(h) * Ttot + start + r] : 1e30f;
      del_r = r < len ? delta[static_cast<long>(h) * Ttot + start + r] : 0.f;
    }
  };
  load_block(0);
  for (int rb = 0; rb < nrb; ++rb) {
    if (rb) __syncthreads();
    if (!PF && rb) load_block(rb);
    img_store(Q_i, qr);
    img_store(O_i, orr);
    if (tid < IR) {
      lse_s[tid] = lse_r;
      del_s[tid] = del_r;
    }
    __syncthreads();
    if (PF && rb + 1 < nrb) load_block(rb + 1);
    f4 scp[2], dpp[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      f4 sc = img_row_dot(Q_i, n, ks);     // [i]: row 16 n + 4 lg + i, key lr
      f4 dp;
      if constexpr (RAWV) dp = img_row_dot_raw(O_i, n, vf);
      else dp = img_row_dot(O_i, n, *reinterpret_cast<const Split3(*)[4]>(vs));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 16 * n + 4 * lg + i;
        const float p = kval ? ex2(sc[i] * scale_log2 - lse_s[rl]) : 0.f;   // padded rows: lse = +inf
        sc[i] = p;
        dp[i] = p * (dp[i] - del_s[rl]);
      }
      scp[n] = sc;
      dpp[n] = dp;
    }
    const Split3 sp = split_pair_regs(scp[0], scp[1]);
    const Split3 sd = split_pair_regs(dpp[0], dpp[1]);
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      dv[nd] = mfma16_x6(img_tr(O_i, nd), sp, dv[nd]);
      dk[nd] = mfma16_x6(img_tr(Q_i, nd), sd, dk[nd]);
    }
  }
  if (kval) {
    const long tok = static_cast<long>(start) + key;
    float* dkp = dqkv + tok * 3 * HD + HD + h * D + 4 * lg;
    float* dvp = dqkv + tok * 3 * HD + 2 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      *reinterpret_cast<float4*>(dkp + 16 * nd) = make_float4(dk[nd][0] * scale, dk[nd][1] * scale,
                                                              dk[nd][2] * scale, dk[nd][3] * scale);
      *reinterpret_cast<float4*>(dvp + 16 * nd) = make_float4(dv[nd][0], dv[nd][1], dv[nd][2], dv[nd][3]);
    }
  }
}

}  // namespace

// split-path variant (APPLESTAR_F32_ATTN_IMG, or attn_f32_variant() at run time).  Default 23 = images, forward at
// 3 waves / SIMD without prefetch, dK/dV with V pre-split: at the learner's shape (384 sequences of 1-512, 2 heads)
// forward 516 -> 303 us, backward 1464 -> 1002 us against the per-wave split (0) (profiles/r4z_attn_f32_img.txt).
// bit 0 = pre-split images (else
// the per-wave split kernels above); bit 1 = forward at 3 waves / SIMD (168 VGPRs, spills); bit 2 = forward without
// the register prefetch of the next block; bit 3 = dQ without it; bit 4 = dK/dV with the V fragment pre-split
// (spills at 256 VGPRs; default: split on the fly).  Measured and removed: dK / dV with each 16-key slice on a
// wave PAIR (8 waves: one holds the K fragment, computes P, accumulates dV; the other the V fragment, dP -> dS, dK;
// P through LDS): 162 VGPRs, 1161 us backward (1378 us held to 128 VGPRs, 200 B spilled) vs 1001 us.
static int g_attn_variant = [] {
  const char* e = std::getenv("APPLESTAR_F32_ATTN_IMG");
  return e ? std::atoi(e) : 23;
}();

int attn_f32_variant(int v) {
  const int old = g_attn_variant;
  if (v >= 0) g_attn_variant = v;
  return old;
}

namespace {

}  // namespace

void varlen_attn_fwd_f32(const float* qkv, const int* cu, float* out, float* lse2, int S, int max_len, int H, long Ttot,
                         float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const int QB = (max_len + BR - 1) / BR;
  const dim3 grid(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
  const int v = g_attn_variant;
  if (f32_mfma_mode() && (v & 1)) {
    auto k = (v & 2) ? ((v & 4) ? attn_f32_fwd_img_kernel<false, 3> : attn_f32_fwd_img_kernel<true, 3>)
                     : ((v & 4) ? attn_f32_fwd_img_kernel<false, 2> : attn_f32_fwd_img_kernel<true, 2>);
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, qkv, cu, out, lse2, H, Ttot, scale_log2, QB, S);
  } else if (f32_mfma_mode())
    hipLaunchKernelGGL(attn_f32_fwd_kernel<true>, grid, dim3(256), 0, s, qkv, cu, out, lse2, H, Ttot, scale_log2, QB, S);
  else
    hipLaunchKernelGGL(attn_f32_fwd_kernel<false>, grid, dim3(256), 0, s, qkv, cu, out, lse2, H, Ttot, scale_log2, QB, S);
}

void varlen_attn_bwd_f32(const float* qkv, const float* out, const float* dout, const float* lse2, const int* cu,
                         float* dqkv, float* delta, int S, int max_len, int H, long Ttot, float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const int QB = (max_len + BR - 1) / BR;
  const dim3 grid(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
  // split backward (profiles/r3z_attn_bwd_variants.txt): exact 1933 us, dQ split 1809, both split 1636 with dK/dV
  // held to two waves per SIMD (its K / V fragments split on the fly; at 276 VGPRs, one workgroup per CU, it was
  // slower than exact).  APPLESTAR_F32_ATTN_BWD_SPLIT = both (default) | dq | none
  static const int bwd_split = [] {
    const char* e = std::getenv("APPLESTAR_F32_ATTN_BWD_SPLIT");
    const std::string v = e ? e : "both";
    return v == "both" ? 3 : (v == "none" ? 0 : 1);
  }();
  const bool sq = f32_mfma_mode() && (bwd_split & 1), skv = f32_mfma_mode() && (bwd_split & 2);
  if (f32_mfma_mode() && (g_attn_variant & 1)) {
    auto kq = (g_attn_variant & 8) ? attn_f32_bwd_dq_img_kernel<false> : attn_f32_bwd_dq_img_kernel<true>;
    hipLaunchKernelGGL(kq, grid, dim3(256), 0, s, qkv, out, dout, lse2, delta, cu, dqkv, H,
                       Ttot, scale_log2, scale, QB, S);
    auto kk = (g_attn_variant & 16) ? attn_f32_bwd_dkdv_img_kernel<false, false> : attn_f32_bwd_dkdv_img_kernel<false, true>;
    hipLaunchKernelGGL(kk, grid, dim3(256), 0, s, qkv, dout, lse2, delta, cu, dqkv, H, Ttot,
                       scale_log2, scale, QB, S);
    return;
  }
  if (sq)
    hipLaunchKernelGGL(attn_f32_bwd_dq_kernel<true>, grid, dim3(256), 0, s, qkv, out, dout, lse2, delta, cu, dqkv, H,
                       Ttot, scale_log2, scale, QB, S);
  else
    hipLaunchKernelGGL(attn_f32_bwd_dq_kernel<false>, grid, dim3(256), 0, s, qkv, out, dout, lse2, delta, cu, dqkv, H,
                       Ttot, scale_log2, scale, QB, S);
  if (skv)
    hipLaunchKernelGGL(attn_f32_bwd_dkdv_kernel<true>, grid, dim3(256), 0, s, qkv, dout, lse2, delta, cu, dqkv, H, Ttot,
                       scale_log2, scale, QB, S);
  else
    hipLaunchKernelGGL(attn_f32_bwd_dkdv_kernel<false>, grid, dim3(256), 0, s, qkv, dout, lse2, delta, cu, dqkv, H,
                       Ttot, scale_log2, scale, QB, S);
}

}  // namespace as
