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
  for (int q = 0; q < 8; ++q) v[q] = ok ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  float* row = T + swz(r, 32 * c);
#pragma unroll
  for (int q = 0; q < 8; ++q) *reinterpret_cast<float4*>(row + 4 * q) = v[q];
}

// 32 consecutive floats of one row (this lane group's dims) -> registers
__device__ __forceinline__ void load_row32(float (&f)[32], const float* __restrict__ p, bool ok) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = ok ? reinterpret_cast<const float4*>(p)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
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
      const float4 v = rval ? orow[q] : make_float4(0.f, 0.f, 0.f, 0.f);
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

}  // namespace

void varlen_attn_fwd_f32(const float* qkv, const int* cu, float* out, float* lse2, int S, int max_len, int H, long Ttot,
                         float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const int QB = (max_len + BR - 1) / BR;
  const dim3 grid(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
  if (f32_mfma_mode())
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
