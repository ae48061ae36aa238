// Variable-length (packed) multi-head self-attention for the entity transformer, forward and
// backward, bf16 MFMA (v_mfma_f32_16x16x32_bf16) with fp32 softmax state.  gfx950.
//
// The reference materialises [B, 2, N, N] fp32 scores over the zero-padded entity batch and masks
// padded keys with -1e9 (module_utils.py:88-111).  Here entities of all observations are packed
// ([T_total, 3*H*D] rows = q | k | v, cu_seqlens delimits each observation) and one workgroup owns
// one (observation, head, 64-row block): only real entities are touched, scores never leave
// registers (online softmax, flash style), and the key mask becomes the loop bound.
// Backward = two kernels with recomputation (no atomics, deterministic):
//   attn_bwd_dq   : per 64-row block (also emits delta = rowsum(dO * O)), loops key blocks:
//                   S^T, dP^T, dS^T, dQ^T += K^T dS^T
//   attn_bwd_dkdv : per 64-key block, loops row blocks: S, dP, dV^T += dO^T P, dK^T += Q^T dS
// LSE is stored in the log2 domain (lse2 = m + log2(l) of scale*log2(e)-scaled scores).
// r2: the first generation (scores in the C layout, P / dS bounced through LDS, V / Q / dO staged
// transposed by scalar LDS writes, three barriers per tile) measured fwd 253 us / bwd 747 us on the
// learner's shape; this one 132 / 426 (profiles/r2ad_attention_microbench.jsonl).
#include "../common.h"
#include "../kernels.h"

#include <cstdlib>

namespace as {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf8;
typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int D = 128;     // head dim
constexpr int BR = 64;     // rows / keys per block
constexpr int PD = D + 8;  // padded LDS row (d-major tiles)
constexpr int PK = BR + 8; // padded LDS row (key/row-major tiles)

__device__ __forceinline__ bf8 ld8(const bf16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  bf8 r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

__device__ __forceinline__ bf8 zero8() {
  const uint4 u = make_uint4(0, 0, 0, 0);
  bf8 r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

__device__ __forceinline__ f4 mfma(const bf8& a, const bf8& b, const f4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// =================================================================================================
// v2: register-resident P / dS ("swapped" products), transposed operands by ds_read_b64_tr_b16.
//
// Every product whose reduction runs over keys (or rows) is computed TRANSPOSED so the softmax row
// (or the key) is lane-local: S^T = K Q^T leaves lane (lg, lr) of a wave holding query row lr and
// keys 16 n + 4 lg + i in its C registers.  The next product's B operand needs, per lane, 8 keys of
// one k-step for that row; the k-slot -> key assignment of an MFMA is free as long as A and B agree,
// so lane group lg takes keys {32 ks + 4 lg + i, 32 ks + 16 + 4 lg + i} - exactly its own C values:
// P^T / dS^T feed the next MFMA straight from registers (no LDS bounce, no barrier).  The A operand
// is then the transposed row-major tile (V^T, dO^T, Q^T, K^T), read with ds_read_b64_tr_b16: group lg
// fetches rows {32 ks + 4 lg + q} (and +16), columns 16 nd .. 16 nd + 15, and lane lr receives column
// lr - i.e. T[key][16 nd + lr] for its 4 keys.  Tiles are staged row-major once (no scalar transposed
// LDS writes), 288-B rows (conflict-free transposed reads, 2-way row reads), and the next tile's
// global loads are issued before the current tile's MFMAs (register staging, written after a barrier).
constexpr int PT = D + 16;   // LDS row pitch (bf16) of the v2 tiles

typedef short v4s __attribute__((ext_vector_type(4)));

// bare v_exp_f32: every argument here is <= 0 (or -1e30-ish for masked entries -> 0), so the libm
// range guards of exp2f (compare + ldexp + branch) are dead weight
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ uint2 ld_tr(const bf16_t* p) {
  const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
  uint2 r;
  __builtin_memcpy(&r, &v, 8);
  return r;
}

// A fragment of T^T for a row-major LDS tile T[64][PT]: A[d = 16 nd + lr][slot 8 lg + e] with slots
// e < 4 <-> tile row 32 ks + 4 lg + e, e >= 4 <-> tile row 32 ks + 16 + 4 lg + (e - 4)
__device__ __forceinline__ bf8 tr_frag(const bf16_t* T, int ks, int nd) {
  const int l = threadIdx.x & 63, lg = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const bf16_t* b = T + (32 * ks + 4 * lg + q) * PT + 16 * nd + 4 * p;
  const uint2 lo = ld_tr(b), hi = ld_tr(b + 16 * PT);
  const uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
  bf8 r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// B fragment from C registers of row/key tiles n = 2 ks, 2 ks + 1 (same slot order as tr_frag)
__device__ __forceinline__ bf8 c_frag(const f4& a, const f4& b) {
  const uint4 u = make_uint4(f2bf2(a[0], a[1]),
                             f2bf2(a[2], a[3]),
                             f2bf2(b[0], b[1]),
                             f2bf2(b[2], b[3]));
  bf8 r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// row-major row read (A operand rows 16 n + lr, k-step ks)
__device__ __forceinline__ bf8 row_frag(const bf16_t* T, int n, int ks) {
  const int l = threadIdx.x & 63;
  return ld8(T + (16 * n + (l & 15)) * PT + 32 * ks + 8 * (l >> 4));
}

// one [64 x 128] tile (rows r0.., valid < nvalid) -> 4 x 16 B registers per thread, and back to LDS
struct TileRegs {
  uint4 v[4];
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long ld, int r0, int nvalid) {
    const int t = threadIdx.x, r = t >> 2, c = t & 3;
    const bool ok = r0 + r < nvalid;
    const bf16_t* src = base + static_cast<long>(ok ? r0 + r : 0) * ld + 32 * c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = *reinterpret_cast<const uint4*>(src + 8 * q);
      if (!ok) v[q] = make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(bf16_t* T) const {
    const int t = threadIdx.x, r = t >> 2, c = t & 3;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4*>(T + r * PT + 32 * c + 8 * q) = v[q];
  }
};

__device__ __forceinline__ float xor_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float xor_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// XCD-aware work mapping for the v2 kernels: a 1-D grid of 8 * ceil(QB * S * H / 8) workgroups; the
// dispatcher deals workgroup ids round-robin over the 8 XCDs, so id i is given work item
// (i % 8) * (grid / 8) + i / 8 - every XCD walks a contiguous range of (observation, head, block)
// items and the blocks of one (observation, head), which re-read the same K / V (Q / dO) tiles, share
// that XCD's L2 instead of fetching the tiles once per XCD.
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

__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, const int* __restrict__ cu,
                                                        bf16_t* __restrict__ out, float* __restrict__ lse2, int H,
                                                        long Ttot, float scale_log2, int QB, int S) {
  __shared__ __attribute__((aligned(16))) bf16_t K_s[BR * PT];
  __shared__ __attribute__((aligned(16))) bf16_t V_s[BR * PT];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;
  const int qrow = qb * BR + w * 16 + lr;   // this lane's query row
  bf8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = qrow < len ? ld8(seq + qrow * ROW + h * D + 32 * ks + 8 * lg) : zero8();
  f4 o[8];   // O^T: o[nd][i] = O[qrow][16 nd + 4 lg + i]
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f4{0.f, 0.f, 0.f, 0.f};
  float m = -1e30f, lsum = 0.f;
  const int nkb = (len + BR - 1) / BR;
  TileRegs rk, rv;
  rk.load(seq + HD + h * D, ROW, 0, len);
  rv.load(seq + 2 * HD + h * D, ROW, 0, len);
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    rk.store(K_s);
    rv.store(V_s);
    __syncthreads();
    if (kb + 1 < nkb) {
      rk.load(seq + HD + h * D, ROW, (kb + 1) * BR, len);
      rv.load(seq + 2 * HD + h * D, ROW, (kb + 1) * BR, len);
    }
    f4 st[4];   // S^T: st[n][i] = S[qrow][key kb*64 + 16 n + 4 lg + i]
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      st[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) st[n] = mfma(row_frag(K_s, n, ks), qf[ks], st[n]);
    }
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
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 pb = c_frag(st[2 * ks], st[2 * ks + 1]);
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) o[nd] = mfma(tr_frag(V_s, ks, nd), pb, o[nd]);
    }
  }
  if (qrow < len) {
    const float inv = 1.f / lsum;
    bf16_t* dst = out + (static_cast<long>(start) + qrow) * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      uint2 u;
      u.x = f2bf2(o[nd][0] * inv, o[nd][1] * inv);
      u.y = f2bf2(o[nd][2] * inv, o[nd][3] * inv);
      *reinterpret_cast<uint2*>(dst + 16 * nd) = u;
    }
    if (lg == 0) lse2[static_cast<long>(h) * Ttot + start + qrow] = m + log2f(lsum);
  }
}

// dK, dV for 64 keys: S = Q K^T and dP = dO V^T leave lane (lg, lr) holding key lr and rows
// 16 n + 4 lg + i; dV^T += dO^T P and dK^T += Q^T dS take P / dS from registers.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse2, const float* __restrict__ delta,
                                                             const int* __restrict__ cu, bf16_t* __restrict__ dqkv, int H,
                                                             long Ttot, float scale_log2, float scale, int QB, int S) {
  __shared__ __attribute__((aligned(16))) bf16_t Q_s[BR * PT];
  __shared__ __attribute__((aligned(16))) bf16_t dO_s[BR * PT];
  __shared__ float lse_s[BR], del_s[BR];
  int kb, s, h;
  if (!attn_item(QB, S, H, kb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (kb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;
  const bf16_t* dseq = dout + static_cast<long>(start) * HD;
  const int key = kb * BR + w * 16 + lr;   // this lane's key
  const bool kval = key < len;
  bf8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = kval ? ld8(seq + key * ROW + HD + h * D + 32 * ks + 8 * lg) : zero8();
    vf[ks] = kval ? ld8(seq + key * ROW + 2 * HD + h * D + 32 * ks + 8 * lg) : zero8();
  }
  f4 dk[8], dv[8];   // dK^T / dV^T: [nd][i] = d(key)[16 nd + 4 lg + i]
#pragma unroll
  for (int n = 0; n < 8; ++n) { dk[n] = f4{0.f, 0.f, 0.f, 0.f}; dv[n] = f4{0.f, 0.f, 0.f, 0.f}; }
  const int nrb = (len + BR - 1) / BR;
  TileRegs rq, rd;
  rq.load(seq + h * D, ROW, 0, len);
  rd.load(dseq + h * D, HD, 0, len);
  for (int rb = 0; rb < nrb; ++rb) {
    if (rb) __syncthreads();
    rq.store(Q_s);
    rd.store(dO_s);
    if (tid < BR) {
      const int r = rb * BR + tid;
      lse_s[tid] = r < len ? lse2[static_cast<long>(h) * Ttot + start + r] : 1e30f;
      del_s[tid] = r < len ? delta[static_cast<long>(h) * Ttot + start + r] : 0.f;
    }
    __syncthreads();
    if (rb + 1 < nrb) {
      rq.load(seq + h * D, ROW, (rb + 1) * BR, len);
      rd.load(dseq + h * D, HD, (rb + 1) * BR, len);
    }
    f4 sc[4], dp[4];   // [n][i]: row 16 n + 4 lg + i, key lr
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sc[n] = f4{0.f, 0.f, 0.f, 0.f};
      dp[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc[n] = mfma(row_frag(Q_s, n, ks), kf[ks], sc[n]);
        dp[n] = mfma(row_frag(dO_s, n, ks), vf[ks], dp[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 16 * n + 4 * lg + i;
        const float p = kval ? ex2(sc[n][i] * scale_log2 - lse_s[rl]) : 0.f;   // padded rows: lse = +inf
        sc[n][i] = p;
        dp[n][i] = p * (dp[n][i] - del_s[rl]);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 pb = c_frag(sc[2 * ks], sc[2 * ks + 1]);
      const bf8 db = c_frag(dp[2 * ks], dp[2 * ks + 1]);
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) {
        dv[nd] = mfma(tr_frag(dO_s, ks, nd), pb, dv[nd]);
        dk[nd] = mfma(tr_frag(Q_s, ks, nd), db, dk[nd]);
      }
    }
  }
  if (kval) {
    const long tok = static_cast<long>(start) + key;
    bf16_t* dkp = dqkv + tok * 3 * HD + HD + h * D + 4 * lg;
    bf16_t* dvp = dqkv + tok * 3 * HD + 2 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      uint2 u;
      u.x = f2bf2(dk[nd][0] * scale, dk[nd][1] * scale);
      u.y = f2bf2(dk[nd][2] * scale, dk[nd][3] * scale);
      *reinterpret_cast<uint2*>(dkp + 16 * nd) = u;
      u.x = f2bf2(dv[nd][0], dv[nd][1]);
      u.y = f2bf2(dv[nd][2], dv[nd][3]);
      *reinterpret_cast<uint2*>(dvp + 16 * nd) = u;
    }
  }
}

// dQ for 64 rows: S^T = K Q^T and dP^T = V dO^T leave lane (lg, lr) holding row lr and keys
// 16 n + 4 lg + i; dQ^T += K^T dS^T takes dS^T from registers.
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse2, float* __restrict__ delta,
                                                           const int* __restrict__ cu, bf16_t* __restrict__ dqkv, int H,
                                                           long Ttot, float scale_log2, float scale, int QB, int S) {
  __shared__ __attribute__((aligned(16))) bf16_t K_s[BR * PT];
  __shared__ __attribute__((aligned(16))) bf16_t V_s[BR * PT];
  int qb, s, h;
  if (!attn_item(QB, S, H, qb, s, h)) return;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;
  const bf16_t* dseq = dout + static_cast<long>(start) * HD;
  const int qrow = qb * BR + w * 16 + lr;
  const bool rval = qrow < len;
  bf8 qf[4], df[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = rval ? ld8(seq + qrow * ROW + h * D + 32 * ks + 8 * lg) : zero8();
    df[ks] = rval ? ld8(dseq + static_cast<long>(qrow) * HD + h * D + 32 * ks + 8 * lg) : zero8();
  }
  const float ls = rval ? lse2[static_cast<long>(h) * Ttot + start + qrow] : 1e30f;
  // delta = rowsum(dO * O) for this lane's row: the dO fragments are already in registers; the 4 lane
  // groups hold disjoint 32-column slices, summed by two xor shuffles
  float dl = 0.f;
  {
    const bf16_t* orow = o + (static_cast<long>(start) + (rval ? qrow : 0)) * HD + h * D + 8 * lg;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 ov = rval ? *reinterpret_cast<const uint4*>(orow + 32 * ks) : make_uint4(0, 0, 0, 0);
      uint4 dv;
      __builtin_memcpy(&dv, &df[ks], 16);
      const uint32_t a[4] = {ov.x, ov.y, ov.z, ov.w}, b[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dl += __uint_as_float(a[e] << 16) * __uint_as_float(b[e] << 16) +
              __uint_as_float(a[e] & 0xffff0000u) * __uint_as_float(b[e] & 0xffff0000u);
    }
    dl = xor_sum(dl);
  }
  if (rval && lg == 0) delta[static_cast<long>(h) * Ttot + start + qrow] = dl;
  f4 dq[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) dq[n] = f4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (len + BR - 1) / BR;
  TileRegs rk, rv;
  rk.load(seq + HD + h * D, ROW, 0, len);
  rv.load(seq + 2 * HD + h * D, ROW, 0, len);
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb) __syncthreads();
    rk.store(K_s);
    rv.store(V_s);
    __syncthreads();
    if (kb + 1 < nkb) {
      rk.load(seq + HD + h * D, ROW, (kb + 1) * BR, len);
      rv.load(seq + 2 * HD + h * D, ROW, (kb + 1) * BR, len);
    }
    f4 st[4], dpt[4];   // [n][i]: key 16 n + 4 lg + i, row qrow
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      st[n] = f4{0.f, 0.f, 0.f, 0.f};
      dpt[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        st[n] = mfma(row_frag(K_s, n, ks), qf[ks], st[n]);
        dpt[n] = mfma(row_frag(V_s, n, ks), df[ks], dpt[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool kv = kb * BR + 16 * n + 4 * lg + i < len;
        const float p = kv ? ex2(st[n][i] * scale_log2 - ls) : 0.f;
        dpt[n][i] = p * (dpt[n][i] - dl);
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 db = c_frag(dpt[2 * ks], dpt[2 * ks + 1]);
#pragma unroll
      for (int nd = 0; nd < 8; ++nd) dq[nd] = mfma(tr_frag(K_s, ks, nd), db, dq[nd]);
    }
  }
  if (rval) {
    bf16_t* dqp = dqkv + (static_cast<long>(start) + qrow) * 3 * HD + h * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < 8; ++nd) {
      uint2 u;
      u.x = f2bf2(dq[nd][0] * scale, dq[nd][1] * scale);
      u.y = f2bf2(dq[nd][2] * scale, dq[nd][3] * scale);
      *reinterpret_cast<uint2*>(dqp + 16 * nd) = u;
    }
  }
}

}  // namespace

void varlen_attn_fwd(const void* qkv, const int* cu, void* out, float* lse2, int S, int max_len, int H, long Ttot,
                     float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const int QB = (max_len + BR - 1) / BR;
  const dim3 grid(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv), cu,
                     static_cast<bf16_t*>(out), lse2, H, Ttot, scale_log2, QB, S);
}

void varlen_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, const int* cu, void* dqkv,
                     float* delta, int S, int max_len, int H, long Ttot, float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const int QB = (max_len + BR - 1) / BR;
  const dim3 grid(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
  // dQ first: it also writes delta, which the dK / dV kernel reads
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                     static_cast<const bf16_t*>(out), static_cast<const bf16_t*>(dout), lse2, delta, cu,
                     static_cast<bf16_t*>(dqkv), H, Ttot, scale_log2, scale, QB, S);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                     static_cast<const bf16_t*>(dout), lse2, delta, cu, static_cast<bf16_t*>(dqkv), H, Ttot,
                     scale_log2, scale, QB, S);
}

}  // namespace as
