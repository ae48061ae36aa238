// Variable-length (packed) multi-head self-attention for the entity transformer, forward and
// backward, bf16 MFMA (v_mfma_f32_16x16x32_bf16) with fp32 softmax state.  gfx950.
//
// The reference materialises [B, 2, N, N] fp32 scores over the zero-padded entity batch and masks
// padded keys with -1e9 (module_utils.py:88-111).  Here entities of all observations are packed
// ([T_total, 3*H*D] rows = q | k | v, cu_seqlens delimits each observation) and one workgroup owns
// one (observation, head, 64-row block): only real entities are touched, scores never leave
// registers (online softmax, flash style), and the key mask becomes the loop bound.
//
// Tiling (D = 128, 4 waves x 16 query rows):
//   S   = Q K^T : A = Q rows from global (16 B / lane), B = K tile in LDS [key][d]   (16 MFMA/wave)
//   O  += P V   : A = P via a per-wave LDS bounce,     B = V^T tile in LDS [d][key]  (16 MFMA/wave)
// LDS rows are padded by 16 B so the 16-lane ds_read_b128 groups hit distinct banks.
// Backward = two kernels with recomputation (no atomics, deterministic):
//   attn_bwd_dkdv : per 64-key block, loops row blocks: S^T = K Q^T, P^T, dV += P^T dO,
//                   dP^T = V dO^T, dS^T = P^T (dP^T - delta), dK += dS^T Q
//   attn_bwd_dq   : per 64-row block, loops key blocks: S, P, dP = dO V^T, dS, dQ += dS K
// LSE is stored in the log2 domain (lse2 = m + log2(l) of scale*log2(e)-scaled scores).
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

__device__ __forceinline__ float grp16_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  v = fmaxf(v, __shfl_xor(v, 8, 64));
  return v;
}

__device__ __forceinline__ float grp16_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// Stage a [64 x 128] bf16 tile (rows r0.. of column block `col`) into LDS row-major [64][PD] and,
// if tr != nullptr, transposed [128][PK].  256 threads, 4 x 16 B per thread.
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ base, long ld, int r0, int nvalid,
                                           bf16_t (*rm)[PD], bf16_t (*tr)[PK]) {
  const int t = threadIdx.x;
  const int r = t >> 2, c = t & 3;
  const bool ok = (r0 + r) < nvalid;
  const bf16_t* src = base + static_cast<long>(r0 + r) * ld + 32 * c;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint4 v = ok ? *reinterpret_cast<const uint4*>(src + 8 * q) : make_uint4(0, 0, 0, 0);
    if (rm) *reinterpret_cast<uint4*>(&rm[r][32 * c + 8 * q]) = v;
    if (tr) {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tr[32 * c + 8 * q + 2 * j][r] = static_cast<bf16_t>(w[j] & 0xffffu);
        tr[32 * c + 8 * q + 2 * j + 1][r] = static_cast<bf16_t>(w[j] >> 16);
      }
    }
  }
}

// ------------------------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, const int* __restrict__ cu,
                                                       bf16_t* __restrict__ out, float* __restrict__ lse2, int H,
                                                       long Ttot, float scale_log2) {
  __shared__ __attribute__((aligned(16))) bf16_t K_s[BR][PD];
  __shared__ __attribute__((aligned(16))) bf16_t Vt_s[D][PK];
  __shared__ __attribute__((aligned(16))) bf16_t P_s[4][16][PK];
  const int qb = blockIdx.x, s = blockIdx.y, h = blockIdx.z;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;

  const int qrow = qb * BR + w * 16 + lr;
  bf8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
    qf[ks] = qrow < len ? ld8(seq + qrow * ROW + h * D + 32 * ks + 8 * lg) : zero8();

  f4 o[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = f4{0.f, 0.f, 0.f, 0.f};
  float m[4], lsum[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -1e30f; lsum[i] = 0.f; }

  const int nkb = (len + BR - 1) / BR;
  for (int kb = 0; kb < nkb; ++kb) {
    stage_tile(seq + HD + h * D, ROW, kb * BR, len, K_s, nullptr);
    stage_tile(seq + 2 * HD + h * D, ROW, kb * BR, len, nullptr, Vt_s);
    __syncthreads();
    f4 sc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sc[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sc[n] = mfma(qf[ks], ld8(&K_s[16 * n + lr][32 * ks + 8 * lg]), sc[n]);
    }
    float mx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) mx[i] = -1e30f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bool valid = (kb * BR + 16 * n + lr) < len;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = valid ? sc[n][i] * scale_log2 : -1e30f;
        sc[n][i] = v;
        mx[i] = fmaxf(mx[i], v);
      }
    }
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mn = fmaxf(m[i], grp16_max(mx[i]));
      alpha[i] = exp2f(m[i] - mn);
      m[i] = mn;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sc[n][i] - m[i]);
        sc[n][i] = p;
        rs += p;
      }
      lsum[i] = lsum[i] * alpha[i] + grp16_sum(rs);
    }
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= alpha[i];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) P_s[w][4 * lg + i][16 * n + lr] = f2bf(sc[n][i]);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 pf = ld8(&P_s[w][lr][32 * ks + 8 * lg]);
#pragma unroll
      for (int n = 0; n < 8; ++n) o[n] = mfma(pf, ld8(&Vt_s[16 * n + lr][32 * ks + 8 * lg]), o[n]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = qb * BR + w * 16 + 4 * lg + i;
    if (row < len) {
      const float inv = 1.f / lsum[i];
      bf16_t* dst = out + (static_cast<long>(start) + row) * HD + h * D;
#pragma unroll
      for (int n = 0; n < 8; ++n) dst[16 * n + lr] = f2bf(o[n][i] * inv);
      if (lr == 0) lse2[static_cast<long>(h) * Ttot + start + row] = m[i] + log2f(lsum[i]);
    }
  }
}

// delta[h][t] = sum_d dO[t, h, d] * O[t, h, d]   (one wave per (t, h))
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ o,
                                                         float* __restrict__ delta, int H, long Ttot) {
  const long wave = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  if (wave >= Ttot * H) return;
  const long t = wave / H;
  const int h = static_cast<int>(wave % H);
  const long base = t * H * D + h * D + 2 * l;
  const float v = bf2f(dout[base]) * bf2f(o[base]) + bf2f(dout[base + 1]) * bf2f(o[base + 1]);
  const float s = wave_sum(v);
  if (l == 0) delta[static_cast<long>(h) * Ttot + t] = s;
}

// ------------------------------------------------------------------------------- backward dK dV
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                            const float* __restrict__ lse2, const float* __restrict__ delta,
                                                            const int* __restrict__ cu, bf16_t* __restrict__ dqkv, int H,
                                                            long Ttot, float scale_log2, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t Q_s[BR][PD];
  __shared__ __attribute__((aligned(16))) bf16_t Qt_s[D][PK];
  __shared__ __attribute__((aligned(16))) bf16_t dO_s[BR][PD];
  __shared__ __attribute__((aligned(16))) bf16_t dOt_s[D][PK];
  __shared__ __attribute__((aligned(16))) bf16_t T_s[4][16][PK];  // per-wave transpose bounce
  __shared__ float lse_s[BR], del_s[BR];
  const int kb = blockIdx.x, s = blockIdx.y, h = blockIdx.z;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (kb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;
  const bf16_t* dseq = dout + static_cast<long>(start) * HD;

  // this wave's 16 keys as A fragments (K for S^T, V for dP^T)
  const int key = kb * BR + w * 16 + lr;
  bf8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = key < len ? ld8(seq + key * ROW + HD + h * D + 32 * ks + 8 * lg) : zero8();
    vf[ks] = key < len ? ld8(seq + key * ROW + 2 * HD + h * D + 32 * ks + 8 * lg) : zero8();
  }
  f4 dk[8], dv[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) { dk[n] = f4{0.f, 0.f, 0.f, 0.f}; dv[n] = f4{0.f, 0.f, 0.f, 0.f}; }
  // key validity of this lane's C-rows (keys 4lg+i of the wave)
  bool kvalid[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) kvalid[i] = (kb * BR + w * 16 + 4 * lg + i) < len;

  const int nrb = (len + BR - 1) / BR;
  for (int rb = 0; rb < nrb; ++rb) {
    stage_tile(seq + h * D, ROW, rb * BR, len, Q_s, Qt_s);
    stage_tile(dseq + h * D, HD, rb * BR, len, dO_s, dOt_s);
    if (tid < BR) {
      const int r = rb * BR + tid;
      lse_s[tid] = r < len ? lse2[static_cast<long>(h) * Ttot + start + r] : 1e30f;
      del_s[tid] = r < len ? delta[static_cast<long>(h) * Ttot + start + r] : 0.f;
    }
    __syncthreads();
    // S^T [16 keys x 64 rows] and dP^T
    f4 st[4], dpt[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      st[n] = f4{0.f, 0.f, 0.f, 0.f};
      dpt[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        st[n] = mfma(kf[ks], ld8(&Q_s[16 * n + lr][32 * ks + 8 * lg]), st[n]);
        dpt[n] = mfma(vf[ks], ld8(&dO_s[16 * n + lr][32 * ks + 8 * lg]), dpt[n]);
      }
    }
    // P^T and dS^T (C layout: row = key 4lg+i, col = query row 16n+lr)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int rl = 16 * n + lr;
      const float ls = lse_s[rl], dl = del_s[rl];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = kvalid[i] ? exp2f(st[n][i] * scale_log2 - ls) : 0.f;  // ls = +inf for padded rows -> 0
        st[n][i] = p;
        dpt[n][i] = p * (dpt[n][i] - dl);
      }
    }
    // dV += P^T dO  (A = P^T via LDS bounce, B = dO^T tile)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) T_s[w][4 * lg + i][16 * n + lr] = f2bf(st[n][i]);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 pf = ld8(&T_s[w][lr][32 * ks + 8 * lg]);
#pragma unroll
      for (int n = 0; n < 8; ++n) dv[n] = mfma(pf, ld8(&dOt_s[16 * n + lr][32 * ks + 8 * lg]), dv[n]);
    }
    __syncthreads();
    // dK += dS^T Q
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) T_s[w][4 * lg + i][16 * n + lr] = f2bf(dpt[n][i]);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 df = ld8(&T_s[w][lr][32 * ks + 8 * lg]);
#pragma unroll
      for (int n = 0; n < 8; ++n) dk[n] = mfma(df, ld8(&Qt_s[16 * n + lr][32 * ks + 8 * lg]), dk[n]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (!kvalid[i]) continue;
    const long tok = static_cast<long>(start) + kb * BR + w * 16 + 4 * lg + i;
    bf16_t* dkp = dqkv + tok * 3 * HD + HD + h * D;
    bf16_t* dvp = dqkv + tok * 3 * HD + 2 * HD + h * D;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      dkp[16 * n + lr] = f2bf(dk[n][i] * scale);
      dvp[16 * n + lr] = f2bf(dv[n][i]);
    }
  }
}

// ---------------------------------------------------------------------------------- backward dQ
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                          const float* __restrict__ lse2, const float* __restrict__ delta,
                                                          const int* __restrict__ cu, bf16_t* __restrict__ dqkv, int H,
                                                          long Ttot, float scale_log2, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t K_s[BR][PD];
  __shared__ __attribute__((aligned(16))) bf16_t Kt_s[D][PK];
  __shared__ __attribute__((aligned(16))) bf16_t V_s[BR][PD];
  __shared__ __attribute__((aligned(16))) bf16_t T_s[4][16][PK];
  const int qb = blockIdx.x, s = blockIdx.y, h = blockIdx.z;
  const int start = cu[s];
  const int len = cu[s + 1] - start;
  if (qb * BR >= len) return;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, lg = l >> 4;
  const int HD = H * D;
  const long ROW = 3L * HD;
  const bf16_t* seq = qkv + static_cast<long>(start) * ROW;
  const bf16_t* dseq = dout + static_cast<long>(start) * HD;

  const int qrow = qb * BR + w * 16 + lr;
  bf8 qf[4], df[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = qrow < len ? ld8(seq + qrow * ROW + h * D + 32 * ks + 8 * lg) : zero8();
    df[ks] = qrow < len ? ld8(dseq + static_cast<long>(qrow) * HD + h * D + 32 * ks + 8 * lg) : zero8();
  }
  float ls[4], dl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = qb * BR + w * 16 + 4 * lg + i;
    ls[i] = r < len ? lse2[static_cast<long>(h) * Ttot + start + r] : 1e30f;
    dl[i] = r < len ? delta[static_cast<long>(h) * Ttot + start + r] : 0.f;
  }
  f4 dq[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) dq[n] = f4{0.f, 0.f, 0.f, 0.f};

  const int nkb = (len + BR - 1) / BR;
  for (int kb = 0; kb < nkb; ++kb) {
    stage_tile(seq + HD + h * D, ROW, kb * BR, len, K_s, Kt_s);
    stage_tile(seq + 2 * HD + h * D, ROW, kb * BR, len, V_s, nullptr);
    __syncthreads();
    f4 sc[4], dp[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sc[n] = f4{0.f, 0.f, 0.f, 0.f};
      dp[n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc[n] = mfma(qf[ks], ld8(&K_s[16 * n + lr][32 * ks + 8 * lg]), sc[n]);
        dp[n] = mfma(df[ks], ld8(&V_s[16 * n + lr][32 * ks + 8 * lg]), dp[n]);
      }
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const bool valid = (kb * BR + 16 * n + lr) < len;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = valid ? exp2f(sc[n][i] * scale_log2 - ls[i]) : 0.f;
        T_s[w][4 * lg + i][16 * n + lr] = f2bf(p * (dp[n][i] - dl[i]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf8 sf = ld8(&T_s[w][lr][32 * ks + 8 * lg]);
#pragma unroll
      for (int n = 0; n < 8; ++n) dq[n] = mfma(sf, ld8(&Kt_s[16 * n + lr][32 * ks + 8 * lg]), dq[n]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = qb * BR + w * 16 + 4 * lg + i;
    if (row >= len) continue;
    bf16_t* dqp = dqkv + (static_cast<long>(start) + row) * 3 * HD + h * D;
#pragma unroll
    for (int n = 0; n < 8; ++n) dqp[16 * n + lr] = f2bf(dq[n][i] * scale);
  }
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

__global__ __launch_bounds__(256) void attn2_fwd_kernel(const bf16_t* __restrict__ qkv, const int* __restrict__ cu,
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
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn2_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
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
__global__ __launch_bounds__(256) void attn2_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse2, const float* __restrict__ delta,
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
  const float dl = rval ? delta[static_cast<long>(h) * Ttot + start + qrow] : 0.f;
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

bool attn_v2() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_ATTN_V2");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

void varlen_attn_fwd(const void* qkv, const int* cu, void* out, float* lse2, int S, int max_len, int H, long Ttot,
                     float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid((max_len + BR - 1) / BR, S, H);
  if (attn_v2()) {
    const int QB = (max_len + BR - 1) / BR;
    const dim3 g1(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
    hipLaunchKernelGGL(attn2_fwd_kernel, g1, dim3(256), 0, s, static_cast<const bf16_t*>(qkv), cu,
                       static_cast<bf16_t*>(out), lse2, H, Ttot, scale_log2, QB, S);
    return;
  }
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv), cu,
                     static_cast<bf16_t*>(out), lse2, H, Ttot, scale_log2);
}

void varlen_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, const int* cu, void* dqkv,
                     float* delta, int S, int max_len, int H, long Ttot, float scale, hipStream_t s) {
  const float scale_log2 = scale * 1.4426950408889634f;
  const long waves = Ttot * H;
  hipLaunchKernelGGL(attn_delta_kernel, dim3(static_cast<unsigned>((waves * 64 + 255) / 256)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(dout), static_cast<const bf16_t*>(out), delta, H, Ttot);
  dim3 grid((max_len + BR - 1) / BR, S, H);
  if (attn_v2()) {
    const int QB = (max_len + BR - 1) / BR;
    const dim3 g1(static_cast<unsigned>((static_cast<long>(QB) * S * H + 7) / 8 * 8));
    hipLaunchKernelGGL(attn2_bwd_dkdv_kernel, g1, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                       static_cast<const bf16_t*>(dout), lse2, delta, cu, static_cast<bf16_t*>(dqkv), H, Ttot,
                       scale_log2, scale, QB, S);
    hipLaunchKernelGGL(attn2_bwd_dq_kernel, g1, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                       static_cast<const bf16_t*>(dout), lse2, delta, cu, static_cast<bf16_t*>(dqkv), H, Ttot,
                       scale_log2, scale, QB, S);
    return;
  }
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                     static_cast<const bf16_t*>(dout), lse2, delta, cu, static_cast<bf16_t*>(dqkv), H, Ttot, scale_log2,
                     scale);
  hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(qkv),
                     static_cast<const bf16_t*>(dout), lse2, delta, cu, static_cast<bf16_t*>(dqkv), H, Ttot, scale_log2,
                     scale);
}

}  // namespace as
