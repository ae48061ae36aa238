// The value baseline's residual MLP stack: n x ResFCBlock2 over 256 features,
//   x <- LN( fc2(relu(fc1(x))) + x )          (res_block.py:110-140, value.py:31-39)
// as ONE forward kernel and ONE backward-data kernel (the weight gradients are one batched wgrad launch).
//
// As torch ops the 16-block stack of one baseline is ~55 forward and ~170 backward launches on
// 390 x 256 activations (r2f attribution: 228 launches, 1.5 ms).  Here a 256-thread workgroup owns 16
// rows for the whole stack: the rows stay in LDS (fp32 residual stream + its bf16 MFMA copy), each
// 256 x 256 GEMM is 16 x 16 x 32 bf16 MFMAs with the weight fragments read straight from L2 (wave w
// owns output columns 64 w .. 64 w + 63), bias / ReLU / residual / LayerNorm are fused around them.
// The forward saves per block the bf16 input, the bf16 hidden activation, the fp32 normalised sum and
// its rstd; the backward walks the blocks in reverse (LN backward, then the two GEMMs against
// transposed weights), saves dY / dH for the batched weight gradient and writes per-workgroup
// LayerNorm-affine partials (no atomics, deterministic).
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int DIM = 256, RB = 16, AP = DIM + 8;  // rows per workgroup, padded bf16 LDS row

typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ bf8v ld_frag(const bf16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  bf8v r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// acc[j] (j < 4) = rows 0..15 of  A[16][256] (LDS, pitch AP) . W^T,  W [256][256] row-major (global);
// lane l of wave w holds C[4 (l >> 4) + i][64 w + 16 j + (l & 15)] in acc[j][i]
__device__ __forceinline__ void gemm16(const bf16_t* A, const bf16_t* __restrict__ W, f4 acc[4]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = l & 15, lg = l >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
  const bf16_t* wrow = W + static_cast<long>(64 * w + lr) * DIM + 8 * lg;
#pragma unroll
  for (int ks = 0; ks < DIM / 32; ++ks) {
    const bf8v a = ld_frag(A + lr * AP + ks * 32 + 8 * lg);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
        a, ld_frag(wrow + static_cast<long>(16 * j) * DIM + ks * 32), acc[j], 0, 0, 0);
  }
}

__device__ __forceinline__ float ldv(const void* p, int dt, long i) {
  return dt == DT_BF16 ? bf2f(static_cast<const bf16_t*>(p)[i]) : static_cast<const float*>(p)[i];
}

__global__ __launch_bounds__(256) void resmlp_fwd_kernel(const void* __restrict__ x0, int x0_dt, const ResMlpW w,
                                                         int nblk, float* __restrict__ out, bf16_t* __restrict__ sv_x,
                                                         bf16_t* __restrict__ sv_h, float* __restrict__ sv_xhat,
                                                         float* __restrict__ sv_rstd, long R) {
  __shared__ float X[RB][DIM];
  __shared__ float S[RB][DIM];
  __shared__ __attribute__((aligned(16))) bf16_t Xb[RB * AP];
  __shared__ __attribute__((aligned(16))) bf16_t Hb[RB * AP];
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, lr = l & 15, lg = l >> 4;
  const long r0 = static_cast<long>(blockIdx.x) * RB;
  const bool save = sv_x != nullptr;
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    const float v = r0 + r < R ? ldv(x0, x0_dt, (r0 + r) * DIM + c) : 0.f;
    X[r][c] = v;
    Xb[r * AP + c] = f2bf(v);
  }
  __syncthreads();
  for (int k = 0; k < nblk; ++k) {
    const long so = static_cast<long>(k) * R * DIM;
    if (save)
      for (int i = tid; i < RB * DIM; i += 256) {
        const int r = i / DIM, c = i - r * DIM;
        if (r0 + r < R) sv_x[so + (r0 + r) * DIM + c] = Xb[r * AP + c];
      }
    f4 acc[4];
    gemm16(Xb, static_cast<const bf16_t*>(w.w1[k]), acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
      const float b = bf2f(static_cast<const bf16_t*>(w.b1[k])[c]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lg + i;
        const bf16_t h = f2bf(fmaxf(acc[j][i] + b, 0.f));
        Hb[r * AP + c] = h;
        if (save && r0 + r < R) sv_h[so + (r0 + r) * DIM + c] = h;
      }
    }
    __syncthreads();
    gemm16(Hb, static_cast<const bf16_t*>(w.w2[k]), acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
      const float b = bf2f(static_cast<const bf16_t*>(w.b2[k])[c]);
#pragma unroll
      for (int i = 0; i < 4; ++i) S[4 * lg + i][c] = acc[j][i] + b + X[4 * lg + i][c];
    }
    __syncthreads();
    // LayerNorm per row: wave wv owns rows 4 wv .. 4 wv + 3, lane l columns 4 l .. 4 l + 3
    for (int rr = 0; rr < 4; ++rr) {
      const int r = 4 * wv + rr;
      float v[4], s1 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = S[r][4 * l + e];
        s1 += v[e];
      }
      const float mean = wave_sum(s1) * (1.f / DIM);
      float s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) s2 += (v[e] - mean) * (v[e] - mean);
      const float rs = rsqrtf(wave_sum(s2) * (1.f / DIM) + 1e-5f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * l + e;
        const float xh = (v[e] - mean) * rs;
        const float y = xh * w.g[k][c] + w.be[k][c];
        X[r][c] = y;
        Xb[r * AP + c] = f2bf(y);
        if (save && r0 + r < R) sv_xhat[so + (r0 + r) * DIM + c] = xh;
      }
      if (save && l == 0 && r0 + r < R) sv_rstd[static_cast<long>(k) * R + r0 + r] = rs;
    }
    __syncthreads();
  }
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    if (r0 + r < R) out[(r0 + r) * DIM + c] = X[r][c];
  }
}

__global__ __launch_bounds__(256) void resmlp_bwd_kernel(const float* __restrict__ dout, const ResMlpW w, int nblk,
                                                         const bf16_t* __restrict__ sv_h, const float* __restrict__ sv_xhat,
                                                         const float* __restrict__ sv_rstd, bf16_t* __restrict__ sv_dy,
                                                         bf16_t* __restrict__ sv_dh, float* __restrict__ ln_part,
                                                         float* __restrict__ dx0, long R) {
  __shared__ float dX[RB][DIM];
  __shared__ float T[RB][DIM];
  __shared__ float red[4][2 * DIM];
  __shared__ __attribute__((aligned(16))) bf16_t Ab[RB * AP];
  __shared__ __attribute__((aligned(16))) bf16_t Hd[RB * AP];
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, lr = l & 15, lg = l >> 4;
  const long r0 = static_cast<long>(blockIdx.x) * RB;
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    dX[r][c] = r0 + r < R ? dout[(r0 + r) * DIM + c] : 0.f;
  }
  __syncthreads();
  for (int k = nblk - 1; k >= 0; --k) {
    const long so = static_cast<long>(k) * R * DIM;
    // LayerNorm backward (rows >= R have dX = 0 and contribute nothing)
    float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
    for (int rr = 0; rr < 4; ++rr) {
      const int r = 4 * wv + rr;
      const bool ok = r0 + r < R;
      const float rs = ok ? sv_rstd[static_cast<long>(k) * R + r0 + r] : 0.f;
      float xh[4], dxh[4], m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * l + e;
        xh[e] = ok ? sv_xhat[so + (r0 + r) * DIM + c] : 0.f;
        const float d = dX[r][c];
        pg[e] += d * xh[e];
        pb[e] += d;
        dxh[e] = d * w.g[k][c];
        m1 += dxh[e];
        m2 += dxh[e] * xh[e];
      }
      m1 = wave_sum(m1) * (1.f / DIM);
      m2 = wave_sum(m2) * (1.f / DIM);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * l + e;
        const float ds = rs * (dxh[e] - m1 - xh[e] * m2);
        T[r][c] = ds;
        const bf16_t db = f2bf(ds);
        Ab[r * AP + c] = db;
        if (ok) sv_dy[so + (r0 + r) * DIM + c] = db;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[wv][4 * l + e] = pg[e];
      red[wv][DIM + 4 * l + e] = pb[e];
    }
    __syncthreads();
    for (int c = tid; c < 2 * DIM; c += 256)
      ln_part[(static_cast<long>(blockIdx.x) * nblk + k) * 2 * DIM + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    // dH = (dS W2) * (h > 0)     (W2^T row-major = w.w2t)
    f4 acc[4];
    gemm16(Ab, static_cast<const bf16_t*>(w.w2t[k]), acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lg + i;
        const bool ok = r0 + r < R;
        const bool act = ok && bf2f(sv_h[so + (r0 + r) * DIM + c]) > 0.f;
        const bf16_t d = f2bf(act ? acc[j][i] : 0.f);
        Hd[r * AP + c] = d;
        if (ok) sv_dh[so + (r0 + r) * DIM + c] = d;
      }
    }
    __syncthreads();
    // dX = dS + dH W1    (W1^T row-major = w.w1t)
    gemm16(Hd, static_cast<const bf16_t*>(w.w1t[k]), acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) dX[4 * lg + i][c] = T[4 * lg + i][c] + acc[j][i];
    }
    __syncthreads();
  }
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    if (r0 + r < R) dx0[(r0 + r) * DIM + c] = dX[r][c];
  }
}

// dst[m] = src[m]^T for m < nmat 256 x 256 bf16 matrices (32 x 32 LDS tiles)
__global__ __launch_bounds__(256) void transpose256_kernel(const ResMlpW w, int nblk, bf16_t* __restrict__ dst) {
  __shared__ bf16_t tile[32][33];
  const int m = blockIdx.y;              // 0 .. 2 nblk - 1: W1 of block m / 2 (even), W2 (odd)
  const bf16_t* src = static_cast<const bf16_t*>((m & 1) ? w.w2[m >> 1] : w.w1[m >> 1]);
  const int tr = blockIdx.x / 8, tc = blockIdx.x % 8;
  const int x = threadIdx.x & 31, y0 = threadIdx.x >> 5;
  for (int y = y0; y < 32; y += 8) tile[y][x] = src[(32 * tr + y) * DIM + 32 * tc + x];
  __syncthreads();
  bf16_t* d = dst + static_cast<long>(m) * DIM * DIM;
  for (int y = y0; y < 32; y += 8) d[(32 * tc + y) * DIM + 32 * tr + x] = tile[x][y];
}

}  // namespace

void resmlp_fwd(const void* x0, int x0_dt, const ResMlpW& w, int nblk, float* out, bf16_t* sv_x, bf16_t* sv_h,
                float* sv_xhat, float* sv_rstd, long R, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(resmlp_fwd_kernel, dim3(static_cast<unsigned>((R + RB - 1) / RB)), dim3(256), 0, s, x0, x0_dt, w,
                     nblk, out, sv_x, sv_h, sv_xhat, sv_rstd, R);
}

void resmlp_transpose(const ResMlpW& w, int nblk, bf16_t* dst, hipStream_t s) {
  hipLaunchKernelGGL(transpose256_kernel, dim3(64, 2 * nblk), dim3(256), 0, s, w, nblk, dst);
}

int resmlp_row_blocks(long R) { return static_cast<int>((R + RB - 1) / RB); }

void resmlp_bwd(const float* dout, const ResMlpW& w, int nblk, const bf16_t* sv_h, const float* sv_xhat,
                const float* sv_rstd, bf16_t* sv_dy, bf16_t* sv_dh, float* ln_part, float* dx0, long R, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(resmlp_bwd_kernel, dim3(static_cast<unsigned>((R + RB - 1) / RB)), dim3(256), 0, s, dout, w, nblk,
                     sv_h, sv_xhat, sv_rstd, sv_dy, sv_dh, ln_part, dx0, R);
}

}  // namespace as
