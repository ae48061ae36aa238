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

// Weight fragments of one 256 x 256 GEMM for this wave (output columns 64 w .. 64 w + 63): lane l holds
// W[64 w + 16 j + (l & 15)][32 ks + 8 (l >> 4) .. +8] in wf[ks][j] (32 x 16 B = 128 VGPRs).  The stack is
// latency-bound (ceil(R / 16) workgroups walk 32 GEMMs in sequence, each streaming the whole weight set
// through ONE CU), so (a) the operands are pre-packed in exactly this fragment order (resmlp_pack): each
// wave load instruction is one contiguous 1-KB run of full cache lines instead of 16 half lines, and
// (b) the fragments of the NEXT GEMM are requested as soon as the current one has consumed each k-slice:
// their latency overlaps the epilogue, the LayerNorm and the barrier.
typedef uint4 WFrag[DIM / 32][4];
constexpr long kImg = static_cast<long>(DIM) * DIM;   // elements per packed matrix

__device__ __forceinline__ const uint4* frag_base(const bf16_t* img) {
  return reinterpret_cast<const uint4*>(img) + (threadIdx.x >> 6) * (8 * 4 * 64) + (threadIdx.x & 63);
}

__device__ __forceinline__ void load_w(const bf16_t* __restrict__ img, WFrag& wf) {
  const uint4* p = frag_base(img);
#pragma unroll
  for (int ks = 0; ks < DIM / 32; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[ks][j] = p[(ks * 4 + j) * 64];
}

// acc[j] (j < 4) = rows 0..15 of  A[16][256] (LDS, pitch AP) . W^T  with W's fragments in wf; refills wf
// with Wnext's fragments slice by slice (always a valid matrix: the code stays branch-free, so hipcc's
// counted vmcnt waits let the prefetch stay in flight across the epilogue).
// lane l of wave w holds C[4 (l >> 4) + i][64 w + 16 j + (l & 15)] in acc[j][i]
__device__ __forceinline__ void gemm16(const bf16_t* A, WFrag& wf, const bf16_t* __restrict__ Wnext, f4 acc[4]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = l & 15, lg = l >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
  const uint4* nrow = frag_base(Wnext);
#pragma unroll
  for (int ks = 0; ks < DIM / 32; ++ks) {
    const bf8v a = ld_frag(A + lr * AP + ks * 32 + 8 * lg);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf8v b;
      __builtin_memcpy(&b, &wf[ks][j], 16);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[ks][j] = nrow[(ks * 4 + j) * 64];
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
  __shared__ float Pp[4][kResMax][DIM];   // b1, b2, LN gamma, LN beta of every block (fp32)
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, lr = l & 15, lg = l >> 4;
  const long r0 = static_cast<long>(blockIdx.x) * RB;
  const bool save = sv_x != nullptr;
  // the small per-block parameters are staged once: a global load of them inside the block loop would
  // make hipcc drain the in-flight weight prefetch (vmcnt(0)) at every epilogue
  for (int i = tid; i < nblk * DIM; i += 256) {
    const int k = i / DIM, c = i - k * DIM;
    Pp[0][k][c] = bf2f(static_cast<const bf16_t*>(w.b1[k])[c]);
    Pp[1][k][c] = bf2f(static_cast<const bf16_t*>(w.b2[k])[c]);
    Pp[2][k][c] = w.g[k][c];
    Pp[3][k][c] = w.be[k][c];
  }
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    const float v = r0 + r < R ? ldv(x0, x0_dt, (r0 + r) * DIM + c) : 0.f;
    X[r][c] = v;
    Xb[r * AP + c] = f2bf(v);
  }
  WFrag wf;
  const bf16_t* pk = static_cast<const bf16_t*>(w.pk);
  load_w(pk, wf);
  __syncthreads();
  for (int k = 0; k < nblk; ++k) {
    const long so = static_cast<long>(k) * R * DIM;
    if (save)
      for (int i = tid; i < RB * DIM; i += 256) {
        const int r = i / DIM, c = i - r * DIM;
        if (r0 + r < R) sv_x[so + (r0 + r) * DIM + c] = Xb[r * AP + c];
      }
    f4 acc[4];
    gemm16(Xb, wf, pk + (2 * k + 1) * kImg, acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
      const float b = Pp[0][k][c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lg + i;
        const bf16_t h = f2bf(fmaxf(acc[j][i] + b, 0.f));
        Hb[r * AP + c] = h;
        if (save && r0 + r < R) sv_h[so + (r0 + r) * DIM + c] = h;
      }
    }
    __syncthreads();
    gemm16(Hb, wf, pk + 2 * (k + 1 < nblk ? k + 1 : 0) * kImg, acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
      const float b = Pp[1][k][c];
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
        const float y = xh * Pp[2][k][c] + Pp[3][k][c];
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
  __shared__ float Pg[kResMax][DIM];   // LN gamma of every block
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, lr = l & 15, lg = l >> 4;
  const long r0 = static_cast<long>(blockIdx.x) * RB;
  for (int i = tid; i < RB * DIM; i += 256) {
    const int r = i / DIM, c = i - r * DIM;
    dX[r][c] = r0 + r < R ? dout[(r0 + r) * DIM + c] : 0.f;
  }
  for (int i = tid; i < nblk * DIM; i += 256) Pg[i / DIM][i % DIM] = w.g[i / DIM][i % DIM];
  // saved activations this lane reads, fetched one phase ahead (branch-free, rows clamped to R - 1 and
  // masked): LN backward rows 4 wv + rr, columns 4 l .. 4 l + 3; the ReLU mask at the MFMA C positions
  const long rl = R - 1;
  float xh_n[4][4], rs_n[4];
  auto load_ln = [&](int k) {
    const long so = static_cast<long>(k) * R * DIM;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const long row = r0 + 4 * wv + rr < R ? r0 + 4 * wv + rr : rl;
      const float4 v = *reinterpret_cast<const float4*>(sv_xhat + so + row * DIM + 4 * l);
      xh_n[rr][0] = v.x; xh_n[rr][1] = v.y; xh_n[rr][2] = v.z; xh_n[rr][3] = v.w;
      rs_n[rr] = sv_rstd[static_cast<long>(k) * R + row];
    }
  };
  WFrag wf;
  load_ln(nblk - 1);
  const bf16_t* pk = static_cast<const bf16_t*>(w.pk);
  load_w(pk + 2 * (nblk - 1) * kImg, wf);
  __syncthreads();
  for (int k = nblk - 1; k >= 0; --k) {
    const long so = static_cast<long>(k) * R * DIM;
    // LayerNorm backward (rows >= R have dX = 0 and contribute nothing)
    float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r = 4 * wv + rr;
      const bool ok = r0 + r < R;
      const float rs = ok ? rs_n[rr] : 0.f;
      float xh[4], dxh[4], m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 4 * l + e;
        xh[e] = ok ? xh_n[rr][e] : 0.f;
        const float d = dX[r][c];
        pg[e] += d * xh[e];
        pb[e] += d;
        dxh[e] = d * Pg[k][c];
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
    // ReLU mask of this block's hidden activation at the lane's C positions, requested before the
    // GEMM (whose weight prefetch would otherwise sit in front of it in the load queue)
    bf16_t hm[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long row = r0 + 4 * lg + i < R ? r0 + 4 * lg + i : rl;
        hm[j][i] = sv_h[so + row * DIM + 64 * wv + 16 * j + lr];
      }
    __syncthreads();
    for (int c = tid; c < 2 * DIM; c += 256)
      ln_part[(static_cast<long>(blockIdx.x) * nblk + k) * 2 * DIM + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    // dH = (dS W2) * (h > 0)     (packed W2^T)
    f4 acc[4];
    gemm16(Ab, wf, pk + (2 * k + 1) * kImg, acc);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 64 * wv + 16 * j + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lg + i;
        const bool ok = r0 + r < R;
        const bool act = ok && bf2f(hm[j][i]) > 0.f;
        const bf16_t d = f2bf(act ? acc[j][i] : 0.f);
        Hd[r * AP + c] = d;
        if (ok) sv_dh[so + (r0 + r) * DIM + c] = d;
      }
    }
    load_ln(k > 0 ? k - 1 : 0);   // next block's LN inputs, ahead of the second GEMM's weight prefetch
    __syncthreads();
    // dX = dS + dH W1    (packed W1^T)
    gemm16(Hd, wf, pk + 2 * (k > 0 ? k - 1 : 0) * kImg, acc);
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

// packed image m (blockIdx.y) of the 2 nblk GEMM operands: thread = one 16-B fragment piece
// p = ((wave * 8 + ks) * 4 + j) * 64 + lane  <-  op[64 wave + 16 j + (lane & 15)][32 ks + 8 (lane >> 4) .. +8]
// op = W1_k / W2_k (forward), W2_k^T / W1_k^T (backward: a strided gather of 8 elements)
__global__ __launch_bounds__(256) void resmlp_pack_kernel(const ResMlpW w, int bwd, bf16_t* __restrict__ dst) {
  const int m = blockIdx.y, k = m >> 1, second = m & 1;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int l = p & 63, j = (p >> 6) & 3, ks = (p >> 8) & 7, wv = p >> 11;
  const int n = 64 * wv + 16 * j + (l & 15), k0 = 32 * ks + 8 * (l >> 4);
  uint4 v;
  if (!bwd) {
    const bf16_t* src = static_cast<const bf16_t*>(second ? w.w2[k] : w.w1[k]);
    v = *reinterpret_cast<const uint4*>(src + n * DIM + k0);
  } else {
    const bf16_t* src = static_cast<const bf16_t*>(second ? w.w1[k] : w.w2[k]);
    uint32_t q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      q[e] = static_cast<uint32_t>(src[(k0 + 2 * e) * DIM + n]) | (static_cast<uint32_t>(src[(k0 + 2 * e + 1) * DIM + n]) << 16);
    v = make_uint4(q[0], q[1], q[2], q[3]);
  }
  reinterpret_cast<uint4*>(dst + m * kImg)[p] = v;
}

}  // namespace

void resmlp_fwd(const void* x0, int x0_dt, const ResMlpW& w, int nblk, float* out, bf16_t* sv_x, bf16_t* sv_h,
                float* sv_xhat, float* sv_rstd, long R, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(resmlp_fwd_kernel, dim3(static_cast<unsigned>((R + RB - 1) / RB)), dim3(256), 0, s, x0, x0_dt, w,
                     nblk, out, sv_x, sv_h, sv_xhat, sv_rstd, R);
}

void resmlp_pack(const ResMlpW& w, int nblk, bool bwd, bf16_t* dst, hipStream_t s) {
  hipLaunchKernelGGL(resmlp_pack_kernel, dim3(static_cast<unsigned>(kImg / 8 / 256), 2 * nblk), dim3(256), 0, s, w,
                     bwd ? 1 : 0, dst);
}

int resmlp_row_blocks(long R) { return static_cast<int>((R + RB - 1) / RB); }

void resmlp_bwd(const float* dout, const ResMlpW& w, int nblk, const bf16_t* sv_h, const float* sv_xhat,
                const float* sv_rstd, bf16_t* sv_dy, bf16_t* sv_dh, float* ln_part, float* dx0, long R, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(resmlp_bwd_kernel, dim3(static_cast<unsigned>((R + RB - 1) / RB)), dim3(256), 0, s, dout, w, nblk,
                     sv_h, sv_xhat, sv_rstd, sv_dy, sv_dh, ln_part, dx0, R);
}

}  // namespace as
