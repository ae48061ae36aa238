// bf16 GEMM with a fused epilogue for the mixed-precision step's large linears (SURVEY K3/K4 in bf16; the
// reference's fc_block, distar/ctools/torch_utils/network/nn_module.py:231-270, and the entity transformer's
// projections and FFN, distar/agent/default/model/module_utils.py:130-139):
//
//   Y[m, n] = bf16( epi( sum_k A[m, k] B[n, k] ) )   A [M, K], B [N, K] bf16 row-major, fp32 accumulation
//   epi(v)  = act( v + bias[n] + res[m, n] ) | (v + bias[n]) * [res[m, n] > 0] (ACT_DRELU)     act: none / ReLU
//
// Forward takes B = W, the input gradient dX = dY W takes B = W^T (the derived transposed form) and adds the
// residual gradient a closing LayerNorm hands over (GradLink) in the epilogue.  The main loop is the fp32 step's
// LDS-DMA ring (f32_pipe.h) in its bf16 form: a 128 x BN tile per 256-thread workgroup, stages of 32 bf16 (64-B
// rows, swizzled 16-B slots), three stages in flight (48 KB: three workgroups per CU), one barrier per stage,
// two 32x32x16 bf16 MFMAs per fragment pair and stage.  K % 8 == 0 (a 16-B piece never straddles K; pieces past
// K read zeros through the buffer range check).  Products of fewer than 128 tiles take gemm_bf16_small.
#include <cstdlib>

#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(16))) float f16v;

// the LDS-staged (row-coalesced) epilogue; -DBF16_STAGED=0 keeps the per-lane register stores (A/B builds)
#ifndef BF16_STAGED
#define BF16_STAGED 1
#endif

// wave tile epilogue (transposed accumulators as pipe::store_tile): 4 bf16 per (i, j, g) in one 8-B store
template <int FM, int FN>
__device__ __forceinline__ void store_tile_bf16(const f16v (&acc)[FM][FN], bf16_t* __restrict__ out,
                                                const float* __restrict__ bias, const bf16_t* __restrict__ res, long M,
                                                int N, long mw, int nw, int act) {
  const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const bool vec = (N & 3) == 0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long m = mw + 32 * i + l32;
    if (m >= M) continue;
    bf16_t* orow = out + m * N;
    const bf16_t* rrow = res ? res + m * N : nullptr;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = nw + 32 * j + 8 * g + 4 * h;
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (vec && n + 3 < N) {
          if (bias) {
            const float4 bv = *reinterpret_cast<const float4*>(bias + n);
            v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
          }
          if (rrow) {
            const uint2 rv = *reinterpret_cast<const uint2*>(rrow + n);
            const float r[4] = {__uint_as_float(rv.x << 16), __uint_as_float(rv.x & 0xffff0000u),
                                __uint_as_float(rv.y << 16), __uint_as_float(rv.y & 0xffff0000u)};
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = act == ACT_DRELU ? (r[q] > 0.f ? v[q] : 0.f) : v[q] + r[q];
          }
          if (act == ACT_RELU)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
          *reinterpret_cast<uint2*>(orow + n) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (n + q >= N) continue;
            float x = v[q] + (bias ? bias[n + q] : 0.f);
            if (rrow) x = act == ACT_DRELU ? (bf2f(rrow[n + q]) > 0.f ? x : 0.f) : x + bf2f(rrow[n + q]);
            if (act == ACT_RELU) x = fmaxf(x, 0.f);
            orow[n + q] = f2bf(x);
          }
        }
      }
    }
  }
}

__device__ __forceinline__ bool bf16_staged_epilogue() { return BF16_STAGED != 0; }

// BKF: the ring's K-step in fp32 units of pipe::Cfg (a stage row = 4 BKF bytes = 2 BKF bf16)
template <int BN, int NS, int BKF, int BM = 128>
__global__ __launch_bounds__(256, NS * (BN + BM) * BKF * 4 <= 56 * 1024 ? 3 : (NS * (BN + BM) * BKF * 4 <= 80 * 1024 ? 2 : 1))
void gemm_bf16_pipe_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, const float* __restrict__ bias,
                           const bf16_t* __restrict__ res, bf16_t* __restrict__ out, long M, int N, int K, int act) {
  using C = pipe::Cfg<BN, NS, BKF, BM>;
  constexpr int BKB = 2 * BKF;                 // bf16 per stage row
  __shared__ __attribute__((aligned(16))) char s0[C::STAGE], s1[C::STAGE], s2[NS > 2 ? C::STAGE : 16],
      s3[NS > 3 ? C::STAGE : 16];
  char* const all[4] = {s0, s1, s2, s3};
  char* smem[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) smem[i] = all[i];
  const int ntn = (N + BN - 1) / BN;
  const int wg = pipe::xcd_remap();
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const pipe::i32x4 ar = pipe::rsrc(a, M * K * 2), br = pipe::rsrc(b, static_cast<long>(N) * K * 2);
  // this lane's DMA piece per chunk: 8 bf16 (column piece p of its row, swizzled)
  int a_off[C::A_PW], a_k[C::A_PW], b_off[C::B_PW], b_k[C::B_PW];
#pragma unroll
  for (int c = 0; c < C::A_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane), p = C::dma_piece(row, lane);
    const long m = m0 + row;
    a_k[c] = 8 * p;
    a_off[c] = m < M ? static_cast<int>((m * K + 8 * p) * 2) : -1;
  }
#pragma unroll
  for (int c = 0; c < C::B_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane), p = C::dma_piece(row, lane);
    b_k[c] = 8 * p;
    b_off[c] = n0 + row < N ? ((n0 + row) * K + 8 * p) * 2 : -1;
  }
  auto asrc = [&](int c, int kt) {
    return a_off[c] >= 0 && kt * BKB + a_k[c] < K ? a_off[c] + kt * BKB * 2 : pipe::kOOB;
  };
  auto bsrc = [&](int c, int kt) {
    return b_off[c] >= 0 && kt * BKB + b_k[c] < K ? b_off[c] + kt * BKB * 2 : pipe::kOOB;
  };
  f16v acc[C::FM][C::FN];
  pipe::mainloop<C, decltype(asrc), decltype(bsrc), true>(smem, ar, br, (K + BKB - 1) / BKB, asrc, bsrc, acc);
  if (bf16_staged_epilogue()) {
    pipe::store_tile_staged<C, bf16_t>(acc, smem[0], out, bias, res, M, N, m0, n0, act);
  } else {
    const int wm = wid / C::WN, wn = wid % C::WN;
    store_tile_bf16<C::FM, C::FN>(acc, out, bias, res, M, N, m0 + wm * C::TM, n0 + wn * C::TN, act);
  }
}

int bf16_pipe_variant() {
  static const int v = [] {
    const char* e = std::getenv("APPLESTAR_BF16_PIPE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

template <int BN>
void launch_bf16(const bf16_t* a, const bf16_t* b, const float* bias, const bf16_t* res, bf16_t* out, long M, int N,
                 int K, int act, hipStream_t s) {
  const long nwg = (M + 127) / 128 * ((N + BN - 1) / BN);
  if (nwg == 0) return;
  const dim3 g(static_cast<unsigned>(nwg)), blk(256);
  if constexpr (BN == 128) {
    // 256-row tiles: each wave owns 128 x 64 (four A and two B fragments per chunk: 0.75 LDS reads per MFMA
    // instead of 1.0 - the 128 x 128 tile's fragment reads alone fill the CU's LDS port at full MFMA rate)
    const int v = bf16_pipe_variant();
    if (v == 3 || v == 4) {
      const dim3 g2(static_cast<unsigned>((M + 255) / 256 * (N / 128)));
      if (v == 3)
        hipLaunchKernelGGL((gemm_bf16_pipe_kernel<128, 3, 16, 256>), g2, blk, 0, s, a, b, bias, res, out, M, N, K, act);
      else
        hipLaunchKernelGGL((gemm_bf16_pipe_kernel<128, 2, 32, 256>), g2, blk, 0, s, a, b, bias, res, out, M, N, K, act);
      return;
    }
  }
  switch (bf16_pipe_variant()) {
    case 1: hipLaunchKernelGGL((gemm_bf16_pipe_kernel<BN, 2, 32>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act); break;
    case 2: hipLaunchKernelGGL((gemm_bf16_pipe_kernel<BN, 4, 16>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act); break;
    default: hipLaunchKernelGGL((gemm_bf16_pipe_kernel<BN, 3, 16>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act);
  }
}

}  // namespace

void gemm_bf16(const void* a, const void* b, const float* bias, const void* res, void* out, long M, int N, int K,
               int act, hipStream_t s) {
  if (gemm_f32_is_small(M, N)) {
    gemm_bf16_small(a, b, bias, res, out, M, N, K, act, s);
    return;
  }
  const auto* A = static_cast<const bf16_t*>(a);
  const auto* B = static_cast<const bf16_t*>(b);
  const auto* R = static_cast<const bf16_t*>(res);
  auto* O = static_cast<bf16_t*>(out);
  if (N % 128 == 0) launch_bf16<128>(A, B, bias, R, O, M, N, K, act, s);
  else if (N > 32) launch_bf16<64>(A, B, bias, R, O, M, N, K, act, s);
  else launch_bf16<32>(A, B, bias, R, O, M, N, K, act, s);
}

}  // namespace as
