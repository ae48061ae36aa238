// fp32 GEMM with a fused epilogue for the fp32 learner step's linears (SURVEY K3/K4 in fp32; the reference's
// fc_block, distar/ctools/torch_utils/network/nn_module.py:231-270, and the post-LN transformer's projections,
// distar/agent/default/model/module_utils.py:130-139), on the exact-f32 MFMA v_mfma_f32_32x32x2_f32:
//
//   Y[m, n] = epi( sum_k A[m, k] * B[n, k] )      A [M, K] row-major, B [N, K] row-major (nn.Linear weight)
//   epi(v)  = act( v + bias[n] + res[m, n] )        act: none / ReLU
//           | (v + bias[n]) * [res[m, n] > 0]       (ACT_DRELU: an input gradient masked by the ReLU output res)
//
// Forward Y = act(X W^T + b) takes B = W; the input gradient dX = dY W takes B = W^T (a [K, N] copy), and can
// add the residual gradient handed over by a closing LayerNorm (GradLink) or apply the previous layer's ReLU
// mask in the same epilogue - the separate [M, N] elementwise pass of a library GEMM disappears.
//
// Tiling as conv3x3_f32.hip (its implicit GEMM with one tap): 128 x BN tile per 256-thread workgroup, K-steps
// of BK = 16 (APPLESTAR_GEMM_F32_BK=32 selects 32-deep stages: half the barriers, but 74 KB of LDS leaves 2
// workgroups per CU and measured 2-8 % slower on the learner's shapes, r3i),
// register-staged LDS double buffer, BK + 4-float LDS rows (conflict-free float4 fragment reads: rows r * 36
// and r * 20 fall in distinct 4-bank groups over each ds_read_b128 lane group), k-slot kk of lane half h =
// column (BK / 2) h + kk, XCD-aware tile order.  K % 4 == 0; a K tail reads zeros through the buffer range
// check.
#include <cstdlib>
#include <string>

#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(16))) float f16v;

constexpr int kOOB = 0x7ffffff0;

// GF_ABL: timing-ablation bits for tools/native/gemm_f32_ablation.cpp only (1: no K-step loads after the first,
// 2: no MFMAs (fragments kept live), 4: no epilogue stores); 0 in every library build
#ifndef GF_ABL
#define GF_ABL 0
#endif

template <int BN_, int BK_>
struct GemmF32Cfg {
  static constexpr int BM = 128, BN = BN_, BK = BK_, NT = 256;
  static constexpr int CH = BK / 4;            // 16-B pieces per tile row
  static constexpr int KH = BK / 2;            // floats per lane half per stage (= MFMA k-steps)
  // 16-B piece idx -> (tile row, column piece): 8 consecutive pieces = 8 rows of one column piece, so the 8
  // contiguous lanes of a ds_write_b128 bank group hit disjoint banks (as conv3x3_f32.hip)
  static __device__ __forceinline__ int prow(int idx) { return (idx & 7) + 8 * (idx / (8 * CH)); }
  static __device__ __forceinline__ int pcol(int idx) { return (idx >> 3) % CH; }
  static constexpr int WN = BN_ >= 128 ? 2 : 1, WM = 4 / WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 32, FN = TN / 32;
  static constexpr int P = BK + 4;
  static constexpr int A_IT = BM * CH / NT;
  static constexpr int B_PIECES = BN * CH;
  static constexpr int B_IT = (B_PIECES + NT - 1) / NT;
  static constexpr int STAGE = (BM + BN) * P;
  // split staging (SPLIT == 2): row = three bf16 planes of BK values + 16 B pad, 3 BK / 2 + 4 dwords (28 / 52:
  // the 16 rows of a ds_read_b128 lane group start on 16 distinct 4-bank groups)
  static constexpr int PS = 3 * BK / 2 + 4;
  static constexpr int STAGE_S = (BM + BN) * PS;
  static constexpr int SMEM = STAGE > STAGE_S ? STAGE : STAGE_S;
};

// SPLIT: 0 exact-f32 MFMA; 1 bf16x6 split in registers after the fp32 LDS read; 2 bf16x6 split once at staging
// (three bf16 planes per LDS row, fragments read as bf16x8)
template <int BN, int BK, int SPLIT>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                       const float* __restrict__ bias, const float* __restrict__ res,
                                                       float* __restrict__ out, long M, int N, int K, int act) {
  using C = GemmF32Cfg<BN, BK>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SPLIT == 2 ? C::STAGE_S : C::STAGE)];
  const int ntn = (N + BN - 1) / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int tn = wg % ntn;
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a), 0, static_cast<int>(M * K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(b), 0, static_cast<int>(static_cast<long>(N) * K * 4), 0x00020000);

  int a_base[C::A_IT], a_row[C::A_IT], a_c4[C::A_IT];
#pragma unroll
  for (int i = 0; i < C::A_IT; ++i) {
    const int idx = tid + i * C::NT;
    a_row[i] = C::prow(idx);
    a_c4[i] = C::pcol(idx);
    const long m = m0 + a_row[i];
    a_base[i] = m < M ? static_cast<int>(m * K) : -1;
  }
  int b_base[C::B_IT];
#pragma unroll
  for (int i = 0; i < C::B_IT; ++i) {
    const int idx = tid + i * C::NT;
    const int n = C::prow(idx);
    b_base[i] = (idx < C::B_PIECES && n0 + n < N) ? (n0 + n) * K : -1;
  }

  uint4 ra[1][C::A_IT], rb[1][C::B_IT];
  auto load_regs = [&](int kt, uint4 (&xa)[C::A_IT], uint4 (&xb)[C::B_IT]) {
    const int k0 = kt * C::BK;
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const int k = k0 + 4 * a_c4[i];
      const int off = (a_base[i] >= 0 && k < K) ? (a_base[i] + k) * 4 : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0);
      xa[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int k = k0 + 4 * C::pcol(tid + i * C::NT);
      const int off = (b_base[i] >= 0 && k < K) ? (b_base[i] + k) * 4 : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(br, off, 0, 0);
      xb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_lds = [&](int s, const uint4 (&xa)[C::A_IT], const uint4 (&xb)[C::B_IT]) {
    if constexpr (SPLIT == 2) {
      unsigned* A = reinterpret_cast<unsigned*>(smem) + s * C::STAGE_S;
      unsigned* Bs = A + C::BM * C::PS;
      auto put = [](unsigned* d, const uint4& v) {
        uint2 s0, s1, s2;
        split4(v, s0, s1, s2);
        *reinterpret_cast<uint2*>(d) = s0;
        *reinterpret_cast<uint2*>(d + C::BK / 2) = s1;
        *reinterpret_cast<uint2*>(d + C::BK) = s2;
      };
#pragma unroll
      for (int i = 0; i < C::A_IT; ++i) put(A + a_row[i] * C::PS + 2 * a_c4[i], xa[i]);
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i) {
        const int idx = tid + i * C::NT;
        if (C::B_PIECES % C::NT == 0 || idx < C::B_PIECES) put(Bs + C::prow(idx) * C::PS + 2 * C::pcol(idx), xb[i]);
      }
    } else {
      float* A = smem + s * C::STAGE;
      float* Bs = A + C::BM * C::P;
#pragma unroll
      for (int i = 0; i < C::A_IT; ++i) *reinterpret_cast<uint4*>(A + a_row[i] * C::P + 4 * a_c4[i]) = xa[i];
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i) {
        const int idx = tid + i * C::NT;
        if (C::B_PIECES % C::NT == 0 || idx < C::B_PIECES)
          *reinterpret_cast<uint4*>(Bs + C::prow(idx) * C::P + 4 * C::pcol(idx)) = xb[i];
      }
    }
  };

  f16v acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  auto compute = [&](int cur) {
    if constexpr (SPLIT == 2) {
      // chunk c of lane half h: columns 16 c + 8 h .. + 7 = the MFMA's k-slots 8 h .. 8 h + 7
      const unsigned* A = reinterpret_cast<const unsigned*>(smem) + cur * C::STAGE_S;
      const unsigned* Bs = A + C::BM * C::PS;
#pragma unroll
      for (int c = 0; c < C::BK / 16; ++c) {
        Split3 sa[C::FM], sb[C::FN];
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
          const unsigned* p = A + (wm * C::TM + 32 * i + l32) * C::PS + 8 * c + 4 * h;
#pragma unroll
          for (int q = 0; q < 3; ++q) sa[i].p[q] = *reinterpret_cast<const u32v4*>(p + q * (C::BK / 2));
        }
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const unsigned* p = Bs + (wn * C::TN + 32 * j + l32) * C::PS + 8 * c + 4 * h;
#pragma unroll
          for (int q = 0; q < 3; ++q) sb[j].p[q] = *reinterpret_cast<const u32v4*>(p + q * (C::BK / 2));
        }
        if constexpr ((GF_ABL & 2) != 0) {
#pragma unroll
          for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int q = 0; q < 3; ++q) asm volatile("" ::"v"(sa[i].p[q]));
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) asm volatile("" ::"v"(sb[j].p[q]));
        } else {
#pragma unroll
          for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
        }
      }
      return;
    }
    const float* A = smem + cur * C::STAGE;
    const float* Bs = A + C::BM * C::P;
    float af[C::FM][C::KH], bfr[C::FN][C::KH];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const float* p = A + (wm * C::TM + 32 * i + l32) * C::P + C::KH * h;
#pragma unroll
      for (int q = 0; q < C::KH / 4; ++q) {
        const float4 u = *reinterpret_cast<const float4*>(p + 4 * q);
        af[i][4 * q] = u.x; af[i][4 * q + 1] = u.y; af[i][4 * q + 2] = u.z; af[i][4 * q + 3] = u.w;
      }
    }
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const float* p = Bs + (wn * C::TN + 32 * j + l32) * C::P + C::KH * h;
#pragma unroll
      for (int q = 0; q < C::KH / 4; ++q) {
        const float4 u = *reinterpret_cast<const float4*>(p + 4 * q);
        bfr[j][4 * q] = u.x; bfr[j][4 * q + 1] = u.y; bfr[j][4 * q + 2] = u.z; bfr[j][4 * q + 3] = u.w;
      }
    }
    if constexpr (SPLIT == 1) {
      // bf16x6 (split_mfma.h): lane half h's 8-float run of a fragment is the MFMA's k-slots 8h..8h+7
#pragma unroll
      for (int c = 0; c < C::KH / 8; ++c) {
        Split3 sa[C::FM], sb[C::FN];
#pragma unroll
        for (int i = 0; i < C::FM; ++i) sa[i] = split8(*reinterpret_cast<const float(*)[8]>(&af[i][8 * c]));
#pragma unroll
        for (int j = 0; j < C::FN; ++j) sb[j] = split8(*reinterpret_cast<const float(*)[8]>(&bfr[j][8 * c]));
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < C::KH; ++kk)
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(bfr[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    }
  };

  // LDS buffer kt & 1 holds K-step kt, the registers kt + 1 (a second register set two K-steps ahead
  // measured no faster and made the unrolled loop copy the accumulators)
  const int KT = (K + C::BK - 1) / C::BK;
  load_regs(0, ra[0], rb[0]);
  store_lds(0, ra[0], rb[0]);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT && ((GF_ABL & 1) == 0 || kt == 0)) load_regs(kt + 1, ra[0], rb[0]);
    compute(cur);
    if (kt + 1 < KT) store_lds(cur ^ 1, ra[0], rb[0]);
    __syncthreads();
  }

  if constexpr ((GF_ABL & 4) != 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) t += acc[i][j][e];
    if (t != 12345.678f) return;
  }
  // operands enter the MFMA swapped (B fragment first), so the accumulator is the transposed tile: lane l32 is
  // output row m, registers 4 g .. 4 g + 3 are four consecutive columns n - one 16-B load / store per group
  // (the untransposed tile stored one float per lane and register: 64 stores per tile, 35 % of a K = 256 GEMM)
  const bool vec = (N & 3) == 0;
#pragma unroll
  for (int i = 0; i < C::FM; ++i) {
    const long m = m0 + wm * C::TM + 32 * i + l32;
    if (m >= M) continue;
    float* orow = out + m * N;
    const float* rrow = res ? res + m * N : nullptr;
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * C::TN + 32 * j + 8 * g + 4 * h;
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (vec && n + 3 < N) {
          if (bias) {
            const float4 bv = *reinterpret_cast<const float4*>(bias + n);
            v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
          }
          if (rrow) {
            const float4 rv = *reinterpret_cast<const float4*>(rrow + n);
            const float r[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = act == ACT_DRELU ? (r[q] > 0.f ? v[q] : 0.f) : v[q] + r[q];
          }
          if (act == ACT_RELU)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
          *reinterpret_cast<float4*>(orow + n) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (n + q >= N) continue;
            float x = v[q] + (bias ? bias[n + q] : 0.f);
            if (rrow) x = act == ACT_DRELU ? (rrow[n + q] > 0.f ? x : 0.f) : x + rrow[n + q];
            if (act == ACT_RELU) x = fmaxf(x, 0.f);
            orow[n + q] = x;
          }
        }
      }
    }
  }
}

// split-MFMA mode: LDS-DMA ring + register split (f32_pipe.h)
// NW = 8: the 256 x 256 tile (8 waves of 128 x 64, two per SIMD, one workgroup per CU)
template <int BN, int NS, int BK, bool STAGED = false, int BM = 128, int NW = 4, bool DMA_MID = false>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 2 : 3) void gemm_f32_pipe_kernel(
    const float* __restrict__ a, const float* __restrict__ b, const float* __restrict__ bias,
    const float* __restrict__ res, float* __restrict__ out, long M, int N, int K, int act) {
  using C = pipe::Cfg<BN, NS, BK, BM, NW>;
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
  const pipe::i32x4 ar = pipe::rsrc(a, M * K * 4), br = pipe::rsrc(b, static_cast<long>(N) * K * 4);
  // this lane's DMA piece per chunk (column piece p of its row, swizzled)
  int a_off[C::A_PW], a_k[C::A_PW], b_off[C::B_PW], b_k[C::B_PW];
#pragma unroll
  for (int c = 0; c < C::A_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane), p = C::dma_piece(row, lane);
    const long m = m0 + row;
    a_k[c] = 4 * p;
    a_off[c] = m < M ? static_cast<int>((m * K + 4 * p) * 4) : -1;
  }
#pragma unroll
  for (int c = 0; c < C::B_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane), p = C::dma_piece(row, lane);
    b_k[c] = 4 * p;
    b_off[c] = n0 + row < N ? ((n0 + row) * K + 4 * p) * 4 : -1;
  }
  auto asrc = [&](int c, int kt) {
    return a_off[c] >= 0 && kt * BK + a_k[c] < K ? a_off[c] + kt * BK * 4 : pipe::kOOB;
  };
  auto bsrc = [&](int c, int kt) {
    return b_off[c] >= 0 && kt * BK + b_k[c] < K ? b_off[c] + kt * BK * 4 : pipe::kOOB;
  };
  f16v acc[C::FM][C::FN];
  pipe::mainloop<C, decltype(asrc), decltype(bsrc), false, DMA_MID>(smem, ar, br, (K + BK - 1) / BK, asrc, bsrc, acc);
  if constexpr (STAGED) {
    pipe::store_tile_staged<C, float>(acc, smem[0], out, bias, res, M, N, m0, n0, act);
  } else {
    const int wm = wid / C::WN, wn = wid % C::WN;
    pipe::store_tile<C::FM, C::FN>(acc, out, bias, res, M, N, m0 + wm * C::TM, n0 + wn * C::TN, act);
  }
}

// row-coalesced LDS-staged epilogue (pipe::store_tile_staged): 1-4 % faster on the learner's GEMM shapes
// (profiles/r4p_gemm_f32_staged_epilogue.txt); APPLESTAR_GEMM_F32_STAGED=0 restores the register stores
bool f32_staged() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_GEMM_F32_STAGED");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// Few-row products: fewer than 128 of the pipe kernel's 128 x 64 tiles (the heads, the scalar encoder and the
// value projections on ~400 rows; the location head's 1-row-per-sample GEMVs).  There the 128-row tile leaves
// most of the chip idle and the library's smallest kernels floor at ~19 us per call.  Here a 256-thread
// workgroup owns one 32 x 32 output tile and its four waves split the reduction (wave w takes K-steps w, w + 4,
// ...): operands stream from global memory (L2-resident at these sizes) straight into registers, KU K-steps of
// loads in flight per wave, no LDS staging; the four partial tiles meet once in LDS and wave 0 applies the same
// fused epilogue (bias, ReLU, residual, ReLU-mask) - so a linear's bias / ReLU / ReLU-mask hand-off work here too.
//   lane (l32, h): A row m0 + l32 and B row n0 + l32, the 8 floats at k = 16 kt + 8 h .. + 7 of K-step kt;
//   split mode: one bf16x6 product per K-step (k-slots 8 h .. 8 h + 7 of lane half h);
//   exact mode: eight v_mfma_f32_32x32x2_f32, instruction t pairing k = 16 kt + 8 h + t on both operands.
// The accumulator is the transposed tile (lane = output row), stored by pipe::store_tile.
template <int KU, int SPLIT>
__global__ __launch_bounds__(256) void gemm_f32_small_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ res, float* __restrict__ out,
                                                             long M, int N, int K, int act, int tiles_n) {
  __shared__ float red[3][16][64];
  const int tn = blockIdx.x % tiles_n;
  const long tm = blockIdx.x / tiles_n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const long m = tm * 32 + l32;
  const int n = tn * 32 + l32;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a), 0,
                                                                      static_cast<int>(M * K * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), 0,
                                                                      static_cast<int>(static_cast<long>(N) * K * 4),
                                                                      0x00020000);
  const int a_row = m < M ? static_cast<int>(m * K) * 4 : -1;
  const int b_row = n < N ? n * K * 4 : -1;
  const int KT = (K + 15) / 16;
  // pieces past K (K % 4 == 0) or of rows past M / N read zeros (out-of-range buffer offset)
  auto off = [&](int row, int kt, int q) {
    const int k = 16 * kt + 8 * h + 4 * q;
    return row >= 0 && k < K ? row + 4 * k : kOOB;
  };
  float4 ra[KU][2], rb[KU][2];
  auto load = [&](int u, int kt) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const auto va = __builtin_amdgcn_raw_buffer_load_b128(ar, off(a_row, kt, q), 0, 0);
      const auto vb = __builtin_amdgcn_raw_buffer_load_b128(br, off(b_row, kt, q), 0, 0);
      ra[u][q] = make_float4(__uint_as_float(va[0]), __uint_as_float(va[1]), __uint_as_float(va[2]),
                             __uint_as_float(va[3]));
      rb[u][q] = make_float4(__uint_as_float(vb[0]), __uint_as_float(vb[1]), __uint_as_float(vb[2]),
                             __uint_as_float(vb[3]));
    }
  };
  // this wave's K-steps: w, w + 4, w + 8, ...
  const int nk = KT > w ? (KT - w + 3) / 4 : 0;
#pragma unroll
  for (int u = 0; u < KU; ++u) load(u, w + 4 * u);
  f16v acc[1][1];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[0][0][e] = 0.f;
  for (int i0 = 0; i0 < nk; i0 += KU) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (i0 + u >= nk) break;
      const float va[8] = {ra[u][0].x, ra[u][0].y, ra[u][0].z, ra[u][0].w,
                           ra[u][1].x, ra[u][1].y, ra[u][1].z, ra[u][1].w};
      const float vb[8] = {rb[u][0].x, rb[u][0].y, rb[u][0].z, rb[u][0].w,
                           rb[u][1].x, rb[u][1].y, rb[u][1].z, rb[u][1].w};
      load(u, w + 4 * (i0 + u + KU));     // refill the slot just read (zeros past the last K-step)
      if constexpr (SPLIT) {
        acc[0][0] = mfma_x6(split8(vb), split8(va), acc[0][0]);
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(vb[t], va[t], acc[0][0], 0, 0, 0);
      }
    }
  }
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w - 1][e][lane] = acc[0][0][e];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[0][0][e] += red[0][e][lane] + red[1][e][lane] + red[2][e][lane];
    pipe::store_tile<1, 1>(acc, out, bias, res, M, N, tm * 32, tn * 32, act);
  }
}

// bf16 form of the few-row kernel (the mixed-precision step's heads / scalar encoder / value projections):
// bf16 operands, one v_mfma_f32_32x32x16_bf16 per K-step, fp32 accumulation and epilogue, bf16 output.
//   out[m, n] = bf16( act( sum_k A[m, k] B[n, k] + bias[n] (+ res[m, n] | * [res[m, n] > 0]) ) )
// lane (l32, h): A row m0 + l32 / B row n0 + l32, the 8 bf16 at k = 16 kt + 8 h (one 16-B load each).
template <int KU>
__global__ __launch_bounds__(256) void gemm_bf16_small_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                              const float* __restrict__ bias,
                                                              const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                                                              long M, int N, int K, int act, int tiles_n) {
  __shared__ float red[3][16][64];
  const int tn = blockIdx.x % tiles_n;
  const long tm = blockIdx.x / tiles_n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const long m = tm * 32 + l32;
  const int n = tn * 32 + l32;
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a), 0,
                                                                      static_cast<int>(M * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(b), 0,
                                                                      static_cast<int>(static_cast<long>(N) * K * 2),
                                                                      0x00020000);
  const int a_row = m < M ? static_cast<int>(m * K) * 2 : -1;
  const int b_row = n < N ? n * K * 2 : -1;
  const int KT = (K + 15) / 16;
  auto off = [&](int row, int kt) {
    const int k = 16 * kt + 8 * h;
    return row >= 0 && k < K ? row + 2 * k : kOOB;      // K % 8 == 0: a piece never straddles K
  };
  u32v4 ra[KU], rb[KU];
  auto load = [&](int u, int kt) {
    const auto va = __builtin_amdgcn_raw_buffer_load_b128(ar, off(a_row, kt), 0, 0);
    const auto vb = __builtin_amdgcn_raw_buffer_load_b128(br, off(b_row, kt), 0, 0);
    ra[u] = u32v4{va[0], va[1], va[2], va[3]};
    rb[u] = u32v4{vb[0], vb[1], vb[2], vb[3]};
  };
  const int nk = KT > w ? (KT - w + 3) / 4 : 0;
#pragma unroll
  for (int u = 0; u < KU; ++u) load(u, w + 4 * u);
  f16v acc[1][1];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[0][0][e] = 0.f;
  for (int i0 = 0; i0 < nk; i0 += KU) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      if (i0 + u >= nk) break;
      const u32v4 va = ra[u], vb = rb[u];
      load(u, w + 4 * (i0 + u + KU));
      acc[0][0] = mfma_bf16(vb, va, acc[0][0]);
    }
  }
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w - 1][e][lane] = acc[0][0][e];
  }
  __syncthreads();
  if (w != 0) return;
  // transposed tile: lane = output row m0 + l32, register 4 g + q = column n0 + 8 g + 4 h + q
  if (m >= M) return;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n0 = tn * 32 + 8 * g + 4 * h;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * g + q;
      v[q] = acc[0][0][e] + red[0][e][lane] + red[1][e][lane] + red[2][e][lane];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nn = n0 + q;
      if (nn >= N) continue;
      float x = v[q] + (bias ? bias[nn] : 0.f);
      if (res) {
        const float r = bf2f(res[m * N + nn]);
        x = act == ACT_DRELU ? (r > 0.f ? x : 0.f) : x + r;
      }
      if (act == ACT_RELU) x = fmaxf(x, 0.f);
      out[m * N + nn] = f2bf(x);
    }
  }
}

int& pipe_variant_ref() {
  static int v = [] {
    const char* e = std::getenv("APPLESTAR_F32_PIPE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
int pipe_variant() { return pipe_variant_ref(); }

template <int BN>
void launch_pipe(const float* a, const float* b, const float* bias, const float* res, float* out, long M, int N, int K,
                 int act, hipStream_t s, long nwg) {
  const dim3 g(static_cast<unsigned>(nwg)), blk(256);
  // ring depth / K-step measured on the entity-transformer shapes (profiles/r3x_pipe_variants.txt): 3 stages of 16
  // (48 KB: 3 workgroups per CU) beat 4 x 16 by 4-7 %, 2 x 32 by 7-10 %, 3 x 32 and 6 x 16 (1 workgroup per CU)
  // by 25-40 % - occupancy, not ring depth, hides the DMA latency
  switch (pipe_variant()) {
    case 3:
      if constexpr (BN == 128) {
        if (N % 256 == 0) {    // 256 x 256 tiles, 8 waves
          const dim3 g8(static_cast<unsigned>((M + 255) / 256 * (N / 256))), blk8(512);
          hipLaunchKernelGGL((gemm_f32_pipe_kernel<256, 3, 16, true, 256, 8>), g8, blk8, 0, s, a, b, bias, res, out, M,
                             N, K, act);
          break;
        }
      }
      hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 3, 16, true>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act);
      break;
    case 4:
      if constexpr (BN == 128) {
        if (N % 256 == 0) {    // 256 x 256 tiles, 8 waves, 4-stage ring (128 KB)
          const dim3 g8(static_cast<unsigned>((M + 255) / 256 * (N / 256))), blk8(512);
          hipLaunchKernelGGL((gemm_f32_pipe_kernel<256, 4, 16, true, 256, 8>), g8, blk8, 0, s, a, b, bias, res, out, M,
                             N, K, act);
          break;
        }
      }
      hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 3, 16, true>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act);
      break;
    case 5:      // DMA issue between the K-step's MFMA halves
      hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 3, 16, true, 128, 4, true>), g, blk, 0, s, a, b, bias, res, out, M, N,
                         K, act);
      break;
    case 1: hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 4, 16>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act); break;
    case 2: hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 2, 32>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act); break;
    default:
      if (f32_staged())
        hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 3, 16, true>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act);
      else
        hipLaunchKernelGGL((gemm_f32_pipe_kernel<BN, 3, 16>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act);
  }
}

template <int BN, int BK>
void launch_gemm(const float* a, const float* b, const float* bias, const float* res, float* out, long M, int N, int K,
                 int act, hipStream_t s) {
  const long nwg = (M + 127) / 128 * ((N + BN - 1) / BN);
  if (nwg == 0) return;
  const int mode = f32_mfma_mode();
  if (mode == 1)
    launch_pipe<BN>(a, b, bias, res, out, M, N, K, act, s, nwg);
  else if (mode == 3)
    hipLaunchKernelGGL((gemm_f32_kernel<BN, BK, 2>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a, b, bias, res,
                       out, M, N, K, act);
  else if (mode == 2)
    hipLaunchKernelGGL((gemm_f32_kernel<BN, BK, 1>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a, b, bias, res,
                       out, M, N, K, act);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<BN, BK, 0>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a, b, bias, res,
                       out, M, N, K, act);
}

int gemm_bk() {
  static const int bk = [] {
    const char* e = std::getenv("APPLESTAR_GEMM_F32_BK");
    return e && std::atoi(e) == 32 ? 32 : 16;
  }();
  return bk;
}

int& mode_ref() {
  static int mode = [] {
    const char* e = std::getenv("APPLESTAR_F32_MFMA");
    const std::string v = e ? e : "";
    return v == "exact" ? 0 : (v == "regsplit" ? 2 : (v == "stagesplit" ? 3 : 1));
  }();
  return mode;
}

}  // namespace

int f32_mfma_mode() { return mode_ref(); }
void set_f32_pipe_variant(int v) { pipe_variant_ref() = v; }

int& conv_variant_ref() {
  static int v = [] {
    // default 3 (DMA issue between the MFMA halves): 1.0-1.8 % faster on the learner's 128-channel convs
    // (profiles/r5d_dma_mid_variants.jsonl); 0 = the plain ring
    const char* e = std::getenv("APPLESTAR_F32_CONV_PIPE");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}
int f32_conv_variant() { return conv_variant_ref(); }
void set_f32_conv_variant(int v) { conv_variant_ref() = v; }
void set_f32_mfma_mode(int mode) { mode_ref() = mode >= 0 && mode <= 3 ? mode : 1; }

void gemm_bf16_small(const void* a, const void* b, const float* bias, const void* res, void* out, long M, int N, int K,
                     int act, hipStream_t s) {
  const int tn = (N + 31) / 32;
  hipLaunchKernelGGL((gemm_bf16_small_kernel<4>), dim3(static_cast<unsigned>((M + 31) / 32 * tn)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(a), static_cast<const bf16_t*>(b), bias,
                     static_cast<const bf16_t*>(res), static_cast<bf16_t*>(out), M, N, K, act, tn);
}

bool gemm_f32_is_small(long M, int N) { return (M + 127) / 128 * ((N + 63) / 64) < 128; }

void gemm_f32(const float* a, const float* b, const float* bias, const float* res, float* out, long M, int N, int K,
              int act, hipStream_t s) {
  if (gemm_f32_is_small(M, N)) {
    const int tn = (N + 31) / 32;
    const dim3 g(static_cast<unsigned>((M + 31) / 32 * tn)), blk(256);
    if (f32_mfma_mode() == 0)
      hipLaunchKernelGGL((gemm_f32_small_kernel<4, 0>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act, tn);
    else
      hipLaunchKernelGGL((gemm_f32_small_kernel<4, 1>), g, blk, 0, s, a, b, bias, res, out, M, N, K, act, tn);
    return;
  }
  const bool deep = gemm_bk() == 32 && K >= 64;
  if (N % 128 == 0 && (M + 127) / 128 * (N / 128) >= 1024) {
    if (deep) launch_gemm<128, 32>(a, b, bias, res, out, M, N, K, act, s);
    else launch_gemm<128, 16>(a, b, bias, res, out, M, N, K, act, s);
  } else if (N > 32) {
    if (deep) launch_gemm<64, 32>(a, b, bias, res, out, M, N, K, act, s);
    else launch_gemm<64, 16>(a, b, bias, res, out, M, N, K, act, s);
  } else {
    launch_gemm<32, 16>(a, b, bias, res, out, M, N, K, act, s);
  }
}

}  // namespace as
