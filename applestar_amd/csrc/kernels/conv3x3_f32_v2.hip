// 3 x 3 / pad 1 convolution, fp32 operands, fp32-accurate bf16x6 split MFMAs (split_mfma.h), second design
// (experimental, selected by variant): BOTH operands staged through one LDS-DMA ring per workgroup.
//
// conv3x3_f32_psb_kernel (gemm_f32_psb.hip) streams the pre-split weight planes straight from L2 into each wave's
// registers: the two waves that share a weight fragment both load it, so a 128 x 128 tile moves 8 KB of activation
// rows + 24 KB of weight planes per 16-deep K-step (2.7 GB of L2 -> CU traffic per ResBlock conv).  Here a stage
// holds the activation rows (8 KB, fp32, the ring's swizzled image) AND the tile's weight planes for the K-step
// (12 KB: 4 column blocks x 3 planes x 1 KB, in MFMA fragment order, read back with one conflict-free ds_read_b128
// per plane): 20 KB per K-step, every byte loaded once per workgroup.
//
// Wave layouts: WM x WN waves over the 128 x 128 tile.  4 x 1: each wave owns 32 rows x 128 columns (one
// activation fragment split per K-step - no fragment is split twice in the workgroup - and four weight fragments
// from LDS); 2 x 2: 64 x 64 per wave (the psb kernel's layout).  NS: ring depth (2-4 stages of 20 KB).
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

using pipe::f16v;
using pipe::i32x4;

constexpr int kV2BM = 128;

// SUB: 16-deep MFMA K-steps per ring stage (1: 20 KB stages; 2: 40 KB, half the barriers and DMA bookkeeping)
// CONV: the implicit im2col of a 3x3 / pad 1 conv over NHWC x [B, H, W, Cin] (K = 9 Cin); else a dense GEMM with
// A = x [Mg, Kg] row-major (Kg % 4 == 0; the pre-split planes are zero past Kg)
template <int WM, int NS, int SUB = 1, bool CONV = true, int kV2BN = 128>
__global__ __launch_bounds__(256, 2) void conv3x3_f32_v2_kernel(const float* __restrict__ x,
                                                                const u32v4* __restrict__ bs,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ res,
                                                                float* __restrict__ out, int B, int H, int W,
                                                                int Cin, int Cout, int act, const pipe::Epi2 e2,
                                                                long Mg, int Kg) {
  constexpr int BK = 16 * SUB;
  constexpr int kV2A = kV2BM * BK * 4;                  // activation rows per stage (BK fp32 per row)
  constexpr int kV2B1 = (kV2BN / 32) * 3 * 1024;        // weight planes of one 16-deep K-step (12 KB)
  constexpr int kV2Stage = kV2A + SUB * kV2B1;
  using CA = pipe::Cfg<kV2BN, NS, BK, kV2BM, 4>;     // the activation half of the ring: rows, swizzle, DMA pieces
  constexpr int WN = 4 / WM, TM = kV2BM / WM, TN = kV2BN / WN, FM = TM / 32, FN = TN / 32;
  // DMA pieces per wave per stage: A_PW activation pieces; the QB weight pieces are dealt round-robin (wave w takes
  // pieces w, w + 4, ...: 3 each for 128 columns, 2 / 1 for 64 - the waits are then vmcnt(0), NS = 2)
  constexpr int A_PW = kV2A / 1024 / 4, QB = SUB * kV2B1 / 1024, B_PW = (QB + 3) / 4;
  static_assert(QB % 4 == 0 || NS == 2, "uneven weight pieces need the 2-stage ring");
  __shared__ __attribute__((aligned(16))) char ring[NS * kV2Stage];
  const int HW = H * W;
  const long M = CONV ? static_cast<long>(B) * HW : Mg;
  const int K = CONV ? 9 * Cin : Kg, KT16 = (K + 15) / 16, KT = (K + BK - 1) / BK;
  const int ntn = Cout / kV2BN;
  const int wg = pipe::xcd_remap();
  const long m0 = static_cast<long>(wg / ntn) * kV2BM;
  const int n0 = (wg % ntn) * kV2BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int l32 = lane & 31, h = lane >> 5;
  const i32x4 xr = pipe::rsrc(x, CONV ? M * Cin * 4 : M * K * 4);
  const long nbt = Cout / 32;
  const i32x4 br = pipe::rsrc(bs, nbt * KT16 * 3 * 1024);
  // activation pieces: the implicit im2col of conv3x3_f32_psb_kernel (a lane's piece = 4 channels of its pixel
  // shifted by the K-step's tap, zeros outside the image)
  int a_pix[A_PW], a_ok[A_PW], a_c[A_PW];
#pragma unroll
  for (int c = 0; c < A_PW; ++c) {
    const int row = CA::dma_row(wid + 4 * c, lane);
    const long m = m0 + row;
    a_c[c] = 4 * CA::dma_piece(row, lane);
    a_pix[c] = static_cast<int>(m);
    a_ok[c] = 0;
    if (!CONV) {
      a_ok[c] = m < M;
    } else if (m < M) {
      const int rem = static_cast<int>(m % HW);
      const int yy = rem / W, xx = rem - yy * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y2 = yy + t / 3 - 1, x2 = xx + t % 3 - 1;
        a_ok[c] |= (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W) << t;
      }
    }
  }
  // weight pieces: stage chunk q = wid + 4 c = (16-deep sub-step q / QB1, column block q % QB1 / 3, plane q % 3)
  constexpr int QB1 = kV2B1 / 1024;
  int b_off[B_PW];
#pragma unroll
  for (int c = 0; c < B_PW; ++c) {
    const int q = wid + 4 * c, sub = q / QB1, r = q % QB1;
    b_off[c] = static_cast<int>(((n0 / 32 + r / 3) * KT16 * 3 + sub * 3 + r % 3) * 1024 + 16 * lane);
  }
  auto stage = [&](int kt) { return ring + (kt % NS) * kV2Stage; };
  auto issue = [&](int kt) {
    char* st = stage(kt);
    const int k0 = kt * BK;
    if constexpr (CONV) {
      const int tap = k0 / Cin, c0 = k0 - tap * Cin;
      const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
#pragma unroll
      for (int c = 0; c < A_PW; ++c)
        pipe::dma16(xr, st + (wid + 4 * c) * 1024,
                    kt < KT && ((a_ok[c] >> tap) & 1) ? ((a_pix[c] + shift) * Cin + c0 + a_c[c]) * 4 : pipe::kOOB);
    } else {
#pragma unroll
      for (int c = 0; c < A_PW; ++c)
        pipe::dma16(xr, st + (wid + 4 * c) * 1024,
                    kt < KT && a_ok[c] && k0 + a_c[c] < K ? (a_pix[c] * K + k0 + a_c[c]) * 4 : pipe::kOOB);
    }
#pragma unroll
    for (int c = 0; c < B_PW; ++c)
      if (QB % 4 == 0 || wid + 4 * c < QB)            // wave-uniform
        pipe::dma16(br, st + kV2A + (wid + 4 * c) * 1024, kt < KT ? b_off[c] + kt * SUB * 3 * 1024 : pipe::kOOB);
  };
  f16v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  for (int kt = 0; kt < KT; ++kt) {
    // this wave's pieces of step kt landed (the NS - 2 later steps may fly); the barrier: everyone's did, and
    // everyone finished reading step kt - 1, whose slot step kt + NS - 1 refills
    pipe::wait_vm<(NS - 2) * (A_PW + B_PW)>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(kt + NS - 1);
    const char* st = stage(kt);
#pragma unroll
    for (int sub = 0; sub < SUB; ++sub) {
      Split3 sa[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) sa[i] = pipe::frag<CA>(st, wm * TM + 32 * i + l32, 4 * sub + 2 * h);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const char* bp = st + kV2A + sub * kV2B1 + (wn * FN + j) * 3 * 1024 + 16 * lane;
        Split3 sb;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const uint4 u = *reinterpret_cast<const uint4*>(bp + p * 1024);
          sb.p[p] = u32v4{u.x, u.y, u.z, u.w};
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) acc[i][j] = mfma_x6(sb, sa[i], acc[i][j]);
      }
    }
  }
  pipe::wait_vm<0>();
  pipe::store_tile<FM, FN>(acc, out, bias, res, M, Cout, m0 + wm * TM, n0 + wn * TN, act, e2);
}

template <int WM, int NS, int SUB = 1, int BN = 128>
void launch_v2(const float* x, const void* ws, const float* bias, const float* res, const pipe::Epi2& e2, float* out,
               int B, int H, int W, int Cin, int Cout, int act, hipStream_t s) {
  const long M = static_cast<long>(B) * H * W;
  const long nwg = (M + kV2BM - 1) / kV2BM * (Cout / BN);
  hipLaunchKernelGGL((conv3x3_f32_v2_kernel<WM, NS, SUB, true, BN>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0,
                     s, x, static_cast<const u32v4*>(ws), bias, res, out, B, H, W, Cin, Cout, act, e2, 0L, 0);
}

}  // namespace

// variant: 0 = 4 x 1 waves, 3 stages; 1 = 4 x 1, 4 stages; 2 = 4 x 1, 2 stages; 3 = 2 x 2, 3 stages;
// 4 = 4 x 1, 2 stages of 32-deep K (Cin % 32 == 0)
void conv3x3_f32_v2(const float* x, const void* wsplit, const float* bias, const float* res, const float* res2,
                    long res2_rows, const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int act,
                    int variant, hipStream_t s) {
  if (static_cast<long>(B) * H * W == 0) return;
  pipe::Epi2 e2;
  e2.res2 = res2;
  e2.res2_rows = res2_rows;
  e2.mask = mask;
  if (Cout % 128 != 0) {        // 64 / 32 output channels: 128 x 64 / 128 x 32 tiles (each wave 32 rows), 2 stages
    // 32-deep K-steps per stage (half the barriers / DMA bookkeeping): 32 outputs 858 -> 743 us on the location
    // head's 76 x 80 64 -> 32 conv, but 64 outputs slower (574 -> 607, 634 -> 729 us; profiles/r10r_conv_narrow_sub*.jsonl)
    // - so by default for 32 outputs only (APPLESTAR_CONV_V2_NARROW_SUB = 1: never, 2: both widths)
    static const int sub_mode = [] {
      const char* e = std::getenv("APPLESTAR_CONV_V2_NARROW_SUB");
      return e ? std::atoi(e) : 0;
    }();
    const bool sub2 = Cin % 32 == 0 && (sub_mode == 2 || (sub_mode == 0 && Cout % 64 != 0));
    if (sub2) {
      if (Cout % 64 == 0) launch_v2<4, 2, 2, 64>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
      else launch_v2<4, 2, 2, 32>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
      return;
    }
    if (Cout % 64 == 0) launch_v2<4, 2, 1, 64>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
    else launch_v2<4, 2, 1, 32>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
    return;
  }
  switch (variant) {
    case 1: launch_v2<4, 4>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s); break;
    case 2: launch_v2<4, 2>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s); break;
    case 3: launch_v2<2, 3>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s); break;
    case 4:
      if (Cin % 32 == 0) {
        launch_v2<4, 2, 2>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
        break;
      }
      launch_v2<4, 2>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s);
      break;
    default: launch_v2<4, 3>(x, wsplit, bias, res, e2, out, B, H, W, Cin, Cout, act, s); break;
  }
}

// dense GEMM out[M, N] = act(A[M, K] B[N, K]^T + bias (+ res)) on the same ring (B pre-split by presplit_b;
// N % 128 == 0, K % 4 == 0): variant 2 = 4 x 1 waves, 2 stages (0: 3 stages; 4: 32-deep K-steps, K % 32 == 0)
void gemm_f32_v2(const float* a, const void* bsplit, const float* bias, const float* res, float* out, long M, int N,
                 int K, int act, int variant, hipStream_t s) {
  const long nwg = (M + kV2BM - 1) / kV2BM * (N / 128);
  if (nwg == 0) return;
  const pipe::Epi2 e2;
  const auto* bs = static_cast<const u32v4*>(bsplit);
  const dim3 g(static_cast<unsigned>(nwg)), b(256);
  if (variant == 0)
    hipLaunchKernelGGL((conv3x3_f32_v2_kernel<4, 3, 1, false>), g, b, 0, s, a, bs, bias, res, out, 1, 1, 1, 1, N, act,
                       e2, M, K);
  else if (variant == 4 && K % 32 == 0)
    hipLaunchKernelGGL((conv3x3_f32_v2_kernel<4, 2, 2, false>), g, b, 0, s, a, bs, bias, res, out, 1, 1, 1, 1, N, act,
                       e2, M, K);
  else
    hipLaunchKernelGGL((conv3x3_f32_v2_kernel<4, 2, 1, false>), g, b, 0, s, a, bs, bias, res, out, 1, 1, 1, 1, N, act,
                       e2, M, K);
}

}  // namespace as
