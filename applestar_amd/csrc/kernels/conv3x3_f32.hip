// 3x3 / stride 1 / pad 1 convolution in fp32 (the fp32 learner step, like-for-like with the reference's fp32
// convolutions: spatial_encoder.py:74-86, res_block.py:50-65, action_arg_head.py:417-446), NHWC, on the
// exact-f32 MFMA v_mfma_f32_32x32x2_f32 (gfx950 has no xf32/TF32 mode), with bias / residual / ReLU (and the
// input-gradient form's ReLU mask) fused into the epilogue.
//
//   out[m, n] = act( bias[n] + res[m, n] + sum_{tap, c} x[shift_tap(m), c] * w[n, tap, c] )
//
// Implicit GEMM as the bf16 kernel (conv3x3.hip): M = B*H*W output pixels, N = Cout, K = 9*Cin tap-major
// (the memory order of a channels_last [Cout, Cin, 3, 3] weight).  K-step = one tap x 16 input channels:
// the A tile is 128 pixels x 16 channels gathered from the shifted pixels (one 16-B buffer load per 4
// channels; taps outside the image read zeros through the buffer range check), the B tile BN x 16 weight
// rows.  Register-staged double buffer, one barrier per K-step.
//
// 32x32x2 f32 MFMA: lane l holds A[row l&31][k l>>5] and B[k l>>5][col l&31] (one f32 each), C[row (r&3) +
// 8(r>>2) + 4(l>>5)][col l&31] in 16 accumulators.  The k-slot assignment is free as long as A and B agree:
// k-step kk of a 16-channel K-step gives lane half h channel 8h + kk, so a lane's 8 k-steps of a fragment are
// 8 consecutive floats of one LDS row (two ds_read_b128).  LDS rows are 20 floats: 20 = 4 mod 16, the 16
// rows read by a 16-lane group land on 16 distinct 4-bank groups.  Staging pieces (16 B) are dealt so that
// the 8 contiguous lanes of a ds_write_b128 bank group write 8 different rows of one 4-float column (row
// pitches 20 r mod 32 for r = 0..7 are disjoint 4-bank windows; row-major dealing put two rows' 16 floats
// on overlapping banks: 2-way on every staging write).  The epilogue stores straight from the
// accumulators: 32 lanes write 32 consecutive channels (128 B) of one pixel.
#include <algorithm>
#include <cstdlib>

#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(16))) float f16v;

constexpr int kOOB = 0x7ffffff0;

template <int BN_>
struct ConvF32Cfg {
  // 16-B piece idx -> (tile row, 4-float column): 8 consecutive pieces = 8 rows of one column
  static __device__ __forceinline__ int prow(int idx) { return (idx & 7) + 8 * (idx >> 5); }
  static __device__ __forceinline__ int pcol(int idx) { return (idx >> 3) & 3; }
  static constexpr int BM = 128, BN = BN_, BK = 16, NT = 256;
  static constexpr int WN = BN_ >= 128 ? 2 : 1;   // waves along N
  static constexpr int WM = 4 / WN;                // waves along M
  static constexpr int TM = BM / WM, TN = BN / WN; // wave tile
  static constexpr int FM = TM / 32, FN = TN / 32; // 32x32 MFMA tiles per wave
  static constexpr int P = BK + 4;                 // LDS row pitch (floats)
  static constexpr int A_IT = BM * (BK / 4) / NT;  // 16-B pieces per thread
  static constexpr int B_PIECES = BN * (BK / 4);
  static constexpr int B_IT = (B_PIECES + NT - 1) / NT;
  static constexpr int STAGE = (BM + BN) * P;      // floats
  // split staging (SPLIT == 2, split_mfma.h): row = three bf16 planes of 16 channels + 16 B pad = 28 dwords
  // (the 16 rows of a ds_read_b128 lane group start on 16 distinct 4-bank groups)
  static constexpr int PS = 28;
  static constexpr int STAGE_S = (BM + BN) * PS;
  static constexpr int SMEM = STAGE > STAGE_S ? STAGE : STAGE_S;
  static_assert(A_IT * NT == BM * (BK / 4), "A tile pieces");
};

// SPLIT: 0 exact-f32 MFMA; 1 bf16x6 split in registers after the fp32 LDS read; 2 bf16x6 split once at staging
template <int BN, int SPLIT>
__global__ __launch_bounds__(256) void conv3x3_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ res, float* __restrict__ out,
                                                          int B, int H, int W, int Cin, int Cout, int act) {
  using C = ConvF32Cfg<BN>;
  __shared__ __attribute__((aligned(16))) float smem[2 * (SPLIT == 2 ? C::STAGE_S : C::STAGE)];

  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  const int K = 9 * Cin;
  const int ntn = (Cout + BN - 1) / BN;
  // XCD-aware bijective remap (8 XCDs, round-robin dispatch): consecutive M-tiles share input halo rows
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int tn = wg % ntn;
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x), 0, static_cast<int>(M * Cin * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(w), 0, static_cast<int>(static_cast<long>(Cout) * K * 4), 0x00020000);

  // A pieces: row = pixel of the tile, ch4 = which 4-channel group of the 16-channel K-step
  int a_pix[C::A_IT], a_row[C::A_IT], a_c4[C::A_IT], a_ok[C::A_IT];
#pragma unroll
  for (int i = 0; i < C::A_IT; ++i) {
    const int idx = tid + i * C::NT;
    a_row[i] = C::prow(idx);
    a_c4[i] = C::pcol(idx);
    const long m = m0 + a_row[i];
    a_pix[i] = static_cast<int>(m);
    a_ok[i] = 0;
    if (m < M) {
      const int rem = static_cast<int>(m % HW);
      const int yy = rem / W, xx = rem - yy * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y2 = yy + t / 3 - 1, x2 = xx + t % 3 - 1;
        a_ok[i] |= (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W) << t;
      }
    }
  }
  int b_off[C::B_IT];
#pragma unroll
  for (int i = 0; i < C::B_IT; ++i) {
    const int idx = tid + i * C::NT;
    const int n = C::prow(idx), c4 = C::pcol(idx);
    b_off[i] = (idx < C::B_PIECES && n0 + n < Cout) ? ((n0 + n) * K + 4 * c4) * 4 : kOOB;
  }

  uint4 ra[C::A_IT], rb[C::B_IT];
  auto load_regs = [&](int kt) {
    const int k0 = kt * C::BK;
    const int tap = k0 / Cin, c0 = k0 - tap * Cin;
    const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const int off = ((a_ok[i] >> tap) & 1) ? ((a_pix[i] + shift) * Cin + c0 + 4 * a_c4[i]) * 4 : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int off = b_off[i] == kOOB ? kOOB : b_off[i] + k0 * 4;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_lds = [&](int s) {
    if constexpr (SPLIT == 2) {
      unsigned* A = reinterpret_cast<unsigned*>(smem) + s * C::STAGE_S;
      unsigned* Bs = A + C::BM * C::PS;
      auto put = [](unsigned* d, const uint4& v) {
        uint2 s0, s1, s2;
        split4(v, s0, s1, s2);
        *reinterpret_cast<uint2*>(d) = s0;
        *reinterpret_cast<uint2*>(d + 8) = s1;
        *reinterpret_cast<uint2*>(d + 16) = s2;
      };
#pragma unroll
      for (int i = 0; i < C::A_IT; ++i) put(A + a_row[i] * C::PS + 2 * a_c4[i], ra[i]);
#pragma unroll
      for (int i = 0; i < C::B_IT; ++i) {
        const int idx = tid + i * C::NT;
        if (C::B_PIECES % C::NT == 0 || idx < C::B_PIECES) put(Bs + C::prow(idx) * C::PS + 2 * C::pcol(idx), rb[i]);
      }
      return;
    }
    float* A = smem + s * C::STAGE;
    float* Bs = A + C::BM * C::P;
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) *reinterpret_cast<uint4*>(A + a_row[i] * C::P + 4 * a_c4[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int idx = tid + i * C::NT;
      if (C::B_PIECES % C::NT == 0 || idx < C::B_PIECES)
        *reinterpret_cast<uint4*>(Bs + C::prow(idx) * C::P + 4 * C::pcol(idx)) = rb[i];
    }
  };

  f16v acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int KT = K / C::BK;      // Cin % 16 == 0 (host check): every K-step lies inside one tap
  load_regs(0);
  store_lds(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_regs(kt + 1);
    if constexpr (SPLIT == 2) {
      // lane half h: channels 8 h .. 8 h + 7 of the K-step = the MFMA's k-slots 8 h .. 8 h + 7
      const unsigned* A = reinterpret_cast<const unsigned*>(smem) + cur * C::STAGE_S;
      const unsigned* Bs = A + C::BM * C::PS;
      Split3 sa[C::FM], sb[C::FN];
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const unsigned* p = A + (wm * C::TM + 32 * i + l32) * C::PS + 4 * h;
#pragma unroll
        for (int q = 0; q < 3; ++q) sa[i].p[q] = *reinterpret_cast<const u32v4*>(p + 8 * q);
      }
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const unsigned* p = Bs + (wn * C::TN + 32 * j + l32) * C::PS + 4 * h;
#pragma unroll
        for (int q = 0; q < 3; ++q) sb[j].p[q] = *reinterpret_cast<const u32v4*>(p + 8 * q);
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
      if (kt + 1 < KT) store_lds(cur ^ 1);
      __syncthreads();
      continue;
    }
    const float* A = smem + cur * C::STAGE;
    const float* Bs = A + C::BM * C::P;
    float af[C::FM][8], bfr[C::FN][8];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const float* p = A + (wm * C::TM + 32 * i + l32) * C::P + 8 * h;
      const float4 u0 = *reinterpret_cast<const float4*>(p), u1 = *reinterpret_cast<const float4*>(p + 4);
      af[i][0] = u0.x; af[i][1] = u0.y; af[i][2] = u0.z; af[i][3] = u0.w;
      af[i][4] = u1.x; af[i][5] = u1.y; af[i][6] = u1.z; af[i][7] = u1.w;
    }
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const float* p = Bs + (wn * C::TN + 32 * j + l32) * C::P + 8 * h;
      const float4 u0 = *reinterpret_cast<const float4*>(p), u1 = *reinterpret_cast<const float4*>(p + 4);
      bfr[j][0] = u0.x; bfr[j][1] = u0.y; bfr[j][2] = u0.z; bfr[j][3] = u0.w;
      bfr[j][4] = u1.x; bfr[j][5] = u1.y; bfr[j][6] = u1.z; bfr[j][7] = u1.w;
    }
    if constexpr (SPLIT == 1) {
      // bf16x6 (split_mfma.h): lane half h's 8 channels are the MFMA's k-slots 8h..8h+7
      Split3 sa[C::FM], sb[C::FN];
#pragma unroll
      for (int i = 0; i < C::FM; ++i) sa[i] = split8(af[i]);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) sb[j] = split8(bfr[j]);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(bfr[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_lds(cur ^ 1);
    __syncthreads();
  }

  // operands enter the MFMA swapped (B fragment first), so the accumulator is the transposed tile: lane l32 is
  // output row m, registers 4 g .. 4 g + 3 are four consecutive columns n - one 16-B load / store per group
  // (the untransposed tile stored one float per lane and register: 64 stores per tile, 35 % of a K = 256 GEMM)
  const bool vec = (Cout & 3) == 0;
#pragma unroll
  for (int i = 0; i < C::FM; ++i) {
    const long m = m0 + wm * C::TM + 32 * i + l32;
    if (m >= M) continue;
    float* orow = out + m * Cout;
    const float* rrow = res ? res + m * Cout : nullptr;
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * C::TN + 32 * j + 8 * g + 4 * h;
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (vec && n + 3 < Cout) {
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
            if (n + q >= Cout) continue;
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

// split-MFMA mode: the LDS-DMA ring of f32_pipe.h with the A rows gathered per tap (a lane's DMA piece is 4
// channels of its row's shifted pixel; taps outside the image read zeros through the buffer range check)
// NW = 8: 256-pixel tiles on 8 waves (each wave 64 x 64 as in the 4-wave tile), the B (weight) stage shared by
// twice the MFMA work
template <int BN, int NS, int BM = 128, bool STAGED = false, int NW = 4, bool DMA_MID = false>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 2 : (BM == 128 ? 3 : 2))
void conv3x3_f32_pipe_kernel(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
                             const float* __restrict__ res, float* __restrict__ out, int B, int H, int W, int Cin,
                             int Cout, int act, const pipe::Epi2 e2 = pipe::Epi2()) {
  using C = pipe::Cfg<BN, NS, 16, BM, NW>;
  __shared__ __attribute__((aligned(16))) char s0[C::STAGE], s1[C::STAGE], s2[NS > 2 ? C::STAGE : 16],
      s3[NS > 3 ? C::STAGE : 16];
  char* const all[4] = {s0, s1, s2, s3};
  char* smem[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) smem[i] = all[i];
  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  const int K = 9 * Cin;
  const int ntn = (Cout + BN - 1) / BN;
  const int wg = pipe::xcd_remap();
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const pipe::i32x4 xr = pipe::rsrc(x, M * Cin * 4), wr = pipe::rsrc(w, static_cast<long>(Cout) * K * 4);
  int a_pix[C::A_PW], a_ok[C::A_PW], a_c[C::A_PW], b_off[C::B_PW];
#pragma unroll
  for (int c = 0; c < C::A_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane);
    const long m = m0 + row;
    a_c[c] = 4 * C::dma_piece(row, lane);
    a_pix[c] = static_cast<int>(m);
    a_ok[c] = 0;
    if (m < M) {
      const int rem = static_cast<int>(m % HW);
      const int yy = rem / W, xx = rem - yy * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y2 = yy + t / 3 - 1, x2 = xx + t % 3 - 1;
        a_ok[c] |= (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W) << t;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < C::B_PW; ++c) {
    const int row = C::dma_row(wid + C::NW * c, lane);
    b_off[c] = n0 + row < Cout ? ((n0 + row) * K + 4 * C::dma_piece(row, lane)) * 4 : -1;
  }
  const int KT = K / 16;      // Cin % 16 == 0 (host check): every K-step lies inside one tap
  auto asrc = [&](int c, int kt) {
    const int k0 = kt * 16, tap = k0 / Cin, c0 = k0 - tap * Cin;
    const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
    return kt < KT && ((a_ok[c] >> tap) & 1) ? ((a_pix[c] + shift) * Cin + c0 + a_c[c]) * 4 : pipe::kOOB;
  };
  auto bsrc = [&](int c, int kt) { return b_off[c] >= 0 && kt < KT ? b_off[c] + kt * 64 : pipe::kOOB; };
  f16v acc[C::FM][C::FN];
  pipe::mainloop<C, decltype(asrc), decltype(bsrc), false, DMA_MID>(smem, xr, wr, KT, asrc, bsrc, acc);
  if constexpr (STAGED) {
    pipe::store_tile_staged<C, float>(acc, smem[0], out, bias, res, M, Cout, m0, n0, act);
  } else {
    const int wm = wid / C::WN, wn = wid % C::WN;
    pipe::store_tile<C::FM, C::FN>(acc, out, bias, res, M, Cout, m0 + wm * C::TM, n0 + wn * C::TN, act, e2);
  }
}

// the LDS-staged epilogue measured -3 ... +6 % on the conv shapes (profiles/r4p_conv_f32_staged_epilogue.txt):
// opt-in (APPLESTAR_CONV_F32_STAGED=1)
bool conv_f32_staged() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_CONV_F32_STAGED");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

// 256-row tiles for the narrow (32-channel) outputs: each wave then owns 64 x 32 (two A fragments per B
// fragment instead of one) - APPLESTAR_CONV_F32_N32_BM256=1 (A/B switch)
bool conv_n32_bm256() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_CONV_F32_N32_BM256");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

// ---- narrow convolutions (Cin 16 / 32, Cout a multiple of 16: the value encoder's spatial tower) as direct
// convolutions on 16x16x32 split MFMAs with no LDS.  The ring kernel's 128 x 32 tile wastes half of every MFMA at
// Cout 16 and pads K = 144 to 256 (16 -> 16 at 76 x 80: 50 TF/s forward, 30 TF/s weight gradient).  Here a wave
// owns 16 pixels x 16 NT output channels and computes C^T[cout][pixel] = W[cout][:] . im2col[pixel][:]: the
// weight rows (A, cout = lr, k = 32 ks + 8 lg + t) are split once into registers and kept for the wave's whole
// pixel range; the im2col operand (B, pixel = lr) is 8 consecutive channels of one tap - two 16-B loads per lane,
// zero outside the image - split in registers; each lane ends with 4 consecutive channels of one pixel (16-B
// NHWC stores).  K = 9 Cin is padded to whole 32-deep steps (144 -> 160 at Cin 16).
typedef __attribute__((ext_vector_type(4))) float nf4;
__device__ __forceinline__ nf4 nmfma_x6(const Split3& a, const Split3& b, nf4 c) {
  auto mm = [](u32v4 x, u32v4 y, nf4 acc) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(x), as_bf(y), acc, 0, 0, 0); };
  c = mm(a.p[1], b.p[1], c);
  c = mm(a.p[0], b.p[2], c);
  c = mm(a.p[2], b.p[0], c);
  c = mm(a.p[0], b.p[1], c);
  c = mm(a.p[1], b.p[0], c);
  return mm(a.p[0], b.p[0], c);
}

template <int CIN, int NT>
__global__ __launch_bounds__(256) void conv3x3_f32_narrow_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ res, float* __restrict__ out,
                                                                int B, int H, int W, int Cout, int act, long ntiles) {
  constexpr int K = 9 * CIN, KS = (K + 31) / 32;
  const int lane = threadIdx.x & 63, lg = lane >> 4, lr = lane & 15;
  const int ncb = Cout / (16 * NT);                       // output-channel blocks
  const long gw = static_cast<long>(blockIdx.x) * 4 + (threadIdx.x >> 6), nw = static_cast<long>(gridDim.x) * 4;
  const int cb = static_cast<int>(gw % ncb);
  const int n_base = cb * 16 * NT;
  Split3 wf[NT][KS];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 32 * ks + 8 * lg;
      float f[8];
      if (k0 < K) {
        const float4* src = reinterpret_cast<const float4*>(w + static_cast<long>(n_base + 16 * j + lr) * K + k0);
        const float4 u = src[0], v = src[1];
        f[0] = u.x; f[1] = u.y; f[2] = u.z; f[3] = u.w; f[4] = v.x; f[5] = v.y; f[6] = v.z; f[7] = v.w;
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) f[t] = 0.f;
      }
      wf[j][ks] = split8(f);
    }
  float4 bv[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    bv[j] = bias ? *reinterpret_cast<const float4*>(bias + n_base + 16 * j + 4 * lg) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  for (long tile = gw / ncb; tile < ntiles; tile += nw / ncb) {
    const long p = tile * 16 + lr;
    const bool pv = p < M;
    const long pc = pv ? p : 0;
    const int rem = static_cast<int>(pc % HW), yy = rem / W, xx = rem - yy * W;
    nf4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = nf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 32 * ks + 8 * lg, tap = k0 / CIN, c0 = k0 - tap * CIN;
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const bool ok = pv && tap < 9 && yy + dy >= 0 && yy + dy < H && xx + dx >= 0 && xx + dx < W;
      const long q = ok ? pc + dy * W + dx : pc;          // clamped, loaded unconditionally, zeroed by select
      const float4* src = reinterpret_cast<const float4*>(x + q * CIN + (tap < 9 ? c0 : 0));
      const float4 u = src[0], v = src[1];
      const float f[8] = {ok ? u.x : 0.f, ok ? u.y : 0.f, ok ? u.z : 0.f, ok ? u.w : 0.f,
                          ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f};
      const Split3 xb = split8(f);
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = nmfma_x6(wf[j][ks], xb, acc[j]);
    }
    if (pv) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n_base + 16 * j + 4 * lg;
        float v[4] = {acc[j][0] + bv[j].x, acc[j][1] + bv[j].y, acc[j][2] + bv[j].z, acc[j][3] + bv[j].w};
        if (res) {
          const float4 rv = *reinterpret_cast<const float4*>(res + p * Cout + n);
          const float r[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act == ACT_DRELU ? (r[e] > 0.f ? v[e] : 0.f) : v[e] + r[e];
        }
        if (act == ACT_RELU)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        *reinterpret_cast<float4*>(out + p * Cout + n) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

// narrow direct conv in split mode (APPLESTAR_CONV_F32_NARROW = 1 (default) | 0 | all).  Measured against the ring
// kernel (profiles/r4z_conv_f32_narrow.txt, 390 images): 16 -> 16 at 76 x 80 158 vs 227 us; 16 -> 32 at 38 x 40
// 87 vs 77, 32 -> 16 118 vs 115, 32 -> 32 at 19 x 20 66 vs 37 - so by default only Cin = Cout = 16 takes it
// ('all': every {16, 32} x {16, 32} shape).
int conv_narrow_mode() {
  static const int m = [] {
    const char* e = std::getenv("APPLESTAR_CONV_F32_NARROW");
    if (e && e[0] == '0') return 0;
    if (e && e[0] == 'a') return 2;
    return 1;
  }();
  return m;
}

bool launch_narrow(const float* x, const float* w, const float* bias, const float* res, float* out, int B, int H,
                   int W, int Cin, int Cout, int act, hipStream_t s) {
  const int nm = conv_narrow_mode();
  if (f32_mfma_mode() != 1 || nm == 0 || (Cin != 16 && Cin != 32) || (Cout != 16 && Cout != 32)) return false;
  if (nm == 1 && (Cin != 16 || Cout != 16)) return false;
  const long M = static_cast<long>(B) * H * W;
  const long ntiles = (M + 15) / 16;
  if (ntiles == 0) return true;
  // ~8 workgroups per CU, each wave walking its tiles (the split weight rows amortised over them)
  const int nt = (Cin == 16 && Cout == 32) ? 2 : 1;
  const long ncb = Cout / (16 * nt);
  long nwg = std::min<long>(2048, (ntiles * ncb + 3) / 4);
  nwg = std::max<long>(nwg, 1);
  // every wave's output-channel block is (wave id % ncb): keep the wave count a multiple of ncb
  if (Cin == 16 && nt == 2)
    hipLaunchKernelGGL((conv3x3_f32_narrow_kernel<16, 2>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias,
                       res, out, B, H, W, Cout, act, ntiles);
  else if (Cin == 16)
    hipLaunchKernelGGL((conv3x3_f32_narrow_kernel<16, 1>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias,
                       res, out, B, H, W, Cout, act, ntiles);
  else
    hipLaunchKernelGGL((conv3x3_f32_narrow_kernel<32, 1>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias,
                       res, out, B, H, W, Cout, act, ntiles);
  return true;
}

template <int BN>
void launch_f32(const float* x, const float* w, const float* bias, const float* res, float* out, int B, int H, int W,
                int Cin, int Cout, int act, hipStream_t s) {
  const long M = static_cast<long>(B) * H * W;
  const long nwg = (M + 127) / 128 * ((Cout + BN - 1) / BN);
  if (nwg == 0) return;
  const int mode = f32_mfma_mode();
  if constexpr (BN == 128) {
    const int cv = f32_conv_variant();
    if (mode == 1 && cv == 3) {                   // DMA issue between the K-step's MFMA halves (A/B switch)
      hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<128, 3, 128, false, 4, true>), dim3(static_cast<unsigned>(nwg)),
                         dim3(256), 0, s, x, w, bias, res, out, B, H, W, Cin, Cout, act);
      return;
    }
    if (mode == 1 && (cv == 1 || cv == 2)) {      // 256-pixel tiles on 8 waves (A/B switch)
      const long nwg8 = (M + 255) / 256 * ((Cout + BN - 1) / BN);
      if (cv == 1)
        hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<128, 4, 256, false, 8>), dim3(static_cast<unsigned>(nwg8)),
                           dim3(512), 0, s, x, w, bias, res, out, B, H, W, Cin, Cout, act);
      else
        hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<128, 4, 256, true, 8>), dim3(static_cast<unsigned>(nwg8)),
                           dim3(512), 0, s, x, w, bias, res, out, B, H, W, Cin, Cout, act);
      return;
    }
  }
  if constexpr (BN == 32) {
    if (mode == 1 && conv_n32_bm256()) {
      const long nwg2 = (M + 255) / 256 * ((Cout + BN - 1) / BN);
      hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<32, 3, 256>), dim3(static_cast<unsigned>(nwg2)), dim3(256), 0, s, x,
                         w, bias, res, out, B, H, W, Cin, Cout, act);
      return;
    }
  }
  if (mode == 1 && conv_f32_staged())
    hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<BN, 3, 128, true>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x,
                       w, bias, res, out, B, H, W, Cin, Cout, act);
  else if (mode == 1)
    hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<BN, 3>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias,
                       res, out, B, H, W, Cin, Cout, act);
  else if (mode == 3)
    hipLaunchKernelGGL((conv3x3_f32_kernel<BN, 2>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias, res,
                       out, B, H, W, Cin, Cout, act);
  else if (mode == 2)
    hipLaunchKernelGGL((conv3x3_f32_kernel<BN, 1>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias, res,
                       out, B, H, W, Cin, Cout, act);
  else
    hipLaunchKernelGGL((conv3x3_f32_kernel<BN, 0>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias, res,
                       out, B, H, W, Cin, Cout, act);
}

}  // namespace

bool conv3x3_f32_supported(int Cin, int Cout) { return Cin % 16 == 0 && Cin > 0 && Cout > 0; }

// the extended input-gradient epilogue (second residual on the first rows + ReLU mask of the layer input) runs on
// the split ring kernel's register epilogue: 128-multiple output channels, split-MFMA mode
bool conv3x3_f32_epi2_supported(int Cin, int Cout) {
  return conv3x3_f32_supported(Cin, Cout) && Cout % 128 == 0 && Cin > 32 && f32_mfma_mode() == 1;
}

void conv3x3_f32_fwd_epi2(const float* x, const float* w, const float* res, const float* res2, long res2_rows,
                          const float* mask, float* out, int B, int H, int W, int Cin, int Cout, hipStream_t s) {
  const long M = static_cast<long>(B) * H * W;
  const long nwg = (M + 127) / 128 * (Cout / 128);
  if (nwg == 0) return;
  pipe::Epi2 e2;
  e2.res2 = res2;
  e2.res2_rows = res2_rows;
  e2.mask = mask;
  if (f32_conv_variant() == 3)
    hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<128, 3, 128, false, 4, true>), dim3(static_cast<unsigned>(nwg)),
                       dim3(256), 0, s, x, w, nullptr, res, out, B, H, W, Cin, Cout, 0, e2);
  else
    hipLaunchKernelGGL((conv3x3_f32_pipe_kernel<128, 3>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w,
                       nullptr, res, out, B, H, W, Cin, Cout, 0, e2);
}

void conv3x3_f32_fwd(const float* x, const float* w, const float* bias, const float* res, float* out, int B, int H,
                     int W, int Cin, int Cout, int act, hipStream_t s) {
  if (launch_narrow(x, w, bias, res, out, B, H, W, Cin, Cout, act, s)) return;
  if (Cout % 128 == 0) launch_f32<128>(x, w, bias, res, out, B, H, W, Cin, Cout, act, s);
  else if (Cout > 32) launch_f32<64>(x, w, bias, res, out, B, H, W, Cin, Cout, act, s);
  else launch_f32<32>(x, w, bias, res, out, B, H, W, Cin, Cout, act, s);
}

}  // namespace as
