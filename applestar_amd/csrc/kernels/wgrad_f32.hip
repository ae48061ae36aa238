// fp32 weight (and bias) gradients of the tall-skinny GEMMs and 3x3 convolutions of the fp32 learner step, on
// the exact-f32 MFMA v_mfma_f32_32x32x2_f32.  Same decomposition as the bf16 kernel (wgrad.hip):
//
//   dW[n, k] = sum_r dY[r, n] * X(r, k)          db[n] = sum_r dY[r, n]
//
// with R = 10^4 .. 10^7 reduction rows split over S slices (grid = N-tiles x K-tiles x S), one fp32 partial
// per slice, summed afterwards by one deterministic column reduction.  X(r, k) is either dense ([R, K]
// row-major: nn.Linear, 1x1 conv on NHWC pixels) or the implicit im2col of a pad-1 3x3 conv on an NHWC image
// (k = tap * Cin + c, zero outside the image): the [Cout, 3, 3, Cin] (channels_last) weight order.
//
// Both operands are reduction-major in memory (row r holds all n / all k) and are staged row-major in LDS as
// loaded.  The 32x32x2 MFMA takes A[i][k] = dY[r][n0 + i] and B[k][j] = X(r, k0 + j) with lane l holding
// row/column l&31 and reduction slot l>>5; k-step kk of a 32-row stage gives lane half h the row 16h + kk, so
// each half-wave reads 32 consecutive floats of one LDS row (one conflict-free ds_read_b32 per operand).
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(16))) float f16v;

constexpr int kOOB = 0x7ffffff0;

template <int BN_, int BK_>
struct WgF32Cfg {
  static constexpr int BN = BN_, BK = BK_, BR = 32, NT = 256;
  static constexpr int WN = BN_ >= 64 ? 2 : 1, WK = 4 / WN;   // waves: 2 x 2, or 1 x 4 for a 32-wide N tile
  static constexpr int TN = BN / WN, TK = BK / WK;
  static constexpr int FN = TN / 32, FK = TK / 32;   // 32x32 tiles per wave
  static constexpr int PA = BN + 4, PB = BK + 4;     // LDS row pitch (floats)
  static constexpr int CHA = BN / 4, CHB = BK / 4;   // 16-B pieces per row
  static constexpr int A_IT = BR * CHA / NT, B_IT = BR * CHB / NT;
  static constexpr int STAGE = BR * (PA + PB);       // floats
  static_assert(A_IT * NT == BR * CHA && B_IT * NT == BR * CHB, "tile / thread mismatch");
};

template <int BN, int BK, bool CONV, int SPLIT>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                        float* __restrict__ dw_part, float* __restrict__ db_part,
                                                        long part_stride, long R, int N, int K, int H, int W, int Cin,
                                                        long rows_per_split, int tiles_n, int tiles_k) {
  using C = WgF32Cfg<BN, BK>;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::STAGE];

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tk = wg % tiles_k;
  const int tn = (wg / tiles_k) % tiles_n;
  const int s = wg / (tiles_k * tiles_n);
  const int n0 = tn * BN, k0 = tk * BK;
  const long r_begin = static_cast<long>(s) * rows_per_split;
  const long r_end = r_begin + rows_per_split < R ? r_begin + rows_per_split : R;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid / C::WK, wk = wid % C::WK;
  const int l32 = lane & 31, h = lane >> 5;
  const long HW = static_cast<long>(H) * W;

  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), 0,
                                                                      static_cast<int>(R * N * 4), 0x00020000);
  const long xbytes = CONV ? R * Cin * 4 : R * K * 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0,
                                                                      static_cast<int>(xbytes), 0x00020000);
  // per-thread piece columns (fixed across stages): CHA and CHB divide NT
  const int a_col = n0 + 4 * (tid % C::CHA);
  const int b_col = k0 + 4 * (tid % C::CHB);
  int b_c = b_col, b_dy = 0, b_dx = 0;
  if (CONV) {
    const int tap = b_col / Cin;
    b_c = b_col - tap * Cin;
    b_dy = tap / 3 - 1;
    b_dx = tap % 3 - 1;
  }
  const bool a_ok = a_col < N, b_ok = b_col < K;
  // conv pieces: image coordinates of each piece's row, advanced by BR rows per stage (32-bit offsets: the
  // host keeps every operand below 2^31 bytes).  Replaces a 64-bit modulo and two divisions per piece and
  // stage, which were the bulk of the loop's VALU work on the narrow (Cout 32 / 64) tiles.
  int py[C::B_IT], px[C::B_IT];
  const int adv_y = C::BR / W, adv_x = C::BR % W;
  if (CONV) {
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const long r = r_begin + (tid + i * C::NT) / C::CHB;
      const int rem = static_cast<int>(r % HW);
      py[i] = rem / W;
      px[i] = rem - py[i] * W;
    }
  }

  uint4 ra[C::A_IT], rb[C::B_IT];
  auto load_regs = [&](long rs) {
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const long r = rs + (tid + i * C::NT) / C::CHA;
      const int off = (a_ok && r < r_end) ? (static_cast<int>(r) * N + a_col) * 4 : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(yr, off, 0, 0);
      ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const long r = rs + (tid + i * C::NT) / C::CHB;
      int off = kOOB;
      if (CONV) {
        const int yy = py[i] + b_dy, xx = px[i] + b_dx;
        if (b_ok && r < r_end && yy >= 0 && yy < H && xx >= 0 && xx < W)
          off = ((static_cast<int>(r) + b_dy * W + b_dx) * Cin + b_c) * 4;
        px[i] += adv_x;
        py[i] += adv_y;
        if (px[i] >= W) { px[i] -= W; ++py[i]; }
        while (py[i] >= H) py[i] -= H;
      } else if (b_ok && r < r_end) {
        off = (static_cast<int>(r) * K + b_col) * 4;
      }
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_lds = [&](int st) {
    float* A = smem + st * C::STAGE;
    float* Bt = A + C::BR * C::PA;
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i) {
      const int idx = tid + i * C::NT;
      *reinterpret_cast<uint4*>(A + (idx / C::CHA) * C::PA + 4 * (idx % C::CHA)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int idx = tid + i * C::NT;
      *reinterpret_cast<uint4*>(Bt + (idx / C::CHB) * C::PB + 4 * (idx % C::CHB)) = rb[i];
    }
  };

  f16v acc[C::FN][C::FK];
#pragma unroll
  for (int i = 0; i < C::FN; ++i)
#pragma unroll
    for (int j = 0; j < C::FK; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const bool do_bias = db_part != nullptr && tk == 0 && wk == 0;
  float bsum[C::FN];
#pragma unroll
  for (int i = 0; i < C::FN; ++i) bsum[i] = 0.f;

  const long nsteps = r_end > r_begin ? (r_end - r_begin + C::BR - 1) / C::BR : 0;
  if (nsteps > 0) {
    load_regs(r_begin);
    store_lds(0);
    __syncthreads();
  }
  for (long it = 0; it < nsteps; ++it) {
    const int cur = static_cast<int>(it & 1);
    if (it + 1 < nsteps) load_regs(r_begin + (it + 1) * C::BR);
    const float* A = smem + cur * C::STAGE + (16 * h) * C::PA + wn * C::TN + l32;
    const float* Bt = smem + cur * C::STAGE + C::BR * C::PA + (16 * h) * C::PB + wk * C::TK + l32;
    if constexpr (SPLIT == 1) {
      // bf16x6 (split_mfma.h): 16-row chunk c of lane half h = the MFMA's k-slots 8h..8h+7
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        float av[C::FN][8], bv[C::FK][8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
#pragma unroll
          for (int i = 0; i < C::FN; ++i) av[i][t] = A[(8 * c + t) * C::PA + 32 * i];
#pragma unroll
          for (int j = 0; j < C::FK; ++j) bv[j][t] = Bt[(8 * c + t) * C::PB + 32 * j];
        }
        Split3 sa[C::FN], sb[C::FK];
#pragma unroll
        for (int i = 0; i < C::FN; ++i) sa[i] = split8(av[i]);
#pragma unroll
        for (int j = 0; j < C::FK; ++j) sb[j] = split8(bv[j]);
#pragma unroll
        for (int i = 0; i < C::FN; ++i)
#pragma unroll
          for (int j = 0; j < C::FK; ++j) acc[i][j] = mfma_x6(sa[i], sb[j], acc[i][j]);
        if (do_bias) {
#pragma unroll
          for (int i = 0; i < C::FN; ++i)
#pragma unroll
            for (int t = 0; t < 8; ++t) bsum[i] += av[i][t];
        }
      }
    } else {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float af[C::FN], bfr[C::FK];
#pragma unroll
      for (int i = 0; i < C::FN; ++i) af[i] = A[kk * C::PA + 32 * i];
#pragma unroll
      for (int j = 0; j < C::FK; ++j) bfr[j] = Bt[kk * C::PB + 32 * j];
#pragma unroll
      for (int i = 0; i < C::FN; ++i)
#pragma unroll
        for (int j = 0; j < C::FK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < C::FN; ++i) bsum[i] += af[i];
      }
    }
    }
    if (it + 1 < nsteps) store_lds(cur ^ 1);
    __syncthreads();
  }

  // accumulator (i, j) register e: n = n0 + wn TN + 32 i + (e&3) + 8 (e>>2) + 4 h, k = k0 + wk TK + 32 j + l32:
  // 32 lanes store 128 contiguous bytes of one dW row
  float* outp = dw_part + static_cast<long>(s) * part_stride;
#pragma unroll
  for (int i = 0; i < C::FN; ++i)
#pragma unroll
    for (int j = 0; j < C::FK; ++j) {
      const int k = k0 + wk * C::TK + 32 * j + l32;
      if (k >= K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + wn * C::TN + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (n < N) outp[static_cast<long>(n) * K + k] = acc[i][j][e];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < C::FN; ++i) {
      const float v = bsum[i] + __shfl_xor(bsum[i], 32, kWave);
      const int n = n0 + wn * C::TN + 32 * i + l32;
      if (h == 0 && n < N) db_part[static_cast<long>(s) * part_stride + n] = v;
    }
  }
}

// split-MFMA mode on the LDS-DMA ring of f32_pipe.h: K-steps of RS = 16 reduction rows, stage = the dY rows
// [16][BN] then the X rows [16][BK] as loaded (lane-linear, 1 KB per DMA wave-instruction = 1024 / (4 BN) rows).
// Fragments: lane (l32, h) takes rows 8 h .. 8 h + 7 of its column (eight ds_read_b32; the 32 lanes of a b32 group
// read 32 consecutive floats of one row).  The conv form's X piece of a lane is a fixed 4-channel group of one tap
// (the lane's column is the same in every stage); its row's image coordinates advance by 16 rows per issued step.
template <int BN, int BK, bool CONV, int NS>
__global__ __launch_bounds__(256, ((BN == 128 && BK >= 128) || BN == 32) ? 2 : 3) void wgrad_f32_pipe_kernel(const float* __restrict__ dy,
                                                                const float* __restrict__ x,
                                                                float* __restrict__ dw_part, float* __restrict__ db_part,
                                                                long part_stride, long R, int N, int K, int H, int W,
                                                                int Cin, long rows_per_split, int tiles_n, int tiles_k) {
  // a 32-wide N tile takes 32 reduction rows per stage (two MFMA K-steps) so its dY rows still fill one 4-KB
  // DMA wave-instruction per wave
  constexpr int RS = BN == 32 ? 32 : 16, SUB = RS / 16;
  constexpr int A_BYTES = RS * BN * 4, B_BYTES = RS * BK * 4, STAGE = A_BYTES + B_BYTES;
  constexpr int A_PW = A_BYTES / 4096, B_PW = B_BYTES / 4096;          // DMA wave-instructions per wave
  constexpr int A_CPR = BN / 4, B_CPR = BK / 4;                       // 16-B pieces per row
  constexpr int A_RPI = 64 / A_CPR, B_RPI = 64 / B_CPR;               // rows per wave-instruction
  static_assert(A_PW >= 1 && B_PW >= 1 && A_PW * 4096 == A_BYTES && B_PW * 4096 == B_BYTES, "tile / DMA mismatch");
  constexpr int WN = BN >= 64 ? 2 : 1, WK = 4 / WN;
  constexpr int TN = BN / WN, TK = BK / WK, FN = TN / 32, FK = TK / 32;
  static_assert(NS == 3, "three stage arrays");
  __shared__ __attribute__((aligned(16))) char s0[STAGE], s1[STAGE], s2[STAGE];
  char* const smem[3] = {s0, s1, s2};

  const int wg = pipe::xcd_remap();
  const int tk = wg % tiles_k;
  const int tn = (wg / tiles_k) % tiles_n;
  const int s = wg / (tiles_k * tiles_n);
  const int n0 = tn * BN, k0 = tk * BK;
  const long r_begin = static_cast<long>(s) * rows_per_split;
  const long r_end = r_begin + rows_per_split < R ? r_begin + rows_per_split : R;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / WK, wk = wid % WK;
  const int l32 = lane & 31, h = lane >> 5;
  const long HW = static_cast<long>(H) * W;
  const pipe::i32x4 yr = pipe::rsrc(dy, R * N * 4), xr = pipe::rsrc(x, CONV ? R * Cin * 4 : R * K * 4);

  // DMA pieces: fixed column per lane, row (within a step) per chunk
  const int a_col = n0 + 4 * (lane % A_CPR), b_col = k0 + 4 * (lane % B_CPR);
  int a_row[A_PW], b_row[B_PW];
#pragma unroll
  for (int c = 0; c < A_PW; ++c) a_row[c] = (wid + 4 * c) * A_RPI + lane / A_CPR;
#pragma unroll
  for (int c = 0; c < B_PW; ++c) b_row[c] = (wid + 4 * c) * B_RPI + lane / B_CPR;
  int b_c = b_col, b_dy = 0, b_dx = 0;
  if (CONV) {
    const int tap = b_col / Cin;
    b_c = b_col - tap * Cin;
    b_dy = tap / 3 - 1;
    b_dx = tap % 3 - 1;
  }
  const bool a_ok = a_col < N, b_ok = b_col < K;
  // conv: image coordinates of each chunk's row for the next step to issue (advanced by RS rows per issue)
  int py[B_PW], px[B_PW];
  const int adv_y = RS / W, adv_x = RS % W;
  if (CONV) {
#pragma unroll
    for (int c = 0; c < B_PW; ++c) {
      const int rem = static_cast<int>((r_begin + b_row[c]) % HW);
      py[c] = rem / W;
      px[c] = rem - py[c] * W;
    }
  }
  const long nsteps = r_end > r_begin ? (r_end - r_begin + RS - 1) / RS : 0;
  auto issue = [&](char* st, long kt) {
    const long r0 = r_begin + kt * RS;
#pragma unroll
    for (int c = 0; c < A_PW; ++c) {
      const long r = r0 + a_row[c];
      pipe::dma16(yr, st + (wid + 4 * c) * 1024,
                  (kt < nsteps && a_ok && r < r_end) ? (static_cast<int>(r) * N + a_col) * 4 : pipe::kOOB);
    }
#pragma unroll
    for (int c = 0; c < B_PW; ++c) {
      const long r = r0 + b_row[c];
      int off = pipe::kOOB;
      if (CONV) {
        const int yy = py[c] + b_dy, xx = px[c] + b_dx;
        if (kt < nsteps && b_ok && r < r_end && yy >= 0 && yy < H && xx >= 0 && xx < W)
          off = ((static_cast<int>(r) + b_dy * W + b_dx) * Cin + b_c) * 4;
        px[c] += adv_x;
        py[c] += adv_y;
        if (px[c] >= W) { px[c] -= W; ++py[c]; }
        while (py[c] >= H) py[c] -= H;
      } else if (kt < nsteps && b_ok && r < r_end) {
        off = (static_cast<int>(r) * K + b_col) * 4;
      }
      pipe::dma16(xr, st + A_BYTES + (wid + 4 * c) * 1024, off);
    }
  };

  f16v acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const bool do_bias = db_part != nullptr && tk == 0 && wk == 0;
  float bsum[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) bsum[i] = 0.f;

  auto step = [&](const char* st, char* next, long kt) {
    pipe::wait_vm<(NS - 2) * (A_PW + B_PW)>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(next, kt + NS - 1);
#pragma unroll
    for (int sub = 0; sub < SUB; ++sub) {
      const float* A = reinterpret_cast<const float*>(st) + (16 * sub + 8 * h) * BN + wn * TN + l32;
      const float* Bt = reinterpret_cast<const float*>(st + A_BYTES) + (16 * sub + 8 * h) * BK + wk * TK + l32;
      float av[FN][8];
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int i = 0; i < FN; ++i) av[i][t] = A[t * BN + 32 * i];
      Split3 sa[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) sa[i] = split8(av[i]);
      if constexpr (FK <= 2) {
        float bv[FK][8];
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int j = 0; j < FK; ++j) bv[j][t] = Bt[t * BK + 32 * j];
        Split3 sb[FK];
#pragma unroll
        for (int j = 0; j < FK; ++j) sb[j] = split8(bv[j]);
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FK; ++j) acc[i][j] = mfma_x6(sa[i], sb[j], acc[i][j]);
      } else {
        // the wide tile (64 x 128 per wave: 2 dY + 4 X fragments per 48 MFMAs, 25 % less split VALU per MFMA than
        // 64 x 64): X fragments streamed one at a time
#pragma unroll
        for (int j = 0; j < FK; ++j) {
          float bv[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) bv[t] = Bt[t * BK + 32 * j];
          const Split3 sb = split8(bv);
#pragma unroll
          for (int i = 0; i < FN; ++i) acc[i][j] = mfma_x6(sa[i], sb, acc[i][j]);
        }
      }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int t = 0; t < 8; ++t) bsum[i] += av[i][t];
      }
    }
  };
  issue(smem[0], 0);
  issue(smem[1], 1);
  for (long kt = 0; kt < nsteps; kt += NS) {
    step(smem[0], smem[2], kt);
    if (kt + 1 >= nsteps) break;
    step(smem[1], smem[0], kt + 1);
    if (kt + 2 >= nsteps) break;
    step(smem[2], smem[1], kt + 2);
  }
  pipe::wait_vm<0>();

  // accumulator (i, j) register e: n = n0 + wn TN + 32 i + (e&3) + 8 (e>>2) + 4 h, k = k0 + wk TK + 32 j + l32
  float* outp = dw_part + static_cast<long>(s) * part_stride;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = k0 + wk * TK + 32 * j + l32;
      if (k >= K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + wn * TN + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (n < N) outp[static_cast<long>(n) * K + k] = acc[i][j][e];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const float v = bsum[i] + __shfl_xor(bsum[i], 32, kWave);
      const int n = n0 + wn * TN + 32 * i + l32;
      if (h == 0 && n < N) db_part[static_cast<long>(s) * part_stride + n] = v;
    }
  }
}

// Split-once staging (the 128 x 128 tiles of the split-MFMA mode, APPLESTAR_WGRAD_STG): in the ring kernel above every
// wave splits each fragment it reads, and in its 2 x 2 wave layout every dY and every X fragment is split by two
// waves - the split is ~80 % of the loop's VALU (9-11 VALU per MFMA, profiles/r8h_pmc_wgrad_*).  Here each fp32
// value of a stage is split ONCE per workgroup into three bf16 planes stored in MFMA fragment order, which the
// waves then read with one conflict-free ds_read_b128 per plane:
//
//   fp32 ring F[2] (16 reduction rows x (128 dY + 128 X) columns, LDS-DMA as loaded)
//   planes P[2]: P[p][block(4)][half(2)][lane(32)] x 16 B for dY and for X (24 KB per stage)
//   step kt: wait F(kt + 1) -> s_barrier -> DMA F(kt + 2) into F(kt)'s slot -> split F(kt + 1) into P(kt + 1)
//            (thread t: column t % 128, rows 8 (t / 128) .. + 7, of dY and of X) beside MFMA(kt) on P(kt)
// so the split of the next step and the products of this one share a barrier interval.  80 KB of LDS: 2
// workgroups per CU.  db: each thread's dY column sums, the two row halves combined through LDS at the end.
// Narrow N tiles (BN = 32 / 64: the 76x80 / 19x20 convs with 32 / 64 output channels, round 6): the same stages
// with the four waves along K (each wave 32 (BN = 32) or 64 x 32 of the tile), the dY stage DMA'd by the first
// A_N waves, and dY split by the first 2 BN threads; 50 / 60 KB of LDS (3 / 2 workgroups per CU).
template <int BN>
struct StgCfg {
  static constexpr int BK = 128, RS = 16;
  static constexpr int WN = BN == 128 ? 2 : 1, WK = 4 / WN;
  static constexpr int FN = BN / (32 * WN), FK = BK / (32 * WK);   // 32 x 32 blocks per wave along N / K
  static constexpr int A_BYTES = RS * BN * 4, B_BYTES = RS * BK * 4, FST = A_BYTES + B_BYTES;
  static constexpr int A_N = A_BYTES / 1024, B_N = B_BYTES / 1024;  // 1 KB DMA wave-instructions per stage
  static constexpr int A_PW = (A_N + 3) / 4, B_PW = B_N / 4;
  static constexpr int A_CPR = BN / 4, B_CPR = BK / 4, A_RPI = 64 / A_CPR, B_RPI = 64 / B_CPR;
  static constexpr int PLA = (BN / 32) * 2 * 32 * 16, PLB = (BK / 32) * 2 * 32 * 16;   // one plane of dY / X
  static constexpr int PST = 3 * (PLA + PLB);
  static constexpr int OCC = BN == 32 ? 3 : 2;
  static_assert(B_N % 4 == 0 && (A_N % 4 == 0 || A_N < 4), "stage DMA split");
};

template <int BN, bool CONV>
__global__ __launch_bounds__(256, StgCfg<BN>::OCC) void wgrad_f32_stg_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                              float* __restrict__ dw_part, float* __restrict__ db_part,
                                                              long part_stride, long R, int N, int K, int H, int W,
                                                              int Cin, long rows_per_split, int tiles_n, int tiles_k) {
  using C = StgCfg<BN>;
  constexpr int BK = C::BK, RS = C::RS, A_BYTES = C::A_BYTES, FST = C::FST, A_PW = C::A_PW, B_PW = C::B_PW;
  constexpr int A_CPR = C::A_CPR, B_CPR = C::B_CPR, A_RPI = C::A_RPI, B_RPI = C::B_RPI;
  constexpr int PLA = C::PLA, PLB = C::PLB, PST = C::PST, FN = C::FN, FK = C::FK;
  __shared__ __attribute__((aligned(16))) char F[2 * FST];
  __shared__ __attribute__((aligned(16))) char P[2 * PST];

  const int wg = pipe::xcd_remap();
  const int tk = wg % tiles_k;
  const int tn = (wg / tiles_k) % tiles_n;
  const int s = wg / (tiles_k * tiles_n);
  const int n0 = tn * BN, k0 = tk * BK;
  const long r_begin = static_cast<long>(s) * rows_per_split;
  const long r_end = r_begin + rows_per_split < R ? r_begin + rows_per_split : R;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid / C::WK, wk = wid % C::WK;
  const int l32 = lane & 31, h = lane >> 5;
  const long HW = static_cast<long>(H) * W;
  const pipe::i32x4 yr = pipe::rsrc(dy, R * N * 4), xr = pipe::rsrc(x, CONV ? R * Cin * 4 : R * K * 4);
  // waves past the dY stage's A_N DMA instructions (BN = 32) issue only their X pieces
  const bool a_wave = A_PW * 4 == C::A_N || wid < C::A_N;

  // DMA pieces (the ring kernel's): fixed column per lane, row (within a step) per chunk
  const int a_col = n0 + 4 * (lane % A_CPR), b_col = k0 + 4 * (lane % B_CPR);
  int a_row[A_PW], b_row[B_PW];
#pragma unroll
  for (int c = 0; c < A_PW; ++c) a_row[c] = (wid + 4 * c) * A_RPI + lane / A_CPR;
#pragma unroll
  for (int c = 0; c < B_PW; ++c) b_row[c] = (wid + 4 * c) * B_RPI + lane / B_CPR;
  int b_c = b_col, b_dy = 0, b_dx = 0;
  if (CONV) {
    const int tap = b_col / Cin;
    b_c = b_col - tap * Cin;
    b_dy = tap / 3 - 1;
    b_dx = tap % 3 - 1;
  }
  const bool a_ok = a_col < N, b_ok = b_col < K;
  int py[B_PW], px[B_PW];
  const int adv_y = RS / W, adv_x = RS % W;
  if (CONV) {
#pragma unroll
    for (int c = 0; c < B_PW; ++c) {
      const int rem = static_cast<int>((r_begin + b_row[c]) % HW);
      py[c] = rem / W;
      px[c] = rem - py[c] * W;
    }
  }
  const long nsteps = r_end > r_begin ? (r_end - r_begin + RS - 1) / RS : 0;
  auto issue = [&](long kt) {
    char* st = F + (kt & 1) * FST;
    const long r0 = r_begin + kt * RS;
    if (a_wave) {
#pragma unroll
      for (int c = 0; c < A_PW; ++c) {
        const long r = r0 + a_row[c];
        pipe::dma16(yr, st + (wid + 4 * c) * 1024,
                    (kt < nsteps && a_ok && r < r_end) ? (static_cast<int>(r) * N + a_col) * 4 : pipe::kOOB);
      }
    }
#pragma unroll
    for (int c = 0; c < B_PW; ++c) {
      const long r = r0 + b_row[c];
      int off = pipe::kOOB;
      if (CONV) {
        const int yy = py[c] + b_dy, xx = px[c] + b_dx;
        if (kt < nsteps && b_ok && r < r_end && yy >= 0 && yy < H && xx >= 0 && xx < W)
          off = ((static_cast<int>(r) + b_dy * W + b_dx) * Cin + b_c) * 4;
        px[c] += adv_x;
        py[c] += adv_y;
        if (px[c] >= W) { px[c] -= W; ++py[c]; }
        while (py[c] >= H) py[c] -= H;
      } else if (kt < nsteps && b_ok && r < r_end) {
        off = (static_cast<int>(r) * K + b_col) * 4;
      }
      pipe::dma16(xr, st + A_BYTES + (wid + 4 * c) * 1024, off);
    }
  };

  // split work of this thread: column sc of X, rows 8 sh .. 8 sh + 7 of the stage; column ac of dY (rows 8 ah ..)
  // for the first 2 BN threads
  const int sc = tid & (BK - 1), sh = tid >> 7;
  const int ac = tid & (BN - 1), ah = tid / BN;
  const bool a_split = tid < 2 * BN;
  const bool do_bias = db_part != nullptr && tk == 0;
  float bsum = 0.f;
  auto split_stage = [&](long j) {
    const float* fa = reinterpret_cast<const float*>(F + (j & 1) * FST);
    const float* fb = fa + RS * BN;
    char* pa = P + (j & 1) * PST;
    char* pb = pa + 3 * PLA;
    float vb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) vb[q] = fb[(8 * sh + q) * BK + sc];
    const Split3 sb = split8(vb);
    const int bslot = (((sc >> 5) * 2 + sh) * 32 + (sc & 31)) * 16;
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<u32v4*>(pb + p * PLB + bslot) = sb.p[p];
    if (a_split) {
      float va[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) va[q] = fa[(8 * ah + q) * BN + ac];
      const Split3 sa = split8(va);
      const int aslot = (((ac >> 5) * 2 + ah) * 32 + (ac & 31)) * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<u32v4*>(pa + p * PLA + aslot) = sa.p[p];
      if (do_bias) {
#pragma unroll
        for (int q = 0; q < 8; ++q) bsum += va[q];
      }
    }
  };

  f16v acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if (nsteps > 0) {
    issue(0);
    issue(1);
    if (a_wave) pipe::wait_vm<A_PW + B_PW>();          // this wave's pieces of step 0
    else pipe::wait_vm<B_PW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    split_stage(0);
  }
  for (long kt = 0; kt < nsteps; ++kt) {
    // F(kt + 1) landed (this wave's pieces, then everyone's); everyone finished split(kt) (P(kt) complete, F(kt)
    // free) and MFMA(kt - 1) (P(kt + 1)'s slot free)
    pipe::wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(kt + 2);
    if (kt + 1 < nsteps) split_stage(kt + 1);
    const char* pa = P + (kt & 1) * PST;
    const char* pb = pa + 3 * PLA;
    Split3 fa[FN], fb[FK];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        fa[i].p[p] = *reinterpret_cast<const u32v4*>(pa + p * PLA + (((wn * FN + i) * 2 + h) * 32 + l32) * 16);
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        fb[j].p[p] = *reinterpret_cast<const u32v4*>(pb + p * PLB + (((wk * FK + j) * 2 + h) * 32 + l32) * 16);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FK; ++j) acc[i][j] = mfma_x6(fa[i], fb[j], acc[i][j]);
  }
  pipe::wait_vm<0>();

  // accumulator (i, j) register e: n = n0 + wn 32 FN + 32 i + (e&3) + 8 (e>>2) + 4 h, k = k0 + wk 32 FK + 32 j + l32
  float* outp = dw_part + static_cast<long>(s) * part_stride;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = k0 + wk * 32 * FK + 32 * j + l32;
      if (k >= K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + wn * 32 * FN + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (n < N) outp[static_cast<long>(n) * K + k] = acc[i][j][e];
      }
    }
  if (do_bias) {
    float* bred = reinterpret_cast<float*>(F);      // the ring is idle: every DMA landed (wait_vm<0> above)
    __syncthreads();
    if (a_split && ah == 1) bred[ac] = bsum;
    __syncthreads();
    if (a_split && ah == 0 && n0 + ac < N) db_part[static_cast<long>(s) * part_stride + n0 + ac] = bsum + bred[ac];
  }
}

// The 32-wide ring kernel is opt-in (APPLESTAR_WGRAD32_PIPE=1): on the learner's narrow convs it measured
// 5-13 % slower than the register-staged kernel (76x80 64->32: 1358 vs 1283 us; 19x20 32->32: 66.7 vs
// 59.2 us; profiles/r3v2_wgrad32_ab.jsonl) - 60 KB of stages hold it at 2 workgroups per CU.
bool wgrad_f32_pipe32_off() {
  static const bool off = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD32_PIPE");
    return e == nullptr || e[0] != '1';
  }();
  return off;
}

// APPLESTAR_WGRAD_STG=0: the 128 x 128 tiles on the per-wave-split ring kernel instead of split-once staging
bool wgrad_stg() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_STG");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// APPLESTAR_WGRAD_STG_NARROW=1: the 32 / 64-wide N tiles on split-once staging too.  Measured slower than the
// per-wave-split kernels on every narrow learner shape (76x80 64 -> 32: 1266 vs 1142 us, 32 -> 64: 1142 vs 959 us;
// fp32 step 55.25 / 55.35 vs 54.79 / 54.74 ms; profiles/r10b_wgrad32_stg_narrow_{on,off}.jsonl): off
bool wgrad_stg_narrow() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_STG_NARROW");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

template <int BN, int BK, bool CONV>
void launch(const float* dy, const float* x, float* dwp, float* dbp, long ps, long R, int N, int K, int H, int W,
            int Cin, int S, long rps, hipStream_t st) {
  const int tn = (N + BN - 1) / BN, tk = (K + BK - 1) / BK;
  const long nwg = static_cast<long>(tn) * tk * S;
  if constexpr (BK == 128) {
    if (f32_mfma_mode() == 1 && wgrad_stg() && (BN == 128 || wgrad_stg_narrow())) {
      hipLaunchKernelGGL((wgrad_f32_stg_kernel<BN, CONV>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, st, dy, x,
                         dwp, dbp, ps, R, N, K, H, W, Cin, rps, tn, tk);
      return;
    }
  }
  if constexpr (BN >= 32 && (BK <= 128 || (BN == 128 && BK == 256))) {
    if (f32_mfma_mode() == 1 && !(BN == 32 && wgrad_f32_pipe32_off())) {
      hipLaunchKernelGGL((wgrad_f32_pipe_kernel<BN, BK, CONV, 3>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, st,
                         dy, x, dwp, dbp, ps, R, N, K, H, W, Cin, rps, tn, tk);
      return;
    }
  }
  if (f32_mfma_mode())
    hipLaunchKernelGGL((wgrad_f32_kernel<BN, BK, CONV, 1>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, st, dy, x,
                       dwp, dbp, ps, R, N, K, H, W, Cin, rps, tn, tk);
  else
    hipLaunchKernelGGL((wgrad_f32_kernel<BN, BK, CONV, 0>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, st, dy,
                       x, dwp, dbp, ps, R, N, K, H, W, Cin, rps, tn, tk);
}

int pick(int n) { return n <= 32 ? 32 : (n <= 64 ? 64 : 128); }
// A/B switch: the 32-wide N tile with a 256-wide K tile (each wave 32 x 64: the dY fragment feeds two MFMA
// blocks) for K >= 256 (APPLESTAR_WGRAD32_BK=256).  Measured 20 % slower on the learner's narrow convs
// (profiles/r3v6_wgrad32_bk256_ab.jsonl: 75 KB of stages, 2 workgroups per CU), so off by default.
bool wgrad32_bk256() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD32_BK");
    return e != nullptr && e[0] == '2';
  }();
  return on;
}
// APPLESTAR_WGRAD_WIDE=1: 128 x 256 tiles (each wave 64 x 128) for N >= 128, K >= 256 in split-MFMA mode
bool wgrad_wide() {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_WIDE");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}
// the K tile: a wave covers >= 32 columns (2 waves along K for BN >= 64, 4 for the 32-wide N tile)
int pick_k(int k, int bn) {
  if (bn == 32) return (k >= 256 && wgrad32_bk256()) ? 256 : 128;
  if (bn == 128 && k >= 256 && wgrad_wide() && f32_mfma_mode() == 1) return 256;
  return k <= 64 ? 64 : 128;
}

}  // namespace

// target workgroup count of the split-R decomposition (APPLESTAR_WGRAD_F32_WG): fp32 step 62.4 / 62.5 ms at
// 1024, 61.6 / 62.0 at 3072, flat to 8192, 64.5 at 512, 68.5 at 256 (profiles/r4t_wgrad_f32_wg_sweep.txt)
long wgrad_f32_target_wg() {
  static const long v = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_F32_WG");
    const long x = e ? std::atol(e) : 3072;
    return x >= 64 ? x : 3072;
  }();
  return v;
}

// few-row products (R < 2048: the heads' / critics' MLPs at R = 384 / 390 - 33 weight gradients per fp32 step, each
// ~4 workgroups walking all R rows in ~32 us): slices of at least this many rows plus one column reduction
// (APPLESTAR_WGRAD_SMALL_R; 0 = one slice).  fp32 step 54.50 / 54.30 ms (0) -> 53.96 / 53.89 (48), 54.08 / 54.03
// (96), 54.21 / 54.31 (192) on one box (profiles/r10c_bench_small_r.txt)
long wgrad_f32_small_r_rows() {
  static const long v = [] {
    const char* e = std::getenv("APPLESTAR_WGRAD_SMALL_R");
    return e ? std::atol(e) : 48L;
  }();
  return v;
}

int wgrad_f32_splits(long R, int N, int K) {
  const int bn = pick(N), bk = pick_k(K, bn);
  const long tiles = static_cast<long>((N + bn - 1) / bn) * ((K + bk - 1) / bk);
  const long target = wgrad_f32_target_wg();
  long S = (target + tiles - 1) / tiles;                 // ~target workgroups
  const long small = wgrad_f32_small_r_rows();
  const long max_s = R < 2048 ? (small > 0 && R >= 2 * small ? R / small : 1)
                              : (R + 127) / 128;         // >= 4 stages per slice
  if (S > max_s) S = max_s;
  const long max_part = (16L << 20) / (static_cast<long>(N) * K);   // partials <= 64 MB
  if (S > max_part) S = max_part;
  if (S < 1) S = 1;
  if (S > 4096) S = 4096;
  return static_cast<int>(S);
}

void wgrad_f32(const float* dy, const float* x, float* dw_part, float* db_part, long part_stride, long R, int N, int K,
               int H, int W, int Cin, int S, hipStream_t st) {
  long rps = (R + S - 1) / S;
  rps = (rps + 31) / 32 * 32;
  const bool conv = Cin > 0;
  const int bn = pick(N), bk = pick_k(K, bn);
#define AS_WGF(BNv, BKv)                                                                   \
  if (bn == BNv && bk == BKv) {                                                            \
    if (conv) launch<BNv, BKv, true>(dy, x, dw_part, db_part, part_stride, R, N, K, H, W, Cin, S, rps, st); \
    else launch<BNv, BKv, false>(dy, x, dw_part, db_part, part_stride, R, N, K, H, W, Cin, S, rps, st);     \
    return;                                                                                \
  }
  AS_WGF(128, 128) AS_WGF(128, 64) AS_WGF(64, 128) AS_WGF(64, 64) AS_WGF(32, 128) AS_WGF(32, 256) AS_WGF(128, 256)
#undef AS_WGF
}

}  // namespace as
