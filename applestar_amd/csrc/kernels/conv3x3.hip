// 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on the MFMA matrix cores (gfx950), NHWC bf16,
// with the bias, residual add and ReLU fused into the epilogue.  SURVEY K7/K8: the spatial-encoder
// downsample convs and ResBlocks (spatial_encoder.py:74-86, res_block.py:50-65), the location head's
// gated res-blocks and upsample convs (action_arg_head.py:417-446, module_utils.py:204-231).
//
//   out[m, n] = act( bias[n] + res[m, n] + sum_{tap, c} x[shift_tap(m), c] * w[n, tap, c] )
//
// GEMM view: M = B*H*W output pixels, N = Cout, K = 9*Cin (tap-major, channel-minor: exactly the
// memory order of a channels_last [Cout, Cin, 3, 3] weight, so the weight needs no repacking).
// The A operand is gathered on the fly: K-step (tap, c0..c0+BK) of tile row m reads BK contiguous
// channels of input pixel (y+dy, x+dx) - one 16-B load per 8 channels, zeros outside the image.
//
// Tiling (per 256-thread workgroup): BM = 128 pixels x BN (128 / 64 / 32) output channels, BK = 64
// (or 32 when Cin = 32).  Register-staged double buffer: the global loads of K-step k+1 are issued
// before the MFMAs of step k and written to the other LDS buffer after them (one barrier per step).
// LDS rows are padded by 16 B so each 16-lane ds_read_b128 group of an MFMA fragment read hits 16
// distinct 4-bank groups.  v_mfma_f32_16x16x32_bf16: lane l holds A[row l&15][k 8(l>>4)..+8] and
// B[k 8(l>>4)..+8][col l&15]; C[row 4(l>>4)+i][col l&15].  Epilogue: fp32 accumulators -> LDS ->
// 16-B coalesced rows (+bias +residual, ReLU, bf16).  Workgroup ids are remapped so consecutive
// M-tiles (which share input halo rows) run on one XCD's L2.
// The input gradient of a conv is the same operation on dy with the flipped, transposed weight.
#include <cstdlib>

#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ __forceinline__ bf8v as_bf8(const uint4& u) {
  bf8v r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// fp32 tile cs [128][CPAD] (LDS) -> out rows m0.., channels n0..n0+BN in 16-B pieces:
//   v = cs + bias (+ res | * [res > 0] for ACT_DRELU), then ReLU for ACT_RELU; bf16.
// ACT_DRELU is the input-gradient form: dpre = dx * (y > 0) with y (the layer's ReLU output) in res.
// A thread's 8-channel piece is the same in every row it handles (256 % (BN / 8) == 0): its bias is loaded
// once and every residual row is requested before the first is used, so the epilogue pays one memory
// latency, not one per row (the per-row form cost 29 us of an 89 us ResBlock conv, r2bu ablation).
template <int BN, int CPAD>
__device__ __forceinline__ void conv_epilogue(const float* cs, long m0, int n0, long M, int Cout,
                                              const float* __restrict__ bias, const bf16_t* __restrict__ res,
                                              bf16_t* __restrict__ out, int act) {
  constexpr int CPR = BN / 8;          // 8-channel pieces per row
  constexpr int RSTEP = 256 / CPR;     // rows between a thread's consecutive pieces
  constexpr int IT = 128 / RSTEP;
  static_assert(256 % CPR == 0, "epilogue piece mapping");
  const int c8 = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  const int n = n0 + 8 * c8;
  if (n >= Cout) return;
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = bias ? bias[n + e] : 0.f;
  uint4 rv[IT];
  if (res) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const long m = m0 + r0 + k * RSTEP;
      rv[k] = m < M ? *reinterpret_cast<const uint4*>(res + m * Cout + n) : make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int rr = r0 + k * RSTEP;
    const long m = m0 + rr;
    if (m >= M) break;
    float v[8];
    const float4 c0 = *reinterpret_cast<const float4*>(cs + rr * CPAD + 8 * c8);
    const float4 c1 = *reinterpret_cast<const float4*>(cs + rr * CPAD + 8 * c8 + 4);
    v[0] = c0.x + bv[0]; v[1] = c0.y + bv[1]; v[2] = c0.z + bv[2]; v[3] = c0.w + bv[3];
    v[4] = c1.x + bv[4]; v[5] = c1.y + bv[5]; v[6] = c1.z + bv[6]; v[7] = c1.w + bv[7];
    if (res) {
      const uint32_t q4[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
      if (act == ACT_DRELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(__uint_as_float(q4[e] << 16) > 0.f)) v[2 * e] = 0.f;
          if (!(__uint_as_float(q4[e] & 0xffff0000u) > 0.f)) v[2 * e + 1] = 0.f;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] += __uint_as_float(q4[e] << 16);
          v[2 * e + 1] += __uint_as_float(q4[e] & 0xffff0000u);
        }
      }
    }
    if (act == ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    uint4 u;
    u.x = f2bf2(v[0], v[1]);
    u.y = f2bf2(v[2], v[3]);
    u.z = f2bf2(v[4], v[5]);
    u.w = f2bf2(v[6], v[7]);
    *reinterpret_cast<uint4*>(out + m * Cout + n) = u;
  }
}

template <int BN_, int BK_>
struct ConvCfg {
  static constexpr int BM = 128, BN = BN_, BK = BK_;
  static constexpr int NT = 256;
  static constexpr int WN = BN_ >= 128 ? 2 : 1;  // waves along N
  static constexpr int WM = 4 / WN;              // waves along M
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int LDK = BK + 16;            // padded LDS row (bf16) = 16 mod 32: conflict-free b128 reads
  static constexpr int CH = BK / 8;              // 16-B chunks per row
  static constexpr int A_IT = (BM * CH + NT - 1) / NT;
  static constexpr int B_IT = (BN * CH + NT - 1) / NT;
  static constexpr int STAGE = (BM + BN) * LDK;  // bf16 elements per pipeline stage
  static constexpr int CPAD = BN + 4;            // fp32 epilogue tile pitch
  static constexpr int SMEM_BYTES = (2 * STAGE * 2 > BM * CPAD * 4) ? 2 * STAGE * 2 : BM * CPAD * 4;
  static_assert((BM * CH) % NT == 0, "A tile chunks");
};

// SPLIT_TAP: Cin < BK (Cin = 16), so one K-step spans several taps: every 16-B chunk finds its own tap,
// and K = 9 Cin is not a multiple of BK (the tail reads zeros).  Cout need not be a multiple of BN.
template <int BN, int BK, bool SPLIT_TAP>
__global__ __launch_bounds__(256) void conv3x3_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const float* __restrict__ bias, const bf16_t* __restrict__ res,
                                                      bf16_t* __restrict__ out, int B, int H, int W, int Cin, int Cout,
                                                      int act) {
  using C = ConvCfg<BN, BK>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM_BYTES];
  bf16_t* st = reinterpret_cast<bf16_t*>(smem);

  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  const int K = 9 * Cin;
  const int ntn = (Cout + BN - 1) / BN;
  // XCD-aware bijective remap of the flat workgroup id (8 XCDs, round-robin dispatch)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int tn = wg % ntn;
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lr = lane & 15, lg = lane >> 4;

  // Operand fetch through buffer descriptors: out-of-image taps and rows past M use an offset beyond
  // num_records, which the hardware range check turns into zeros - no branches around the loads, so all
  // A_IT + B_IT loads of a K-step issue back to back and stay in flight under the MFMAs of the previous one.
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x), 0, static_cast<int>(M * Cin * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(w), 0, static_cast<int>(static_cast<long>(Cout) * K * 2), 0x00020000);
  constexpr int kOOB = 0x7ffffff0;

  // per-thread A rows (fixed across K-steps): pixel index and a 9-bit in-image mask over the taps
  int a_pix[C::A_IT], a_row[C::A_IT], a_ch[C::A_IT], a_ok[C::A_IT];
#pragma unroll
  for (int i = 0; i < C::A_IT; ++i) {
    const int idx = tid + i * C::NT;
    a_row[i] = idx / C::CH;
    a_ch[i] = idx % C::CH;
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
    const int n = idx / C::CH, ch = idx % C::CH;
    b_off[i] = (idx < BN * C::CH && n0 + n < Cout) ? ((n0 + n) * K + 8 * ch) * 2 : kOOB;
  }

  uint4 ra[C::A_IT], rb[C::B_IT];
  auto load_regs = [&](int kt) {
    const int k0 = kt * BK;
    if (SPLIT_TAP) {
#pragma unroll
      for (int i = 0; i < C::A_IT; ++i) {
        const int k = k0 + 8 * a_ch[i];
        const int tap = k / Cin, c = k - tap * Cin;
        const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
        const int off = (k < K && ((a_ok[i] >> tap) & 1)) ? ((a_pix[i] + shift) * Cin + c) * 2 : kOOB;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
        ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    } else {
      const int tap = k0 / Cin, c0 = k0 - tap * Cin;
      const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
#pragma unroll
      for (int i = 0; i < C::A_IT; ++i) {
        const int off = ((a_ok[i] >> tap) & 1) ? ((a_pix[i] + shift) * Cin + c0 + 8 * a_ch[i]) * 2 : kOOB;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
        ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int kc = k0 + 8 * ((tid + i * C::NT) % C::CH);
      const int off = (b_off[i] == kOOB || (SPLIT_TAP && kc >= K)) ? kOOB : b_off[i] + k0 * 2;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_lds = [&](int s) {
    bf16_t* A = st + s * C::STAGE;
    bf16_t* Bs = A + C::BM * C::LDK;
#pragma unroll
    for (int i = 0; i < C::A_IT; ++i)
      *reinterpret_cast<uint4*>(A + a_row[i] * C::LDK + 8 * a_ch[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int idx = tid + i * C::NT;
      if ((BN * C::CH) % C::NT == 0 || idx < BN * C::CH) {
        const int n = idx / C::CH, ch = idx % C::CH;
        *reinterpret_cast<uint4*>(Bs + n * C::LDK + 8 * ch) = rb[i];
      }
    }
  };

  f4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int KT = (K + BK - 1) / BK;
  load_regs(0);
  store_lds(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_regs(kt + 1);
    const bf16_t* A = st + cur * C::STAGE;
    const bf16_t* Bs = A + C::BM * C::LDK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf8v af[C::FM], bfr[C::FN];
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
        af[i] = as_bf8(*reinterpret_cast<const uint4*>(A + (wm * C::TM + i * 16 + lr) * C::LDK + ks * 32 + 8 * lg));
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        bfr[j] = as_bf8(*reinterpret_cast<const uint4*>(Bs + (wn * C::TN + j * 16 + lr) * C::LDK + ks * 32 + 8 * lg));
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_lds(cur ^ 1);
    __syncthreads();
  }

  // epilogue: accumulators -> LDS (fp32) -> coalesced 16-B rows with bias / residual / activation
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        cs[(wm * C::TM + i * 16 + 4 * lg + e) * C::CPAD + wn * C::TN + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  conv_epilogue<BN, C::CPAD>(cs, m0, n0, M, Cout, bias, res, out, act);
}

// ------------------------------------------------------------------------------------------------
// Halo-window variant for narrow maps (W <= 40, Cin % 64 == 0): the implicit GEMM above gathers every
// input pixel once per tap (9x the image through LDS, and its LDS stores plus fragment reads saturate
// the LDS port before the MFMAs do).  Here a 128-pixel tile's input is staged ONCE per 64-channel
// chunk as a window of 128 + 2W + 2 consecutive pixel rows (the tile plus one image row and one pixel
// of halo on each side); every tap then reads its A fragments from that window at a constant row
// offset dy*W + dx and zeroes the rows whose neighbour falls outside the image (per-lane 9-bit masks).
// Only the weight tile is re-staged per (tap, chunk) step, double-buffered through registers.
// HALO_ABL: timing-ablation bits for tools/native/conv_ablation.cpp only (1: no weight restaging, 2: no window
// restaging, 8: no loop barriers, 16: two K-steps only, 32: no epilogue, 64: no prologue loads); 0 in every
// library build
#ifndef HALO_ABL
#define HALO_ABL 0
#endif

template <int BN, int WP>
struct HaloCfg {
  static constexpr int BM = 128, CK = 64, NT = 256;
  static constexpr int WN = BN >= 128 ? 2 : 1, WM = 4 / WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int P = CK + 16;                // LDS row pitch (bf16) = 16 mod 32: conflict-free ds_read_b128 groups
  static constexpr int NR = WP * NT / 8;           // window rows covered by WP 16-B pieces per thread
  static constexpr int B_IT = BN * (CK / 8) / NT;  // weight pieces per thread
  static constexpr int WIN = NR * P, BT = BN * P;  // bf16 elements
  static constexpr int MAIN = (WIN + 2 * BT) * 2;  // bytes
  static constexpr int CPAD = BN + 4;
  static constexpr int SMEM = MAIN > BM * CPAD * 4 ? MAIN : BM * CPAD * 4;
  static_assert(B_IT * NT == BN * (CK / 8), "weight tile pieces");
};

template <int BN, int WP>
__global__ __launch_bounds__(256) void conv3x3_halo_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                           const float* __restrict__ bias,
                                                           const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                                                           int B, int H, int W, int Cin, int Cout, int act) {
  using C = HaloCfg<BN, WP>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::SMEM];
  bf16_t* win = reinterpret_cast<bf16_t*>(smem);
  bf16_t* bts = win + C::WIN;

  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  const int K = 9 * Cin;
  const int ntn = (Cout + BN - 1) / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int tn = wg % ntn;
  const long m0 = static_cast<long>(wg / ntn) * C::BM;
  const int n0 = tn * BN;
  const long wb0 = m0 - (W + 1);                    // window row 0 <-> pixel wb0
  const int nrows = C::BM + 2 * W + 2;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lr = lane & 15, lg = lane >> 4;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x), 0, static_cast<int>(M * Cin * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(w), 0, static_cast<int>(static_cast<long>(Cout) * K * 2), 0x00020000);
  constexpr int kOOB = 0x7ffffff0;

  // 9-bit in-image masks of this lane's A-fragment rows (pixel wm*TM + 16 i + lr of the tile)
  int ok9[C::FM];
#pragma unroll
  for (int i = 0; i < C::FM; ++i) {
    const long m = m0 + wm * C::TM + 16 * i + lr;
    ok9[i] = 0;
    if (m < M) {
      const int rem = static_cast<int>(m % HW);
      const int yy = rem / W, xx = rem - yy * W;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int y2 = yy + t / 3 - 1, x2 = xx + t % 3 - 1;
        ok9[i] |= (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W) << t;
      }
    }
  }

  uint4 rw[WP], rb[C::B_IT];
  auto load_win = [&](int c0) {
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int piece = tid + i * C::NT;
      const int row = piece >> 3, ch = (piece & 7) * 8;
      const long pix = wb0 + row;
      const int off = (row < nrows && pix >= 0 && pix < M) ? static_cast<int>((pix * Cin + c0 + ch) * 2) : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0);
      rw[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_win = [&]() {
#pragma unroll
    for (int i = 0; i < WP; ++i) {
      const int piece = tid + i * C::NT;
      const int row = piece >> 3, ch = (piece & 7) * 8;
      if (row < nrows) *reinterpret_cast<uint4*>(win + row * C::P + ch) = rw[i];
    }
  };
  auto load_b = [&](int step) {
    const int tap = step % 9, c0 = (step / 9) * C::CK;
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int piece = tid + i * C::NT;
      const int n = piece >> 3, ch = (piece & 7) * 8;
      const int off = n0 + n < Cout ? ((n0 + n) * K + tap * Cin + c0 + ch) * 2 : kOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_b = [&](int buf) {
    bf16_t* Bs = bts + buf * C::BT;
#pragma unroll
    for (int i = 0; i < C::B_IT; ++i) {
      const int piece = tid + i * C::NT;
      const int n = piece >> 3, ch = (piece & 7) * 8;
      *reinterpret_cast<uint4*>(Bs + n * C::P + ch) = rb[i];
    }
  };

  f4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = (HALO_ABL & 16) ? 2 : 9 * (Cin / C::CK);
  if (!(HALO_ABL & 64)) {
    load_win(0);
    load_b(0);
    store_win();
    store_b(0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = (HALO_ABL & 1) ? 0 : (step & 1);
    const int tap = step % 9;
    const bool next = step + 1 < nsteps && !(HALO_ABL & 1);
    const bool new_chunk = step + 1 < nsteps && (step + 1) % 9 == 0 && !(HALO_ABL & 2);
    if (next) load_b(step + 1);
    if (new_chunk) load_win(((step + 1) / 9) * C::CK);
    const int shift = (W + 1) + (tap / 3 - 1) * W + (tap % 3 - 1);
    const bf16_t* Bs = bts + cur * C::BT;
    // every fragment of the step is read before the first MFMA: the reads of the second k-slice land while
    // the first slice's MFMAs run, so the LDS latency is exposed once per step instead of once per slice
    // (with the loop barrier keeping a CU's waves in phase, the other wave on the SIMD cannot hide it)
    constexpr int KS = C::CK / 32;
    uint4 ua[KS][C::FM], ub[KS][C::FN];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
        ua[ks][i] = *reinterpret_cast<const uint4*>(win + (wm * C::TM + 16 * i + lr + shift) * C::P + ks * 32 + 8 * lg);
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        ub[ks][j] = *reinterpret_cast<const uint4*>(Bs + (wn * C::TN + 16 * j + lr) * C::P + ks * 32 + 8 * lg);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf8v af[C::FM];
#pragma unroll
      for (int i = 0; i < C::FM; ++i) af[i] = as_bf8(((ok9[i] >> tap) & 1) ? ua[ks][i] : make_uint4(0, 0, 0, 0));
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], as_bf8(ub[ks][j]), acc[i][j], 0, 0, 0);
    }
    if (new_chunk) {
      if (!(HALO_ABL & 8)) __syncthreads();           // every wave is done reading the old window
      store_win();
    }
    if (next) store_b(cur ^ 1);
    if (!(HALO_ABL & 8)) __syncthreads();
  }

  if (HALO_ABL & 32) {            // ablation: no epilogue (one value per lane keeps the MFMAs alive)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == 12345.f) out[threadIdx.x] = 1;
    return;
  }
  // epilogue (as conv3x3_kernel): fp32 tile in LDS -> 16-B rows with bias / residual / activation
  float* cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        cs[(wm * C::TM + i * 16 + 4 * lg + e) * C::CPAD + wn * C::TN + j * 16 + lr] = acc[i][j][e];
  __syncthreads();
  conv_epilogue<BN, C::CPAD>(cs, m0, n0, M, Cout, bias, res, out, act);
}

template <int BN, int WP>
void launch_halo(const bf16_t* x, const bf16_t* w, const float* bias, const bf16_t* res, bf16_t* out, int B, int H,
                 int W, int Cin, int Cout, int act, hipStream_t s) {
  const long M = static_cast<long>(B) * H * W;
  const long nwg = (M + 127) / 128 * ((Cout + BN - 1) / BN);
  if (nwg == 0) return;
  hipLaunchKernelGGL((conv3x3_halo_kernel<BN, WP>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w, bias, res,
                     out, B, H, W, Cin, Cout, act);
}

// window pieces per thread for a map width: (128 + 2W + 2) rows x 8 pieces over 256 threads
bool halo_pieces(int W, int* wp) {
  const int need = ((128 + 2 * W + 2) * 8 + 255) / 256;
  if (need <= 6) *wp = 6;
  else if (need <= 8) *wp = 8;
  else return false;
  return true;
}

bool use_halo(int W, int Cin, int Cout) {
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_CONV_HALO");
    return e == nullptr || e[0] != '0';
  }();
  int wp = 0;
  return on && Cin % 64 == 0 && (Cout % 128 == 0 || Cout == 64) && halo_pieces(W, &wp);
}

template <int BN, int BK, bool SPLIT_TAP = false>
void launch(const bf16_t* x, const bf16_t* w, const float* bias, const bf16_t* res, bf16_t* out, int B, int H, int W,
            int Cin, int Cout, int act, hipStream_t s) {
  const long M = static_cast<long>(B) * H * W;
  const long mt = (M + 127) / 128;
  const long nwg = mt * ((Cout + BN - 1) / BN);
  if (nwg == 0) return;
  hipLaunchKernelGGL((conv3x3_kernel<BN, BK, SPLIT_TAP>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x, w,
                     bias, res, out, B, H, W, Cin, Cout, act);
}

bool small_m_bk128() {   // APPLESTAR_CONV_SMALLM_BK=64: the 64-wide K-steps (A/B)
  static const bool on = [] {
    const char* e = std::getenv("APPLESTAR_CONV_SMALLM_BK");
    return e == nullptr || std::atoi(e) != 64;
  }();
  return on;
}

}  // namespace

bool conv3x3_supported(int Cin, int Cout) {  // (the host wrapper also bounds B*H*W*Cin*2 < 2^31)
  const bool cin_ok = Cin == 16 || (Cin % 32 == 0 && Cin >= 32);
  const bool cout_ok = Cout == 16 || Cout == 32 || Cout == 64 || Cout % 128 == 0;
  return cin_ok && cout_ok;
}

void conv3x3_fwd(const void* x, const void* w, const float* bias, const void* res, void* out, int B, int H, int W,
                 int Cin, int Cout, int act, hipStream_t s) {
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(w);
  const bf16_t* rp = static_cast<const bf16_t*>(res);
  bf16_t* op = static_cast<bf16_t*>(out);
  const bool k64 = Cin % 64 == 0;
  static const bool small_m = [] {
    const char* e = std::getenv("APPLESTAR_CONV_SMALLM");
    return e == nullptr || e[0] != '0';
  }();
  const long mt = (static_cast<long>(B) * H * W + 127) / 128;
  if (small_m && Cin % 32 == 0 && Cout % 32 == 0 && mt * ((Cout + 127) / 128) < 64) {
    // few output tiles (the actor's B = 1..16 forwards: a 19 x 20 map is 3 row tiles - 3 workgroups walking all of
    // K for ~20 us): 32-wide output tiles give 4x the workgroups.  Each K-step of these few workgroups waits out a
    // whole memory latency, so 128-wide K-steps (Cin % 128) halve the dependent chain.  (A split-K form - fp32
    // partials reduced by the last-arriving workgroup - measured slower, 22 vs 15 us: the device-scope release /
    // acquire fences around the partials write back and invalidate the L2, profiles/r8v_timeline_b1_splitk_conv.txt)
    if (Cin % 128 == 0 && small_m_bk128()) launch<32, 128>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else if (k64) launch<32, 64>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else launch<32, 32>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    return;
  }
  if (use_halo(W, Cin, Cout)) {        // narrow maps: halo window staged once per channel chunk
    int npc = 0;
    halo_pieces(W, &npc);
    if (Cout % 128 == 0) {
      if (npc == 6) launch_halo<128, 6>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
      else launch_halo<128, 8>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    } else {
      if (npc == 6) launch_halo<64, 6>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
      else launch_halo<64, 8>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    }
    return;
  }
  if (Cin == 16) {                     // K-steps straddle taps
    if (Cout % 128 == 0) launch<128, 32, true>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else if (Cout == 64) launch<64, 32, true>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else launch<32, 32, true>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    return;
  }
  if (Cout % 128 == 0) {
    if (k64) launch<128, 64>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else launch<128, 32>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
  } else if (Cout == 64) {
    if (k64) launch<64, 64>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else launch<64, 32>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
  } else {
    if (k64) launch<32, 64>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
    else launch<32, 32>(xp, wp, bias, rp, op, B, H, W, Cin, Cout, act, s);
  }
}

}  // namespace as
