// fp32 GEMM  out[M, N] = act(A[M, K] B[N, K]^T + bias (+ res))  with the weight operand PRE-SPLIT (split-MFMA mode).
//
// The split ring GEMM (gemm_f32.hip + f32_pipe.h) splits both operands into three bf16 parts in registers, in every
// wave that reads them: ~44 VALU per fragment, 4 fragments per 24 MFMAs, and the B fragment of a 2 x 2 wave tile is
// split twice per workgroup.  B is a weight: it changes once per optimizer step and is read by every M-tile.  Here
// it is split ONCE per step (presplit_b_kernel, a derived weight form) into the MFMA's own fragment order:
//
//   planes[nb][kt][p][lane] = 8 bf16 (16 B): part p of B[32 nb + (lane & 31)][16 kt + 8 (lane >> 5) + 0..7]
//
// so a wave's fragment of (32-row block nb, 16-deep K-step kt) is three fully coalesced 1-KB loads.  The B
// fragments bypass LDS: each wave streams its two fragments straight into registers one K-step ahead (inline-asm
// buffer loads counted with the ring's own vmcnt waits), while the LDS-DMA ring (f32_pipe.h) carries only the A
// rows (8 KB a stage).  Per K-step a wave splits 2 fragments instead of 4; the LDS traffic per step halves.
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"
#include "../f32_pipe.h"

namespace as {
namespace {

using pipe::f16v;
using pipe::i32x4;

constexpr int kPsbBM = 128, kPsbBN = 128, kPsbNS = 3, kPsbRB = 64;   // 16 fp32 per A row and K-step
constexpr int kPsbAStage = kPsbBM * kPsbRB;                             // 8 KB of A rows per stage

// trans: the source is B^T ([K][N] row-major, e.g. a weight W [N_out][K_in] whose transpose feeds the dX product)
__global__ __launch_bounds__(256) void presplit_b_kernel(const float* __restrict__ b, int N, int K, int KT, long total,
                                                         bool trans, u32v4* __restrict__ out) {
  const long gid = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (gid >= total) return;
  const int lane = static_cast<int>(gid & 63);
  const long rest = gid >> 6;
  const int kt = static_cast<int>(rest % KT);
  const long nb = rest / KT;
  const long n = nb * 32 + (lane & 31);
  const int k0 = kt * 16 + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
    v[t] = (n < N && k0 + t < K) ? (trans ? b[static_cast<long>(k0 + t) * N + n] : b[n * K + k0 + t]) : 0.f;
  const Split3 s = split8(v);
  u32v4* o = out + (nb * KT + kt) * 3 * 64 + lane;
  o[0] = s.p[0];
  o[64] = s.p[1];
  o[128] = s.p[2];
}

// many weights' planes in one launch (the per-optimizer-step rebuild of every pre-split form)
__global__ __launch_bounds__(256) void multi_presplit_kernel(const PresplitArgs a) {
  const int blk = blockIdx.x;
  int t = 0;
  while (t + 1 < a.n && a.block_start[t + 1] <= blk) ++t;
  const int N = a.N[t], K = a.K[t], KT = (K + 15) / 16;
  const long total = static_cast<long>((N + 31) / 32) * KT * 64;
  const long gid = static_cast<long>(blk - a.block_start[t]) * 256 + threadIdx.x;
  if (gid >= total) return;
  const float* b = a.src[t];
  const bool trans = a.trans[t] != 0;
  const int lane = static_cast<int>(gid & 63);
  const long rest = gid >> 6;
  const int kt = static_cast<int>(rest % KT);
  const long nb = rest / KT;
  const long n = nb * 32 + (lane & 31);
  const int k0 = kt * 16 + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    v[q] = (n < N && k0 + q < K) ? (trans ? b[static_cast<long>(k0 + q) * N + n] : b[n * K + k0 + q]) : 0.f;
  const Split3 sp = split8(v);
  u32v4* o = static_cast<u32v4*>(a.dst[t]) + (nb * KT + kt) * 3 * 64 + lane;
  o[0] = sp.p[0];
  o[64] = sp.p[1];
  o[128] = sp.p[2];
}

// 16 B of a B fragment plane into registers, outside the compiler's waitcnt tracking (counted with the DMA ring)
__device__ __forceinline__ void bload(u32v4& dst, i32x4 r, int voff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(dst) : "v"(voff), "s"(r) : "memory");
}

// wait until at most N vector-memory ops are outstanding; ties the B registers about to be read to the wait
template <int N>
__device__ __forceinline__ void wait_b(Split3 (&b)[2]) {
  asm volatile("s_waitcnt vmcnt(%6)"
               : "+v"(b[0].p[0]), "+v"(b[0].p[1]), "+v"(b[0].p[2]), "+v"(b[1].p[0]), "+v"(b[1].p[1]), "+v"(b[1].p[2])
               : "n"(N)
               : "memory");
}

// The one-register-set main loop (128 VGPRs): per K-step kt [barrier] MFMAs of B fragment 0, B(kt + 1) fragment 0
// into the freed registers, MFMAs of fragment 1, B(kt + 1) fragment 1, then the A rows of kt + 2 into the ring
// stage read at kt - 1.  The wait for B(kt + 1) / A(kt + 1) sits at the END of step kt (vmcnt(A_PW): A(kt + 2) may
// fly), so a register the compiler carries around the loop is never copied before its load returned.
template <class C, int A_PW, class IssueA>
__device__ __forceinline__ void psb_sb_loop(char* ring, const IssueA& issue_a, i32x4 br, const int (&b_off)[2], int KT,
                                            f16v (&acc)[2][2], int wm, int l32, int h) {
  Split3 b[2];
  auto stage = [&](int kt) { return ring + (kt % 3) * kPsbAStage; };
  auto load_frag = [&](int j, int kt) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bload(b[j].p[p], br, b_off[j] >= 0 && kt < KT ? b_off[j] + (kt * 3 + p) * 1024 : pipe::kOOB);
  };
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  load_frag(0, 0);
  load_frag(1, 0);
  issue_a(stage(0), 0);
  issue_a(stage(1), 1);
  wait_b<A_PW>(b);
  for (int kt = 0; kt < KT; ++kt) {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const char* st = stage(kt);
    const Split3 sa0 = pipe::frag<C>(st, wm * C::TM + l32, 2 * h);
    const Split3 sa1 = pipe::frag<C>(st, wm * C::TM + 32 + l32, 2 * h);
    acc[0][0] = mfma_x6(b[0], sa0, acc[0][0]);
    acc[1][0] = mfma_x6(b[0], sa1, acc[1][0]);
    load_frag(0, kt + 1);
    acc[0][1] = mfma_x6(b[1], sa0, acc[0][1]);
    acc[1][1] = mfma_x6(b[1], sa1, acc[1][1]);
    load_frag(1, kt + 1);
    issue_a(stage(kt + 2), kt + 2);
    wait_b<A_PW>(b);
  }
  pipe::wait_vm<0>();
}

// DB: two B register sets (the next K-step's fragments load during this step's MFMAs: 204 VGPRs, 2 waves / SIMD);
// else one set, each fragment reloaded right after its last MFMA (3 waves / SIMD)
template <bool STAGED, bool DB>
__global__ __launch_bounds__(256, DB ? 2 : 3) void gemm_f32_psb_kernel(const float* __restrict__ a,
                                                              const u32v4* __restrict__ bs, int KT,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ res, float* __restrict__ out,
                                                              long M, int N, int K, int act) {
  // the staged epilogue reuses stage 0 for 32 x 128 floats (16 KB)
  using C = pipe::Cfg<kPsbBN, kPsbNS, 16, kPsbBM, 4>;
  // one ring array (stage = kt % 3, addressed at run time: the DMA is inline asm, so the compiler adds no waits
  // for it whatever it can prove about the stages); 32 KB so the staged epilogue can take its first 16 KB
  __shared__ __attribute__((aligned(16))) char ring[4 * kPsbAStage];
  constexpr int A_PW = kPsbAStage / 1024 / 4;                // A DMA chunks per wave per step (2)
  const int ntn = (N + kPsbBN - 1) / kPsbBN;
  const int wg = pipe::xcd_remap();
  const long m0 = static_cast<long>(wg / ntn) * kPsbBM;
  const int n0 = (wg % ntn) * kPsbBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;
  const i32x4 ar = pipe::rsrc(a, M * K * 4);
  const long nbt = (N + 31) / 32;
  const i32x4 br = pipe::rsrc(bs, nbt * KT * 3 * 1024);
  // A DMA pieces (the ring's lane-linear, swizzled layout: f32_pipe.h)
  int a_off[A_PW], a_k[A_PW];
#pragma unroll
  for (int c = 0; c < A_PW; ++c) {
    const int row = C::dma_row(wid + 4 * c, lane), p = C::dma_piece(row, lane);
    const long m = m0 + row;
    a_k[c] = 4 * p;
    a_off[c] = m < M ? static_cast<int>((m * K + 4 * p) * 4) : -1;
  }
  auto issue_a = [&](char* st, int kt) {
#pragma unroll
    for (int c = 0; c < A_PW; ++c)
      pipe::dma16(ar, st + (wid + 4 * c) * 1024,
                  a_off[c] >= 0 && kt < KT && kt * 16 + a_k[c] < K ? a_off[c] + kt * 64 : pipe::kOOB);
  };
  // this lane's B fragment j at K-step kt: ((nb KT + kt) 3 + p) KB + 16 lane
  const int nb0 = (n0 + wn * C::TN) / 32;
  int b_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b_off[j] = nb0 + j < nbt ? static_cast<int>((nb0 + j) * KT * 3 * 1024 + 16 * lane) : -1;
  auto issue_b = [&](Split3 (&dst)[2], int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bload(dst[j].p[p], br, b_off[j] >= 0 && kt < KT ? b_off[j] + (kt * 3 + p) * 1024 : pipe::kOOB);
  };

  f16v acc[C::FM][2];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  Split3 bq[2][2];
  auto stage = [&](int kt) { return ring + (kt % 3) * kPsbAStage; };
  if constexpr (DB) {
    // issue order per step kt (after its barrier): B(kt + 1), then A(kt + 2).  At the top of step kt the A rows of
    // kt (issued two steps back) and B(kt) (issued one step back, before A(kt + 1)) must have landed; A(kt + 1)
    // may stay in flight: vmcnt(A_PW)
    // The wait for a register set sits at the END of the step that loaded it (the top of the next step waits for
    // the same things): a register the compiler carries around the loop (a phi copy at the back edge) is then
    // never read before its load returned.
    auto step = [&](const char* st, char* next, int kt, Split3 (&bu)[2], Split3 (&bn)[2]) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_b(bn, kt + 1);
      issue_a(next, kt + 2);
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const Split3 sa = pipe::frag<C>(st, wm * C::TM + 32 * i + l32, 2 * h);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x6(bu[j], sa, acc[i][j]);
      }
      wait_b<A_PW>(bn);
    };
    issue_b(bq[0], 0);
    issue_a(stage(0), 0);
    issue_a(stage(1), 1);
    wait_b<A_PW>(bq[0]);
    // unrolled by the 2 register sets (a 6-step unroll - stages and sets all compile-time - blew the register
    // budget: 500+ VGPRs demanded, 255 spilled)
    for (int kt = 0; kt < KT; kt += 2) {
      step(stage(kt), stage(kt + 2), kt, bq[0], bq[1]);
      if (kt + 1 >= KT) break;
      step(stage(kt + 1), stage(kt + 3), kt + 1, bq[1], bq[0]);
    }
  } else {
    // issue order per step kt: [barrier] MFMAs of fragment 0, B(kt + 1) fragment 0 into its registers, MFMAs of
    // fragment 1, B(kt + 1) fragment 1, A(kt + 2).  At the top of step kt + 1: A(kt + 1) and B(kt + 1) landed,
    // A(kt + 2) may stay in flight: vmcnt(A_PW)
    Split3 (&b)[2] = bq[0];
    auto load_frag = [&](int j, int kt) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bload(b[j].p[p], br, b_off[j] >= 0 && kt < KT ? b_off[j] + (kt * 3 + p) * 1024 : pipe::kOOB);
    };
    load_frag(0, 0);
    load_frag(1, 0);
    issue_a(stage(0), 0);
    issue_a(stage(1), 1);
    wait_b<A_PW>(b);
    for (int kt = 0; kt < KT; ++kt) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* st = stage(kt);
      const Split3 sa0 = pipe::frag<C>(st, wm * C::TM + l32, 2 * h);
      const Split3 sa1 = pipe::frag<C>(st, wm * C::TM + 32 + l32, 2 * h);
      acc[0][0] = mfma_x6(b[0], sa0, acc[0][0]);
      acc[1][0] = mfma_x6(b[0], sa1, acc[1][0]);
      load_frag(0, kt + 1);
      acc[0][1] = mfma_x6(b[1], sa0, acc[0][1]);
      acc[1][1] = mfma_x6(b[1], sa1, acc[1][1]);
      load_frag(1, kt + 1);
      issue_a(stage(kt + 2), kt + 2);
      // at the end of the step (see the two-set form): B(kt + 1) and A(kt + 1) landed, A(kt + 2) may fly
      wait_b<A_PW>(b);
    }
  }
  pipe::wait_vm<0>();
  if constexpr (STAGED) {
    pipe::store_tile_staged<C, float>(acc, ring, out, bias, res, M, N, m0, n0, act);
  } else {
    pipe::store_tile<C::FM, 2>(acc, out, bias, res, M, N, m0 + wm * C::TM, n0 + wn * C::TN, act);
  }
}

// 3 x 3 / pad 1 convolution (NHWC x [B, H, W, Cin], Cout % 128 == 0, Cin % 16 == 0) on the pre-split weight planes
// of w [Cout, 3, 3, Cin] (= B [Cout, 9 Cin]); the A rows are the implicit im2col of the ring conv kernel
// (conv3x3_f32.hip): a lane's DMA piece is 4 channels of its pixel shifted by the K-step's tap, zeros outside
// the image.  Epilogue: bias / residual / ReLU (/ ReLU-mask of the residual) and the input-gradient extras (Epi2).
__global__ __launch_bounds__(256, 3) void conv3x3_f32_psb_kernel(const float* __restrict__ x,
                                                                 const u32v4* __restrict__ bs,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ res,
                                                                 float* __restrict__ out, int B, int H, int W,
                                                                 int Cin, int Cout, int act, const pipe::Epi2 e2) {
  using C = pipe::Cfg<kPsbBN, kPsbNS, 16, kPsbBM, 4>;
  __shared__ __attribute__((aligned(16))) char ring[4 * kPsbAStage];
  constexpr int A_PW = kPsbAStage / 1024 / 4;
  const int HW = H * W;
  const long M = static_cast<long>(B) * HW;
  const int K = 9 * Cin, KT = K / 16;
  const int ntn = Cout / kPsbBN;
  const int wg = pipe::xcd_remap();
  const long m0 = static_cast<long>(wg / ntn) * kPsbBM;
  const int n0 = (wg % ntn) * kPsbBN;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;
  const i32x4 xr = pipe::rsrc(x, M * Cin * 4);
  const long nbt = Cout / 32;
  const i32x4 br = pipe::rsrc(bs, nbt * KT * 3 * 1024);
  int a_pix[A_PW], a_ok[A_PW], a_c[A_PW];
#pragma unroll
  for (int c = 0; c < A_PW; ++c) {
    const int row = C::dma_row(wid + 4 * c, lane);
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
  auto issue_a = [&](char* st, int kt) {
    const int k0 = kt * 16, tap = k0 / Cin, c0 = k0 - tap * Cin;
    const int shift = (tap / 3 - 1) * W + (tap % 3 - 1);
#pragma unroll
    for (int c = 0; c < A_PW; ++c)
      pipe::dma16(xr, st + (wid + 4 * c) * 1024,
                  kt < KT && ((a_ok[c] >> tap) & 1) ? ((a_pix[c] + shift) * Cin + c0 + a_c[c]) * 4 : pipe::kOOB);
  };
  const int nb0 = (n0 + wn * C::TN) / 32;
  int b_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b_off[j] = static_cast<int>((nb0 + j) * KT * 3 * 1024 + 16 * lane);
  f16v acc[2][2];
  psb_sb_loop<C, A_PW>(ring, issue_a, br, b_off, KT, acc, wm, l32, h);
  pipe::store_tile<2, 2>(acc, out, bias, res, M, Cout, m0 + wm * C::TM, n0 + wn * C::TN, act, e2);
}

}  // namespace

long presplit_b_bytes(int N, int K) {
  const long nbt = (N + 31) / 32, KT = (K + 15) / 16;
  return nbt * KT * 3 * 1024;
}

void presplit_b(const float* b, int N, int K, bool trans, void* out, hipStream_t s) {
  const int KT = (K + 15) / 16;
  const long total = static_cast<long>((N + 31) / 32) * KT * 64;
  if (total == 0) return;
  hipLaunchKernelGGL(presplit_b_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, s, b, N, K, KT,
                     total, trans, static_cast<u32v4*>(out));
}

// N % 128 == 0 and K % 4 == 0 (the A rows stream in 16-B pieces); B pre-split by presplit_b
bool gemm_f32_psb_supported(long M, int N, int K) {
  return N % kPsbBN == 0 && K % 4 == 0 && K > 0 && M > 0 && M * K * 4 < 0x7ffffff0L &&
         presplit_b_bytes(N, K) < 0x7ffffff0L;
}

// variant: 0 = two B register sets (2 waves / SIMD), 1 = one set (3 waves / SIMD); >= 10: gemm_f32_v2 variant - 10
void gemm_f32_psb(const float* a, const void* bsplit, const float* bias, const float* res, float* out, long M, int N,
                  int K, int act, int variant, hipStream_t s) {
  if (variant >= 10) {        // both operands staged through the LDS ring (conv3x3_f32_v2.hip), variant - 10
    gemm_f32_v2(a, bsplit, bias, res, out, M, N, K, act, variant - 10, s);
    return;
  }
  const long nwg = (M + kPsbBM - 1) / kPsbBM * (N / kPsbBN);
  if (nwg == 0) return;
  const int KT = (K + 15) / 16;
  if (variant == 1)
    hipLaunchKernelGGL((gemm_f32_psb_kernel<true, false>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a,
                       static_cast<const u32v4*>(bsplit), KT, bias, res, out, M, N, K, act);
  else
    hipLaunchKernelGGL((gemm_f32_psb_kernel<true, true>), dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a,
                       static_cast<const u32v4*>(bsplit), KT, bias, res, out, M, N, K, act);
}

int conv_v2_variant();
// Cout % 128 (or 64 / 32 on the ring-staged kernel), Cin % 16 (every 16-deep K-step inside one tap), 32-bit offsets
bool conv3x3_f32_psb_supported(long M, int Cin, int Cout) {
  return (Cout % kPsbBN == 0 || ((Cout == 64 || Cout == 32) && conv_v2_variant() >= 0)) && Cin % 16 == 0 && Cin > 0 &&
         M * Cin * 4 < 0x7ffffff0L &&
         presplit_b_bytes(Cout, 9 * Cin) < 0x7ffffff0L && M * Cout < 0x7ffffff0L;
}

// APPLESTAR_CONV_V2: the design with both operands staged through the LDS ring (conv3x3_f32_v2.hip) and its
// variant (default 2: 4 x 1 waves, 2 stages, 4 workgroups per CU: 218 vs 235 us on the ResBlock conv,
// profiles/r8d_conv_v2.jsonl); -1 = the register-streamed weight planes below
int conv_v2_variant() {
  static const int v = [] {
    const char* e = std::getenv("APPLESTAR_CONV_V2");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

void conv3x3_f32_psb(const float* x, const void* wsplit, const float* bias, const float* res, const float* res2,
                     long res2_rows, const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int act,
                     hipStream_t s) {
  if (conv_v2_variant() >= 0) {
    conv3x3_f32_v2(x, wsplit, bias, res, res2, res2_rows, mask, out, B, H, W, Cin, Cout, act, conv_v2_variant(), s);
    return;
  }
  const long M = static_cast<long>(B) * H * W;
  const long nwg = (M + kPsbBM - 1) / kPsbBM * (Cout / kPsbBN);
  if (nwg == 0) return;
  pipe::Epi2 e2;
  e2.res2 = res2;
  e2.res2_rows = res2_rows;
  e2.mask = mask;
  hipLaunchKernelGGL(conv3x3_f32_psb_kernel, dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, x,
                     static_cast<const u32v4*>(wsplit), bias, res, out, B, H, W, Cin, Cout, act, e2);
}

void multi_presplit(const PresplitArgs& a, hipStream_t s) {
  const int nblk = a.block_start[a.n];
  if (nblk > 0) hipLaunchKernelGGL(multi_presplit_kernel, dim3(nblk), dim3(256), 0, s, a);
}

}  // namespace as
