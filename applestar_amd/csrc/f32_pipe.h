// The fp32 GEMM main loop shared by gemm_f32.hip and conv3x3_f32.hip (split-MFMA mode): a 128 x BN output tile per
// 256-thread workgroup, K-steps of BK (16 / 32) floats, tiles streamed global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds)
// through an NS-deep ring, products as bf16x6 split MFMAs (split_mfma.h) on fragments split in registers.
//
// Why this shape (measured, profiles/r3u_gemm_f32_ablation_*): the register-staged double buffer kept one 16 KB
// K-step in flight per workgroup and its memory side alone ran at 1.7 TB/s (the ablation without MFMAs took as
// long as the one without loads, and the two barely overlapped).  LDS-DMA needs no staging registers, so NS - 1
// K-steps stay in flight; the waits are counted (s_waitcnt vmcnt(N), never 0 in the loop) and the barrier is the
// raw s_barrier (a __syncthreads() would drain the DMA queue).
//
// LDS image (lane-linear, as the DMA writes it): a stage holds the A rows then the B rows, BK floats per row
// (BK / 4 16-B slots); one wave-instruction fills 1 KB of rows.  Slot s of row r holds column piece s ^ swz(r) -
// the swizzle rides on the per-lane SOURCE address - so the 16 rows read by a ds_read_b128 lane group land on 16
// distinct 4-bank groups.
//
// Loop (one barrier per K-step):  wait until this wave's loads of step kt landed (vmcnt((NS-2) * loads per
// step)) -> s_barrier (every wave's step kt landed; every wave finished reading step kt - 1) -> issue step
// kt + NS - 1 into the slot of step kt - 1 -> compute step kt.  Loads past the last step use an out-of-range
// offset (zeros into a slot nobody reads) so the counts stay uniform.
#pragma once
#include "common.h"
#include "split_mfma.h"

namespace as {
namespace pipe {

typedef __attribute__((ext_vector_type(16))) float f16v;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) int i32x4;

constexpr int kOOB = 0x7ffffff0;

// PIPE_ABL: timing-ablation bits for tools/native/gemm_f32_ablation.cpp only (1: fragments bit-cast instead of
// split (wrong values, no split VALU), 2: no MFMAs); 0 in every library build
#ifndef PIPE_ABL
#define PIPE_ABL 0
#endif

// NW waves per workgroup (4: 2 x 2 / 4 x 1 waves; 8: the 256-row / 256-column tiles, 2 waves per SIMD at one
// workgroup per CU - twice the MFMA work per staged byte of the 128 x 128 tile)
template <int BN_, int NS_, int BK_ = 16, int BM_ = 128, int NW_ = 4>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, NS = NS_, BK = BK_, NW = NW_, NT = 64 * NW_;
  static constexpr int WN = NW_ == 8 ? (BN_ >= 256 ? 4 : (BN_ >= 128 ? 2 : 1)) : (BN_ >= 128 ? 2 : 1);
  static constexpr int WM = NW_ / WN;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 32, FN = TN / 32;
  static constexpr int RB = BK * 4, SL = BK / 4;              // bytes / 16-B slots per LDS row
  static constexpr int RPI = 1024 / RB;                       // rows per DMA wave-instruction (1 KB)
  static constexpr int A_CH = BM / RPI, B_CH = BN / RPI;      // DMA chunks per stage
  static constexpr int A_PW = A_CH / NW;                      // A chunks per wave
  static constexpr int B_PW = B_CH >= NW ? B_CH / NW : 1;     // B chunks per wave (waves >= B_CH issue none)
  static_assert(A_PW >= 1 && A_CH % NW == 0, "A chunks must split evenly over the waves");
  static constexpr int STAGE = (BM + BN) * RB;                // bytes per stage array
  // slot swizzle: the 16 rows of a ds_read_b128 lane group on 16 distinct 4-bank groups (64-B rows: XOR with
  // bits 2-3 of the row; 128-B rows: bits 1-3)
  static __device__ __forceinline__ int swz(int r) { return BK == 16 ? (r >> 2) & 3 : (r >> 1) & 7; }
  static __device__ __forceinline__ int slot_of(int r, int p) { return p ^ swz(r); }
  // the DMA piece of `lane` in chunk `ch` (global chunk index within the A or B rows): row and column piece
  static __device__ __forceinline__ int dma_row(int ch, int lane) { return RPI * ch + lane / SL; }
  static __device__ __forceinline__ int dma_piece(int row, int lane) { return slot_of(row, lane % SL); }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// raw buffer resource (base, size in bytes; out-of-range offsets read zeros) as an SGPR quad for the asm DMA
__device__ __forceinline__ i32x4 rsrc(const void* base, long bytes) {
  const unsigned long a = reinterpret_cast<unsigned long>(base);
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>((a >> 32) & 0xffff));
  r[2] = static_cast<int>(bytes);
  r[3] = 0x00020000;
  return r;
}

// one LDS-DMA piece: 16 B from the buffer at byte offset voff (kOOB: zeros) to dst + 16 * lane.  Inline asm, so
// the compiler's waitcnt pass does not see the DMA: through the builtin it could not tell the stage being
// written from the stage being read and put an s_waitcnt vmcnt(0) before the fragment reads of every K-step
// (the loop's own counted waits order the DMA; M0 is set here and needs one wait state before the load)
__device__ __forceinline__ void dma16(i32x4 r, char* dst, int voff) {
  const unsigned lds = static_cast<unsigned>(reinterpret_cast<size_t>((lds_void*)dst));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
               : "memory", "m0");
}

// fragment of 8 consecutive floats (pieces p0, p0 + 1) of LDS row r
template <class C>
__device__ __forceinline__ Split3 frag(const char* stage, int r, int p0) {
  const float4 u0 = *reinterpret_cast<const float4*>(stage + r * C::RB + 16 * C::slot_of(r, p0));
  const float4 u1 = *reinterpret_cast<const float4*>(stage + r * C::RB + 16 * C::slot_of(r, p0 + 1));
  if constexpr ((PIPE_ABL & 1) != 0) {
    Split3 x;
    x.p[0] = u32v4{__float_as_uint(u0.x), __float_as_uint(u0.y), __float_as_uint(u0.z), __float_as_uint(u0.w)};
    x.p[1] = u32v4{__float_as_uint(u1.x), __float_as_uint(u1.y), __float_as_uint(u1.z), __float_as_uint(u1.w)};
    x.p[2] = x.p[0] ^ x.p[1];
    return x;
  }
  const float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  return split8(v);
}

// bf16 fragment: the 8 bf16 (one 16-B slot, piece p) of LDS row r (the bf16 form of the ring: a stage row holds
// 2 BK bf16, piece p = k 8 p .. 8 p + 7)
template <class C>
__device__ __forceinline__ u32v4 frag_bf16(const char* stage, int r, int p) {
  const uint4 u = *reinterpret_cast<const uint4*>(stage + r * C::RB + 16 * C::slot_of(r, p));
  return u32v4{u.x, u.y, u.z, u.w};
}

// The main loop.  ASrc / BSrc: (chunk index within the wave's share, K-step) -> byte offset of this lane's 16-B
// piece (the piece is column slot_of(row, lane & 3) of row 16 chunk + lane / 4), or kOOB.  smem: NS stage arrays
// (separate __shared__ objects) and the loop unrolled by NS, so every DMA target and every fragment read names a
// compile-time stage: with one array and a runtime stage index the compiler cannot tell the DMA just issued from
// the stage being read and drains the DMA queue (s_waitcnt vmcnt(0)) before every K-step's first ds_read.
// BF16: the ring carries bf16 operands (a stage row = 2 BK bf16 = BK / 8 chunks of 16): plain bf16 MFMAs on
// one fragment read per operand and chunk, no split (gemm_bf16.hip).
// DMA_MID: issue the next stage's LDS-DMA between the two halves of the K-step's MFMAs (pinned with
// sched_barrier) instead of right after the barrier, so the DMA issue overlaps the matrix pipe (A/B switch)
template <class C, class ASrc, class BSrc, bool BF16 = false, bool DMA_MID = false>
__device__ __forceinline__ void mainloop(char* const (&smem)[C::NS], i32x4 ar, i32x4 br, int KT, const ASrc& asrc,
                                         const BSrc& bsrc, f16v (&acc)[C::FM][C::FN]) {
  constexpr int NS = C::NS;
  // the wave id in a scalar register: the per-wave branches below are uniform (s_cbranch, and only the taken
  // side's s_waitcnt executes)
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;
  const bool b_wave = C::B_CH >= C::NW || wid < C::B_CH;
  auto issue = [&](char* st, int kt) {
#pragma unroll
    for (int c = 0; c < C::A_PW; ++c) dma16(ar, st + (wid + C::NW * c) * 1024, asrc(c, kt));
    if (b_wave) {
#pragma unroll
      for (int c = 0; c < C::B_PW; ++c) dma16(br, st + C::BM * C::RB + (wid + C::NW * c) * 1024, bsrc(c, kt));
    }
  };
  auto step = [&](const char* st, char* next, int kt) {
    // this wave's loads of step kt: NS - 2 later steps may stay in flight
    if (b_wave) wait_vm<(NS - 2) * (C::A_PW + C::B_PW)>();
    else wait_vm<(NS - 2) * C::A_PW>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (!DMA_MID) issue(next, kt + NS - 1);
    if constexpr (BF16) {
#pragma unroll
      for (int c = 0; c < C::BK / 8; ++c) {
        u32v4 fa[C::FM], fb[C::FN];
#pragma unroll
        for (int i = 0; i < C::FM; ++i) fa[i] = frag_bf16<C>(st, wm * C::TM + 32 * i + l32, 2 * c + h);
#pragma unroll
        for (int j = 0; j < C::FN; ++j) fb[j] = frag_bf16<C>(st + C::BM * C::RB, wn * C::TN + 32 * j + l32, 2 * c + h);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_bf16(fb[j], fa[i], acc[i][j]);
      }
      return;
    }
#pragma unroll
    for (int c = 0; c < C::BK / 16; ++c) {
    // chunk c of lane half h: columns 16 c + 8 h .. + 7 = the MFMA's k-slots 8 h .. 8 h + 7
    Split3 sa[C::FM], sb[C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) sa[i] = frag<C>(st, wm * C::TM + 32 * i + l32, 4 * c + 2 * h);
#pragma unroll
    for (int j = 0; j < C::FN; ++j) sb[j] = frag<C>(st + C::BM * C::RB, wn * C::TN + 32 * j + l32, 4 * c + 2 * h);
    // swapped operands: the accumulator is the transposed tile (lane = output row, registers = columns)
    if constexpr ((PIPE_ABL & 2) != 0) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) asm volatile("" ::"v"(sa[i].p[q]));
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) asm volatile("" ::"v"(sb[j].p[q]));
    } else if constexpr (DMA_MID) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
          if (c == 0 && i * C::FN + j == (C::FM * C::FN) / 2 - 1) {
            __builtin_amdgcn_sched_barrier(0);
            issue(next, kt + NS - 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    } else {
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma_x6(sb[j], sa[i], acc[i][j]);
    }
    }
  };
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(smem[s], s);
  for (int kt = 0; kt < KT; kt += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (kt + s >= KT) break;
      step(smem[s], smem[(s + NS - 1) % NS], kt + s);
    }
  }
  wait_vm<0>();
}

// Epilogue of a wave's transposed accumulator tiles: lane l32 of tile (i, j) is output row mw + 32 i + l32,
// registers 4 g .. 4 g + 3 are columns nw + 32 j + 8 g + 4 h + 0..3.  out / res rows have N floats.
//   v = acc + bias[n] (+ res[m, n] | masked by res[m, n] > 0 for ACT_DRELU), then ReLU for ACT_RELU
// Extra (input-gradient) terms: + res2[m, n] for rows m < res2_rows (a gradient handed over for the first rows
// only, e.g. the location head's use of an encoder skip map), then the ReLU mask of the layer input:
// v = mask[m, n] > 0 ? v : 0.
struct Epi2 {
  const float* res2 = nullptr;
  long res2_rows = 0;
  const float* mask = nullptr;
};

template <int FM, int FN>
__device__ __forceinline__ void store_tile(const f16v (&acc)[FM][FN], float* __restrict__ out,
                                           const float* __restrict__ bias, const float* __restrict__ res, long M,
                                           int N, long mw, int nw, int act, const Epi2 e2 = Epi2()) {
  const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const bool vec = (N & 3) == 0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long m = mw + 32 * i + l32;
    if (m >= M) continue;
    float* orow = out + m * N;
    const float* rrow = res ? res + m * N : nullptr;
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
            const float4 rv = *reinterpret_cast<const float4*>(rrow + n);
            const float r[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = act == ACT_DRELU ? (r[q] > 0.f ? v[q] : 0.f) : v[q] + r[q];
          }
          if (e2.res2 != nullptr && m < e2.res2_rows) {
            const float4 r2 = *reinterpret_cast<const float4*>(e2.res2 + m * N + n);
            v[0] += r2.x; v[1] += r2.y; v[2] += r2.z; v[3] += r2.w;
          }
          if (e2.mask != nullptr) {
            const float4 mk = *reinterpret_cast<const float4*>(e2.mask + m * N + n);
            v[0] = mk.x > 0.f ? v[0] : 0.f; v[1] = mk.y > 0.f ? v[1] : 0.f;
            v[2] = mk.z > 0.f ? v[2] : 0.f; v[3] = mk.w > 0.f ? v[3] : 0.f;
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
            if (e2.res2 != nullptr && m < e2.res2_rows) x += e2.res2[m * N + n + q];
            if (e2.mask != nullptr && !(e2.mask[m * N + n + q] > 0.f)) x = 0.f;
            if (act == ACT_RELU) x = fmaxf(x, 0.f);
            orow[n + q] = x;
          }
        }
      }
    }
  }
}

// Epilogue through LDS (after the main loop; `lds` >= 32 x BN floats, e.g. one ring stage): the tile is written
// 32 rows at a time into LDS (float4 granules XOR-swizzled by row: the 32 lanes of a fragment column hit 16
// distinct 4-bank groups) and read back row-major, so each thread finishes 8 consecutive columns of one row
// and 16 / 32 lanes store one contiguous row segment (the register layout stores one 8- / 16-B piece per row
// and lane: every store instruction touched 64 rows).  Bias / residual / ReLU / ReLU-mask as store_tile.
template <class C, typename TO>
__device__ __forceinline__ void store_tile_staged(const f16v (&acc)[C::FM][C::FN], char* lds, TO* __restrict__ out,
                                                  const float* __restrict__ bias, const TO* __restrict__ res, long M,
                                                  int N, long m0, int n0, int act) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l32 = lane & 31, h = lane >> 5;
  constexpr int G = C::BN / 4;            // float4 granules per staged row
  constexpr int CPR = C::BN / 8;          // 8-column pieces per row
  float* t = reinterpret_cast<float*>(lds);
  const bool vec = (N & 7) == 0;
#pragma unroll 1
  for (int pass = 0; pass < C::WM * C::FM; ++pass) {
    const int pw = pass / C::FM, pi = pass % C::FM;     // tile rows pw TM + 32 pi .. + 31
    __syncthreads();                                     // the ring / the previous pass is no longer read
    if (wm == pw) {
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        if (i != pi) continue;
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int gr = (wn * C::TN + 32 * j + 8 * g + 4 * h) / 4;
            *reinterpret_cast<float4*>(t + (l32 * G + (gr ^ (l32 % G))) * 4) =
                make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          }
      }
    }
    __syncthreads();
    for (int c = tid; c < 32 * CPR; c += C::NT) {
      const int r = c / CPR, cc = c % CPR;
      const long m = m0 + pw * C::TM + 32 * pi + r;
      const int n = n0 + 8 * cc;
      if (m >= M || n >= N) continue;
      const float4 u0 = *reinterpret_cast<const float4*>(t + (r * G + ((2 * cc) ^ (r % G))) * 4);
      const float4 u1 = *reinterpret_cast<const float4*>(t + (r * G + ((2 * cc + 1) ^ (r % G))) * 4);
      float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      TO* orow = out + m * N;
      const TO* rrow = res ? res + m * N : nullptr;
      if (vec) {
        if (bias) {
          const float4 b0 = *reinterpret_cast<const float4*>(bias + n), b1 = *reinterpret_cast<const float4*>(bias + n + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (rrow) {
          float r8[8];
          if constexpr (sizeof(TO) == 2) {
            const uint4 rv = *reinterpret_cast<const uint4*>(rrow + n);
            const unsigned rw[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              r8[2 * q] = __uint_as_float(rw[q] << 16);
              r8[2 * q + 1] = __uint_as_float(rw[q] & 0xffff0000u);
            }
          } else {
            const float4 r0 = *reinterpret_cast<const float4*>(rrow + n), r1 = *reinterpret_cast<const float4*>(rrow + n + 4);
            r8[0] = r0.x; r8[1] = r0.y; r8[2] = r0.z; r8[3] = r0.w; r8[4] = r1.x; r8[5] = r1.y; r8[6] = r1.z; r8[7] = r1.w;
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = act == ACT_DRELU ? (r8[q] > 0.f ? v[q] : 0.f) : v[q] + r8[q];
        }
        if (act == ACT_RELU)
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
        if constexpr (sizeof(TO) == 2) {
          *reinterpret_cast<uint4*>(orow + n) =
              make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7]));
        } else {
          *reinterpret_cast<float4*>(orow + n) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(orow + n + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (n + q >= N) continue;
          float x = v[q] + (bias ? bias[n + q] : 0.f);
          if (rrow) {
            const float r = Cvt<TO>::load(rrow, n + q);
            x = act == ACT_DRELU ? (r > 0.f ? x : 0.f) : x + r;
          }
          if (act == ACT_RELU) x = fmaxf(x, 0.f);
          Cvt<TO>::store(orow, n + q, x);
        }
      }
    }
  }
}

// XCD-aware bijective remap of the workgroup id (8 XCDs, round-robin dispatch): consecutive logical ids share an
// XCD's L2
__device__ __forceinline__ int xcd_remap() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
}

}  // namespace pipe
}  // namespace as
