// fp32-accurate products on the bf16 MFMA: an fp32 value is split exactly into three bf16 parts and a 32x32x16
// block product is six bf16 MFMAs into one fp32 accumulator.
//
//   a = a0 + a1 + a2      a0 = a truncated to bf16 (top 8 significand bits), r1 = a - a0 (exact in fp32),
//                         a1 = r1 truncated to bf16, a2 = r1 - a1 (at most 8 significant bits left: exact bf16)
//   a b ~ a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0)          dropped: a1 b2 + a2 b1 + a2 b2  (~2^-25 |a b|)
//
// Each kept partial product is exact in the MFMA (8 x 8 significand bits) and accumulates in fp32, so the result
// carries fp32 rounding (the dropped terms sit below half an fp32 ulp of the product); tests compare it with the
// exact-f32 MFMA against float64.  Rate: the exact-f32 MFMA (v_mfma_f32_32x32x2_f32) runs 64 FLOP/clk/SIMD, the
// bf16 MFMA 1024, so six bf16 MFMAs per product deliver 2.67x the f32 rate (the split is VALU work beside them).
// This is the BF16x6 scheme of Henry, Tang & Heinecke, "Leveraging the bfloat16 Artificial Intelligence Datatype
// for Higher-Precision Computations" (ARITH 2019).
#pragma once
#include "common.h"

namespace as {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8;
typedef __attribute__((ext_vector_type(4))) unsigned u32v4;

struct Split3 {
  u32v4 p[3];   // parts 0 (high) .. 2 (low); dword q holds the bf16 pair of floats 2q, 2q + 1
};

// upper halves of two fp32 words -> one packed bf16 pair (x in bits 0..15): one v_perm_b32
__device__ __forceinline__ unsigned hi_pair(unsigned x, unsigned y) { return __builtin_amdgcn_perm(y, x, 0x07060302u); }

__device__ __forceinline__ float trunc_rest(float v) { return v - __uint_as_float(__float_as_uint(v) & 0xffff0000u); }

// split two floats into the three packed bf16 pairs
__device__ __forceinline__ void split_pair(float x, float y, unsigned& s0, unsigned& s1, unsigned& s2) {
  s0 = hi_pair(__float_as_uint(x), __float_as_uint(y));
  const float rx = trunc_rest(x), ry = trunc_rest(y);
  s1 = hi_pair(__float_as_uint(rx), __float_as_uint(ry));
  s2 = hi_pair(__float_as_uint(trunc_rest(rx)), __float_as_uint(trunc_rest(ry)));
}

// 8 floats (one MFMA lane fragment) -> three bf16x8 fragments
__device__ __forceinline__ Split3 split8(const float (&v)[8]) {
  Split3 s;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned s0, s1, s2;
    split_pair(v[2 * q], v[2 * q + 1], s0, s1, s2);
    s.p[0][q] = s0;
    s.p[1][q] = s1;
    s.p[2][q] = s2;
  }
  return s;
}

// 4 floats (one 16-B piece) -> three 8-B packed bf16 pieces
__device__ __forceinline__ void split4(const uint4 v, uint2& s0, uint2& s1, uint2& s2) {
  split_pair(__uint_as_float(v.x), __uint_as_float(v.y), s0.x, s1.x, s2.x);
  split_pair(__uint_as_float(v.z), __uint_as_float(v.w), s0.y, s1.y, s2.y);
}

__device__ __forceinline__ bf16v8 as_bf(u32v4 v) { return __builtin_bit_cast(bf16v8, v); }

__device__ __forceinline__ f32x16 mfma_bf16(u32v4 a, u32v4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(a), as_bf(b), c, 0, 0, 0);
}

// acc += A B over one 16-deep k block, fp32-accurate: smallest terms first
__device__ __forceinline__ f32x16 mfma_x6(const Split3& a, const Split3& b, f32x16 c) {
  c = mfma_bf16(a.p[1], b.p[1], c);
  c = mfma_bf16(a.p[0], b.p[2], c);
  c = mfma_bf16(a.p[2], b.p[0], c);
  c = mfma_bf16(a.p[0], b.p[1], c);
  c = mfma_bf16(a.p[1], b.p[0], c);
  return mfma_bf16(a.p[0], b.p[0], c);
}

}  // namespace as
