// Shared device helpers for the applestar_amd gfx950 (CDNA4) kernels.
// Wavefront = 64 lanes; all cross-lane reductions below are 64-wide.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace as {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // raw bfloat16 bits
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(4))) short bf16x4;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// round-to-nearest-even float -> bf16 (NaN preserved): the fptrunc lowers to gfx950's v_cvt_pk_bf16_f32
// (the former integer rounding sequence carried a NaN branch - an exec-mask branch per conversion)
__device__ __forceinline__ bf16_t f2bf(float f) {
  const __bf16 b = static_cast<__bf16>(f);
  bf16_t u;
  __builtin_memcpy(&u, &b, 2);
  return u;
}

// two floats -> packed bf16 pair (lo in bits 0..15): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t f2bf2(float lo, float hi) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 b = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  uint32_t u;
  __builtin_memcpy(&u, &b, 4);
  return u;
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float load(const float* p, long i) { return p[i]; }
  __device__ __forceinline__ static void store(float* p, long i, float v) { p[i] = v; }
};
template <> struct Cvt<bf16_t> {
  __device__ __forceinline__ static float load(const bf16_t* p, long i) { return bf2f(p[i]); }
  __device__ __forceinline__ static void store(bf16_t* p, long i, float v) { p[i] = f2bf(v); }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ long wave_sum_long(long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3, ACT_DRELU = 4 };  // DRELU: conv epilogue only

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(x, 0.f);
    case ACT_SIGMOID: return sigmoidf_(x);
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

// d act / d pre, expressed through the activation *output* y
__device__ __forceinline__ float act_grad_from_out(float y, int act) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    default: return 1.f;
  }
}

}  // namespace as
