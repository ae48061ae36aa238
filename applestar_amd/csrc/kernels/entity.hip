// Entity-encoder input embedding without the 997-wide one-hot tensor.
//
// The reference concatenates 29 one-hot / 2 x 11-bit binary / 7 scalar encodings of each unit into a
// [B, N, 997] fp32 tensor and multiplies by W[256, 997] (entity_encoder.py:61-78, K1 in SURVEY).
// one-hot(v) @ W^T is a row gather of W^T, so the forward here is an embedding-bag: one wave per
// (packed, real) entity, each lane accumulating 4 of the 256 output channels from the selected
// W^T rows (8-16 B per lane, L2-resident 0.5 MB table), + bias, ReLU.  For the weight gradient the
// sparse input is materialised once in bf16 by entity_onehot() and fed to one GEMM.
#include "../common.h"
#include "../kernels.h"
#include <hip/hip_fp16.h>

namespace as {
namespace {

__device__ __forceinline__ float load_field(const void* p, int dt, long i) {
  switch (dt) {
    case SRC_U8: return static_cast<float>(static_cast<const uint8_t*>(p)[i]);
    case SRC_I8: return static_cast<float>(static_cast<const int8_t*>(p)[i]);
    case SRC_I16: return static_cast<float>(static_cast<const int16_t*>(p)[i]);
    case SRC_I32: return static_cast<float>(static_cast<const int32_t*>(p)[i]);
    case SRC_I64: return static_cast<float>(static_cast<const int64_t*>(p)[i]);
    case SRC_F16: return __half2float(static_cast<const __half*>(p)[i]);
    case SRC_F32: return static_cast<const float*>(p)[i];
    default: return 0.f;
  }
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

template <typename TW> struct Row4;
template <> struct Row4<float> {
  __device__ static void add(const float* w, float s, float* acc) {
    const float4 t = *reinterpret_cast<const float4*>(w);
    acc[0] = fmaf(s, t.x, acc[0]); acc[1] = fmaf(s, t.y, acc[1]);
    acc[2] = fmaf(s, t.z, acc[2]); acc[3] = fmaf(s, t.w, acc[3]);
  }
};
template <> struct Row4<bf16_t> {
  __device__ static void add(const bf16_t* w, float s, float* acc) {
    const uint2 t = *reinterpret_cast<const uint2*>(w);
    acc[0] = fmaf(s, __uint_as_float(t.x << 16), acc[0]); acc[1] = fmaf(s, __uint_as_float(t.x & 0xffff0000u), acc[1]);
    acc[2] = fmaf(s, __uint_as_float(t.y << 16), acc[2]); acc[3] = fmaf(s, __uint_as_float(t.y & 0xffff0000u), acc[3]);
  }
};

// wT [K_in][256]; out [T][256]
template <typename TW, typename TO>
__global__ __launch_bounds__(256) void entity_embed_fwd_kernel(EntityFields f, const int64_t* __restrict__ index,
                                                               const TW* __restrict__ wT, const float* __restrict__ bias,
                                                               TO* __restrict__ out, long T) {
  constexpr int C = 256;
  const int lane = threadIdx.x & 63;
  const long wave = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const long nwave = (static_cast<long>(gridDim.x) * blockDim.x) >> 6;
  const float4 bv = *reinterpret_cast<const float4*>(bias + lane * 4);
  for (long t = wave; t < T; t += nwave) {
    const long src = index[t];
    float acc[4] = {bv.x, bv.y, bv.z, bv.w};
    for (int k = 0; k < f.n; ++k) {
      const float v = load_field(f.ptr[k], f.dtype[k], src);
      const int off = f.offset[k], width = f.width[k];
      if (f.kind[k] == FIELD_ONE_HOT) {
        const int col = off + clampi(static_cast<int>(v), 0, width - 1);
        Row4<TW>::add(wT + static_cast<long>(col) * C + lane * 4, 1.f, acc);
      } else if (f.kind[k] == FIELD_BINARY) {
        const int iv = clampi(static_cast<int>(v), 0, (1 << width) - 1);
        for (int bit = 0; bit < width; ++bit)
          if ((iv >> (width - 1 - bit)) & 1) Row4<TW>::add(wT + static_cast<long>(off + bit) * C + lane * 4, 1.f, acc);
      } else {
        Row4<TW>::add(wT + static_cast<long>(off) * C + lane * 4, v, acc);
      }
    }
    float o[4] = {fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f), fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f)};
#pragma unroll
    for (int i = 0; i < 4; ++i) Cvt<TO>::store(out, t * C + lane * 4 + i, o[i]);
  }
}

// X [T][K_in] (pre-zeroed): one thread per (token, field)
template <typename TX>
__global__ __launch_bounds__(256) void entity_onehot_kernel(EntityFields f, const int64_t* __restrict__ index,
                                                            TX* __restrict__ X, long T, int K_in) {
  const long gid = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gid >= T * f.n) return;
  const long t = gid / f.n;
  const int k = static_cast<int>(gid % f.n);
  const float v = load_field(f.ptr[k], f.dtype[k], index[t]);
  TX* row = X + t * K_in;
  const int off = f.offset[k], width = f.width[k];
  if (f.kind[k] == FIELD_ONE_HOT) {
    Cvt<TX>::store(row, off + clampi(static_cast<int>(v), 0, width - 1), 1.f);
  } else if (f.kind[k] == FIELD_BINARY) {
    const int iv = clampi(static_cast<int>(v), 0, (1 << width) - 1);
    for (int bit = 0; bit < width; ++bit) Cvt<TX>::store(row, off + bit, static_cast<float>((iv >> (width - 1 - bit)) & 1));
  } else {
    Cvt<TX>::store(row, off, v);
  }
}

}  // namespace

void entity_embed_fwd(const EntityFields& f, const int64_t* index, const void* wT, int w_dt, const float* bias,
                      void* out, int out_dt, long T, hipStream_t s) {
  long blocks = (T + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
#define EE(TW, TO)                                                                                          \
  hipLaunchKernelGGL((entity_embed_fwd_kernel<TW, TO>), grid, block, 0, s, f, index, static_cast<const TW*>(wT), \
                     bias, static_cast<TO*>(out), T)
  if (w_dt == DT_BF16 && out_dt == DT_BF16) EE(bf16_t, bf16_t);
  else if (w_dt == DT_BF16) EE(bf16_t, float);
  else if (out_dt == DT_BF16) EE(float, bf16_t);
  else EE(float, float);
#undef EE
}

void entity_onehot(const EntityFields& f, const int64_t* index, void* X, int x_dt, long T, int K_in, hipStream_t s) {
  const long n = T * f.n;
  dim3 grid(static_cast<unsigned>((n + 255) / 256)), block(256);
  if (n == 0) return;
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(entity_onehot_kernel<bf16_t>, grid, block, 0, s, f, index, static_cast<bf16_t*>(X), T, K_in);
  else
    hipLaunchKernelGGL(entity_onehot_kernel<float>, grid, block, 0, s, f, index, static_cast<float*>(X), T, K_in);
}

}  // namespace as
