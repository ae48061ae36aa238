// Entity-encoder input embedding without the 997-wide one-hot tensor.
//
// The reference concatenates 29 one-hot / 2 x 11-bit binary / 7 scalar encodings of each unit into a
// [B, N, 997] fp32 tensor and multiplies by W[256, 997] (entity_encoder.py:61-78, K1 in SURVEY).
// one-hot(v) @ W^T is a row gather of W^T, so the forward here is an embedding-bag: one wave per
// (packed, real) entity, each lane accumulating 4 of the 256 output channels from the selected
// W^T rows (8-16 B per lane, L2-resident 0.5 MB table), + bias, ReLU.  The weight gradient is the
// same sparse structure transposed: entity_embed_wgrad() scatters dpre = dout * [out > 0] into an LDS
// [997][32] fp32 tile per (32-channel group, token chunk) - ~58 nonzero columns per token instead of
// the 997-wide materialised one-hot and a [256 x T] x [T x 997] library GEMM (r2an: 0.46 ms).
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


// dW partials: workgroup (chunk, channel group g) accumulates, for tokens of its chunk, dpre[t][32 g + c]
// times each nonzero input column of token t into acc[col][c] (LDS float atomics; lanes 0-31 / 32-63
// take two tokens, lane c = channel), then writes its [32][K_in] block (and the 32 bias sums) into row
// `chunk` of part [nchunk][256 * K_in + 256] (reduced over chunks afterwards).  Tokens go in passes of
// 128: the pass's field values are first staged in LDS by all threads (independent loads, so their
// latency overlaps - read one field at a time per token they serialised: 8.6 ms, r2ap), and each
// wave fetches its 16 tokens' dpre before scattering.
constexpr int kEwKin = 1024;   // LDS rows (K_in <= 1024)
constexpr int kEwPass = 128;   // tokens per pass
template <typename TD>
__global__ __launch_bounds__(256) void entity_wgrad_kernel(EntityFields f, const int64_t* __restrict__ index,
                                                           const TD* __restrict__ dout, const TD* __restrict__ out,
                                                           float* __restrict__ part, long T, int K_in, int nchunk) {
  __shared__ float acc[kEwKin * 32 + 32];   // [K_in][32] (+ 32 bias sums); static: > 64 KB
  __shared__ float fv[kMaxFields][kEwPass];
  const int g = blockIdx.x & 7, chunk = blockIdx.x >> 3;
  const int tid = threadIdx.x, c = tid & 31, half = (tid >> 5) & 1, w = tid >> 6;
  for (int i = tid; i < K_in * 32 + 32; i += 256) acc[i] = 0.f;
  const long per = (T + nchunk - 1) / nchunk;
  const long t0 = chunk * per, t1 = t0 + per < T ? t0 + per : T;
  float db = 0.f;
  for (long base = t0; base < t1; base += kEwPass) {
    __syncthreads();   // previous pass consumed (and acc zeroed)
    {
      const int tl = tid & (kEwPass - 1), fh = tid >> 7;
      const long t = base + tl < t1 ? base + tl : t0;
      const long src = index[t];
      float vals[kMaxFields / 2];
#pragma unroll
      for (int i = 0; i < kMaxFields / 2; ++i) {
        const int k = 2 * i + fh;
        vals[i] = k < f.n ? load_field(f.ptr[k], f.dtype[k], src) : 0.f;
      }
#pragma unroll
      for (int i = 0; i < kMaxFields / 2; ++i)
        if (2 * i + fh < f.n) fv[2 * i + fh][tl] = vals[i];
    }
    // this lane's 16 tokens of the pass: dpre = dout * [out > 0]
    float dv[kEwPass / 8];
#pragma unroll
    for (int j = 0; j < kEwPass / 8; ++j) {
      const long t = base + 2 * w + half + 8 * j;
      const long o = (t < t1 ? t : t0) * 256 + 32 * g + c;
      const float ov = Cvt<TD>::load(out, o), dd = Cvt<TD>::load(dout, o);
      dv[j] = (t < t1 && ov > 0.f) ? dd : 0.f;
    }
    __syncthreads();
#pragma unroll 1
    for (int j = 0; j < kEwPass / 8; ++j) {
      const int tl = 2 * w + half + 8 * j;
      if (base + tl >= t1) break;
      const float d = dv[j];
      db += d;
      for (int k = 0; k < f.n; ++k) {
        const float v = fv[k][tl];
        const int off = f.offset[k], width = f.width[k];
        if (f.kind[k] == FIELD_ONE_HOT) {
          atomicAdd(&acc[(off + clampi(static_cast<int>(v), 0, width - 1)) * 32 + c], d);
        } else if (f.kind[k] == FIELD_BINARY) {
          const int iv = clampi(static_cast<int>(v), 0, (1 << width) - 1);
          for (int bit = 0; bit < width; ++bit)
            if ((iv >> (width - 1 - bit)) & 1) atomicAdd(&acc[(off + bit) * 32 + c], d);
        } else if (v != 0.f) {
          atomicAdd(&acc[off * 32 + c], d * v);
        }
      }
    }
  }
  atomicAdd(&acc[K_in * 32 + c], db);
  __syncthreads();
  float* row = part + static_cast<long>(chunk) * (256L * K_in + 256);
  for (int i = tid; i < 32 * K_in; i += 256) {
    const int cc = i / K_in, col = i - cc * K_in;   // consecutive threads -> consecutive columns
    row[static_cast<long>(32 * g + cc) * K_in + col] = acc[col * 32 + cc];
  }
  if (tid < 32) row[256L * K_in + 32 * g + tid] = acc[K_in * 32 + tid];
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

int entity_wgrad_chunks(long T) {
  long n = (T + 2047) / 2048;   // ~2k tokens per workgroup, <= 64 chunks (x 8 channel groups)
  return static_cast<int>(n < 1 ? 1 : (n > 64 ? 64 : n));
}

void entity_embed_wgrad(const EntityFields& f, const int64_t* index, const void* dout, const void* out, int dt,
                        float* part, long T, int K_in, int nchunk, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(nchunk) * 8);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(entity_wgrad_kernel<bf16_t>, grid, dim3(256), 0, s, f, index, static_cast<const bf16_t*>(dout),
                       static_cast<const bf16_t*>(out), part, T, K_in, nchunk);
  else
    hipLaunchKernelGGL(entity_wgrad_kernel<float>, grid, dim3(256), 0, s, f, index, static_cast<const float*>(dout),
                       static_cast<const float*>(out), part, T, K_in, nchunk);
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
