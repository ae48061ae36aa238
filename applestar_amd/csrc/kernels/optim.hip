// Fused gradient clip + Adam for the RL learner (distar/agent/default/rl_learner.py:114-132:
// pytorch_norm clip at 1.0, then Adam(betas=(0, 0.99), eps=1e-5)), as two launches over every optimizer
// tensor, whatever their number:
//
//   1. mt_sumsq: one workgroup per 32K-element chunk of the (tensor, offset) chunk table writes the chunk's
//      sum of squared gradients into part[chunk]  (fixed order: deterministic, identical on every rank);
//   2. mt_adam:  every workgroup sums part[] in the same fixed order (a few KB from L2), forms
//      coef = min(1, max_norm / (||g|| + 1e-6)) * gate, and updates its chunk in place:
//          g' = coef g (+ wd p),  m = b1 m + (1 - b1) g',  v = b2 v + (1 - b2) g'^2,
//          p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)            (torch.optim.Adam's formula)
//      and workgroup 0 stores ||g|| (the pre-clip norm the learner logs).
// The per-tensor pointer table is built once on the host (parameters, gradients and moments never move), so
// a step passes two device pointers.  Replaces ~10 foreach / fused-Adam launches and the norm's host-visible
// intermediates.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

constexpr int kChunk = 1 << 15;
constexpr int kOptT = 256;

struct TensorRec {   // mirrors the host table layout (6 x int64)
  float* p;
  const float* g;
  float* m;
  float* v;
  long n;
  long pad;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x < 64) {
    t = threadIdx.x < kOptT / 64 ? red[threadIdx.x] : 0.f;
    t = wave_sum(t);
  }
  return t;   // valid in threads 0..63
}

__global__ __launch_bounds__(kOptT) void mt_sumsq_kernel(const TensorRec* __restrict__ tt,
                                                         const long* __restrict__ chunks, float* __restrict__ part) {
  __shared__ float red[kOptT / 64];
  const long t = chunks[2 * blockIdx.x], off = chunks[2 * blockIdx.x + 1];
  const TensorRec r = tt[t];
  const long end = off + kChunk < r.n ? off + kChunk : r.n;
  float s = 0.f;
  if ((reinterpret_cast<uintptr_t>(r.g) & 15) == 0 && (off & 3) == 0) {
    const long n4 = (end - off) >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(r.g + off);
    for (long i = threadIdx.x; i < n4; i += kOptT) {
      const float4 v = g4[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (long i = off + 4 * n4 + threadIdx.x; i < end; i += kOptT) s += r.g[i] * r.g[i];
  } else {
    for (long i = off + threadIdx.x; i < end; i += kOptT) s += r.g[i] * r.g[i];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(kOptT) void mt_adam_kernel(const TensorRec* __restrict__ tt, const long* __restrict__ chunks,
                                                        const float* __restrict__ part, int nchunks,
                                                        const float* __restrict__ gate, float* __restrict__ norm_out,
                                                        float max_norm, float lr_bc1, float b1, float b2,
                                                        float inv_sqrt_bc2, float eps, float wd, int decoupled) {
  __shared__ float red[kOptT / 64];
  __shared__ float coef_s;
  float s = 0.f;
  for (int i = threadIdx.x; i < nchunks; i += kOptT) s += part[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    float c = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    if (gate != nullptr) c *= gate[0];
    coef_s = c;
    if (blockIdx.x == 0 && norm_out != nullptr) norm_out[0] = norm;
  }
  __syncthreads();
  const float coef = coef_s;
  const long t = chunks[2 * blockIdx.x], off = chunks[2 * blockIdx.x + 1];
  const TensorRec r = tt[t];
  const long end = off + kChunk < r.n ? off + kChunk : r.n;
  for (long i = off + threadIdx.x; i < end; i += kOptT) {
    float g = r.g[i] * coef;
    float p = r.p[i];
    if (decoupled) p *= 1.f - wd;          // AdamW: lr * weight_decay folded by the host into wd
    else g += wd * p;
    const float m = b1 * r.m[i] + (1.f - b1) * g;
    const float v = b2 * r.v[i] + (1.f - b2) * g * g;
    r.m[i] = m;
    r.v[i] = v;
    r.p[i] = p - lr_bc1 * m / (sqrtf(v) * inv_sqrt_bc2 + eps);
  }
}

}  // namespace

int fused_adam_chunk() { return kChunk; }

void fused_clip_adam(const void* table, const long* chunks, int nchunks, float* part, const float* gate, float* norm_out,
                     float max_norm, float lr_bc1, float b1, float b2, float inv_sqrt_bc2, float eps, float wd,
                     int decoupled, hipStream_t s) {
  if (nchunks <= 0) return;
  const TensorRec* tt = static_cast<const TensorRec*>(table);
  hipLaunchKernelGGL(mt_sumsq_kernel, dim3(nchunks), dim3(kOptT), 0, s, tt, chunks, part);
  hipLaunchKernelGGL(mt_adam_kernel, dim3(nchunks), dim3(kOptT), 0, s, tt, chunks, part, nchunks, gate, norm_out,
                     max_norm, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd, decoupled);
}

}  // namespace as
