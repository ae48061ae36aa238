// Fused gradient clip + Adam for the learners, as two or three launches over every optimizer tensor,
// whatever their number:
//
//   RL (distar/agent/default/rl_learner.py:114-132): pytorch_norm clip at 1.0, Adam(betas=(0, 0.99), eps=1e-5);
//   SL (distar/agent/default/sl_learner.py:46-77, ctools/torch_utils/grad_clip.py:73-106): momentum_norm - each
//      tensor's gradient norm against an EMA of its past clipped norms - then Adam with L2 weight decay.
//
//   1. mt_sumsq: one workgroup per 32K-element chunk of the (tensor, offset) chunk table writes the chunk's
//      sum of squared gradients into part[chunk]  (fixed order: deterministic, identical on every rank);
//   2. (momentum_norm only) mt_momentum_clip: one workgroup; per tensor t the norm g_t from its chunks'
//      partials, scale_t = g_t < thr * mom_t ? 1 : thr * mom_t / (g_t + 1e-6) (1 until the EMA is initialised),
//      mom_t = 0.99 mom_t + 0.01 g_t scale_t (mom_t = g_t on the initialising step), and the global norm of the
//      clipped gradients.  "Initialised" is a device flag set by the first KEPT step: a gated first step leaves
//      the EMA uninitialised (a host-side flag would mark it live at 0 and every later scale would be 0);
//   3. mt_adam: coef = min(1, max_norm / (||g|| + 1e-6)) (every workgroup sums part[] in the same fixed
//      order, a few KB from L2) or scale_t, then per element:
//          g' = coef g (+ wd p),  m = b1 m + (1 - b1) g',  v = b2 v + (1 - b2) g'^2,
//          p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)            (torch.optim.Adam's formula)
//      and workgroup 0 stores the norm the learner logs.
// A step whose device gate is 0 (a timed-out LSTM exchange on any rank: the gate is all-reduced with the
// gradients) leaves p, m, v and the momentum EMA untouched: the update is skipped, not multiplied by 0
// (NaN * 0 is NaN, and v would still decay).
// The per-tensor pointer table is built once on the host (parameters, gradients and moments never move), so
// a step passes two device pointers.  The step-dependent scalars (lr / bc1, 1 / sqrt(bc2), decoupled decay)
// come either as kernel arguments (eager step) or from a 3-float device buffer that the host refreshes before
// each replay (a HIP graph captures the pointer, not the values).
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
  long chunk0;       // index of the tensor's first chunk in the chunk table
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

__device__ __forceinline__ bool gated_off(const float* gate) { return gate != nullptr && !(gate[0] > 0.f); }

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

__global__ __launch_bounds__(kOptT) void mt_momentum_clip_kernel(const TensorRec* __restrict__ tt, int ntensors,
                                                                 const float* __restrict__ part, float thr,
                                                                 float* __restrict__ mom, float* __restrict__ scale,
                                                                 float* __restrict__ init_flag, const float* __restrict__ gate,
                                                                 float* __restrict__ norm_out) {
  __shared__ float red[kOptT / 64];
  const bool keep = !gated_off(gate);
  const bool init = !(init_flag[0] > 0.f);    // read by every thread before thread 0 may set it (block_sum syncs)
  float acc = 0.f;
  for (int t = threadIdx.x; t < ntensors; t += kOptT) {
    const TensorRec r = tt[t];
    const long nc = (r.n + kChunk - 1) / kChunk;
    float s = 0.f;
    for (long c = 0; c < nc; ++c) s += part[r.chunk0 + c];
    const float g = sqrtf(s);
    float sc = 1.f;
    if (!init) {
      const float lim = thr * mom[t];
      sc = g < lim ? 1.f : lim / (g + 1e-6f);
    }
    const float nw = g * sc;
    if (keep) mom[t] = init ? nw : mom[t] * 0.99f + nw * 0.01f;
    scale[t] = sc;
    acc += nw * nw;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) {
    norm_out[0] = sqrtf(acc);
    if (keep) init_flag[0] = 1.f;
  }
}

__global__ __launch_bounds__(kOptT) void mt_adam_kernel(const TensorRec* __restrict__ tt, const long* __restrict__ chunks,
                                                        const float* __restrict__ part, int nchunks,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ gate, float* __restrict__ norm_out,
                                                        float max_norm, const float* __restrict__ hp, float lr_bc1,
                                                        float b1, float b2, float inv_sqrt_bc2, float eps, float wd,
                                                        int decoupled) {
  __shared__ float red[kOptT / 64];
  __shared__ float coef_s;
  const long t = chunks[2 * blockIdx.x], off = chunks[2 * blockIdx.x + 1];
  if (scale == nullptr) {
    float s = 0.f;
    for (int i = threadIdx.x; i < nchunks; i += kOptT) s += part[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) {
      const float norm = sqrtf(s);
      coef_s = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
      if (blockIdx.x == 0 && norm_out != nullptr) norm_out[0] = norm;
    }
    __syncthreads();
  } else if (threadIdx.x == 0) {
    coef_s = scale[t];
  }
  __syncthreads();
  if (gated_off(gate)) return;   // uniform across the grid
  const float coef = coef_s;
  if (hp != nullptr) {
    lr_bc1 = hp[0];
    inv_sqrt_bc2 = hp[1];
    wd = hp[2];
  }
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

void fused_clip_adam(const void* table, const long* chunks, int nchunks, int ntensors, float* part,
                     const float* gate, float* norm_out, float max_norm, float* mom, float* scale, float* mom_init,
                     const float* hp, float lr_bc1, float b1, float b2, float inv_sqrt_bc2, float eps, float wd,
                     int decoupled, hipStream_t s) {
  if (nchunks <= 0) return;
  const TensorRec* tt = static_cast<const TensorRec*>(table);
  hipLaunchKernelGGL(mt_sumsq_kernel, dim3(nchunks), dim3(kOptT), 0, s, tt, chunks, part);
  if (mom != nullptr) {
    hipLaunchKernelGGL(mt_momentum_clip_kernel, dim3(1), dim3(kOptT), 0, s, tt, ntensors, part, max_norm, mom, scale,
                       mom_init, gate, norm_out);
  }
  hipLaunchKernelGGL(mt_adam_kernel, dim3(nchunks), dim3(kOptT), 0, s, tt, chunks, part, nchunks,
                     mom != nullptr ? static_cast<const float*>(scale) : nullptr, gate,
                     mom != nullptr ? nullptr : norm_out, max_norm, hp, lr_bc1, b1, b2, inv_sqrt_bc2, eps, wd,
                     decoupled);
}

}  // namespace as
