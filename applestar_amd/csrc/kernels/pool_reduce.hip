// NHWC 2x2 max-pool (forward + backward), sorted-segment row sums, small-table row-gather
// gradients and the partial-sum column reduction, for gfx950.
//
// maxpool2: the spatial and value encoders downsample with max_pool2d(x, 2, 2) three times each
//   (spatial_encoder.py:74-80, value_encoder.py:43-50).  torch's channels_last kernels cost ~3 ms
//   per learner step (the backward zero-fills dx, then scatters through int64 argmax indices).  Here
//   one thread owns 8 channels (16 B) of one output pixel: the forward reads the 2x2 window with four
//   16-B loads and writes y plus the window position per channel (one byte); the backward writes
//   every dx element exactly once (dy where the position matches, else 0): no memset, no atomics.
//   Selection matches torch: scan (0,0),(0,1),(1,0),(1,1), replace on (v > max) || isnan(v).
// segment_sum: out[s, c] = sum_{t in [cu[s], cu[s+1])} x[t, c] over packed entity rows (the entity
//   encoder's masked mean, entity_encoder.py:85-87): one workgroup per segment, no atomics.
// table_grad: dT[v, :] = sum_u [idx[u] == v] src[u, :] for tiny lookup tables (the value encoder's
//   unit-type / alliance tables, value_encoder.py:32-41): block-private LDS accumulators (LDS float
//   atomics), one global atomic per table entry per block - instead of ~2e5 contended bf16 CAS
//   atomics into 260 (or 2) rows.
// column_reduce: out[c] = sum_r part[r][c] for the per-block partials of the LayerNorm / upconv
//   weight gradients.  <= 1024 rows: one 1024-thread block per 64 columns (16 row groups x 4
//   independent accumulators).  More rows: 256-row slabs per block, fp32 atomics into a zeroed out.
#include <algorithm>

#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

struct V8 {
  float v[8];
};

template <typename T> __device__ __forceinline__ V8 load8(const T* p);
template <> __device__ __forceinline__ V8 load8<bf16_t>(const bf16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  V8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r.v[2 * j] = __uint_as_float(w[j] << 16);
    r.v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
  return r;
}
template <> __device__ __forceinline__ V8 load8<float>(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  V8 r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

template <typename T> __device__ __forceinline__ void store8(T* p, const V8& r);
template <> __device__ __forceinline__ void store8<bf16_t>(bf16_t* p, const V8& r) {
  uint4 u;
  u.x = f2bf2(r.v[0], r.v[1]);
  u.y = f2bf2(r.v[2], r.v[3]);
  u.z = f2bf2(r.v[4], r.v[5]);
  u.w = f2bf2(r.v[6], r.v[7]);
  *reinterpret_cast<uint4*>(p) = u;
}
template <> __device__ __forceinline__ void store8<float>(float* p, const V8& r) {
  *reinterpret_cast<float4*>(p) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return static_cast<int>(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

// x [B][H][W][C] -> y [B][H/2][W/2][C], pos (window position 0..3 per element); C % 8 == 0
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                           uint8_t* __restrict__ pos, int B, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1, C8 = C >> 3;
  const long total = static_cast<long>(B) * Ho * Wo * C8;
  const long rowstride = static_cast<long>(W) * C;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % C8);
    long r = i / C8;
    const int ox = static_cast<int>(r % Wo);
    r /= Wo;
    const int oy = static_cast<int>(r % Ho);
    const long b = r / Ho;
    const long p00 = ((b * H + 2 * oy) * W + 2 * ox) * C + 8 * c8;
    const V8 a = load8<T>(x + p00), q1 = load8<T>(x + p00 + C), q2 = load8<T>(x + p00 + rowstride),
             q3 = load8<T>(x + p00 + rowstride + C);
    V8 o;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float m = a.v[k];
      uint32_t p = 0;
      if (q1.v[k] > m || isnan(q1.v[k])) { m = q1.v[k]; p = 1; }
      if (q2.v[k] > m || isnan(q2.v[k])) { m = q2.v[k]; p = 2; }
      if (q3.v[k] > m || isnan(q3.v[k])) { m = q3.v[k]; p = 3; }
      o.v[k] = m;
      if (k < 4) lo |= p << (8 * k);
      else hi |= p << (8 * (k - 4));
    }
    store8<T>(y + i * 8, o);
    *reinterpret_cast<uint2*>(pos + i * 8) = make_uint2(lo, hi);
  }
}

// dy [B][Ho][Wo][C], pos -> dx [B][H][W][C] (every element written; an odd trailing row/col gets 0)
// mask (optional): the pool's input x when it is a ReLU output - dx is also multiplied by [x > 0] (the
// producer's ReLU backward folded in; its separate threshold pass is then skipped, ops/native.py _premasked)
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ pos,
                                                           T* __restrict__ dx, int B, int H, int W, int C,
                                                           const T* __restrict__ mask) {
  const int Ho = H >> 1, Wo = W >> 1, C8 = C >> 3;
  const long total = static_cast<long>(B) * H * W * C8;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c8 = static_cast<int>(i % C8);
    long r = i / C8;
    const int ix = static_cast<int>(r % W);
    r /= W;
    const int iy = static_cast<int>(r % H);
    const long b = r / H;
    const int oy = iy >> 1, ox = ix >> 1;
    V8 o;
    if (oy < Ho && ox < Wo) {
      const long oi = ((b * Ho + oy) * Wo + ox) * C + 8 * c8;
      const V8 g = load8<T>(dy + oi);
      const uint2 pp = *reinterpret_cast<const uint2*>(pos + oi);
      const uint32_t me = static_cast<uint32_t>((iy & 1) * 2 + (ix & 1));
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t p = ((k < 4 ? pp.x : pp.y) >> (8 * (k & 3))) & 0xffu;
        o.v[k] = p == me ? g.v[k] : 0.f;
      }
      if (mask) {
        const V8 xm = load8<T>(mask + i * 8);
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = xm.v[k] > 0.f ? o.v[k] : 0.f;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = 0.f;
    }
    store8<T>(dx + i * 8, o);
  }
}

// one workgroup (256 threads = 4 waves) per segment; each lane covers 4 channels per pass, C <= 1024
template <typename T>
__global__ __launch_bounds__(256) void segment_sum_kernel(const T* __restrict__ x, const int* __restrict__ cu,
                                                          float* __restrict__ out, int C) {
  __shared__ float red[4][1024];
  const int s = blockIdx.x;
  const int t0 = cu[s], t1 = cu[s + 1];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int c0 = 4 * l; c0 < C; c0 += 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = t0 + w; t < t1; t += 4) {
      const long base = static_cast<long>(t) * C + c0;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += Cvt<T>::load(x, base + k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) red[w][c0 + k] = acc[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256)
    out[static_cast<long>(s) * C + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// out [V][D] fp32 (zeroed) += rows of src [U][D] grouped by idx[u]; rows with idx outside [0, V) skipped.
// V * D floats of dynamic LDS (<= 64 KiB).
template <typename T>
__global__ __launch_bounds__(256) void table_grad_kernel(const T* __restrict__ src, const int64_t* __restrict__ idx,
                                                         float* __restrict__ out, long U, int V, int D) {
  extern __shared__ float acc[];
  const int VD = V * D;
  for (int i = threadIdx.x; i < VD; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  const long total = U * D;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const long u = i / D;
    const int d = static_cast<int>(i - u * D);
    const int64_t v = idx[u];
    if (v >= 0 && v < V) atomicAdd(&acc[v * D + d], Cvt<T>::load(src, i));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < VD; i += blockDim.x) {
    const float a = acc[i];
    if (a != 0.f) atomicAdd(out + i, a);
  }
}

// Embedding lookup + ReLU of the scalar encoder's small tables (the index column in its stored integer dtype,
// clamped to [0, V)): out[u][d] = max(table[clamp(idx[u])][d], 0) - one launch instead of the integer cast,
// clamp, gather and ReLU passes.  The backward sums the ReLU-masked rows into dtable with ONE workgroup for the
// tiniest batches (LDS accumulation, plain stores: no zero fill of the output) or the LDS-then-global-atomic form.
template <typename I>
__device__ __forceinline__ int clamp_idx(const I* idx, long u, int V) {
  long v = static_cast<long>(idx[u]);
  return static_cast<int>(v < 0 ? 0 : (v >= V ? V - 1 : v));
}

template <typename T, typename I>
__global__ __launch_bounds__(256) void embed_relu_fwd_kernel(const T* __restrict__ table, const I* __restrict__ idx,
                                                             T* __restrict__ out, long U, int V, int D) {
  const long total = U * D;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const long u = i / D;
    const int d = static_cast<int>(i - u * D);
    const float v = Cvt<T>::load(table, static_cast<long>(clamp_idx(idx, u, V)) * D + d);
    Cvt<T>::store(out, i, fmaxf(v, 0.f));
  }
}

template <typename T, typename I>
__global__ __launch_bounds__(256) void embed_relu_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                                             const I* __restrict__ idx, float* __restrict__ dtab,
                                                             long U, int V, int D, int direct) {
  extern __shared__ float acc[];
  const int VD = V * D;
  for (int i = threadIdx.x; i < VD; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  const long total = U * D;
  for (long i = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const long u = i / D;
    const int d = static_cast<int>(i - u * D);
    if (Cvt<T>::load(out, i) > 0.f) atomicAdd(&acc[clamp_idx(idx, u, V) * D + d], Cvt<T>::load(dout, i));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < VD; i += blockDim.x) {
    if (direct) dtab[i] = acc[i];
    else if (acc[i] != 0.f) atomicAdd(dtab + i, acc[i]);
  }
}

// Entity packing tables in one launch (one workgroup per observation b; len_b = min(num[b], N) clamped at 0):
//   valid[b][j] = j < len_b;  cu[b] = sum_{b' < b} len_b' (cu[B] = total);  for the packed rows k = cu[b] + j:
//   flat[k] = b N + j (packed -> padded row), seg[k] = b.  Rows past `total` (the host's count) are not written.
// Replaces sequence_mask + nonzero_static + clamp + cumsum + pad + repeat_interleave (~8 launches, 0.2 ms).
template <typename NT>
__global__ __launch_bounds__(256) void entity_pack_kernel(const NT* __restrict__ num, int B, int N, long total,
                                                          bool* __restrict__ valid, int64_t* __restrict__ flat,
                                                          int64_t* __restrict__ seg, int* __restrict__ cu) {
  const int b = blockIdx.x;
  __shared__ long base_s;
  auto len_of = [&](int i) {
    const long v = static_cast<long>(num[i]);
    return v < 0 ? 0L : (v > N ? static_cast<long>(N) : v);
  };
  if (threadIdx.x < 64) {
    long acc = 0;
    for (int i = threadIdx.x; i < b; i += 64) acc += len_of(i);
    acc = wave_sum_long(acc);
    if (threadIdx.x == 0) {
      base_s = acc;
      cu[b] = static_cast<int>(acc);
      if (b == B - 1) cu[B] = static_cast<int>(acc + len_of(b));
    }
  }
  __syncthreads();
  const long base = base_s, len = len_of(b);
  for (int j = threadIdx.x; j < N; j += 256) {
    valid[static_cast<long>(b) * N + j] = j < len;
    const long k = base + j;
    if (j < len && k < total) {
      flat[k] = static_cast<int64_t>(b) * N + j;
      seg[k] = b;
    }
  }
}

// OutT = bf16_t fuses the cast of the reduced weight gradient to the bf16 compute parameter dtype
// (one launch instead of reduce + cast, wgrad callers under master weights)
template <typename OutT>
__global__ __launch_bounds__(1024) void column_reduce_kernel(const float* __restrict__ part, OutT* __restrict__ out,
                                                             int nrows, int cols, long rstride) {
  __shared__ float red[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    int r = g;
    for (; r + 48 < nrows; r += 64) {
      s0 += part[static_cast<long>(r) * rstride + c];
      s1 += part[static_cast<long>(r + 16) * rstride + c];
      s2 += part[static_cast<long>(r + 32) * rstride + c];
      s3 += part[static_cast<long>(r + 48) * rstride + c];
    }
    for (; r < nrows; r += 16) s0 += part[static_cast<long>(r) * rstride + c];
  }
  red[g][threadIdx.x & 63] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][threadIdx.x];
    if constexpr (sizeof(OutT) == 2) out[c] = f2bf(s);
    else out[c] = s;
  }
}

// first pass of a long reduction (nrows > 1024): grid (ceil(cols/64), ceil(nrows/256)); workgroup (cb, rb) sums rows
// 256 rb .. 256 rb + 255 of its 64 columns in a fixed order and writes the sum over the chunk's FIRST row (rows only
// it reads), so the second pass (column_reduce_kernel with rstride = 256 cols) is deterministic too.  Replaced a zero
// fill + atomicAdd pass whose summation order varied run to run (tools/diag/poison_probe.py).
__global__ __launch_bounds__(256) void column_reduce_chunk_kernel(float* __restrict__ part, int nrows, int cols) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int r0 = blockIdx.y * 256, r1 = min(r0 + 256, nrows);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    int r = r0 + g;
    for (; r + 12 < r1; r += 16) {
      s0 += part[static_cast<long>(r) * cols + c];
      s1 += part[static_cast<long>(r + 4) * cols + c];
      s2 += part[static_cast<long>(r + 8) * cols + c];
      s3 += part[static_cast<long>(r + 12) * cols + c];
    }
    for (; r < r1; r += 4) s0 += part[static_cast<long>(r) * cols + c];
  }
  red[g][threadIdx.x & 63] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < cols)
    part[static_cast<long>(r0) * cols + c] = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                                             (red[2][threadIdx.x] + red[3][threadIdx.x]);
}


// LayerNorm affine gradients over rows: part[s][c] = sum_r dy[r][c] * xh[r][c], part[s][C + c] = sum_r dy[r][c]
// for the rows of slice s (kAffRows rows per slice); 64 columns per block, the 4 waves take every 4th row
constexpr int kAffRows = 512;
__global__ __launch_bounds__(256) void ln_affine_grads_kernel(const float* __restrict__ dy, const float* __restrict__ xh,
                                                              float* __restrict__ part, long R, int C) {
  __shared__ float sw[4][64], sb[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const long r0 = static_cast<long>(blockIdx.y) * kAffRows;
  const long r1 = r0 + kAffRows < R ? r0 + kAffRows : R;
  float aw = 0.f, ab = 0.f;
  if (c < C) {
#pragma unroll 4
    for (long r = r0 + w; r < r1; r += 4) {
      const float g = dy[r * C + c];
      aw += g * xh[r * C + c];
      ab += g;
    }
  }
  sw[w][lane] = aw;
  sb[w][lane] = ab;
  __syncthreads();
  if (w == 0 && c < C) {
    float* o = part + static_cast<long>(blockIdx.y) * 2 * C;
    o[c] = (sw[0][lane] + sw[1][lane]) + (sw[2][lane] + sw[3][lane]);
    o[C + c] = (sb[0][lane] + sb[1][lane]) + (sb[2][lane] + sb[3][lane]);
  }
}
}  // namespace

namespace {
// Backward of relu -> maxpool2 for even H, W (bf16): one thread per pooled pixel and 8 channels writes its
// 2x2 input pixels; the gradient passes at the argmax when the pooled value (= the ReLU output there) is
// positive.  Used by the fused spatial embed + pool stage, which keeps no full-resolution output.
__global__ __launch_bounds__(256) void maxpool2_bwd_relu_kernel(const bf16_t* __restrict__ dy,
                                                                const uint8_t* __restrict__ pos,
                                                                const bf16_t* __restrict__ y, bf16_t* __restrict__ dx,
                                                                int B, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1, C8 = C >> 3;
  const int total = B * Ho * Wo * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    int r = i / C8;
    const int ox = r % Wo;
    r /= Wo;
    const int oy = r % Ho;
    const int b = r / Ho;
    const long oi = static_cast<long>(i) * 8;
    const uint4 g = *reinterpret_cast<const uint4*>(dy + oi);
    const uint4 yv = *reinterpret_cast<const uint4*>(y + oi);
    const uint2 pp = *reinterpret_cast<const uint2*>(pos + oi);
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
    uint32_t outw[4][4];   // [window position][dword]
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) outw[t][j] = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t p = ((k < 4 ? pp.x : pp.y) >> (8 * (k & 3))) & 3u;
      const uint32_t raw = (k & 1) ? (gw[k >> 1] >> 16) : (gw[k >> 1] & 0xffffu);     // bf16 bits of dy
      const float yk = __uint_as_float((k & 1) ? (yw[k >> 1] & 0xffff0000u) : (yw[k >> 1] << 16));
      const uint32_t bits = yk > 0.f ? raw : 0u;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (p == static_cast<uint32_t>(t)) outw[t][k >> 1] |= bits << ((k & 1) ? 16 : 0);
    }
    const long row = static_cast<long>(W) * C;
    const long i00 = ((static_cast<long>(b) * H + 2 * oy) * W + 2 * ox) * C + 8 * c8;
    *reinterpret_cast<uint4*>(dx + i00) = make_uint4(outw[0][0], outw[0][1], outw[0][2], outw[0][3]);
    *reinterpret_cast<uint4*>(dx + i00 + C) = make_uint4(outw[1][0], outw[1][1], outw[1][2], outw[1][3]);
    *reinterpret_cast<uint4*>(dx + i00 + row) = make_uint4(outw[2][0], outw[2][1], outw[2][2], outw[2][3]);
    *reinterpret_cast<uint4*>(dx + i00 + row + C) = make_uint4(outw[3][0], outw[3][1], outw[3][2], outw[3][3]);
  }
}
// fp32 form (the fp32 step's fused spatial embed + pool): 8 channels of one pooled pixel per thread, the gradient
// written at the argmax when the pooled ReLU output there is positive, zeros elsewhere (two 16-B stores per window
// position)
__global__ __launch_bounds__(256) void maxpool2_bwd_relu_f32_kernel(const float* __restrict__ dy,
                                                                    const uint8_t* __restrict__ pos,
                                                                    const float* __restrict__ y, float* __restrict__ dx,
                                                                    int B, int H, int W, int C) {
  const int Ho = H >> 1, Wo = W >> 1, C8 = C >> 3;
  const int total = B * Ho * Wo * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8;
    int r = i / C8;
    const int ox = r % Wo;
    r /= Wo;
    const int oy = r % Ho;
    const int b = r / Ho;
    const long oi = static_cast<long>(i) * 8;
    const float4 g0 = *reinterpret_cast<const float4*>(dy + oi), g1 = *reinterpret_cast<const float4*>(dy + oi + 4);
    const float4 y0 = *reinterpret_cast<const float4*>(y + oi), y1 = *reinterpret_cast<const float4*>(y + oi + 4);
    const uint2 pp = *reinterpret_cast<const uint2*>(pos + oi);
    const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
    float o[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t p = ((k < 4 ? pp.x : pp.y) >> (8 * (k & 3))) & 3u;
      const float v = yv[k] > 0.f ? gv[k] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t][k] = p == static_cast<uint32_t>(t) ? v : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long px = (static_cast<long>(b) * H + 2 * oy + (t >> 1)) * W + 2 * ox + (t & 1);
      float* d = dx + px * C + 8 * c8;
      *reinterpret_cast<float4*>(d) = make_float4(o[t][0], o[t][1], o[t][2], o[t][3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(o[t][4], o[t][5], o[t][6], o[t][7]);
    }
  }
}

}  // namespace

void maxpool2_bwd_relu(const void* dy, const uint8_t* pos, const void* y, void* dx, int B, int H, int W, int C,
                       hipStream_t s, bool f32) {
  const long n = static_cast<long>(B) * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return;
  if (f32)
    hipLaunchKernelGGL(maxpool2_bwd_relu_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(dy),
                       pos, static_cast<const float*>(y), static_cast<float*>(dx), B, H, W, C);
  else
    hipLaunchKernelGGL(maxpool2_bwd_relu_kernel, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const bf16_t*>(dy), pos,
                       static_cast<const bf16_t*>(y), static_cast<bf16_t*>(dx), B, H, W, C);
}

void maxpool2_fwd(const void* x, void* y, uint8_t* pos, int dt, int B, int H, int W, int C, hipStream_t s) {
  const long n = static_cast<long>(B) * (H / 2) * (W / 2) * (C / 8);
  if (n == 0) return;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const bf16_t*>(x),
                       static_cast<bf16_t*>(y), pos, B, H, W, C);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), pos, B, H, W, C);
}

void maxpool2_bwd(const void* dy, const uint8_t* pos, void* dx, int dt, int B, int H, int W, int C, hipStream_t s,
                  const void* mask) {
  const long n = static_cast<long>(B) * H * W * (C / 8);
  if (n == 0) return;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const bf16_t*>(dy),
                       pos, static_cast<bf16_t*>(dx), B, H, W, C, static_cast<const bf16_t*>(mask));
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, static_cast<const float*>(dy),
                       pos, static_cast<float*>(dx), B, H, W, C, static_cast<const float*>(mask));
}

namespace {
// mean over the valid entity rows of x [B, N, C] (valid [B, N] bool, count num[b] clamped to >= 1), fp32 accumulation,
// output in x's dtype: the static (graphed) inference path's entity pooling in one launch (was mask cast, multiply,
// sum, count clamp / cast, divide and the output cast: seven small launches per forward).  grid (B, C / 64): the four
// waves take every 4th row of the 64 columns, then sum through LDS in a fixed order.
template <typename T, typename TN>
__global__ __launch_bounds__(256) void entity_mean_pool_kernel(const T* __restrict__ x, const bool* __restrict__ valid,
                                                               const TN* __restrict__ num, T* __restrict__ out, int N,
                                                               int C) {
  __shared__ float red[4][64];
  const int b = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    int n = w;
    for (; n + 4 < N; n += 8) {
      const long r0 = static_cast<long>(b) * N + n, r1 = r0 + 4;
      const float v0 = Cvt<T>::load(x, r0 * C + c), v1 = Cvt<T>::load(x, r1 * C + c);
      a0 += valid[r0] ? v0 : 0.f;
      a1 += valid[r1] ? v1 : 0.f;
    }
    for (; n < N; n += 4) {
      const long r = static_cast<long>(b) * N + n;
      a0 += valid[r] ? Cvt<T>::load(x, r * C + c) : 0.f;
    }
  }
  red[w][threadIdx.x & 63] = a0 + a1;
  __syncthreads();
  if (w == 0 && c < C) {
    const long cnt = static_cast<long>(num[b]);
    const float s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
    Cvt<T>::store(out, static_cast<long>(b) * C + c, s / static_cast<float>(cnt > 1 ? cnt : 1));
  }
}
}  // namespace

void entity_mean_pool(const void* x, int dt, const bool* valid, const void* num, bool num64, void* out, int B, int N,
                      int C, hipStream_t s) {
  if (B == 0 || C == 0) return;
  const dim3 g(B, (C + 63) / 64);
#define AS_EMP(T, TN)                                                                                            \
  hipLaunchKernelGGL((entity_mean_pool_kernel<T, TN>), g, dim3(256), 0, s, static_cast<const T*>(x), valid,      \
                     static_cast<const TN*>(num), static_cast<T*>(out), N, C)
  if (dt == DT_BF16) {
    if (num64) AS_EMP(bf16_t, int64_t); else AS_EMP(bf16_t, int);
  } else {
    if (num64) AS_EMP(float, int64_t); else AS_EMP(float, int);
  }
#undef AS_EMP
}

void segment_sum(const void* x, int dt, const int* cu, float* out, int S, int C, hipStream_t s) {
  if (S == 0) return;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(segment_sum_kernel<bf16_t>, dim3(S), dim3(256), 0, s, static_cast<const bf16_t*>(x), cu, out, C);
  else
    hipLaunchKernelGGL(segment_sum_kernel<float>, dim3(S), dim3(256), 0, s, static_cast<const float*>(x), cu, out, C);
}

void table_grad(const void* src, int dt, const int64_t* idx, float* out, long U, int V, int D, hipStream_t s) {
  const long n = U * D;
  if (n == 0) return;
  long blocks = (n + 4095) / 4096;  // >= 16 elements per thread before the per-block flush
  if (blocks > 256) blocks = 256;
  if (blocks < 1) blocks = 1;
  const size_t lds = static_cast<size_t>(V) * D * sizeof(float);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(table_grad_kernel<bf16_t>, dim3(static_cast<unsigned>(blocks)), dim3(256), lds, s,
                       static_cast<const bf16_t*>(src), idx, out, U, V, D);
  else
    hipLaunchKernelGGL(table_grad_kernel<float>, dim3(static_cast<unsigned>(blocks)), dim3(256), lds, s,
                       static_cast<const float*>(src), idx, out, U, V, D);
}

// idt: 0 int64, 1 int32, 2 int16, 3 uint8, 4 int8
#define AS_EMB_IDX(IDT, BODY)                                      \
  switch (IDT) {                                                   \
    case 0: { using I = int64_t; BODY; } break;                    \
    case 1: { using I = int32_t; BODY; } break;                    \
    case 2: { using I = int16_t; BODY; } break;                    \
    case 3: { using I = uint8_t; BODY; } break;                    \
    default: { using I = int8_t; BODY; } break;                    \
  }

void embed_relu_fwd(const void* table, int dt, const void* idx, int idt, void* out, long U, int V, int D,
                    hipStream_t s) {
  const long n = U * D;
  if (n == 0) return;
  const unsigned blocks = static_cast<unsigned>(std::min<long>((n + 255) / 256, 1024));
  if (dt == DT_BF16) {
    AS_EMB_IDX(idt, hipLaunchKernelGGL((embed_relu_fwd_kernel<bf16_t, I>), dim3(blocks), dim3(256), 0, s,
                                       static_cast<const bf16_t*>(table), static_cast<const I*>(idx),
                                       static_cast<bf16_t*>(out), U, V, D))
  } else {
    AS_EMB_IDX(idt, hipLaunchKernelGGL((embed_relu_fwd_kernel<float, I>), dim3(blocks), dim3(256), 0, s,
                                       static_cast<const float*>(table), static_cast<const I*>(idx),
                                       static_cast<float*>(out), U, V, D))
  }
}

// direct (one workgroup; tiny U * D): dtab written outright; else dtab must be zeroed and takes one atomic per
// nonzero LDS slot of each workgroup (~4 elements per thread: the loop is latency-bound, not bandwidth-bound)
void embed_relu_bwd(const void* dout, const void* out, int dt, const void* idx, int idt, float* dtab, long U, int V,
                    int D, bool direct, hipStream_t s) {
  const long n = U * D;
  long blocks = direct ? 1 : std::min<long>(std::max<long>((n + 1023) / 1024, 1), 256);
  const size_t lds = static_cast<size_t>(V) * D * sizeof(float);
  if (dt == DT_BF16) {
    AS_EMB_IDX(idt, hipLaunchKernelGGL((embed_relu_bwd_kernel<bf16_t, I>), dim3(static_cast<unsigned>(blocks)),
                                       dim3(256), lds, s, static_cast<const bf16_t*>(dout),
                                       static_cast<const bf16_t*>(out), static_cast<const I*>(idx), dtab, U, V, D,
                                       direct ? 1 : 0))
  } else {
    AS_EMB_IDX(idt, hipLaunchKernelGGL((embed_relu_bwd_kernel<float, I>), dim3(static_cast<unsigned>(blocks)),
                                       dim3(256), lds, s, static_cast<const float*>(dout),
                                       static_cast<const float*>(out), static_cast<const I*>(idx), dtab, U, V, D,
                                       direct ? 1 : 0))
  }
}
#undef AS_EMB_IDX

void entity_pack(const void* num, bool num64, int B, int N, long total, bool* valid, int64_t* flat, int64_t* seg,
                 int* cu, hipStream_t s) {
  if (B == 0) return;
  if (num64)
    hipLaunchKernelGGL(entity_pack_kernel<int64_t>, dim3(B), dim3(256), 0, s, static_cast<const int64_t*>(num), B, N,
                       total, valid, flat, seg, cu);
  else
    hipLaunchKernelGGL(entity_pack_kernel<int>, dim3(B), dim3(256), 0, s, static_cast<const int*>(num), B, N, total,
                       valid, flat, seg, cu);
}

// part is scratch: a long reduction (> 1024 rows) overwrites the first row of every 256-row chunk
void column_reduce(const float* part, float* out, int nrows, int cols, hipStream_t s) {
  if (nrows <= 1024) {
    hipLaunchKernelGGL(column_reduce_kernel<float>, dim3((cols + 63) / 64), dim3(1024), 0, s, part, out, nrows, cols,
                       static_cast<long>(cols));
    return;
  }
  const int nchunk = (nrows + 255) / 256;
  hipLaunchKernelGGL(column_reduce_chunk_kernel, dim3((cols + 63) / 64, nchunk), dim3(256), 0, s,
                     const_cast<float*>(part), nrows, cols);
  hipLaunchKernelGGL(column_reduce_kernel<float>, dim3((cols + 63) / 64), dim3(1024), 0, s, part, out, nchunk, cols,
                     256L * cols);
}

void column_reduce_bf16(const float* part, void* out, int nrows, int cols, hipStream_t s) {
  hipLaunchKernelGGL(column_reduce_kernel<bf16_t>, dim3((cols + 63) / 64), dim3(1024), 0, s, part,
                     static_cast<bf16_t*>(out), nrows, cols, static_cast<long>(cols));
}

int ln_affine_slices(long R) { return static_cast<int>((R + kAffRows - 1) / kAffRows); }

void ln_affine_grads(const float* dy, const float* xh, float* part, long R, int C, hipStream_t s) {
  const int S = ln_affine_slices(R);
  if (S == 0 || C == 0) return;
  hipLaunchKernelGGL(ln_affine_grads_kernel, dim3((C + 63) / 64, S), dim3(256), 0, s, dy, xh, part, R, C);
}

}  // namespace as
