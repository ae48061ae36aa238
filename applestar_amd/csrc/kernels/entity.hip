// Entity-encoder input embedding without the 997-wide one-hot tensor.
//
// The reference concatenates 29 one-hot / 2 x 11-bit binary / 7 scalar encodings of each unit into a
// [B, N, 997] fp32 tensor and multiplies by W[256, 997] (entity_encoder.py:61-78, K1 in SURVEY).
// one-hot(v) @ W^T is a row gather of W^T, so the forward here is an embedding-bag: one wave per
// (packed, real) entity, each lane accumulating 4 of the 256 output channels from the selected
// W^T rows (8-16 B per lane, L2-resident 0.5 MB table), + bias, ReLU.  The weight gradient
// (entity_embed_wgrad) runs on MFMA with the one-hot input generated in registers from the raw fields
// instead of materialising the [T, 997] input for a library GEMM (r2an: 0.46 ms).  (A first version
// scattered dpre into an LDS [997][32] tile with float atomics: 7.6 ms - LDS atomics are slow.)
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

// wT [K_in][256]; out [T][256].  Per entity, lane k < f.n loads field k's value (one memory latency for all
// fields), expands it into its (W^T row, scale) entries - 1 for one-hot / scalar fields, one per set bit of a
// binary field - and writes them at its exclusive prefix offset into the wave's LDS list; the wave then
// gathers the rows four at a time (four row loads in flight) and accumulates them in list order, i.e. the same
// order (and so the same bits) as a field-by-field loop.  Lists longer than kEeList entries fall back to that
// loop.
constexpr int kEeList = 128;

template <typename TW>
__device__ __forceinline__ void ee_fields_serial(const EntityFields& f, long src, const TW* __restrict__ wT, int lane,
                                                 float* acc) {
  constexpr int C = 256;
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
}

template <typename TW, typename TO>
__global__ __launch_bounds__(256) void entity_embed_fwd_kernel(EntityFields f, const int64_t* __restrict__ index,
                                                               const TW* __restrict__ wT, const float* __restrict__ bias,
                                                               TO* __restrict__ out, long T) {
  constexpr int C = 256;
  __shared__ int s_col[4][kEeList];
  __shared__ float s_scale[4][kEeList];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long wave = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const long nwave = (static_cast<long>(gridDim.x) * blockDim.x) >> 6;
  const float4 bv = *reinterpret_cast<const float4*>(bias + lane * 4);
  const int nf = f.n;
  // this lane's field (lane < nf): kind / offset / width / source, fixed for the whole kernel
  const int kk = lane < nf ? lane : 0;
  int kind = 0, off = 0, width = 1, fdt = 0;
  const void* fptr = nullptr;
  for (int k = 0; k < nf; ++k)      // uniform loop: picks the lane's entry without dynamic kernarg indexing
    if (k == kk) { kind = f.kind[k]; off = f.offset[k]; width = f.width[k]; fdt = f.dtype[k]; fptr = f.ptr[k]; }
  for (long t = wave; t < T; t += nwave) {
    const long src = index[t];
    float acc[4] = {bv.x, bv.y, bv.z, bv.w};
    int cnt = 0, iv = 0;
    float v = 0.f;
    if (lane < nf) {
      v = load_field(fptr, fdt, src);
      if (kind == FIELD_BINARY) {
        iv = clampi(static_cast<int>(v), 0, (1 << width) - 1);
        cnt = __popc(iv);
      } else {
        cnt = 1;
      }
    }
    // exclusive prefix sum of cnt over the wave
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    const int total = __shfl(incl, 63, 64);
    if (total > kEeList) {
      ee_fields_serial<TW>(f, src, wT, lane, acc);
    } else {
      int pos = incl - cnt;
      if (lane < nf) {
        if (kind == FIELD_ONE_HOT) {
          s_col[wv][pos] = off + clampi(static_cast<int>(v), 0, width - 1);
          s_scale[wv][pos] = 1.f;
        } else if (kind == FIELD_BINARY) {
          for (int bit = 0; bit < width; ++bit)
            if ((iv >> (width - 1 - bit)) & 1) {
              s_col[wv][pos] = off + bit;
              s_scale[wv][pos] = 1.f;
              ++pos;
            }
        } else {
          s_col[wv][pos] = off;
          s_scale[wv][pos] = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      int e = 0;
      for (; e + 4 <= total; e += 4) {
        int col[4];
        float sc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) { col[u] = s_col[wv][e + u]; sc[u] = s_scale[wv][e + u]; }
        float r[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u][0] = r[u][1] = r[u][2] = r[u][3] = 0.f;
          Row4<TW>::add(wT + static_cast<long>(col[u]) * C + lane * 4, 1.f, r[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = fmaf(sc[u], r[u][i], acc[i]);
      }
      for (; e < total; ++e) Row4<TW>::add(wT + static_cast<long>(s_col[wv][e]) * C + lane * 4, s_scale[wv][e], acc);
      __builtin_amdgcn_wave_barrier();     // the list is rewritten for the next entity
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


// Weight gradient on the matrix cores: dW [256][K_in] = dpre^T X with the sparse X built per step.
// Workgroup = (64-channel slice cs, token chunk), 8 waves; wave w owns output columns 128 w .. 128 w + 127
// (8 column tiles x 4 channel tiles of 16x16x32 MFMA accumulators).  Per 32-token step: dpre = dout *
// [out > 0] of the slice is staged transposed in LDS ([64 n][32 t], the A operand), and X^T
// ([1024 cols][32 t] bf16, zeroed each step) receives the step's ~58 nonzeros per token, one thread per
// (token, field) pair - the B fragments are then plain 16-B row reads.  Column K_in (< 1024) is a ones
// column whose accumulator is db.  The next step's dout / out / field values are loaded during the
// current step's MFMAs.  Partials: part[chunk] = [256 * K_in] dW | [256] db, reduced over chunks.
// (Per-lane generation of X from the field values was VALU-bound: 0.56 ms.)
typedef __attribute__((ext_vector_type(8))) __bf16 ew_bf8;
typedef __attribute__((ext_vector_type(4))) float ew_f4;
constexpr int kEwStep = 32, kEwDP = kEwStep + 8;   // tokens per MFMA step, padded LDS row (bf16)

template <typename TD>
__global__ __launch_bounds__(512) void entity_wgrad_kernel(EntityFields f, const int64_t* __restrict__ index,
                                                           const TD* __restrict__ dout, const TD* __restrict__ out,
                                                           float* __restrict__ part, long T, int K_in, int nchunk) {
  __shared__ __attribute__((aligned(16))) bf16_t dT[64 * kEwDP];
  __shared__ __attribute__((aligned(16))) bf16_t xT[1024 * kEwDP];
  const int cs = blockIdx.x & 3, chunk = blockIdx.x >> 2;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6, lr = l & 15, lg = l >> 4;
  ew_f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = ew_f4{0.f, 0.f, 0.f, 0.f};
  const long per = (T + nchunk - 1) / nchunk;
  const long t0 = chunk * per, t1 = t0 + per < T ? t0 + per : T;
  const int tt_d = tid >> 4, c4 = 4 * (tid & 15);
  float dreg[4], freg[3];
  auto load_step = [&](long base) {
    {
      const long t = base + tt_d;
      const bool ok = t < t1;
      const long o = (ok ? t : t0) * 256 + 64 * cs + c4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float ov = Cvt<TD>::load(out, o + e), dv = Cvt<TD>::load(dout, o + e);
        dreg[e] = (ok && ov > 0.f) ? dv : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int i = tid + 512 * r;
      const int k = i / kEwStep, tt = i - k * kEwStep;
      const long t = base + tt < t1 ? base + tt : t0;
      freg[r] = k < f.n ? load_field(f.ptr[k], f.dtype[k], index[t]) : 0.f;
    }
  };
  static_assert(kMaxFields * kEwStep <= 3 * 512, "field staging: 3 values per thread");
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  if (t0 < t1) load_step(t0);
  for (long base = t0; base < t1; base += kEwStep) {
    __syncthreads();   // previous step's tiles consumed
    // zero X^T (1024 rows x 64 B of data per row; the pad columns are never read)
    for (int i = tid; i < 1024 * 4; i += 512) *reinterpret_cast<uint4*>(xT + (i >> 2) * kEwDP + 8 * (i & 3)) = z4;
#pragma unroll
    for (int e = 0; e < 4; ++e) dT[(c4 + e) * kEwDP + tt_d] = f2bf(dreg[e]);
    __syncthreads();
    if (tid < kEwStep) xT[K_in * kEwDP + tid] = base + tid < t1 ? 0x3F80 : 0;   // ones column (db)
#pragma unroll
    for (int r = 0; r < 3; ++r) {   // scatter the nonzeros of (token tt, field k)
      const int i = tid + 512 * r;
      const int k = i / kEwStep, tt = i - k * kEwStep;
      if (k < f.n && base + tt < t1) {
        const float v = freg[r];
        const int off = f.offset[k], width = f.width[k];
        if (f.kind[k] == FIELD_ONE_HOT) {
          xT[(off + clampi(static_cast<int>(v), 0, width - 1)) * kEwDP + tt] = 0x3F80;
        } else if (f.kind[k] == FIELD_BINARY) {
          const int iv = clampi(static_cast<int>(v), 0, (1 << width) - 1);
          for (int bit = 0; bit < width; ++bit)
            if ((iv >> (width - 1 - bit)) & 1) xT[(off + bit) * kEwDP + tt] = 0x3F80;
        } else {
          xT[off * kEwDP + tt] = f2bf(v);
        }
      }
    }
    __syncthreads();
    if (base + kEwStep < t1) load_step(base + kEwStep);
    ew_bf8 af[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const uint4 u = *reinterpret_cast<const uint4*>(dT + (16 * nt + lr) * kEwDP + 8 * lg);
      __builtin_memcpy(&af[nt], &u, 16);
    }
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) {
      const uint4 u = *reinterpret_cast<const uint4*>(xT + (128 * w + 16 * ct + lr) * kEwDP + 8 * lg);
      ew_bf8 bx;
      __builtin_memcpy(&bx, &u, 16);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[ct][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bx, acc[ct][nt], 0, 0, 0);
    }
  }
  // C[n = 16 nt + 4 lg + i][col = 128 w + 16 ct + lr]
  float* row = part + static_cast<long>(chunk) * (256L * K_in + 256);
#pragma unroll
  for (int ct = 0; ct < 8; ++ct) {
    const int col = 128 * w + 16 * ct + lr;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = 64 * cs + 16 * nt + 4 * lg + i;
        if (col < K_in) row[static_cast<long>(n) * K_in + col] = acc[ct][nt][i];
        else if (col == K_in) row[256L * K_in + n] = acc[ct][nt][i];
      }
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

int entity_wgrad_chunks(long T) {
  long n = (T + 1023) / 1024;   // ~1k+ tokens per workgroup, <= 64 chunks (x 4 channel slices)
  return static_cast<int>(n < 1 ? 1 : (n > 64 ? 64 : n));
}

void entity_embed_wgrad(const EntityFields& f, const int64_t* index, const void* dout, const void* out, int dt,
                        float* part, long T, int K_in, int nchunk, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(nchunk) * 4);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(entity_wgrad_kernel<bf16_t>, grid, dim3(512), 0, s, f, index, static_cast<const bf16_t*>(dout),
                       static_cast<const bf16_t*>(out), part, T, K_in, nchunk);
  else
    hipLaunchKernelGGL(entity_wgrad_kernel<float>, grid, dim3(512), 0, s, f, index, static_cast<const float*>(dout),
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
