// Few-row products of ANY shape, both directions, in fp32 (bf16x6 split or exact-f32 MFMA) and bf16:
//   small_nt: out [M, N] = epi( mask(A) [M, K] . B [N, K]^T )        (forward, and dX = dY . W against W^T)
//   small_tn: dW [N, K] = mask(dY)^T [N, R] . X [R, K],  db [N] = sum_r mask(dY)[r, :]
// The scalar encoder's one-hot inputs (K = 10, 90, 167, 269), the 327-, 2- and 1-wide head / value outputs and
// the GLU gates (sigmoid) of the heads do not meet the aligned kernels' K % 4 / K % 8 rule, so until r4 every
// such layer was three library GEMMs (forward, dX, dW) + a ones-row GEMV for db + a separate ReLU-mask pass.
// Here one workgroup owns one 32 x 32 output tile and its four waves split the reduction; operands are read
// element by element with bounds checks (rows of odd length are not 16-B aligned), straight from L2 into
// registers; the four partial tiles meet once in LDS.  The activation gradient of the layer's output
// ("mask": ReLU y > 0, or sigmoid y (1 - y), from the saved output y) is applied to the gradient operand as it
// is loaded, so backward is two launches (dX, dW + db) with no elementwise pass.
//   lane (l32, h): output row side index l32, k-slots 8 h .. 8 h + 7 of each 16-deep reduction step
//   split mode: one bf16x6 product per step; exact mode: eight v_mfma_f32_32x32x2_f32; bf16: one bf16 MFMA
// The accumulator is the transposed tile: lane = output row, registers 4 g + q = column 8 g + 4 h + q.
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"

namespace as {
namespace {

__device__ __forceinline__ float grad_mask(float y, int mode) {
  return mode == ACT_RELU ? (y > 0.f ? 1.f : 0.f) : (mode == ACT_SIGMOID ? y * (1.f - y) : 1.f);
}

// acc += one 16-deep step: va = the output-row side (8 k values), vb = the output-column side
template <typename T, int SPLIT>
__device__ __forceinline__ void step_mfma(const float (&va)[8], const float (&vb)[8], f32x16& acc) {
  if constexpr (sizeof(T) == 2) {
    const u32v4 a = u32v4{f2bf2(va[0], va[1]), f2bf2(va[2], va[3]), f2bf2(va[4], va[5]), f2bf2(va[6], va[7])};
    const u32v4 b = u32v4{f2bf2(vb[0], vb[1]), f2bf2(vb[2], vb[3]), f2bf2(vb[4], vb[5]), f2bf2(vb[6], vb[7])};
    acc = mfma_bf16(b, a, acc);
  } else if constexpr (SPLIT) {
    acc = mfma_x6(split8(vb), split8(va), acc);
  } else {
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vb[t], va[t], acc, 0, 0, 0);
  }
}

// 8 values of row `row` (element offset, < 0: none) at k0 .. k0 + 7 through 16-B buffer loads (rows 16-B aligned:
// K % 4 fp32 / K % 8 bf16); a piece at or past K, or of a missing row, reads zeros (out-of-range offset)
template <typename T>
__device__ __forceinline__ void load8_vec(__amdgpu_buffer_rsrc_t r, long row, int k0, int K, float (&v)[8]) {
  constexpr int kOOBv = 0x7ffffff0;
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int off = row >= 0 && k0 + 4 * q < K ? static_cast<int>((row + k0 + 4 * q) * 4) : kOOBv;
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * q + j] = __uint_as_float(x[j]);
    }
  } else {
    const int off = row >= 0 && k0 < K ? static_cast<int>((row + k0) * 2) : kOOBv;
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(x[j] << 16);
      v[2 * j + 1] = __uint_as_float(x[j] & 0xffff0000u);
    }
  }
}

template <typename T, int SPLIT, bool VEC = false>
__global__ __launch_bounds__(256) void small_nt_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                       const float* __restrict__ bias, const T* __restrict__ res,
                                                       const T* __restrict__ amask, int mask_mode,
                                                       T* __restrict__ out, long M, int N, int K, int act,
                                                       int tiles_n, int kspan, float* __restrict__ part) {
  __shared__ float red[3][16][64];
  const int tn = blockIdx.x % tiles_n;
  const long tm = blockIdx.x / tiles_n;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const long m = tm * 32 + l32;
  const int n = tn * 32 + l32;
  const bool mok = m < M, nok = n < N;
  const long arow = mok ? m * K : 0, brow = nok ? static_cast<long>(n) * K : 0;
  // split-K (part != nullptr): slice blockIdx.y covers K-steps [y kspan, (y + 1) kspan) and stores its raw
  // partial tile to part[y] (small_nt_finish sums the slices in order and applies the epilogue)
  const int KT = (K + 15) / 16;
  const int kt0 = part ? blockIdx.y * kspan : 0;
  const int kt1 = part ? min(KT, kt0 + kspan) : KT;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;

  if constexpr (VEC) {
    // aligned rows: 16-B buffer loads, KU K-steps of both operands in flight per wave (the long-K split-K slices
    // and the aligned few-row products); the activation-gradient mask is not used on this path
    constexpr int KU = 4;
    const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(a), 0,
                                                                        static_cast<int>(M * K * sizeof(T)), 0x00020000);
    const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(b), 0, static_cast<int>(static_cast<long>(N) * K * sizeof(T)), 0x00020000);
    const long ra0 = mok ? arow : -1, rb0 = nok ? brow : -1;
    float va[KU][8], vb[KU][8];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int kt = kt0 + w + 4 * u;
      load8_vec<T>(ar, kt < kt1 ? ra0 : -1, 16 * kt + 8 * h, K, va[u]);
      load8_vec<T>(br, kt < kt1 ? rb0 : -1, 16 * kt + 8 * h, K, vb[u]);
    }
    for (int kt = kt0 + w; kt < kt1; kt += 4 * KU) {
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const int kc = kt + 4 * u;
        if (kc >= kt1) break;
        float xa[8], xb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { xa[j] = va[u][j]; xb[j] = vb[u][j]; }
        const int kn = kc + 4 * KU;          // refill the slot just read (zeros past the slice)
        load8_vec<T>(ar, kn < kt1 ? ra0 : -1, 16 * kn + 8 * h, K, va[u]);
        load8_vec<T>(br, kn < kt1 ? rb0 : -1, 16 * kn + 8 * h, K, vb[u]);
        step_mfma<T, SPLIT>(xa, xb, acc);
      }
    }
  } else {
    for (int kt = kt0 + w; kt < kt1; kt += 4) {
      const int k0 = 16 * kt + 8 * h;
      float va[8], vb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool kok = k0 + j < K;
        va[j] = mok && kok ? Cvt<T>::load(a, arow + k0 + j) : 0.f;
        vb[j] = nok && kok ? Cvt<T>::load(b, brow + k0 + j) : 0.f;
        if (amask != nullptr && mok && kok) va[j] *= grad_mask(Cvt<T>::load(amask, arow + k0 + j), mask_mode);
      }
      step_mfma<T, SPLIT>(va, vb, acc);
    }
  }
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w - 1][e][lane] = acc[e];
  }
  __syncthreads();
  if (w != 0 || !mok) return;
  if (part != nullptr) {
    float* prow = part + (static_cast<long>(blockIdx.y) * M + m) * N;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = 4 * g + q, nn = tn * 32 + 8 * g + 4 * h + q;
        if (nn < N) prow[nn] = acc[e] + red[0][e][lane] + red[1][e][lane] + red[2][e][lane];
      }
    return;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * g + q, nn = tn * 32 + 8 * g + 4 * h + q;
      if (nn >= N) continue;
      float x = acc[e] + red[0][e][lane] + red[1][e][lane] + red[2][e][lane];
      if (bias) x += bias[nn];
      if (res) {
        const float r = Cvt<T>::load(res, m * N + nn);
        x = act == ACT_DRELU ? (r > 0.f ? x : 0.f) : x + r;
      }
      if (act == ACT_RELU) x = fmaxf(x, 0.f);
      else if (act == ACT_SIGMOID) x = 1.f / (1.f + expf(-x));
      Cvt<T>::store(out, m * N + nn, x);
    }
  }
}

// dW tile (rows n0 .. n0 + 31 of dW = columns of dY, columns k0 .. k0 + 31 = columns of X); the workgroups of the
// first column tile also produce db.  lane (l32, h): dY column n0 + l32 and X column k0 + l32 at rows
// 16 s + 8 h .. + 7 of reduction step s (wave w takes steps w, w + NW, ...): every load instruction reads 32
// consecutive elements of one row (coalesced).  NW = 16 waves once the reduction has >= 32 steps (R >= 512,
// small_tn_waves): each wave's loop is a chain of dependent L2 round trips, so more waves = shorter chains.
template <typename T, typename TO, int SPLIT, int NW>
__global__ __launch_bounds__(64 * NW) void small_tn_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ ymask, int mask_mode,
                                                       TO* __restrict__ dw, TO* __restrict__ db, long R, int N,
                                                       int K, int tiles_k) {
  __shared__ float red[NW - 1][16][64];
  __shared__ float dbs[NW][64];
  const int tk = blockIdx.x % tiles_k, tn = blockIdx.x / tiles_k;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
  const int n = tn * 32 + l32, k = tk * 32 + l32;
  const bool nok = n < N, kok = k < K;
  const bool want_db = db != nullptr && tk == 0;
  const long RT = (R + 15) / 16;
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  float dsum = 0.f;
  // one reduction step's operands: 8 rows of the lane's dY column (masked) and X column; the next step's are
  // loaded before this one's MFMAs (the loop is latency-bound: a handful of steps per wave)
  auto load = [&](long s, float (&va)[8], float (&vb)[8]) {
    const long r0 = 16 * s + 8 * h;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool rok = s < RT && r0 + j < R;
      va[j] = rok && nok ? Cvt<T>::load(dy, (r0 + j) * N + n) : 0.f;
      if (ymask != nullptr && rok && nok) va[j] *= grad_mask(Cvt<T>::load(ymask, (r0 + j) * N + n), mask_mode);
      vb[j] = rok && kok ? Cvt<T>::load(x, (r0 + j) * K + k) : 0.f;
    }
  };
  float ca[8], cb[8];
  load(w, ca, cb);
  for (long s = w; s < RT; s += NW) {
    float na[8], nb[8];
    load(s + NW, na, nb);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += ca[j];
    step_mfma<T, SPLIT>(ca, cb, acc);
#pragma unroll
    for (int j = 0; j < 8; ++j) { ca[j] = na[j]; cb[j] = nb[j]; }
  }
  if (w > 0) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[w - 1][e][lane] = acc[e];
  }
  if (want_db) dbs[w][lane] = dsum;
  __syncthreads();
  if (w != 0) return;
  if (want_db && h == 0 && nok) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += dbs[q][l32] + dbs[q][l32 + 32];
    Cvt<TO>::store(db, n, t);
  }
  if (!nok) return;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = 4 * g + q, kk = tk * 32 + 8 * g + 4 * h + q;
      if (kk >= K) continue;
      float v = acc[e];
#pragma unroll
      for (int q = 0; q < NW - 1; ++q) v += red[q][e][lane];
      Cvt<TO>::store(dw, static_cast<long>(n) * K + kk, v);
    }
  }
}

// out[m, n] = epi(sum_s part[s, m, n]) in slice order (deterministic), the small_nt epilogue (bias, act)
template <typename T>
__global__ __launch_bounds__(256) void small_nt_finish_kernel(const float* __restrict__ part, int S,
                                                              const float* __restrict__ bias, T* __restrict__ out,
                                                              long MN, int N, int act) {
  const long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= MN) return;
  float x = 0.f;
  for (int s = 0; s < S; ++s) x += part[s * MN + i];
  if (bias) x += bias[i % N];
  if (act == ACT_RELU) x = fmaxf(x, 0.f);
  else if (act == ACT_SIGMOID) x = 1.f / (1.f + expf(-x));
  Cvt<T>::store(out, i, x);
}

}  // namespace

// the 16-B-load path: rows 16-B aligned (K % 4 fp32 / K % 8 bf16), 16-B aligned bases, byte sizes < 2^31
bool small_vec_ok(const void* a, const void* b, long M, int N, int K, bool bf16) {
  const long es = bf16 ? 2 : 4;
  return K % (16 / es) == 0 && (reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(b) & 15) == 0 &&
         M * K * es < 0x7ffffff0L && static_cast<long>(N) * K * es < 0x7ffffff0L;
}

int small_nt_splits(long M, int N, int K) {
  // few tiles and a long reduction (the spatial encoder's 48,640-wide fc over ~400 rows): slice K so that the
  // grid reaches ~2 workgroups per CU, each slice >= 64 K-steps of 16
  const long tiles = (M + 31) / 32 * ((N + 31) / 32);
  const int kt = (K + 15) / 16;
  if (tiles >= 256 || kt < 256) return 1;
  int s = static_cast<int>((2048 + tiles - 1) / tiles);   // ~2048 workgroups, slices of >= 32 K-steps
  s = min(s, kt / 32);
  return max(1, min(s, 64));
}

void small_nt_splitk(const void* a, const void* b, const float* bias, float* part, int S, void* out, long M, int N,
                     int K, int act, bool bf16, hipStream_t s) {
  const int tn = (N + 31) / 32;
  const long nwg = (M + 31) / 32 * tn;
  if (nwg == 0) return;
  const int KT = (K + 15) / 16, kspan = (KT + S - 1) / S;
  const dim3 g(static_cast<unsigned>(nwg), static_cast<unsigned>(S)), blk(256);
  const long MN = M * N;
  const dim3 gf(static_cast<unsigned>((MN + 255) / 256));
  const bool vec = small_vec_ok(a, b, M, N, K, bf16);
  if (bf16) {
    if (vec)
      hipLaunchKernelGGL((small_nt_kernel<bf16_t, 0, true>), g, blk, 0, s, static_cast<const bf16_t*>(a),
                         static_cast<const bf16_t*>(b), nullptr, nullptr, nullptr, 0, nullptr, M, N, K, 0, tn, kspan,
                         part);
    else
      hipLaunchKernelGGL((small_nt_kernel<bf16_t, 0>), g, blk, 0, s, static_cast<const bf16_t*>(a),
                         static_cast<const bf16_t*>(b), nullptr, nullptr, nullptr, 0, nullptr, M, N, K, 0, tn, kspan,
                         part);
    hipLaunchKernelGGL(small_nt_finish_kernel<bf16_t>, gf, blk, 0, s, part, S, bias, static_cast<bf16_t*>(out), MN,
                       N, act);
  } else {
    if (f32_mfma_mode() == 0)
      hipLaunchKernelGGL((small_nt_kernel<float, 0>), g, blk, 0, s, static_cast<const float*>(a),
                         static_cast<const float*>(b), nullptr, nullptr, nullptr, 0, nullptr, M, N, K, 0, tn, kspan,
                         part);
    else if (vec)
      hipLaunchKernelGGL((small_nt_kernel<float, 1, true>), g, blk, 0, s, static_cast<const float*>(a),
                         static_cast<const float*>(b), nullptr, nullptr, nullptr, 0, nullptr, M, N, K, 0, tn, kspan,
                         part);
    else
      hipLaunchKernelGGL((small_nt_kernel<float, 1>), g, blk, 0, s, static_cast<const float*>(a),
                         static_cast<const float*>(b), nullptr, nullptr, nullptr, 0, nullptr, M, N, K, 0, tn, kspan,
                         part);
    hipLaunchKernelGGL(small_nt_finish_kernel<float>, gf, blk, 0, s, part, S, bias, static_cast<float*>(out), MN, N,
                       act);
  }
}

void small_nt(const void* a, const void* b, const float* bias, const void* res, const void* amask, int mask_mode,
              void* out, long M, int N, int K, int act, bool bf16, hipStream_t s) {
  const int tn = (N + 31) / 32;
  const long nwg = (M + 31) / 32 * tn;
  if (nwg == 0) return;
  const dim3 g(static_cast<unsigned>(nwg)), blk(256);
  if ((amask == nullptr || mask_mode == 0) && small_vec_ok(a, b, M, N, K, bf16) && (bf16 || f32_mfma_mode() != 0)) {
    if (bf16)
      hipLaunchKernelGGL((small_nt_kernel<bf16_t, 0, true>), g, blk, 0, s, static_cast<const bf16_t*>(a),
                         static_cast<const bf16_t*>(b), bias, static_cast<const bf16_t*>(res), nullptr, 0,
                         static_cast<bf16_t*>(out), M, N, K, act, tn, 0, nullptr);
    else
      hipLaunchKernelGGL((small_nt_kernel<float, 1, true>), g, blk, 0, s, static_cast<const float*>(a),
                         static_cast<const float*>(b), bias, static_cast<const float*>(res), nullptr, 0,
                         static_cast<float*>(out), M, N, K, act, tn, 0, nullptr);
    return;
  }
  if (bf16) {
    hipLaunchKernelGGL((small_nt_kernel<bf16_t, 0>), g, blk, 0, s, static_cast<const bf16_t*>(a),
                       static_cast<const bf16_t*>(b), bias, static_cast<const bf16_t*>(res),
                       static_cast<const bf16_t*>(amask), mask_mode, static_cast<bf16_t*>(out), M, N, K, act, tn, 0,
                       nullptr);
  } else if (f32_mfma_mode() == 0) {
    hipLaunchKernelGGL((small_nt_kernel<float, 0>), g, blk, 0, s, static_cast<const float*>(a),
                       static_cast<const float*>(b), bias, static_cast<const float*>(res),
                       static_cast<const float*>(amask), mask_mode, static_cast<float*>(out), M, N, K, act, tn, 0,
                       nullptr);
  } else {
    hipLaunchKernelGGL((small_nt_kernel<float, 1>), g, blk, 0, s, static_cast<const float*>(a),
                       static_cast<const float*>(b), bias, static_cast<const float*>(res),
                       static_cast<const float*>(amask), mask_mode, static_cast<float*>(out), M, N, K, act, tn, 0,
                       nullptr);
  }
}

// waves per workgroup of small_tn: 16 when the reduction has >= 32 steps (R >= 512), else 4
// (APPLESTAR_SMALL_TN_WAVES = 4 | 16 forces one)
int small_tn_waves(long R) {
  static const int forced = [] {
    const char* e = std::getenv("APPLESTAR_SMALL_TN_WAVES");
    return e ? std::atoi(e) : 0;
  }();
  if (forced == 4 || forced == 16) return forced;
  return (R + 15) / 16 >= 32 ? 16 : 4;
}

template <int NW>
void small_tn_launch(const void* dy, const void* x, const void* ymask, int mask_mode, void* dw, void* db, long R,
                     int N, int K, bool bf16_in, bool bf16_out, hipStream_t s) {
  const int tk = (K + 31) / 32;
  const long nwg = static_cast<long>((N + 31) / 32) * tk;
  if (nwg == 0) return;
  const dim3 g(static_cast<unsigned>(nwg)), blk(64 * NW);
  if (bf16_in) {
    if (bf16_out)
      hipLaunchKernelGGL((small_tn_kernel<bf16_t, bf16_t, 0, NW>), g, blk, 0, s, static_cast<const bf16_t*>(dy),
                         static_cast<const bf16_t*>(x), static_cast<const bf16_t*>(ymask), mask_mode,
                         static_cast<bf16_t*>(dw), static_cast<bf16_t*>(db), R, N, K, tk);
    else
      hipLaunchKernelGGL((small_tn_kernel<bf16_t, float, 0, NW>), g, blk, 0, s, static_cast<const bf16_t*>(dy),
                         static_cast<const bf16_t*>(x), static_cast<const bf16_t*>(ymask), mask_mode,
                         static_cast<float*>(dw), static_cast<float*>(db), R, N, K, tk);
  } else if (f32_mfma_mode() == 0) {
    hipLaunchKernelGGL((small_tn_kernel<float, float, 0, NW>), g, blk, 0, s, static_cast<const float*>(dy),
                       static_cast<const float*>(x), static_cast<const float*>(ymask), mask_mode,
                       static_cast<float*>(dw), static_cast<float*>(db), R, N, K, tk);
  } else {
    hipLaunchKernelGGL((small_tn_kernel<float, float, 1, NW>), g, blk, 0, s, static_cast<const float*>(dy),
                       static_cast<const float*>(x), static_cast<const float*>(ymask), mask_mode,
                       static_cast<float*>(dw), static_cast<float*>(db), R, N, K, tk);
  }
}

void small_tn(const void* dy, const void* x, const void* ymask, int mask_mode, void* dw, void* db, long R, int N,
              int K, bool bf16_in, bool bf16_out, hipStream_t s) {
  if (small_tn_waves(R) == 16) small_tn_launch<16>(dy, x, ymask, mask_mode, dw, db, R, N, K, bf16_in, bf16_out, s);
  else small_tn_launch<4>(dy, x, ymask, mask_mode, dw, db, R, N, K, bf16_in, bf16_out, s);
}

}  // namespace as
