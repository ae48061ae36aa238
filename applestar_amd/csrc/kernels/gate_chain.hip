// Chain of four 128 x 128 pointwise (1x1-conv) layers over NHWC pixel rows with the activation tile kept in
// LDS between layers — the location head's GatedResBlock gate path (module_utils.py:204-231 in the
// reference):
//
//   forward   a1 = relu(x W1^T + b1), a2 = relu(a1 W2^T + b2), a3 = relu(a2 W3^T + b3), g = a3 W4^T + b4
//   backward  d3 = (dg W4) * [a3 > 0], d2 = (d3 W3) * [a2 > 0], d1 = (d2 W2) * [a1 > 0], dx = d1 W1 + dres
//
// Both directions are one launch of the same kernel: per layer L the operand M_L is staged as Ms[n][k]
// (forward passes W_L, backward W_L^T), a 128-row tile is multiplied on MFMA (4 waves, 64 x 64 each), the
// epilogue applies bias / ReLU (forward) or the ReLU mask of a saved activation / the residual gradient
// (backward), writes the layer's output rows to HBM (needed by the weight gradients) and leaves them in LDS
// as the next layer's input.  As four library GEMMs (+ three act_grad passes backward) each layer re-read its
// input from HBM: ~25 us per layer per direction on the 145,920-row location-head map (r2cs).
#include "../common.h"
#include "../kernels.h"
#include "../split_mfma.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 gc_bf8v;
typedef __attribute__((ext_vector_type(4))) float gc_f4;

constexpr int kGC = 128;              // channels
constexpr int kGP = kGC + 16;         // LDS row pitch (bf16), 16 mod 32: conflict-free b128 fragment reads
constexpr int kGRows = 128;           // rows per workgroup

__device__ __forceinline__ gc_bf8v gc_frag(const bf16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  gc_bf8v r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

__global__ __launch_bounds__(256) void gate_chain_kernel(GateChainArgs a, long P) {
  const bf16_t* ax = reinterpret_cast<const bf16_t*>(a.x);
  __shared__ __attribute__((aligned(16))) bf16_t xs[kGRows * kGP];
  __shared__ __attribute__((aligned(16))) bf16_t ms[kGC * kGP];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, lr = lane & 15, lg = lane >> 4;
  // bijective XCD-grouped tile order, as in the other tiled kernels
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const long m0 = static_cast<long>(wg) * kGRows;
  constexpr int PIECES = kGRows * kGC / 8 / 256;   // 16-B pieces per thread for a 128 x 128 tile (= 8)

  // input tile and the first operand
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const int piece = tid + 256 * i, r = piece >> 4, c = (piece & 15) * 8;
    const long row = m0 + r;
    const uint4 v = row < P ? *reinterpret_cast<const uint4*>(ax + row * kGC + c) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(xs + r * kGP + c) = v;
    *reinterpret_cast<uint4*>(ms + r * kGP + c) = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.m[0]) + r * kGC + c);
  }
  __syncthreads();
#pragma unroll 1
  for (int L = 0; L < 4; ++L) {
    gc_f4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = gc_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < kGC / 32; ++ks) {
      gc_bf8v af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = gc_frag(xs + (64 * wm + 16 * i + lr) * kGP + 32 * ks + 8 * lg);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = gc_frag(ms + (64 * wn + 16 * j + lr) * kGP + 32 * ks + 8 * lg);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();   // every wave is done reading xs and ms
    // next operand -> ms (overlaps the epilogue)
    if (L < 3) {
#pragma unroll
      for (int i = 0; i < PIECES; ++i) {
        const int piece = tid + 256 * i, r = piece >> 4, c = (piece & 15) * 8;
        *reinterpret_cast<uint4*>(ms + r * kGP + c) = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(a.m[L + 1]) + r * kGC + c);
      }
    }
    // fragments (+ bias, ReLU) -> xs as bf16
    const float* bias = a.bias[L];
    const bool relu = (a.relu_mask >> L) & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = 64 * wn + 16 * j + lr;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][j][e] + bv;
          if (relu) v = fmaxf(v, 0.f);
          xs[(64 * wm + 16 * i + 4 * lg + e) * kGP + col] = f2bf(v);
        }
    }
    __syncthreads();
    // row pieces: ReLU mask of a saved activation / residual gradient, then HBM (and back to xs if masked)
    const bf16_t* msk = reinterpret_cast<const bf16_t*>(a.mask[L]);
    const bf16_t* res = reinterpret_cast<const bf16_t*>(a.res[L]);
    bf16_t* out = reinterpret_cast<bf16_t*>(a.out[L]);
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int piece = tid + 256 * i, r = piece >> 4, c = (piece & 15) * 8;
      const long row = m0 + r;
      if (row >= P) continue;
      uint4 v = *reinterpret_cast<const uint4*>(xs + r * kGP + c);
      if (msk != nullptr || res != nullptr) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        if (msk != nullptr) {
          const uint4 m = *reinterpret_cast<const uint4*>(msk + row * kGC + c);
          const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t lo = __uint_as_float(mw[q] << 16) > 0.f ? 0x0000ffffu : 0u;
            const uint32_t hi = __uint_as_float(mw[q] & 0xffff0000u) > 0.f ? 0xffff0000u : 0u;
            w[q] &= lo | hi;
          }
        }
        if (res != nullptr) {
          const uint4 rr = *reinterpret_cast<const uint4*>(res + row * kGC + c);
          const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            w[q] = f2bf2(__uint_as_float(w[q] << 16) + __uint_as_float(rw[q] << 16),
                         __uint_as_float(w[q] & 0xffff0000u) + __uint_as_float(rw[q] & 0xffff0000u));
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
        *reinterpret_cast<uint4*>(xs + r * kGP + c) = v;
      }
      *reinterpret_cast<uint4*>(out + row * kGC + c) = v;
    }
    __syncthreads();
  }
}

// ---- fp32 chain (the fp32 learner step) on bf16x6 split products (split_mfma.h).  A 64-row tile lives in LDS
// as a pre-split image (three bf16 planes of [64 rows][128 ch], 256-B rows, 16-B chunk index XORed by
// 2 (row & 7) | ((row >> 3) & 1): conflict-free b128 row reads, the attention_f32.hip image).  The product is
// computed transposed, C^T[n][r] = M[n][:] . X[r][:], so each lane ends a layer holding 4 consecutive channels of
// one row: 16-B fp32 stores to HBM and 8-B plane writes of the next layer's image.  Wave w owns channels
// 32 w .. 32 w + 31 (two 16-row A tiles of M, split once per layer into 96 VGPRs) over all 64 rows (four B tiles
// read from the image per k-step).  Measured against four gemm_f32 launches on the 145,920-row location-head map
// (profiles/r4z_gate_chain_f32.txt): forward 164 vs 183 us, backward 243 vs ~200 us, fp32 step unchanged
// (58.2 / 58.2 vs 58.1 / 58.4 ms) - latency-bound at 3 workgroups per CU with a layer-serial chain, so it stays
// behind APPLESTAR_GATE_CHAIN_F32=1 (default off).
constexpr int kFR = 64;                      // rows per workgroup
constexpr int kFPlane = kFR * 256;           // bytes per bf16 plane
__device__ __forceinline__ int gcf_off(int r, int ch) { return 256 * r + 16 * (ch ^ ((2 * (r & 7)) | ((r >> 3) & 1))); }

__device__ __forceinline__ gc_f4 gcf_x6(const Split3& a, const Split3& b, gc_f4 c) {
  auto mm = [](u32v4 x, u32v4 y, gc_f4 acc) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(x), as_bf(y), acc, 0, 0, 0); };
  c = mm(a.p[1], b.p[1], c);
  c = mm(a.p[0], b.p[2], c);
  c = mm(a.p[2], b.p[0], c);
  c = mm(a.p[0], b.p[1], c);
  c = mm(a.p[1], b.p[0], c);
  return mm(a.p[0], b.p[0], c);
}

__global__ __launch_bounds__(256, 2) void gate_chain_f32_kernel(GateChainF32Args a, long P) {
  __shared__ __attribute__((aligned(16))) char img[3 * kFPlane];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lg = lane >> 4;
  const long m0 = static_cast<long>(blockIdx.x) * kFR;
  // input tile -> image: thread t takes row t >> 2 (0..63), chunks 4 (t & 3) .. 4 (t & 3) + 3 (32 floats);
  // rows past P are zero (clamped unconditional loads)
  {
    const int r = tid >> 2, c0 = 4 * (tid & 3);
    const bool ok = m0 + r < P;
    const float4* src = reinterpret_cast<const float4*>(a.x + (ok ? m0 + r : 0) * 128 + 8 * c0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 u = src[2 * c], v = src[2 * c + 1];
      const float f[8] = {ok ? u.x : 0.f, ok ? u.y : 0.f, ok ? u.z : 0.f, ok ? u.w : 0.f,
                          ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f};
      const Split3 sp = split8(f);
      const int o = gcf_off(r, c0 + c);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32v4*>(img + pl * kFPlane + o) = sp.p[pl];
    }
  }
#pragma unroll 1
  for (int L = 0; L < 4; ++L) {
    // this wave's rows of M_L (channels 32 w + 16 j + lr), k = 32 ks + 8 lg + t, split once.  (Loading the next
    // layer's rows during the epilogue: 192 VGPRs, 2 waves / SIMD, 189 us vs 164 - measured, reverted.)
    Split3 mf[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4* mrow = reinterpret_cast<const float4*>(a.m[L] + (32 * w + 16 * j + lr) * 128 + 8 * lg);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float4 u = mrow[8 * ks], v = mrow[8 * ks + 1];
        const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
        mf[j][ks] = split8(f);
      }
    }
    __syncthreads();   // the image holds this layer's input
    gc_f4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[j][m] = gc_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int o = gcf_off(16 * m + lr, 4 * ks + lg);
        Split3 xb;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) xb.p[pl] = *reinterpret_cast<const u32v4*>(img + pl * kFPlane + o);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j][m] = gcf_x6(mf[j][ks], xb, acc[j][m]);
      }
    __syncthreads();   // every wave is done reading the image
    const bool relu = (a.relu_mask >> L) & 1;
    const float* bias = a.bias[L];
    const float* msk = a.mask[L];
    const float* res = a.res[L];
    float* out = a.out[L];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 32 * w + 16 * j + 4 * lg;   // channels n .. n + 3
      const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int r = 16 * m + lr;
        const long row = m0 + r;
        const bool ok = row < P;
        const long ro = (ok ? row : 0) * 128 + n;
        float v[4] = {acc[j][m][0] + bv.x, acc[j][m][1] + bv.y, acc[j][m][2] + bv.z, acc[j][m][3] + bv.w};
        if (relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (msk) {
          const float4 mk = *reinterpret_cast<const float4*>(msk + ro);
          v[0] = mk.x > 0.f ? v[0] : 0.f;
          v[1] = mk.y > 0.f ? v[1] : 0.f;
          v[2] = mk.z > 0.f ? v[2] : 0.f;
          v[3] = mk.w > 0.f ? v[3] : 0.f;
        }
        if (res) {
          const float4 rr = *reinterpret_cast<const float4*>(res + ro);
          v[0] += rr.x;
          v[1] += rr.y;
          v[2] += rr.z;
          v[3] += rr.w;
        }
        if (ok) *reinterpret_cast<float4*>(out + ro) = make_float4(v[0], v[1], v[2], v[3]);
        if (L < 3) {
          uint2 s0, s1, s2;
          split4(make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])),
                 s0, s1, s2);
          const int o = gcf_off(r, n >> 3) + 8 * ((n >> 2) & 1);
          *reinterpret_cast<uint2*>(img + o) = s0;
          *reinterpret_cast<uint2*>(img + kFPlane + o) = s1;
          *reinterpret_cast<uint2*>(img + 2 * kFPlane + o) = s2;
        }
      }
    }
  }
}

}  // namespace

void gate_chain_f32(const GateChainF32Args& a, long P, hipStream_t s) {
  const long nwg = (P + kFR - 1) / kFR;
  if (nwg > 0) hipLaunchKernelGGL(gate_chain_f32_kernel, dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a, P);
}

void gate_chain(const GateChainArgs& a, long P, hipStream_t s) {
  const long nwg = (P + kGRows - 1) / kGRows;
  if (nwg > 0) hipLaunchKernelGGL(gate_chain_kernel, dim3(static_cast<unsigned>(nwg)), dim3(256), 0, s, a, P);
}

}  // namespace as
