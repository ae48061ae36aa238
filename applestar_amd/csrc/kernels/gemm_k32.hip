// out [R][N] = a [R][32] . W [32][N] (bf16 in / out, fp32 accumulate) for the thin-K products of the
// heads: the input gradient of the 256 -> 32 key projections (dX = dK W, R = 196k entity rows) and
// the 32-wide selected-units layers.  hipBLASLt runs these at ~0.19 ms for 100 MB of output (r2an);
// with K = 32 every 16 x 16 output tile is ONE v_mfma_f32_16x16x32_bf16, so the kernel is a pure
// store stream: wave = 16 rows, lane (lg, lr) holds a[row lr][8 lg .. +8] as the B operand and
// W^T[16 j + lr][8 lg .. +8] as the A operand of C^T = W^T a^T, and writes out[row lr][16 j + 4 lg .. +3]
// (8 B) per column tile.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 k32_bf8;
typedef __attribute__((ext_vector_type(4))) float k32_f4;

__device__ __forceinline__ k32_bf8 ld_k32(const bf16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  k32_bf8 r;
  __builtin_memcpy(&r, &u, 16);
  return r;
}

// wT [N][32]; grid = ceil(R / 64), 256 threads (4 waves x 16 rows)
__global__ __launch_bounds__(256) void mm_k32_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ wT,
                                                     bf16_t* __restrict__ out, long R, int N) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, lr = l & 15, lg = l >> 4;
  const long row = static_cast<long>(blockIdx.x) * 64 + 16 * w + lr;
  const bool ok = row < R;
  const k32_bf8 bx = ld_k32(a + (ok ? row : 0) * 32 + 8 * lg);
  bf16_t* dst = out + row * N + 4 * lg;
  for (int j = 0; j < N / 16; ++j) {
    const k32_bf8 aw = ld_k32(wT + (16 * j + lr) * 32 + 8 * lg);
    const k32_f4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx, k32_f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    if (ok) *reinterpret_cast<uint2*>(dst + 16 * j) = make_uint2(f2bf2(c[0], c[1]), f2bf2(c[2], c[3]));
  }
}

}  // namespace

void mm_k32(const void* a, const void* wT, void* out, long R, int N, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(mm_k32_kernel, dim3(static_cast<unsigned>((R + 63) / 64)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(a), static_cast<const bf16_t*>(wT), static_cast<bf16_t*>(out), R, N);
}

}  // namespace as
