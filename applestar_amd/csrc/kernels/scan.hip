// Batched reverse linear recurrence  y[t] = a[t] * y[t+1] + b[t]  (t = T-1 .. 0, y[T] = init).
//
// V-trace (vs - V), TD(lambda) and UPGO lambda-returns are all this recurrence
// (as_rl_utils.py:157-312); the loss stacks the six policy heads (and every baseline field) into K
// independent [T, B] problems so one launch replaces 6 x T x ~4 tiny torch kernels.  One lane owns
// one (k, b) column and walks time backwards; loads across lanes are contiguous in b.
#include "../common.h"
#include "../kernels.h"

namespace as {
namespace {

__global__ __launch_bounds__(256) void reverse_scan_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ init, float* __restrict__ y,
                                                           int K, int T, int B) {
  const long col = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (col >= static_cast<long>(K) * B) return;
  const int k = static_cast<int>(col / B);
  const int bb = static_cast<int>(col % B);
  const long base = static_cast<long>(k) * T * B + bb;
  float acc = init[col];
  for (int t = T - 1; t >= 0; --t) {
    const long i = base + static_cast<long>(t) * B;
    acc = fmaf(a[i], acc, b[i]);
    y[i] = acc;
  }
}

}  // namespace

void reverse_scan(const float* a, const float* b, const float* init, float* y, int K, int T, int B, hipStream_t s) {
  const long n = static_cast<long>(K) * B;
  hipLaunchKernelGGL(reverse_scan_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, a, b, init,
                     y, K, T, B);
}

}  // namespace as
