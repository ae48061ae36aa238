// Timing ablation of gemm_f32.hip (split mode) on the entity transformer's shapes.  Built once per GF_ABL
// value (see gemm_f32.hip); prints "abl M N K us tflops".
#include "../../applestar_amd/csrc/kernels/gemm_f32.hip"

#include <cstdio>
#include <vector>

static void run(long M, int N, int K) {
  std::vector<float> ha(M * K), hb(static_cast<long>(N) * K);
  for (long i = 0; i < M * K; ++i) ha[i] = static_cast<float>((i * 2654435761u) % 2001) / 1000.f - 1.f;
  for (long i = 0; i < static_cast<long>(N) * K; ++i) hb[i] = static_cast<float>((i * 40503u) % 2001) / 1000.f - 1.f;
  float *a, *b, *o;
  if (hipMalloc(&a, M * K * 4) != hipSuccess || hipMalloc(&b, static_cast<long>(N) * K * 4) != hipSuccess ||
      hipMalloc(&o, M * N * 4) != hipSuccess) return;
  (void)hipMemcpy(a, ha.data(), M * K * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, hb.data(), static_cast<long>(N) * K * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) as::gemm_f32(a, b, nullptr, nullptr, o, M, N, K, 0, 0);
  (void)hipEventRecord(e0, 0);
  const int n = 20;
  for (int i = 0; i < n; ++i) as::gemm_f32(a, b, nullptr, nullptr, o, M, N, K, 0, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = 1e3 * ms / n;
  std::printf("abl %d %ld %d %d us %.1f tflops %.1f\n", GF_ABL, M, N, K, us, 2.0 * M * N * K / us / 1e6);
  (void)hipFree(a);
  (void)hipFree(b);
  (void)hipFree(o);
}

int main() {
  run(100000, 256, 256);
  run(100000, 768, 256);
  run(100000, 256, 1024);
  return 0;
}
