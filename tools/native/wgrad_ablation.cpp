// Timing ablation of the split-R weight-gradient kernel on the ResBlock conv shape (dW of a 3x3 conv over
// 390 x 19 x 20 pixels, 128 -> 128 channels: R = 148200, N = 128, K = 1152) and on a dense [148200 x 128]
// pair.  Built once per WG_ABL value (see wgrad.hip); prints "abl form us tflops".
#include "../../applestar_amd/csrc/kernels/wgrad.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

static void run(bool conv, int S_override) {
  const int B = 390, H = 19, W = 20, C = 128, N = 128;
  const long R = static_cast<long>(B) * H * W;
  const int K = conv ? 9 * C : C;
  std::vector<uint16_t> hy(R * N), hx(R * C);
  for (long i = 0; i < R * N; ++i) hy[i] = 0x3f80 ^ static_cast<uint16_t>((i * 2654435761u) & 0x807f);
  for (long i = 0; i < R * C; ++i) hx[i] = 0x3c00 ^ static_cast<uint16_t>((i * 40503u) & 0x807f);
  void *dy, *x;
  float *part, *db;
  const int S = S_override > 0 ? S_override : as::wgrad_splits(R, N, K);
  if (hipMalloc(&dy, R * N * 2) != hipSuccess || hipMalloc(&x, R * C * 2) != hipSuccess ||
      hipMalloc(&part, static_cast<size_t>(S) * N * K * 4 + N * 4) != hipSuccess ||
      hipMalloc(&db, static_cast<size_t>(S) * N * K * 4) != hipSuccess) return;
  (void)hipMemcpy(dy, hy.data(), R * N * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(x, hx.data(), R * C * 2, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipMemset(part, 0, static_cast<size_t>(S) * N * K * 4 + N * 4);
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const long ps = static_cast<long>(N) * K;
  for (int i = 0; i < 5; ++i) as::wgrad(dy, x, part, db, ps, R, N, K, H, W, conv ? C : 0, S, 0, false);
  (void)hipEventRecord(a, 0);
  const int n = 40;
  for (int i = 0; i < n; ++i) as::wgrad(dy, x, part, db, ps, R, N, K, H, W, conv ? C : 0, S, 0, false);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = 1e3 * ms / n, flop = 2.0 * R * N * K;
  std::printf("abl %d %s S=%d us %.1f tflops %.1f\n", WG_ABL, conv ? "conv" : "dense", S, us, flop / us / 1e6);
  (void)hipFree(dy);
  (void)hipFree(x);
  (void)hipFree(part);
  (void)hipFree(db);
}

int main(int argc, char** argv) {
  if (argc > 1) {                       // explicit slice counts: conv form only
    for (int i = 1; i < argc; ++i) run(true, std::atoi(argv[i]));
    return 0;
  }
  run(true, 0);
  run(false, 0);
  return 0;
}
