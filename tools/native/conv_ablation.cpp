// Timing ablation of the halo conv3x3 kernel on the spatial-encoder ResBlock shape (390 x 19 x 20, 128 -> 128).
// Built once per HALO_ABL value (see conv3x3.hip); prints "abl us tflops".
//   hipcc --offload-arch=gfx950 -O3 -DHALO_ABL=1 -I applestar_amd/csrc tools/native/conv_ablation.cpp -o /tmp/x
#include "../../applestar_amd/csrc/kernels/conv3x3.hip"

#include <cstdio>
#include <vector>

int main() {
  const int B = 390, H = 19, W = 20, Cin = 128, Cout = 128;
  const size_t nx = static_cast<size_t>(B) * H * W * Cin, nw = static_cast<size_t>(Cout) * 9 * Cin;
  std::vector<uint16_t> hx(nx), hw(nw);
  for (size_t i = 0; i < nx; ++i) hx[i] = 0x3f80 ^ static_cast<uint16_t>((i * 2654435761u) & 0x807f);
  for (size_t i = 0; i < nw; ++i) hw[i] = 0x3c00 ^ static_cast<uint16_t>((i * 40503u) & 0x807f);
  void *x, *w, *out;
  float* bias;
  if (hipMalloc(&x, nx * 2) != hipSuccess || hipMalloc(&w, nw * 2) != hipSuccess ||
      hipMalloc(&out, static_cast<size_t>(B) * H * W * Cout * 2) != hipSuccess ||
      hipMalloc(&bias, Cout * 4) != hipSuccess) return 1;
  hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice);
  hipMemset(bias, 0, Cout * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) as::conv3x3_fwd(x, w, bias, nullptr, out, B, H, W, Cin, Cout, 1, 0);
  hipEventRecord(a, 0);
  const int n = 50;
  for (int i = 0; i < n; ++i) as::conv3x3_fwd(x, w, bias, nullptr, out, B, H, W, Cin, Cout, 1, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double us = 1e3 * ms / n, flop = 2.0 * B * H * W * Cout * 9.0 * Cin;
  std::printf("abl %d us %.1f tflops %.1f\n", HALO_ABL, us, flop / us / 1e6);
  return 0;
}
