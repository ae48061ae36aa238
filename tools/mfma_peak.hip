// Achievable MFMA throughput on this MI355X (the speed of light the fp32 / bf16 kernels are judged against):
// register-only MFMA streams - 8 independent accumulators per wave, no memory traffic in the loop - over a
// grid of 256 CUs x {1, 2, 4} waves per SIMD, timed with HIP events.  Compares the measured rate with the
// nominal dense peak (2.4 GHz x 256 CUs x 4 SIMDs x flops/cycle) to expose clock throttling under load.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_peak tools/mfma_peak.hip && /tmp/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(16))) float f16v;
typedef __attribute__((ext_vector_type(4))) float f4v;
typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

// flops per MFMA: 32x32x2 f32 = 4096, 16x16x4 f32 = 2048, 32x32x16 bf16 = 32768, 16x16x32 bf16 = 16384
__global__ __launch_bounds__(256) void k_f32_32x32x2(float* out, int iters, float s) {
  f16v acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  float a = s * threadIdx.x, b = s + threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
  float t = 0.f;
  for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_f32_16x16x4(float* out, int iters, float s) {
  f4v acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 4; ++e) acc[j][e] = 0.f;
  float a = s * threadIdx.x, b = s + threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
  float t = 0.f;
  for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_bf16_32x32x16(float* out, int iters, float s) {
  f16v acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  bf8v a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = static_cast<__bf16>(s * (threadIdx.x + e));
    b[e] = static_cast<__bf16>(s - e);
  }
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
  float t = 0.f;
  for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_bf16_16x16x32(float* out, int iters, float s) {
  f4v acc[8];
  for (int j = 0; j < 8; ++j)
    for (int e = 0; e < 4; ++e) acc[j][e] = 0.f;
  bf8v a, b;
  for (int e = 0; e < 8; ++e) {
    a[e] = static_cast<__bf16>(s * (threadIdx.x + e));
    b[e] = static_cast<__bf16>(s - e);
  }
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
  float t = 0.f;
  for (int j = 0; j < 8; ++j) t += acc[j][0] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

typedef void (*Kern)(float*, int, float);

int run(const char* name, Kern k, double flops_per_mfma, double nominal_per_cu_clk, float* out, int cus) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int wps : {1, 2, 4}) {           // waves per SIMD: 256-thread blocks = 1 wave per SIMD each
    const int blocks = cus * wps;
    int iters = 2000;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 50, 1.f);   // warm-up
    CHECK(hipDeviceSynchronize());
    float ms = 0.f;
    for (;;) {                           // grow until the run takes >= 20 ms (bounded: iters <= 2^24)
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (ms >= 20.f || iters >= (1 << 24)) break;
      iters *= 4;
    }
    const double mfmas = static_cast<double>(blocks) * 4 /* waves */ * iters * 8;
    const double tf = mfmas * flops_per_mfma / (ms * 1e-3) / 1e12;
    const double nominal = nominal_per_cu_clk * cus * 2.4e9 / 1e12;
    std::printf("{\"mfma\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.2f, \"tflops\": %.1f, \"nominal_tflops\": %.1f, "
                "\"pct_nominal\": %.1f, \"implied_mfma_clock_ghz\": %.2f}\n",
                name, wps, ms, tf, nominal, 100.0 * tf / nominal, 2.4 * tf / nominal);
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float* out;
  CHECK(hipMalloc(&out, sizeof(float) * 256 * cus * 4));
  // nominal flops / CU / clock: 4 SIMDs x (flops per MFMA / cycles per MFMA)
  if (run("f32_32x32x2", k_f32_32x32x2, 4096, 4 * 4096.0 / 64, out, cus)) return 1;
  if (run("f32_16x16x4", k_f32_16x16x4, 2048, 4 * 2048.0 / 32, out, cus)) return 1;
  if (run("bf16_32x32x16", k_bf16_32x32x16, 32768, 4 * 32768.0 / 32, out, cus)) return 1;
  if (run("bf16_16x16x32", k_bf16_16x16x32, 16384, 4 * 16384.0 / 16, out, cus)) return 1;
  CHECK(hipFree(out));
  return 0;
}
