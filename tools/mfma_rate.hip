// Measurement tool: bf16 MFMA issue rate on gfx950 for the shapes the K2 / K4 kernels use
// (16x16x16 bf16 "_1k" -- the K2 r = 64 split path --, 16x16x32 bf16, 32x32x16 bf16, 16x16x4 f32).
// Every CU runs 4 waves (one per SIMD), each a chain of independent accumulators on random data.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o tools/bin/mfma_rate && tools/bin/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 4096;
constexpr int kAcc = 8;

template <int KIND>
__global__ __launch_bounds__(256) void mfma_loop(float* out, float seed) {
  f32x4 acc[kAcc];
  f32x16 acc32[2];
  for (int i = 0; i < kAcc; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc32[0] = acc32[1] = f32x16{};
  const float v = seed + threadIdx.x * 1e-3f;
  bf16x4 a4, b4;
  bf16x8 a8, b8;
  for (int e = 0; e < 4; ++e) {
    a4[e] = (short)(0x3f80 + threadIdx.x + e);
    b4[e] = (short)(0x3f00 + threadIdx.x * 3 + e);
  }
  for (int e = 0; e < 8; ++e) {
    a8[e] = (__bf16)(v + e);
    b8[e] = (__bf16)(v - e);
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < kAcc; ++i) {
      if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[i], 0, 0, 0);
      if constexpr (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[i], 0, 0, 0);
      if constexpr (KIND == 2) acc32[i & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, acc32[i & 1], 0, 0, 0);
      if constexpr (KIND == 3) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v * 0.5f, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < kAcc; ++i) s += acc[i][0] + acc[i][3];
  s += acc32[0][0] + acc32[1][5];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
static void run(const char* name, double flop_per_mfma) {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out = nullptr;
  hipMalloc(&out, (size_t)cus * 256 * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(mfma_loop<KIND>, dim3(cus), dim3(256), 0, 0, out, 1.0f);
  hipEventRecord(a);
  const int reps = 20;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mfma_loop<KIND>, dim3(cus), dim3(256), 0, 0, out, 1.0f + r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double mfmas = (double)reps * cus * 4 /*waves*/ * kIters * kAcc;
  const double tf = mfmas * flop_per_mfma / (ms * 1e-3) / 1e12;
  // cycles per MFMA per SIMD at the clock the loop held: unknown here, so report TF/s and the
  // SIMD-cycle count implied at 2.4 GHz
  const double cyc = (ms * 1e-3) * 2.4e9 / ((double)reps * kIters * kAcc);
  printf("%-26s %8.1f TFLOP/s   ~%5.1f cyc/MFMA/SIMD at 2.4 GHz\n", name, tf, cyc);
  hipFree(out);
}

int main() {
  run<0>("16x16x16 bf16 (_1k)", 2.0 * 16 * 16 * 16);
  run<1>("16x16x32 bf16", 2.0 * 16 * 16 * 32);
  run<2>("32x32x16 bf16", 2.0 * 32 * 32 * 16);
  run<3>("16x16x4 f32", 2.0 * 16 * 16 * 4);
  return 0;
}
