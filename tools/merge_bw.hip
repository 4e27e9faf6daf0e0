// K5 merge (W += dW, float32) bandwidth variants (measurement tool, not part of the library).
// 12 B per element over a buffer far beyond the 256 MB Infinity Cache; reports TB/s of the
// algorithmic bytes for: grid-stride with U vectors in flight per lane (the shipped form is U = 2,
// 2048 workgroups), and contiguous per-workgroup chunks.
//   hipcc --offload-arch=gfx950 -O3 tools/merge_bw.hip -o tools/bin/merge_bw && tools/bin/merge_bw
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define G1 __attribute__((address_space(1)))

template <int U, bool NT>
__global__ __launch_bounds__(256) void stride_kernel(float* W, const float* dW, long n4) {
  G1 f32x4* W4 = (G1 f32x4*)W;
  const G1 f32x4* D4 = (const G1 f32x4*)dW;
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f32x4 d[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d[u] = NT ? __builtin_nontemporal_load(D4 + i + u * stride) : D4[i + u * stride];
      w[u] = NT ? __builtin_nontemporal_load(W4 + i + u * stride) : W4[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(w[u] + d[u], W4 + i + u * stride);
      else W4[i + u * stride] = w[u] + d[u];
    }
  }
  for (; i < n4; i += stride) W4[i] = W4[i] + D4[i];
}

// each workgroup owns contiguous chunks of 256 * U vectors (U * 4 KB of W per chunk)
template <int U, bool NT>
__global__ __launch_bounds__(256) void chunk_kernel(float* W, const float* dW, long n4) {
  G1 f32x4* W4 = (G1 f32x4*)W;
  const G1 f32x4* D4 = (const G1 f32x4*)dW;
  const long chunk = 256L * U;
  for (long c = (long)blockIdx.x * chunk; c < n4; c += (long)gridDim.x * chunk) {
    f32x4 d[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = c + u * 256 + threadIdx.x;
      if (i < n4) {
        d[u] = NT ? __builtin_nontemporal_load(D4 + i) : D4[i];
        w[u] = NT ? __builtin_nontemporal_load(W4 + i) : W4[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = c + u * 256 + threadIdx.x;
      if (i < n4) {
        if (NT) __builtin_nontemporal_store(w[u] + d[u], W4 + i);
        else W4[i] = w[u] + d[u];
      }
    }
  }
}

template <class K>
static void run(const char* name, K kern, int grid, float* W, const float* dW, long n4) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, W, dW, n4);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, W, dW, n4);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double tbs = 12.0 * 4 * n4 * reps / (ms * 1e-3) / 1e12;
  printf("%-34s grid %5d  %6.3f ms  %5.2f TB/s  (%.3f of 8)\n", name, grid, ms / reps, tbs, tbs / 8.0);
}

int main() {
  const long n = 256L << 20;  // 1 GiB of W, 1 GiB of dW
  float *W = nullptr, *dW = nullptr;
  (void)hipMalloc(&W, n * 4);
  (void)hipMalloc(&dW, n * 4);
  (void)hipMemset(W, 0, n * 4);
  (void)hipMemset(dW, 0, n * 4);
  const long n4 = n / 4;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run("stride U2 nt (shipped)", stride_kernel<2, true>, 2048, W, dW, n4);
  run("stride U2 plain", stride_kernel<2, false>, 2048, W, dW, n4);
  run("stride U4 nt", stride_kernel<4, true>, 2048, W, dW, n4);
  run("stride U4 nt", stride_kernel<4, true>, cus * 4, W, dW, n4);
  run("stride U8 nt", stride_kernel<8, true>, cus * 4, W, dW, n4);
  run("stride U4 plain", stride_kernel<4, false>, cus * 4, W, dW, n4);
  run("chunk U4 nt", chunk_kernel<4, true>, cus * 8, W, dW, n4);
  run("chunk U8 nt", chunk_kernel<8, true>, cus * 4, W, dW, n4);
  run("chunk U8 nt", chunk_kernel<8, true>, cus * 8, W, dW, n4);
  run("chunk U16 nt", chunk_kernel<16, true>, cus * 4, W, dW, n4);
  run("chunk U8 plain", chunk_kernel<8, false>, cus * 8, W, dW, n4);
  return 0;
}
