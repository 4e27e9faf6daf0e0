// Measurement tool (not part of the library): calibrates rocprofv3's FETCH_SIZE for the load widths the
// kernels use.  Each kernel streams the same 1 GiB buffer once, every lane reading W bytes per load at
// consecutive addresses (W = 4, 8, 16) and the sum goes to a sink so nothing is elided; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/bin/fetch_calib
// and compare FETCH_SIZE (KiB) x 1024 with the 1 GiB each kernel reads.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

template <class V>
__global__ void stream_kernel(const V* __restrict__ p, size_t n, float* sink) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const V v = __builtin_nontemporal_load(p + i);
    if constexpr (sizeof(V) == 4) acc += v;
    else if constexpr (sizeof(V) == 8) acc += v[0] + v[1];
    else acc += v[0] + v[1] + v[2] + v[3];
  }
  if (acc == 12345.678f) sink[0] = acc;  // practically never: keeps the loads
}

int main() {
  const size_t bytes = 1ull << 30;
  void* buf;
  float* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(buf, 0, bytes));
  const dim3 grid(256 * 8), block(256);
  hipLaunchKernelGGL(stream_kernel<float>, grid, block, 0, 0, (const float*)buf, bytes / 4, sink);
  hipLaunchKernelGGL(stream_kernel<f32x2>, grid, block, 0, 0, (const f32x2*)buf, bytes / 8, sink);
  hipLaunchKernelGGL(stream_kernel<f32x4>, grid, block, 0, 0, (const f32x4*)buf, bytes / 16, sink);
  CHECK(hipDeviceSynchronize());
  printf("streamed 1 GiB with 4-, 8- and 16-byte loads per lane (kernels in that order)\n");
  return 0;
}
