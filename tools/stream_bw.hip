// Read-bandwidth microbenchmark for the probe sweep's access patterns (measurement tool, not
// part of the library).  Reads a T x N fp32 matrix once per launch and writes one float per
// thread (sum), for several workgroup tilings:
//   linear : grid-stride float4 over the flat array
//   tile   : workgroup = TT rows x 512 columns, wave = 64 columns x TT rows, 4 rows x 256 B per
//            wave-instruction, two 16-row blocks in flight (the sweep kernel's pattern)
//   rows   : workgroup = 16 rows x all N columns, wave = 2 rows (full 16-KB rows)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/stream_bw tools/stream_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void linear_kernel(const f32x4* __restrict__ x, int64_t n4, float* out) {
  f32x4 s{0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) s += x[i];
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <int DEPTH, bool STRIPE_MAJOR = false>
__global__ __launch_bounds__(512) void tile_kernel(const float* __restrict__ x, int64_t T, int64_t N, int TT,
                                                   float* out) {
  const int nct = (int)(N / 512);
  const int nrt = (int)(T / TT);
  // row-major order: consecutive workgroups = adjacent stripes of the same rows;
  // stripe-major: consecutive workgroups = consecutive row tiles of one stripe
  const int rt = STRIPE_MAJOR ? blockIdx.x % nrt : blockIdx.x / nct;
  const int ct = STRIPE_MAJOR ? blockIdx.x / nrt : blockIdx.x % nct;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  const int64_t col = (int64_t)ct * 512 + 64 * wave + 4 * li;
  const int64_t t0 = (int64_t)rt * TT;
  const int NI = TT / 16;
  f32x4 s{0, 0, 0, 0};
  f32x4 z[DEPTH][4];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
#pragma unroll
    for (int p = 0; p < 4; ++p)
      z[d][p] = *reinterpret_cast<const f32x4*>(x + (t0 + 16 * d + 4 * p + g) * N + col);
  for (int i = 0; i < NI; i += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int p = 0; p < 4; ++p) s += z[d][p];
      int blk = i + d + DEPTH;
      blk = blk < NI ? blk : NI - 1;
#pragma unroll
      for (int p = 0; p < 4; ++p) z[d][p] = *reinterpret_cast<const f32x4*>(x + (t0 + 16 * blk + 4 * p + g) * N + col);
    }
  }
  out[(int64_t)blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(512) void rows_kernel(const float* __restrict__ x, int64_t T, int64_t N, float* out) {
  // workgroup: 16 rows; wave: 2 rows, each lane 16 B per 1 KB step along the row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 16 + 2 * wave;
  f32x4 s{0, 0, 0, 0};
  for (int rr = 0; rr < 2; ++rr) {
    const float* row = x + (r0 + rr) * N;
    for (int64_t c = 4 * lane; c < N; c += 4 * 64 * 4) {
      f32x4 a = *reinterpret_cast<const f32x4*>(row + c);
      f32x4 b = (c + 256 < N) ? *reinterpret_cast<const f32x4*>(row + c + 256) : f32x4{0, 0, 0, 0};
      f32x4 cc = (c + 512 < N) ? *reinterpret_cast<const f32x4*>(row + c + 512) : f32x4{0, 0, 0, 0};
      f32x4 dd = (c + 768 < N) ? *reinterpret_cast<const f32x4*>(row + c + 768) : f32x4{0, 0, 0, 0};
      s += a + b + cc + dd;
    }
  }
  out[(int64_t)blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int64_t T = 1024, N = 4096;
  const int nmat = argc > 1 ? atoi(argv[1]) : 48;  // 48 x 16 MB = 768 MB: beyond the 256 MB MALL
  std::vector<float*> mats(nmat);
  for (auto& m : mats) {
    CK(hipMalloc(&m, T * N * 4));
    CK(hipMemset(m, 0, T * N * 4));
  }
  float* out;
  CK(hipMalloc(&out, 64 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w)
      for (int m = 0; m < nmat; ++m) launch(mats[m]);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    const int reps = 3;
    for (int rep = 0; rep < reps; ++rep)
      for (int m = 0; m < nmat; ++m) launch(mats[m]);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double bytes = (double)reps * nmat * T * N * 4;
    printf("%-28s %8.2f us/matrix  %7.0f GB/s\n", name, 1e3 * ms / (reps * nmat), bytes / (ms * 1e-3) / 1e9);
  };
  for (int grid : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "linear grid=%d", grid);
    run(nm, [&](float* m) { hipLaunchKernelGGL(linear_kernel, dim3(grid), dim3(256), 0, 0, (const f32x4*)m, T * N / 4, out); });
  }
  for (int TT : {64, 128, 256, 512}) {
    char nm[64];
    snprintf(nm, sizeof nm, "tile TT=%d depth2", TT);
    const int nwg = (int)((T / TT) * (N / 512));
    run(nm, [&](float* m) { hipLaunchKernelGGL(tile_kernel<2>, dim3(nwg), dim3(512), 0, 0, m, T, N, TT, out); });
    snprintf(nm, sizeof nm, "tile TT=%d depth4", TT);
    run(nm, [&](float* m) { hipLaunchKernelGGL(tile_kernel<4>, dim3(nwg), dim3(512), 0, 0, m, T, N, TT, out); });
  }
  run("rows 16/wg", [&](float* m) { hipLaunchKernelGGL(rows_kernel, dim3((unsigned)(T / 16)), dim3(512), 0, 0, m, T, N, out); });
  // one 768 MB launch (48 stacked matrices): the streaming rate without per-launch ramp/tail
  float* big;
  CK(hipMalloc(&big, 48 * T * N * 4));
  CK(hipMemset(big, 0, 48 * T * N * 4));
  for (int TT : {128, 256}) {
    const int nwg = (int)((48 * T / TT) * (N / 512));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(tile_kernel<2>, dim3(nwg), dim3(512), 0, 0, big, 48 * T, N, TT, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int rep = 0; rep < 10; ++rep)
      hipLaunchKernelGGL(tile_kernel<2>, dim3(nwg), dim3(512), 0, 0, big, 48 * T, N, TT, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("tile 768MB-launch TT=%-4d     %8.2f us/launch  %7.0f GB/s\n", TT, 1e3 * ms / 10,
           10.0 * 48 * T * N * 4 / (ms * 1e-3) / 1e9);
  }
  // occupancy limited to 2 (or 1) 512-thread workgroups per CU by dynamic LDS, as in the sweep kernels
  for (int lds : {56 << 10, 96 << 10}) {
    for (int depth : {2, 4}) {
      const int TT = 128;
      const int nwg = (int)((48 * T / TT) * (N / 512));
      auto go = [&] {
        if (depth == 2) hipLaunchKernelGGL(tile_kernel<2>, dim3(nwg), dim3(512), lds, 0, big, 48 * T, N, TT, out);
        else hipLaunchKernelGGL(tile_kernel<4>, dim3(nwg), dim3(512), lds, 0, big, 48 * T, N, TT, out);
      };
      for (int w = 0; w < 3; ++w) go();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, 0));
      for (int rep = 0; rep < 10; ++rep) go();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("tile TT=128 depth%d lds=%dK    %8.2f us/launch  %7.0f GB/s\n", depth, lds >> 10, 1e3 * ms / 10,
             10.0 * 48 * T * N * 4 / (ms * 1e-3) / 1e9);
    }
  }
  // launch size: the first 14 matrices of the stack (224 MB, one sweep phase of a 14-module group)
  for (int nm : {14, 28}) {
    const int TT = 128;
    const int nwg = (int)((nm * T / TT) * (N / 512));
    auto go = [&] { hipLaunchKernelGGL((tile_kernel<2, false>), dim3(nwg), dim3(512), 0, 0, big, nm * T, N, TT, out); };
    for (int w = 0; w < 3; ++w) go();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int rep = 0; rep < 10; ++rep) go();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("tile %3d MB launch TT=128    %8.2f us/launch  %7.0f GB/s\n", nm * 16, 1e3 * ms / 10,
           10.0 * nm * T * N * 4 / (ms * 1e-3) / 1e9);
  }
  // stripe-major order on 16 MB matrices stacked 48 deep (one launch): each stripe is 48 K rows tall
  for (int TT : {128, 256}) {
    const int nwg = (int)((48 * T / TT) * (N / 512));
    auto go = [&] { hipLaunchKernelGGL((tile_kernel<2, true>), dim3(nwg), dim3(512), 0, 0, big, 48 * T, N, TT, out); };
    for (int w = 0; w < 3; ++w) go();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int rep = 0; rep < 10; ++rep) go();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("tile stripe-major TT=%-4d     %8.2f us/launch  %7.0f GB/s\n", TT, 1e3 * ms / 10,
           10.0 * 48 * T * N * 4 / (ms * 1e-3) / 1e9);
  }
  {
    const int64_t n4 = 48 * T * N / 4;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(linear_kernel, dim3(8192), dim3(256), 0, 0, (const f32x4*)big, n4, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int rep = 0; rep < 10; ++rep)
      hipLaunchKernelGGL(linear_kernel, dim3(8192), dim3(256), 0, 0, (const f32x4*)big, n4, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("linear 768MB-launch           %8.2f us/launch  %7.0f GB/s\n", 1e3 * ms / 10,
           10.0 * 48 * T * N * 4 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
