// Read-modify-write bandwidth microbenchmark for K4's merge epilogue (measurement tool, not
// part of the library): W[i] += c over a 1.6 GB float32 buffer with
//   acc   : the K4 accumulator layout -- per 64x64 wave tile, 64 dword loads + 64 dword stores per
//           lane (register e of block (bo, bc) = row (e&3) + 8(e>>2) + 4h + 32bo, column l32 + 32bc),
//           through a buffer descriptor, as delta_group_kernel's epilogue does
//   vec4  : the same tiles, row-major float4 per lane (4 rows x 256 B per wave-instruction)
// Both persistent over the tiles (grid = 512 workgroups of 256 threads, 4 waves x 64x64).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/rmw_bw tools/rmw_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(256, 2) void rmw_acc(float* W, int rows, int cols, float c) {
  const int ntc = cols / 128, ntr = rows / 128, nt = ntr * ntc;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  auto rs = __builtin_amdgcn_make_buffer_rsrc(W, 0, 0x7fffffff, 0x00020000);
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const int o_w = (t / ntc) * 128 + (wave >> 1) * 64, c_w = (t % ntc) * 128 + (wave & 1) * 64;
    const int voff = ((4 * h) * cols + l32) * 4;
    float w[2][2][16];
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int so = ((o_w + 32 * bo + (e & 3) + 8 * (e >> 2)) * cols + c_w + 32 * bc) * 4;
          w[bo][bc][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, so, AUX));
        }
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int so = ((o_w + 32 * bo + (e & 3) + 8 * (e >> 2)) * cols + c_w + 32 * bc) * 4;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w[bo][bc][e] + c), rs, voff, so, AUX);
        }
  }
}

__global__ __launch_bounds__(256, 2) void rmw_vec4(float* W, int rows, int cols, float c) {
  const int ntc = cols / 128, ntr = rows / 128, nt = ntr * ntc;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const int o_w = (t / ntc) * 128 + (wave >> 1) * 64, c_w = (t % ntc) * 128 + (wave & 1) * 64;
    f32x4 w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // 64 rows x 64 cols: lane -> row 4k + (lane >> 4), col 4 (lane & 15)
      const int64_t idx = (int64_t)(o_w + 4 * k + (lane >> 4)) * cols + c_w + 4 * (lane & 15);
      w[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(W + idx));
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int64_t idx = (int64_t)(o_w + 4 * k + (lane >> 4)) * cols + c_w + 4 * (lane & 15);
      __builtin_nontemporal_store(w[k] + c, reinterpret_cast<f32x4*>(W + idx));
    }
  }
}

int main() {
  const int rows = 11008 * 8, cols = 4096;  // 1.44 GB
  float* W;
  if (hipMalloc(&W, (size_t)rows * cols * 4) != hipSuccess) return 1;
  (void)hipMemset(W, 0, (size_t)rows * cols * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const double bytes = 2.0 * rows * (double)cols * 4;
  for (int grid : {512, 1024}) {
    for (int v = 0; v < 3; ++v) {
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        for (int i = 0; i < 5; ++i) {
          if (v == 0) hipLaunchKernelGGL(rmw_acc<0>, dim3(grid), dim3(256), 0, 0, W, rows, cols, 1.f);
          if (v == 1) hipLaunchKernelGGL(rmw_acc<2>, dim3(grid), dim3(256), 0, 0, W, rows, cols, 1.f);
          if (v == 2) hipLaunchKernelGGL(rmw_vec4, dim3(grid), dim3(256), 0, 0, W, rows, cols, 1.f);
        }
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep == 1)
          printf("%-12s grid=%5d  %8.3f ms  %7.0f GB/s\n", v == 0 ? "acc" : v == 1 ? "acc-nt" : "vec4-nt", grid, ms / 5,
                 bytes / (ms / 5 * 1e-3) / 1e9);
      }
    }
  }
  return 0;
}
