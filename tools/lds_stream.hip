// Stripe-streaming microbenchmark for the probe sweep (measurement tool, not part of the library).
// A T x N fp32 matrix read once per launch in the sweep's geometry: persistent workgroups of 8 waves,
// each workgroup a contiguous range of 16-row steps of one 512-column stripe, each wave 64 columns.
//   reg  DEPTH : global loads into registers, DEPTH steps in flight (the shipped sweep: 2)
//   lds  DEPTH : global_load_lds_dwordx4 into a wave-private LDS ring of DEPTH 4-KB slots, consumed
//                with ds_read_b128 (no workgroup barrier: a wave reads only its own slots)
// Either form can run NM dummy v_mfma_f32_16x16x4_f32 per step and wave (the phase-B load is 32).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/lds_stream tools/lds_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define G1 __attribute__((address_space(1)))
#define L3 __attribute__((address_space(3)))

constexpr int vmcnt_imm(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }

template <int NM>
__device__ __forceinline__ void mfma_load(const f32x4 (&z)[4], f32x4 (&acc)[4]) {
#pragma unroll
  for (int m = 0; m < NM; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(z[m & 3][(m >> 2) & 3], z[(m + 1) & 3][m & 3], acc[m & 3], 0, 0, 0);
}

// steps of this workgroup: [w * U / G, (w + 1) * U / G) of U = nct * (T / 16), stripe-major
template <int DEPTH, int NM>
__global__ __launch_bounds__(512, 1) void reg_kernel(const float* __restrict__ x, int64_t T, int64_t N, float* out) {
  const int64_t S = T / 16, U = (N / 512) * S;
  const int64_t lo = (int64_t)blockIdx.x * U / gridDim.x, hi = (int64_t)(blockIdx.x + 1) * U / gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  f32x4 acc[4] = {};
  f32x4 s{0, 0, 0, 0};
  f32x4 z[DEPTH][4];
  auto addr = [&](int64_t u, int p) {
    const int64_t ct = u / S, st = u % S;
    return x + (16 * st + 4 * p + g) * N + ct * 512 + 64 * wave + 4 * li;
  };
  auto load = [&](int d, int64_t u) {
#pragma unroll
    for (int p = 0; p < 4; ++p) z[d][p] = *(const G1 f32x4*)(addr(u < hi ? u : hi - 1, p));
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, lo + d);
  for (int64_t u = lo; u < hi; u += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (u + d < hi) {
        mfma_load<NM>(z[d], acc);
#pragma unroll
        for (int p = 0; p < 4; ++p) s += z[d][p];
      }
      load(d, u + d + DEPTH);
    }
  }
  out[(int64_t)blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3] + acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

// LDS ring: slot = 16 rows x 64 floats (4 KB) per wave, row-major with the 16-B chunk XOR-swizzled by
// the row (chunk' = chunk ^ row): fragment reads of one chunk across 16 rows and reads of 16 chunks of
// one row are both conflict-free
template <int DEPTH, int NM>
__global__ __launch_bounds__(512, 1) void lds_kernel(const float* __restrict__ x, int64_t T, int64_t N, float* out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int64_t S = T / 16, U = (N / 512) * S;
  const int64_t lo = (int64_t)blockIdx.x * U / gridDim.x, hi = (int64_t)(blockIdx.x + 1) * U / gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  float* ring = lds + wave * DEPTH * 1024;
  f32x4 acc[4] = {};
  f32x4 s{0, 0, 0, 0};
  // instruction p writes rows 4p .. 4p + 3: lane (g, li) -> LDS slot (row 4p + g, chunk' li) holds
  // global chunk li ^ (row & 15)
  auto issue = [&](int d, int64_t u) {
    const int64_t uu = u < hi ? u : hi - 1;
    const int64_t ct = uu / S, st = uu % S;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int row = 4 * p + g;
      const float* src = x + (16 * st + row) * N + ct * 512 + 64 * wave + 4 * (li ^ row);
      __builtin_amdgcn_global_load_lds((const G1 void*)(src), (L3 void*)(ring + d * 1024 + p * 256), 16, 0, 0);
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) issue(d, lo + d);
  for (int64_t u = lo; u < hi; u += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(4 * (DEPTH - 1)));  // slot d landed (in-order completion)
      f32x4 z[4];
      if (u + d < hi) {
        const float* sl = ring + d * 1024;
#pragma unroll
        for (int p = 0; p < 4; ++p) {  // OUTER view: row 4p + g, global chunk li
          const int row = 4 * p + g;
          z[p] = *reinterpret_cast<const f32x4*>(sl + row * 64 + 4 * (li ^ row));
        }
        mfma_load<NM>(z, acc);
#pragma unroll
        for (int p = 0; p < 4; ++p) s += z[p];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(d, u + d + DEPTH);
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
  out[(int64_t)blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3] + acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

// bf16-row geometry (the r = 64 sweep): lane (li, g) of wave w loads LB bytes of row 4 p + g at byte
// 16 LB w + LB li of the stripe (LB = 8: the shipped sweep, 4 columns; 16: 8 columns), NM dummy
// v_mfma_f32_16x16x32_bf16 per step (the phase-C load at LB = 8 is 24, at LB = 16 48)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int DEPTH, int NM, int LB>
__global__ __launch_bounds__(512, 1) void regb_kernel(const char* __restrict__ x, int64_t T, int64_t RBYTES, float* out) {
  const int64_t S = T / 16, SW = 128 * LB, U = (RBYTES / SW) * S;
  const int64_t lo = (int64_t)blockIdx.x * U / gridDim.x, hi = (int64_t)(blockIdx.x + 1) * U / gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
  f32x4 acc[4] = {};
  typedef typename std::conditional<LB == 8, u32x2, u32x4>::type V;
  V z[DEPTH][4];
  auto load = [&](int d, int64_t u) {
    u = u < hi ? u : hi - 1;
    const int64_t ct = u / S, st = u % S;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      z[d][p] = *(const G1 V*)(x + (16 * st + 4 * p + g) * RBYTES + ct * SW + LB * 16 * wave + LB * li);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, lo + d);
  for (int64_t u = lo; u < hi; u += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (u + d < hi) {
        u32x4 w;
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = z[d][k & 3][0] ^ z[d][(k + 1) & 3][1];
        const bf16x8 a = __builtin_bit_cast(bf16x8, w);
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, acc[m & 3], 0, 0, 0);
      }
      load(d, u + d + DEPTH);
    }
  }
  out[(int64_t)blockIdx.x * 512 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

template <class K>
static void run(const char* name, K kern, int grid, size_t lds, const float* x, int64_t T, int64_t N, float* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, 0, x, T, N, out);
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, 0, x, T, N, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double tbs = 4.0 * T * N * reps / (ms * 1e-3) / 1e12;
  printf("%-28s grid %4d  %7.3f ms  %5.2f TB/s\n", name, grid, ms / reps, tbs);
  fflush(stdout);
}

int main() {
  const int64_t T = 16384, N = 16384;  // 1 GiB
  float *x = nullptr, *out = nullptr;
  (void)hipMalloc(&x, 4 * T * N);
  (void)hipMalloc(&out, 4 << 20);
  (void)hipMemset(x, 0, 4 * T * N);
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipFuncSetAttribute((const void*)lds_kernel<4, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
#define R(D, NM) run("reg  depth " #D " mfma " #NM, reg_kernel<D, NM>, cus, 0, x, T, N, out)
#define L(D, NM)                                                                                         \
  do {                                                                                                   \
    (void)hipFuncSetAttribute((const void*)lds_kernel<D, NM>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              8 * D * 4096);                                                             \
    run("lds  depth " #D " mfma " #NM, lds_kernel<D, NM>, cus, 8 * D * 4096, x, T, N, out);              \
  } while (0)
#define B(D, NM, LB)                                                                                        \
  do {                                                                                                      \
    hipEvent_t a, b;                                                                                        \
    (void)hipEventCreate(&a);                                                                               \
    (void)hipEventCreate(&b);                                                                               \
    hipLaunchKernelGGL((regb_kernel<D, NM, LB>), dim3(cus), dim3(512), 0, 0, (const char*)x, T, N * 4, out);  \
    (void)hipEventRecord(a);                                                                                \
    for (int r = 0; r < 10; ++r)                                                                            \
      hipLaunchKernelGGL((regb_kernel<D, NM, LB>), dim3(cus), dim3(512), 0, 0, (const char*)x, T, N * 4, out); \
    (void)hipEventRecord(b);                                                                                \
    (void)hipEventSynchronize(b);                                                                           \
    float ms = 0.f;                                                                                         \
    (void)hipEventElapsedTime(&ms, a, b);                                                                   \
    printf("bf16 rows LB %2d depth %d mfma %2d   %7.3f ms  %5.2f TB/s\n", LB, D, NM, ms / 10,              \
           4.0 * T * N * 10 / (ms * 1e-3) / 1e12);                                                          \
    fflush(stdout);                                                                                         \
  } while (0)
  B(2, 0, 8); B(3, 0, 8); B(4, 0, 8); B(2, 24, 8); B(4, 24, 8); B(2, 0, 16); B(3, 0, 16); B(2, 48, 16); B(3, 48, 16);
  R(2, 0); R(3, 0); R(2, 32); R(3, 32); R(2, 48);
  L(2, 0); L(3, 0); L(4, 0); L(3, 32); L(4, 32); L(4, 48); L(3, 48);
  return 0;
}
