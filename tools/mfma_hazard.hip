// Measurement tool (not part of the library): how many wait states gfx950 needs between an MFMA and a
// vector-memory read of its result.  For each MFMA form and pad N, every lane stores the accumulator
// registers with `global_store_dwordx4` N + 1 wait states after the MFMA issued (one asm block: no
// compiler padding), and the stored values are compared with the same MFMA read after 2 x 16 wait states.
// Prints, per form, the mismatching lanes per pad.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_hazard.hip -o tools/bin/mfma_hazard && tools/bin/mfma_hazard
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

// N = pad (s_nop N gives N + 1 wait states; the store itself issues after them).  Two stores of the
// 16x16 result: at the pad and after 32 more wait states (the reference).
#define PAD_16(N)                                                                                         \
  template <int F>                                                                                         \
  __global__ void k16_##N(const float* in, float* out, float* ref) {                                      \
    const int l = threadIdx.x, w = blockIdx.x;                                                            \
    const float* p = in + (w * 64 + l) * 8;                                                               \
    f32x4 acc;                                                                                             \
    float* o = out + (w * 64 + l) * 4;                                                                     \
    float* r = ref + (w * 64 + l) * 4;                                                                     \
    if constexpr (F == 0) {                                                                                \
      bf16x8 a, b;                                                                                         \
      for (int e = 0; e < 8; ++e) { a[e] = (__bf16)p[e]; b[e] = (__bf16)p[(e + 3) & 7]; }                  \
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0\n\ts_nop " #N                                    \
                   "\n\tglobal_store_dwordx4 %3, %0, off\n\ts_nop 15\n\ts_nop 15\n\t"                       \
                   "global_store_dwordx4 %4, %0, off\n\ts_waitcnt vmcnt(0)"                               \
                   : "=&v"(acc) : "v"(a), "v"(b), "v"(o), "v"(r) : "memory");                             \
    } else if constexpr (F == 1) {                                                                         \
      bf16x4 a, b;                                                                                         \
      for (int e = 0; e < 4; ++e) { a[e] = (__bf16)p[e]; b[e] = (__bf16)p[4 + e]; }                        \
      asm volatile("v_mfma_f32_16x16x16_bf16 %0, %1, %2, 0\n\ts_nop " #N                                    \
                   "\n\tglobal_store_dwordx4 %3, %0, off\n\ts_nop 15\n\ts_nop 15\n\t"                       \
                   "global_store_dwordx4 %4, %0, off\n\ts_waitcnt vmcnt(0)"                               \
                   : "=&v"(acc) : "v"(a), "v"(b), "v"(o), "v"(r) : "memory");                             \
    } else {                                                                                               \
      const float a = p[0], b = p[1];                                                                      \
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0\n\ts_nop " #N                                      \
                   "\n\tglobal_store_dwordx4 %3, %0, off\n\ts_nop 15\n\ts_nop 15\n\t"                       \
                   "global_store_dwordx4 %4, %0, off\n\ts_waitcnt vmcnt(0)"                               \
                   : "=&v"(acc) : "v"(a), "v"(b), "v"(o), "v"(r) : "memory");                             \
    }                                                                                                      \
  }

PAD_16(0)
PAD_16(2)
PAD_16(4)
PAD_16(5)
PAD_16(6)
PAD_16(7)
PAD_16(8)
PAD_16(9)
PAD_16(10)
PAD_16(11)
PAD_16(12)
PAD_16(13)
PAD_16(14)
PAD_16(15)

// explicit registers (v40..v55, clobbered): RAW of the first four result registers of a 32x32 form,
// and WAW: a VALU write of the first result register N + 1 wait states after the MFMA (the stored value
// must be the VALU's, 1.0, unless the MFMA's write lands after it)
#define PAD_XG(TAG, NOPS)                                                                                          \
  template <int F>                                                                                         \
  __global__ void kx_##TAG(const float* in, float* out, float* ref) {                                       \
    const int l = threadIdx.x, w = blockIdx.x;                                                            \
    const float* p = in + (w * 64 + l) * 8;                                                               \
    float* o = out + (w * 64 + l) * 4;                                                                     \
    float* r = ref + (w * 64 + l) * 4;                                                                     \
    bf16x8 a, b;                                                                                           \
    for (int e = 0; e < 8; ++e) { a[e] = (__bf16)p[e]; b[e] = (__bf16)p[(e + 5) & 7]; }                    \
    if constexpr (F == 0) {                                                                                \
      asm volatile("v_mfma_f32_32x32x16_bf16 v[40:55], %0, %1, 0\n\t" NOPS                            \
                   "\n\tglobal_store_dwordx4 %2, v[40:43], off\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"  \
                   "global_store_dwordx4 %3, v[40:43], off\n\ts_waitcnt vmcnt(0)"                         \
                   :: "v"(a), "v"(b), "v"(o), "v"(r)                                                       \
                   : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",     \
                     "v49", "v50", "v51", "v52", "v53", "v54", "v55");                               \
    } else if constexpr (F == 1) {                                                                         \
      asm volatile("v_mfma_f32_32x32x16_bf16 v[40:55], %0, %1, 0\n\t" NOPS                            \
                   "\n\tv_mov_b32 v40, 1.0\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"                         \
                   "global_store_dwordx4 %2, v[40:43], off\n\ts_waitcnt vmcnt(0)"                         \
                   :: "v"(a), "v"(b), "v"(o), "v"(r)                                                       \
                   : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",     \
                     "v49", "v50", "v51", "v52", "v53", "v54", "v55");                               \
      if (l == 0 && w == 0) r[0] = 0.f;                                                                    \
    } else if constexpr (F == 3) {                                                                         \
      asm volatile("v_mfma_f32_32x32x16_bf16 v[40:55], %0, %1, 0\n\t" NOPS                                    \
                   "\n\tglobal_store_dwordx4 %2, v[52:55], off\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"  \
                   "global_store_dwordx4 %3, v[52:55], off\n\ts_waitcnt vmcnt(0)"                         \
                   :: "v"(a), "v"(b), "v"(o), "v"(r)                                                       \
                   : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",     \
                     "v49", "v50", "v51", "v52", "v53", "v54", "v55");                               \
    } else if constexpr (F == 4 || F == 5) {                                                               \
      const float fa = p[0], fb = p[1];                                                                    \
      if constexpr (F == 4)                                                                                \
        asm volatile("v_mfma_f32_32x32x2_f32 v[40:55], %0, %1, 0\n\t" NOPS                                 \
                     "\n\tglobal_store_dwordx4 %2, v[40:43], off\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t" \
                     "global_store_dwordx4 %3, v[40:43], off\n\ts_waitcnt vmcnt(0)"                       \
                     :: "v"(fa), "v"(fb), "v"(o), "v"(r)                                                   \
                     : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",   \
                       "v49", "v50", "v51", "v52", "v53", "v54", "v55");                             \
      else                                                                                                 \
        asm volatile("v_mfma_f32_32x32x2_f32 v[40:55], %0, %1, 0\n\t" NOPS                                 \
                     "\n\tglobal_store_dwordx4 %2, v[52:55], off\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t" \
                     "global_store_dwordx4 %3, v[52:55], off\n\ts_waitcnt vmcnt(0)"                       \
                     :: "v"(fa), "v"(fb), "v"(o), "v"(r)                                                   \
                     : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",   \
                       "v49", "v50", "v51", "v52", "v53", "v54", "v55");                             \
    } else {                                                                                               \
      asm volatile("v_mfma_f32_16x16x32_bf16 v[40:43], %0, %1, 0\n\t" NOPS                            \
                   "\n\tv_mov_b32 v40, 1.0\n\ts_nop 15\n\ts_nop 15\n\t"                                     \
                   "global_store_dwordx4 %2, v[40:43], off\n\ts_waitcnt vmcnt(0)"                         \
                   :: "v"(a), "v"(b), "v"(o), "v"(r) : "memory", "v40", "v41", "v42", "v43");         \
    }                                                                                                      \
  }
PAD_XG(0, "s_nop 0")
PAD_XG(2, "s_nop 2")
PAD_XG(4, "s_nop 4")
PAD_XG(6, "s_nop 6")
PAD_XG(7, "s_nop 7")
PAD_XG(8, "s_nop 8")
PAD_XG(9, "s_nop 9")
PAD_XG(10, "s_nop 10")
PAD_XG(11, "s_nop 11")
PAD_XG(12, "s_nop 12")
PAD_XG(13, "s_nop 13")
PAD_XG(14, "s_nop 14")
PAD_XG(15, "s_nop 15")
PAD_XG(17, "s_nop 15\n\ts_nop 0")
PAD_XG(19, "s_nop 15\n\ts_nop 2")
PAD_XG(21, "s_nop 15\n\ts_nop 4")
PAD_XG(23, "s_nop 15\n\ts_nop 6")


int main() {
  const int waves = 4096, n = waves * 64;
  std::vector<float> h(n * 8);
  srand(7);
  for (auto& x : h) x = (float)(rand() % 2001 - 1000) / 256.f;
  float *din, *dout, *dref;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMalloc(&dout, n * 16));
  CHECK(hipMalloc(&dref, n * 16));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> o(n * 4), r(n * 4);
  auto run = [&](void (*k)(const float*, float*, float*), const char* form, int pad, bool waw = false) {
    CHECK(hipMemset(dout, 0xff, n * 16));
    CHECK(hipMemset(dref, 0xff, n * 16));
    hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, din, dout, dref);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(o.data(), dout, n * 16, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(r.data(), dref, n * 16, hipMemcpyDeviceToHost));
    long bad = 0;
    if (waw) {
      for (int i = 0; i < n; ++i) bad += o[4 * i] != 1.0f;
    } else {
      for (int i = 0; i < n * 4; ++i) bad += o[i] != r[i];
    }
    printf("%-22s wait states %2d: %ld of %d values differ\n", form, pad + 1, bad, n * 4);
    fflush(stdout);
  };
#define R16(F, name, N) run(k16_##N<F>, name, N)
#define ALL16(F, name)                                                                                    \
  R16(F, name, 0); R16(F, name, 2); R16(F, name, 4); R16(F, name, 5); R16(F, name, 6); R16(F, name, 7);  \
  R16(F, name, 8); R16(F, name, 9); R16(F, name, 10); R16(F, name, 11); R16(F, name, 12);                 \
  R16(F, name, 13); R16(F, name, 14); R16(F, name, 15)
  ALL16(0, "16x16x32_bf16");
  ALL16(1, "16x16x16_bf16");
  ALL16(2, "16x16x4_f32");
#define RX(F, name, N, waw) run(kx_##N<F>, name, N, waw)
#define ALLX(F, name, waw)                                                                                \
  RX(F, name, 0, waw); RX(F, name, 2, waw); RX(F, name, 4, waw); RX(F, name, 6, waw); RX(F, name, 7, waw); \
  RX(F, name, 8, waw); RX(F, name, 9, waw); RX(F, name, 10, waw); RX(F, name, 11, waw);                    \
  RX(F, name, 12, waw); RX(F, name, 13, waw); RX(F, name, 14, waw); RX(F, name, 15, waw);                  \
  RX(F, name, 17, waw); RX(F, name, 19, waw); RX(F, name, 21, waw); RX(F, name, 23, waw)
  ALLX(0, "32x32x16_bf16 RAW", false);
  ALLX(1, "32x32x16_bf16 WAW", true);
  ALLX(2, "16x16x32_bf16 WAW", true);
  ALLX(3, "32x32x16_bf16 RAW r12", false);
  ALLX(4, "32x32x2_f32 RAW r0", false);
  ALLX(5, "32x32x2_f32 RAW r12", false);
  return 0;
}
