// Shared helpers for libhdpissa (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/hdpissa.h"

namespace hdp {

// ---- error reporting (host) -------------------------------------------------------------
void set_error(const char* fmt, ...);

#define HDP_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      ::hdp::set_error(__VA_ARGS__);      \
      return HDP_EINVAL;                  \
    }                                     \
  } while (0)

#define HDP_CHECK_HIP(expr)                                                            \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ::hdp::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                       __LINE__);                                                      \
      return HDP_EHIP;                                                                 \
    }                                                                                  \
  } while (0)

// HDP_SYNC_DEBUG=1: synchronise after every launch so an asynchronous fault names its kernel
bool sync_debug();
#define HDP_CHECK_LAUNCH()                                                                    \
  do {                                                                                        \
    HDP_CHECK_HIP(hipGetLastError());                                                         \
    if (::hdp::sync_debug()) HDP_CHECK_HIP(hipDeviceSynchronize());                           \
  } while (0)
#define HDP_POST_LAUNCH(st)                                                                   \
  do {                                                                                        \
    if (::hdp::sync_debug()) HDP_CHECK_HIP(hipStreamSynchronize(st));                         \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- live per-kernel timing (hdp_timing_*): HIP events bracket each launch on its stream --
enum KernelId {
  K_MERGE = 0, K_ADAM, K_DELTA, K_DELTA_MULTI, K_PROBE_P1, K_PROBE_P2, K_PROBE_FINISH, K_PROBE_REDUCE, K_SWEEP_A, K_SWEEP_B, K_SWEEP_C,
  K_SVD_GEMM, K_DELTA_PACK, K_FOLD, K_COUNT
};
bool timing_on();
void timing_record(int kid, hipEvent_t a, hipEvent_t b, double bytes, double flops);
// device-memory copy of the probe's hand-off error word (the probe sets it together with the
// host-mapped word), or null before any probe launch (hdp_probe.hip); K3 reads it stream-ordered, once
// per workgroup, and applies no update while it is set
const int* probe_err_device();
hipEvent_t timing_event();
// RAII: construct immediately before a launch, destroy right after it (one kernel per scope).
// `bytes` / `flops` = the launch's ALGORITHMIC work (every operand byte once).
struct KTimer {
  int kid;
  hipStream_t st;
  double bytes, flops;
  hipEvent_t a = nullptr;
  KTimer(int k, hipStream_t s, double by, double fl = 0.0) : kid(k), st(s), bytes(by), flops(fl) {
    if (timing_on() && (a = timing_event()) != nullptr) (void)hipEventRecord(a, st);
  }
  ~KTimer() {
    if (a == nullptr) return;
    hipEvent_t b = timing_event();
    if (b == nullptr) return;
    (void)hipEventRecord(b, st);
    timing_record(kid, a, b, bytes, flops);
  }
};

// ---- bf16 (torch's float -> bfloat16 is round-to-nearest-even, NaN -> quiet NaN) -------
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
__device__ __forceinline__ float round_bf16(float f) { return bf16_to_f32(f32_to_bf16(f)); }
// two f32 -> packed bf16 (a in the low half), round-to-nearest-even: one v_cvt_pk_bf16_f32, the bits
// f32_to_bf16 gives for every finite input
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}

// Explicit wait states between the MFMAs above and any non-MFMA access of their results below (on every
// path: the sched barriers keep the MFMAs before and the readers after the pad).  hipcc pads such reads
// itself but misses paths through a taken branch: r04 found a v_mfma_f32_16x16x32_bf16 result read 3 wait
// states after issue behind `s_cbranch_vccnz` (the r-block-1 K32 probe's wrong projections); measured
// requirements (tools/mfma_hazard.hip, profiles/r04_mfma_hazard.txt): 6 for 16x16x32 bf16, 9 for 16x16x4
// f32, 10 for 32x32x16 bf16, 18 for 32x32x2 f32.  18 here; the static scan
// tests/isa_scan.py::mfma_result_hazards checks the shipped code object.
#define HDP_MFMA_FENCE()                                           \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 1" ::: "memory");  \
    __builtin_amdgcn_sched_barrier(0);                             \
  } while (0)

// s_waitcnt immediate for vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] bits 3:0, vmcnt[5:4] bits 15:14)
constexpr int vmcnt_imm(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }

// ---- vector types -----------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// ---- global address space -----------------------------------------------------------------
// A pointer the compiler cannot prove global (one LOADED from a device descriptor table, as the
// persistent plans and the probe's group tables hold them) is generic, and generic accesses
// compile to flat_load/flat_store: those retire out of order and count in BOTH vmcnt and lgkmcnt,
// so every use of one waits vmcnt(0) lgkmcnt(0) -- all loads in flight, the prefetched steps
// included.  Every HBM access of the hot kernels goes through these casts (global_load /
// global_store, in-order vmcnt).
#define HDP_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const HDP_GLOBAL T* gptr(const T* p) {
  return (const HDP_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ HDP_GLOBAL T* gptr(T* p) {
  return (HDP_GLOBAL T*)p;
}
__device__ __forceinline__ f32x4 gld4(const float* p) { return *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(p)); }
__device__ __forceinline__ f32x4 gld4(const HDP_GLOBAL float* p) { return *reinterpret_cast<const HDP_GLOBAL f32x4*>(p); }
__device__ __forceinline__ float gld1(const float* p) { return *gptr(p); }
__device__ __forceinline__ void gst4(float* p, f32x4 v) { *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(p)) = v; }
__device__ __forceinline__ void gst1(float* p, float v) { *gptr(p) = v; }

// load 4 consecutive model-dtype elements as float (p must be 8/16-B aligned for the
// vector path; callers guarantee it on the fast path)
template <int DT>
__device__ __forceinline__ f32x4 load4(const void* p, int64_t idx);
template <>
__device__ __forceinline__ f32x4 load4<HDP_F32>(const void* p, int64_t idx) {
  return gld4(reinterpret_cast<const float*>(p) + idx);
}
template <>
__device__ __forceinline__ f32x4 load4<HDP_BF16>(const void* p, int64_t idx) {
  u16x4 h = *reinterpret_cast<const HDP_GLOBAL u16x4*>(gptr(reinterpret_cast<const uint16_t*>(p) + idx));
  return f32x4{bf16_to_f32(h[0]), bf16_to_f32(h[1]), bf16_to_f32(h[2]), bf16_to_f32(h[3])};
}
// the same with a non-temporal (streaming) hint: data read exactly once
template <int DT>
__device__ __forceinline__ f32x4 load4_nt(const void* p, int64_t idx) {
  if constexpr (DT == HDP_F32) {
    return __builtin_nontemporal_load(reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(reinterpret_cast<const float*>(p) + idx)));
  } else {
    u16x4 h = __builtin_nontemporal_load(reinterpret_cast<const HDP_GLOBAL u16x4*>(gptr(reinterpret_cast<const uint16_t*>(p) + idx)));
    return f32x4{bf16_to_f32(h[0]), bf16_to_f32(h[1]), bf16_to_f32(h[2]), bf16_to_f32(h[3])};
  }
}
template <int DT>
__device__ __forceinline__ float load1(const void* p, int64_t idx) {
  if constexpr (DT == HDP_F32) return gld1(reinterpret_cast<const float*>(p) + idx);
  else return bf16_to_f32(*gptr(reinterpret_cast<const uint16_t*>(p) + idx));
}

// bijective XCD-aware remap of a linear block id (cdna_hip_programming.md T1): blocks that
// the dispatcher deals to one XCD (id % 8 equal) get a contiguous range of tile ids.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  constexpr int NX = 8;
  if (nwg < NX) return id;
  const int q = nwg / NX, r = nwg % NX, xcd = id % NX, loc = id / NX;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + loc;
}

// ---------------------------------------------------------------------------------------
// Adam on factors (hp:356-373), shared by K3 (hdp_elementwise.hip) and K4's fused Adam + H2 pack
// (hdp_delta.hip).  Every operation is rounded separately (contract(off) on plain operators) so the
// float32 result follows torch's op-by-op evaluation.
// ---------------------------------------------------------------------------------------
struct AdamScalars {
  float grad_scale, b1, omb1, b2, omb2, bc1, bc2, lr, eps;
};

__device__ __forceinline__ void adam1(float& g, float& m, float& v, float& d, const AdamScalars& s) {
#pragma clang fp contract(off)
  // plain operators in this contract(off) scope: every product/sum rounds on its own
  const float gs = g * s.grad_scale;
  const float b1m = s.b1 * m, og = s.omb1 * gs;
  m = b1m + og;
  const float g2 = gs * gs;
  const float b2v = s.b2 * v, og2 = s.omb2 * g2;
  v = b2v + og2;
  const float mh = m / s.bc1;  // IEEE division / sqrt (hipcc default: correctly rounded)
  const float vh = v / s.bc2;
  const float num = s.lr * mh;
  d = num / (sqrtf(vh) + s.eps);
}

// The probe's hand-off error word: while it is set the update is refused on the device
// (m and v stay as they were, delta = 0, so the merge that follows adds exactly 0 to W_res)
__device__ __forceinline__ bool adam_refused(const int* err) {
  return __builtin_amdgcn_readfirstlane(
             err != nullptr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ? 1 : 0) != 0;
}

}  // namespace hdp
