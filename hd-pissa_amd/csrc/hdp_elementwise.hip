// K5 merge (hp:394) and K3 Adam-on-factors (hp:356-373): HBM-streaming kernels.
//
// Both are pure streams with no reuse: 16-byte vector accesses per lane, a grid of at most
// 256 CUs x 8 blocks striding over the array, two vectors in flight per lane.  Roofline:
//   merge f32 W : 12 B/element (read W, read dW, write W)
//   merge bf16 W:  8 B/element (read W 2, read dW 4, write W 2)
//   adam        : 24 B/element (read g, m, v; write m, v, delta) (+4 with zero_grad)
#include "hdp_common.h"

namespace hdp {

constexpr int kEwThreads = 256;
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

static int ew_grid(int64_t vec_items, int per_thread) {
  int64_t blocks = (vec_items + (int64_t)kEwThreads * per_thread - 1) / ((int64_t)kEwThreads * per_thread);
  if (blocks > 256 * 8) blocks = 256 * 8;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

// ---------------------------------------------------------------------------------------
// merge: W += dW
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kEwThreads) void merge_f32_kernel(float* __restrict__ W,
                                                               const float* __restrict__ dW,
                                                               int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  f32x4* W4 = reinterpret_cast<f32x4*>(W);
  const f32x4* D4 = reinterpret_cast<const f32x4*>(dW);
  for (; i + stride < n4; i += 2 * stride) {
    f32x4 d0 = __builtin_nontemporal_load(D4 + i);
    f32x4 d1 = __builtin_nontemporal_load(D4 + i + stride);
    f32x4 w0 = W4[i];
    f32x4 w1 = W4[i + stride];
    W4[i] = w0 + d0;
    W4[i + stride] = w1 + d1;
  }
  if (i < n4) W4[i] = W4[i] + __builtin_nontemporal_load(D4 + i);
}

__global__ __launch_bounds__(kEwThreads) void merge_bf16_kernel(uint16_t* __restrict__ W,
                                                                const float* __restrict__ dW,
                                                                int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  u16x8* W8 = reinterpret_cast<u16x8*>(W);
  const f32x4* D4 = reinterpret_cast<const f32x4*>(dW);
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < n8; i += stride) {
    f32x4 d0 = __builtin_nontemporal_load(D4 + 2 * i);
    f32x4 d1 = __builtin_nontemporal_load(D4 + 2 * i + 1);
    u16x8 w = W8[i];
    u16x8 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = f32_to_bf16(bf16_to_f32(w[q]) + round_bf16(d0[q]));
      o[q + 4] = f32_to_bf16(bf16_to_f32(w[q + 4]) + round_bf16(d1[q]));
    }
    W8[i] = o;
  }
}

// grouped merge: one exchange bucket's modules in one launch; every item
// 16-B aligned with a whole number of vectors (the host checks, else it merges item by item)
constexpr int kMergeGroupMax = 64;
struct MergeGroupArgs {
  int n, bf16;
  void* W[kMergeGroupMax];
  const float* dW[kMergeGroupMax];
  int64_t nv[kMergeGroupMax];  // f32: float4 vectors; bf16: 8-element vectors
};
static_assert(sizeof(MergeGroupArgs) <= 4096, "merge group kernel arguments must stay within 4 KB");

__global__ __launch_bounds__(kEwThreads) void merge_group_kernel(MergeGroupArgs ga) {
  // persistent: every workgroup strides through every item in turn (one launch-sized grid, as the
  // single-slab kernel, instead of a grid per item)
  for (int it = 0; it < ga.n; ++it) {
  const int64_t nv = ga.nv[it];
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  const HDP_GLOBAL f32x4* D4 = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(ga.dW[it]));
  if (!ga.bf16) {
    HDP_GLOBAL f32x4* W4 = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(reinterpret_cast<float*>(ga.W[it])));
    int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
    // every byte is touched once: non-temporal loads AND stores (the K4 merge epilogue measured
    // +12 % from the same policy, profiles/r01_k4_wn1_cache_policy.txt)
    for (; i + stride < nv; i += 2 * stride) {
      const f32x4 d0 = __builtin_nontemporal_load(D4 + i), d1 = __builtin_nontemporal_load(D4 + i + stride);
      const f32x4 w0 = __builtin_nontemporal_load(W4 + i), w1 = __builtin_nontemporal_load(W4 + i + stride);
      __builtin_nontemporal_store(w0 + d0, W4 + i);
      __builtin_nontemporal_store(w1 + d1, W4 + i + stride);
    }
    if (i < nv) __builtin_nontemporal_store(__builtin_nontemporal_load(W4 + i) + __builtin_nontemporal_load(D4 + i), W4 + i);
  } else {
    HDP_GLOBAL u16x8* W8 = reinterpret_cast<HDP_GLOBAL u16x8*>(gptr(reinterpret_cast<uint16_t*>(ga.W[it])));
    for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < nv; i += stride) {
      const f32x4 d0 = __builtin_nontemporal_load(D4 + 2 * i), d1 = __builtin_nontemporal_load(D4 + 2 * i + 1);
      const u16x8 w = __builtin_nontemporal_load(W8 + i);
      u16x8 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        o[q] = f32_to_bf16(bf16_to_f32(w[q]) + round_bf16(d0[q]));
        o[q + 4] = f32_to_bf16(bf16_to_f32(w[q + 4]) + round_bf16(d1[q]));
      }
      __builtin_nontemporal_store(o, W8 + i);
    }
  }
  }
}

// scalar tail / unaligned fallback
__global__ void merge_scalar_kernel(void* W, int dt, const float* dW, int64_t begin, int64_t n) {
  for (int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (dt == HDP_F32) {
      reinterpret_cast<float*>(W)[i] += dW[i];
    } else {
      uint16_t* w = reinterpret_cast<uint16_t*>(W);
      w[i] = f32_to_bf16(bf16_to_f32(w[i]) + round_bf16(dW[i]));
    }
  }
}

// ---------------------------------------------------------------------------------------
// Adam on factors.  Every operation is rounded separately (contract(off) on plain operators:
// HIP's __fmul_rn / __fadd_rn are header-scope * and + that hipcc still fuses into FMAs) so the
// float32 result follows torch's op-by-op evaluation of hp:356-373.
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

template <bool ZERO>
__global__ __launch_bounds__(kEwThreads) void adam_kernel(float* __restrict__ grad, float* __restrict__ m,
                                                          float* __restrict__ v, float* __restrict__ delta,
                                                          int64_t n4, AdamScalars s) {
  const int64_t stride = (int64_t)gridDim.x * kEwThreads;
  f32x4* G = reinterpret_cast<f32x4*>(grad);
  f32x4* M = reinterpret_cast<f32x4*>(m);
  f32x4* V = reinterpret_cast<f32x4*>(v);
  f32x4* D = reinterpret_cast<f32x4*>(delta);
  for (int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x; i < n4; i += stride) {
    f32x4 g = G[i], mm = M[i], vv = V[i], dd;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float gq = g[q], mq = mm[q], vq = vv[q], dq;
      adam1(gq, mq, vq, dq, s);
      mm[q] = mq;
      vv[q] = vq;
      dd[q] = dq;
    }
    M[i] = mm;
    V[i] = vv;
    D[i] = dd;
    if (ZERO) G[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

__global__ void adam_scalar_kernel(float* grad, float* m, float* v, float* delta, int64_t begin,
                                   int64_t n, AdamScalars s, int zero) {
  for (int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float g = grad[i], mq = m[i], vq = v[i], d;
    adam1(g, mq, vq, d, s);
    m[i] = mq;
    v[i] = vq;
    delta[i] = d;
    if (zero) grad[i] = 0.f;
  }
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace hdp

using namespace hdp;

extern "C" int hdp_merge(void* W, int w_dtype, const float* dW, int64_t n, void* stream) {
  HDP_CHECK_ARG(n >= 0, "hdp_merge: n < 0");
  HDP_CHECK_ARG(w_dtype == HDP_F32 || w_dtype == HDP_BF16, "hdp_merge: bad dtype %d", w_dtype);
  if (n == 0) return HDP_OK;
  HDP_CHECK_ARG(W && dW, "hdp_merge: null pointer");
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  const bool al = aligned16(W) && aligned16(dW);
  if (w_dtype == HDP_F32 && al) {
    const int64_t n4 = n / 4;
    if (n4) {
      KTimer kt(K_MERGE, st, 12.0 * 4 * n4);
      hipLaunchKernelGGL(merge_f32_kernel, dim3(ew_grid(n4, 2)), dim3(kEwThreads), 0, st,
                         reinterpret_cast<float*>(W), dW, n4);
      HDP_CHECK_LAUNCH();
    }
    done = n4 * 4;
  } else if (w_dtype == HDP_BF16 && al) {
    const int64_t n8 = n / 8;
    if (n8) {
      KTimer kt(K_MERGE, st, 8.0 * 8 * n8);
      hipLaunchKernelGGL(merge_bf16_kernel, dim3(ew_grid(n8, 1)), dim3(kEwThreads), 0, st,
                         reinterpret_cast<uint16_t*>(W), dW, n8);
      HDP_CHECK_LAUNCH();
    }
    done = n8 * 8;
  }
  if (done < n) {
    const int64_t rest = n - done;
    int blocks = (int)((rest + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    {
      KTimer kt(K_MERGE, st, (w_dtype == HDP_F32 ? 12.0 : 8.0) * rest);
      hipLaunchKernelGGL(merge_scalar_kernel, dim3(blocks), dim3(256), 0, st, W, w_dtype, dW, done, n);
    }
    HDP_CHECK_LAUNCH();
  }
  return HDP_OK;
}

extern "C" int hdp_merge_group(int n, const hdp_merge_item* items, int w_dtype, void* stream) {
  HDP_CHECK_ARG(n >= 0 && (n == 0 || items), "hdp_merge_group: bad item list");
  HDP_CHECK_ARG(w_dtype == HDP_F32 || w_dtype == HDP_BF16, "hdp_merge_group: bad dtype %d", w_dtype);
  hipStream_t st = as_stream(stream);
  const int64_t vec = w_dtype == HDP_F32 ? 4 : 8;
  MergeGroupArgs ga;
  ga.n = 0;
  ga.bf16 = w_dtype == HDP_BF16;
  int64_t big = 0;
  double bytes = 0;
  auto launch = [&]() -> int {
    if (ga.n == 0) return HDP_OK;
    int64_t gx = (big + (int64_t)kEwThreads * 2 - 1) / ((int64_t)kEwThreads * 2);
    gx = gx < 1 ? 1 : (gx > 2048 ? 2048 : gx);
    {
      KTimer kt(K_MERGE, st, bytes);
      hipLaunchKernelGGL(merge_group_kernel, dim3((unsigned)gx), dim3(kEwThreads), 0, st, ga);
    }
    HDP_CHECK_LAUNCH();
    ga.n = 0;
    big = 0;
    bytes = 0;
    return HDP_OK;
  };
  for (int i = 0; i < n; ++i) {
    const hdp_merge_item& it = items[i];
    HDP_CHECK_ARG(it.n >= 0 && (it.n == 0 || (it.W && it.dW)), "hdp_merge_group: bad item %d", i);
    if (it.n == 0) continue;
    if (!aligned16(it.W) || !aligned16(it.dW) || it.n % vec != 0) {  // this item on its own
      const int rc = hdp_merge(it.W, w_dtype, it.dW, it.n, stream);
      if (rc) return rc;
      continue;
    }
    ga.W[ga.n] = it.W;
    ga.dW[ga.n] = it.dW;
    ga.nv[ga.n] = it.n / vec;
    big = ga.nv[ga.n] > big ? ga.nv[ga.n] : big;
    bytes += (w_dtype == HDP_F32 ? 12.0 : 8.0) * it.n;
    if (++ga.n == kMergeGroupMax) {
      const int rc = launch();
      if (rc) return rc;
    }
  }
  return launch();
}

extern "C" int hdp_adam_factors(float* grad, float* m, float* v, float* delta, int64_t n,
                                float grad_scale, float beta1, float one_minus_beta1, float beta2,
                                float one_minus_beta2, float bc1, float bc2, float lr, float eps,
                                int zero_grad, void* stream) {
  HDP_CHECK_ARG(n >= 0, "hdp_adam_factors: n < 0");
  if (n == 0) return HDP_OK;
  HDP_CHECK_ARG(grad && m && v && delta, "hdp_adam_factors: null pointer");
  HDP_CHECK_ARG(bc1 != 0.f && bc2 != 0.f, "hdp_adam_factors: bias correction is zero (t == 0?)");
  AdamScalars s{grad_scale, beta1, one_minus_beta1, beta2, one_minus_beta2, bc1, bc2, lr, eps};
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned16(grad) && aligned16(m) && aligned16(v) && aligned16(delta)) {
    const int64_t n4 = n / 4;
    if (n4) {
      KTimer kt(K_ADAM, st, 28.0 * 4 * n4);
      if (zero_grad)
        hipLaunchKernelGGL(adam_kernel<true>, dim3(ew_grid(n4, 1)), dim3(kEwThreads), 0, st, grad, m, v,
                           delta, n4, s);
      else
        hipLaunchKernelGGL(adam_kernel<false>, dim3(ew_grid(n4, 1)), dim3(kEwThreads), 0, st, grad, m, v,
                           delta, n4, s);
      HDP_CHECK_LAUNCH();
    }
    done = n4 * 4;
  }
  if (done < n) {
    const int64_t rest = n - done;
    int blocks = (int)((rest + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    {
      KTimer kt(K_ADAM, st, 28.0 * rest);
      hipLaunchKernelGGL(adam_scalar_kernel, dim3(blocks), dim3(256), 0, st, grad, m, v, delta, done, n, s,
                         zero_grad);
    }
    HDP_CHECK_LAUNCH();
  }
  return HDP_OK;
}
