// K5 merge (hp:394) and K3 Adam-on-factors (hp:356-373): HBM-streaming kernels.
//
// Both are pure streams with no reuse: 16-byte vector accesses per lane.  Roofline:
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
// merge: W += dW.  Contiguous chunks: a workgroup owns kMergeU x 256 consecutive vectors at a time
// (every load of the chunk issued before its first store; each byte touched once, so non-temporal
// loads and stores) and walks chunks blockIdx.x, + grid, ... of one flat chunk space over a bucket's
// items.  tools/merge_bw.hip on a 1 GiB float32 slab: this form 5.76 TB/s (0.72 of 8) against 4.61 for
// the grid-stride loop with two vectors per lane it replaces (profiles/r03_merge_bw_v2.txt).
// ---------------------------------------------------------------------------------------
constexpr int kMergeU = 4;            // vectors per lane per chunk
constexpr int kMergeGrid = 2048;      // workgroups (8 per CU)
constexpr int kMergeGroupMax = 64;
struct MergeGroupArgs {
  int n;
  void* W[kMergeGroupMax];
  const float* dW[kMergeGroupMax];
  int64_t nv[kMergeGroupMax];  // f32: float4 vectors; bf16: 8-element vectors
};
static_assert(sizeof(MergeGroupArgs) <= 4096, "merge group kernel arguments must stay within 4 KB");

template <bool BF>
__global__ __launch_bounds__(kEwThreads) void merge_chunk_kernel(MergeGroupArgs ga) {
  // bf16 W with float32 dW: 8 vectors per lane (r04, tools/merge_bench.py: 0.69 -> 0.735 of HBM; float32 W and
  // the bf16-dW merge are faster at 4)
  constexpr int U = BF ? 2 * kMergeU : kMergeU;
  constexpr int64_t CH = (int64_t)kEwThreads * U;  // vectors per chunk
  int it = 0;
  int64_t base = 0, nch = (ga.nv[0] + CH - 1) / CH;      // item it owns chunks [base, base + nch)
  for (int64_t c = blockIdx.x;; c += gridDim.x) {        // c, it, base: workgroup-uniform
    while (c >= base + nch) {
      base += nch;
      if (++it == ga.n) return;
      nch = (ga.nv[it] + CH - 1) / CH;
    }
    const int64_t nv = ga.nv[it];
    const int64_t v0 = (c - base) * CH + threadIdx.x;
    const HDP_GLOBAL f32x4* D4 = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(ga.dW[it]));
    if constexpr (!BF) {
      HDP_GLOBAL f32x4* W4 = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(reinterpret_cast<float*>(ga.W[it])));
      f32x4 w[U], d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = v0 + u * kEwThreads;
        if (i < nv) {
          d[u] = __builtin_nontemporal_load(D4 + i);
          w[u] = __builtin_nontemporal_load(W4 + i);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = v0 + u * kEwThreads;
        if (i < nv) __builtin_nontemporal_store(w[u] + d[u], W4 + i);
      }
    } else {
      HDP_GLOBAL u16x8* W8 = reinterpret_cast<HDP_GLOBAL u16x8*>(gptr(reinterpret_cast<uint16_t*>(ga.W[it])));
      u16x8 w[U];
      f32x4 d0[U], d1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = v0 + u * kEwThreads;
        if (i < nv) {
          d0[u] = __builtin_nontemporal_load(D4 + 2 * i);
          d1[u] = __builtin_nontemporal_load(D4 + 2 * i + 1);
          w[u] = __builtin_nontemporal_load(W8 + i);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = v0 + u * kEwThreads;
        if (i < nv) {  // bf16(W + bf16(dW)), two elements per packed conversion
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 wv = __builtin_bit_cast(u32x4, w[u]);
          u32x4 o;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const f32x4& dd = k < 2 ? d0[u] : d1[u];
            const uint32_t dp = cvt_pk_bf16(dd[(2 * k) & 3], dd[(2 * k + 1) & 3]);
            o[k] = cvt_pk_bf16(__uint_as_float(wv[k] << 16) + __uint_as_float(dp << 16),
                               __uint_as_float(wv[k] & 0xffff0000u) + __uint_as_float(dp & 0xffff0000u));
          }
          __builtin_nontemporal_store(__builtin_bit_cast(u16x8, o), W8 + i);
        }
      }
    }
  }
}

// bf16 W += bf16 dW (the rank-ordered bf16 exchange): 8-element vectors, 6 B per element
__global__ __launch_bounds__(kEwThreads) void merge_bf16dw_kernel(MergeGroupArgs ga) {
  constexpr int64_t CH = (int64_t)kEwThreads * kMergeU;
  int it = 0;
  int64_t base = 0, nch = (ga.nv[0] + CH - 1) / CH;
  for (int64_t c = blockIdx.x;; c += gridDim.x) {
    while (c >= base + nch) {
      base += nch;
      if (++it == ga.n) return;
      nch = (ga.nv[it] + CH - 1) / CH;
    }
    const int64_t nv = ga.nv[it];
    const int64_t v0 = (c - base) * CH + threadIdx.x;
    HDP_GLOBAL u16x8* W8 = reinterpret_cast<HDP_GLOBAL u16x8*>(gptr(reinterpret_cast<uint16_t*>(ga.W[it])));
    const HDP_GLOBAL u16x8* D8 =
        reinterpret_cast<const HDP_GLOBAL u16x8*>(gptr(reinterpret_cast<const uint16_t*>(ga.dW[it])));
    u16x8 w[kMergeU], d[kMergeU];
#pragma unroll
    for (int u = 0; u < kMergeU; ++u) {
      const int64_t i = v0 + u * kEwThreads;
      if (i < nv) {
        d[u] = __builtin_nontemporal_load(D8 + i);
        w[u] = __builtin_nontemporal_load(W8 + i);
      }
    }
#pragma unroll
    for (int u = 0; u < kMergeU; ++u) {
      const int64_t i = v0 + u * kEwThreads;
      if (i < nv) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 wv = __builtin_bit_cast(u32x4, w[u]), dv = __builtin_bit_cast(u32x4, d[u]);
        u32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          o[k] = cvt_pk_bf16(__uint_as_float(wv[k] << 16) + __uint_as_float(dv[k] << 16),
                             __uint_as_float(wv[k] & 0xffff0000u) + __uint_as_float(dv[k] & 0xffff0000u));
        __builtin_nontemporal_store(__builtin_bit_cast(u16x8, o), W8 + i);
      }
    }
  }
}

__global__ void merge_bf16dw_scalar_kernel(uint16_t* W, const uint16_t* dW, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    W[i] = f32_to_bf16(bf16_to_f32(W[i]) + bf16_to_f32(dW[i]));
}

// ---------------------------------------------------------------------------------------
// Rank-ordered bf16 fold (hp:389-392 for a bf16 model): out = 0; out = bf16(out + parts[i]) for
// i = 0 .. nparts - 1, one 4-element vector per lane and grid-stride; the parts are read once.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kEwThreads) void fold_bf16_kernel(const float* __restrict__ parts, int nparts,
                                                                int64_t stride, uint16_t* __restrict__ out,
                                                                int64_t n, int vec) {
  const int64_t nv = vec ? n / 4 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float run[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < nparts; ++p) {
      const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(parts + p * stride)) + i);
#pragma unroll
      for (int q = 0; q < 4; ++q) run[q] = bf16_to_f32(f32_to_bf16(run[q] + v[q]));
    }
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 o{(uint32_t)f32_to_bf16(run[0]) | ((uint32_t)f32_to_bf16(run[1]) << 16),
                  (uint32_t)f32_to_bf16(run[2]) | ((uint32_t)f32_to_bf16(run[3]) << 16)};
    *reinterpret_cast<HDP_GLOBAL u32x2*>(gptr(out + 4 * i)) = o;
  }
  for (int64_t e = 4 * nv + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float run = 0.f;
    for (int p = 0; p < nparts; ++p) run = bf16_to_f32(f32_to_bf16(run + parts[p * stride + e]));
    out[e] = f32_to_bf16(run);
  }
}

static int merge_chunk_launch(const MergeGroupArgs& ga, bool bf16, double bytes, hipStream_t st) {
  // the chunk the kernel walks (merge_chunk_kernel<BF>'s U): the grid never exceeds the chunk count
  const int64_t CH = (int64_t)kEwThreads * (bf16 ? 2 * kMergeU : kMergeU);
  int64_t chunks = 0;
  for (int i = 0; i < ga.n; ++i) chunks += (ga.nv[i] + CH - 1) / CH;
  if (chunks == 0) return HDP_OK;
  const unsigned grid = (unsigned)(chunks < kMergeGrid ? chunks : kMergeGrid);
  KTimer kt(K_MERGE, st, bytes);
  if (bf16) hipLaunchKernelGGL(merge_chunk_kernel<true>, dim3(grid), dim3(kEwThreads), 0, st, ga);
  else hipLaunchKernelGGL(merge_chunk_kernel<false>, dim3(grid), dim3(kEwThreads), 0, st, ga);
  HDP_CHECK_LAUNCH();
  return HDP_OK;
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
// float32 result follows torch's op-by-op evaluation of hp:356-373 (AdamScalars, adam1 and
// adam_refused live in hdp_common.h: K4's fused Adam + H2 pack runs the same arithmetic).
// ---------------------------------------------------------------------------------------
// The probe's hand-off error word: the step's host check sees only probe launches that
// have completed, so the last groups of the accumulation window may still be running when it passes.
// Adam reads the word in stream order: while it is set the update is refused on the device -- m and v
// stay as they were and delta is written as 0, so the K4 / K5 merge that follows adds exactly 0 to
// W_res -- and the next flush / step raises on the host.

// contiguous chunks of kAdamU x 256 vectors per workgroup step (the merge's form: every load of the
// chunk issued before its stores)
constexpr int kAdamU = 2;
template <bool ZERO>
__global__ __launch_bounds__(kEwThreads) void adam_kernel(float* __restrict__ grad, float* __restrict__ m,
                                                          float* __restrict__ v, float* __restrict__ delta,
                                                          int64_t n4, AdamScalars s, const int* err) {
  constexpr int64_t CH = (int64_t)kEwThreads * kAdamU;
  const bool refused = adam_refused(err);
  HDP_GLOBAL f32x4* G = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(grad));
  HDP_GLOBAL f32x4* M = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(m));
  HDP_GLOBAL f32x4* V = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(v));
  HDP_GLOBAL f32x4* D = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(delta));
  for (int64_t c = (int64_t)blockIdx.x * CH; c < n4; c += (int64_t)gridDim.x * CH) {
    f32x4 g[kAdamU], mm[kAdamU], vv[kAdamU];
#pragma unroll
    for (int u = 0; u < kAdamU; ++u) {
      const int64_t i = c + u * kEwThreads + threadIdx.x;
      if (i < n4) {
        g[u] = G[i];
        mm[u] = M[i];
        vv[u] = V[i];
      }
    }
#pragma unroll
    for (int u = 0; u < kAdamU; ++u) {
      const int64_t i = c + u * kEwThreads + threadIdx.x;
      if (i >= n4) continue;
      if (refused) {
        D[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (ZERO) G[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      f32x4 dd;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float gq = g[u][q], mq = mm[u][q], vq = vv[u][q], dq;
        adam1(gq, mq, vq, dq, s);
        mm[u][q] = mq;
        vv[u][q] = vq;
        dd[q] = dq;
      }
      M[i] = mm[u];
      V[i] = vv[u];
      D[i] = dd;
      if (ZERO) G[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

__global__ void adam_scalar_kernel(float* grad, float* m, float* v, float* delta, int64_t begin,
                                   int64_t n, AdamScalars s, int zero, const int* err) {
  const bool refused = adam_refused(err);
  for (int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (refused) {
      delta[i] = 0.f;
      if (zero) grad[i] = 0.f;
      continue;
    }
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
  if (al) {
    const int64_t vec = w_dtype == HDP_F32 ? 4 : 8;
    MergeGroupArgs ga;
    ga.n = 1;
    ga.W[0] = W;
    ga.dW[0] = dW;
    ga.nv[0] = n / vec;
    if (ga.nv[0]) {
      const int rc = merge_chunk_launch(ga, w_dtype == HDP_BF16, (w_dtype == HDP_F32 ? 12.0 : 8.0) * vec * ga.nv[0], st);
      if (rc) return rc;
    }
    done = ga.nv[0] * vec;
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
  double bytes = 0;
  auto launch = [&]() -> int {
    if (ga.n == 0) return HDP_OK;
    const int rc = merge_chunk_launch(ga, w_dtype == HDP_BF16, bytes, st);
    ga.n = 0;
    bytes = 0;
    return rc;
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
  const int* err = probe_err_device();
  int64_t done = 0;
  if (aligned16(grad) && aligned16(m) && aligned16(v) && aligned16(delta)) {
    const int64_t n4 = n / 4;
    if (n4) {
      KTimer kt(K_ADAM, st, 28.0 * 4 * n4);
      const dim3 grid(ew_grid(n4, kAdamU));
      if (zero_grad)
        hipLaunchKernelGGL(adam_kernel<true>, grid, dim3(kEwThreads), 0, st, grad, m, v, delta, n4, s, err);
      else
        hipLaunchKernelGGL(adam_kernel<false>, grid, dim3(kEwThreads), 0, st, grad, m, v, delta, n4, s, err);
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
                         zero_grad, err);
    }
    HDP_CHECK_LAUNCH();
  }
  return HDP_OK;
}

extern "C" int hdp_merge_group_bf16dw(int n, const hdp_merge_item* items, void* stream) {
  HDP_CHECK_ARG(n >= 0 && (n == 0 || items), "hdp_merge_group_bf16dw: bad item list");
  hipStream_t st = as_stream(stream);
  MergeGroupArgs ga;
  ga.n = 0;
  double bytes = 0;
  int64_t chunks = 0;
  constexpr int64_t CH = (int64_t)kEwThreads * kMergeU;
  auto launch = [&]() -> int {
    if (ga.n == 0) return HDP_OK;
    const unsigned grid = (unsigned)(chunks < kMergeGrid ? chunks : kMergeGrid);
    {
      KTimer kt(K_MERGE, st, bytes);
      hipLaunchKernelGGL(merge_bf16dw_kernel, dim3(grid), dim3(kEwThreads), 0, st, ga);
    }
    HDP_CHECK_LAUNCH();
    ga.n = 0;
    bytes = 0;
    chunks = 0;
    return HDP_OK;
  };
  for (int i = 0; i < n; ++i) {
    const hdp_merge_item& it = items[i];
    HDP_CHECK_ARG(it.n >= 0 && (it.n == 0 || (it.W && it.dW)), "hdp_merge_group_bf16dw: bad item %d", i);
    if (it.n == 0) continue;
    if (!aligned16(it.W) || !aligned16(it.dW) || it.n % 8 != 0) {  // this item element-wise
      int blocks = (int)((it.n + 255) / 256);
      if (blocks > 2048) blocks = 2048;
      {
        KTimer kt(K_MERGE, st, 6.0 * it.n);
        hipLaunchKernelGGL(merge_bf16dw_scalar_kernel, dim3(blocks), dim3(256), 0, st,
                           reinterpret_cast<uint16_t*>(it.W), reinterpret_cast<const uint16_t*>(it.dW), it.n);
      }
      HDP_CHECK_LAUNCH();
      continue;
    }
    ga.W[ga.n] = it.W;
    ga.dW[ga.n] = it.dW;
    ga.nv[ga.n] = it.n / 8;
    chunks += (ga.nv[ga.n] + CH - 1) / CH;
    bytes += 6.0 * it.n;
    if (++ga.n == kMergeGroupMax) {
      const int rc = launch();
      if (rc) return rc;
    }
  }
  return launch();
}

extern "C" int hdp_fold_bf16(const float* parts, int nparts, int64_t stride, void* out, int64_t n, void* stream) {
  HDP_CHECK_ARG(n >= 0 && nparts >= 1 && stride >= n, "hdp_fold_bf16: bad sizes (n=%lld nparts=%d stride=%lld)",
                (long long)n, nparts, (long long)stride);
  if (n == 0) return HDP_OK;
  HDP_CHECK_ARG(parts && out, "hdp_fold_bf16: null pointer");
  const int vec = aligned16(parts) && stride % 4 == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0;
  int64_t blocks = ((vec ? n / 4 : n) + kEwThreads - 1) / kEwThreads;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipStream_t st = as_stream(stream);
  {
    KTimer kt(K_FOLD, st, (4.0 * nparts + 2.0) * n);
    hipLaunchKernelGGL(fold_bf16_kernel, dim3((unsigned)blocks), dim3(kEwThreads), 0, st, parts, nparts, stride,
                       reinterpret_cast<uint16_t*>(out), n, vec);
  }
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}
