// K2: adapter probe backward -- replaces the autograd of hp:139's adapter term.
//
// The reference materialises M = 1e-16*alpha*B@A (out x in), runs an extra full fp32
// T x in x out GEMM in the forward and three full GEMMs in the backward (dX, dM = G^T X,
// then dA = B^T dM, dB = dM A^T).  Algebraically
//     A.grad += s (G B)^T X        B.grad += s G^T (X A^T),     s = alpha_eff * 1e-16
// so only skinny products are needed (4 T r (in+out) flop; X and G are read once each for
// the projections and once for the outer products, the second read mostly from MALL):
//   P1 (proj) : H = X A^T  (T x r, K = in),  J = G B  (T x r, K = out)  -> split-K slabs
//               (B may be passed transposed, r x out: B is frozen, so the host keeps B^T)
//   P2 (outer): dA_part = J^T X,  dB_part = H^T G  (r x N, K = T)       -> split-T slabs;
//               each workgroup first reduces its rows of the P1 slabs into LDS
//   P3        : g += s * sum(parts)   (fixed summation order: deterministic)
// All products on fp32 MFMA v_mfma_f32_16x16x4_f32 (guide sec. 3):
//   operand a: lane l -> Am[i = l&15][kk = l>>4];  operand b: Bm[kk = l>>4][j = l&15]
//   result   : lane l holds D[row = 4(l>>4) + reg][col = l&15], reg in [0,4)
// A 16-byte load of 4 consecutive k per lane feeds 4 MFMAs (k = base + 4 kk + q, q-th
// MFMA), which keeps every global access of X and G a wide coalesced vector.
#include "hdp_common.h"

namespace hdp {

constexpr int kTC = 64;   // P2 T-chunk per workgroup
constexpr int kNW = 256;  // P2 columns per workgroup (4 waves x 64)

struct ProbePlan {
  int64_t T, in, out;
  int r, rp, RB;
  int ksh, ksj;      // P1 K splits for H (K=in) and J (K=out)
  int64_t kch, kcj;  // P1 K-chunk lengths (multiples of 64)
  int kst;           // P2 T splits
  size_t off_slabH, off_slabJ, off_partA, off_partB, bytes;
};

// P1 split: ~1024 waves per side so that every CU keeps several 1-KB loads in flight
static void split_k(int64_t K, int64_t tblk, int64_t& kc, int& ks) {
  int64_t target = (1024 + tblk - 1) / tblk;
  if (target < 1) target = 1;
  kc = (K + target - 1) / target;
  kc = (kc + 63) / 64 * 64;
  ks = (int)((K + kc - 1) / kc);
}

static ProbePlan make_plan(int64_t T, int64_t in, int64_t out, int r) {
  ProbePlan p;
  p.T = T;
  p.in = in;
  p.out = out;
  p.r = r;
  const int rb = (r + 15) / 16;
  p.RB = rb <= 1 ? 1 : rb <= 2 ? 2 : rb <= 4 ? 4 : 8;
  p.rp = 16 * p.RB;
  const int64_t tblk = (T + 15) / 16;
  split_k(in, tblk, p.kch, p.ksh);
  split_k(out, tblk, p.kcj, p.ksj);
  p.kst = (int)((T + kTC - 1) / kTC);
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n * 4 + 255) / 256 * 256; return o; };
  p.off_slabH = take((size_t)p.ksh * T * p.rp);
  p.off_slabJ = take((size_t)p.ksj * T * p.rp);
  p.off_partA = take((size_t)p.kst * p.rp * in);
  p.off_partB = take((size_t)p.kst * p.rp * out);
  p.bytes = off;
  return p;
}

// ---------------------------------------------------------------------------------------
// P1: slab[ks][t][j] = sum_{k in chunk ks} Z[t][k] F(k, j)
//   F_RK: F given as [r][K] (A, or B^T);  otherwise as [K][r] (B)
// One wave = 16 rows x one K-chunk; U 16-column steps are loaded back to back before their
// MFMAs so each wave keeps U x 1 KB of Z (plus the F rows) in flight.
// ---------------------------------------------------------------------------------------
struct ProjJob {
  const void* Z;
  const float* F;
  float* slab;
  int64_t K, kc;
  int ks;
  int nwaves;
  int f_rk;
};
struct ProjArgs {
  ProjJob job[2];
  int64_t T;
  int r, rp;
};

template <bool F_RK>
__device__ __forceinline__ f32x4 load_f4(const ProjArgs& a, const ProjJob& jb, int j, int64_t k, bool full) {
  f32x4 f;
  if (F_RK) {
    if (j < a.r && full) return *reinterpret_cast<const f32x4*>(jb.F + (int64_t)j * jb.K + k);
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = (j < a.r && k + q < jb.K) ? jb.F[(int64_t)j * jb.K + k + q] : 0.f;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = (j < a.r && k + q < jb.K) ? jb.F[(k + q) * a.r + j] : 0.f;
  }
  return f;
}

template <int DT, int RB, bool F_RK>
__device__ __forceinline__ void proj_wave(const ProjArgs& a, const ProjJob& jb, int wid, int lane) {
  constexpr int U = RB >= 4 ? 1 : 4 / RB;
  const int li = lane & 15, g = lane >> 4;
  const int64_t tb = (int64_t)(wid / jb.ks) * 16;
  const int ks = wid % jb.ks;
  const int64_t k0 = (int64_t)ks * jb.kc;
  const int64_t k1 = min(jb.K, k0 + jb.kc);
  const int64_t zrow = min(tb + li, a.T - 1) * jb.K;
  f32x4 acc[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  int64_t k = k0;
  if (jb.K % 4 == 0) {
    for (; k + 16 * U <= k1; k += 16 * U) {
      f32x4 z[U], f[U][RB];
#pragma unroll
      for (int u = 0; u < U; ++u) z[u] = load4<DT>(jb.Z, zrow + k + 16 * u + 4 * g);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int b = 0; b < RB; ++b) f[u][b] = load_f4<F_RK>(a, jb, b * 16 + li, k + 16 * u + 4 * g, true);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(z[u][q], f[u][b][q], acc[b], 0, 0, 0);
    }
  }
  for (; k < k1; k += 16) {  // tail: guarded 16-column steps
    const int64_t kq = k + 4 * g;
    const bool full = (k + 16 <= k1) && (jb.K % 4 == 0);
    f32x4 z;
    if (full) {
      z = load4<DT>(jb.Z, zrow + kq);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) z[q] = (kq + q < k1) ? load1<DT>(jb.Z, zrow + kq + q) : 0.f;
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      f32x4 f = load_f4<F_RK>(a, jb, b * 16 + li, kq, full);
      if (!full) {
#pragma unroll
        for (int q = 0; q < 4; ++q) f[q] = (kq + q < k1) ? f[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(z[q], f[q], acc[b], 0, 0, 0);
    }
  }
#pragma unroll
  for (int b = 0; b < RB; ++b) {
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int64_t t = tb + 4 * g + reg;
      if (t < a.T) jb.slab[((int64_t)ks * a.T + t) * a.rp + b * 16 + li] = acc[b][reg];
    }
  }
}

template <int DT, int RB>
__global__ __launch_bounds__(256) void probe_proj_kernel(ProjArgs a) {
  const int lane = threadIdx.x & 63;
  int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid < a.job[0].nwaves) {
    proj_wave<DT, RB, true>(a, a.job[0], wid, lane);
  } else {
    wid -= a.job[0].nwaves;
    if (wid < a.job[1].nwaves) {
      if (a.job[1].f_rk) proj_wave<DT, RB, true>(a, a.job[1], wid, lane);
      else proj_wave<DT, RB, false>(a, a.job[1], wid, lane);
    }
  }
}

// ---------------------------------------------------------------------------------------
// P2: part[kt] = sum_{t in chunk kt} Y[t][j] Z[t][n],  Y = sum_ks slabY[ks]
//   layout of part[kt]: [rp][N] (dA) or, with TRANS, [N][rp] (dB, so P3 writes B's layout)
// ---------------------------------------------------------------------------------------
struct OuterJob {
  const void* Z;
  const float* slabY;
  float* part;
  int64_t N;
  int ksY;
  int nblocks;  // = ceil(N / kNW) * kst
  int trans;
};
struct OuterArgs {
  OuterJob job[2];
  int64_t T;
  int r, rp, kst;
};

template <int DT, int RB>
__device__ __forceinline__ void outer_block(const OuterArgs& a, const OuterJob& jb, int bid, float* Ys) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int kt = bid % a.kst;
  const int64_t nb = (int64_t)(bid / a.kst) * kNW;
  const int64_t tb = (int64_t)kt * kTC;
  const int rp = a.rp;
  // reduce the P1 slabs for rows [tb, tb + kTC) into LDS (16-B granules, 4 independent sums)
  const int r4 = rp / 4;
  for (int e = tid; e < kTC * r4; e += 256) {
    const int tt = e / r4, j = (e % r4) * 4;
    const int64_t t = tb + tt;
    f32x4 s0{0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    if (t < a.T) {
      const f32x4* src = reinterpret_cast<const f32x4*>(jb.slabY + t * rp + j);
      const int64_t step4 = a.T * rp / 4;
      int ks = 0;
      for (; ks + 4 <= jb.ksY; ks += 4) {
        s0 += src[(ks + 0) * step4];
        s1 += src[(ks + 1) * step4];
        s2 += src[(ks + 2) * step4];
        s3 += src[(ks + 3) * step4];
      }
      for (; ks < jb.ksY; ++ks) s0 += src[ks * step4];
    }
    *reinterpret_cast<f32x4*>(Ys + tt * rp + j) = (s0 + s1) + (s2 + s3);
  }
  __syncthreads();
  const int64_t ncol = nb + 64 * wave + 4 * li;  // lane's 4 columns: ncol + q
  const bool vecN = (jb.N % 4 == 0) && (ncol + 3 < jb.N);
  f32x4 acc[RB][4];
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tlen = (int)min((int64_t)kTC, a.T - tb);
  constexpr int U = 4;
  for (int tt = 0; tt < tlen; tt += 4 * U) {
    f32x4 z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = tt + 4 * u + g;
      z[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < tlen) {
        const int64_t base = (tb + row) * jb.N + ncol;
        if (vecN) {
          z[u] = load4<DT>(jb.Z, base);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) z[u][q] = (ncol + q < jb.N) ? load1<DT>(jb.Z, base + q) : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const float y = Ys[(tt + 4 * u + g) * rp + b * 16 + li];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(y, z[u][q], acc[b][q], 0, 0, 0);
      }
    }
  }
  // lane holds D[j = 16b + 4g + reg][n = ncol + q]
  if (!jb.trans) {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int j = b * 16 + 4 * g + reg;
        float* dst = jb.part + ((int64_t)kt * rp + j) * jb.N + ncol;
        f32x4 v{acc[b][0][reg], acc[b][1][reg], acc[b][2][reg], acc[b][3][reg]};
        if (vecN) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (ncol + q < jb.N) dst[q] = v[q];
        }
      }
    }
  } else {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ncol + q >= jb.N) continue;
        float* dst = jb.part + ((int64_t)kt * jb.N + ncol + q) * rp + b * 16 + 4 * g;
        *reinterpret_cast<f32x4*>(dst) = acc[b][q];
      }
    }
  }
}

template <int DT, int RB>
__global__ __launch_bounds__(256) void probe_outer_kernel(OuterArgs a) {
  extern __shared__ __attribute__((aligned(16))) float Ys[];
  int bid = blockIdx.x;
  if (bid < a.job[0].nblocks) {
    outer_block<DT, RB>(a, a.job[0], bid, Ys);
  } else {
    bid -= a.job[0].nblocks;
    outer_block<DT, RB>(a, a.job[1], bid, Ys);
  }
}

// ---------------------------------------------------------------------------------------
// P3: gA[j][n] (+)= s * sum_kt partA[kt][j][n];  gB[n][j] (+)= s * sum_kt partB[kt][n][j]
// ---------------------------------------------------------------------------------------
struct FinishArgs {
  const float* partA;
  const float* partB;
  float* gA;
  float* gB;
  int64_t in, out;
  int r, rp, kst;
  float scale;
  int accumulate;
};

__device__ __forceinline__ float sum_parts(const float* p, int64_t stride, int n) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int k = 0;
  for (; k + 4 <= n; k += 4) {
    s0 += p[(k + 0) * stride];
    s1 += p[(k + 1) * stride];
    s2 += p[(k + 2) * stride];
    s3 += p[(k + 3) * stride];
  }
  for (; k < n; ++k) s0 += p[k * stride];
  return (s0 + s1) + (s2 + s3);
}

__global__ __launch_bounds__(256) void probe_finish_kernel(FinishArgs a) {
#pragma clang fp contract(off)  // g + s*sum as two roundings, like autograd's mul then add
  const int64_t nA = (int64_t)a.r * a.in, nB = (int64_t)a.r * a.out;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nA + nB; e += (int64_t)gridDim.x * 256) {
    if (e < nA) {
      const float s = sum_parts(a.partA + e, (int64_t)a.rp * a.in, a.kst);  // rows j < r are a prefix
      const float v = a.scale * s;
      a.gA[e] = a.accumulate ? a.gA[e] + v : v;
    } else {
      const int64_t f = e - nA;
      const int64_t n = f / a.r, j = f % a.r;
      const float s = sum_parts(a.partB + n * a.rp + j, (int64_t)a.out * a.rp, a.kst);
      const float v = a.scale * s;
      a.gB[f] = a.accumulate ? a.gB[f] + v : v;
    }
  }
}

template <int DT, int RB>
static int launch_probe(const ProbePlan& p, const void* X, const void* G, const float* A, const float* B,
                        int b_transposed, float* gA, float* gB, float scale, int accumulate, char* ws,
                        hipStream_t st) {
  float* slabH = reinterpret_cast<float*>(ws + p.off_slabH);
  float* slabJ = reinterpret_cast<float*>(ws + p.off_slabJ);
  float* partA = reinterpret_cast<float*>(ws + p.off_partA);
  float* partB = reinterpret_cast<float*>(ws + p.off_partB);
  const int64_t tblk = (p.T + 15) / 16;
  ProjArgs pa;
  pa.T = p.T;
  pa.r = p.r;
  pa.rp = p.rp;
  pa.job[0] = ProjJob{X, A, slabH, p.in, p.kch, p.ksh, (int)(tblk * p.ksh), 1};
  pa.job[1] = ProjJob{G, B, slabJ, p.out, p.kcj, p.ksj, (int)(tblk * p.ksj), b_transposed ? 1 : 0};
  const int w1 = pa.job[0].nwaves + pa.job[1].nwaves;
  hipLaunchKernelGGL((probe_proj_kernel<DT, RB>), dim3((w1 + 3) / 4), dim3(256), 0, st, pa);
  HDP_CHECK_LAUNCH();

  OuterArgs oa;
  oa.T = p.T;
  oa.r = p.r;
  oa.rp = p.rp;
  oa.kst = p.kst;
  // dA = J^T X (Y = J, Z = X, N = in);  dB = (H^T G)^T (Y = H, Z = G, N = out, transposed parts)
  oa.job[0] = OuterJob{X, slabJ, partA, p.in, p.ksj, (int)(((p.in + kNW - 1) / kNW) * p.kst), 0};
  oa.job[1] = OuterJob{G, slabH, partB, p.out, p.ksh, (int)(((p.out + kNW - 1) / kNW) * p.kst), 1};
  const size_t lds = (size_t)kTC * p.rp * sizeof(float);
  hipLaunchKernelGGL((probe_outer_kernel<DT, RB>), dim3(oa.job[0].nblocks + oa.job[1].nblocks), dim3(256), lds,
                     st, oa);
  HDP_CHECK_LAUNCH();

  FinishArgs fa{partA, partB, gA, gB, p.in, p.out, p.r, p.rp, p.kst, scale, accumulate};
  const int64_t tot = (int64_t)p.r * (p.in + p.out);
  int blocks = (int)min((int64_t)2048, (tot + 255) / 256);
  hipLaunchKernelGGL(probe_finish_kernel, dim3(blocks), dim3(256), 0, st, fa);
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}

}  // namespace hdp

using namespace hdp;

extern "C" size_t hdp_probe_workspace_bytes(int64_t T, int64_t in, int64_t out, int r) {
  if (T <= 0 || in <= 0 || out <= 0 || r <= 0 || r > 128) return 0;
  return make_plan(T, in, out, r).bytes;
}

extern "C" int hdp_probe_grads(int64_t T, int64_t in, int64_t out, int r, const void* X, const void* G,
                               int x_dtype, const float* A, const float* B, int b_transposed, float* gA, float* gB,
                               float scale, int accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  HDP_CHECK_ARG(in > 0 && out > 0 && r > 0 && T >= 0, "hdp_probe_grads: bad shape");
  HDP_CHECK_ARG(r <= 128, "hdp_probe_grads: r = %d > 128 is not supported", r);
  HDP_CHECK_ARG(x_dtype == HDP_F32 || x_dtype == HDP_BF16, "hdp_probe_grads: bad dtype %d", x_dtype);
  HDP_CHECK_ARG(A && B && gA && gB, "hdp_probe_grads: null pointer");
  hipStream_t st = as_stream(stream);
  if (T == 0) {
    if (!accumulate) {
      HDP_CHECK_HIP(hipMemsetAsync(gA, 0, sizeof(float) * r * in, st));
      HDP_CHECK_HIP(hipMemsetAsync(gB, 0, sizeof(float) * r * out, st));
    }
    return HDP_OK;
  }
  HDP_CHECK_ARG(X && G && workspace, "hdp_probe_grads: null pointer");
  const ProbePlan p = make_plan(T, in, out, r);
  HDP_CHECK_ARG(workspace_bytes >= p.bytes, "hdp_probe_grads: workspace %zu < %zu bytes", workspace_bytes,
                p.bytes);
  HDP_CHECK_ARG((reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
                    (!b_transposed || (reinterpret_cast<uintptr_t>(B) & 15) == 0) &&
                    (reinterpret_cast<uintptr_t>(G) & 15) == 0,
                "hdp_probe_grads: X, G and A must be 16-byte aligned");
  char* ws = reinterpret_cast<char*>(workspace);
#define HDP_PROBE(D, R) return launch_probe<D, R>(p, X, G, A, B, b_transposed, gA, gB, scale, accumulate, ws, st)
  if (x_dtype == HDP_F32) {
    switch (p.RB) {
      case 1: HDP_PROBE(HDP_F32, 1);
      case 2: HDP_PROBE(HDP_F32, 2);
      case 4: HDP_PROBE(HDP_F32, 4);
      default: HDP_PROBE(HDP_F32, 8);
    }
  } else {
    switch (p.RB) {
      case 1: HDP_PROBE(HDP_BF16, 1);
      case 2: HDP_PROBE(HDP_BF16, 2);
      case 4: HDP_PROBE(HDP_BF16, 4);
      default: HDP_PROBE(HDP_BF16, 8);
    }
  }
#undef HDP_PROBE
}
