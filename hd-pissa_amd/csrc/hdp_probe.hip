// K2: adapter probe backward -- replaces the autograd of hp:139's adapter term.
//
// The reference materialises M = 1e-16*alpha*B@A (out x in), runs an extra full fp32
// T x in x out GEMM in the forward and three full GEMMs in the backward (dX, dM = G^T X,
// then dA = B^T dM, dB = dM A^T).  Algebraically
//     A.grad += s (G B)^T X        B.grad += s G^T (X A^T),     s = alpha_eff * 1e-16
// so only skinny products are needed (4 T r (in+out) flop):
//   P1 (proj) : H = X A^T  (T x r, K = in),  J = G B  (T x r, K = out)
//               8-wave workgroups (16 rows x 8 K-slices, reduced in LDS) -> ceil(K/2048) slabs
//   P2 (outer): dA_part = J^T X,  dB_part = H^T G  (r x N, K = T): 8-wave workgroups over 128
//               rows x 256 columns; the P1 slabs of its rows are reduced into LDS first
//   P3        : g (+)= s * sum(parts)   (fixed summation order: deterministic)
// X and G are read from HBM by P1 and re-read by P2 while a group's bytes still sit in the
// 256 MB Infinity Cache (the host sizes groups for that).
//
// GROUPED: one launch of each pass serves up to kMaxGroup modules (same r-block and dtype);
// the per-module descriptors travel by value in the kernel arguments, each workgroup finds
// its module by a prefix-sum lookup.  This replaces 3 launches + 3 host calls per module with
// 3 per group.
//
// All products on fp32 MFMA v_mfma_f32_16x16x4_f32 (guide sec. 3):
//   operand a: lane l -> Am[i = l&15][kk = l>>4];  operand b: Bm[kk = l>>4][j = l&15]
//   result   : lane l holds D[row = 4(l>>4) + reg][col = l&15], reg in [0,4)
// A 16-byte load of 4 consecutive k per lane feeds 4 MFMAs (k = base + 4 kk + q, q-th
// MFMA), which keeps every global access of X and G a wide coalesced vector.
#include <cstdlib>

#include "hdp_common.h"

namespace hdp {

constexpr int kMaxGroup = 16;  // keeps GroupArgs (kernel arguments, by value) near 2.6 KB
constexpr int kP1Waves = 8;       // P1 workgroup: 8 waves x 16 rows, K split over the waves

// P1 tuning knobs (defaults measured on MI355X; HDP_P1_COLS / HDP_P1_U override for sweeps)
static int p1_cols() {
  static const int v = [] { const char* e = getenv("HDP_P1_COLS"); return e ? atoi(e) : 128; }();
  return v;
}
static int p1_u() {
  static const int v = [] { const char* e = getenv("HDP_P1_U"); return e ? atoi(e) : 1; }();
  return v;
}
constexpr int kTC = 128;      // P2 rows per workgroup (8 waves: 2 row halves x 4 column groups)
constexpr int kNW = 256;      // P2 columns per workgroup

struct ProbeDesc {
  const void* X;
  const void* G;
  const float* A;
  const float* B;   // B (out x r) or B^T (r x out) when b_t
  float* gA;
  float* gB;
  float* slabH;     // [ksh][T][rp]
  float* slabJ;     // [ksj][T][rp]
  float* partA;     // [kst][rp][in]
  float* partB;     // [kst][out][rp]
  int64_t T, in, out;
  float scale;
  int r, b_t, accumulate;
  int ksh, ksj, kst;
  int colh, colj;   // P1 columns per wave (multiples of 16)
};

struct GroupArgs {
  int n, rp, RB;
  int p1_pre[kMaxGroup + 1];      // P1 workgroups: per module (ksh + ksj) x tblk
  int p2_pre[kMaxGroup + 1];      // P2 workgroups: per module (in + out tiles) x kst
  int64_t p3_pre[kMaxGroup + 1];  // P3 elements: r (in + out)
  ProbeDesc d[kMaxGroup];
};

__device__ __forceinline__ int find_module(const int* pre, int n, int bid) {
  int m = 0;
  while (m + 1 < n && bid >= pre[m + 1]) ++m;
  return m;
}

// ---------------------------------------------------------------------------------------
// P1
// ---------------------------------------------------------------------------------------
template <bool F_RK>
__device__ __forceinline__ f32x4 load_f4(const float* F, int64_t K, int r, int j, int64_t k, int64_t k1, bool full) {
  f32x4 f;
  if (F_RK) {
    if (j < r && full) return *reinterpret_cast<const f32x4*>(F + (int64_t)j * K + k);
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = (j < r && k + q < k1) ? F[(int64_t)j * K + k + q] : 0.f;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) f[q] = (j < r && k + q < k1) ? F[(k + q) * r + j] : 0.f;
  }
  return f;
}

// one wave: 16 rows x columns [k0, k1) of Z (T x K) against F -> acc[RB]
//
// Z is read in full 128-byte lines: per 64-column tile each lane loads 4 consecutive
// elements of row 4p + (lane >> 4) at column 4 (lane & 15) (p = 0..3: 4 rows x 256 B per f32
// wave-instruction), stages them in a wave-private padded LDS tile [16][64 + 4] and reads the
// MFMA fragments back (row lane & 15, columns 16 s + 4 (lane >> 4)) with ds_read_b128 -- the
// fragment-shaped global pattern (16 rows x 64 B per instruction) costs 18-45 % (guide sec. 5).
constexpr int kTileLd = 68;  // padded LDS row (floats)

template <int DT, int RB, int U, bool F_RK>
__device__ __forceinline__ void proj_wave(const void* Z, const float* F, int64_t T, int64_t K, int r, int64_t tb,
                                          int64_t k0, int64_t k1, int lane, float* tile, f32x4 (&acc)[RB]) {
  // U = 64-column tiles whose loads are issued together (bytes in flight per wave).
  // r >= 64 (RB >= 4): the F fragments, not Z's access pattern, dominate -> tail path only.
  const int li = lane & 15, g = lane >> 4;
  int64_t k = k0;
  if (RB < 4 && K % 4 == 0) {
    int64_t srow[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) srow[p] = min(tb + 4 * p + g, T - 1) * K;
    for (; k + 64 * U <= k1; k += 64 * U) {
      f32x4 z[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int p = 0; p < 4; ++p) z[u][p] = load4<DT>(Z, srow[p] + k + 64 * u + 4 * li);
      f32x4 f[U][4][RB];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int b = 0; b < RB; ++b)
            f[u][s][b] = load_f4<F_RK>(F, K, r, b * 16 + li, k + 64 * u + 16 * s + 4 * g, k1, true);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float* tl = tile + u * 16 * kTileLd;
#pragma unroll
        for (int p = 0; p < 4; ++p)
          *reinterpret_cast<f32x4*>(tl + (4 * p + g) * kTileLd + 4 * li) = z[u][p];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float* tl = tile + u * 16 * kTileLd;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const f32x4 zf = *reinterpret_cast<const f32x4*>(tl + li * kTileLd + 16 * s + 4 * g);
#pragma unroll
          for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[q], f[u][s][b][q], acc[b], 0, 0, 0);
        }
      }
    }
  }
  const int64_t zrow = min(tb + li, T - 1) * K;
  for (; k < k1; k += 16) {  // tail: guarded 16-column steps, fragment-shaped loads
    const int64_t kq = k + 4 * g;
    const bool full = (k + 16 <= k1) && (K % 4 == 0);
    f32x4 zz;
    if (full) {
      zz = load4<DT>(Z, zrow + kq);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) zz[q] = (kq + q < k1) ? load1<DT>(Z, zrow + kq + q) : 0.f;
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const f32x4 ff = load_f4<F_RK>(F, K, r, b * 16 + li, kq, k1, full);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zz[q], ff[q], acc[b], 0, 0, 0);
    }
  }
}

template <int DT, int RB, int U>
__global__ __launch_bounds__(kP1Waves * 64) void probe_proj_kernel(GroupArgs ga) {
  // LDS: [kP1Waves][16 rows][rp] reduction tiles, then [kP1Waves][U][16][kTileLd] staging
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int m = find_module(ga.p1_pre, ga.n, blockIdx.x);
  const ProbeDesc& d = ga.d[m];
  int loc = blockIdx.x - ga.p1_pre[m];
  const int64_t tblk = (d.T + 15) / 16;
  const int nH = (int)tblk * d.ksh;
  const bool sideH = loc < nH;
  if (!sideH) loc -= nH;
  const int ks_n = sideH ? d.ksh : d.ksj;
  const int64_t K = sideH ? d.in : d.out;
  const int64_t tb = (int64_t)(loc / ks_n) * 16;
  const int ks = loc % ks_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t cols = sideH ? d.colh : d.colj;
  const int64_t k0 = (ks * kP1Waves + wave) * cols;
  const int64_t k1 = min(K, k0 + cols);
  f32x4 acc[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rp = ga.rp, li = lane & 15, g = lane >> 4;
  float* tile = red + kP1Waves * 16 * rp + wave * U * 16 * kTileLd;
  if (k0 < k1) {
    if (sideH) proj_wave<DT, RB, U, true>(d.X, d.A, d.T, K, d.r, tb, k0, k1, lane, tile, acc);
    else if (d.b_t) proj_wave<DT, RB, U, true>(d.G, d.B, d.T, K, d.r, tb, k0, k1, lane, tile, acc);
    else proj_wave<DT, RB, U, false>(d.G, d.B, d.T, K, d.r, tb, k0, k1, lane, tile, acc);
  }
  // reduce the 8 waves' 16 x rp tiles in LDS (fixed order), write one slab row-block
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) red[(wave * 16 + 4 * g + reg) * rp + b * 16 + li] = acc[b][reg];
  __syncthreads();
  float* slab = sideH ? d.slabH : d.slabJ;
  for (int e = threadIdx.x; e < 16 * rp; e += kP1Waves * 64) {
    const int row = e / rp, j = e % rp;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kP1Waves; ++w) s += red[(w * 16 + row) * rp + j];
    const int64_t t = tb + row;
    if (t < d.T) slab[((int64_t)ks * d.T + t) * rp + j] = s;
  }
}

// ---------------------------------------------------------------------------------------
// P2: part[kt] = sum_{t in chunk kt} Y[t][j] Z[t][n],  Y = sum_ks slabY[ks]
//   dA parts [kt][rp][N];  dB parts [kt][N][rp] (so P3 writes B's out x r layout)
// ---------------------------------------------------------------------------------------
template <int DT, int RB>
__global__ __launch_bounds__(512) void probe_outer_kernel(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) float Ys[];  // max([kTC][rp], 4096): Y tile, then half reduce
  const int m = find_module(ga.p2_pre, ga.n, blockIdx.x);
  const ProbeDesc& d = ga.d[m];
  int loc = blockIdx.x - ga.p2_pre[m];
  const int nA = (int)((d.in + kNW - 1) / kNW) * d.kst;
  const bool sideA = loc < nA;  // dA: Y = J, Z = X, N = in;  dB: Y = H, Z = G, N = out
  if (!sideA) loc -= nA;
  const void* Z = sideA ? d.X : d.G;
  const float* slabY = sideA ? d.slabJ : d.slabH;
  const int ksY = sideA ? d.ksj : d.ksh;
  const int64_t N = sideA ? d.in : d.out;
  const int kt = loc % d.kst;
  const int64_t nb = (int64_t)(loc / d.kst) * kNW;
  const int64_t tb = (int64_t)kt * kTC;
  const int rp = ga.rp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  // 1. Y rows [tb, tb + kTC) from the ksY slabs (16-B granules, two independent sums)
  const int r4 = rp / 4;
  for (int e = tid; e < kTC * r4; e += 512) {
    const int tt = e / r4, j = (e % r4) * 4;
    const int64_t t = tb + tt;
    f32x4 s0{0.f, 0.f, 0.f, 0.f}, s1 = s0;
    if (t < d.T) {
      const f32x4* src = reinterpret_cast<const f32x4*>(slabY + t * rp + j);
      const int64_t step4 = d.T * rp / 4;
      int ks = 0;
      for (; ks + 2 <= ksY; ks += 2) {
        s0 += src[ks * step4];
        s1 += src[(ks + 1) * step4];
      }
      if (ks < ksY) s0 += src[ks * step4];
    }
    *reinterpret_cast<f32x4*>(Ys + tt * rp + j) = s0 + s1;
  }
  __syncthreads();
  // 2. wave (half, cg): rows [64 half, 64 half + 64), columns nb + 64 cg + 4 li + q
  const int half = wave >> 2, cg = wave & 3;
  const int64_t ncol = nb + 64 * cg + 4 * li;
  const bool vecN = (N % 4 == 0) && (ncol + 3 < N);
  f32x4 acc[RB][4];
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tlen = (int)min((int64_t)kTC, d.T - tb);
  constexpr int U = RB >= 8 ? 4 : 8;
  for (int tt = 64 * half; tt < 64 * half + 64 && tt < tlen; tt += 4 * U) {
    f32x4 z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = tt + 4 * u + g;
      z[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < tlen) {
        const int64_t base = (tb + row) * N + ncol;
        if (vecN) {
          z[u] = load4<DT>(Z, base);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) z[u][q] = (ncol + q < N) ? load1<DT>(Z, base + q) : 0.f;
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
  // 3. add the two row halves through LDS, one r-block per round (half 1 publishes its
  //    [4 cg][4 q][4 reg][64 lanes] = 4096 floats, half 0 adds); LDS holds >= 4096 floats
  float* X1 = Ys;
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    __syncthreads();  // previous readers of the buffer are done
    if (half == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) X1[((cg * 4 + q) * 4 + reg) * 64 + lane] = acc[b][q][reg];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) acc[b][q][reg] += X1[((cg * 4 + q) * 4 + reg) * 64 + lane];
    }
  }
  if (half == 1) return;
  // lane holds D[j = 16b + 4g + reg][n = ncol + q]
  if (sideA) {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int j = b * 16 + 4 * g + reg;
        float* dst = d.partA + ((int64_t)kt * rp + j) * N + ncol;
        f32x4 v{acc[b][0][reg], acc[b][1][reg], acc[b][2][reg], acc[b][3][reg]};
        if (vecN) {
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (ncol + q < N) dst[q] = v[q];
        }
      }
    }
  } else {
#pragma unroll
    for (int b = 0; b < RB; ++b) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ncol + q >= N) continue;
        float* dst = d.partB + ((int64_t)kt * N + ncol + q) * rp + b * 16 + 4 * g;
        *reinterpret_cast<f32x4*>(dst) = acc[b][q];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// P3: gA[j][n] (+)= s * sum_kt partA[kt][j][n];  gB[n][j] (+)= s * sum_kt partB[kt][n][j]
// ---------------------------------------------------------------------------------------
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

__global__ __launch_bounds__(256) void probe_finish_kernel(GroupArgs ga) {
#pragma clang fp contract(off)  // g + s*sum as two roundings, like autograd's mul then add
  const int64_t total = ga.p3_pre[ga.n];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    int m = 0;
    while (m + 1 < ga.n && e >= ga.p3_pre[m + 1]) ++m;
    const ProbeDesc& d = ga.d[m];
    const int64_t f = e - ga.p3_pre[m];
    const int64_t nA = (int64_t)d.r * d.in;
    if (f < nA) {
      const float s = sum_parts(d.partA + f, (int64_t)ga.rp * d.in, d.kst);  // rows j < r are a prefix
      const float v = d.scale * s;
      d.gA[f] = d.accumulate ? d.gA[f] + v : v;
    } else {
      const int64_t fb = f - nA;
      const int64_t n = fb / d.r, j = fb % d.r;
      const float s = sum_parts(d.partB + n * ga.rp + j, d.out * ga.rp, d.kst);
      const float v = d.scale * s;
      d.gB[fb] = d.accumulate ? d.gB[fb] + v : v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// host planning
// ---------------------------------------------------------------------------------------
static int rb_of(int r) {
  const int rb = (r + 15) / 16;
  return rb <= 1 ? 1 : rb <= 2 ? 2 : rb <= 4 ? 4 : 8;
}

struct ModPlan {
  int ksh, ksj, kst, colh, colj;
  size_t off_slabH, off_slabJ, off_partA, off_partB, bytes;
};

static void p1_split(int64_t K, int& ks, int& cols) {
  const int64_t span = (int64_t)kP1Waves * p1_cols();
  ks = (int)((K + span - 1) / span);
  int64_t c = (K + (int64_t)ks * kP1Waves - 1) / ((int64_t)ks * kP1Waves);
  cols = (int)((c + 15) / 16 * 16);
}

static ModPlan plan_module(int64_t T, int64_t in, int64_t out, int r) {
  ModPlan p;
  const int rp = 16 * rb_of(r);
  p1_split(in, p.ksh, p.colh);
  p1_split(out, p.ksj, p.colj);
  p.kst = (int)((T + kTC - 1) / kTC);
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n * 4 + 255) / 256 * 256; return o; };
  p.off_slabH = take((size_t)p.ksh * T * rp);
  p.off_slabJ = take((size_t)p.ksj * T * rp);
  p.off_partA = take((size_t)p.kst * rp * in);
  p.off_partB = take((size_t)p.kst * rp * out);
  p.bytes = off;
  return p;
}

template <int DT, int RB>
static int launch_group(const GroupArgs& ga, hipStream_t st) {
  const int rp = ga.rp;
  const dim3 g1(ga.p1_pre[ga.n]), b1(kP1Waves * 64);
  auto lds1 = [&](int U) { return (size_t)kP1Waves * (16 * rp + U * 16 * kTileLd) * sizeof(float); };
  if constexpr (RB >= 4) {
    hipLaunchKernelGGL((probe_proj_kernel<DT, RB, 1>), g1, b1, lds1(1), st, ga);
  } else if constexpr (RB == 2) {
    hipLaunchKernelGGL((probe_proj_kernel<DT, RB, 1>), g1, b1, lds1(1), st, ga);
  } else {
    switch (p1_u()) {
      case 1: hipLaunchKernelGGL((probe_proj_kernel<DT, RB, 1>), g1, b1, lds1(1), st, ga); break;
      case 3: hipLaunchKernelGGL((probe_proj_kernel<DT, RB, 3>), g1, b1, lds1(3), st, ga); break;
      default: hipLaunchKernelGGL((probe_proj_kernel<DT, RB, 2>), g1, b1, lds1(2), st, ga); break;
    }
  }
  HDP_CHECK_LAUNCH();
  hipLaunchKernelGGL((probe_outer_kernel<DT, RB>), dim3(ga.p2_pre[ga.n]), dim3(512),
                     (size_t)(kTC * rp > 4096 ? kTC * rp : 4096) * sizeof(float), st, ga);
  HDP_CHECK_LAUNCH();
  const int64_t tot = ga.p3_pre[ga.n];
  const int blocks = (int)min((int64_t)4096, (tot + 255) / 256);
  hipLaunchKernelGGL(probe_finish_kernel, dim3(blocks), dim3(256), 0, st, ga);
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}

}  // namespace hdp

using namespace hdp;

extern "C" size_t hdp_probe_workspace_bytes(int64_t T, int64_t in, int64_t out, int r) {
  if (T <= 0 || in <= 0 || out <= 0 || r <= 0 || r > 128) return 0;
  return plan_module(T, in, out, r).bytes;
}

extern "C" int hdp_probe_group_max(void) { return kMaxGroup; }

extern "C" int hdp_probe_grads_group(int n, const hdp_probe_item* items, int x_dtype, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  HDP_CHECK_ARG(n >= 0 && n <= kMaxGroup, "hdp_probe_grads_group: n = %d not in [0, %d]", n, kMaxGroup);
  HDP_CHECK_ARG(x_dtype == HDP_F32 || x_dtype == HDP_BF16, "hdp_probe_grads_group: bad dtype %d", x_dtype);
  if (n == 0) return HDP_OK;
  HDP_CHECK_ARG(items != nullptr, "hdp_probe_grads_group: null items");
  hipStream_t st = as_stream(stream);
  GroupArgs ga;
  ga.n = 0;
  ga.RB = rb_of(items[0].r);
  ga.rp = 16 * ga.RB;
  ga.p1_pre[0] = ga.p2_pre[0] = 0;
  ga.p3_pre[0] = 0;
  size_t off = 0;
  char* ws = reinterpret_cast<char*>(workspace);
  for (int i = 0; i < n; ++i) {
    const hdp_probe_item& it = items[i];
    HDP_CHECK_ARG(it.in > 0 && it.out > 0 && it.r > 0 && it.T >= 0, "hdp_probe_grads: bad shape (item %d)", i);
    HDP_CHECK_ARG(it.r <= 128, "hdp_probe_grads: r = %d > 128 is not supported", it.r);
    HDP_CHECK_ARG(rb_of(it.r) == ga.RB, "hdp_probe_grads_group: items of one group need the same r-block");
    HDP_CHECK_ARG(it.A && it.B && it.gA && it.gB, "hdp_probe_grads: null pointer (item %d)", i);
    for (int k = 0; k < i; ++k)
      HDP_CHECK_ARG(items[k].gA != it.gA && items[k].gB != it.gB,
                    "hdp_probe_grads_group: items %d and %d accumulate into the same gradient", k, i);
    if (it.T == 0) {
      if (!it.accumulate) {
        HDP_CHECK_HIP(hipMemsetAsync(it.gA, 0, sizeof(float) * it.r * it.in, st));
        HDP_CHECK_HIP(hipMemsetAsync(it.gB, 0, sizeof(float) * it.r * it.out, st));
      }
      continue;
    }
    HDP_CHECK_ARG(it.X && it.G && workspace, "hdp_probe_grads: null pointer (item %d)", i);
    HDP_CHECK_ARG((reinterpret_cast<uintptr_t>(it.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(it.X) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(it.G) & 15) == 0 &&
                      (!it.b_transposed || (reinterpret_cast<uintptr_t>(it.B) & 15) == 0),
                  "hdp_probe_grads: X, G, A (and B^T) must be 16-byte aligned (item %d)", i);
    const ModPlan p = plan_module(it.T, it.in, it.out, it.r);
    HDP_CHECK_ARG(off + p.bytes <= workspace_bytes, "hdp_probe_grads: workspace %zu bytes too small (need %zu)",
                  workspace_bytes, off + p.bytes);
    ProbeDesc& d = ga.d[ga.n];
    d.X = it.X;
    d.G = it.G;
    d.A = it.A;
    d.B = it.B;
    d.gA = it.gA;
    d.gB = it.gB;
    d.slabH = reinterpret_cast<float*>(ws + off + p.off_slabH);
    d.slabJ = reinterpret_cast<float*>(ws + off + p.off_slabJ);
    d.partA = reinterpret_cast<float*>(ws + off + p.off_partA);
    d.partB = reinterpret_cast<float*>(ws + off + p.off_partB);
    d.T = it.T;
    d.in = it.in;
    d.out = it.out;
    d.scale = it.scale;
    d.r = it.r;
    d.b_t = it.b_transposed ? 1 : 0;
    d.accumulate = it.accumulate ? 1 : 0;
    d.ksh = p.ksh;
    d.ksj = p.ksj;
    d.kst = p.kst;
    d.colh = p.colh;
    d.colj = p.colj;
    off += p.bytes;
    const int64_t tblk = (it.T + 15) / 16;
    const int64_t w1 = tblk * (p.ksh + p.ksj);
    const int64_t w2 = ((it.in + kNW - 1) / kNW + (it.out + kNW - 1) / kNW) * p.kst;
    HDP_CHECK_ARG(ga.p1_pre[ga.n] + w1 < (1ll << 31) && ga.p2_pre[ga.n] + w2 < (1ll << 31),
                  "hdp_probe_grads_group: grid too large");
    ga.p1_pre[ga.n + 1] = ga.p1_pre[ga.n] + (int)w1;
    ga.p2_pre[ga.n + 1] = ga.p2_pre[ga.n] + (int)w2;
    ga.p3_pre[ga.n + 1] = ga.p3_pre[ga.n] + (int64_t)it.r * (it.in + it.out);
    ++ga.n;
  }
  if (ga.n == 0) return HDP_OK;
#define HDP_PROBE(D, R) return launch_group<D, R>(ga, st)
  if (x_dtype == HDP_F32) {
    switch (ga.RB) {
      case 1: HDP_PROBE(HDP_F32, 1);
      case 2: HDP_PROBE(HDP_F32, 2);
      case 4: HDP_PROBE(HDP_F32, 4);
      default: HDP_PROBE(HDP_F32, 8);
    }
  } else {
    switch (ga.RB) {
      case 1: HDP_PROBE(HDP_BF16, 1);
      case 2: HDP_PROBE(HDP_BF16, 2);
      case 4: HDP_PROBE(HDP_BF16, 4);
      default: HDP_PROBE(HDP_BF16, 8);
    }
  }
#undef HDP_PROBE
}

extern "C" int hdp_probe_grads(int64_t T, int64_t in, int64_t out, int r, const void* X, const void* G,
                               int x_dtype, const float* A, const float* B, int b_transposed, float* gA, float* gB,
                               float scale, int accumulate, void* workspace, size_t workspace_bytes, void* stream) {
  HDP_CHECK_ARG(in > 0 && out > 0 && r > 0 && T >= 0, "hdp_probe_grads: bad shape");
  HDP_CHECK_ARG(r <= 128, "hdp_probe_grads: r = %d > 128 is not supported", r);
  hdp_probe_item it;
  it.X = X;
  it.G = G;
  it.A = A;
  it.B = B;
  it.gA = gA;
  it.gB = gB;
  it.T = T;
  it.in = in;
  it.out = out;
  it.r = r;
  it.b_transposed = b_transposed;
  it.scale = scale;
  it.accumulate = accumulate;
  return hdp_probe_grads_group(1, &it, x_dtype, workspace, workspace_bytes, stream);
}
