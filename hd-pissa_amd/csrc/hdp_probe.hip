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
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "hdp_probe_int.h"

namespace hdp {

constexpr int kMaxGroup = 1024;  // modules per group (sweep path: device descriptor tables)
constexpr int kMaxSplit = 16;  // split path: GroupArgs (kernel arguments, by value) near 2.6 KB
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

template <int CAP>
struct GroupArgsT {
  int n, rp, RB;
  int p1_pre[CAP + 1];      // P1 workgroups: per module (ksh + ksj) x tblk
  int p2_pre[CAP + 1];      // P2 workgroups: per module (in + out tiles) x kst
  int64_t p3_pre[CAP + 1];  // P3 elements: r (in + out)
  ProbeDesc d[CAP];
};
using GroupArgs = GroupArgsT<kMaxSplit>;  // split-path kernel arguments
static_assert(sizeof(GroupArgs) <= 4096, "split-path kernel arguments must stay within 4 KB");

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
// kTileLd (hdp_probe_int.h): padded LDS row (floats): conflict-free 16-B writes and fragment reads

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

// P3 with the module from blockIdx.y and 4 consecutive elements per thread (16-B loads of the parts and
// of g; side A: same j, n..n+3; side B: same n, j..j+3): same per-element summation order as above.
// The host takes it when every module has r % 4 == 0, in % 4 == 0 and 16-B aligned gradients.
__global__ __launch_bounds__(256) void probe_finish4_kernel(GroupArgs ga) {
#pragma clang fp contract(off)
  const int m = blockIdx.y;
  const ProbeDesc& d = ga.d[m];
  const int64_t f = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t nA = (int64_t)d.r * d.in;
  if (f >= nA + (int64_t)d.r * d.out) return;
  const bool sideA = f < nA;
  const float* p;
  int64_t stride;
  if (sideA) {
    p = d.partA + f;  // rows j < r of [kt][rp][in] are a prefix
    stride = (int64_t)ga.rp * d.in;
  } else {
    const int64_t fb = f - nA, n = fb / d.r, j = fb % d.r;
    p = d.partB + n * ga.rp + j;
    stride = d.out * ga.rp;
  }
  f32x4 s0{0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
  int k = 0;
  for (; k + 4 <= d.kst; k += 4) {
    s0 += gld4(p + (k + 0) * stride);
    s1 += gld4(p + (k + 1) * stride);
    s2 += gld4(p + (k + 2) * stride);
    s3 += gld4(p + (k + 3) * stride);
  }
  for (; k < d.kst; ++k) s0 += gld4(p + k * stride);
  const f32x4 v = d.scale * ((s0 + s1) + (s2 + s3));
  float* g = sideA ? d.gA + f : d.gB + (f - nA);
  gst4(g, d.accumulate ? gld4(g) + v : v);
}

// ---------------------------------------------------------------------------------------
// SWEEP path (r <= 32): X and G are each a row-major stream "Z" (T x N).  A sweep kernel walks
// 16-row steps of 512-column stripes of Z and can do, from the SAME registers:
//   PROJ : slab_out[ct][t][j] = sum_{n in stripe ct} Z[t][n] F[j][n]      (H = X A^T or J = G B)
//   OUTER: piece[ct][k][j][n] = sum_{t in segment k} Y[t][j] Z[t][n]      (J^T X or H^T G)
// with Y = the other stream's projection (slabs summed by probe_yreduce_kernel).  Per module,
// S1 = the smaller of X, G:
//   phase A  PROJ  over S1                       (reads S1)
//   R1       Y_S1 = sum of S1's slabs
//   phase B  PROJ + OUTER over S2 (Y_S1)         (reads S2 once for both of its products)
//   R2       Y_S2 = sum of S2's slabs
//   phase C  OUTER over S1 (Y_S2)                (re-reads S1)
//   phase D  probe_sweep_finish_kernel: g (+)= s * sum of pieces
// => X + G + min(X, G) bytes per module instead of 2 (X + G) for the P1/P2 split.
//
// PERSISTENT schedule: a launch has exactly G resident workgroups (occupancy x CUs, capped so
// each gets >= kSwMinSteps steps); the U steps of the group, flattened as (module, stripe,
// row step), are split into G equal contiguous ranges -- no tail quantization, one launch per
// phase however large the group.  A workgroup's range crosses few stripes; OUTER accumulators
// live in registers over a stripe segment and are flushed as one piece per segment.
//
// Workgroup: 8 waves, each owning 64 columns of the stripe.  A lane loads 4 consecutive columns
// of rows 4p + g (full 128-B lines), which are directly the OUTER MFMA's B operand.  PROJ re-
// reads them as A-operand fragments through a wave-private padded LDS tile against F fragments
// held in registers for the segment; the 8 waves' 16-row partials are summed through a
// double-buffered LDS area (one barrier per step).  Rows are clamped to T - 1 and columns to
// N - 4 (rows past T meet zero Y and unwritten slab rows; columns past N meet zero F and
// unwritten pieces), so the loop is branch-free; loads run two steps ahead with three register
// sets in fixed roles.
// ---------------------------------------------------------------------------------------
constexpr int kSwMinSteps = 8;       // >= 128 rows per workgroup: bounds the pieces per stripe
// bf16 activations on bf16 MFMA (v_mfma_f32_16x16x16_bf16): X and G are exact in bf16, the f32 operand
// (a factor fragment, or a row of the other stream's projection) is split exactly into three bf16
// parts v = hi + mid + lo (24 significant bits), and the MFMA sums the three exact products in f32 --
// the error of the f32 chain it replaces, at 3 MFMAs of 16x16x16 bf16 instead of 4 of 16x16x4 f32
// (5.3x the rate).  Operand maps: lane l holds A[i = l & 15][k = 4 (l >> 4) + e] and
// B[k = 4 (l >> 4) + e][j = l & 15], e = 0..3; the result layout equals the 16x16x4 f32 one, so
// k = 4 g + e can stand for row 16 s + 4 e + g (OUTER: the rows as loaded, no data movement) or for
// column 16 ss + 4 g + e (PROJ: the transposed tile as read).
typedef short bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3(const f32x4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint16_t a = f32_to_bf16(v[e]);
    const float r1 = v[e] - bf16_to_f32(a);
    const uint16_t b = f32_to_bf16(r1);
    h[e] = (short)a;
    m[e] = (short)b;
    l[e] = (short)f32_to_bf16(r1 - bf16_to_f32(b));
  }
}
// an f32 holding a bf16 value (bf16 data as loaded) back to its exact bits
__device__ __forceinline__ short bf16_bits(float v) { return (short)(__float_as_uint(v) >> 16); }
// K32 forms (v_mfma_f32_16x16x32_bf16: twice the k per instruction of 16x16x16 at about the same
// cycles -- tools/mfma_rate.hip: 1.89 vs 0.88 PFLOP/s): lane l holds A[i = l & 15][k = 8 (l >> 4) + e]
// and B[k = 8 (l >> 4) + e][j = l & 15], e = 0..7; the result layout is the 16x16x4 / 16x16x16 one
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // exact: v = h + m + l (24 significant bits)
    const __bf16 a = (__bf16)v[e];
    const float r1 = v[e] - (float)a;
    const __bf16 b = (__bf16)r1;
    h[e] = a;
    m[e] = b;
    l[e] = (__bf16)(r1 - (float)b);
  }
}
// an f32 holding a bf16 value back to __bf16 (exact)
__device__ __forceinline__ __bf16 as_bf16(float v) { return __builtin_bit_cast(__bf16, bf16_bits(v)); }
// the same exact 3-way split on packed conversions (two values per v_cvt_pk_bf16_f32): the float32
// activations of the X6 forms are split per step, the factors once per segment
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split8p(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma clang fp contract(off)
  u32x4s H, M, L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float a0 = v[2 * e], a1 = v[2 * e + 1];
    const uint32_t ph = cvt_pk_bf16(a0, a1);
    const float r0 = a0 - __uint_as_float(ph << 16), r1 = a1 - __uint_as_float(ph & 0xffff0000u);
    const uint32_t pm = cvt_pk_bf16(r0, r1);
    const float s0 = r0 - __uint_as_float(pm << 16), s1 = r1 - __uint_as_float(pm & 0xffff0000u);
    H[e] = ph;
    M[e] = pm;
    L[e] = cvt_pk_bf16(s0, s1);
  }
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}
// x y for x, y split exactly into 3 bf16 parts: the six partial products that reach f32 resolution
// (hi hi, hi mid, mid hi, hi lo, lo hi, mid mid; the dropped ones are below 2^-24 relative) -- the K4
// MX3 scheme on v_mfma_f32_16x16x32_bf16, 6 x 16 cycles per 32 k where f32 MFMA takes 8 x 32
__device__ __forceinline__ f32x4 mfma_x6(const bf16x8 (&x)[3], const bf16x8 (&y)[3], f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[2], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[1], c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[0], c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

constexpr int kSwRedBufs = 4;        // PROJ partial buffers in rotation (arrival-counter hand-off)
// r = 64 (RB = 4): two buffers keep the PROJ LDS at 101 KB (four would exceed the 160 KB of a CU);
// the shared-X instance (FUSE, 4 r-blocks of up to 4 modules): three (132 KB)
template <int RB, bool FUSE = false>
constexpr int sw_nbuf() { return FUSE ? 3 : RB >= 4 ? 2 : kSwRedBufs; }
constexpr int kSwMaxBlk = 4;         // r-blocks of one stream side (FUSE: of all modules sharing its X)
#ifndef HDP_BF_SETS
#define HDP_BF_SETS 3
#endif
constexpr int kBfSets = HDP_BF_SETS;  // register sets of the bf16 PROJ phases (loads kBfSets - 1 steps ahead)
enum { kSwProj = 1, kSwOuter = 2 };

struct SweepDesc {
  const void* Z;          // T x N, row-major, x_dtype
  const float* F;         // f_rk: F[j][n] at j * N + n (A, B^T);  else F[n][j] at n * r + j (B)
  float* slab_out;        // PROJ:  [nct][T][rp] stripe partials of Z F^T
  const float* y_in;      // OUTER: the other stream's projection, row t at y_in + t * yrs, a lane's
                          //        RB values at + li * yls (probe_yreduce_kernel's layout)
  float* part;            // OUTER: [nct][kmax][rp][kSwC]  or  [nct][kmax][kSwC][rp] (part_t)
  int64_t T, N, pre;      // pre: first flattened step of this module side
  int r, f_rk, part_t, nct, S, kmax;  // S = 16-row steps per stripe
  // OUTER, a stripe covered by ONE workgroup segment: its gradient block written directly,
  // g (+)= scale * acc (part_t 0: gA [r][N]; 1: gB [N][ldb]); the finish pass skips it
  float* g;
  float scale;
  int acc, ldb;
  int yrs, yls;           // Y row / lane strides (floats)
  // Shared-X instances (FUSE): the side is r-block-wise -- nb blocks of 16 rows, block b possibly of
  // another module that reads the same X (q/k/v, gate/up).  Block b: F rows Fb[b] (rbr[b] of them),
  // slab columns slab_b[b] and pieces part_b[b] (row strides rpm = the members' 16 RB), gradient
  // rows gb[b] with scale sc[b] / accumulate accb[b].
  int nb, rpm;
  const float* Fb[kSwMaxBlk];
  float* slab_b[kSwMaxBlk];
  float* part_b[kSwMaxBlk];
  float* gb[kSwMaxBlk];
  float sc[kSwMaxBlk];
  int rbr[kSwMaxBlk], accb[kSwMaxBlk];
};

// g (+)= s * acc for this wave's columns of one stripe (the finish kernel's arithmetic on a single
// piece: s * (piece + 0) == s * piece, then g + v as two roundings)
template <int RB>
__device__ __forceinline__ void sw_store_g(const SweepDesc& d, const f32x4 (&acc2)[RB][4], int64_t col, int g,
                                           bool vec) {
#pragma clang fp contract(off)
  const float sc = d.scale;
  const int r = d.r;
  const int64_t N = d.N;
  if (!d.part_t) {  // gA [r][N]: row j = 16 b + 4 g + reg, columns col .. col + 3
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int j = 16 * b + 4 * g + reg;
        if (j >= r) continue;
        float* p = d.g + (int64_t)j * N + col;
        const f32x4 v{sc * acc2[b][0][reg], sc * acc2[b][1][reg], sc * acc2[b][2][reg], sc * acc2[b][3][reg]};
        if (vec) {
          gst4(p, d.acc ? gld4(p) + v : v);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (col + q < N) gst1(p + q, d.acc ? gld1(p + q) + v[q] : v[q]);
        }
      }
  } else {  // gB [N][ldb]: row n = col + q, columns j = 16 b + 4 g .. + 3
    const bool v4 = (d.ldb & 3) == 0 && (reinterpret_cast<uintptr_t>(d.g) & 15) == 0;
#pragma unroll
    for (int b = 0; b < RB; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (col + q >= N) continue;
        const int j0 = 16 * b + 4 * g;
        float* p = d.g + (col + q) * d.ldb + j0;
        const f32x4 v = sc * acc2[b][q];
        if (v4 && j0 + 3 < r) {
          gst4(p, d.acc ? gld4(p) + v : v);
        } else {
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            if (j0 + reg < r) gst1(p + reg, d.acc ? gld1(p + reg) + v[reg] : v[reg]);
        }
      }
  }
}

// the same for a FUSE side: gA rows per r-block (block b = 16 rows of module Fb's gradient gb[b]); a
// part_t side (gB, never shared) as sw_store_g over its nb blocks
__device__ __forceinline__ void sw_store_g_fuse(const SweepDesc& d, const f32x4 (&acc2)[kSwMaxBlk][4], int64_t col,
                                                int g, bool vec) {
#pragma clang fp contract(off)
  const int64_t N = d.N;
  if (!d.part_t) {
#pragma unroll
    for (int b = 0; b < kSwMaxBlk; ++b) {
      if (b >= d.nb) break;
      const float sc = d.sc[b];
      const int acc = d.accb[b];
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int j = 4 * g + reg;
        if (j >= d.rbr[b]) continue;
        float* p = d.gb[b] + (int64_t)j * N + col;
        const f32x4 v{sc * acc2[b][0][reg], sc * acc2[b][1][reg], sc * acc2[b][2][reg], sc * acc2[b][3][reg]};
        if (vec) {
          gst4(p, acc ? gld4(p) + v : v);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (col + q < N) gst1(p + q, acc ? gld1(p + q) + v[q] : v[q]);
        }
      }
    }
  } else {
    const float sc = d.scale;
    const int r = d.r;
    const bool v4 = (d.ldb & 3) == 0 && (reinterpret_cast<uintptr_t>(d.g) & 15) == 0;
#pragma unroll
    for (int b = 0; b < kSwMaxBlk; ++b) {
      if (b >= d.nb) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (col + q >= N) continue;
        const int j0 = 16 * b + 4 * g;
        float* p = d.g + (col + q) * d.ldb + j0;
        const f32x4 v = sc * acc2[b][q];
        if (v4 && j0 + 3 < r) {
          gst4(p, d.acc ? gld4(p) + v : v);
        } else {
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            if (j0 + reg < r) gst1(p + reg, d.acc ? gld1(p + reg) + v[reg] : v[reg]);
        }
      }
    }
  }
}

// Kernel arguments stay small (a few pointers): a group's descriptors live in a device table
// uploaded once per flush (probe_tables_upload), so a group can hold every module of a
// backward pass (hundreds) instead of what 4 KB of kernel arguments allowed (32).
struct SweepArgs {
  int n, G;
  int spin;       // bound of one PROJ hand-off wait (sleeps); < 0 = fail every wait (test knob, HDP_PROBE_SPIN)
  int64_t U;      // total steps
  int* err;       // device error word (host-mapped): set when a hand-off wait gives up
  int* errd;      // its device-memory copy (set together): what K3 reads in stream order (L2, not PCIe)
  const SweepDesc* d;  // [n] this phase's module sides (device)
  const int* wst;      // [3 G] where workgroup w starts: module, stripe, step (device; host-planned)
};

__device__ __forceinline__ int64_t sw_lo(int w, int64_t U, int G) { return (int64_t)w * U / G; }
// the workgroup whose range holds step u: the largest w with sw_lo(w) <= u
__device__ __forceinline__ int sw_owner(int64_t u, int64_t U, int G) { return (int)(((u + 1) * G - 1) / U); }

// one stripe segment: steps [s0, s0 + n) of stripe ct of d.  `i0` = the workgroup's step count
// before it (parity of the PROJ reduction buffer).  Steps whose 16 rows are all < T run a
// pipelined loop on incremented pointers; a final partial step (T % 16 != 0) is clamped.
// OCC = resident workgroups per CU the kernel is built for: 1 (two steps of loads in flight,
// three register sets) or 2 (one step in flight, two sets: <= 128 VGPRs, 16 waves per CU)
template <int DT, int RB, int MODE, bool VEC, int OCC, bool FUSE, bool K32>
__device__ __forceinline__ void sweep_segment(const SweepDesc& d, int ct, int s0, int n, int64_t i0, int w,
                                              const SweepArgs& sa, float* tile, float* red, int* flags, int wave,
                                              int lane) {
  constexpr bool PROJ = (MODE & kSwProj) != 0, OUTER = (MODE & kSwOuter) != 0;
  constexpr int rp = 16 * RB, r4 = rp / 4, ES = DT == HDP_F32 ? 4 : 2;
  const int li = lane & 15, g = lane >> 4;
  const int64_t T = d.T, N = d.N;
  const int64_t c = (int64_t)ct * kSwC + 64 * wave;  // this wave's 64 columns
  const int64_t col = c + 4 * li;
  const int64_t colc = VEC ? (col < N ? col : N - 4) : col;
  const char* Zb = reinterpret_cast<const char*>(d.Z);

  // bf16 data, PROJ-only phase: the fragments split once into hi / mid / lo for bf16 MFMA; with OUTER
  // in the same phase (B) the split fragments would not fit beside the accumulators: f32 MFMA there
  constexpr bool SPLIT_F = DT == HDP_BF16 && MODE == kSwProj;
  // K32 (bf16 activations): PROJ over 32-column chunks, OUTER over PAIRS of 16-row steps (the 8 k of
  // a lane = its 4 rows of each step), both on v_mfma_f32_16x16x32_bf16.  X6 (float32 activations, r04):
  // the same forms with the activations split exactly into 3 bf16 parts as well, 6 products per 32 k
  // (mfma_x6) instead of 8 v_mfma_f32_16x16x4_f32 of twice the cycles
  constexpr bool X6 = K32 && DT == HDP_F32;
  constexpr bool K32P = K32 && MODE == kSwProj, K32O = K32 && MODE == kSwOuter;
  // DL (r04): bf16 PROJ-only phases load Z straight in the 16x16x32 A-operand layout -- lane (li, g) reads row
  // 16 s + li, columns c + 32 ch + 8 g .. + 7 as one 16-B load per ch (z[ch] holds the 8 bf16 bits) -- instead of
  // 4 rows x 4 columns per lane transposed through the LDS tile (the tile store + read was 20 % of these phases,
  // tools/probe_ablate.py notile).  VEC for bf16 means rows of whole 16-B granules (host).
  constexpr bool DL = K32P && DT == HDP_BF16 && !X6 && VEC;
  // the lane's two DL column groups, clamped to the row (columns past N meet zero factor fragments)
  const int64_t cdl0 = c + 8 * g < N ? c + 8 * g : N - 8, cdl1 = c + 32 + 8 * g < N ? c + 32 + 8 * g : N - 8;
  f32x4 f[K32P ? 1 : 4][RB];
  bf16x4 fs[K32P ? 1 : 4][RB][3];
  bf16x8 fs8[K32P ? 2 : 1][RB][3];
  if constexpr (K32P) {  // fs8[ch][b] = split of F[j = 16 b + li][c + 32 ch + 8 g + e], e = 0..7
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int j = 16 * b + li;
        const int64_t k = c + 32 * ch + 8 * g;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
        const float* Fp = nullptr;
        int rows = d.r;
        if constexpr (FUSE) {
          Fp = b < d.nb ? d.Fb[b] : nullptr;
          rows = b < d.nb ? d.rbr[b] : 0;
        }
        const bool ok = FUSE ? (Fp != nullptr && li < rows) : (j < d.r);
        if (ok) {
          if (FUSE) Fp += (int64_t)li * N;
          if ((FUSE || d.f_rk) && N % 4 == 0 && k + 7 < N) {
            const float* P = FUSE ? Fp : d.F + (int64_t)j * N;
            const f32x4 a = gld4(P + k), bq = gld4(P + k + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = a[e];
              v[4 + e] = bq[e];
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (k + e < N)
                v[e] = FUSE ? gld1(Fp + k + e)
                            : d.f_rk ? gld1(d.F + (int64_t)j * N + k + e) : gld1(d.F + (k + e) * d.r + j);
          }
        }
        split8(v, fs8[ch][b][0], fs8[ch][b][1], fs8[ch][b][2]);
#pragma unroll
        for (int t = 0; t < 3; ++t) asm volatile("" : "+v"(fs8[ch][b][t]));
      }
  }
  if constexpr (PROJ && !K32P) {  // this stripe's F fragments: f[s][b] = F[j = 16 b + li][c + 16 s + 4 g + q]
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const int j = 16 * b + li;
        const int64_t k = c + 16 * s + 4 * g;
        f32x4 v{0.f, 0.f, 0.f, 0.f};
        if constexpr (FUSE) {  // block b's rows: F rows of the module owning it (row-major, f_rk)
          if (b < d.nb && li < d.rbr[b]) {
            const float* Fp = d.Fb[b] + (int64_t)li * N;
            if (N % 4 == 0 && k + 3 < N) {
              v = gld4(Fp + k);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q)
                if (k + q < N) v[q] = gld1(Fp + k + q);
            }
          }
        } else if (j < d.r) {
          if (d.f_rk && N % 4 == 0 && k + 3 < N) {
            v = gld4(d.F + (int64_t)j * N + k);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (k + q < N) v[q] = d.f_rk ? gld1(d.F + (int64_t)j * N + k + q) : gld1(d.F + (k + q) * d.r + j);
          }
        }
        f[s][b] = v;
      }
    // consume the fragments here: otherwise the compiler cannot prove them landed later and
    // waits vmcnt(0) on every step
    if constexpr (SPLIT_F) {  // split once per segment (F is constant)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
          split3(f[s][b], fs[s][b][0], fs[s][b][1], fs[s][b][2]);
#pragma unroll
          for (int t = 0; t < 3; ++t) asm volatile("" : "+v"(fs[s][b][t]));
        }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int b = 0; b < RB; ++b) asm volatile("" : "+v"(f[s][b]));
    }
  }
  bool hs_broken = false;  // set once a hand-off wait gave up (reported through sa.err; no more waits)
  f32x4 acc2[OUTER ? RB : 1][4];
#pragma unroll
  for (int b = 0; b < (OUTER ? RB : 1); ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc2[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};

  // PROJ hand-off at r-block >= 4 without FUSE (r04): every wave sums ITS slice (2 of the 16 rows) of a step's 8
  // partials one step later, instead of the last-arriving wave summing all of them (32 dependent LDS reads per
  // lane on one wave: the bf16 r = 64 / 128 phases A / B ran 30 % faster with that sum removed,
  // tools/probe_ablate.py noreduce).  Same fixed wave order per element: the same bits.
  constexpr bool DIST = PROJ && !FUSE && RB >= 4;
  int pend_i = -1, pend_s = 0;
  bool pend_tail = false;
  // bounded wait for *p >= target (a wait that gives up is REPORTED, as below)
  auto wait_ge = [&](const int* p, int target) {
    if (hs_broken) return;
    int it = 0;
    while (sa.spin < 0 || __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
      if (it++ >= sa.spin) {
        hs_broken = true;
        if (lane == 0) {
          __hip_atomic_store(sa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(sa.errd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
  };
  // this wave's slice of step pi: rows 2 wave, 2 wave + 1, one float pair per lane
  auto reduce_slice = [&](int pi, int ps, bool ptail) {
    if constexpr (DIST) {
      constexpr int NB = sw_nbuf<RB, FUSE>();
      const int pb = pi % NB, pr = pi / NB;
      wait_ge(flags + pb, kSwWaves * (pr + 1));  // every partial of step pi is in LDS
      const float* rs = red + pb * kSwWaves * 16 * rp;
      const int idx = 2 * lane;
      if (idx < 2 * rp) {
        const int row = 2 * wave + idx / rp, j = idx % rp;
        typedef float f32x2s __attribute__((ext_vector_type(2)));
        f32x2s acc{0.f, 0.f};
#pragma unroll
        for (int ww = 0; ww < kSwWaves; ++ww) acc += *reinterpret_cast<const f32x2s*>(rs + (ww * 16 + row) * rp + j);
        const int64_t t = 16 * (int64_t)ps + row;
        if (!ptail || t < T) *reinterpret_cast<HDP_GLOBAL f32x2s*>(gptr(d.slab_out + ((int64_t)ct * T + t) * rp + j)) = acc;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slice is read: count it
      if (lane == 0) (void)__hip_atomic_fetch_add(flags + NB + pb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };

  // one step of compute on registers z (rows 16 s + 4 p + g) / y; `i` = the workgroup's step index
  auto compute = [&](const f32x4 (&z)[4], const float (&y)[4][RB], int s, int64_t i, bool tail) {
    if constexpr (OUTER) {
      if constexpr (DT == HDP_BF16) {
        // k = 4 g + e <-> row 16 s + 4 e + g: the four loaded rows are one bf16 operand (exact)
#pragma unroll
        for (int b = 0; b < RB; ++b) {
          if (FUSE && b >= d.nb) break;
          f32x4 yv;
#pragma unroll
          for (int p = 0; p < 4; ++p) yv[p] = (!tail || 16 * (int64_t)s + 4 * p + g < T) ? y[p][b] : 0.f;
          bf16x4 yh, ym, yl;
          split3(yv, yh, ym, yl);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bf16x4 zb{bf16_bits(z[0][q]), bf16_bits(z[1][q]), bf16_bits(z[2][q]), bf16_bits(z[3][q])};
            acc2[b][q] = mfma_bf16(yl, zb, acc2[b][q]);
            acc2[b][q] = mfma_bf16(ym, zb, acc2[b][q]);
            acc2[b][q] = mfma_bf16(yh, zb, acc2[b][q]);
          }
        }
      } else {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const bool rok = !tail || 16 * (int64_t)s + 4 * p + g < T;
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            if (FUSE && b >= d.nb) break;
            const float yv = rok ? y[p][b] : 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) acc2[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(yv, z[p][q], acc2[b][q], 0, 0, 0);
          }
        }
      }
    }
    if constexpr (PROJ) {
#pragma unroll
      for (int p = 0; p < (DL ? 0 : 4); ++p) *reinterpret_cast<f32x4*>(tile + (4 * p + g) * kTileLd + 4 * li) = z[p];
      f32x4 a0[RB], a1[RB];
#pragma unroll
      for (int b = 0; b < RB; ++b) a0[b] = a1[b] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (K32P) {
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {  // row li, columns 32 ch + 8 g .. + 7
          f32x4 lo4{0.f, 0.f, 0.f, 0.f}, hi4{0.f, 0.f, 0.f, 0.f};
          if constexpr (!DL) {
            lo4 = *reinterpret_cast<const f32x4*>(tile + li * kTileLd + 32 * ch + 8 * g);
            hi4 = *reinterpret_cast<const f32x4*>(tile + li * kTileLd + 32 * ch + 8 * g + 4);
          }
          if constexpr (X6) {  // float32 values: split exactly, 6 products
            const float zv[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            bf16x8 zs[3];
            split8p(zv, zs[0], zs[1], zs[2]);
#pragma unroll
            for (int b = 0; b < RB; ++b) {
              if (FUSE && b >= d.nb) break;
              f32x4& a = ch ? a1[b] : a0[b];
              a = mfma_x6(zs, fs8[ch][b], a);
            }
          } else {  // bf16 values: exact as they are
            bf16x8 zb;
            if constexpr (DL) {
              zb = __builtin_bit_cast(bf16x8, z[ch]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                zb[e] = as_bf16(lo4[e]);
                zb[4 + e] = as_bf16(hi4[e]);
              }
            }
#pragma unroll
            for (int b = 0; b < RB; ++b) {
              if (FUSE && b >= d.nb) break;
              f32x4& a = ch ? a1[b] : a0[b];
              a = mfma32(zb, fs8[ch][b][2], a);
              a = mfma32(zb, fs8[ch][b][1], a);
              a = mfma32(zb, fs8[ch][b][0], a);
            }
          }
        }
      }
#pragma unroll
      for (int ss = 0; ss < (K32P ? 0 : 4); ++ss) {
        const f32x4 zf = *reinterpret_cast<const f32x4*>(tile + li * kTileLd + 16 * ss + 4 * g);
        if constexpr (SPLIT_F) {
          const bf16x4 zb{bf16_bits(zf[0]), bf16_bits(zf[1]), bf16_bits(zf[2]), bf16_bits(zf[3])};
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            if (FUSE && b >= d.nb) break;
            f32x4& a = (ss & 1) ? a1[b] : a0[b];
            a = mfma_bf16(zb, fs[ss][b][2], a);
            a = mfma_bf16(zb, fs[ss][b][1], a);
            a = mfma_bf16(zb, fs[ss][b][0], a);
          }
        } else {
#pragma unroll
          for (int b = 0; b < RB; ++b) {
            if (FUSE && b >= d.nb) break;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (ss & 1) a1[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[q], f[ss][b][q], a1[b], 0, 0, 0);
              else a0[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[q], f[ss][b][q], a0[b], 0, 0, 0);
            }
          }
        }
      }
      HDP_MFMA_FENCE();  // the partial sums below read the accumulators (see hdp_common.h)
      // lane holds rows 4 g + reg, column j = 16 b + li of this step's 16 x rp partial.  The 8
      // waves' partials of a step are summed (fixed wave order: deterministic) by the wave that
      // delivers the LAST one -- an arrival counter in LDS instead of a workgroup barrier per
      // step, so the waves drift freely and keep their loads in flight.  kSwRedBufs buffers in
      // rotation; a wave reuses buffer b for step i only after step i - kSwRedBufs was summed.
      constexpr int NBUF = sw_nbuf<RB, FUSE>();
      const int bsel = (int)(i % NBUF);
      const int round = (int)(i / NBUF);
      int* arrive = flags + bsel;
      int* done = flags + NBUF + bsel;
      if constexpr (DIST) {
        // distributed reduction (r04, r-block >= 4 without FUSE): cumulative counters; the buffer is free once
        // every wave has reduced its slice of step i - NBUF
        if (round > 0) wait_ge(done, kSwWaves * round);
        float* rb = red + (bsel * kSwWaves + wave) * 16 * rp;
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) rb[(4 * g + reg) * rp + 16 * b + li] = a0[b][reg] + a1[b][reg];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's partial is in LDS
        if (lane == 0) (void)__hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (pend_i >= 0) reduce_slice(pend_i, pend_s, pend_tail);  // the previous step: its partials are in
        pend_i = i;
        pend_s = s;
        pend_tail = tail;
      } else {
        if (round > 0 && !hs_broken) {
          // the waves of a workgroup are co-resident, so the wait ends; it is still bounded (never hang
          // the GPU on a bug) and a wait that gives up is REPORTED: the error word is checked by the
          // host at the next flush / step (hdp_probe_errors), which fails loudly
          int it = 0;
          while (sa.spin < 0 || __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < round) {
            if (it++ >= sa.spin) {
              hs_broken = true;
              if (lane == 0) {
                __hip_atomic_store(sa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(sa.errd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          asm volatile("" ::: "memory");
        }
        float* rb = red + (bsel * kSwWaves + wave) * 16 * rp;
#pragma unroll
        for (int b = 0; b < RB; ++b) {
          if (FUSE && b >= d.nb) break;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) rb[(4 * g + reg) * rp + 16 * b + li] = a0[b][reg] + a1[b][reg];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's partial is in LDS
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __builtin_amdgcn_readfirstlane(old);
        if (old == kSwWaves - 1) {  // last arrival: every partial of this step is in LDS
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const float* rs = red + bsel * kSwWaves * 16 * rp;
          if constexpr (FUSE) {  // one r-block per round (16 rows x 4 granules = 64 lanes): its own slab
#pragma unroll
            for (int b = 0; b < RB; ++b) {
              if (b >= d.nb) break;
              const int row = lane >> 2, jj = (lane & 3) * 4;
              f32x4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ww = 0; ww < kSwWaves; ++ww)
                acc += *reinterpret_cast<const f32x4*>(rs + (ww * 16 + row) * rp + 16 * b + jj);
              const int64_t t = 16 * (int64_t)s + row;
              if (!tail || t < T) gst4(d.slab_b[b] + ((int64_t)ct * T + t) * d.rpm + jj, acc);
            }
          } else {
#pragma unroll
            for (int e0 = 0; e0 < 16 * r4; e0 += 64) {
              const int e = e0 + lane, row = e / r4, j = (e % r4) * 4;
              f32x4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ww = 0; ww < kSwWaves; ++ww) acc += *reinterpret_cast<const f32x4*>(rs + (ww * 16 + row) * rp + j);
              const int64_t t = 16 * (int64_t)s + row;
              if (!tail || t < T) gst4(d.slab_out + ((int64_t)ct * T + t) * rp + j, acc);
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the partials are read: release the buffer
          if (lane == 0) {
            __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(done, round + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
  };

  // K32 OUTER on a PAIR of steps (rows 16 s .. 16 s + 31): k = 8 g + e <-> row 16 s + 4 e + g (e < 4,
  // first step) or 16 (s + 1) + 4 (e - 4) + g (second step) -- the lane's own rows of both steps, for Y
  // (A operand) and Z (B operand) alike; vB = false: the second step is absent (its Y taken as 0)
  auto pair = [&](const f32x4 (&zA)[4], const float (&yA)[4][RB], const f32x4 (&zB)[4], const float (&yB)[4][RB],
                  int s, bool vB, bool tail) {
    if constexpr (K32O && X6) {  // float32 Z: every column's 8 rows split exactly, 6 products
      bf16x8 zs[4][3];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float zv[8] = {zA[0][q], zA[1][q], zA[2][q], zA[3][q],
                             vB ? zB[0][q] : 0.f, vB ? zB[1][q] : 0.f, vB ? zB[2][q] : 0.f, vB ? zB[3][q] : 0.f};
        split8p(zv, zs[q][0], zs[q][1], zs[q][2]);
      }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        if (FUSE && b >= d.nb) break;
        float yv[8];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          yv[p] = (!tail || 16 * (int64_t)s + 4 * p + g < T) ? yA[p][b] : 0.f;
          yv[4 + p] = vB ? yB[p][b] : 0.f;
        }
        bf16x8 ys[3];
        split8p(yv, ys[0], ys[1], ys[2]);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc2[b][q] = mfma_x6(ys, zs[q], acc2[b][q]);
      }
    } else if constexpr (K32O) {
      bf16x8 zq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          zq[q][p] = as_bf16(zA[p][q]);
          zq[q][4 + p] = as_bf16(zB[p][q]);
        }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        if (FUSE && b >= d.nb) break;
        float yv[8];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          yv[p] = (!tail || 16 * (int64_t)s + 4 * p + g < T) ? yA[p][b] : 0.f;
          yv[4 + p] = vB ? yB[p][b] : 0.f;
        }
        bf16x8 yh, ym, yl;
        split8(yv, yh, ym, yl);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc2[b][q] = mfma32(yl, zq[q], acc2[b][q]);
          acc2[b][q] = mfma32(ym, zq[q], acc2[b][q]);
          acc2[b][q] = mfma32(yh, zq[q], acc2[b][q]);
        }
      }
    }
  };

  const int full_end = (int)min((int64_t)(s0 + n), T / 16);
  const int nfull = full_end > s0 ? full_end - s0 : 0;
  if (nfull > 0) {
    // load cursor: byte offsets of rows 16 s + 4 p + g (no clamping needed on full steps)
    int64_t zo[4];
    int yo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      zo[p] = ((16 * (int64_t)s0 + 4 * p + g) * N + colc) * ES;
      yo[p] = (16 * s0 + 4 * p + g) * d.yrs + li * d.yls;  // Y stored [t][li][b] (probe_yreduce_kernel)
    }
    const int64_t zstep = 16 * N * ES;
    int64_t zd = (16 * (int64_t)s0 + li) * N * ES;  // DL: the lane's row
    int lk = 0;  // step the load cursor points at
    auto load = [&](f32x4 (&z)[4], float (&y)[4][RB]) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DL) {
        typedef uint32_t u32x4d __attribute__((ext_vector_type(4)));
        z[0] = __builtin_bit_cast(f32x4, *reinterpret_cast<const HDP_GLOBAL u32x4d*>(gptr(Zb + zd + cdl0 * ES)));
        z[1] = __builtin_bit_cast(f32x4, *reinterpret_cast<const HDP_GLOBAL u32x4d*>(gptr(Zb + zd + cdl1 * ES)));
      }
#pragma unroll
      for (int p = 0; p < (DL ? 0 : 4); ++p) {
        if constexpr (VEC) {
          // float32 Z: non-temporal (each row is read once per phase; 7B probe group 2.13 -> 2.06 ms,
          // tools/probe_ablate.py ntz, r04); bf16 measured equal and keeps the plain load
          if constexpr (DT == HDP_F32)
            z[p] = load4_nt<DT>(Zb + zo[p], 0);
          else
            z[p] = load4<DT>(Zb + zo[p], 0);
        } else {
          const int64_t rowoff = zo[p] / ES - colc;  // element offset of the row start
#pragma unroll
          for (int q = 0; q < 4; ++q) z[p][q] = load1<DT>(d.Z, rowoff + (col + q < N ? col + q : N - 1));
        }
        if constexpr (OUTER) {  // this lane's RB values of the row: one 4 RB-byte load
          if constexpr (RB == 4) {
            const f32x4 v = gld4(d.y_in + yo[p]);
#pragma unroll
            for (int b = 0; b < RB; ++b) y[p][b] = v[b];
          } else if constexpr (RB == 2) {
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            const f32x2 v = *reinterpret_cast<const HDP_GLOBAL f32x2*>(gptr(d.y_in + yo[p]));
            y[p][0] = v[0];
            y[p][1] = v[1];
          } else {
#pragma unroll
            for (int b = 0; b < RB; ++b) y[p][b] = gld1(d.y_in + yo[p] + b);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (lk + 1 < nfull) {  // uniform; advance (the last step is re-loaded past the end)
        ++lk;
        zd += zstep;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          zo[p] += zstep;
          yo[p] += 16 * d.yrs;
        }
      }
    };
    if constexpr (K32O) {
      // pairs of steps, two pairs in fixed register roles: the next pair's loads in flight
      f32x4 za0[4], za1[4], zb0[4], zb1[4];
      float ya0[4][RB], ya1[4][RB], yb0[4][RB], yb1[4][RB];
      load(za0, ya0);
      load(za1, ya1);
      for (int k = 0; k < nfull; k += 4) {  // nfull is uniform over the workgroup
        load(zb0, yb0);
        load(zb1, yb1);
        pair(za0, ya0, za1, ya1, s0 + k, k + 1 < nfull, false);
        load(za0, ya0);
        load(za1, ya1);
        if (k + 2 < nfull) pair(zb0, yb0, zb1, yb1, s0 + k + 2, k + 3 < nfull, false);
      }
    } else if constexpr (OCC == 1) {
      // NS register sets in fixed roles (a rotation by copies would wait on the new loads); loads run NS - 1
      // steps ahead.  float32: three sets (four or non-temporal loads measured the same, r02).  bf16 PROJ
      // phases: a set is 4 x 8 B per lane (the loads stay packed until the step's compute), half the bytes in
      // flight of a float32 set, and the phase is bound by load latency (SQ r04: waves parked 0.5 of their
      // cycles) -- kBfSets sets
      constexpr int NS = (DT == HDP_BF16 && MODE == kSwProj) ? kBfSets : 3;
      f32x4 zz[NS][4];
      float yy[NS][4][RB];
#pragma unroll
      for (int j = 0; j + 1 < NS; ++j) load(zz[j], yy[j]);
      for (int k = 0; k < nfull; k += NS) {  // nfull is uniform over the workgroup
#pragma unroll
        for (int j = 0; j < NS; ++j) {
          load(zz[(j + NS - 1) % NS], yy[(j + NS - 1) % NS]);
          if (j == 0 || k + j < nfull) compute(zz[j], yy[j], s0 + k + j, i0 + k + j, false);
        }
      }
    } else {
      f32x4 z0[4], z1[4];
      float y0[4][RB], y1[4][RB];
      load(z0, y0);
      for (int k = 0; k < nfull; k += 2) {
        load(z1, y1);
        compute(z0, y0, s0 + k, i0 + k, false);
        load(z0, y0);
        if (k + 1 < nfull) compute(z1, y1, s0 + k + 1, i0 + k + 1, false);
      }
    }
  }
  if (nfull < n) {  // the stripe's last step holds rows past T: clamped loads
    const int s = s0 + nfull;
    f32x4 z[4];
    float y[4][RB];
    if constexpr (DL) {
      typedef uint32_t u32x4d __attribute__((ext_vector_type(4)));
      int64_t row = 16 * (int64_t)s + li;
      row = row < T ? row : T - 1;
      z[0] = __builtin_bit_cast(f32x4, *reinterpret_cast<const HDP_GLOBAL u32x4d*>(gptr(Zb + (row * N + cdl0) * ES)));
      z[1] = __builtin_bit_cast(f32x4, *reinterpret_cast<const HDP_GLOBAL u32x4d*>(gptr(Zb + (row * N + cdl1) * ES)));
    }
#pragma unroll
    for (int p = 0; p < (DL ? 0 : 4); ++p) {
      int64_t row = 16 * (int64_t)s + 4 * p + g;
      row = row < T ? row : T - 1;
      if constexpr (VEC) {
        z[p] = load4<DT>(d.Z, row * N + colc);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) z[p][q] = load1<DT>(d.Z, row * N + (col + q < N ? col + q : N - 1));
      }
      if constexpr (OUTER) {
#pragma unroll
        for (int b = 0; b < RB; ++b) y[p][b] = gld1(d.y_in + row * d.yrs + li * d.yls + b);
      }
    }
    if constexpr (K32O)
      pair(z, y, z, y, s, false, true);
    else
      compute(z, y, s, i0 + nfull, true);
  }
  if constexpr (DIST) {  // the segment's last step
    if (pend_i >= 0) reduce_slice(pend_i, pend_s, pend_tail);
  }
  if constexpr (OUTER) {  // flush this segment's piece
    HDP_MFMA_FENCE();
    const int64_t u0 = d.pre + (int64_t)ct * d.S;
    const int first = sw_owner(u0, sa.U, sa.G);
    const int piece = w - first;
    if (sw_owner(u0 + d.S - 1, sa.U, sa.G) == first) {  // the stripe's only segment: the gradient itself
      if constexpr (FUSE) {
        if (col < N) sw_store_g_fuse(d, acc2, col, g, VEC);
      } else {
        if (col < N) sw_store_g<RB>(d, acc2, col, g, VEC);
      }
    } else if (FUSE && col < N) {  // per r-block: the pieces of the module owning the block
      const int64_t pofs = ((int64_t)ct * d.kmax + piece) * d.rpm * kSwC;
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        if (b >= d.nb) break;
        float* base = d.part_b[b] + pofs;
        if (!d.part_t) {
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            gst4(base + (4 * g + reg) * kSwC + 64 * wave + 4 * li,
                 f32x4{acc2[b][0][reg], acc2[b][1][reg], acc2[b][2][reg], acc2[b][3][reg]});
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) gst4(base + (64 * wave + 4 * li + q) * d.rpm + 4 * g, acc2[b][q]);
        }
      }
    } else if (col < N) {
      float* base = d.part + ((int64_t)ct * d.kmax + piece) * rp * kSwC;
      if (!d.part_t) {
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            gst4(base + (16 * b + 4 * g + reg) * kSwC + 64 * wave + 4 * li,
                 f32x4{acc2[b][0][reg], acc2[b][1][reg], acc2[b][2][reg], acc2[b][3][reg]});
      } else {
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            gst4(base + (64 * wave + 4 * li + q) * rp + 16 * b + 4 * g, acc2[b][q]);
      }
    }
  }
}

// OCC: 1 = one workgroup per CU, three register sets (loads two steps ahead); 2 = two per CU, two
// sets; 3 = one per CU, two sets (r = 64 phase B: PROJ + OUTER registers of 4 r-blocks)
template <int DT, int RB, int MODE, bool VEC, int OCC, bool FUSE = false, bool K32 = false>
__global__ __launch_bounds__(512, OCC == 2 ? 4 : 2) void probe_sweep_kernel(SweepArgs sa) {
  // LDS (PROJ): [staging 8 x 16 x kTileLd] [red kSwRedBufs x 8 x 16 x rp] [flags 2 x kSwRedBufs]
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = blockIdx.x;
  const int64_t lo = sw_lo(w, sa.U, sa.G), nsteps = sw_lo(w + 1, sa.U, sa.G) - lo;
  if (nsteps <= 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* tile = lds + wave * 16 * kTileLd;
  float* red = lds + kSwWaves * 16 * kTileLd;
  int* flags = reinterpret_cast<int*>(red + sw_nbuf<RB, FUSE>() * kSwWaves * 16 * 16 * RB);
  if constexpr ((MODE & kSwProj) != 0) {
    if (threadIdx.x < 2 * sw_nbuf<RB, FUSE>()) flags[threadIdx.x] = 0;
    __syncthreads();
  }
  int m = sa.wst[3 * w], ct = sa.wst[3 * w + 1], s = sa.wst[3 * w + 2];
  for (int64_t done = 0; done < nsteps;) {  // stripe segments of this workgroup's range
    const SweepDesc d = sa.d[m];  // a register copy: the segment's stores cannot alias it
    const int n = (int)min((int64_t)(d.S - s), nsteps - done);
    sweep_segment<DT, RB, MODE, VEC, OCC, FUSE, K32>(d, ct, s, n, done, w, sa, tile, red, flags, wave, lane);
    done += n;
    s = 0;
    if (++ct == d.nct) {
      ct = 0;
      ++m;
    }
  }
}

// Y[t][j] = sum_ct slab[ct][t][j] (fixed order), all modules of a group in one launch:
// blockIdx.y = module, blockIdx.x = 256-granule chunk of its T x rp / 4 f32x4 granules.
struct YRedDesc {
  const float* slab;  // [nct][T][rp] (rp = 16 RB of the module)
  float* y;           // element (t, j = 16 b + li) -> y[t * ys + b + li * sl]
  int64_t T;
  int nct, ys, sl, pad;
};
struct YReduceArgs {
  int n, rp;
  const YRedDesc* d;  // [n] (device)
};

__global__ __launch_bounds__(256) void probe_yreduce_kernel(YReduceArgs ya) {
  const YRedDesc d = ya.d[blockIdx.y];
  const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t step4 = d.T * ya.rp / 4;
  if (f >= step4) return;
  const f32x4* src = reinterpret_cast<const f32x4*>(d.slab) + f;
  f32x4 acc{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < d.nct; c0 += 8) {  // 8 loads in flight, summed in stripe order
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = c0 + u < d.nct ? gld4(reinterpret_cast<const float*>(src + (c0 + u) * step4)) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  // stored [t][li][b] (j = 16 b + li): a sweep lane's RB values of a row are one vector load.  The
  // plain layout is ys = rp, sl = RB; the shared-X layout pads every lane to 4 blocks (ys = 64, sl =
  // 4) and y points at the module's first block within its X-sharing set
  const int rp = ya.rp;
  const int64_t e = 4 * f, t = e / rp;
  const int j0 = (int)(e % rp), b = j0 / 16, li0 = j0 % 16;
  float* dst = d.y + t * d.ys + b;
#pragma unroll
  for (int k = 0; k < 4; ++k) gst1(dst + (li0 + k) * d.sl, acc[k]);
}

// gA[j][n] (+)= s * sum_k pieceA[ct][k][j][n % kSwC];  gB[n][j] (+)= s * sum_k pieceB[ct][k][n % kSwC][j]
struct SwFinishSide {
  const float* part;
  int64_t pre;     // the OUTER phase's flattened steps before this side
  int S, kmax;
  int ph;          // which OUTER phase wrote the pieces: 0 = phase B, 1 = phase C
  int pad;
};
struct FinDesc {
  float* gA;
  float* gB;
  int in, out, r, acc;
  float scale;
  int ldb;  // row stride of gB (= r, or the full rank when the module is an r-slice of a wider one)
  SwFinishSide sx, sg;
};
struct SwFinishArgs {
  int n, rp;
  int64_t U[2];    // phase B / C total steps
  int G[2];        // phase B / C workgroups
  const FinDesc* d;  // [n] (device)
  const int* jobs;   // [njobs][2]: module, 2 stripe + side (1 = B side) -- the split stripes only
  int bx;            // workgroups per job
};

// One job = one stripe that more than one workgroup segment covered (the host lists them; a stripe
// covered by one segment had its gradient block written by that segment, so it gets no job and no
// workgroup): r x kSwC elements, workgroup blockIdx.x % bx of job blockIdx.x / bx.
// V = 4: every thread finishes 4 consecutive elements of one row (side A: same j, n..n+3;
// side B: same n, j..j+3) with 16-B loads of the pieces and of g -- same per-element
// summation order as V = 1 (deterministic, identical bits).  The host picks V = 4 when every
// module has r % 4 == 0, in % 4 == 0 and 16-B aligned gradients.
template <int V>
__global__ __launch_bounds__(256) void probe_sweep_finish_kernel(SwFinishArgs fa) {
#pragma clang fp contract(off)  // g + s*sum as two roundings, like autograd's mul then add
  typedef float vec __attribute__((ext_vector_type(V)));
  const int job = blockIdx.x / fa.bx;
  const FinDesc& dm = fa.d[fa.jobs[2 * job]];
  const int code = fa.jobs[2 * job + 1], ct = code >> 1;
  const bool sideA = (code & 1) == 0;
  const int r = dm.r;
  const int e = ((int)(blockIdx.x % fa.bx) * 256 + (int)threadIdx.x) * V;  // element of the r x kSwC job
  if (e >= r * kSwC) return;
  int nn, j;
  if (sideA) {
    j = e / kSwC;
    nn = e % kSwC;
  } else {
    nn = e / r;
    j = e % r;
  }
  const int64_t n = (int64_t)ct * kSwC + nn;
  if (n >= (sideA ? dm.in : dm.out)) return;
  const SwFinishSide& sd = sideA ? dm.sx : dm.sg;
  const int64_t u0 = sd.pre + (int64_t)ct * sd.S;
  const int64_t U = fa.U[sd.ph];
  const int Gw = fa.G[sd.ph];
  const int k0 = sw_owner(u0, U, Gw), np = sw_owner(u0 + sd.S - 1, U, Gw) - k0 + 1;
  if (np == 1) return;  // one segment covered the stripe and wrote its gradient block itself
  const float* p = sd.part + (int64_t)ct * sd.kmax * fa.rp * kSwC + (sideA ? (int64_t)j * kSwC + nn : (int64_t)nn * fa.rp + j);
  const int64_t stride = (int64_t)fa.rp * kSwC;
  vec s0 = 0.f, s1 = 0.f;
  int k = 0;
  for (; k + 2 <= np; k += 2) {
    s0 += *reinterpret_cast<const HDP_GLOBAL vec*>(gptr(p + k * stride));
    s1 += *reinterpret_cast<const HDP_GLOBAL vec*>(gptr(p + (k + 1) * stride));
  }
  if (k < np) s0 += *reinterpret_cast<const HDP_GLOBAL vec*>(gptr(p + k * stride));
  const vec v = dm.scale * (s0 + s1);
  HDP_GLOBAL vec* gp = reinterpret_cast<HDP_GLOBAL vec*>(gptr(sideA ? dm.gA + (int64_t)j * dm.in + n : dm.gB + n * dm.ldb + j));
  *gp = dm.acc ? *gp + v : v;
}

// Per-flush descriptor tables: one host blob copied to the head of the group's device workspace
// in stream order.  The host side goes through a ring of pinned staging buffers, each reused only
// after the copy that last read it has executed (its event).
constexpr size_t kTableFixed = 3 * 4096 * 3 * sizeof(int) + 4096;  // WG start tables, up to 4096 WGs/phase
constexpr size_t kTablePerModule = 3 * sizeof(SweepDesc) + 2 * sizeof(YRedDesc) + sizeof(FinDesc) + 64;

// Device error word of the sweep's PROJ hand-off: pinned host memory mapped into the device, so the
// host reads it without synchronising (it reflects every launch that has completed).  Written only
// when a bounded wait gives up; hdp_probe_queue_flush / hdp_probe_grads_group refuse to run while
// it is set, hdp_probe_errors reads (and clears) it.
static std::mutex g_err_mu;
static int* g_err_host = nullptr;
static int* g_err_dev = nullptr;
static int* g_err_local = nullptr;  // device-memory copy (hipMalloc): read by every K3 workgroup -- a read
                                    // of the host-mapped word crosses PCIe and serialises (+1.4 ms per Adam)
int* probe_err_word() {
  std::lock_guard<std::mutex> lk(g_err_mu);
  if (!g_err_host) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 256, hipHostMallocMapped) != hipSuccess) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return nullptr;
    }
    void* l = nullptr;
    if (hipMalloc(&l, 256) != hipSuccess || hipMemset(l, 0, 256) != hipSuccess) {
      (void)hipHostFree(h);
      return nullptr;
    }
    *reinterpret_cast<volatile int*>(h) = 0;
    g_err_host = reinterpret_cast<int*>(h);
    g_err_dev = reinterpret_cast<int*>(d);
    g_err_local = reinterpret_cast<int*>(l);
  }
  return g_err_dev;
}
int* probe_err_local() {
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err_local;
}
const int* probe_err_device() { return probe_err_local(); }
int probe_err_read(int clear) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  if (!g_err_host) return 0;
  volatile int* w = g_err_host;
  const int v = *w;
  if (clear && v != 0) {  // (the error path only: a synchronous clear of the device copy too)
    *w = 0;
    (void)hipMemset(g_err_local, 0, sizeof(int));
  }
  return v;
}
// hand-off wait bound (sleeps of ~64 cycles): env HDP_PROBE_SPIN, read per launch (tests force
// the failure path with a negative value)
static int probe_spin() {
  const char* e = getenv("HDP_PROBE_SPIN");
  return e ? atoi(e) : (1 << 22);
}

struct Staging {
  void* host = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};
// 64 slots: a LLaMA-2-7B step flushes 8 groups, so the host can run ~8 steps ahead of the GPU
// before a slot's copy must have executed (with 8 the host waited on the GPU every step)
constexpr int kStageSlots = 64;
static std::mutex g_stage_mu;
static Staging g_stage[kStageSlots];
static int g_stage_next = 0;
static int64_t g_wait_ns = 0;  // host time blocked on the ring (the GPU is behind): measurement

int probe_tables_upload(const std::vector<char>& blob, void* dst, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  Staging& s = g_stage[g_stage_next];
  g_stage_next = (g_stage_next + 1) % kStageSlots;
  if (s.pending) {
    if (hipEventQuery(s.ev) == hipErrorNotReady) {  // back-pressure: the host is kStageSlots flushes ahead
      const auto t0 = std::chrono::steady_clock::now();
      HDP_CHECK_HIP(hipEventSynchronize(s.ev));
      g_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    s.pending = false;
  }
  if (s.cap < blob.size()) {
    if (s.host) HDP_CHECK_HIP(hipHostFree(s.host));
    s.host = nullptr;
    s.cap = 0;
    const size_t sz = blob.size() * 2 > 65536 ? blob.size() * 2 : 65536;
    HDP_CHECK_HIP(hipHostMalloc(&s.host, sz, hipHostMallocDefault));
    s.cap = sz;
  }
  if (!s.ev) HDP_CHECK_HIP(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
  memcpy(s.host, blob.data(), blob.size());
  HDP_CHECK_HIP(hipMemcpyAsync(dst, s.host, blob.size(), hipMemcpyHostToDevice, st));
  HDP_CHECK_HIP(hipEventRecord(s.ev, st));
  s.pending = true;
  return HDP_OK;
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
  size_t off_slabH, off_slabJ, off_partA, off_partB, off_yH, off_yJ, area, bytes;
};

static void p1_split(int64_t K, int& ks, int& cols) {
  const int64_t span = (int64_t)kP1Waves * p1_cols();
  ks = (int)((K + span - 1) / span);
  int64_t c = (K + (int64_t)ks * kP1Waves - 1) / ((int64_t)ks * kP1Waves);
  cols = (int)((c + 15) / 16 * 16);
}

// r <= 64 runs the sweep path (phases A-D); HDP_PROBE_PATH=split forces the P1/P2 split
// (read per call: the workspace query and the launch must agree; tests flip it per case)
static bool use_sweep(int RB) {
  const char* e = getenv("HDP_PROBE_PATH");
  return RB <= 4 && !(e && e[0] == 's' && e[1] == 'p');
}
// group-level tables per module (sweep descriptors)
static size_t table_per_module() { return kTablePerModule; }

// 64 < r <= 128 (r-block 8): the probe is separable in r -- A.grad rows j and B.grad columns j only
// involve A's row j and B's column j -- so such a module runs as r-slices of at most 64 on the
// pipelined sweep (RB 4) instead of the split path: A / B^T / A.grad sliced by rows, B.grad by
// columns (leading dimension = the full r).  X and G are streamed once per slice.  Needs B^T (the
// slice of B^T is contiguous); HDP_PROBE_R128=split keeps the split path.
static bool slice_r(int r, int b_transposed) {
  const char* e = getenv("HDP_PROBE_R128");
  return r > 64 && r <= 128 && b_transposed && use_sweep(4) && !(e && e[0] == 's');
}
static int n_slices(int r) { return (r + 63) / 64; }

// the finish's job list (one int2 per split stripe) is part of the group's tables: room for every stripe
static size_t finish_jobs_bytes(int64_t in, int64_t out) {
  return (size_t)(((in + kSwC - 1) / kSwC + (out + kSwC - 1) / kSwC) * 8 + 255) / 256 * 256;
}

static int sweep_kmax(int64_t T) { return (int)(((T + 15) / 16 + kSwMinSteps - 1) / kSwMinSteps) + 2; }

static ModPlan plan_module(int64_t T, int64_t in, int64_t out, int r) {
  ModPlan p;
  const int RB = rb_of(r), rp = 16 * RB;
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n * 4 + 255) / 256 * 256; return o; };
  if (use_sweep(RB)) {
    p.ksh = (int)((in + kSwC - 1) / kSwC);
    p.ksj = (int)((out + kSwC - 1) / kSwC);
    p.colh = p.colj = 0;
    p.kst = sweep_kmax(T);  // pieces per stripe (capacity)
    // slabs [nct][T16][rp] and projections [T16][rp] floats (T16 = T rounded up to 16 rows)
    const size_t T16 = (size_t)((T + 15) / 16) * 16;
    p.off_slabH = take((size_t)p.ksh * T16 * rp);
    p.off_slabJ = take((size_t)p.ksj * T16 * rp);
    p.off_partA = take((size_t)p.ksh * p.kst * rp * kSwC);
    p.off_partB = take((size_t)p.ksj * p.kst * rp * kSwC);
    // projections: [T16][rp], or the padded shared-X layout [T16][16 lanes][4 blocks] (r-block <= 2)
    const size_t yrow = RB <= 2 ? 64 : 2 * (size_t)rp;
    p.off_yH = take(T16 * yrow);
    p.off_yJ = take(T16 * yrow);
  } else {
    p1_split(in, p.ksh, p.colh);
    p1_split(out, p.ksj, p.colj);
    p.kst = (int)((T + kTC - 1) / kTC);
    p.off_slabH = take((size_t)p.ksh * T * rp);
    p.off_slabJ = take((size_t)p.ksj * T * rp);
    p.off_partA = take((size_t)p.kst * rp * in);
    p.off_partB = take((size_t)p.kst * rp * out);
    p.off_yH = p.off_yJ = 0;
  }
  p.area = off;
  // + this module's share of the group's tables and counters
  p.bytes = off + table_per_module() + kTableFixed + 256 + (use_sweep(RB) ? finish_jobs_bytes(in, out) : 0);
  return p;
}

// algorithmic work of a group's passes: X and G once (+ the factors once), 2 T r (in|out) flop
struct GroupWork {
  double xg = 0, fac = 0, x = 0, g = 0, s1 = 0, s2 = 0, fl_x = 0, fl_g = 0, fl_s1 = 0, fl_s2 = 0, grads = 0;
};
template <class GA>
static GroupWork group_work(const GA& ga, int es) {
  GroupWork w;
  for (int i = 0; i < ga.n; ++i) {
    const ProbeDesc& d = ga.d[i];
    const double X = (double)es * d.T * d.in, G = (double)es * d.T * d.out;
    const double fx = 2.0 * d.T * d.r * d.in, fg = 2.0 * d.T * d.r * d.out;
    w.x += X;
    w.g += G;
    w.fac += 4.0 * d.r * (d.in + d.out);
    w.fl_x += fx;
    w.fl_g += fg;
    const bool s1x = d.in <= d.out;
    w.s1 += s1x ? X : G;
    w.s2 += s1x ? G : X;
    w.fl_s1 += s1x ? fx : fg;
    w.fl_s2 += s1x ? fg : fx;
    w.grads += 4.0 * d.r * (d.in + d.out) * (d.accumulate ? 2 : 1);
  }
  w.xg = w.x + w.g;
  return w;
}

template <int DT, int RB>
static int launch_group(const GroupArgs& ga, hipStream_t st) {
  const GroupWork w = group_work(ga, DT == HDP_F32 ? 4 : 2);
  const int rp = ga.rp;
  const dim3 g1(ga.p1_pre[ga.n]), b1(kP1Waves * 64);
  auto lds1 = [&](int U) { return (size_t)kP1Waves * (16 * rp + U * 16 * kTileLd) * sizeof(float); };
  {
  KTimer kt(K_PROBE_P1, st, w.xg + w.fac, w.fl_x + w.fl_g);
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
  }
  HDP_CHECK_LAUNCH();
  {
    KTimer kt(K_PROBE_P2, st, w.xg, w.fl_x + w.fl_g);
    hipLaunchKernelGGL((probe_outer_kernel<DT, RB>), dim3(ga.p2_pre[ga.n]), dim3(512),
                       (size_t)(kTC * rp > 4096 ? kTC * rp : 4096) * sizeof(float), st, ga);
  }
  HDP_CHECK_LAUNCH();
  const int64_t tot = ga.p3_pre[ga.n];
  const int blocks = (int)min((int64_t)4096, (tot + 255) / 256);
  bool v4 = true;
  int64_t per = 1;
  for (int i = 0; i < ga.n; ++i) {
    const ProbeDesc& d = ga.d[i];
    v4 = v4 && d.r % 4 == 0 && d.in % 4 == 0 && (reinterpret_cast<uintptr_t>(d.gA) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(d.gB) & 15) == 0 && (reinterpret_cast<uintptr_t>(d.partA) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(d.partB) & 15) == 0;
    const int64_t e = ((int64_t)d.r * (d.in + d.out) + 1023) / 1024;
    per = e > per ? e : per;
  }
  {
    KTimer kt(K_PROBE_FINISH, st, w.grads);
    if (v4 && per < 65536)
      hipLaunchKernelGGL(probe_finish4_kernel, dim3((unsigned)per, (unsigned)ga.n), dim3(256), 0, st, ga);
    else
      hipLaunchKernelGGL(probe_finish_kernel, dim3(blocks), dim3(256), 0, st, ga);
  }
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}

// resident 512-thread workgroups of one sweep kernel instance x CUs (cached per instance/device)
template <int DT, int RB, int MODE, bool VEC, int OCC, bool FUSE = false, bool K32 = false>
static int sweep_slots(size_t lds) {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, probe_sweep_kernel<DT, RB, MODE, VEC, OCC, FUSE, K32>, 512,
                                                     lds) != hipSuccess ||
        per <= 0)
      per = 1;
    cached[dev] = cus * per;
  }
  return cached[dev];
}

// resident workgroups of one phase: occupancy x CUs, capped so each gets >= kSwMinSteps steps
template <int DT, int RB, int MODE, bool VEC, int OCC, bool FUSE = false, bool K32 = false>
static int phase_grid(int64_t U, size_t lds) {
  const int64_t cap = U / kSwMinSteps;
  const int slots = sweep_slots<DT, RB, MODE, VEC, OCC, FUSE, K32>(lds);
  return (int)(cap < 1 ? 1 : (cap < slots ? cap : slots));
}

// where workgroup w of G starts: (module, stripe, step) of flattened step w * U / G
static void phase_starts(const std::vector<SweepDesc>& d, int64_t U, int G, int* out) {
  int m = 0;
  for (int w = 0; w < G; ++w) {
    const int64_t lo = (int64_t)w * U / G;
    while (m + 1 < (int)d.size() && lo >= d[m + 1].pre) ++m;
    const int64_t rem = lo - d[m].pre;
    out[3 * w] = m;
    out[3 * w + 1] = (int)(rem / d[m].S);
    out[3 * w + 2] = (int)(rem % d[m].S);
  }
}

// Shared X (hp:139 is called with ONE hidden state per projection group of a decoder layer: q/k/v
// read the same normed x, gate/up the same x; autograd saves that one tensor for each of them).
// Modules of a group whose X is the same tensor (same pointer, T and in; B given transposed) are
// packed into sets of at most kSwMaxBlk r-blocks; a set streams its X ONCE per pass for all of its
// modules (phase A: PROJ against the stacked A rows; phase C: OUTER against the stacked
// projections of their G) instead of once per module.  A set is formed only when X is the smaller
// side (in <= sum of its modules' out): X is then the stream read twice.  env HDP_PROBE_SHARE_X=0
// turns it off (A/B measurements, tests).
// 0: off (HDP_PROBE_K32=0); 1: r-block 4 only (HDP_PROBE_K32=4); 2 (default): PROJ phases at every r-block,
// the OUTER phase at r-block 4 (its r-block-1 instance spills 24 VGPRs); 3: every phase and r-block
// (HDP_PROBE_K32=all)
static int probe_k32() {
  const char* e = getenv("HDP_PROBE_K32");
  return !e ? 2 : e[0] == '0' ? 0 : e[0] == '4' ? 1 : e[0] == 'a' ? 3 : 2;
}
// float32 activations: phase A (the shared-X FUSE instance, 4 r-block template) on the exact 6-product
// bf16 split (X6, r04); env HDP_PROBE_X6=0 keeps f32 MFMA
static bool probe_x6() {
  const char* e = getenv("HDP_PROBE_X6");
  return !(e && e[0] == '0');
}
static bool share_x_enabled() {
  const char* e = getenv("HDP_PROBE_SHARE_X");
  return !(e && e[0] == '0');
}
static std::vector<std::vector<int>> shared_x_sets(const HostGroup& ga) {
  std::vector<std::vector<int>> sets;
  const int n = ga.n;
  if (ga.RB > 2 || !share_x_enabled()) return sets;
  for (int i = 0; i < n; ++i)
    if (!ga.d[i].b_t) return sets;
  std::vector<char> used(n, 0);
  for (int i = 0; i < n; ++i) {
    if (used[i]) continue;
    const ProbeDesc& p = ga.d[i];
    std::vector<int> cur{i};
    int64_t outs = p.out;
    for (int k = i + 1; k < n && (int)(cur.size() + 1) * ga.RB <= kSwMaxBlk; ++k) {
      const ProbeDesc& q = ga.d[k];
      if (!used[k] && q.X == p.X && q.T == p.T && q.in == p.in) {
        cur.push_back(k);
        outs += q.out;
      }
    }
    if (cur.size() < 2 || outs < p.in) continue;
    for (int k : cur) used[k] = 1;
    sets.push_back(cur);
  }
  return sets;
}

// the plain side descriptor of one module stream (X: PROJ -> H, OUTER with J -> pieces A; G: PROJ
// -> J, OUTER with H -> pieces B^T), its r-block view filled for the FUSE instances
static SweepDesc side_desc(const ProbeDesc& p, bool xs, int RB, int S) {
  const int rp = 16 * RB;
  SweepDesc d{};
  d.Z = xs ? p.X : p.G;
  d.F = xs ? p.A : p.B;
  d.slab_out = xs ? p.slabH : p.slabJ;
  d.y_in = xs ? p.yJ : p.yH;
  d.part = xs ? p.partA : p.partB;
  d.T = p.T;
  d.N = xs ? p.in : p.out;
  d.pre = 0;
  d.r = p.r;
  d.f_rk = xs ? 1 : p.b_t;
  d.part_t = xs ? 0 : 1;
  d.nct = xs ? p.ksh : p.ksj;
  d.S = S;
  d.kmax = p.kst;
  d.g = xs ? p.gA : p.gB;
  d.scale = p.scale;
  d.acc = p.accumulate;
  d.ldb = xs ? p.r : p.ldb;
  d.yrs = rp;
  d.yls = RB;
  d.nb = RB;
  d.rpm = rp;
  for (int b = 0; b < kSwMaxBlk; ++b) {
    const int rows = p.r - 16 * b;
    d.rbr[b] = b < RB ? (rows < 0 ? 0 : rows > 16 ? 16 : rows) : 0;
    d.Fb[b] = d.F + (int64_t)16 * b * d.N;  // f_rk rows (FUSE requires B^T)
    d.slab_b[b] = d.slab_out + 16 * b;
    d.part_b[b] = d.part_t ? d.part + 16 * b : d.part + (int64_t)16 * b * kSwC;
    d.gb[b] = d.part_t ? d.g + 16 * b : d.g + (int64_t)16 * b * d.N;
    d.sc[b] = p.scale;
    d.accb[b] = p.accumulate;
  }
  return d;
}

// phases A (PROJ over S1), R1 (reduce S1 slabs), B (PROJ + OUTER over S2), R2 (reduce S2
// slabs), C (OUTER over S1), D (finish); `tab` = the group's device table region
// occupancy per phase (measured r02, LLaMA-2-7B shapes): PROJ + OUTER (B) gains from two
// resident workgroups per CU (-4 %), PROJ (A) and OUTER (C) from two steps of loads in flight
// With X-sharing sets (shared_x_sets) phases A and C run the FUSE instance (4 r-blocks, runtime nb)
// over every S1 side; phase B, the reduces and the finish keep their kernels (descriptor strides).
template <int DT, int RB, bool VEC>
static int launch_sweep(const HostGroup& ga, char* tab, hipStream_t st) {
  constexpr int rp = 16 * RB;
  // bf16 data at r-block 4: phase B is PROJ only (bf16 MFMA, split fragments -- fused with OUTER they
  // do not fit beside its accumulators) and S2's OUTER joins S1's in phase C: S2 is read twice, its
  // projection costs a fifth of the f32 MFMA issue time
  constexpr bool SPLIT_B = RB >= 4 && DT == HDP_BF16;
  constexpr int ES = DT == HDP_F32 ? 4 : 2;
  const int n = ga.n;
  const std::vector<std::vector<int>> sets = SPLIT_B ? std::vector<std::vector<int>>{} : shared_x_sets(ga);
  const bool fuse = !sets.empty();
  std::vector<int> set_of(n, -1), blk0(n, 0);
  for (int k = 0; k < (int)sets.size(); ++k)
    for (int m = 0; m < (int)sets[k].size(); ++m) {
      set_of[sets[k][m]] = k;
      blk0[sets[k][m]] = m * RB;
    }
  std::vector<SweepDesc> sd[3];
  std::vector<YRedDesc> yd[2];
  std::vector<FinDesc> fd(n);
  std::vector<char> s1x(n);
  std::vector<int> at_c(n, -1), at_b(n, -1);  // each module's X / G side: index in its OUTER phase
  int64_t U[3] = {0, 0, 0};
  double bytes_ph[3] = {0, 0, 0}, flop_ph[3] = {0, 0, 0};
  auto add = [&](int ph, SweepDesc d) {
    d.pre = U[ph];
    U[ph] += (int64_t)d.nct * d.S;
    int rows = 0;
    for (int b = 0; b < d.nb && b < kSwMaxBlk; ++b) rows += d.rbr[b];
    bytes_ph[ph] += (double)ES * d.T * d.N;
    flop_ph[ph] += 2.0 * d.T * d.N * (fuse && (ph != 1) ? rows : d.r) * (ph == 1 && !SPLIT_B ? 2.0 : 1.0);
    sd[ph].push_back(d);
    return (int)sd[ph].size() - 1;
  };
  for (int k = 0; k < 2; ++k) yd[k].resize(n);
  int64_t yblk = 1;
  bool v4 = true;  // 4 elements per finish thread when every module allows it
  for (int i = 0; i < n; ++i) {
    const ProbeDesc& p = ga.d[i];
    const int S = (int)((p.T + 15) / 16);
    const int si = set_of[i];
    s1x[i] = si >= 0 ? 1 : (p.in <= p.out);  // S1 = the smaller stream, read twice (a set: its X)
    SweepDesc x = side_desc(p, true, RB, S), gg = side_desc(p, false, RB, S);
    if (si >= 0) {
      const ProbeDesc& lead = ga.d[sets[si][0]];
      // this module's G side reads its H in phase B: member m's [T][16 lanes][RB] slice of the set's
      // H buffer (lead's yH, rows of 64 floats: the plain layout per member, member-major)
      gg.y_in = lead.yH + 16 * blk0[i];
      gg.yrs = 4 * 16;
      if (sets[si][0] == i) {  // the set's X side (phases A and C), r-blocks of every member
        SweepDesc fx = x;
        fx.nb = RB * (int)sets[si].size();
        fx.y_in = lead.yJ;  // the set's padded J (phase C)
        fx.yrs = 4 * 16;
        fx.yls = 4;
        for (int m = 0; m < (int)sets[si].size(); ++m) {
          const SweepDesc xm = side_desc(ga.d[sets[si][m]], true, RB, S);
          for (int bb = 0; bb < RB; ++bb) {
            const int b = m * RB + bb;
            fx.Fb[b] = xm.Fb[bb];
            fx.rbr[b] = xm.rbr[bb];
            fx.slab_b[b] = xm.slab_b[bb];
            fx.part_b[b] = xm.part_b[bb];
            fx.gb[b] = xm.gb[bb];
            fx.sc[b] = xm.sc[bb];
            fx.accb[b] = xm.accb[bb];
          }
        }
        add(0, fx);
        at_c[i] = add(2, fx);
        for (int m : sets[si]) at_c[m] = at_c[i];
      }
      at_b[i] = add(1, gg);
    } else {
      const SweepDesc& d1 = s1x[i] ? x : gg;
      SweepDesc d2 = s1x[i] ? gg : x;
      SweepDesc d1c = d1;
      if (fuse) {  // phase C runs the FUSE instance: Y_S2 in the padded layout
        d1c.yrs = 4 * 16;
        d1c.yls = 4;
      }
      add(0, d1);
      if (SPLIT_B) {  // S2's OUTER, right after S1's in phase C
        add(1, d2);
        const int c1 = add(2, d1c);
        const int c2 = add(2, d2);
        at_c[i] = s1x[i] ? c1 : c2;  // X side
        at_b[i] = s1x[i] ? c2 : c1;  // G side (both in phase C)
      } else {
        const int bi = add(1, d2);
        const int ci = add(2, d1c);
        at_c[i] = s1x[i] ? ci : bi;
        at_b[i] = s1x[i] ? bi : ci;
      }
    }
    // R1: S1's slabs -> the projection phase B reads; R2: S2's slabs -> the one phase C reads
    if (si >= 0) {
      const ProbeDesc& lead = ga.d[sets[si][0]];
      yd[0][i] = YRedDesc{p.slabH, lead.yH + 16 * blk0[i], p.T, p.ksh, 4 * 16, RB, 0};
      yd[1][i] = YRedDesc{p.slabJ, lead.yJ + blk0[i], p.T, p.ksj, 4 * 16, 4, 0};
    } else {
      const SweepDesc& d1 = s1x[i] ? x : gg;
      const SweepDesc& d2 = s1x[i] ? gg : x;
      yd[0][i] = YRedDesc{d1.slab_out, s1x[i] ? p.yH : p.yJ, p.T, d1.nct, rp, RB, 0};
      yd[1][i] = YRedDesc{d2.slab_out, s1x[i] ? p.yJ : p.yH, p.T, d2.nct, fuse ? 4 * 16 : rp, fuse ? 4 : RB, 0};
    }
    const int64_t yb = (p.T * rp / 4 + 255) / 256;
    yblk = yb > yblk ? yb : yblk;
    fd[i] = FinDesc{p.gA, p.gB, (int)p.in, (int)p.out, p.r, p.accumulate, p.scale, p.ldb, {}, {}};
    v4 = v4 && p.r % 4 == 0 && p.ldb % 4 == 0 && p.in % 4 == 0 && (reinterpret_cast<uintptr_t>(p.gA) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(p.gB) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.partA) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(p.partB) & 15) == 0;
  }
  const int V = v4 ? 4 : 1;
  const size_t proj_lds =
      ((size_t)kSwWaves * 16 * kTileLd + (size_t)sw_nbuf<RB>() * kSwWaves * 16 * rp) * sizeof(float) +
      2 * sw_nbuf<RB>() * 4;
  const size_t fuse_lds =
      ((size_t)kSwWaves * 16 * kTileLd + (size_t)sw_nbuf<kSwMaxBlk, true>() * kSwWaves * 16 * 16 * kSwMaxBlk) *
          sizeof(float) +
      2 * sw_nbuf<kSwMaxBlk, true>() * 4;
  constexpr int OCC_B = SPLIT_B ? 1 : RB >= 4 ? 3 : VEC ? 2 : 1;
  constexpr int MODE_B = SPLIT_B ? kSwProj : kSwProj | kSwOuter;
  constexpr int RBF = RB <= 2 ? kSwMaxBlk : RB;  // the FUSE instances' r-blocks (only built for RB <= 2)
  // bf16 activations: the PROJ-only and OUTER-only phases on 16x16x32 bf16 MFMA (K32; env
  // HDP_PROBE_K32=0 keeps the 16x16x16 forms)
  constexpr bool BF = DT == HDP_BF16;
  // (every r-block: r03 restricted them to r-block 4 after wrong projections at r <= 32, whose cause was an
  // MFMA result read 3 wait states after issue behind a taken branch -- HDP_MFMA_FENCE, r04;
  // tests/test_gpu_kernels.py::test_probe_k32_all_rblocks)
  const int k32m = BF ? probe_k32() : 0;
  const bool k32 = k32m >= 2 || (k32m == 1 && RB >= 4);
  const bool k32c = k32m == 3 || (k32m >= 1 && RB >= 4);  // the OUTER phase (C)
  // phase A's FUSE instance (4 r-block template) on float32 activations: X6 (the K32 PROJ form on split
  // activations; phase C's X6 OUTER form spills at 256 VGPRs beside four load sets: kept on f32 MFMA)
  const bool x6 = !BF && fuse && probe_x6();
  const bool kf = k32 || x6;  // phase A's K32 template (bf16 split fragments / X6)
  int G[3];
  if (fuse) {
    if constexpr (RB <= 2) {
      G[0] = kf ? phase_grid<DT, RBF, kSwProj, VEC, 1, true, true>(U[0], fuse_lds)
                : phase_grid<DT, RBF, kSwProj, VEC, 1, true>(U[0], fuse_lds);
      G[2] = k32 ? phase_grid<DT, RBF, kSwOuter, VEC, 1, true, BF>(U[2], 0)  // (the FUSE instance is r-block 4)
                 : phase_grid<DT, RBF, kSwOuter, VEC, 1, true>(U[2], 0);
    }
  } else {
    G[0] = k32 ? phase_grid<DT, RB, kSwProj, VEC, 1, false, BF>(U[0], proj_lds)
               : phase_grid<DT, RB, kSwProj, VEC, 1>(U[0], proj_lds);
    G[2] = k32c ? phase_grid<DT, RB, kSwOuter, VEC, 1, false, BF>(U[2], 0)
               : phase_grid<DT, RB, kSwOuter, VEC, 1>(U[2], 0);
  }
  constexpr bool K32B = BF && MODE_B == kSwProj;  // phase B is PROJ-only on the split (r-block 4) path
  G[1] = k32 ? phase_grid<DT, RB, MODE_B, VEC, OCC_B, false, K32B>(U[1], proj_lds)
             : phase_grid<DT, RB, MODE_B, VEC, OCC_B>(U[1], proj_lds);
  HDP_CHECK_ARG(G[0] <= 4096 && G[1] <= 4096 && G[2] <= 4096, "probe sweep: grid above the table size");
  HDP_CHECK_ARG(yblk < 65536 && n < 65536, "probe sweep: group too large");
  // finish: the pieces of X's OUTER and of G's (phase index 0 = B, 1 = C in fa.U / fa.G); every
  // module's pieces are in its own part buffers (a shared-X set's OUTER writes each member's rows there)
  for (int i = 0; i < n; ++i) {
    const ProbeDesc& p = ga.d[i];
    const bool x_in_c = SPLIT_B || s1x[i], g_in_c = SPLIT_B || !s1x[i];
    const SweepDesc& dx = sd[x_in_c ? 2 : 1][at_c[i]];
    const SweepDesc& dg = sd[g_in_c ? 2 : 1][at_b[i]];
    fd[i].sx = SwFinishSide{p.partA, dx.pre, dx.S, dx.kmax, x_in_c ? 1 : 0, 0};
    fd[i].sg = SwFinishSide{p.partB, dg.pre, dg.S, dg.kmax, g_in_c ? 1 : 0, 0};
  }
  // one blob: [sd A | sd B | sd C | wst A | wst B | wst C | yd R1 | yd R2 | fd]
  size_t off = 0;
  auto place = [&](size_t bytes) { size_t o = off; off += (bytes + 255) / 256 * 256; return o; };
  size_t o_sd[3], o_w[3], o_y[2];
  for (int ph = 0; ph < 3; ++ph) o_sd[ph] = place(sizeof(SweepDesc) * sd[ph].size());
  for (int ph = 0; ph < 3; ++ph) o_w[ph] = place(sizeof(int) * 3 * G[ph]);
  for (int k = 0; k < 2; ++k) o_y[k] = place(sizeof(YRedDesc) * n);
  const size_t o_f = place(sizeof(FinDesc) * n);
  // the finish's jobs: the stripes that more than one workgroup segment covered (the others wrote their
  // gradient blocks in phase B / C)
  std::vector<int> jobs;
  double pieces = 0;
  {
    auto owner = [](int64_t u, int64_t UU, int GG) { return (int64_t)(((u + 1) * GG - 1) / UU); };
    for (int i = 0; i < n; ++i) {
      const ProbeDesc& p = ga.d[i];
      for (int side = 0; side < 2; ++side) {
        const SwFinishSide& sd2 = side == 0 ? fd[i].sx : fd[i].sg;
        const int nct = side == 0 ? p.ksh : p.ksj;
        const int ph = sd2.ph + 1;  // phase B = 1, C = 2
        for (int ct = 0; ct < nct; ++ct) {
          const int64_t u0 = sd2.pre + (int64_t)ct * sd2.S;
          const int64_t np = owner(u0 + sd2.S - 1, U[ph], G[ph]) - owner(u0, U[ph], G[ph]) + 1;
          if (np > 1) {
            jobs.push_back(i);
            jobs.push_back(2 * ct + side);
            // the finish reads the pieces and updates the gradient of split stripes only
            pieces += 4.0 * p.r * kSwC * ((double)np + (p.accumulate ? 2 : 1));
          }
        }
      }
    }
  }
  const int njobs = (int)(jobs.size() / 2);
  HDP_CHECK_ARG((int64_t)njobs * (rp * kSwC / 256) < (1ll << 31), "probe sweep: finish grid too large");
  const size_t o_j = place(sizeof(int) * jobs.size());
  size_t tab_cap = kTableFixed + (size_t)n * table_per_module();
  for (int i = 0; i < n; ++i) tab_cap += finish_jobs_bytes(ga.d[i].in, ga.d[i].out);
  HDP_CHECK_ARG(off <= tab_cap, "probe sweep: descriptor tables exceed their space");
  std::vector<char> blob(off);
  for (int ph = 0; ph < 3; ++ph) {
    memcpy(blob.data() + o_sd[ph], sd[ph].data(), sizeof(SweepDesc) * sd[ph].size());
    phase_starts(sd[ph], U[ph], G[ph], reinterpret_cast<int*>(blob.data() + o_w[ph]));
  }
  for (int k = 0; k < 2; ++k) memcpy(blob.data() + o_y[k], yd[k].data(), sizeof(YRedDesc) * n);
  memcpy(blob.data() + o_f, fd.data(), sizeof(FinDesc) * n);
  if (njobs) memcpy(blob.data() + o_j, jobs.data(), sizeof(int) * jobs.size());
  int rc = probe_tables_upload(blob, tab, st);
  if (rc) return rc;

  int* err = probe_err_word();
  HDP_CHECK_ARG(err != nullptr, "probe sweep: error word allocation failed");
  int* errd = probe_err_local();
  const int spin = probe_spin();
  SweepArgs sa[3];
  for (int ph = 0; ph < 3; ++ph)
    sa[ph] = SweepArgs{(int)sd[ph].size(), G[ph], spin, U[ph], err, errd, reinterpret_cast<const SweepDesc*>(tab + o_sd[ph]),
                       reinterpret_cast<const int*>(tab + o_w[ph])};
  // workspace bytes the reduce / finish passes move (slabs + Y; pieces + gradients) -- counted
  // as algorithmic for these launches: they are the price of the stripe decomposition
  double slab[2] = {0, 0};
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 2; ++k) slab[k] += 4.0 * ga.d[i].T * rp * (yd[k][i].nct + 1);
  auto reduce = [&](int k) {
    KTimer kt(K_PROBE_REDUCE, st, slab[k]);
    hipLaunchKernelGGL(probe_yreduce_kernel, dim3((unsigned)yblk, (unsigned)n), dim3(256), 0, st,
                       YReduceArgs{n, rp, reinterpret_cast<const YRedDesc*>(tab + o_y[k])});
  };
  {
    KTimer kt(K_SWEEP_A, st, bytes_ph[0], flop_ph[0]);
    if (fuse) {
      if constexpr (RB <= 2) {
        if (kf)
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwProj, VEC, 1, true, true>), dim3(G[0]), dim3(512), fuse_lds,
                             st, sa[0]);
        else
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwProj, VEC, 1, true>), dim3(G[0]), dim3(512), fuse_lds, st,
                             sa[0]);
      }
    } else if (k32) {
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, kSwProj, VEC, 1, false, BF>), dim3(G[0]), dim3(512), proj_lds, st,
                         sa[0]);
    } else {
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, kSwProj, VEC, 1>), dim3(G[0]), dim3(512), proj_lds, st, sa[0]);
    }
  }
  HDP_CHECK_LAUNCH();
  reduce(0);
  HDP_CHECK_LAUNCH();
  {
    KTimer kt(K_SWEEP_B, st, bytes_ph[1], flop_ph[1]);
    if (k32)
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, MODE_B, VEC, OCC_B, false, K32B>), dim3(G[1]), dim3(512), proj_lds,
                         st, sa[1]);
    else
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, MODE_B, VEC, OCC_B>), dim3(G[1]), dim3(512), proj_lds, st, sa[1]);
  }
  HDP_CHECK_LAUNCH();
  reduce(1);
  HDP_CHECK_LAUNCH();
  {
    KTimer kt(K_SWEEP_C, st, bytes_ph[2], flop_ph[2]);
    if (fuse) {
      if constexpr (RB <= 2) {
        if (k32)
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwOuter, VEC, 1, true, BF>), dim3(G[2]), dim3(512), 0, st,
                             sa[2]);
        else
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwOuter, VEC, 1, true>), dim3(G[2]), dim3(512), 0, st, sa[2]);
      }
    } else if (k32c) {
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, kSwOuter, VEC, 1, false, BF>), dim3(G[2]), dim3(512), 0, st, sa[2]);
    } else {
      hipLaunchKernelGGL((probe_sweep_kernel<DT, RB, kSwOuter, VEC, 1>), dim3(G[2]), dim3(512), 0, st, sa[2]);
    }
  }
  HDP_CHECK_LAUNCH();
  if (njobs) {  // (none when every stripe had one segment: no launch)
    const int bx = (rp * kSwC + 256 * V - 1) / (256 * V);
    SwFinishArgs fa{n, rp, {U[1], U[2]}, {G[1], G[2]}, reinterpret_cast<const FinDesc*>(tab + o_f),
                    reinterpret_cast<const int*>(tab + o_j), bx};
    KTimer kt(K_PROBE_FINISH, st, pieces);
    if (v4)
      hipLaunchKernelGGL(probe_sweep_finish_kernel<4>, dim3((unsigned)(njobs * bx)), dim3(256), 0, st, fa);
    else
      hipLaunchKernelGGL(probe_sweep_finish_kernel<1>, dim3((unsigned)(njobs * bx)), dim3(256), 0, st, fa);
    HDP_CHECK_LAUNCH();
  }
  return HDP_OK;
}

}  // namespace hdp

using namespace hdp;

// workspace of one module: its plan, or (64 < r <= 128) the larger of the split plan and its r-slices'
static size_t module_bytes(int64_t T, int64_t in, int64_t out, int r) {
  size_t b = plan_module(T, in, out, r).bytes;
  if (r > 64 && r <= 128 && use_sweep(4)) {
    size_t sl = 0;
    const int ns = n_slices(r);
    for (int k = 0; k < ns; ++k) sl += plan_module(T, in, out, (r + ns - 1) / ns).bytes;
    b = sl > b ? sl : b;
  }
  return b;
}

extern "C" size_t hdp_probe_workspace_bytes(int64_t T, int64_t in, int64_t out, int r) {
  if (T <= 0 || in <= 0 || out <= 0 || r <= 0 || r > 128) return 0;
  return module_bytes(T, in, out, r);
}

extern "C" int hdp_probe_group_max(void) { return kMaxGroup; }

extern "C" int hdp_probe_errors(int clear) { return probe_err_read(clear); }

extern "C" int64_t hdp_probe_host_wait_us(int reset) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  const int64_t us = g_wait_ns / 1000;
  if (reset) g_wait_ns = 0;
  return us;
}

extern "C" int hdp_probe_grads_group(int n, const hdp_probe_item* items, int x_dtype, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (probe_err_read(0) != 0) {
    set_error("hdp_probe_grads_group: a previous probe launch reported a failed hand-off (device error word "
              "set; those gradients are wrong) -- hdp_probe_errors(1) clears it");
    return HDP_EDEVICE;
  }
  HDP_CHECK_ARG(n >= 0 && n <= kMaxGroup, "hdp_probe_grads_group: n = %d not in [0, %d]", n, kMaxGroup);
  HDP_CHECK_ARG(x_dtype == HDP_F32 || x_dtype == HDP_BF16, "hdp_probe_grads_group: bad dtype %d", x_dtype);
  if (n == 0) return HDP_OK;
  HDP_CHECK_ARG(items != nullptr, "hdp_probe_grads_group: null items");
  // r-slices (64 < r <= 128 with B^T): expand every module into slices of <= 64, one group on RB 4
  std::vector<hdp_probe_item> sliced;
  std::vector<int> ldb_of;
  bool slicing = n > 0;
  for (int i = 0; i < n && slicing; ++i) slicing = slice_r(items[i].r, items[i].b_transposed);
  if (slicing && n * 2 > kMaxGroup) {
    // more slices than a group holds: stream-ordered chunks that reuse the workspace from its start
    const int chunk = kMaxGroup / 2;
    for (int k = 0; k < n; k += chunk) {
      const int rc = hdp_probe_grads_group(n - k < chunk ? n - k : chunk, items + k, x_dtype, workspace,
                                           workspace_bytes, stream);
      if (rc != HDP_OK) return rc;
    }
    return HDP_OK;
  }
  if (slicing) {
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < i; ++k)
        HDP_CHECK_ARG(items[k].gA != items[i].gA && items[k].gB != items[i].gB,
                      "hdp_probe_grads_group: items %d and %d accumulate into the same gradient", k, i);
    for (int i = 0; i < n; ++i) {
      const hdp_probe_item& it = items[i];
      const int ns = n_slices(it.r), rk = (it.r + ns - 1) / ns;
      for (int j0 = 0; j0 < it.r; j0 += rk) {
        hdp_probe_item sl = it;
        sl.r = it.r - j0 < rk ? it.r - j0 : rk;
        sl.A = it.A + (int64_t)j0 * it.in;
        sl.B = it.B + (int64_t)j0 * it.out;
        sl.gA = it.gA + (int64_t)j0 * it.in;
        sl.gB = it.gB + j0;
        sliced.push_back(sl);
        ldb_of.push_back(it.r);
      }
    }
    HDP_CHECK_ARG((int)sliced.size() <= kMaxGroup, "hdp_probe_grads_group: %d r-slices exceed the group size",
                  (int)sliced.size());
    n = (int)sliced.size();
    items = sliced.data();
  }
  const bool sweep = slicing || use_sweep(rb_of(items[0].r));
  if (!sweep && n > kMaxSplit) {
    // the split path's kernel arguments hold kMaxSplit modules: launch in stream-ordered
    // chunks that reuse the workspace from its start
    for (int k = 0; k < n; k += kMaxSplit) {
      const int rc = hdp_probe_grads_group(n - k < kMaxSplit ? n - k : kMaxSplit, items + k, x_dtype, workspace,
                                           workspace_bytes, stream);
      if (rc != HDP_OK) return rc;
    }
    return HDP_OK;
  }
  hipStream_t st = as_stream(stream);
  HostGroup ga;
  ga.RB = slicing ? 4 : rb_of(items[0].r);
  ga.rp = 16 * ga.RB;
  ga.d.reserve(n);
  char* ws = reinterpret_cast<char*>(workspace);
  // the group's descriptor tables first (sweep path), then the modules' work areas
  size_t tab_bytes = 0;
  if (sweep) {
    tab_bytes = kTableFixed + (size_t)n * table_per_module();
    for (int i = 0; i < n; ++i) tab_bytes += finish_jobs_bytes(items[i].in, items[i].out);
  }
  size_t off = tab_bytes;
  HDP_CHECK_ARG(!sweep || off <= workspace_bytes, "hdp_probe_grads: workspace %zu bytes too small (need %zu)",
                workspace_bytes, off);
  if (!slicing)
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < i; ++k)
        HDP_CHECK_ARG(items[k].gA != items[i].gA && items[k].gB != items[i].gB,
                      "hdp_probe_grads_group: items %d and %d accumulate into the same gradient", k, i);
  for (int i = 0; i < n; ++i) {
    const hdp_probe_item& it = items[i];
    HDP_CHECK_ARG(it.in > 0 && it.out > 0 && it.r > 0 && it.T >= 0, "hdp_probe_grads: bad shape (item %d)", i);
    HDP_CHECK_ARG(it.r <= 128, "hdp_probe_grads: r = %d > 128 is not supported", it.r);
    HDP_CHECK_ARG(slicing ? it.r <= 16 * ga.RB : rb_of(it.r) == ga.RB,
                  "hdp_probe_grads_group: items of one group need the same r-block");
    const int ldb = slicing ? ldb_of[i] : it.r;
    HDP_CHECK_ARG(it.A && it.B && it.gA && it.gB, "hdp_probe_grads: null pointer (item %d)", i);
    if (it.T == 0) {
      if (!it.accumulate) {
        HDP_CHECK_HIP(hipMemsetAsync(it.gA, 0, sizeof(float) * it.r * it.in, st));
        if (ldb == it.r)
          HDP_CHECK_HIP(hipMemsetAsync(it.gB, 0, sizeof(float) * it.r * it.out, st));
        else
          HDP_CHECK_HIP(hipMemset2DAsync(it.gB, sizeof(float) * ldb, 0, sizeof(float) * it.r, it.out, st));
      }
      continue;
    }
    HDP_CHECK_ARG(it.X && it.G && workspace, "hdp_probe_grads: null pointer (item %d)", i);
    HDP_CHECK_ARG((reinterpret_cast<uintptr_t>(it.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(it.X) & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(it.G) & 15) == 0 &&
                      (!it.b_transposed || (reinterpret_cast<uintptr_t>(it.B) & 15) == 0),
                  "hdp_probe_grads: X, G, A (and B^T) must be 16-byte aligned (item %d)", i);
    const ModPlan p = plan_module(it.T, it.in, it.out, it.r);
    const size_t mod_bytes = p.area;
    HDP_CHECK_ARG(off + mod_bytes <= workspace_bytes, "hdp_probe_grads: workspace %zu bytes too small (need %zu)",
                  workspace_bytes, off + mod_bytes);
    ProbeDesc d{};
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
    d.yH = reinterpret_cast<float*>(ws + off + p.off_yH);
    d.yJ = reinterpret_cast<float*>(ws + off + p.off_yJ);
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
    d.ldb = ldb;
    off += mod_bytes;
    ga.d.push_back(d);
  }
  ga.n = (int)ga.d.size();
  if (ga.n == 0) return HDP_OK;
  if (sweep) {
    bool vec = true;  // every stream's rows are whole 16-B granules
    for (int i = 0; i < ga.n; ++i) vec = vec && ga.d[i].in % 4 == 0 && ga.d[i].out % 4 == 0;
    // bf16: rows of whole 16-B granules too (8 elements), 16-B aligned bases (the PROJ phases' 16-B loads)
    if (x_dtype == HDP_BF16)
      for (int i = 0; i < ga.n; ++i)
        vec = vec && ga.d[i].in % 8 == 0 && ga.d[i].out % 8 == 0 &&
              (reinterpret_cast<uintptr_t>(ga.d[i].X) & 15) == 0 && (reinterpret_cast<uintptr_t>(ga.d[i].G) & 15) == 0;
#define HDP_SWEEP(D, R) return vec ? launch_sweep<D, R, true>(ga, ws, st) : launch_sweep<D, R, false>(ga, ws, st)
    if (x_dtype == HDP_F32) {
      if (ga.RB == 1) HDP_SWEEP(HDP_F32, 1);
      if (ga.RB == 2) HDP_SWEEP(HDP_F32, 2);
      HDP_SWEEP(HDP_F32, 4);
    }
    if (ga.RB == 1) HDP_SWEEP(HDP_BF16, 1);
    if (ga.RB == 2) HDP_SWEEP(HDP_BF16, 2);
    HDP_SWEEP(HDP_BF16, 4);
#undef HDP_SWEEP
  }
  // split path (n <= kMaxSplit here): descriptors by value in the kernel arguments
  GroupArgs gs;
  gs.n = ga.n;
  gs.rp = ga.rp;
  gs.RB = ga.RB;
  gs.p1_pre[0] = gs.p2_pre[0] = 0;
  gs.p3_pre[0] = 0;
  for (int i = 0; i < ga.n; ++i) {
    const ProbeDesc& d = ga.d[i];
    gs.d[i] = d;
    const int64_t tblk = (d.T + 15) / 16;
    const int64_t w1 = tblk * (d.ksh + d.ksj);
    const int64_t w2 = ((d.in + kNW - 1) / kNW + (d.out + kNW - 1) / kNW) * d.kst;
    HDP_CHECK_ARG(gs.p1_pre[i] + w1 < (1ll << 31) && gs.p2_pre[i] + w2 < (1ll << 31),
                  "hdp_probe_grads_group: grid too large");
    gs.p1_pre[i + 1] = gs.p1_pre[i] + (int)w1;
    gs.p2_pre[i + 1] = gs.p2_pre[i] + (int)w2;
    gs.p3_pre[i + 1] = gs.p3_pre[i] + (int64_t)d.r * (d.in + d.out);
  }
#define HDP_PROBE(D, R) return launch_group<D, R>(gs, st)
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

// ---------------------------------------------------------------------------------------
// Native probe queue (host runtime of the deferred, grouped K2 backward).  The Python
// ProbeQueue used to build every group's item array in ctypes (~15 us of host time per
// module backward, slower than the GPU consumed the groups); here a module's constant fields
// are registered once and each backward is one push of (slot, X, G, T, accumulate, stream).
// The queue launches the pending group before a push that would exceed the group size or
// byte budget, repeat a module, change the stream or the r-block; it owns its device
// workspace (grown on demand after a stream synchronisation -- only when a larger T or group
// appears).
// ---------------------------------------------------------------------------------------
struct hdp_probe_queue_s {
  int dtype = HDP_F32;
  int max_items = kMaxGroup;
  int64_t budget = 0;
  std::vector<hdp_probe_item> mods;   // registered modules (X, G, T, accumulate unset)
  std::vector<int64_t> stamp;         // per slot: the flush generation it was last queued in
  int64_t gen = 1;
  std::vector<hdp_probe_item> pend;
  int npend = 0;
  int64_t bytes = 0;
  void* stream = nullptr;
  int rb = 0;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  void* last_stream = nullptr;  // stream of the previous flush (the workspace's last user)
  bool any_flush = false;
  int64_t flushes = 0;
};

extern "C" int hdp_probe_queue_create(int x_dtype, int max_items, int64_t budget_bytes, hdp_probe_queue* q) {
  HDP_CHECK_ARG(q, "hdp_probe_queue_create: null handle pointer");
  HDP_CHECK_ARG(x_dtype == HDP_F32 || x_dtype == HDP_BF16, "hdp_probe_queue_create: bad dtype %d", x_dtype);
  HDP_CHECK_ARG(max_items >= 1 && max_items <= kMaxGroup, "hdp_probe_queue_create: max_items %d not in [1, %d]",
                max_items, kMaxGroup);
  HDP_CHECK_ARG(budget_bytes > 0, "hdp_probe_queue_create: budget must be positive");
  hdp_probe_queue p = new hdp_probe_queue_s;
  p->pend.resize(max_items);
  p->dtype = x_dtype;
  p->max_items = max_items;
  p->budget = budget_bytes;
  *q = p;
  return HDP_OK;
}

extern "C" int hdp_probe_queue_add_module(hdp_probe_queue q, const float* A, const float* B, int b_transposed,
                                          float* gA, float* gB, int64_t in, int64_t out, int r, float scale,
                                          int* slot) {
  HDP_CHECK_ARG(q && slot, "hdp_probe_queue_add_module: null argument");
  HDP_CHECK_ARG(A && B && gA && gB && in > 0 && out > 0 && r > 0 && r <= 128,
                "hdp_probe_queue_add_module: bad module (in=%lld out=%lld r=%d)", (long long)in, (long long)out, r);
  hdp_probe_item it{};
  it.A = A;
  it.B = B;
  it.gA = gA;
  it.gB = gB;
  it.in = in;
  it.out = out;
  it.r = r;
  it.b_transposed = b_transposed ? 1 : 0;
  it.scale = scale;
  q->mods.push_back(it);
  q->stamp.push_back(0);
  *slot = (int)q->mods.size() - 1;
  return HDP_OK;
}

extern "C" int hdp_probe_queue_flush(hdp_probe_queue q) {
  HDP_CHECK_ARG(q, "hdp_probe_queue_flush: null queue");
  if (q->npend == 0) return HDP_OK;
  if (probe_err_read(0) != 0) {  // refuse BEFORE any queue state changes: the group stays pending
    set_error("hdp_probe_queue_flush: a probe hand-off failed earlier (device error word set; those gradients "
              "are wrong) -- hdp_probe_errors(1) clears it; the %d pending modules stay queued", q->npend);
    return HDP_EDEVICE;
  }
  size_t need = 0;
  for (int i = 0; i < q->npend; ++i) {
    const hdp_probe_item& it = q->pend[i];
    if (it.T > 0) need += module_bytes(it.T, it.in, it.out, it.r);
  }
  if (q->any_flush && q->last_stream != q->stream)  // the workspace is shared: order the two streams
    HDP_CHECK_HIP(hipStreamSynchronize(as_stream(q->last_stream)));
  if (need > q->ws_bytes) {
    // grow geometrically, stream-ordered: the old workspace is released after the kernels
    // already queued on this stream (no host synchronisation inside a training step)
    hipStream_t st = as_stream(q->stream);
    if (q->ws) {
      HDP_CHECK_HIP(hipFreeAsync(q->ws, st));
      q->ws = nullptr;
    }
    const size_t sz = need > 2 * q->ws_bytes ? need + need / 4 : 2 * q->ws_bytes;
    q->ws_bytes = 0;
    HDP_CHECK_HIP(hipMallocAsync(&q->ws, sz, st));
    q->ws_bytes = sz;
  }
  const int n = q->npend;
  q->npend = 0;
  q->bytes = 0;
  ++q->gen;
  ++q->flushes;
  q->last_stream = q->stream;
  q->any_flush = true;
  return hdp_probe_grads_group(n, q->pend.data(), q->dtype, q->ws, q->ws_bytes, q->stream);
}

extern "C" int hdp_probe_queue_push(hdp_probe_queue q, int slot, const void* X, const void* G, int64_t T,
                                    int accumulate, void* stream, int* flushed) {
  HDP_CHECK_ARG(q && slot >= 0 && slot < (int)q->mods.size(), "hdp_probe_queue_push: bad slot %d", slot);
  HDP_CHECK_ARG(T >= 0 && (T == 0 || (X && G)), "hdp_probe_queue_push: bad X / G / T");
  const hdp_probe_item& m = q->mods[slot];
  const int64_t es = q->dtype == HDP_F32 ? 4 : 2;
  const int64_t nb = T * (m.in + m.out) * es;
  const int rb = rb_of(m.r);
  int fl = 0;
  if (q->npend > 0 && (q->stamp[slot] == q->gen || q->npend >= q->max_items || q->bytes + nb > q->budget ||
                       stream != q->stream || rb != q->rb)) {
    const int rc = hdp_probe_queue_flush(q);
    if (rc != HDP_OK) return rc;
    fl = 1;
  }
  if (q->npend == 0) {
    q->stream = stream;
    q->rb = rb;
  }
  hdp_probe_item& it = q->pend[q->npend++];
  it = m;
  it.X = X;
  it.G = G;
  it.T = T;
  it.accumulate = accumulate ? 1 : 0;
  q->stamp[slot] = q->gen;
  q->bytes += nb;
  if (flushed) *flushed = fl;
  return HDP_OK;
}

extern "C" int hdp_probe_queue_pending(hdp_probe_queue q) { return q ? q->npend : 0; }

extern "C" int64_t hdp_probe_queue_flushes(hdp_probe_queue q) { return q ? q->flushes : 0; }

extern "C" int hdp_probe_queue_destroy(hdp_probe_queue q) {
  if (!q) return HDP_OK;
  int rc = HDP_OK;
  if (q->ws) {
    if (q->stream) (void)hipStreamSynchronize(as_stream(q->stream));
    if (hipFreeAsync(q->ws, as_stream(q->stream)) != hipSuccess || hipStreamSynchronize(as_stream(q->stream)) != hipSuccess) {
      set_error("hdp_probe_queue_destroy: hipFree failed");
      rc = HDP_EHIP;
    }
  }
  delete q;
  return rc;
}
