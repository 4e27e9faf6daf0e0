// K1: SVD-slice initializer -- replaces hp:106-125.
//
// The reference runs a full torch.svd of every targeted W on every rank and keeps r
// triplets.  Only the top k = r * nranks triplets are ever used, so here:
//   1. Gram  = W^T W (out >= in) or W W^T (out < in), float64 accumulation of float32/bf16
//      inputs on fp64 MFMA (v_mfma_f64_16x16x4_f64) -- products of fp32 values are exact.
//   2. the top k eigenpairs of the n x n Gram (n = min(out, in)):
//      TRUNCATED (r05, k <= 64 and n >= 2048, k <= 128 at n >= 4096 (r06; r05: n >= 5120) -- every BASELINE config
//      at one GPU, and LLaMA-2-7B r16 at Wn = 8):
//      block Krylov on the Gram, batched over the modules that share n -- m = 1024 directions for k <= 32, 2048
//      for k <= 64, 3072 for k <= 128 (blocks of b = 32 / 64 / 128 from a seeded random start, each the Gram times the previous block,
//      orthogonalised twice against all earlier blocks, Cholesky QR twice), Rayleigh-Ritz on the m x m
//      projection (rocSOLVER dsyevd), Ritz vectors,
//      and an explicit residual check ||G v - theta v|| / theta <= 1e-5 for every pair of every module
//      (the SVD triplet residual ||W^T u - sigma v|| / sigma; the parity bar is 1e-4); a batch that misses
//      it falls back to the full solve below (the Grams are left intact).  O(n^2 m) flops of fp64 GEMM
//      against the full tridiagonalisation's O(n^3) memory-bound gemv chain (HDP_EIG=full forces it).
//      FULL: rocSOLVER dsyevd of all n eigenpairs, batched over the modules that share n (strided
//      batched); the top k columns are used.  HDP_EIG=dsyevdx selects the index-range solver (top k
//      only) for single-matrix calls.
//   3. projection P = W V (tall) or U^T W (wide) on fp64 MFMA, then the factor epilogue
//      A = sqrt(S) V^T, B = U sqrt(S) = W V / sqrt(S)  (tall)  /  B = U sqrt(S),
//      A = U^T W / sqrt(S)  (wide), written per rank: A_all rows d*r.., B_all slab d.
// sigma = sqrt(lambda) keeps ~1e-16 * sigma_max^2 / sigma^2 relative accuracy for the
// leading triplets, far inside the 1e-4 parity bar; vectors are defined up to sign.
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "hdp_common.h"

namespace hdp {

enum { EL_F32 = 0, EL_BF16 = 1, EL_F64 = 2 };

struct GemmF64Args {
  int64_t M, N, K;
  const void* a;
  int64_t a_sm, a_sk;
  const void* b;
  int64_t b_sk, b_sn;
  double* c;
  int64_t ldc;
};

template <int EL>
__device__ __forceinline__ double ldel(const void* p, int64_t i) {
  if constexpr (EL == EL_F32) return (double)reinterpret_cast<const float*>(p)[i];
  else if constexpr (EL == EL_BF16) return (double)bf16_to_f32(reinterpret_cast<const uint16_t*>(p)[i]);
  else return reinterpret_cast<const double*>(p)[i];
}

constexpr int GB = 64, GK = 16;

// C[M][N] = sum_k a(m,k) b(k,n); 256 threads, 64x64 tile, 4 waves of 32x32 (2x2 MFMA blocks).
// SYM (the Gram, a == b as matrices, M == N): only the tiles with block row <= block column run (one
// per blockIdx.x, column-major over the upper triangle: bn (bn + 1) / 2 + bm), and an off-diagonal
// tile also writes its transpose -- half the fp64 MFMA work of the full product (r06, VERDICT r05 #6;
// C[n][m] and C[m][n] are the same exact products summed in the same k order, so the mirror is exact)
__device__ __forceinline__ void tri_tile(int64_t idx, int64_t& bm, int64_t& bn) {
  int64_t c = (int64_t)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
  while (c * (c + 1) / 2 > idx) --c;
  while ((c + 1) * (c + 2) / 2 <= idx) ++c;
  bn = c;
  bm = idx - c * (c + 1) / 2;
}

template <int AEL, int BEL, bool SYM = false>
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmF64Args g) {
  __shared__ double As[GK][GB + 1];
  __shared__ double Bs[GK][GB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int64_t m0, n0;
  if constexpr (SYM) {
    int64_t bm, bn;
    tri_tile((int64_t)blockIdx.x, bm, bn);
    m0 = bm * GB;
    n0 = bn * GB;
  } else {
    const int nN = (int)((g.N + GB - 1) / GB);
    m0 = (int64_t)(blockIdx.x / nN) * GB;
    n0 = (int64_t)(blockIdx.x % nN) * GB;
  }
  const int wm = wave >> 1, wn = wave & 1;
  f64x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  const bool a_m_fast = (g.a_sm == 1), b_n_fast = (g.b_sn == 1);
  for (int64_t k0 = 0; k0 < g.K; k0 += GK) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      int mm, kk;
      if (a_m_fast) { mm = e % GB; kk = e / GB; } else { mm = e / GK; kk = e % GK; }
      const int64_t m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < g.M && k < g.K) ? ldel<AEL>(g.a, m * g.a_sm + k * g.a_sk) : 0.0;
      int nn;
      if (b_n_fast) { nn = e % GB; kk = e / GB; } else { nn = e / GK; kk = e % GK; }
      const int64_t n = n0 + nn, k2 = k0 + kk;
      Bs[kk][nn] = (n < g.N && k2 < g.K) ? ldel<BEL>(g.b, k2 * g.b_sk + n * g.b_sn) : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < GK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double av[2], bv[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) av[x] = As[kk][wm * 32 + x * 16 + (lane & 15)];
#pragma unroll
      for (int y = 0; y < 2; ++y) bv[y] = Bs[kk][wn * 32 + y * 16 + (lane & 15)];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
    }
    __syncthreads();
  }
  // f64 16x16x4 result map: D[row = (lane>>4) + 4*reg][col = lane&15]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t m = m0 + wm * 32 + x * 16 + (lane >> 4) + 4 * reg;
        const int64_t n = n0 + wn * 32 + y * 16 + (lane & 15);
        if (m < g.M && n < g.N) {
          g.c[m * g.ldc + n] = acc[x][y][reg];
          if (SYM && m0 != n0) g.c[n * g.ldc + m] = acc[x][y][reg];
        }
      }
}

template <int AEL, int BEL, bool SYM = false>
static int gemm_f64(const GemmF64Args& g, hipStream_t st) {
  const int64_t nT = (g.N + GB - 1) / GB;
  const int64_t nb = SYM ? nT * (nT + 1) / 2 : ((g.M + GB - 1) / GB) * nT;
  HDP_CHECK_ARG(!SYM || g.M == g.N, "gemm_f64: symmetric product needs M == N");
  {
    // (flops: the MFMA work launched -- the upper-triangle tiles only for SYM)
    KTimer kt(K_SVD_GEMM, st, 8.0 * (g.M * g.K + g.K * g.N + g.M * g.N),
              2.0 * (double)nb * GB * GB * (double)g.K);
    hipLaunchKernelGGL((gemm_f64_kernel<AEL, BEL, SYM>), dim3((unsigned)nb), dim3(256), 0, st, g);
  }
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}

struct FactorArgs {
  const double* Z;     // n x k eigenvectors, column-major (ld n), ascending eigenvalues
  const double* lam;   // k eigenvalues, ascending
  const double* P;     // tall: out x k (ld k) = W V;  wide: k x in (ld in) = U^T W
  int64_t n, out, in;
  int k, r, tall;
  float* A_all;        // k x in
  float* B_all;        // nranks x out x r
  double* S;           // k, descending (may be null)
};

__global__ __launch_bounds__(256) void svd_factor_kernel(FactorArgs f) {
  const int64_t nA = (int64_t)f.k * f.in, nB = (int64_t)f.out * f.k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nA + nB; e += (int64_t)gridDim.x * 256) {
    int t;
    if (e < nA) t = (int)(e / f.in);
    else t = (int)((e - nA) % f.k);
    const int jz = f.k - 1 - t;
    const double lam = f.lam[jz];
    const double sigma = lam > 0.0 ? sqrt(lam) : 0.0;
    const double sq = sqrt(sigma);
    const double inv = sigma > 0.0 ? 1.0 / sq : 0.0;
    if (e < nA) {
      const int64_t c = e % f.in;
      const double v = f.tall ? sq * f.Z[c + (int64_t)jz * f.n] : inv * f.P[(int64_t)jz * f.in + c];
      f.A_all[(int64_t)t * f.in + c] = (float)v;
      if (c == 0 && f.S) f.S[t] = sigma;
    } else {
      const int64_t o = (e - nA) / f.k;
      const double v = f.tall ? inv * f.P[o * f.k + jz] : sq * f.Z[o + (int64_t)jz * f.n];
      const int d = t / f.r, tt = t % f.r;
      f.B_all[((int64_t)d * f.out + o) * f.r + tt] = (float)v;
    }
  }
}

// HDP_EIG=dsyevdx selects rocSOLVER's index-range solver (top k only); the default is the
// full dsyevd (the path torch.linalg.eigh takes), whose top k columns are used.
static bool use_syevdx() {
  const char* e = getenv("HDP_EIG");
  return e && std::string(e) == "dsyevdx";
}

// ---- truncated path (block Krylov) ----------------------------------------------------------
constexpr double kKryTol = 1e-5;   // accepted Ritz residual ||G v - theta v|| / theta (the parity bar: 1e-4)
// Krylov directions m and block b (b divides m: the Ritz values land at [m - k, m)); k > 32 (the bf16
// configs' r = 64 / 128 at Wn = 1) takes a deeper basis (tools/svd_kry_probe.py, profiles/r05_svd_krylov_k64_k128.txt)
static int kry_m(int k) {
  if (const char* e = getenv("HDP_KRY_M")) return atoi(e);
  return k <= 32 ? 1024 : k <= 64 ? 2048 : 3072;
}
static int kry_block(int k) { return k <= 16 ? 32 : k <= 64 ? 64 : 128; }
static bool use_krylov(int64_t n, int k) {
  const char* e = getenv("HDP_EIG");
  if (e && (std::string(e) == "full" || std::string(e) == "dsyevdx")) return false;
  const int m = kry_m(k), b = kry_block(k);
  // k = 128 misses the residual bar at m = 2048 on the bench's Gaussian init (1e-3 .. 5e-5) and meets it at
  // m = 3072 for n = 5120 (4e-7); at smaller n the m x m Rayleigh-Ritz solve is no longer cheaper than the full one
  int kmax = 128;
  if (const char* e = getenv("HDP_KRY_KMAX")) kmax = atoi(e);  // experiments (tools/svd_kry_probe.py)
  // (r06: n = 4096 -- LLaMA-2-7B at Wn = 8 -- runs m = 3072 = 0.75 n; HDP_KRY_NMIN_K128 moves the floor back for
  // A/B timing against the full solve)
  int nmin128 = 4096;
  if (const char* e = getenv("HDP_KRY_NMIN_K128")) nmin128 = atoi(e);
  if (k > 64 && n < nmin128) return false;
  return k <= kmax && n >= 2048 && m <= n && m % b == 0 && m >= 8 * k;
}

// seeded random start block: Q0[i][c] (column-major, ld n) uniform in (-1, 1) from a hash of (item, i, c)
__global__ __launch_bounds__(256) void kry_init_kernel(double* Q, int64_t n, int b, int64_t item_stride, int count) {
  const int64_t tot = n * b;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot * count; e += (int64_t)gridDim.x * 256) {
    const int64_t it = e / tot, loc = e % tot;
    uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(loc + 1) + 0xD1B54A32D192ED03ull * (uint64_t)(it + 7);
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 32;
    Q[it * item_stride + loc] = (double)(x >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  }
}

// per item, per Ritz pair i: R[:, i] (= G V[:, i], from the stored Krylov products) against theta_i V[:, i];
// the worst relative residual over the item's k pairs goes to res[item] (one workgroup per (item, pair))
__global__ __launch_bounds__(256) void kry_resid_kernel(const double* R, const double* V, const double* lam, int64_t n,
                                                        int k, int64_t vstride, int64_t lstride, int m, double* res) {
  const int it = blockIdx.y, i = blockIdx.x;
  const double th = lam[it * lstride + (m - k) + i];
  const double* r = R + it * vstride + (int64_t)i * n;
  const double* v = V + it * vstride + (int64_t)i * n;
  double acc = 0.0;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    const double d = r[e] - th * v[e];
    acc += d * d;
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double rel = th > 0.0 ? sqrt(red[0]) / th : 1.0;
    // max over the item's pairs: doubles compare as unsigned 64-bit for non-negatives
    atomicMax(reinterpret_cast<unsigned long long*>(res + it), (unsigned long long)__double_as_longlong(rel));
  }
}

static std::mutex g_blas_mu;
static rocblas_handle g_blas = nullptr;
static int blas_handle(rocblas_handle* h) {
  std::lock_guard<std::mutex> lk(g_blas_mu);
  if (!g_blas) {
    if (rocblas_create_handle(&g_blas) != rocblas_status_success) {
      set_error("rocblas_create_handle failed");
      return HDP_ESOLVER;
    }
  }
  *h = g_blas;
  return HDP_OK;
}

// One batch of top-k SVDs sharing n = min(out, in): Grams into a strided buffer, ONE
// rocsolver_dsyevd_strided_batched over all of them (rocSOLVER's tridiagonalisation is a chain of
// O(n) small launches per matrix -- latrd/larfg, 150 ms for n = 4096 -- which the batched call
// issues once for the whole batch), then per item the projection and the factor epilogue.
struct BatchWs {
  size_t gram, lam, offd, Z, ints, bytes;
  std::vector<size_t> P;
  // truncated path: Krylov basis and products [item][m][n], projection [item][m][m], its eigenvalues /
  // off-diagonal [item][m], solver infos, C [item][m][b], Ritz vectors / residual products [item][k][n]
  size_t kQ = 0, kY = 0, kT = 0, kLam = 0, kOff = 0, kInf = 0, kC = 0, kV = 0, kR = 0, kRes = 0;
  bool kry = false;
};
static BatchWs batch_ws(const hdp_svd_item* items, int count, int k) {
  BatchWs w;
  const int64_t n = items[0].out < items[0].in ? items[0].out : items[0].in;
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off += (b + 255) / 256 * 256; return o; };
  w.gram = take(sizeof(double) * n * n * count);  // Grams; dsyevd overwrites them with the eigenvectors
  w.lam = take(sizeof(double) * n * count);
  w.offd = take(sizeof(double) * n * count);      // dsyevd's off-diagonal workspace E
  w.kry = use_krylov(n, k);
  if (w.kry) {
    const int64_t m = kry_m(k), b = kry_block(k);
    w.kQ = take(sizeof(double) * n * m * count);
    w.kY = take(sizeof(double) * n * m * count);
    w.kT = take(sizeof(double) * m * m * count);
    w.kLam = take(sizeof(double) * m * count);
    w.kOff = take(sizeof(double) * m * count);
    w.kInf = take(sizeof(int) * count * (1 + 2 * (m / b)));  // dsyevd + two Cholesky factorisations per block
    w.kC = take(sizeof(double) * m * b * count);
    w.kV = take(sizeof(double) * n * k * count);
    w.kR = take(sizeof(double) * n * k * count);
    w.kRes = take(sizeof(double) * count);
  }
  // dsyevdx (single item, HDP_EIG=dsyevdx) writes the selected eigenvectors here and may use all
  // n columns as workspace: sized n x n (an n x k buffer faulted the GPU once)
  w.Z = count == 1 ? take(sizeof(double) * n * n) : 0;
  for (int i = 0; i < count; ++i) {
    const int64_t big = items[i].out > items[i].in ? items[i].out : items[i].in;
    w.P.push_back(take(sizeof(double) * big * k));
  }
  w.ints = take(sizeof(int) * (2 + count));
  w.bytes = off;
  return w;
}

#define HDP_CHECK_BLAS(expr)                                                                    \
  do {                                                                                          \
    rocblas_status s_ = (expr);                                                                 \
    if (s_ != rocblas_status_success) {                                                         \
      ::hdp::set_error("%s failed: %s (%s:%d)", #expr, rocblas_status_to_string(s_), __FILE__, __LINE__); \
      return HDP_ESOLVER;                                                                       \
    }                                                                                           \
  } while (0)

// Block Krylov top-k of `count` Grams (n x n, fp64, column- = row-major: symmetric) at ws + w.gram: on
// success (ok = true) the k Ritz vectors of item i are columns of ws + w.kV (n x k, ld n, ascending with
// the eigenvalues) and the Ritz values are ws + w.kLam[i m + m - k ..] (ascending).  ok = false: the
// residual check failed (or a QR / eigensolver info was nonzero) -- the caller runs the full solve.
static int krylov_topk(rocblas_handle h, hipStream_t st, char* ws, const BatchWs& w, int64_t n, int k, int count,
                       int* infos, bool& ok) {
  ok = false;
  const int m = kry_m(k), b = kry_block(k), q = m / b;
  const int mm = q * b;  // directions used (== m: b divides it)
  HDP_CHECK_ARG(mm == m, "krylov_topk: block %d does not divide %d", b, m);
  const rocblas_stride sG = (rocblas_stride)(n * n), sQ = (rocblas_stride)(n * m), sT = (rocblas_stride)m * m,
                       sC = (rocblas_stride)m * b, sV = (rocblas_stride)(n * k);
  double* G = reinterpret_cast<double*>(ws + w.gram);
  double* Q = reinterpret_cast<double*>(ws + w.kQ);
  double* Y = reinterpret_cast<double*>(ws + w.kY);
  double* T = reinterpret_cast<double*>(ws + w.kT);
  double* lam = reinterpret_cast<double*>(ws + w.kLam);
  double* offd = reinterpret_cast<double*>(ws + w.kOff);
  double* C = reinterpret_cast<double*>(ws + w.kC);
  double* V = reinterpret_cast<double*>(ws + w.kV);
  double* R = reinterpret_cast<double*>(ws + w.kR);
  double* res = reinterpret_cast<double*>(ws + w.kRes);
  int rc_ = HDP_OK;
  const double one = 1.0, zero = 0.0, mone = -1.0;
  HDP_CHECK_BLAS(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host));
  // orthonormalise the n x b block X of every item in place: Cholesky QR twice (S = X^T X = R^T R, X = X R^-1);
  // rocSOLVER has no batched orgqr, and after the block Gram-Schmidt against the earlier blocks X is well
  // conditioned -- a failed factorisation (info != 0) is caught with the other infos and falls back
  int* pinfo = infos;  // [count] accumulated over the factorisations (each call sets 0 or its first bad pivot)
  int nfail_slot = 0;
  auto cholqr = [&](double* X) -> int {
    for (int pass = 0; pass < 2; ++pass) {
      HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_transpose, rocblas_operation_none, b, b,
                                                   (rocblas_int)n, &one, X, (rocblas_int)n, sQ, X, (rocblas_int)n, sQ, &zero,
                                                   C, m, sC, count));
      HDP_CHECK_BLAS(rocsolver_dpotrf_strided_batched(h, rocblas_fill_upper, b, C, m, sC, pinfo + count * (1 + nfail_slot),
                                                      count));
      ++nfail_slot;
      HDP_CHECK_BLAS(rocblas_dtrsm_strided_batched(h, rocblas_side_right, rocblas_fill_upper, rocblas_operation_none,
                                                   rocblas_diagonal_non_unit, (rocblas_int)n, b, &one, C, m, sC, X,
                                                   (rocblas_int)n, sQ, count));
    }
    return HDP_OK;
  };
  {
    const int64_t tot = n * b * count;
    hipLaunchKernelGGL(kry_init_kernel, dim3((unsigned)std::min<int64_t>((tot + 255) / 256, 8192)), dim3(256), 0, st, Q,
                       n, b, (int64_t)sQ, count);
    HDP_CHECK_LAUNCH();
  }
  if ((rc_ = cholqr(Q))) return rc_;
  for (int j = 0; j < q; ++j) {
    double* Qj = Q + (int64_t)j * b * n;
    double* Yj = Y + (int64_t)j * b * n;
    // Y_j = G Q_j
    HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, b,
                                                 (rocblas_int)n, &one, G, (rocblas_int)n, sG, Qj, (rocblas_int)n, sQ, &zero,
                                                 Yj, (rocblas_int)n, sQ, count));
    if (j + 1 == q) break;
    // Q_{j+1} = orth(Y_j) against Q_0 .. Q_j: two passes of X -= Q (Q^T X), then Householder QR
    double* X = Q + (int64_t)(j + 1) * b * n;
    HDP_CHECK_HIP(hipMemcpy2DAsync(X, sizeof(double) * sQ, Yj, sizeof(double) * sQ, sizeof(double) * n * b, count,
                                   hipMemcpyDeviceToDevice, st));
    const int mj = (j + 1) * b;
    for (int pass = 0; pass < 2; ++pass) {
      HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_transpose, rocblas_operation_none, mj, b,
                                                   (rocblas_int)n, &one, Q, (rocblas_int)n, sQ, X, (rocblas_int)n, sQ, &zero,
                                                   C, m, sC, count));
      HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, b,
                                                   mj, &mone, Q, (rocblas_int)n, sQ, C, m, sC, &one, X, (rocblas_int)n,
                                                   sQ, count));
    }
    if ((rc_ = cholqr(X))) return rc_;
  }
  // Rayleigh-Ritz: T = Q^T (G Q) = Q^T Y (mm x mm, ld m), eigenpairs ascending
  HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_transpose, rocblas_operation_none, mm, mm,
                                               (rocblas_int)n, &one, Q, (rocblas_int)n, sQ, Y, (rocblas_int)n, sQ, &zero, T, m,
                                               sT, count));
  HDP_CHECK_BLAS(rocsolver_dsyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, mm, T, m, sT, lam,
                                                  (rocblas_stride)m, offd, (rocblas_stride)m, infos, count));
  // (mm == m: the top k Ritz values sit at lam[i m + m - k ..], as the caller reads them)
  // Ritz vectors V = Q Z_k and their products R = G V = Y Z_k (Z_k = the last k columns of T)
  const double* Zk = T + (int64_t)(mm - k) * m;
  HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, k, mm,
                                               &one, Q, (rocblas_int)n, sQ, Zk, m, sT, &zero, V, (rocblas_int)n, sV, count));
  HDP_CHECK_BLAS(rocblas_dgemm_strided_batched(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, k, mm,
                                               &one, Y, (rocblas_int)n, sQ, Zk, m, sT, &zero, R, (rocblas_int)n, sV, count));
  HDP_CHECK_HIP(hipMemsetAsync(res, 0, sizeof(double) * count, st));
  hipLaunchKernelGGL(kry_resid_kernel, dim3((unsigned)k, (unsigned)count), dim3(256), 0, st, R, V, lam, n, k,
                     (int64_t)sV, (int64_t)m, mm, res);
  HDP_CHECK_LAUNCH();
  std::vector<double> hres(count, 1.0);
  const int ninf = count * (1 + nfail_slot);
  std::vector<int> hinf(ninf, 1);
  HDP_CHECK_HIP(hipMemcpyAsync(hres.data(), res, sizeof(double) * count, hipMemcpyDeviceToHost, st));
  HDP_CHECK_HIP(hipMemcpyAsync(hinf.data(), infos, sizeof(int) * ninf, hipMemcpyDeviceToHost, st));
  HDP_CHECK_HIP(hipStreamSynchronize(st));
  ok = true;
  for (int i = 0; i < ninf; ++i) ok = ok && hinf[i] == 0;
  for (int i = 0; i < count; ++i) ok = ok && hres[i] <= kKryTol && hres[i] == hres[i];
  if (getenv("HDP_EIG_TRACE")) {
    double mx = 0.0;
    for (int i = 0; i < count; ++i) mx = hres[i] > mx ? hres[i] : mx;
    fprintf(stderr, "hdp_svd: block Krylov n=%lld k=%d m=%d count=%d max residual %.3e -> %s\n", (long long)n, k, mm,
            count, mx, ok ? "accepted" : "full solve");
  }
  return HDP_OK;
}

}  // namespace hdp

using namespace hdp;

extern "C" size_t hdp_svd_batch_workspace_bytes(int count, const hdp_svd_item* items, int k) {
  if (count <= 0 || !items || k <= 0) return 0;
  return batch_ws(items, count, k).bytes;
}

extern "C" size_t hdp_svd_workspace_bytes(int64_t out, int64_t in, int k) {
  if (out <= 0 || in <= 0 || k <= 0) return 0;
  hdp_svd_item it{};
  it.out = out;
  it.in = in;
  return batch_ws(&it, 1, k).bytes;
}

extern "C" int hdp_svd_topk_batched(int count, const hdp_svd_item* items, int w_dtype, int r, int nranks,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  HDP_CHECK_ARG(count >= 1 && items, "hdp_svd_topk_batched: count = %d", count);
  HDP_CHECK_ARG(r > 0 && nranks > 0, "hdp_svd_topk: bad r / nranks");
  HDP_CHECK_ARG(w_dtype == HDP_F32 || w_dtype == HDP_BF16, "hdp_svd_topk: bad dtype %d", w_dtype);
  const int64_t n = items[0].out < items[0].in ? items[0].out : items[0].in;
  const int64_t k64 = (int64_t)r * nranks;
  for (int i = 0; i < count; ++i) {
    const hdp_svd_item& it = items[i];
    HDP_CHECK_ARG(it.out > 0 && it.in > 0, "hdp_svd_topk: bad shape (item %d)", i);
    HDP_CHECK_ARG((it.out < it.in ? it.out : it.in) == n,
                  "hdp_svd_topk_batched: items of one batch need the same min(out, in) (item %d)", i);
  }
  HDP_CHECK_ARG(k64 <= n, "hdp_svd_topk: ranks_per_gpu*world_size = %lld exceeds min(out,in) = %lld",
                (long long)k64, (long long)n);
  for (int i = 0; i < count; ++i)
    HDP_CHECK_ARG(items[i].W && items[i].A_all && items[i].B_all, "hdp_svd_topk: null pointer (item %d)", i);
  HDP_CHECK_ARG(n < (1ll << 31) && n * n * count < (1ll << 62), "hdp_svd_topk: matrix too large for rocSOLVER");
  const int k = (int)k64;
  HDP_CHECK_ARG(workspace, "hdp_svd_topk: null workspace");
  const BatchWs w = batch_ws(items, count, k);
  HDP_CHECK_ARG(workspace_bytes >= w.bytes, "hdp_svd_topk: workspace %zu < %zu bytes", workspace_bytes, w.bytes);
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  double* gram0 = reinterpret_cast<double*>(ws + w.gram);
  double* lam0 = reinterpret_cast<double*>(ws + w.lam);
  int* ints = reinterpret_cast<int*>(ws + w.ints);  // [0] nev (dsyevdx), [1] dsyevdx info, [2..] batch infos
  const int el = w_dtype == HDP_F32 ? EL_F32 : EL_BF16;
  int rc;

  // 1. Grams (n x n, float64), one per item
  for (int i = 0; i < count; ++i) {
    const hdp_svd_item& it = items[i];
    GemmF64Args g;
    g.M = n;
    g.N = n;
    g.c = gram0 + (int64_t)i * n * n;
    g.ldc = n;
    g.a = it.W;
    g.b = it.W;
    if (it.out >= it.in) {  // C[i][j] = sum_o W[o][i] W[o][j]
      g.K = it.out;
      g.a_sm = 1; g.a_sk = it.in;
      g.b_sk = it.in; g.b_sn = 1;
    } else {                // C[i][j] = sum_c W[i][c] W[j][c]
      g.K = it.in;
      g.a_sm = it.in; g.a_sk = 1;
      g.b_sk = 1; g.b_sn = it.in;
    }
    rc = el == EL_F32 ? gemm_f64<EL_F32, EL_F32, true>(g, st) : gemm_f64<EL_BF16, EL_BF16, true>(g, st);
    if (rc) return rc;
  }

  // 2. eigenpairs (ascending order; column n-1 is the largest)
  rocblas_handle h;
  if ((rc = blas_handle(&h))) return rc;
  if (rocblas_set_stream(h, st) != rocblas_status_success) {
    set_error("rocblas_set_stream failed");
    return HDP_ESOLVER;
  }
  const bool sx = count == 1 && use_syevdx();
  rocblas_status rs = rocblas_status_success;
  bool kry_ok = false;
  if (w.kry) {
    rc = krylov_topk(h, st, ws, w, n, k, count, reinterpret_cast<int*>(ws + w.kInf), kry_ok);
    if (rc) return rc;
  }
  if (kry_ok) {
    // (the Ritz pairs are in place: projections below read w.kV / w.kLam)
  } else if (sx) {
    double* Z = reinterpret_cast<double*>(ws + w.Z);
    rs = rocsolver_dsyevdx(h, rocblas_evect_original, rocblas_erange_index, rocblas_fill_upper, (rocblas_int)n,
                           gram0, (rocblas_int)n, 0.0, 1.0, (rocblas_int)(n - k + 1), (rocblas_int)n, ints, lam0, Z,
                           (rocblas_int)n, ints + 1);
  } else {
    double* offd = reinterpret_cast<double*>(ws + w.offd);
    rs = rocsolver_dsyevd_strided_batched(h, rocblas_evect_original, rocblas_fill_upper, (rocblas_int)n, gram0,
                                          (rocblas_int)n, (rocblas_stride)(n * n), lam0, (rocblas_stride)n, offd,
                                          (rocblas_stride)n, ints + 2, (rocblas_int)count);
  }
  if (rs != rocblas_status_success) {
    set_error("rocsolver eigensolver failed: %s", rocblas_status_to_string(rs));
    return HDP_ESOLVER;
  }
  HDP_POST_LAUNCH(st);

  // 3. projections + factor epilogues
  for (int i = 0; i < count; ++i) {
    const hdp_svd_item& it = items[i];
    const bool tall = it.out >= it.in;
    // k eigenvectors (column-major, ld n) and eigenvalues, ascending
    const double* Zk = kry_ok ? reinterpret_cast<const double*>(ws + w.kV) + (int64_t)i * n * k
                       : sx   ? reinterpret_cast<const double*>(ws + w.Z)
                              : gram0 + (int64_t)i * n * n + (n - k) * n;
    const double* lamk = kry_ok ? reinterpret_cast<const double*>(ws + w.kLam) + (int64_t)i * kry_m(k) + (kry_m(k) - k)
                         : sx   ? lam0
                                : lam0 + (int64_t)i * n + (n - k);
    double* P = reinterpret_cast<double*>(ws + w.P[i]);
    GemmF64Args p;
    if (tall) {  // P[o][j] = sum_c W[o][c] Z[c][j]
      p.M = it.out; p.N = k; p.K = it.in;
      p.a = it.W; p.a_sm = it.in; p.a_sk = 1;
      p.b = Zk; p.b_sk = 1; p.b_sn = n;
      p.c = P; p.ldc = k;
      rc = el == EL_F32 ? gemm_f64<EL_F32, EL_F64>(p, st) : gemm_f64<EL_BF16, EL_F64>(p, st);
    } else {     // P[j][c] = sum_o Z[o][j] W[o][c]
      p.M = k; p.N = it.in; p.K = it.out;
      p.a = Zk; p.a_sm = n; p.a_sk = 1;
      p.b = it.W; p.b_sk = it.in; p.b_sn = 1;
      p.c = P; p.ldc = it.in;
      rc = el == EL_F32 ? gemm_f64<EL_F64, EL_F32>(p, st) : gemm_f64<EL_F64, EL_BF16>(p, st);
    }
    if (rc) return rc;
    FactorArgs f{Zk, lamk, P, n, it.out, it.in, k, r, tall ? 1 : 0, it.A_all, it.B_all, it.S};
    const int64_t tot = (int64_t)k * (it.in + it.out);
    hipLaunchKernelGGL(svd_factor_kernel, dim3((unsigned)((tot + 255) / 256 < 4096 ? (tot + 255) / 256 : 4096)),
                       dim3(256), 0, st, f);
    HDP_CHECK_LAUNCH();
  }

  std::vector<int> host_ints(2 + count, 0);
  HDP_CHECK_HIP(hipMemcpyAsync(host_ints.data(), ints, sizeof(int) * (2 + count), hipMemcpyDeviceToHost, st));
  HDP_CHECK_HIP(hipStreamSynchronize(st));
  if (kry_ok) {
    // (the Krylov path checked its own infos and residuals before the projections)
  } else if (sx) {
    if (host_ints[1] != 0 || host_ints[0] != k) {
      set_error("rocsolver dsyevdx: info=%d nev=%d (expected %d)", host_ints[1], host_ints[0], k);
      return HDP_ESOLVER;
    }
  } else {
    for (int i = 0; i < count; ++i)
      if (host_ints[2 + i] != 0) {
        set_error("rocsolver dsyevd: info=%d for item %d of the batch", host_ints[2 + i], i);
        return HDP_ESOLVER;
      }
  }
  return HDP_OK;
}

extern "C" int hdp_svd_topk(const void* W, int w_dtype, int64_t out, int64_t in, int r, int nranks, float* A_all,
                            float* B_all, double* S, void* workspace, size_t workspace_bytes, void* stream) {
  HDP_CHECK_ARG(out > 0 && in > 0 && r > 0 && nranks > 0, "hdp_svd_topk: bad shape");
  hdp_svd_item it;
  it.W = W;
  it.out = out;
  it.in = in;
  it.A_all = A_all;
  it.B_all = B_all;
  it.S = S;
  return hdp_svd_topk_batched(1, &it, w_dtype, r, nranks, workspace, workspace_bytes, stream);
}
