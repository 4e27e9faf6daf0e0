// K1: SVD-slice initializer -- replaces hp:106-125.
//
// The reference runs a full torch.svd of every targeted W on every rank and keeps r
// triplets.  Only the top k = r * nranks triplets are ever used, so here:
//   1. Gram  = W^T W (out >= in) or W W^T (out < in), float64 accumulation of float32/bf16
//      inputs on fp64 MFMA (v_mfma_f64_16x16x4_f64) -- products of fp32 values are exact.
//   2. eigenpairs of the n x n Gram (n = min(out, in)) with rocSOLVER dsyevd, batched over the
//      modules that share n (strided batched); the top k columns are used.  HDP_EIG=dsyevdx
//      selects the index-range solver (top k only) for single-matrix calls.
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

// C[M][N] = sum_k a(m,k) b(k,n); 256 threads, 64x64 tile, 4 waves of 32x32 (2x2 MFMA blocks)
template <int AEL, int BEL>
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmF64Args g) {
  __shared__ double As[GK][GB + 1];
  __shared__ double Bs[GK][GB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nN = (int)((g.N + GB - 1) / GB);
  const int64_t m0 = (int64_t)(blockIdx.x / nN) * GB, n0 = (int64_t)(blockIdx.x % nN) * GB;
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
        if (m < g.M && n < g.N) g.c[m * g.ldc + n] = acc[x][y][reg];
      }
}

template <int AEL, int BEL>
static int gemm_f64(const GemmF64Args& g, hipStream_t st) {
  const int64_t nb = ((g.M + GB - 1) / GB) * ((g.N + GB - 1) / GB);
  {
    KTimer kt(K_SVD_GEMM, st, 8.0 * (g.M * g.K + g.K * g.N + g.M * g.N), 2.0 * g.M * g.N * g.K);
    hipLaunchKernelGGL((gemm_f64_kernel<AEL, BEL>), dim3((unsigned)nb), dim3(256), 0, st, g);
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
};
static BatchWs batch_ws(const hdp_svd_item* items, int count, int k) {
  BatchWs w;
  const int64_t n = items[0].out < items[0].in ? items[0].out : items[0].in;
  size_t off = 0;
  auto take = [&](size_t b) { size_t o = off; off += (b + 255) / 256 * 256; return o; };
  w.gram = take(sizeof(double) * n * n * count);  // Grams; dsyevd overwrites them with the eigenvectors
  w.lam = take(sizeof(double) * n * count);
  w.offd = take(sizeof(double) * n * count);      // dsyevd's off-diagonal workspace E
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
    rc = el == EL_F32 ? gemm_f64<EL_F32, EL_F32>(g, st) : gemm_f64<EL_BF16, EL_BF16>(g, st);
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
  rocblas_status rs;
  if (sx) {
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
    const double* Zk = sx ? reinterpret_cast<const double*>(ws + w.Z) : gram0 + (int64_t)i * n * n + (n - k) * n;
    const double* lamk = sx ? lam0 : lam0 + (int64_t)i * n + (n - k);
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
  if (sx) {
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
