/*
 * hdpissa.h -- C-ABI of libhdpissa.so, the MI355X-native (gfx950) implementation of
 * HD-PiSSA's per-step distributed orthogonal-adapter update.
 *
 * The reference (/root/reference/hd_pissa.py, "hp:") is a single Python file with no
 * FFI; its drop-in surface is the Python API (CustomLinearLayer, replace_with_custom_layer,
 * the optimizer-step block).  Every entry point below replaces one piece of arithmetic that
 * the reference performs through torch; the reference site is cited on each declaration.
 * The host mirror (hd-pissa_amd/hdpissa_amd, Python/ctypes) binds exactly these symbols;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain pointers are DEVICE pointers (HBM) unless stated; all matrices are dense
 *     row-major with the leading dimension equal to the row length.
 *   - Every call is asynchronous and ordered on the given HIP stream (hipStream_t passed
 *     as void*; NULL = the default stream).  Calls that allocate device memory:
 *     hdp_svd_topk / hdp_svd_topk_batched (rocSOLVER handle and info words),
 *     hdp_comm_init (RCCL), hdp_delta_plan_create (its descriptor table and, for x3 / H2
 *     plans, the packed operand panels and scale tables), hdp_probe_queue_flush (the queue's
 *     workspace, grown stream-ordered with hipMallocAsync), the first probe launch (a
 *     host-mapped error word) and the probe's pinned staging ring for its per-flush
 *     descriptor tables (host memory).  Everything else runs in caller-owned memory.
 *   - Return value: 0 on success, otherwise an HDP_E* code; hdp_last_error() gives a
 *     message (thread-local).  Shapes are validated on the host before any launch.
 *   - Not thread-safe per communicator: one host thread per process, one process per GPU
 *     (the reference's process model, hp:471-480).
 */
#ifndef HDPISSA_H
#define HDPISSA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDP_ABI_VERSION 1

/* status codes */
#define HDP_OK 0
#define HDP_EINVAL 1   /* bad argument / shape */
#define HDP_EHIP 2     /* HIP runtime error */
#define HDP_ERCCL 3    /* RCCL error */
#define HDP_ESOLVER 4  /* rocSOLVER / rocBLAS error or eigensolver non-convergence */
#define HDP_EDEVICE 5  /* a device-side check failed in an earlier launch (hdp_probe_errors) */

/* element types of model-dtype tensors (W_res, activations) */
#define HDP_F32 0
#define HDP_BF16 1

/* hdp_delta_gemm modes */
#define HDP_DW_STORE 0 /* dst (float32) <- dW                                   */
#define HDP_DW_MERGE 1 /* dst (model dtype W_res) <- W_res + dW  (fused merge)  */

typedef struct hdp_comm_s* hdp_comm; /* opaque: owns an RCCL communicator */

int hdp_abi_version(void);
const char* hdp_last_error(void);

/* ---------------------------------------------------------------------------------------
 * K5 merge -- replaces hp:394  `layer.W_res.data += delta_W_res.to(layer.W_res.dtype)`.
 * W (n elements, dtype w_dtype) += dW (float32).  bf16: W = bf16(W + bf16(dW)).
 * ------------------------------------------------------------------------------------- */
int hdp_merge(void* W, int w_dtype, const float* dW, int64_t n, void* stream);

/* Grouped K5: every module of one exchange bucket in one launch (W_i += dW_i, same semantics as
 * hdp_merge per item; items that are not 16-B aligned or a whole number of vectors fall back to
 * hdp_merge).  items is a HOST array read during the call. */
typedef struct {
  void* W;          /* n elements, w_dtype */
  const float* dW;  /* n float32 */
  int64_t n;
} hdp_merge_item;
int hdp_merge_group(int n, const hdp_merge_item* items, int w_dtype, void* stream);
/* The same with a bfloat16 dW (the rank-ordered bf16 exchange below): bf16 W_i = bf16(W_i + dW_i),
 * hp:394 with delta_W_res already bf16 (`.to(dtype)` is then the identity).  items[i].dW points at
 * n bf16 values (reinterpreted). */
int hdp_merge_group_bf16dw(int n, const hdp_merge_item* items, void* stream);

/* Rank-ordered bf16 fold -- the rounding order of hp:389-392 for a bfloat16 model:
 *   delta_W_res = zeros_like(W_res) (bf16);  for i in 0..nparts-1:  delta_W_res -= bracket_i
 * i.e. out = 0; out = bf16(out + parts[i]) for i = 0, 1, ... with parts[i] = -bracket_i (float32,
 * what K4 STORE writes for one segment).  parts: nparts rows of n floats, row i at parts + i * stride;
 * out: n bf16 values. */
int hdp_fold_bf16(const float* parts, int nparts, int64_t stride, void* out, int64_t n, void* stream);

/* ---------------------------------------------------------------------------------------
 * K3 Adam-on-factors -- replaces hp:356-373 for a flat arena of n float32 factor entries
 * (all modules' A-side and B-side concatenated).  Per element:
 *   g = grad*grad_scale; m = b1*m + omb1*g; v = b2*v + omb2*g*g;
 *   delta = lr*(m/bc1) / (sqrt(v/bc2) + eps)
 * with bc1 = 1-beta1^t, bc2 = 1-beta2^t computed by the caller (t after hp:350's increment).
 * If zero_grad != 0 the grad arena is cleared afterwards (replaces hp:397-398).
 * ------------------------------------------------------------------------------------- */
int hdp_adam_factors(float* grad, float* m, float* v, float* delta, int64_t n, float grad_scale,
                     float beta1, float one_minus_beta1, float beta2, float one_minus_beta2,
                     float bc1, float bc2, float lr, float eps, int zero_grad, void* stream);

/* ---------------------------------------------------------------------------------------
 * K4 delta GEMM -- replaces hp:389-394 (zeros_like, the per-rank loop of 3 GEMMs, merge).
 * For one module (out x in) and nseg rank segments i = 0..nseg-1:
 *   dW = 0; for i: dW -= dB_i @ (A_i - dA_i) + B_i @ dA_i       (== hp:392's bracket)
 * accumulated in rank order like the reference; with round_bf16 != 0 the running sum is
 * rounded to bf16 after every segment (the reference's zeros_like(W_res) is bf16 for a
 * bf16 model).  Segment i's operands live at
 *   dA + i*delta_seg_stride, dB + i*delta_seg_stride   (dA: r x in, dB: out x r)
 *   A  + i*factor_seg_stride, B  + i*factor_seg_stride (A: r x in,  B: out x r)
 * (strides in float elements).  One fused K = 2r*nseg MFMA pass in the math of
 * hdp_delta_set_math (below); the out x in result is never materialised in MERGE mode.
 * mode HDP_DW_STORE: dst is float32 out x in.  mode HDP_DW_MERGE: dst is W_res (dst_dtype).
 * ------------------------------------------------------------------------------------- */
int hdp_delta_gemm(int64_t out, int64_t in, int r, int nseg, const float* dA, const float* dB,
                   int64_t delta_seg_stride, const float* A, const float* B,
                   int64_t factor_seg_stride, void* dst, int dst_dtype, int mode, int round_bf16,
                   void* stream);

/* K4 math.  HDP_MATH_F32: v_mfma_f32_32x32x2_f32, a bit-exact f32 fma chain.  HDP_MATH_X3:
 * each f32 operand split exactly into three bf16 parts (24 significand bits) and the six
 * partial products that reach f32 resolution summed by v_mfma_f32_32x32x16_bf16 in f32 --
 * f32 accuracy (dropped terms < 2^-24 relative) at 2.7x the MFMA rate.  HDP_MATH_H2 (plans
 * with a float32 result -- STORE, or MERGE into float32 W -- and bf16 MERGE plans of ONE
 * segment; others fall back to X3): every k of an item scaled by powers of two (column k of L
 * into (2^13, 2^14], R's rows by 2^E / that, E per item from the live factors), each operand
 * split into fp16 hi + lo and three products summed by v_mfma_f32_32x32x16_f16 -- half the
 * MFMAs of X3, errors ~2^-22 relative (below the f32 chain's rounding; for a bf16 W the merge
 * then rounds bf16(W + bf16(-acc)) once, as the reference's single-rank bf16(W + bf16(dW));
 * when every tile of such a plan has >= 4 chunks of 32 k (r >= 49) the W read-modify-write of a
 * full tile is deferred under the next tile's chunks in 8-byte row groups -- same bits, env
 * HDP_K4_DEFER=0 keeps the immediate epilogue).
 * HDP_MATH_AUTO (the default; env HDP_K4_MATH=auto|f32|x3|h2): F32 while K = 2 r nseg <= 32
 * (HBM-bound); above that H2 where allowed, X3 otherwise (bf16 MERGE with nseg > 1: the
 * per-rank bf16 rounding of the reference's running dW needs the ROUND form on X3).  Returns
 * the previous setting (process-wide; plans keep the math of their creation). */
#define HDP_MATH_AUTO 0
#define HDP_MATH_F32 1
#define HDP_MATH_X3 2
#define HDP_MATH_H2 3
int hdp_delta_set_math(int math);

/* Staging of x3 PLANS (hdp_delta_plan_*; env HDP_K4_X3_STAGE=wide|glds|regs).  HDP_X3_WIDE (default):
 * 256x128 tiles of 8 waves, packed panels loaded straight into a 4-chunk LDS ring;
 * HDP_X3_GLDS: 128x128 tiles, 3-chunk LDS ring; HDP_X3_REGS: 128x128 tiles, 3-slot register ring.
 * Same MFMA chain per output in all three (bitwise-identical results).  A bf16 ROUND merge plan
 * takes GLDS when WIDE is set.  Returns the previous setting, or -1 for a bad stage (message in
 * hdp_last_error; process-wide; plans keep the staging of their creation). */
#define HDP_X3_REGS 0
#define HDP_X3_GLDS 1
#define HDP_X3_WIDE 2
int hdp_delta_set_x3_stage(int stage);

/* Grouped persistent form of hdp_delta_gemm -- the whole per-step loop hp:352-394 over
 * modules (or one exchange bucket of it) in ONE launch.  A plan captures the items' shapes,
 * pointers and strides once (their buffers are persistent: W_res and the factor arenas), in
 * a small device table owned by the plan; every hdp_delta_plan_run then launches one kernel
 * whose resident workgroups walk all tiles of all items, with the next tile's operands in
 * flight across tile and module boundaries.  Items share dst_dtype / mode / round_bf16 and
 * must not write overlapping dst ranges; each item's semantics equal hdp_delta_gemm's. */
typedef struct {
  int64_t out, in;
  int r, nseg;
  const float* dA;
  const float* dB;
  int64_t delta_seg_stride;
  const float* A;
  const float* B;
  int64_t factor_seg_stride;
  void* dst;
} hdp_delta_item;
typedef struct hdp_delta_plan_s* hdp_delta_plan; /* opaque */
int hdp_delta_plan_create(const hdp_delta_item* items, int n, int dst_dtype, int mode, int round_bf16,
                          hdp_delta_plan* plan);
int hdp_delta_plan_run(hdp_delta_plan plan, void* stream);
/* Adam folded into K4's operand preparation (replaces hp:356-373 + the operand pack for
 * single-segment H2 merge plans -- Wn = 1, bf16 W, r >= 32): 1 if hdp_delta_plan_run_adam applies.
 * run_adam = hdp_adam_factors over every factor entry of the plan's items (grad / m / v / delta are the
 * arenas the items' dA / dB point into: entry i of each belongs together; m, v, delta bit-identical to
 * hdp_adam_factors) + the plan run, with no scale pass over the live factors: delta_bound D >= max |delta|
 * (the host's Adam bound, lr (1 - b1) / sqrt(1 - b2) sqrt((1 - rho^t) / (1 - rho)) sqrt(1 - b2^t) /
 * (1 - b1^t), rho = b1^2 / b2, with margin) sets the delta halves' scales; a delta above D (moments not
 * from this Adam sequence) switches the same launch sequence to the live-factor pack (gated kernels). */
int hdp_delta_plan_fused_adam(hdp_delta_plan plan);
int hdp_delta_plan_run_adam(hdp_delta_plan plan, float* grad, float* m, float* v, float* delta, float grad_scale,
                            float beta1, float one_minus_beta1, float beta2, float one_minus_beta2, float bc1,
                            float bc2, float lr, float eps, float delta_bound, int zero_grad, void* stream);
/* 1 if the last run_adam took the live-factor fallback (synchronises; tests / diagnosis) */
int hdp_delta_plan_fused_fallback(hdp_delta_plan plan, int* taken);
/* run_adam packs the CONSTANT operand halves (B, and the max |A| / max |B| scale bounds) once per plan
 * and reuses them on every later run_adam.  A host that rewrites the factors A / B in place (a resumed
 * checkpoint loaded into the same arena, a re-init) calls this before the next run_adam so the constants
 * are re-packed from the new factors.  hdp_delta_plan_run does the same implicitly. */
int hdp_delta_plan_invalidate(hdp_delta_plan plan);
int hdp_delta_plan_tiles(hdp_delta_plan plan, int64_t* tiles, int* grid);
/* the math the plan runs (HDP_MATH_F32 / X3 / H2; -1 for a null plan) -- the MFMA ceiling a
 * measurement of it is priced against */
int hdp_delta_plan_math(hdp_delta_plan plan);
int hdp_delta_plan_destroy(hdp_delta_plan plan);

/* ---------------------------------------------------------------------------------------
 * K2 adapter probe backward -- replaces the autograd of hp:139's adapter term.
 * X: T x in, G: T x out (model dtype x_dtype; G is dL/dy).  B is out x r, or r x out when
 * b_transposed != 0 (B is frozen in HD-PiSSA, hp:375-376, so a host can keep B^T).  Accumulates
 *   gA (r x in)  += scale * (G @ B)^T @ X
 *   gB (out x r) += scale * G^T @ (X @ A^T)
 * (= the reference's A.grad/B.grad with scale = alpha_eff * 1e-16); accumulate == 0
 * overwrites instead.  Skinny MFMA GEMMs that never form the out x in product: float32
 * activations on v_mfma_f32_16x16x4_f32 (an exact f32 chain); bf16 activations (exact in bf16)
 * on bf16 MFMA with the float32 operand split exactly into three bf16 parts (the f32 chain's
 * accuracy).  r <= 64 on the streaming SWEEP path, 64 < r <= 128 as r-slices of 64 (B^T
 * given) or the P1/P2 split path.  workspace: device scratch of hdp_probe_workspace_bytes().
 * ------------------------------------------------------------------------------------- */
size_t hdp_probe_workspace_bytes(int64_t T, int64_t in, int64_t out, int r);
int hdp_probe_grads(int64_t T, int64_t in, int64_t out, int r, const void* X, const void* G,
                    int x_dtype, const float* A, const float* B, int b_transposed, float* gA,
                    float* gB, float scale, int accumulate, void* workspace,
                    size_t workspace_bytes, void* stream);

/* Grouped form: up to hdp_probe_group_max() modules (same ceil(r/16) block, same x_dtype, no
 * two items sharing a gradient) in one launch per pass -- what an autograd backward over a
 * decoder layer produces.  items is a HOST array read during the call; the workspace must
 * hold the sum of hdp_probe_workspace_bytes() over the items. */
typedef struct {
  const void* X;       /* T x in  (x_dtype) */
  const void* G;       /* T x out (x_dtype) */
  const float* A;      /* r x in */
  const float* B;      /* out x r, or r x out when b_transposed */
  float* gA;           /* r x in */
  float* gB;           /* out x r */
  int64_t T, in, out;
  int r;
  int b_transposed;
  int accumulate;
  float scale;
} hdp_probe_item;
int hdp_probe_group_max(void);
/* The sweep path's workgroups hand partial sums between their waves through bounded waits.  A
 * wait that gives up (a bug, never expected) sets a device error word instead of hanging the
 * GPU; while it is set, hdp_probe_grads_group / hdp_probe_queue_flush refuse with HDP_EDEVICE.
 * Returns the word (0 = no failure in any completed launch; no device synchronisation -- the
 * word is host-mapped), clear != 0 resets it. */
int hdp_probe_errors(int clear);
/* Measurement support: microseconds the host has spent blocked because the GPU was behind (a
 * flush waits for the oldest of its 64 pinned descriptor-staging slots, i.e. the host runs at
 * most 64 group flushes ahead); reset != 0 zeroes the counter.  Host time minus this is the
 * host's own cost. */
int64_t hdp_probe_host_wait_us(int reset);
int hdp_probe_grads_group(int n, const hdp_probe_item* items, int x_dtype, void* workspace,
                          size_t workspace_bytes, void* stream);

/* Native deferred-probe queue: the host runtime behind an autograd backward.  Each adapter
 * module is registered once (its constant operands); each module backward pushes (X, G, T,
 * accumulate) on a stream.  The queue launches the pending group (hdp_probe_grads_group) before
 * a push that would exceed max_items or budget_bytes of pending X + G, repeat a module, or
 * change the stream / r-block, and on hdp_probe_queue_flush.  The caller keeps every pushed
 * X and G alive until the push that reports *flushed != 0 (or the flush) has returned; the
 * queue owns a device workspace, grown on demand (after a stream synchronisation). */
typedef struct hdp_probe_queue_s* hdp_probe_queue; /* opaque */
int hdp_probe_queue_create(int x_dtype, int max_items, int64_t budget_bytes, hdp_probe_queue* q);
int hdp_probe_queue_add_module(hdp_probe_queue q, const float* A, const float* B, int b_transposed,
                               float* gA, float* gB, int64_t in, int64_t out, int r, float scale,
                               int* slot);
int hdp_probe_queue_push(hdp_probe_queue q, int slot, const void* X, const void* G, int64_t T,
                         int accumulate, void* stream, int* flushed);
int hdp_probe_queue_flush(hdp_probe_queue q);
int hdp_probe_queue_pending(hdp_probe_queue q);
int64_t hdp_probe_queue_flushes(hdp_probe_queue q);
int hdp_probe_queue_destroy(hdp_probe_queue q);

/* ---------------------------------------------------------------------------------------
 * K1 SVD-slice init -- replaces hp:106-125 (torch.svd of the whole matrix + slicing).
 * Computes only the top k singular triplets of W (out x in, dtype w_dtype) through a
 * float64 Gram matrix (fp64 MFMA), rocSOLVER dsyevd (all eigenpairs of the n x n Gram,
 * n = min(out, in); the top k are used -- env HDP_EIG=dsyevdx selects the index-range solver
 * for single-matrix calls) and an fp64 MFMA projection, and writes every rank's factors
 * (k = r * nranks):
 *   A_all: k x in         rows d*r..(d+1)*r-1 = rank d's A = diag(sqrt S_d) V_d^T
 *   B_all: nranks x out x r   slab d = rank d's B = U_d diag(sqrt S_d)
 *   S (optional, may be NULL): k singular values, descending (device, float64)
 * workspace: device scratch of hdp_svd_workspace_bytes() bytes.  Synchronous w.r.t. the
 * host (checks the solver's info).
 * ------------------------------------------------------------------------------------- */
size_t hdp_svd_workspace_bytes(int64_t out, int64_t in, int k);
int hdp_svd_topk(const void* W, int w_dtype, int64_t out, int64_t in, int r, int nranks,
                 float* A_all, float* B_all, double* S, void* workspace, size_t workspace_bytes,
                 void* stream);

/* Batched form (the init of a whole model: hp:150-156 constructs one CustomLinearLayer per
 * targeted module): count matrices that share n = min(out, in) and the dtype; their Grams go
 * through ONE rocsolver_dsyevd_strided_batched call (the solver's tridiagonalisation is a chain
 * of O(n) small launches per matrix; batched, the chain is paid once per batch).  Each item's
 * outputs are exactly hdp_svd_topk's.  workspace: hdp_svd_batch_workspace_bytes(). */
typedef struct {
  const void* W;   /* out x in, w_dtype */
  int64_t out, in;
  float* A_all;    /* k x in */
  float* B_all;    /* nranks x out x r */
  double* S;       /* k, or NULL */
} hdp_svd_item;
size_t hdp_svd_batch_workspace_bytes(int count, const hdp_svd_item* items, int k);
int hdp_svd_topk_batched(int count, const hdp_svd_item* items, int w_dtype, int r, int nranks,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Factor exchange over RCCL/xGMI -- replaces hp:379-387 (4 all_gathers per module per step)
 * and carries the dense-dW all-reduce variant.  The id is an ncclUniqueId (128 bytes)
 * created on rank 0 by hdp_comm_unique_id and shipped to the other ranks by the host
 * (the reference's TCP rendezvous, hp:216).
 * ------------------------------------------------------------------------------------- */
int hdp_comm_unique_id(unsigned char* id, size_t id_bytes);
int hdp_comm_init(hdp_comm* comm, const unsigned char* id, size_t id_bytes, int nranks, int rank);
int hdp_comm_destroy(hdp_comm comm);
/* recv = [rank0's send | rank1's send | ...]; count = float elements per rank */
int hdp_allgather_f32(hdp_comm comm, const float* send, float* recv, int64_t count, void* stream);
/* in-place sum over ranks */
int hdp_allreduce_sum_f32(hdp_comm comm, float* buf, int64_t count, void* stream);
int hdp_broadcast_bytes(hdp_comm comm, void* buf, int64_t bytes, int root, void* stream);
/* all-to-all with equal blocks: send block j (count floats at send + j * count) goes to rank j,
 * recv block i comes from rank i.  The rank-ordered bf16 exchange sends every rank the float32
 * per-rank terms of its 1/Wn shard of a dW bucket. */
int hdp_alltoall_f32(hdp_comm comm, const float* send, float* recv, int64_t count, void* stream);
/* recv = [rank0's bytes | rank1's | ...]; bytes per rank (the folded bf16 shards) */
int hdp_allgather_bytes(hdp_comm comm, const void* send, void* recv, int64_t bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Live kernel timing (measurement support, no reference counterpart).  While enabled, every
 * kernel launch of this library is bracketed by two HIP events on the stream it is launched
 * on; queries wait for the recorded events and return, per kernel id, the launch count, the
 * summed event time and the summed ALGORITHMIC bytes / flops of those launches.
 * ------------------------------------------------------------------------------------- */
int hdp_timing_enable(int on); /* returns the previous setting */
int hdp_timing_reset(void);
int hdp_timing_kernels(void); /* number of kernel ids */
int hdp_timing_query(int kid, const char** name, int64_t* launches, double* total_ms, double* bytes,
                     double* flops);

#ifdef __cplusplus
}
#endif
#endif /* HDPISSA_H */
