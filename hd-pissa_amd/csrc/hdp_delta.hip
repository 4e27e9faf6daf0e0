// K4: fused low-rank delta GEMM (+ optional merge) -- replaces hp:389-394.
//
//   dW = 0;  for i in 0..nseg-1:  dW -= dB_i (A_i - dA_i) + B_i dA_i      (hp:392 bracket)
//   MODE STORE: dst(f32)  = dW            MODE MERGE: W_res = W_res + dW  (in place)
//
// Per rank segment the bracket is one K = 2r product  L_i R_i  with
//   L_i = [dB_i | B_i]  (out x 2r),   R_i = [A_i - dA_i ; dA_i]  (2r x in),
// the cancellation-free form of B'A' - BA (SURVEY 7.2 hard part 2).
//
// MFMA mapping (v_mfma_f32_32x32x2_f32, exact fp32 fma chain; guide sec. 3):
//   operand a: lane l supplies Am[i = l&31][kk = l>>5]   operand b: Bm[kk = l>>5][j = l&31]
//   result   : lane l holds D[i = (reg&3) + 8(reg>>2) + 4(l>>5)][j = l&31], reg in [0,16)
// We compute D = dW^T tiles: i <-> output column c, j <-> output row o, and at step s the
// two k-slots are kk=0 -> (dB[o][s], A[s][c]-dA[s][c]), kk=1 -> (B[o][s], dA[s][c]).  So a
// lane owns ONE output row o and, per 32x32 block, four runs of 4 consecutive columns
// (c = 8g + 4h + q): every epilogue access is a 16-byte (f32) / 8-byte (bf16) vector.
//
// Rounding: float32 models accumulate all K = 2 r nseg products in one MFMA chain; with
// round_bf16 (bf16 models) each segment's bracket is summed alone and subtracted from a
// running dW that is rounded to bf16 after every segment, as the reference's bf16
// zeros_like(W_res) does (hp:389-392).
//
// Tiling (cdna_hip_programming.md 5, "minimum 2-phase"): 256-thread workgroup = 4 waves
// (2 x 2), workgroup tile 128 (o) x 128 (c), wave tile 64 x 64 = 2 x 2 blocks of 32 x 32.
// Per chunk (one segment, 16 steps = 32 k-slots) the workgroup stages L = [dB | B] rows
// (transposed to [kslot][o]) and R = [A - dA ; dA] (the subtraction done once here) into one
// of two LDS buffers from the natural row-major factor layouts with 16-byte loads; the next
// chunk's global loads are issued before the current chunk's 64 MFMAs per wave, and the W
// tile of a MERGE is prefetched into registers during the last chunk.  LDS reads are
// lane-consecutive (conflict-free).  Tiles are dealt XCD-contiguous (c-minor).
//
// Roofline per output element: STORE 4 B write, MERGE f32 8 B (r+w), bf16 4 B;
// MFMA work 4 r nseg flop.  Ridge (157 TF / 6.3 TB/s) ~ 25 flop/B.
#include <type_traits>

#include "hdp_common.h"

namespace hdp {

struct DeltaArgs {
  int64_t out, in;
  int r, nseg;
  const float* dA;
  const float* dB;
  int64_t dstr;
  const float* A;
  const float* B;
  int64_t fstr;
  void* dst;
  int vec_l;   // L rows 16-B aligned (r % 4 == 0, aligned bases and strides)
  int vec_r;   // R rows 16-B aligned (in % 4 == 0, aligned bases and strides)
  int vec_io;  // dst rows vector-aligned (in % 4 == 0, aligned base)
};

constexpr int kDT = 128;             // workgroup tile (both dims)
constexpr int kSC = 16;              // steps per chunk -> 32 k-slots (16 dB|A-dA, 16 B|dA)
constexpr int kLDS = 2 * 32 * kDT;   // floats per buffer: L [32][128] + R [32][128]

// staging registers of one chunk (per thread): its L row part (16 floats) and two R
// positions (A and dA float4 each)
struct Stage {
  f32x4 l[4];
  f32x4 ra[2], rd[2];
};

// chunk -> (segment, first step)
__device__ __forceinline__ void chunk_pos(const DeltaArgs& a, int c, int& seg, int& s0) {
  const int per = (a.r + kSC - 1) / kSC;
  seg = c / per;
  s0 = (c % per) * kSC;
}

__device__ __forceinline__ void stage_load(const DeltaArgs& a, int c, int64_t o_t, int64_t c_t, int tid, Stage& st) {
  int seg, s0;
  chunk_pos(a, c, seg, s0);
  // L: thread -> (row, part); part 0 = dB row, part 1 = B row; 16 consecutive steps
  const int lrow = tid & (kDT - 1), lpart = tid >> 7;
  const int64_t go = min(o_t + lrow, a.out - 1);
  const float* Lrow = (lpart ? a.B + seg * a.fstr : a.dB + seg * a.dstr) + go * a.r + s0;
  if (a.vec_l && s0 + kSC <= a.r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) st.l[q] = *reinterpret_cast<const f32x4*>(Lrow + 4 * q);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) st.l[q][e] = (s0 + 4 * q + e < a.r) ? Lrow[4 * q + e] : 0.f;
  }
  // R: positions p = tid + 256u over 16 steps x 32 column-quads
  const float* As = a.A + seg * a.fstr;
  const float* dAs = a.dA + seg * a.dstr;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = tid + 256 * u;
    const int s = s0 + (p >> 5);
    const int64_t gc = c_t + 4 * (p & 31);
    if (s < a.r && a.vec_r && gc + 3 < a.in) {
      st.ra[u] = *reinterpret_cast<const f32x4*>(As + (int64_t)s * a.in + gc);
      st.rd[u] = *reinterpret_cast<const f32x4*>(dAs + (int64_t)s * a.in + gc);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = s < a.r && gc + e < a.in;
        st.ra[u][e] = ok ? As[(int64_t)s * a.in + gc + e] : 0.f;
        st.rd[u][e] = ok ? dAs[(int64_t)s * a.in + gc + e] : 0.f;
      }
    }
  }
}

// LDS image per buffer: L[kslot][o_local] then R[kslot][c_local]; kslot = 16*half + step
__device__ __forceinline__ void stage_store(float* buf, int tid, const Stage& st) {
  const int lrow = tid & (kDT - 1), lpart = tid >> 7;
  float* L = buf;
  float* R = buf + 32 * kDT;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) L[(lpart * 16 + 4 * q + e) * kDT + lrow] = st.l[q][e];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = tid + 256 * u;
    const int s = p >> 5, c4 = 4 * (p & 31);
    *reinterpret_cast<f32x4*>(R + s * kDT + c4) = st.ra[u] - st.rd[u];   // A - dA
    *reinterpret_cast<f32x4*>(R + (16 + s) * kDT + c4) = st.rd[u];       // dA
  }
}

template <int MODE, int DT>
struct WPrefetch;
template <>
struct WPrefetch<HDP_DW_STORE, HDP_F32> {
  __device__ __forceinline__ void load(const DeltaArgs&, int64_t, int64_t, int) {}
};
template <int DT>
struct WPrefetch<HDP_DW_MERGE, DT> {
  // 2 (bo) x 2 (bc) x 4 (g) runs of 4 elements, one row per lane
  typename std::conditional<DT == HDP_F32, f32x4, u16x4>::type w[2][2][4];
  __device__ __forceinline__ void load(const DeltaArgs& a, int64_t o_w, int64_t c_w, int lane) {
    const int l32 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int64_t idx = (o_w + 32 * bo + l32) * a.in + c_w + 32 * bc + 8 * g + 4 * h;
          if constexpr (DT == HDP_F32) w[bo][bc][g] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(a.dst) + idx);
          else w[bo][bc][g] = *reinterpret_cast<const u16x4*>(reinterpret_cast<const uint16_t*>(a.dst) + idx);
        }
  }
};

template <int MODE, int DT, bool ROUND>
__global__ __launch_bounds__(256, 2) void delta_gemm_kernel(DeltaArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * kLDS];
  const int nC = (int)((a.in + kDT - 1) / kDT);
  const int nO = (int)((a.out + kDT - 1) / kDT);
  const int id = xcd_remap(blockIdx.x, nO * nC);
  const int tO = id / nC, tC = id % nC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t o_t = (int64_t)tO * kDT, c_t = (int64_t)tC * kDT;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;  // wave offsets inside the tile
  const int64_t o_w = o_t + ow, c_w = c_t + cw;
  const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in) && a.vec_io;
  const int per = (a.r + kSC - 1) / kSC;
  const int nchunks = a.nseg * per;

  f32x16 acc[2][2];
  f32x16 run[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        acc[x][y][e] = 0.f;
        run[x][y][e] = 0.f;
      }
  WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;

  Stage st;
  stage_load(a, 0, o_t, c_t, tid, st);
  stage_store(smem, tid, st);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const float* buf = smem + (c & 1) * kLDS;
    if (c + 1 < nchunks) stage_load(a, c + 1, o_t, c_t, tid, st);       // next chunk in flight
    if constexpr (MODE == HDP_DW_MERGE) {
      if (c + 1 == nchunks && full) wpf.load(a, o_w, c_w, lane);       // W tile in flight
    }
    const float* L = buf;
    const float* R = buf + 32 * kDT;
#pragma unroll
    for (int s = 0; s < kSC; ++s) {
      const int ks = 16 * h + s;
      const float r0 = R[ks * kDT + cw + l32], r1 = R[ks * kDT + cw + 32 + l32];
      const float b0 = L[ks * kDT + ow + l32], b1 = L[ks * kDT + ow + 32 + l32];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(r0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(r0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(r1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(r1, b1, acc[1][1], 0, 0, 0);
    }
    if (ROUND && (c + 1) % per == 0) {  // end of a rank segment: dW = bf16(dW - bracket_i)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            run[x][y][e] = round_bf16(run[x][y][e] - acc[x][y][e]);
            acc[x][y][e] = 0.f;
          }
    }
    if (c + 1 < nchunks) {
      // the other buffer was last read in chunk c-1, before the previous barrier: free
      stage_store(smem + ((c + 1) & 1) * kLDS, tid, st);
      __syncthreads();
    }
  }
  if (!ROUND) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) run[x][y][e] = -acc[x][y][e];
  }

  // ---- epilogue: lane owns row o, columns c = cb + 8g + 4h + q ----
#pragma unroll
  for (int bo = 0; bo < 2; ++bo) {
    const int64_t o = o_w + 32 * bo + l32;
#pragma unroll
    for (int bc = 0; bc < 2; ++bc) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t c = c_w + 32 * bc + 8 * g + 4 * h;
        f32x4 val{run[bc][bo][4 * g + 0], run[bc][bo][4 * g + 1], run[bc][bo][4 * g + 2],
                  run[bc][bo][4 * g + 3]};
        const int64_t idx = o * a.in + c;
        if (full) {
          if constexpr (MODE == HDP_DW_STORE) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.dst) + idx) = val;
          } else if constexpr (DT == HDP_F32) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.dst) + idx) = wpf.w[bo][bc][g] + val;
          } else {
            u16x4 w = wpf.w[bo][bc][g], nw;
#pragma unroll
            for (int q = 0; q < 4; ++q) nw[q] = f32_to_bf16(bf16_to_f32(w[q]) + round_bf16(val[q]));
            *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(a.dst) + idx) = nw;
          }
        } else if (o < a.out) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (c + q >= a.in) continue;
            if constexpr (MODE == HDP_DW_STORE) {
              reinterpret_cast<float*>(a.dst)[idx + q] = val[q];
            } else if constexpr (DT == HDP_F32) {
              reinterpret_cast<float*>(a.dst)[idx + q] += val[q];
            } else {
              uint16_t* p = reinterpret_cast<uint16_t*>(a.dst) + idx + q;
              *p = f32_to_bf16(bf16_to_f32(*p) + round_bf16(val[q]));
            }
          }
        }
      }
    }
  }
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace hdp

using namespace hdp;

extern "C" int hdp_delta_gemm(int64_t out, int64_t in, int r, int nseg, const float* dA, const float* dB,
                              int64_t delta_seg_stride, const float* A, const float* B,
                              int64_t factor_seg_stride, void* dst, int dst_dtype, int mode, int round_bf16,
                              void* stream) {
  HDP_CHECK_ARG(out > 0 && in > 0 && r > 0 && nseg > 0, "hdp_delta_gemm: bad shape out=%lld in=%lld r=%d nseg=%d",
                (long long)out, (long long)in, r, nseg);
  HDP_CHECK_ARG(out * in < (int64_t)1 << 40, "hdp_delta_gemm: matrix too large");
  HDP_CHECK_ARG(dA && dB && A && B && dst, "hdp_delta_gemm: null pointer");
  HDP_CHECK_ARG(mode == HDP_DW_STORE || mode == HDP_DW_MERGE, "hdp_delta_gemm: bad mode %d", mode);
  HDP_CHECK_ARG(dst_dtype == HDP_F32 || dst_dtype == HDP_BF16, "hdp_delta_gemm: bad dtype %d", dst_dtype);
  HDP_CHECK_ARG(mode == HDP_DW_MERGE || dst_dtype == HDP_F32, "hdp_delta_gemm: STORE mode writes float32");
  HDP_CHECK_ARG(!(round_bf16 && mode == HDP_DW_MERGE && dst_dtype == HDP_F32),
                "hdp_delta_gemm: round_bf16 applies to bf16 W_res (or STORE), not to a float32 merge");
  HDP_CHECK_ARG(nseg == 1 || (delta_seg_stride > 0 && factor_seg_stride > 0),
                "hdp_delta_gemm: segment strides must be positive");
  DeltaArgs a;
  a.out = out;
  a.in = in;
  a.r = r;
  a.nseg = nseg;
  a.dA = dA;
  a.dB = dB;
  a.dstr = delta_seg_stride;
  a.A = A;
  a.B = B;
  a.fstr = factor_seg_stride;
  a.dst = dst;
  const bool strides4 = nseg == 1 || (delta_seg_stride % 4 == 0 && factor_seg_stride % 4 == 0);
  a.vec_l = (r % 4 == 0) && al16(dB) && al16(B) && strides4;
  a.vec_r = (in % 4 == 0) && al16(dA) && al16(A) && strides4;
  const int esz = dst_dtype == HDP_F32 ? 16 : 8;
  a.vec_io = (in % 4 == 0) && ((reinterpret_cast<uintptr_t>(dst) % esz) == 0);
  const int64_t nwg = ((out + kDT - 1) / kDT) * ((in + kDT - 1) / kDT);
  HDP_CHECK_ARG(nwg < (1ll << 31), "hdp_delta_gemm: grid too large");
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)nwg), block(256);
  // fp32: one accumulation chain over all K = 2 r nseg (float32 rounding differs from the
  // reference's rank-by-rank sum only at the 1e-7 level); bf16 with round_bf16: the
  // rank-ordered running sum with bf16 rounding after every segment, as hp:389-392 does.
  const bool rnd = round_bf16 != 0;
#define HDP_LAUNCH(M, D, R) hipLaunchKernelGGL((delta_gemm_kernel<M, D, R>), grid, block, 0, st, a)
  // algorithmic work: dst written (and W read for MERGE) once + the 4 factor operands once
  const double wes = (mode == HDP_DW_MERGE && dst_dtype == HDP_BF16) ? 2.0 : 4.0;
  KTimer kt(nseg == 1 ? K_DELTA : K_DELTA_MULTI, st, (double)out * in * (mode == HDP_DW_MERGE ? 2.0 * wes : 4.0) + 8.0 * r * (out + in) * nseg,
            4.0 * out * in * r * nseg);
  if (mode == HDP_DW_STORE) {
    if (rnd) HDP_LAUNCH(HDP_DW_STORE, HDP_F32, true);
    else HDP_LAUNCH(HDP_DW_STORE, HDP_F32, false);
  } else if (dst_dtype == HDP_F32) {
    HDP_LAUNCH(HDP_DW_MERGE, HDP_F32, false);
  } else {
    if (rnd) HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, true);
    else HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, false);
  }
#undef HDP_LAUNCH
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}
