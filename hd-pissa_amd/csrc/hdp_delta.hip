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
// Rank order and rounding follow the reference: each segment's bracket is summed in its own
// accumulator and subtracted from the running dW (f32); with round_bf16 the running sum is
// rounded to bf16 after every segment, as the reference's bf16 zeros_like(W_res) does.
//
// Tiling: 256-thread workgroup = 4 waves (2 x 2), workgroup tile 128 (o) x 128 (c), wave
// tile 64 x 64 = 2 x 2 blocks of 32 x 32.  Operands (L: out x 2r, R: 2r x in per segment)
// are small and L2/MALL resident; each lane keeps its L row in registers per 16-step chunk
// and streams R rows (coalesced 128 B per half-wave).  Tiles are dealt XCD-contiguous
// (c-minor) so workgroups on one XCD share L rows in its L2.
//
// Roofline per output element: STORE 4 B write, MERGE f32 8 B (r+w), bf16 4 B;
// MFMA work 4 r nseg flop.  Ridge (157 TF / 6.3 TB/s) ~ 25 flop/B.
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
  int round_bf16;
  int vec_l;   // L rows 16-B aligned (r % 4 == 0, aligned bases)
  int vec_io;  // dst rows vector-aligned (in % 4 == 0, aligned base)
};

constexpr int kDT = 128;  // workgroup tile (both dims)
constexpr int kSC = 16;   // steps per operand chunk

template <bool GUARD>
__device__ __forceinline__ void load_chunk(const DeltaArgs& a, const float* Lrow0, const float* Lrow1,
                                           const float* dAs, const float* As, int64_t c0, int64_t c1,
                                           int s0, int h, int vec_l, float (&L)[2][kSC],
                                           float (&R)[2][kSC]) {
  if (!GUARD && vec_l) {
#pragma unroll
    for (int q = 0; q < kSC / 4; ++q) {
      f32x4 x0 = *reinterpret_cast<const f32x4*>(Lrow0 + s0 + 4 * q);
      f32x4 x1 = *reinterpret_cast<const f32x4*>(Lrow1 + s0 + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        L[0][4 * q + e] = x0[e];
        L[1][4 * q + e] = x1[e];
      }
    }
  } else {
#pragma unroll
    for (int ss = 0; ss < kSC; ++ss) {
      const bool ok = !GUARD || (s0 + ss < a.r);
      L[0][ss] = ok ? Lrow0[s0 + ss] : 0.f;
      L[1][ss] = ok ? Lrow1[s0 + ss] : 0.f;
    }
  }
#pragma unroll
  for (int ss = 0; ss < kSC; ++ss) {
    const bool ok = !GUARD || (s0 + ss < a.r);
    const int64_t rowoff = (int64_t)(s0 + ss) * a.in;
    float d0 = 0.f, d1 = 0.f, x0 = 0.f, x1 = 0.f;
    if (ok) {
      d0 = dAs[rowoff + c0];
      d1 = dAs[rowoff + c1];
      if (h == 0) {
        x0 = As[rowoff + c0];
        x1 = As[rowoff + c1];
      }
    }
    R[0][ss] = h ? d0 : (x0 - d0);
    R[1][ss] = h ? d1 : (x1 - d1);
  }
}

template <int MODE, int DT, bool MULTI>
__global__ __launch_bounds__(256, 2) void delta_gemm_kernel(DeltaArgs a) {
  const int nC = (int)((a.in + kDT - 1) / kDT);
  const int nO = (int)((a.out + kDT - 1) / kDT);
  const int id = xcd_remap(blockIdx.x, nO * nC);
  const int tO = id / nC, tC = id % nC;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t o_w = (int64_t)tO * kDT + (wave >> 1) * 64;
  const int64_t c_w = (int64_t)tC * kDT + (wave & 1) * 64;
  const int64_t orow0 = min(o_w + l32, a.out - 1);
  const int64_t orow1 = min(o_w + 32 + l32, a.out - 1);
  const int64_t ccol0 = min(c_w + l32, a.in - 1);
  const int64_t ccol1 = min(c_w + 32 + l32, a.in - 1);

  f32x16 acc[2][2];
  f32x16 run[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) run[x][y][e] = 0.f;

  for (int seg = 0; seg < a.nseg; ++seg) {
    const float* Lb = h ? (a.B + seg * a.fstr) : (a.dB + seg * a.dstr);
    const float* Lrow0 = Lb + orow0 * a.r;
    const float* Lrow1 = Lb + orow1 * a.r;
    const float* dAs = a.dA + seg * a.dstr;
    const float* As = a.A + seg * a.fstr;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;

    for (int s0 = 0; s0 < a.r; s0 += kSC) {
      float L[2][kSC], R[2][kSC];
      if (s0 + kSC <= a.r)
        load_chunk<false>(a, Lrow0, Lrow1, dAs, As, ccol0, ccol1, s0, h, a.vec_l, L, R);
      else
        load_chunk<true>(a, Lrow0, Lrow1, dAs, As, ccol0, ccol1, s0, h, a.vec_l, L, R);
#pragma unroll
      for (int ss = 0; ss < kSC; ++ss) {
#pragma unroll
        for (int bc = 0; bc < 2; ++bc)
#pragma unroll
          for (int bo = 0; bo < 2; ++bo)
            acc[bc][bo] = __builtin_amdgcn_mfma_f32_32x32x2f32(R[bc][ss], L[bo][ss], acc[bc][bo], 0, 0, 0);
      }
    }
    if (MULTI) {
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            float v = run[x][y][e] - acc[x][y][e];
            run[x][y][e] = a.round_bf16 ? round_bf16(v) : v;
          }
    }
  }
  if (!MULTI) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float v = -acc[x][y][e];
          run[x][y][e] = a.round_bf16 ? round_bf16(v) : v;
        }
  }

  // ---- epilogue: lane owns row o, columns c = cb + 8g + 4h + q ----
  const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in) && a.vec_io;
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
          if (MODE == HDP_DW_STORE) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.dst) + idx) = val;
          } else if (DT == HDP_F32) {
            f32x4* p = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.dst) + idx);
            *p = *p + val;
          } else {
            u16x4* p = reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(a.dst) + idx);
            u16x4 w = *p, nw;
#pragma unroll
            for (int q = 0; q < 4; ++q) nw[q] = f32_to_bf16(bf16_to_f32(w[q]) + round_bf16(val[q]));
            *p = nw;
          }
        } else if (o < a.out) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (c + q >= a.in) continue;
            if (MODE == HDP_DW_STORE) {
              reinterpret_cast<float*>(a.dst)[idx + q] = val[q];
            } else if (DT == HDP_F32) {
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
  a.round_bf16 = round_bf16 ? 1 : 0;
  a.vec_l = (r % 4 == 0) && al16(dB) && al16(B) && (nseg == 1 || (delta_seg_stride % 4 == 0 && factor_seg_stride % 4 == 0));
  const int esz = dst_dtype == HDP_F32 ? 16 : 8;
  a.vec_io = (in % 4 == 0) && ((reinterpret_cast<uintptr_t>(dst) % esz) == 0);
  const int64_t nwg = ((out + kDT - 1) / kDT) * ((in + kDT - 1) / kDT);
  HDP_CHECK_ARG(nwg < (1ll << 31), "hdp_delta_gemm: grid too large");
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)nwg), block(256);
  const bool multi = nseg > 1;
#define HDP_LAUNCH(M, D, MU) hipLaunchKernelGGL((delta_gemm_kernel<M, D, MU>), grid, block, 0, st, a)
  if (mode == HDP_DW_STORE) {
    if (multi) HDP_LAUNCH(HDP_DW_STORE, HDP_F32, true);
    else HDP_LAUNCH(HDP_DW_STORE, HDP_F32, false);
  } else if (dst_dtype == HDP_F32) {
    if (multi) HDP_LAUNCH(HDP_DW_MERGE, HDP_F32, true);
    else HDP_LAUNCH(HDP_DW_MERGE, HDP_F32, false);
  } else {
    if (multi) HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, true);
    else HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, false);
  }
#undef HDP_LAUNCH
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}
