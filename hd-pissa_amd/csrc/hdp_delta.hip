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
// D = dW tiles: i <-> output row o (a-operand = L = [dB | B] rows), j <-> output column c
// (b-operand = R = [A - dA ; dA] columns); at step s the two k-slots are kk=0 -> (dB[o][s],
// A[s][c]-dA[s][c]) and kk=1 -> (B[o][s], dA[s][c]).  So a lane owns ONE output column per
// 32 x 32 block and 16 of its rows: for every accumulator register the wave's 64 lanes touch
// two rows x 32 consecutive elements -- whole 128-B lines for float32 W -- which is what the
// epilogue's W read-modify-write wants (the transposed, fragment-shaped mapping -- 32 rows x
// 32 B per 16-B-per-lane instruction -- ran the merge at ~4.2 TB/s).
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
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

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
  __bf16* limg;  // packed bf16x3 panels (plans with x3 math; see MX3P), else null
  __bf16* rimg;  //   (fp16x2 panels for H2 plans: the same pointers reinterpreted)
  float* ktab;   // H2 plans: the item's per-k scale table (see H2 below), else null
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
  const HDP_GLOBAL float* Lrow = gptr((lpart ? a.B + seg * a.fstr : a.dB + seg * a.dstr) + go * a.r + s0);
  if (a.vec_l && s0 + kSC <= a.r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) st.l[q] = gld4(Lrow + 4 * q);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) st.l[q][e] = (s0 + 4 * q + e < a.r) ? Lrow[4 * q + e] : 0.f;
  }
  // R: positions p = tid + 256u over 16 steps x 32 column-quads
  const HDP_GLOBAL float* As = gptr(a.A + seg * a.fstr);
  const HDP_GLOBAL float* dAs = gptr(a.dA + seg * a.dstr);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = tid + 256 * u;
    const int s = s0 + (p >> 5);
    const int64_t gc = c_t + 4 * (p & 31);
    if (s < a.r && a.vec_r && gc + 3 < a.in) {
      st.ra[u] = gld4(As + (int64_t)s * a.in + gc);
      st.rd[u] = gld4(dAs + (int64_t)s * a.in + gc);
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

// v_mfma_f32_32x32x2_f32 result register e of lane (l32, h) is row (e & 3) + 8 (e >> 2) + 4 h,
// column l32 of the 32 x 32 block
__device__ __forceinline__ int row_of(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

template <int MODE, int DT>
struct WPrefetch;
struct TileAddr;
template <>
struct WPrefetch<HDP_DW_STORE, HDP_F32> {
  template <int POL = 0>
  __device__ __forceinline__ void load(const TileAddr&) {}
};
// Full tiles address dst through a buffer descriptor: the lane part of an element's byte
// offset, (4 h in + l32) esz, is one VGPR for the whole kernel, and the row / block part is
// wave-uniform (an SGPR soffset per register) -- 64 separate 64-bit addresses per lane
// would not fit beside the accumulators and the W registers.
struct TileAddr {
  __amdgpu_buffer_rsrc_t rs;
  int voff;   // lane part
  int sbase;  // wave part: (o_w in + c_w) esz
  int rowb;   // in * esz
};
template <int ESZ>
__device__ __forceinline__ TileAddr tile_addr(const DeltaArgs& a, int64_t o_w, int64_t c_w, int l32, int h) {
  TileAddr t;
  t.rs = __builtin_amdgcn_make_buffer_rsrc(a.dst, 0, (int)(a.out * a.in * ESZ), 0x00020000);
  t.rowb = (int)(a.in * ESZ);
  t.voff = (4 * h) * t.rowb + l32 * ESZ;
  t.sbase = (int)((o_w * a.in + c_w) * ESZ);
  return t;
}
// soffset of register e of block (bo, bc)
template <int ESZ>
__device__ __forceinline__ int reg_soff(const TileAddr& t, int bo, int bc, int e) {
  return t.sbase + ((e & 3) + 8 * (e >> 2) + 32 * bo) * t.rowb + 32 * bc * ESZ;
}

// float32 W cache policy (plan pol / HDP_DELTA_POL): bit 0 nt stores, bit 1 nt loads, bit 2
// sc1 stores, bit 3 sc1 loads (buffer aux: nt = 2, sc1 = 16).  W is touched once per plan run;
// lines it leaves in the XCD's L2 displace the packed panels the x3 kernels re-read from there.
constexpr int w_store_aux(int pol) { return ((pol & 1) ? 2 : 0) | ((pol & 4) ? 16 : 0); }
constexpr int w_load_aux(int pol) { return ((pol & 2) ? 2 : 0) | ((pol & 8) ? 16 : 0); }

template <int DT>
struct WPrefetch<HDP_DW_MERGE, DT> {
  // [bo][bc][e]: row o_w + 32 bo + row_of(e, h), column c_w + 32 bc + l32 (one element per lane
  // and register: every wave-instruction covers two full row segments of 32 elements)
  typename std::conditional<DT == HDP_F32, float, uint16_t>::type w[2][2][16];
  template <int POL = 0>  // POL bit 1: non-temporal W loads
  __device__ __forceinline__ void load(const TileAddr& t) {
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if constexpr (DT == HDP_F32)
            w[bo][bc][e] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(t.rs, t.voff, reg_soff<4>(t, bo, bc, e), w_load_aux(POL)));
          else
            w[bo][bc][e] = __builtin_amdgcn_raw_buffer_load_b16(t.rs, t.voff, reg_soff<2>(t, bo, bc, e), 0);
        }
  }
};

// one chunk (16 steps = 32 k-slots) of the wave's 64 x 64 tile from an LDS buffer
__device__ __forceinline__ void chunk_mfma(const float* buf, int h, int l32, int ow, int cw, f32x16 (&acc)[2][2]) {
  const float* L = buf;
  const float* R = buf + 32 * kDT;
#pragma unroll
  for (int s = 0; s < kSC; ++s) {
    const int ks = 16 * h + s;
    const float r0 = R[ks * kDT + cw + l32], r1 = R[ks * kDT + cw + 32 + l32];
    const float b0 = L[ks * kDT + ow + l32], b1 = L[ks * kDT + ow + 32 + l32];
    // acc[bo][bc] (rows o = a-operand from L, columns c = b-operand from R)
    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(b0, r0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b0, r1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(b1, r0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(b1, r1, acc[1][1], 0, 0, 0);
  }
}

// ---------------------------------------------------------------------------------------
// Math policies.  MF32: v_mfma_f32_32x32x2_f32 (exact f32 fma chain), 16 steps per chunk.
// MX3: every f32 operand split exactly into three bf16 parts x = x_hi + x_mid + x_lo (24
// significand bits, no rounding: each residual is exact in f32) and the product formed by
// v_mfma_f32_32x32x16_bf16 as hi*hi + hi*mid + mid*hi + hi*lo + mid*mid + lo*hi with f32
// accumulation -- the dropped terms are below 2^-24 relative, so the result carries f32
// accuracy (test_gpu_kernels: error vs fp64 at the level of the f32 chain) at 6 bf16 MFMAs
// (6 x 32 cycles) per 16 k instead of 8 f32 MFMAs (8 x 64): 2.7x the MFMA throughput where
// K4 is MFMA-bound (K = 2 r Wn >= 64).  8 steps per chunk = 16 k-slots = one k-group:
// slots 0..7 = (dB, A - dA) at steps s0..s0+7, slots 8..15 = (B, dA).
// LDS image per buffer (bf16): L parts [3][128 rows o][16 k], R parts [3][128 cols c][16 k]
// (R transposed while staging); each 16-B granule (8 k) of row x sits at granule
// g ^ ((x >> 3) & 1) -- conflict-free ds_read_b128 for the MFMA fragments and ds_write_b128
// for the staging (MI355X_MICROARCH.md LDS lane groups).
// ---------------------------------------------------------------------------------------
struct MF32 {
  static constexpr int kSteps = kSC;
  static constexpr int kBuf = kLDS;  // floats per LDS buffer
  using St = Stage;
  __device__ __forceinline__ static void load(const DeltaArgs& a, int c, int64_t o_t, int64_t c_t, int tid, St& st) {
    stage_load(a, c, o_t, c_t, tid, st);
  }
  __device__ __forceinline__ static void store(float* buf, int tid, const St& st) { stage_store(buf, tid, st); }
  __device__ __forceinline__ static void mfma(const float* buf, int h, int l32, int ow, int cw, f32x16 (&acc)[2][2]) {
    chunk_mfma(buf, h, l32, ow, cw, acc);
  }
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct StageX3 {
  float l[8];   // L row (dB or B) at 8 steps
  float ra[8];  // R column: A (half 0 only)
  float rd[8];  // R column: dA
};

struct MX3 {
  static constexpr int kSteps = 8;
  static constexpr int kBuf = 6 * kDT * 16 / 2;  // floats per LDS buffer (6 parts x 128 x 16 bf16)
  using St = StageX3;

  __device__ __forceinline__ static void load(const DeltaArgs& a, int c, int64_t o_t, int64_t c_t, int tid, St& st) {
    const int per = (a.r + kSteps - 1) / kSteps;
    const int seg = c / per, s0 = (c % per) * kSteps;
    const int x = tid & (kDT - 1), half = tid >> 7;  // half is wave-uniform
    // L: row o_t + x, 8 steps of dB (half 0) or B (half 1)
    const int64_t go = min(o_t + x, a.out - 1);
    const HDP_GLOBAL float* Lrow = gptr((half ? a.B + seg * a.fstr : a.dB + seg * a.dstr) + go * a.r + s0);
    if (a.vec_l && s0 + kSteps <= a.r) {
      const f32x4 v0 = gld4(Lrow), v1 = gld4(Lrow + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        st.l[q] = v0[q];
        st.l[4 + q] = v1[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < kSteps; ++q) st.l[q] = (s0 + q < a.r) ? Lrow[q] : 0.f;
    }
    // R: column c_t + x, 8 steps of A - dA (half 0) or dA (half 1); one dword per lane per
    // step (a wave covers 64 consecutive columns of one factor row)
    const int64_t gc = min(c_t + x, a.in - 1);
    const HDP_GLOBAL float* As = gptr(a.A + seg * a.fstr + gc);
    const HDP_GLOBAL float* dAs = gptr(a.dA + seg * a.dstr + gc);
#pragma unroll
    for (int q = 0; q < kSteps; ++q) {
      const bool ok = s0 + q < a.r;
      const int64_t off = (int64_t)(s0 + q) * a.in;
      st.rd[q] = ok ? dAs[off] : 0.f;
      st.ra[q] = (ok && half == 0) ? As[off] : 0.f;
    }
  }

  // exact three-way split of 8 values into packed bf16 parts
  __device__ __forceinline__ static void split8(const float (&v)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const __bf16 h = (__bf16)v[q];
      const float r1 = v[q] - (float)h;
      const __bf16 m = (__bf16)r1;
      hi[q] = h;
      mid[q] = m;
      lo[q] = (__bf16)(r1 - (float)m);
    }
  }

  __device__ __forceinline__ static int gran(int x, int g) { return g ^ ((x >> 3) & 1); }

  __device__ __forceinline__ static void store(float* buf, int tid, const St& st) {
    __bf16* b = reinterpret_cast<__bf16*>(buf);
    const int x = tid & (kDT - 1), half = tid >> 7;
    const int off = x * 16 + 8 * gran(x, half);
    bf16x8 p0, p1, p2;
    split8(st.l, p0, p1, p2);
    *reinterpret_cast<bf16x8*>(b + 0 * kDT * 16 + off) = p0;
    *reinterpret_cast<bf16x8*>(b + 1 * kDT * 16 + off) = p1;
    *reinterpret_cast<bf16x8*>(b + 2 * kDT * 16 + off) = p2;
    float rv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) rv[q] = half ? st.rd[q] : st.ra[q] - st.rd[q];
    split8(rv, p0, p1, p2);
    *reinterpret_cast<bf16x8*>(b + 3 * kDT * 16 + off) = p0;
    *reinterpret_cast<bf16x8*>(b + 4 * kDT * 16 + off) = p1;
    *reinterpret_cast<bf16x8*>(b + 5 * kDT * 16 + off) = p2;
  }

  __device__ __forceinline__ static void mfma(const float* buf, int h, int l32, int ow, int cw, f32x16 (&acc)[2][2]) {
    const __bf16* b = reinterpret_cast<const __bf16*>(buf);
    bf16x8 fa[2][3], fb[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int xa = ow + 32 * i + l32, xb = cw + 32 * i + l32;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        fa[i][p] = *reinterpret_cast<const bf16x8*>(b + p * kDT * 16 + xa * 16 + 8 * gran(xa, h));
        fb[i][p] = *reinterpret_cast<const bf16x8*>(b + (3 + p) * kDT * 16 + xb * 16 + 8 * gran(xb, h));
      }
    }
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc) {
        f32x16 d = acc[bo][bc];
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][2], fb[bc][0], d, 0, 0, 0);  // lo * hi
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][1], d, 0, 0, 0);  // mid * mid
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][2], d, 0, 0, 0);  // hi * lo
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][0], d, 0, 0, 0);  // mid * hi
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][1], d, 0, 0, 0);  // hi * mid
        d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][0], d, 0, 0, 0);  // hi * hi
        acc[bo][bc] = d;
      }
  }
};

// MX3P: MX3 with the operands PACKED once per plan run by k4_pack_kernel into exactly the
// LDS image MX3 builds -- per (chunk, 128-row / 128-column block) a 12-KB panel [3 parts]
// [128][16 k] with the granule swizzle applied -- so a K4 workgroup's staging is six 16-B
// loads and six linear ds_write_b128 per thread: the split (≈6 VALU per value) and the R
// transpose happen once per factor element instead of once per tile that reads it (32-112
// tiles per element).
struct StageX3P {
  f32x4 v[6];
};
constexpr int kPanel = 3 * kDT * 16;  // bf16 elements per packed panel

struct MX3P {
  static constexpr int kSteps = MX3::kSteps;
  static constexpr int kBuf = MX3::kBuf;
  using St = StageX3P;
  __device__ __forceinline__ static void load(const DeltaArgs& a, int c, int64_t o_t, int64_t c_t, int tid, St& st) {
    const int64_t nRB = (a.out + kDT - 1) / kDT, nCB = (a.in + kDT - 1) / kDT;
    const HDP_GLOBAL f32x4* L = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(a.limg + ((int64_t)c * nRB + o_t / kDT) * kPanel));
    const HDP_GLOBAL f32x4* R = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(a.rimg + ((int64_t)c * nCB + c_t / kDT) * kPanel));
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      st.v[p] = L[p * 256 + tid];
      st.v[3 + p] = R[p * 256 + tid];
    }
  }
  __device__ __forceinline__ static void store(float* buf, int tid, const St& st) {
    f32x4* b = reinterpret_cast<f32x4*>(buf);
#pragma unroll
    for (int p = 0; p < 6; ++p) b[p * 256 + tid] = st.v[p];
  }
  __device__ __forceinline__ static void mfma(const float* buf, int h, int l32, int ow, int cw, f32x16 (&acc)[2][2]) {
    MX3::mfma(buf, h, l32, ow, cw, acc);
  }
};

// Pack every item's panels: one thread per (item, chunk, L row block or R column block, row).
// Items are laid out in the thread space at 256-aligned offsets (workgroup-uniform item).
__global__ __launch_bounds__(256) void k4_pack_kernel(const DeltaArgs* __restrict__ items,
                                                      const int64_t* __restrict__ pack_start, int n) {
  const int64_t e0 = (int64_t)blockIdx.x * 256;
  int m = 0;
  while (m + 1 < n && e0 >= pack_start[m + 1]) ++m;
  const DeltaArgs a = items[m];
  int64_t e = e0 - pack_start[m] + threadIdx.x;
  const int per = (a.r + MX3::kSteps - 1) / MX3::kSteps;
  const int nch = a.nseg * per;
  const int64_t nRB = (a.out + kDT - 1) / kDT, nCB = (a.in + kDT - 1) / kDT;
  const int64_t nL = (int64_t)nch * nRB * kDT, nR = (int64_t)nch * nCB * kDT;
  if (e >= nL + nR) return;
  const bool left = e < nL;
  if (!left) e -= nL;
  const int64_t nb = left ? nRB : nCB;
  const int x = (int)(e % kDT);
  const int64_t pb = e / kDT;             // panel index = c * nb + block
  const int c = (int)(pb / nb);
  const int64_t blk = pb - (int64_t)c * nb;
  const int seg = c / per, s0 = (c % per) * MX3::kSteps;
  float v0[8], v1[8];                     // k-slots 0..7 and 8..15
  if (left) {
    const int64_t o = blk * kDT + x;
    const bool ok = o < a.out;
    const HDP_GLOBAL float* dBr = gptr(a.dB + seg * a.dstr + (ok ? o : 0) * a.r);
    const HDP_GLOBAL float* Br = gptr(a.B + seg * a.fstr + (ok ? o : 0) * a.r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in_r = ok && s0 + j < a.r;
      v0[j] = in_r ? dBr[s0 + j] : 0.f;
      v1[j] = in_r ? Br[s0 + j] : 0.f;
    }
  } else {
    const int64_t col = blk * kDT + x;
    const bool ok = col < a.in;
    const HDP_GLOBAL float* As = gptr(a.A + seg * a.fstr + (ok ? col : 0));
    const HDP_GLOBAL float* dAs = gptr(a.dA + seg * a.dstr + (ok ? col : 0));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool in_r = ok && s0 + j < a.r;
      const float ad = in_r ? dAs[(int64_t)(s0 + j) * a.in] : 0.f;
      const float av = in_r ? As[(int64_t)(s0 + j) * a.in] : 0.f;
      v0[j] = av - ad;
      v1[j] = ad;
    }
  }
  HDP_GLOBAL __bf16* panel = gptr((left ? a.limg : a.rimg) + pb * kPanel);
  bf16x8 p[3];
  MX3::split8(v0, p[0], p[1], p[2]);
#pragma unroll
  for (int q = 0; q < 3; ++q) *reinterpret_cast<HDP_GLOBAL bf16x8*>(panel + q * kDT * 16 + x * 16 + 8 * MX3::gran(x, 0)) = p[q];
  MX3::split8(v1, p[0], p[1], p[2]);
#pragma unroll
  for (int q = 0; q < 3; ++q) *reinterpret_cast<HDP_GLOBAL bf16x8*>(panel + q * kDT * 16 + x * 16 + 8 * MX3::gran(x, 1)) = p[q];
}

__device__ __forceinline__ void zero_tile(f32x16 (&x)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) x[i][j][e] = 0.f;
}

// end of a rank segment (bf16 rounding order): run = bf16(run - bracket_i), acc = 0
__device__ __forceinline__ void fold_segment(f32x16 (&run)[2][2], f32x16 (&acc)[2][2]) {
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

// ---- epilogue: register e of block (bo, bc) is row o_w + 32 bo + row_of(e, h), column
// c_w + 32 bc + l32; val = run (the tile's dW).  Full tiles: buffer stores through `t`;
// edge tiles: bounds-checked element access ----
template <int MODE, int DT, bool NEG, int POL = 0, class WPF>  // POL bit 0: non-temporal stores
__device__ __forceinline__ void epilogue(const DeltaArgs& a, const f32x16 (&run)[2][2], const WPF& wpf,
                                         const TileAddr& t, int64_t o_w, int64_t c_w, bool full, int l32, int h) {
  if (full) {
#pragma unroll
    for (int bo = 0; bo < 2; ++bo)
#pragma unroll
      for (int bc = 0; bc < 2; ++bc)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float val = NEG ? -run[bo][bc][e] : run[bo][bc][e];
          if constexpr (MODE == HDP_DW_STORE) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), t.rs, t.voff, reg_soff<4>(t, bo, bc, e),
                                                  w_store_aux(POL));
          } else if constexpr (DT == HDP_F32) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(wpf.w[bo][bc][e] + val), t.rs, t.voff,
                                                  reg_soff<4>(t, bo, bc, e), w_store_aux(POL));
          } else {
            const uint16_t nw = f32_to_bf16(bf16_to_f32(wpf.w[bo][bc][e]) + round_bf16(val));
            __builtin_amdgcn_raw_buffer_store_b16(nw, t.rs, t.voff, reg_soff<2>(t, bo, bc, e), 0);
          }
        }
    return;
  }
#pragma unroll
  for (int bo = 0; bo < 2; ++bo) {
#pragma unroll
    for (int bc = 0; bc < 2; ++bc) {
      const int64_t c = c_w + 32 * bc + l32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t o = o_w + 32 * bo + row_of(e, h);
        if (o >= a.out || c >= a.in) continue;
        const float val = NEG ? -run[bo][bc][e] : run[bo][bc][e];
        const int64_t idx = o * a.in + c;
        if constexpr (MODE == HDP_DW_STORE) {
          gptr(reinterpret_cast<float*>(a.dst))[idx] = val;
        } else if constexpr (DT == HDP_F32) {
          gptr(reinterpret_cast<float*>(a.dst))[idx] += val;
        } else {
          HDP_GLOBAL uint16_t* p = gptr(reinterpret_cast<uint16_t*>(a.dst)) + idx;
          *p = f32_to_bf16(bf16_to_f32(*p) + round_bf16(val));
        }
      }
    }
  }
}

// Local tile l of a module -> origin.  Tiles are numbered in 8-column bands (band-major, then
// row, then column inside the band), so any 64 consecutive tiles form an 8 x 8 block: the
// factor rows / columns they read (8 L blocks + 8 R blocks per chunk) stay in the XCD's L2
// while the block's workgroups run (see the XCD-contiguous schedule in delta_group_kernel).
// TR = the tile's row count (kDT, or 2 kDT for the wide x3 kernel); columns are always kDT.
template <int TR = kDT>
__device__ __forceinline__ void tile_origin(const DeltaArgs& a, int64_t l, int64_t& o_t, int64_t& c_t) {
  const int64_t nC = (a.in + kDT - 1) / kDT, nO = (a.out + TR - 1) / TR;
  const int64_t band = l / (8 * nO);
  const int64_t w = min((int64_t)8, nC - 8 * band);  // columns in this band
  const int64_t rem = l - band * 8 * nO;
  const int64_t row = rem / w;
  o_t = row * TR;
  c_t = (8 * band + (rem - row * w)) * kDT;
}

template <int MODE, int DT, bool ROUND, class M = MF32>
__global__ __launch_bounds__(256, 2) void delta_gemm_kernel(DeltaArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * M::kBuf];
  const int nC = (int)((a.in + kDT - 1) / kDT);
  const int nO = (int)((a.out + kDT - 1) / kDT);
  const int id = xcd_remap(blockIdx.x, nO * nC);  // XCD-contiguous ranges of banded tiles
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  int64_t o_t, c_t;
  tile_origin(a, id, o_t, c_t);
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;  // wave offsets inside the tile
  const int64_t o_w = o_t + ow, c_w = c_t + cw;
  const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
  constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
  const TileAddr taddr = tile_addr<ESZ>(a, o_w, c_w, l32, h);
  const int per = (a.r + M::kSteps - 1) / M::kSteps;
  const int nchunks = a.nseg * per;

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only: the bf16-rounded running dW
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;

  typename M::St st;
  M::load(a, 0, o_t, c_t, tid, st);
  M::store(smem, tid, st);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const float* buf = smem + (c & 1) * M::kBuf;
    if (c + 1 < nchunks) M::load(a, c + 1, o_t, c_t, tid, st);          // next chunk in flight
    if constexpr (MODE == HDP_DW_MERGE) {
      if (c + 1 == nchunks && full) wpf.load(taddr);                   // W tile in flight
    }
    M::mfma(buf, h, l32, ow, cw, acc);
    if (ROUND && (c + 1) % per == 0) fold_segment(run, acc);  // dW = bf16(dW - bracket_i)
    if (c + 1 < nchunks) {
      // the other buffer was last read in chunk c-1, before the previous barrier: free
      M::store(smem + ((c + 1) & 1) * M::kBuf, tid, st);
      __syncthreads();
    }
  }
  // the tile's dW: ROUND keeps the bf16 running sum in `run`; otherwise it is -acc
  HDP_MFMA_FENCE();
  if constexpr (ROUND) epilogue<MODE, DT, false>(a, run, wpf, taddr, o_w, c_w, full, l32, h);
  else epilogue<MODE, DT, true>(a, acc, wpf, taddr, o_w, c_w, full, l32, h);
}

// ---------------------------------------------------------------------------------------
// GROUPED persistent form (hdp_delta_plan_*): every module of a plan in ONE launch.
// The plan's tiles are numbered module after module (tile_start = prefix sums); workgroup
// b walks tiles b, b + G, b + 2G, ... (G = resident workgroups), and the chunk pipeline runs
// ACROSS tile boundaries: while the MFMAs of the current chunk run, the next chunk's factor
// operands (possibly of the next tile, possibly of the next module) are in flight, and on a
// tile's last chunk its W tile is loaded before the MFMAs.  The next factors are staged into
// LDS before the epilogue's W stores are issued, so the vmcnt-ordered queue never makes the
// staging wait for the stores.  No per-module launch boundary, no tile-count tail per module.
// ---------------------------------------------------------------------------------------
struct DeltaGroup {
  const DeltaArgs* items;
  const int64_t* tile_start;  // n + 1 prefix sums of the modules' tile counts
  int n;
  int64_t total;
};

template <class M>
__device__ __forceinline__ int chunks_of(const DeltaArgs& a) { return a.nseg * ((a.r + M::kSteps - 1) / M::kSteps); }

template <int MODE, int DT, bool ROUND, int POL = 0, class M = MF32>
__global__ __launch_bounds__(256, 2) void delta_group_kernel(const DeltaArgs* __restrict__ items,
                                                             const int64_t* __restrict__ tile_start, int n,
                                                             int64_t total) {
  // (separate __restrict__ parameters: the descriptor loads are provably unclobbered by the
  // kernel's W stores, so they become scalar loads into SGPRs)
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[2 * M::kBuf];
  // XCD-contiguous schedule: the G / 8 workgroups the dispatcher deals to one XCD (blockIdx
  // b, b + 8, ...) walk one contiguous eighth of the plan's tile space, G / 8 tiles apart, so
  // the tiles running at once on an XCD are neighbours (L2 reuse of their factor operands).
  // Speed only: any placement gives the same result.
  const int nx = gridDim.x >= 8 ? 8 : 1;
  const int x = blockIdx.x % nx;
  const int64_t stride = gridDim.x / nx;
  const int64_t t_end = (int64_t)(x + 1) * g.total / nx;
  int64_t t = (int64_t)x * g.total / nx + blockIdx.x / nx;
  if (t >= t_end || (nx == 8 && (int)(blockIdx.x / nx) >= (int)stride)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;

  int m = 0;
  {
    int lo = 0, hi = g.n - 1;  // largest m with tile_start[m] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (g.tile_start[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    m = lo;
  }
  DeltaArgs a = g.items[m];
  int64_t m_end = g.tile_start[m + 1];
  int64_t o_t, c_t;
  tile_origin(a, t - g.tile_start[m], o_t, c_t);
  int c = 0, nch = chunks_of<M>(a), per = (a.r + M::kSteps - 1) / M::kSteps;

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only: the bf16-rounded running dW
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;

  typename M::St st;
  M::load(a, 0, o_t, c_t, tid, st);
  M::store(smem, tid, st);
  __syncthreads();
  int buf = 0;
  for (;;) {
    // ---- the next (tile, chunk) of this workgroup ----
    const bool last = (c + 1 == nch);
    int64_t tn = t, on_t = o_t, cn_t = c_t, mn_end = m_end;
    int cn = c + 1, mn = m;
    DeltaArgs an = a;
    if (last) {
      tn = t + stride;
      cn = 0;
      if (tn < t_end) {
        if (tn >= m_end) {
          do {
            ++mn;
          } while (tn >= g.tile_start[mn + 1]);
          an = g.items[mn];
          mn_end = g.tile_start[mn + 1];
        }
        tile_origin(an, tn - g.tile_start[mn], on_t, cn_t);
      }
    }
    const bool has_next = tn < t_end;
    const int64_t o_w = o_t + ow, c_w = c_t + cw;
    const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
    constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
    const TileAddr taddr = tile_addr<ESZ>(a, o_w, c_w, l32, h);
    if (has_next) M::load(an, cn, on_t, cn_t, tid, st);                // next factors in flight
    if constexpr (MODE == HDP_DW_MERGE) {
      if (last && full) wpf.template load<POL>(taddr);                  // W tile in flight
    }
    M::mfma(smem + buf * M::kBuf, h, l32, ow, cw, acc);
    if (ROUND && (c + 1) % per == 0) fold_segment(run, acc);
    // the other buffer was last read before the previous barrier: free
    if (has_next) M::store(smem + (buf ^ 1) * M::kBuf, tid, st);
    if (last) {
      if constexpr (ROUND) {
        epilogue<MODE, DT, false, POL>(a, run, wpf, taddr, o_w, c_w, full, l32, h);
        zero_tile(run);
      } else {
        epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, full, l32, h);
      }
      zero_tile(acc);
    }
    if (!has_next) break;
    __syncthreads();
    buf ^= 1;
    t = tn;
    c = cn;
    if (mn != m) {
      m = mn;
      a = an;
      m_end = mn_end;
      nch = chunks_of<M>(a);
      per = (a.r + M::kSteps - 1) / M::kSteps;
    }
    o_t = on_t;
    c_t = cn_t;
  }
}

// ---------------------------------------------------------------------------------------
// X3P pipelined form (x3 plans): the MFMA phase of a bf16x3 chunk is 24 MFMAs (768 cycles),
// shorter than a factor-panel load's latency under load, so the packed panels are staged
// through a 3-slot REGISTER ring: at chunk i the workgroup computes on LDS buffer i & 1,
// stores chunk i + 1 (loaded two chunks ago) into the other buffer and issues the loads of
// chunk i + 3 into the slot chunk i vacated -- two chunk phases of latency cover per load.
// The W tile of a MERGE is read in the epilogue (not prefetched: the ring holds those
// registers); with K = 2 r Wn >= 128 a tile has >= 16 chunks, so that exposure is rare.
// ---------------------------------------------------------------------------------------
struct X3Cursor {
  int64_t t, t_end, stride, m_end;
  int m, c, nch;
  int64_t o_t, c_t;
  DeltaArgs a;
  bool valid;
};

template <int TR = kDT>
__device__ __forceinline__ void x3_cursor_tile(const DeltaGroup& g, X3Cursor& k) {
  if (k.t >= k.m_end) {
    do {
      ++k.m;
    } while (k.t >= g.tile_start[k.m + 1]);
    k.a = g.items[k.m];
    k.m_end = g.tile_start[k.m + 1];
    k.nch = chunks_of<MX3>(k.a);
  }
  tile_origin<TR>(k.a, k.t - g.tile_start[k.m], k.o_t, k.c_t);
}

template <int TR = kDT>
__device__ __forceinline__ void x3_advance(const DeltaGroup& g, X3Cursor& k) {
  if (!k.valid) return;
  if (++k.c < k.nch) return;
  k.c = 0;
  k.t += k.stride;
  if (k.t >= k.t_end) {
    k.valid = false;
    return;
  }
  x3_cursor_tile<TR>(g, k);
}

// panel pointers of the load cursor's chunk
__device__ __forceinline__ void x3_panels(const X3Cursor& k, const HDP_GLOBAL f32x4*& lp, const HDP_GLOBAL f32x4*& rp) {
  const int64_t nRB = (k.a.out + kDT - 1) / kDT, nCB = (k.a.in + kDT - 1) / kDT;
  lp = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(k.a.limg + ((int64_t)k.c * nRB + k.o_t / kDT) * kPanel));
  rp = reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(k.a.rimg + ((int64_t)k.c * nCB + k.c_t / kDT) * kPanel));
}

template <int MODE, int DT, bool ROUND, int POL>
__global__ __launch_bounds__(256, 2) void delta_x3p_kernel(const DeltaArgs* __restrict__ items,
                                                           const int64_t* __restrict__ tile_start, int n,
                                                           int64_t total) {
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[2 * MX3P::kBuf];
  const int nx = gridDim.x >= 8 ? 8 : 1;
  const int x = blockIdx.x % nx;
  X3Cursor L;
  L.stride = gridDim.x / nx;
  L.t_end = (int64_t)(x + 1) * g.total / nx;
  L.t = (int64_t)x * g.total / nx + blockIdx.x / nx;
  if (L.t >= L.t_end || (int64_t)(blockIdx.x / nx) >= L.stride) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  {
    int lo = 0, hi = g.n - 1;  // largest m with tile_start[m] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (g.tile_start[mid] <= L.t) lo = mid;
      else hi = mid - 1;
    }
    L.m = lo;
  }
  L.a = g.items[L.m];
  L.m_end = g.tile_start[L.m + 1];
  L.nch = chunks_of<MX3>(L.a);
  L.c = 0;
  L.valid = true;
  tile_origin(L.a, L.t - g.tile_start[L.m], L.o_t, L.c_t);
  X3Cursor C = L;  // compute cursor; L runs ahead as the load cursor

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  StageX3P ring[3];
  const HDP_GLOBAL f32x4 *lp, *rp;  // panels of the load cursor's chunk (the last valid one once L ran out)
  auto ring_load = [&](StageX3P& st) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      st.v[p] = lp[p * 256 + tid];
      st.v[3 + p] = rp[p * 256 + tid];
    }
  };
  x3_panels(L, lp, rp);
  ring_load(ring[0]);
  x3_advance(g, L);
  if (L.valid) x3_panels(L, lp, rp);
  ring_load(ring[1]);
  x3_advance(g, L);
  if (L.valid) x3_panels(L, lp, rp);
  ring_load(ring[2]);
  x3_advance(g, L);
  if (L.valid) x3_panels(L, lp, rp);
  MX3P::store(smem, tid, ring[0]);
  __syncthreads();

  // one chunk; S = the ring slot of chunk i (compile-time), buf = its LDS buffer.  The 24
  // MFMAs are interleaved (sched_group_barrier) with the 6 LDS stores of chunk i + 1 into the
  // other buffer and the 6 loads of chunk i + 3 into slot S.  Stores / loads past the end of
  // the workgroup's work are harmless repeats (never read).
  auto step = [&](auto S_, int buf) -> bool {
    constexpr int S = decltype(S_)::value;
    const __bf16* b = reinterpret_cast<const __bf16*>(smem + buf * MX3P::kBuf);
    bf16x8 fa[2][3], fb[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int xa = ow + 32 * i + l32, xb = cw + 32 * i + l32;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        fa[i][p] = *reinterpret_cast<const bf16x8*>(b + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
        fb[i][p] = *reinterpret_cast<const bf16x8*>(b + (3 + p) * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));
      }
    }
    f32x4* nb = reinterpret_cast<f32x4*>(smem + (buf ^ 1) * MX3P::kBuf);
    const StageX3P& nx_st = ring[(S + 1) % 3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int bo = q >> 1, bc = q & 1;
      f32x16 d = acc[bo][bc];
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][2], fb[bc][0], d, 0, 0, 0);  // lo * hi
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][1], d, 0, 0, 0);  // mid * mid
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][2], d, 0, 0, 0);  // hi * lo
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][0], d, 0, 0, 0);  // mid * hi
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][1], d, 0, 0, 0);  // hi * mid
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][0], d, 0, 0, 0);  // hi * hi
      acc[bo][bc] = d;
    }
#pragma unroll
    for (int p = 0; p < 6; ++p) nb[p * 256 + tid] = nx_st.v[p];
    ring_load(ring[S]);
    // schedule: the 12 fragment reads first, then per 4 MFMAs one LDS store and one load
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    const int per = (C.a.r + MX3::kSteps - 1) / MX3::kSteps;
    if (ROUND && (C.c + 1) % per == 0) fold_segment(run, acc);
    const bool last = C.c + 1 == C.nch;
    const bool has_next = !last || C.t + C.stride < C.t_end;
    x3_advance(g, L);
    if (L.valid) x3_panels(L, lp, rp);
    if (last) {
      const int64_t o_w = C.o_t + ow, c_w = C.c_t + cw;
      const bool full = (o_w + 64 <= C.a.out) && (c_w + 64 <= C.a.in);
      constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
      const TileAddr taddr = tile_addr<ESZ>(C.a, o_w, c_w, l32, h);
      WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;
      if constexpr (MODE == HDP_DW_MERGE) {
        if (full) wpf.template load<POL>(taddr);
      }
      if constexpr (ROUND) {
        epilogue<MODE, DT, false, POL>(C.a, run, wpf, taddr, o_w, c_w, full, l32, h);
        zero_tile(run);
      } else {
        epilogue<MODE, DT, true, POL>(C.a, acc, wpf, taddr, o_w, c_w, full, l32, h);
      }
      zero_tile(acc);
    }
    if (!has_next) return false;
    __syncthreads();
    x3_advance(g, C);
    return true;
  };
  for (;;) {
    if (!step(std::integral_constant<int, 0>(), 0)) break;
    if (!step(std::integral_constant<int, 1>(), 1)) break;
    if (!step(std::integral_constant<int, 2>(), 0)) break;
    if (!step(std::integral_constant<int, 0>(), 1)) break;
    if (!step(std::integral_constant<int, 1>(), 0)) break;
    if (!step(std::integral_constant<int, 2>(), 1)) break;
  }
}

// ---------------------------------------------------------------------------------------
// X3G: the x3 plan kernel with the packed panels staged by LDS-DMA (global_load_lds_dwordx4)
// into a 3-buffer LDS ring.  In the register-ring form hipcc's wait-count pass merged the
// loop's paths (epilogue / no epilogue) into an `s_waitcnt vmcnt(0)` at every chunk: each
// chunk waited for the loads issued one chunk earlier, so the ring hid nothing (34 % MFMA
// busy).  Here the loads have no VGPR destination and the waits are written by hand:
//   chunk i: fragments of buffer i % 3 -> 24 MFMAs -> [tile end: W RMW] -> wait for THIS
//   wave's pieces of chunk i + 1 (s_waitcnt vmcnt(6) leaves chunk i + 2 in flight) -> raw
//   s_barrier (every wave's pieces landed; every wave done reading buffer i % 3) -> issue
//   chunk i + 3 into buffer i % 3 (six 1-KB pieces per wave: the panels are stored in the
//   exact lane-linear LDS image).
// A tile end's W loads are ordinary loads: their first use makes hipcc wait vmcnt(0), which
// also retires the chunks in flight -- so the wait after a MERGE epilogue (and after the one
// before) is skipped; after a STORE epilogue the stores sit in the counter, so it drains.
// ---------------------------------------------------------------------------------------
template <int MODE, int DT, bool ROUND, int POL>
__global__ __launch_bounds__(256, 2) void delta_x3g_kernel(const DeltaArgs* __restrict__ items,
                                                           const int64_t* __restrict__ tile_start, int n,
                                                           int64_t total) {
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[3 * MX3P::kBuf];
  const int nx = gridDim.x >= 8 ? 8 : 1;
  const int x = blockIdx.x % nx;
  X3Cursor L;
  L.stride = gridDim.x / nx;
  L.t_end = (int64_t)(x + 1) * g.total / nx;
  L.t = (int64_t)x * g.total / nx + blockIdx.x / nx;
  if (L.t >= L.t_end || (int64_t)(blockIdx.x / nx) >= L.stride) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  {
    int lo = 0, hi = g.n - 1;  // largest m with tile_start[m] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (g.tile_start[mid] <= L.t) lo = mid;
      else hi = mid - 1;
    }
    L.m = lo;
  }
  L.a = g.items[L.m];
  L.m_end = g.tile_start[L.m + 1];
  L.nch = chunks_of<MX3>(L.a);
  L.c = 0;
  L.valid = true;
  tile_origin(L.a, L.t - g.tile_start[L.m], L.o_t, L.c_t);
  X3Cursor C = L;

  // wave w moves pieces 6w .. 6w + 5 of a chunk's 24 (L panel = pieces 0-11, R panel = 12-23)
  auto issue = [&](int buf) {
    const HDP_GLOBAL f32x4 *lp, *rp;
    x3_panels(L, lp, rp);
    const HDP_GLOBAL f32x4* src = wave < 2 ? lp + (wave * 6) * 64 : rp + ((wave - 2) * 6) * 64;
    float* dst = smem + buf * MX3P::kBuf + wave * 6 * 256;
#pragma unroll
    for (int p = 0; p < 6; ++p)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const HDP_GLOBAL void*>(src + p * 64 + lane),
                                       (__attribute__((address_space(3))) void*)(dst + p * 256), 16, 0, 0);
  };
  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  // prologue: chunks 0, 1, 2 in flight; wait for chunk 0
  int nissued = 0;  // chunks issued so far (the load cursor L points at chunk nissued)
  for (int b = 0; b < 3 && L.valid; ++b) {
    issue(b);
    ++nissued;
    x3_advance(g, L);
  }
  if (nissued == 3) __builtin_amdgcn_s_waitcnt(0x0F70 | 12);       // vmcnt(12)
  else if (nissued == 2) __builtin_amdgcn_s_waitcnt(0x0F70 | 6);   // vmcnt(6)
  else __builtin_amdgcn_s_waitcnt(0x0F70);                          // vmcnt(0)
  __builtin_amdgcn_s_barrier();

  int i = 0;          // chunk index of this workgroup's sequence
  bool prev_epi = false;
  for (;;) {
    const int buf = i % 3;
    MX3::mfma(smem + buf * MX3P::kBuf, h, l32, ow, cw, acc);
    const int per = (C.a.r + MX3::kSteps - 1) / MX3::kSteps;
    if (ROUND && (C.c + 1) % per == 0) fold_segment(run, acc);
    const bool last = C.c + 1 == C.nch;
    const bool has_next = !last || C.t + C.stride < C.t_end;
    if (last) {
      const int64_t o_w = C.o_t + ow, c_w = C.c_t + cw;
      const bool full = (o_w + 64 <= C.a.out) && (c_w + 64 <= C.a.in);
      constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
      const TileAddr taddr = tile_addr<ESZ>(C.a, o_w, c_w, l32, h);
      WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;
      if constexpr (MODE == HDP_DW_MERGE) {
        if (full) wpf.template load<POL>(taddr);
      }
      if constexpr (ROUND) {
        epilogue<MODE, DT, false, POL>(C.a, run, wpf, taddr, o_w, c_w, full, l32, h);
        zero_tile(run);
      } else {
        epilogue<MODE, DT, true, POL>(C.a, acc, wpf, taddr, o_w, c_w, full, l32, h);
      }
      zero_tile(acc);
    }
    if (!has_next) break;
    // chunk i + 1 must have landed (this wave's pieces); chunk i + 2 may stay in flight
    const bool next2 = nissued >= i + 3;  // chunk i + 2 was issued
    const bool drained = MODE == HDP_DW_MERGE && (last || prev_epi);
    if (!drained) {
      if (MODE == HDP_DW_STORE && (last || prev_epi)) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      else if (next2) __builtin_amdgcn_s_waitcnt(0x0F70 | 6);                            // vmcnt(6)
      else __builtin_amdgcn_s_waitcnt(0x0F70);                                            // vmcnt(0)
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();
    if (L.valid) {
      issue(buf);  // chunk i + 3 into the buffer chunk i vacated
      ++nissued;
      x3_advance(g, L);
    }
    prev_epi = last;
    x3_advance(g, C);
    ++i;
  }
}

// ---------------------------------------------------------------------------------------
// X3W: the wide form of X3G (the default for x3 plans).  A workgroup of 8 waves owns a
// 256-row x 128-column tile (wave w computes rows 64 (w >> 1), columns 64 (w & 1)), so a chunk
// stages two L panels and one R panel (36 KB) for 32 K outputs: 1.1 B of panel traffic per
// output and chunk instead of X3G's 1.5 B.  One workgroup per CU with a 4-buffer LDS ring
// (144 KB; three chunks in flight).
// X3G's SQ counters (tools/pmc_delta.sh) showed what held it at 34 % MFMA busy: ~200 SALU /
// VALU instructions per wave and chunk beside 24 MFMAs -- panel addresses recomputed from the
// module descriptor every chunk, two cursors' worth of descriptor state spilled to VGPR lanes,
// data-dependent wait counts.  Here each wave keeps ONE source pointer: waves 0-2 move 4 pieces
// (1 KB each) of the first L panel, waves 3-5 4 of the second, waves 6-7 6 of the R panel, and
// a chunk advance is one 64-bit add (pointer += panel stride).  Every iteration issues exactly
// one chunk (past the end of the workgroup's work it repeats the last one into the buffer just
// vacated, never read), so the wait before the barrier is a constant vmcnt(2 pieces-per-chunk).
// Descriptor fields are read from the item table (scalar loads) only when a cursor changes
// tile.  A tile end drains the counter (vmcnt(0)) before its epilogue, which covers the next
// chunk's wait too; the W tile of a float32 MERGE is prefetched at the top of the last chunk.
// ---------------------------------------------------------------------------------------
constexpr int kWideBuf = 9 * kDT * 16 / 2;  // floats per buffer: L panels 2 x [3][128][16] + R [3][128][16] bf16
constexpr int kWideNB = 4;                  // LDS ring depth (chunks)


__device__ __forceinline__ void x3_frags(const __bf16* Lb, const __bf16* Rb, int h, int l32, int ow, int cw,
                                         bf16x8 (&fa)[2][3], bf16x8 (&fb)[2][3]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int xa = ow + 32 * i + l32, xb = cw + 32 * i + l32;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      fa[i][p] = *reinterpret_cast<const bf16x8*>(Lb + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
      fb[i][p] = *reinterpret_cast<const bf16x8*>(Rb + p * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));
    }
  }
}
__device__ __forceinline__ void x3_mfma_regs(const bf16x8 (&fa)[2][3], const bf16x8 (&fb)[2][3], f32x16 (&acc)[2][2]);
__device__ __forceinline__ void x3_mfma(const __bf16* Lb, const __bf16* Rb, int h, int l32, int ow, int cw,
                                        f32x16 (&acc)[2][2]) {
  bf16x8 fa[2][3], fb[2][3];
  x3_frags(Lb, Rb, h, l32, ow, cw, fa, fb);
  x3_mfma_regs(fa, fb, acc);
}
__device__ __forceinline__ void x3_mfma_regs(const bf16x8 (&fa)[2][3], const bf16x8 (&fb)[2][3], f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int bo = 0; bo < 2; ++bo)
#pragma unroll
    for (int bc = 0; bc < 2; ++bc) {
      f32x16 d = acc[bo][bc];
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][2], fb[bc][0], d, 0, 0, 0);  // lo * hi
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][1], d, 0, 0, 0);  // mid * mid
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][2], d, 0, 0, 0);  // hi * lo
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][1], fb[bc][0], d, 0, 0, 0);  // mid * hi
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][1], d, 0, 0, 0);  // hi * mid
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[bo][0], fb[bc][0], d, 0, 0, 0);  // hi * hi
      acc[bo][bc] = d;
    }
}

// module of tile t at or after module m (cursors only move forward)
__device__ __forceinline__ int x3w_module(const int64_t* __restrict__ ts, int m, int64_t t) {
  while (t >= ts[m + 1]) ++m;
  return m;
}
// tile_origin<2 kDT> in 32-bit arithmetic (make_args bounds out * in < 2^31)
#ifndef HDP_K4_BAND
#define HDP_K4_BAND 8
#endif
__device__ __forceinline__ void x3w_origin(int out, int in, int l, int& o_t, int& c_t) {
  constexpr int BW = HDP_K4_BAND;  // column blocks per band
  const int nC = (in + kDT - 1) / kDT, nO = (out + 2 * kDT - 1) / (2 * kDT);
  const int band = l / (BW * nO);
  const int w = min(BW, nC - BW * band);
  const int rem = l - band * BW * nO;
  const int row = rem / w;
  o_t = row * 2 * kDT;
  c_t = (BW * band + (rem - row * w)) * kDT;
}

struct X3WLoad {
  const char* src;  // this wave's first piece of the current chunk
  int64_t step;     // bytes between consecutive chunks of that panel
  int64_t t;        // tile
  int m, c, nch;
  bool live;
};

__device__ __forceinline__ void x3w_load_tile(const DeltaGroup& g, X3WLoad& L, int wave) {
  L.m = x3w_module(g.tile_start, L.m, L.t);
  const DeltaArgs& a = g.items[L.m];
  const int out = (int)a.out, in = (int)a.in;
  int o_t, c_t;
  x3w_origin(out, in, (int)(L.t - g.tile_start[L.m]), o_t, c_t);
  const int nRB = (out + kDT - 1) / kDT, nCB = (in + kDT - 1) / kDT;
  L.c = 0;
  L.nch = chunks_of<MX3>(a);
  if (wave < 6) {  // rows past the module's last 128 re-read the first panel (never stored)
    const int rb0 = o_t / kDT, rb = wave < 3 ? rb0 : min(rb0 + 1, nRB - 1);
    L.src = reinterpret_cast<const char*>(a.limg + (int64_t)rb * kPanel) + (wave % 3) * 4096;
    L.step = (int64_t)nRB * kPanel * 2;
  } else {
    L.src = reinterpret_cast<const char*>(a.rimg + (int64_t)(c_t / kDT) * kPanel) + (wave - 6) * 6144;
    L.step = (int64_t)nCB * kPanel * 2;
  }
}

// ---- deferred W merge (DEF != 0; float32 MERGE): the epilogue of a full tile is not done at the
// tile end, where a wave would wait for its 16 KB of W behind one chunk of MFMAs (the CU's W
// read-modify-write, 256 KB per tile, takes ~8 us at its share of HBM bandwidth against ~10 us of
// MFMAs per tile).  The finished accumulators move to `pend` and the next tile's first chunks
// carry the W traffic: chunk k loads group k of the pending tile's W (8 PPC registers), chunk
// k + D adds and stores it.  The 64 W registers of the immediate form are replaced by
// (D + 1) x 8 PPC; the pending accumulators take the 64 the W prefetch held.
// Groups of PPC pieces; piece p = block (p >> 2, (p >> 1) & 1), registers 8 (p & 1) .. + 7.
template <int DEF> struct X3WDefer {
  // DEF 4 (H2 only): two pieces per chunk with two chunks between loads and stores (the W loads of a
  // Wn = 8 tile get two chunks of MFMAs to land instead of one; 16 more registers)
  static constexpr int PPC = DEF == 1 ? 1 : 2;  // pieces per chunk
  static constexpr int D = DEF == 2 ? 1 : 2;    // chunks between a group's loads and its stores
  static constexpr int G = 8 / PPC;             // groups per tile
  // W ops (loads + stores) issued in iteration j of a tile that has a pending predecessor
  static constexpr int wops(int j) { return j < 0 ? 0 : 8 * PPC * ((j < G ? 1 : 0) + (j >= D && j - D < G ? 1 : 0)); }
  static constexpr int span = G + D;            // iterations with W ops
  static constexpr int lops(int j) { return j >= 0 && j < G ? 8 * PPC : 0; }
  static constexpr int sops(int j) { return j >= D && j - D < G ? 8 * PPC : 0; }
  // vector-memory ops issued after group J's loads when iteration J + D stores it: iteration
  // order is loads, MFMAs, stores, ring wait, barrier, ring issue (rn ops)
  static constexpr int after_load(int J, int rn) {
    int c = sops(J) + rn;
    for (int j = J + 1; j < J + D; ++j) c += lops(j) + sops(j) + rn;
    return c + lops(J + D);
  }
  // the pending merge must finish inside the next tile's loop (iterations 0 .. nch - 2) before
  // that tile's own accumulators move to `pend`
  static constexpr int min_chunks = span + 1;
};
template <int DEF> int x3w_defer_min_chunks() { return X3WDefer<DEF>::min_chunks; }

// the row offsets are recomputed per access from scalars made opaque here: hoisted out of
// the tile loop they would take 64 SGPRs (the kernel has none to spare)
__device__ __forceinline__ TileAddr opaque_rows(TileAddr t) {
  asm volatile("" : "+s"(t.sbase), "+s"(t.rowb));
  return t;
}
typedef int i32x4 __attribute__((ext_vector_type(4)));
// Every inline-asm VMEM instruction below starts with s_nop 4: its SGPR operands (descriptor, soffset) may be
// re-materialised by v_readlane from the SGPR spill lanes right in front of the asm, and a VALU write of an SGPR
// needs 5 wait states before a VMEM instruction reads it -- the compiler pads that hazard for its own instructions,
// not inside inline asm (r06: with a different register allocation a spill reload one instruction before the first
// deferred bf16 W store made it store through a stale descriptor; tests/isa_scan.py::valu_sgpr_vmem_hazards scans
// the shipped code object for it).
// Pending-tile W loads in inline asm: the compiler's wait-count model would otherwise put a
// vmcnt(0) in front of every use (a load issued two iterations back, LDS-DMA in between),
// draining the LDS ring.  These loads are invisible to it; their consumer waits explicitly
// (wgroup_store) with the count of vector-memory ops issued after them.  rs4 = the dword form of
// the buffer descriptor (__builtin_amdgcn_make_buffer_rsrc's layout).
template <int P0, int N, int POL>
__device__ __forceinline__ void wgroup_load_asm(i32x4 rs4, TileAddr t, float (&w)[8 * N]) {
  t = opaque_rows(t);
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const int p = P0 + q, bo = p >> 2, bc = (p >> 1) & 1, e0 = 8 * (p & 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int so = reg_soff<4>(t, bo, bc, e0 + e);
      if constexpr (POL & 2)
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, %3 offen nt" : "=v"(w[8 * q + e]) : "v"(t.voff), "s"(rs4), "s"(so) : "memory");
      else
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, %3 offen" : "=v"(w[8 * q + e]) : "v"(t.voff), "s"(rs4), "s"(so) : "memory");
    }
  }
}
// the compiler-tracked form (the workgroup's final flush)
template <int P0, int N, int POL>
__device__ __forceinline__ void wgroup_load(TileAddr t, float (&w)[8 * N]) {
  t = opaque_rows(t);
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const int p = P0 + q, bo = p >> 2, bc = (p >> 1) & 1, e0 = 8 * (p & 1);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      w[8 * q + e] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(t.rs, t.voff, reg_soff<4>(t, bo, bc, e0 + e), w_load_aux(POL)));
  }
}
// wait until at most NV vector-memory ops are outstanding, then hand the registers on (the
// empty asms order every later use after the wait)
template <int NV, int M>
__device__ __forceinline__ void wait_regs(float (&w)[M]) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV > 63 ? 63 : NV) : "memory");  // fewer is stricter: safe
#pragma unroll
  for (int i = 0; i < M; ++i) asm volatile("" : "+v"(w[i]));
}
template <int P0, int N, int POL>
__device__ __forceinline__ void wgroup_store(TileAddr t, const f32x16 (&pend)[2][2], const float (&w)[8 * N]) {
  t = opaque_rows(t);
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const int p = P0 + q, bo = p >> 2, bc = (p >> 1) & 1, e0 = 8 * (p & 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float val = -pend[bo][bc][e0 + e];  // the immediate epilogue's NEG merge, same expression
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w[8 * q + e] + val), t.rs, t.voff,
                                            reg_soff<4>(t, bo, bc, e0 + e), w_store_aux(POL));
    }
  }
}
// call f(integral_constant<K>) for the runtime k in [K, KMAX) (wave-uniform branches)
template <int K, int KMAX, class F>
__device__ __forceinline__ void static_case(int k, F&& f) {
  if constexpr (K < KMAX) {
    if (k == K) f(std::integral_constant<int, K>{});
    else static_case<K + 1, KMAX>(k, f);
  }
}

template <class F, int... Ks>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Ks...>) {
  (f(std::integral_constant<int, Ks>{}), ...);
}
// f(integral_constant<0>) .. f(integral_constant<N - 1>), in order, unrolled
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int MODE, int DT, bool ROUND, int POL, int DEF = 0>
__global__ __launch_bounds__(512, 1) void delta_x3w_kernel(const DeltaArgs* __restrict__ items,
                                                           const int64_t* __restrict__ tile_start, int n,
                                                           int64_t total) {
  constexpr int NB = kWideNB;
  constexpr bool kDefer = DEF != 0 && MODE == HDP_DW_MERGE && DT == HDP_F32 && !ROUND;
  using DF = X3WDefer<DEF>;
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[NB * kWideBuf];
  const int nx = gridDim.x >= 8 ? 8 : 1;
  const int x = blockIdx.x % nx;
  const int64_t stride = gridDim.x / nx;
  const int64_t t_end = (int64_t)(x + 1) * g.total / nx;
  const int64_t t0 = (int64_t)x * g.total / nx + blockIdx.x / nx;
  if (t0 >= t_end || (int64_t)(blockIdx.x / nx) >= stride) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  int m0 = 0;
  {
    int lo = 0, hi = g.n - 1;  // largest m with tile_start[m] <= t0
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (g.tile_start[mid] <= t0) lo = mid;
      else hi = mid - 1;
    }
    m0 = lo;
  }
  X3WLoad L;
  L.t = t0;
  L.m = m0;
  L.live = true;
  x3w_load_tile(g, L, wave);

  auto issue = [&](int buf) {
    float* dst = smem + buf * kWideBuf;
    if (wave < 6) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const HDP_GLOBAL void*>(gptr(L.src + j * 1024 + lane * 16)),
                                         (__attribute__((address_space(3))) void*)(dst + (wave * 4 + j) * 256), 16,
                                         0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const HDP_GLOBAL void*>(gptr(L.src + j * 1024 + lane * 16)),
                                         (__attribute__((address_space(3))) void*)(dst + (24 + (wave - 6) * 6 + j) * 256),
                                         16, 0, 0);
    }
  };
  auto advance = [&]() {
    if (!L.live) return;
    if (++L.c < L.nch) {
      L.src += L.step;
      return;
    }
    L.t += stride;
    if (L.t >= t_end) {
      L.live = false;  // src stays on the last chunk: later issues repeat it
      return;
    }
    x3w_load_tile(g, L, wave);
  };

  // compute cursor
  int64_t ct = t0;
  int cm = m0, cnch = 0, cper = 1, cfold = 1, o_t = 0, c_t = 0;
  auto compute_tile = [&]() {
    cm = x3w_module(g.tile_start, cm, ct);
    const DeltaArgs& a = g.items[cm];
    cnch = chunks_of<MX3>(a);
    cper = (a.r + MX3::kSteps - 1) / MX3::kSteps;
    cfold = cper;
    x3w_origin((int)a.out, (int)a.in, (int)(ct - g.tile_start[cm]), o_t, c_t);
  };
  compute_tile();

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    issue(b);
    advance();
  }
  // chunks 0 and 1 landed: the first iteration's wait covers chunk 1 only after a tile-end drain
  if (wave < 6) __builtin_amdgcn_s_waitcnt(vmcnt_imm(4 * (NB - 2)));
  else __builtin_amdgcn_s_waitcnt(vmcnt_imm(6 * (NB - 2)));
  __builtin_amdgcn_s_barrier();

  constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
  constexpr bool kPrefetchW = MODE == HDP_DW_MERGE && DT == HDP_F32 && !ROUND && !kDefer;
  // deferred merge state (kDefer)
  f32x16 pend[2][2];
  float wb[DF::D + 1][8 * DF::PPC];
  // the pending tile's address, kept as wave-uniform scalars (readfirstlane): a buffer
  // descriptor carried around the tile loop is otherwise taken for divergent and every W
  // access becomes a waterfall loop
  int pd_lo = 0, pd_hi = 0, pd_n = 0, pd_sbase = 0, pd_rowb = 0, pd_voff = 0;
  bool pp = false;  // a full tile's merge is pending (wave-uniform)
  auto pend_rs4 = [&]() {
    i32x4 r;
    r[0] = pd_lo;
    r[1] = pd_hi & 0xffff;
    r[2] = pd_n;
    r[3] = 0x00020000;
    return r;
  };
  auto pend_addr = [&]() {
    TileAddr t;
    const uint64_t ptr = ((uint64_t)(uint32_t)pd_hi << 32) | (uint32_t)pd_lo;
    t.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), 0, pd_n, 0x00020000);
    t.voff = pd_voff;
    t.sbase = pd_sbase;
    t.rowb = pd_rowb;
    return t;
  };
  // chunk i + 1 landed: every vector-memory op issued after its LDS-DMA pieces may stay in
  // flight -- two chunks' pieces and, in the first iterations of a tile with a pending merge,
  // the W ops of iterations k - 2 .. k (counts in issue order; vmcnt is in order on gfx9).
  // Ops not counted only make a wait stricter.
  auto plain_wait = [&]() {
    if (wave < 6) __builtin_amdgcn_s_waitcnt(vmcnt_imm(4 * (NB - 2)));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(6 * (NB - 2)));
  };
  int i = 0;
  auto mfma_chunk = [&]() {
    const __bf16* b = reinterpret_cast<const __bf16*>(smem + (i & (NB - 1)) * kWideBuf);
    x3_mfma(b + (ow >> 7) * 3 * kDT * 16, b + 6 * kDT * 16, h, l32, ow & (kDT - 1), cw, acc);
    if constexpr (ROUND) {
      if (--cfold == 0) {
        fold_segment(run, acc);
        cfold = cper;
      }
    }
  };
  // end of chunk i: every wave done with buffer i % NB -> chunk i + NB into it
  auto next_chunk = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();
    issue(i & (NB - 1));
    advance();
    ++i;
  };
  // Tiles, each: chunks 0 .. nch - 2 in the inner loop (no tile-end state: the accumulators
  // keep their registers across iterations), the last chunk peeled with the W prefetch and the
  // epilogue.  Chunk i + 1 must have landed before the barrier ending chunk i (this wave's
  // pieces; i + 2 .. i + NB - 1 stay in flight) -- except after a tile end, whose drain covered
  // the first chunk of the next tile.
  for (;;) {
    int k = 0;
    if constexpr (kDefer) {
      if (pp) {
        // the predecessor's merge rides on iterations 0 .. span - 1, unrolled so that every
        // W register has a fixed home (cnch >= span + 1: X3WDefer::min_chunks).  The loads
        // of group K wait at iteration K + D behind ring chunks the ring wait needs anyway.
        static_for<DF::span>([&](auto kc) {
          constexpr int K = decltype(kc)::value;
          if constexpr (K < DF::G)
            wgroup_load_asm<K * DF::PPC, DF::PPC, POL>(pend_rs4(), pend_addr(), wb[K % (DF::D + 1)]);
          mfma_chunk();
          if constexpr (K >= DF::D) {
            constexpr int J = K - DF::D;
            if (wave < 6) wait_regs<DF::after_load(J, 4)>(wb[J % (DF::D + 1)]);
            else wait_regs<DF::after_load(J, 6)>(wb[J % (DF::D + 1)]);
            wgroup_store<J * DF::PPC, DF::PPC, POL>(pend_addr(), pend, wb[J % (DF::D + 1)]);
          }
          constexpr int w = DF::wops(K - 2) + DF::wops(K - 1) + DF::wops(K);
          if (wave < 6) __builtin_amdgcn_s_waitcnt(vmcnt_imm(w + 4 * (NB - 2) > 63 ? 63 : w + 4 * (NB - 2)));
          else __builtin_amdgcn_s_waitcnt(vmcnt_imm(w + 6 * (NB - 2) > 63 ? 63 : w + 6 * (NB - 2)));
          next_chunk();
        });
        k = DF::span;
      }
    }
    for (; k + 1 < cnch; ++k) {
      mfma_chunk();
      if (kDefer || k != 0) plain_wait();  // (a tile end without kDefer drained the counter)
      next_chunk();
    }
    {
      const DeltaArgs& a = g.items[cm];
      const int64_t o_w = o_t + ow, c_w = c_t + cw;
      const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
      const TileAddr taddr = tile_addr<ESZ>(a, o_w, c_w, l32, h);
      WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;
      if constexpr (kPrefetchW) {
        if (full) wpf.template load<POL>(taddr);  // covered by the last chunk's MFMAs
      }
      mfma_chunk();
      if constexpr (kDefer) {
        // the predecessor's merge finished by iteration span - 1 <= cnch - 2 (min_chunks)
        pp = full;
        if (full) {
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) pend[x][y] = acc[x][y];
          const uint64_t dptr = reinterpret_cast<uint64_t>(a.dst);
          pd_lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)dptr);
          pd_hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(dptr >> 32));
          pd_n = __builtin_amdgcn_readfirstlane((int)(a.out * a.in * ESZ));
          pd_sbase = __builtin_amdgcn_readfirstlane(taddr.sbase);
          pd_rowb = __builtin_amdgcn_readfirstlane(taddr.rowb);
          pd_voff = taddr.voff;
          plain_wait();  // counts no W ops: at most conservative
        } else {
          __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
          epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, false, l32, h);  // edge: element-wise
        }
      } else {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // W and every chunk in flight have landed
        if constexpr (!kPrefetchW && MODE == HDP_DW_MERGE) {
          if (full) wpf.template load<POL>(taddr);
        }
        if constexpr (ROUND) {
          epilogue<MODE, DT, false, POL>(a, run, wpf, taddr, o_w, c_w, full, l32, h);
          zero_tile(run);
        } else {
          epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, full, l32, h);
        }
      }
      zero_tile(acc);
    }
    ct += stride;
    if (ct >= t_end) break;
    compute_tile();
    next_chunk();
  }
  if constexpr (kDefer) {
    if (pp) {  // the workgroup's last tile
      float w[64];
      const TileAddr t = pend_addr();
      wgroup_load<0, 8, POL>(t, w);
      wgroup_store<0, 8, POL>(t, pend, w);
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // no LDS-DMA outstanding when the workgroup retires
}

// ---------------------------------------------------------------------------------------
// H2: fp16x2 split with per-k power-of-two scaling (plans: HDP_MATH_H2, and AUTO for float32
// MERGE / STORE plans whose K = 2 r nseg > 32).  Each product L[o][k] R[k][c] is formed as
// (sl_k L[o][k]) (sr_k R[k][c]) 2^-E with sl_k sr_k = 2^E for every k of the item: sl_k brings
// column k of L into (2^13, 2^14], E is the largest exponent that keeps every scaled row of R
// within 2^14.  The scaled operands split into fp16 hi + lo (22 significand bits; no
// overflow, and underflow only below 2^-24 of the largest operand of its k), and
// v_mfma_f32_32x32x16_f16 sums lo*hi + hi*lo + hi*hi in f32: 3 MFMAs per 16 k where bf16x3
// needs 6.  The dropped lo*lo term and the split residual are ~2^-22 relative, below the f32
// chain's own rounding (test_gpu_kernels: error vs fp64 against the f32 MFMA chain's).
// Every run rebuilds the scales from the live factors (k4_h2_scale_kernel: maxima per 256
// rows / columns; k4_h2_fin_kernel: per item sl, sr, E), k4_h2_pack_kernel writes the
// panels, and delta_h2_kernel runs the wide schedule on them with K = 32 per chunk.
// ---------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kPanelH = 2 * kDT * 16;  // fp16 elements per H2 panel: [2 parts][128][16 k]
// per-item table (floats): [0] = 2^-E, [4 ..) sl[K], then sr[K], then the scale pass's
// partial maxima: L [seg][ceil(out / 256)][2r], R [seg][ceil(in / 256)][2r]; with
// k = (2 seg + half) r + step (half 0: dB | A - dA, half 1: B | dA)
static inline int64_t h2_tab_floats(int64_t out, int64_t in, int r, int nseg) {
  const int64_t K = 2ll * r * nseg;
  return 4 + 2 * K + (int64_t)nseg * ((out + 255) / 256 + (in + 255) / 256) * 2 * r + 2 * r;
}
// the fused Adam + pack path (single-segment plans): constant maxima max_o |B[o][k]| (r floats), then
// max_c |A[k][c]| (r floats), behind the scale pass's partials
__host__ __device__ inline int64_t h2_cmax_off(int64_t out, int64_t in, int r, int nseg) {
  return 4 + 4ll * r * nseg + (int64_t)nseg * ((out + 255) / 256 + (in + 255) / 256) * 2 * r;
}

// partial maxima of |L| per column and |R| per row: one workgroup per (item, segment, side,
// 256 rows of L or 256 columns of R), one row / column per thread
// gate (the fused path's fallback): run only when the word is set; null = always
__device__ __forceinline__ bool h2_gated_off(const int* gate) {
  return gate != nullptr && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

__global__ __launch_bounds__(256) void k4_h2_scale_kernel(const DeltaArgs* __restrict__ items,
                                                          const int* __restrict__ sstart, int n,
                                                          const int* gate) {
  if (h2_gated_off(gate)) return;
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;  // largest m with sstart[m] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (sstart[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const DeltaArgs& a = items[lo];
  const int r = a.r, K = 2 * r * a.nseg;
  const int nbL = (int)((a.out + 255) / 256), nbR = (int)((a.in + 255) / 256);
  int local = b - sstart[lo];
  const int seg = local / (nbL + nbR);
  local -= seg * (nbL + nbR);
  const bool left = local < nbL;
  const int blk = left ? local : local - nbL;
  float* part = a.ktab + 4 + 2 * K +
                (left ? ((int64_t)seg * nbL + blk) * 2 * r
                      : (int64_t)a.nseg * nbL * 2 * r + ((int64_t)seg * nbR + blk) * 2 * r);  // [half][r]
  __shared__ float red[4][16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t x = (int64_t)blk * 256 + tid;
  const bool ok = x < (left ? a.out : a.in);
  for (int s0 = 0; s0 < r; s0 += 8) {
    float mx[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) mx[j] = 0.f;
    if (ok) {
      if (left) {
        const HDP_GLOBAL float* dBr = gptr(a.dB + seg * a.dstr + x * r + s0);
        const HDP_GLOBAL float* Br = gptr(a.B + seg * a.fstr + x * r + s0);
        if (a.vec_l && s0 + 8 <= r) {  // 16-B aligned rows: two 16-B loads per operand
          const f32x4 d0 = gld4(dBr), d1 = gld4(dBr + 4), b0 = gld4(Br), b1 = gld4(Br + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            mx[j] = fabsf(d0[j]);
            mx[4 + j] = fabsf(d1[j]);
            mx[8 + j] = fabsf(b0[j]);
            mx[12 + j] = fabsf(b1[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (s0 + j < r) {
              mx[j] = fabsf(dBr[j]);
              mx[8 + j] = fabsf(Br[j]);
            }
        }
      } else {
        const HDP_GLOBAL float* As = gptr(a.A + seg * a.fstr + x);
        const HDP_GLOBAL float* dAs = gptr(a.dA + seg * a.dstr + x);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (s0 + j < r) {
            const float ad = dAs[(int64_t)(s0 + j) * a.in], av = As[(int64_t)(s0 + j) * a.in];
            mx[j] = fabsf(av - ad);
            mx[8 + j] = fabsf(ad);
          }
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], off));
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) red[wv][j] = mx[j];
    }
    __syncthreads();
    if (tid < 16) {
      const float v = fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid]));
      const int half = tid >> 3, j = tid & 7;
      if (s0 + j < r) part[half * r + s0 + j] = v;
    }
    __syncthreads();
  }
}

// exponent e with x < 2^e (frexp); 0 for zero and non-finite x
__device__ __forceinline__ int h2_exp(float x) {
  if (!(x > 0.f) || !isfinite(x)) return 0;
  int e;
  frexpf(x, &e);
  return e;
}

// per item: maxL_k, maxR_k from the partials; sl_k = 2^(14 - e(maxL_k)),
// E = 14 - max_k (e(maxR_k) - log2 sl_k), sr_k = 2^E / sl_k
__global__ __launch_bounds__(256) void k4_h2_fin_kernel(const DeltaArgs* __restrict__ items, const int* gate) {
  if (h2_gated_off(gate)) return;
  const DeltaArgs& a = items[blockIdx.x];
  const int r = a.r, K = 2 * r * a.nseg, tid = threadIdx.x;
  const int nbL = (int)((a.out + 255) / 256), nbR = (int)((a.in + 255) / 256);
  float* t = a.ktab;
  float* sl = t + 4;
  float* sr = t + 4 + K;
  const float* partL = t + 4 + 2 * K;
  const float* partR = partL + (int64_t)a.nseg * nbL * 2 * r;
  auto maxes = [&](int k, float& mL, float& mR) {
    const int seg = k / (2 * r), hs = k - seg * 2 * r;  // half * r + step
    mL = 0.f;
    mR = 0.f;
    for (int b = 0; b < nbL; ++b) mL = fmaxf(mL, partL[((int64_t)seg * nbL + b) * 2 * r + hs]);
    for (int b = 0; b < nbR; ++b) mR = fmaxf(mR, partR[((int64_t)seg * nbR + b) * 2 * r + hs]);
  };
  __shared__ int red[4];
  int emax = -100000;
  // a k whose L column is zero contributes nothing: it must not pull E down (its R row is
  // zeroed below), nor may a zero R row raise it
  for (int k = tid; k < K; k += 256) {
    float mL, mR;
    maxes(k, mL, mR);
    const int sle = min(100, max(-100, 14 - h2_exp(mL)));
    if (mL > 0.f && mR > 0.f && isfinite(mR)) emax = max(emax, h2_exp(mR) - sle);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) emax = max(emax, __shfl_xor(emax, off));
  if ((tid & 63) == 0) red[tid >> 6] = emax;
  __syncthreads();
  emax = max(max(red[0], red[1]), max(red[2], red[3]));
  const int E = emax == -100000 ? 0 : min(120, max(-120, 14 - emax));
  for (int k = tid; k < K; k += 256) {
    float mL, mR;
    maxes(k, mL, mR);
    const int sle = min(100, max(-100, 14 - h2_exp(mL)));
    sl[k] = ldexpf(1.f, sle);
    sr[k] = mL > 0.f ? ldexpf(1.f, min(126, max(-126, E - sle))) : 0.f;
  }
  if (tid == 0) t[0] = ldexpf(1.f, -E);
}

// H2 panels: one thread per (item, pair of 16-k chunks, L row block or R column block, row):
// both 16-k panels of one delta_h2_kernel chunk (a 64-B row of dB / B when r = 16).  The chunk
// count is padded to even; padding panels are zero.
__global__ __launch_bounds__(256) void k4_h2_pack_kernel(const DeltaArgs* __restrict__ items,
                                                         const int64_t* __restrict__ pack_start, int n,
                                                         const int* gate) {
  if (h2_gated_off(gate)) return;
  const int64_t e0 = (int64_t)blockIdx.x * 256;
  int lo = 0, hi = n - 1;  // largest m with pack_start[m] <= e0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pack_start[mid] <= e0) lo = mid;
    else hi = mid - 1;
  }
  const DeltaArgs a = items[lo];
  int64_t e = e0 - pack_start[lo] + threadIdx.x;
  const int r = a.r, per = (r + MX3::kSteps - 1) / MX3::kSteps;
  const int nch = a.nseg * per, npair = (nch + 1) >> 1, K = 2 * r * a.nseg;
  const int64_t nRB = (a.out + kDT - 1) / kDT, nCB = (a.in + kDT - 1) / kDT;
  const int64_t nL = (int64_t)npair * nRB * kDT, nR = (int64_t)npair * nCB * kDT;
  if (e >= nL + nR) return;
  const bool left = e < nL;
  if (!left) e -= nL;
  const int64_t nb = left ? nRB : nCB;
  const int x = (int)(e % kDT);
  const int64_t pp = e / kDT;  // pair * nb + block
  const int cp = (int)(pp / nb);
  const int64_t blk = pp - (int64_t)cp * nb;
  const int64_t xo = blk * kDT + x;
  const bool ok = xo < (left ? a.out : a.in);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c = 2 * cp + q;
    float v0[8], v1[8];  // k-slots 0..7 and 8..15
#pragma unroll
    for (int j = 0; j < 8; ++j) v0[j] = v1[j] = 0.f;
    if (c < nch) {
      const int seg = c / per, s0 = (c % per) * MX3::kSteps;
      const HDP_GLOBAL float* sc = gptr(a.ktab + 4 + (left ? 0 : K) + 2 * seg * r);  // sl or sr: [half][r]
      if (left && a.vec_l && s0 + 8 <= r) {  // 16-B aligned rows and scale vectors (r % 4 == 0)
        const HDP_GLOBAL float* dBr = gptr(a.dB + seg * a.dstr + (ok ? xo : 0) * r + s0);
        const HDP_GLOBAL float* Br = gptr(a.B + seg * a.fstr + (ok ? xo : 0) * r + s0);
        const f32x4 d0 = gld4(dBr), d1 = gld4(dBr + 4), b0 = gld4(Br), b1 = gld4(Br + 4);
        const f32x4 s00 = gld4(sc + s0), s01 = gld4(sc + s0 + 4), s10 = gld4(sc + r + s0), s11 = gld4(sc + r + s0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v0[j] = ok ? d0[j] * s00[j] : 0.f;
          v0[4 + j] = ok ? d1[j] * s01[j] : 0.f;
          v1[j] = ok ? b0[j] * s10[j] : 0.f;
          v1[4 + j] = ok ? b1[j] * s11[j] : 0.f;
        }
      } else if (left) {
        const HDP_GLOBAL float* dBr = gptr(a.dB + seg * a.dstr + (ok ? xo : 0) * r);
        const HDP_GLOBAL float* Br = gptr(a.B + seg * a.fstr + (ok ? xo : 0) * r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool in_r = ok && s0 + j < r;
          v0[j] = in_r ? dBr[s0 + j] * sc[s0 + j] : 0.f;
          v1[j] = in_r ? Br[s0 + j] * sc[r + s0 + j] : 0.f;
        }
      } else {
        const HDP_GLOBAL float* As = gptr(a.A + seg * a.fstr + (ok ? xo : 0));
        const HDP_GLOBAL float* dAs = gptr(a.dA + seg * a.dstr + (ok ? xo : 0));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const bool in_r = ok && s0 + j < r;
          const float ad = in_r ? dAs[(int64_t)(s0 + j) * a.in] : 0.f;
          const float av = in_r ? As[(int64_t)(s0 + j) * a.in] : 0.f;
          v0[j] = in_r ? (av - ad) * sc[s0 + j] : 0.f;  // powers of two: exact
          v1[j] = in_r ? ad * sc[r + s0 + j] : 0.f;
        }
      }
    }
    HDP_GLOBAL _Float16* panel =
        gptr(reinterpret_cast<_Float16*>(left ? a.limg : a.rimg) + ((int64_t)c * nb + blk) * kPanelH);
    f16x8 h0, l0, h1, l1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      h0[j] = (_Float16)v0[j];
      l0[j] = (_Float16)(v0[j] - (float)h0[j]);
      h1[j] = (_Float16)v1[j];
      l1[j] = (_Float16)(v1[j] - (float)h1[j]);
    }
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 0 * kDT * 16 + x * 16 + 8 * MX3::gran(x, 0)) = h0;
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 0 * kDT * 16 + x * 16 + 8 * MX3::gran(x, 1)) = h1;
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 1 * kDT * 16 + x * 16 + 8 * MX3::gran(x, 0)) = l0;
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 1 * kDT * 16 + x * 16 + 8 * MX3::gran(x, 1)) = l1;
  }
}

// ---- fused Adam + H2 pack (hp:356-373 folded into K4's operand preparation) --------
// Single-segment plans (Wn = 1): every operand half but two is constant across steps -- B (L half 1)
// and A (inside R half 0 = A - dA) never change (hp:375-376) -- and the Adam step bounds the deltas:
// |m_hat / sqrt(v_hat)| <= (1 - b1) / sqrt(1 - b2) sqrt((1 - rho^t) / (1 - rho)) sqrt(1 - b2^t) / (1 - b1^t)
// (Cauchy-Schwarz over the moment sums, rho = b1^2 / b2 < 1; the host passes D = lr x that bound x 1.01).
// So the per-k scales need no pass over the live factors: L half 0 (dB) is scaled by 2^(14 - e(D)),
// L half 1 (B) by its constant column maxima (packed ONCE, at plan creation), and the R rows' bounds are
// max|A[k][:]| + D and D.  Per step: k4_h2_bound_kernel writes the scale table from D and the constant
// maxima, then k4_h2_adam_pack_kernel runs Adam on each factor entry (grad -> m, v, delta; grad cleared)
// and writes the delta-dependent panel granules -- the scale pass, the fin pass and the standalone Adam
// and pack kernels are gone from the step.
struct AdamPackArgs {
  int* gate;           // set when a delta exceeds D: the gated scale / fin / pack kernels then re-pack
                       // every panel from the live deltas (m, v or t not from this Adam sequence)
  float D;
  float* dbase;        // the delta arena (the items' dA / dB point into it; written here)
  float* g;            // grad, m, v arenas: the same layout (element i of each belongs together)
  float* m;
  float* v;
  const int* err;      // probe error word (refusal: delta = 0, m / v untouched)
  AdamScalars s;
  int zero;            // clear grad
};

// constant maxima of one item: one workgroup per (item, side); side 0: max_o |B[o][k]|, side 1:
// max_c |A[k][c]|, k < r; 8 k per pass, rows / columns strided over the 256 threads
__global__ __launch_bounds__(256) void k4_h2_cmax_kernel(const DeltaArgs* __restrict__ items) {
  const DeltaArgs& a = items[blockIdx.x];
  const bool left = blockIdx.y == 0;
  const int r = a.r, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* cmax = a.ktab + h2_cmax_off(a.out, a.in, r, a.nseg) + (left ? 0 : r);
  __shared__ float red[4][8];
  const int64_t nx = left ? a.out : a.in;
  for (int s0 = 0; s0 < r; s0 += 8) {
    float mx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) mx[j] = 0.f;
    for (int64_t x = tid; x < nx; x += 256)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (s0 + j < r) mx[j] = fmaxf(mx[j], fabsf(left ? a.B[x * r + s0 + j] : a.A[(int64_t)(s0 + j) * a.in + x]));
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mx[j] = fmaxf(mx[j], __shfl_xor(mx[j], off));
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wv][j] = mx[j];
    __syncthreads();
    if (tid < 8 && s0 + tid < r) cmax[s0 + tid] = fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid]));
    __syncthreads();
  }
}

// per item: the scale table from the delta bound D and the constant maxima (k4_h2_fin_kernel's rule:
// sl_k = 2^(14 - e(maxL_k)), E = 14 - max_k (e(maxR_k) - log2 sl_k), sr_k = 2^E / sl_k) with
// maxL = (D | max|B[:, k]|) and maxR = (max|A[k, :]| + D | D)
__global__ __launch_bounds__(256) void k4_h2_bound_kernel(const DeltaArgs* __restrict__ items, float D, int* gate) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *gate = 0;  // set again by k4_h2_adam_pack_kernel if a delta exceeds D
  const DeltaArgs& a = items[blockIdx.x];
  const int r = a.r, K = 2 * r, tid = threadIdx.x;
  float* t = a.ktab;
  float* sl = t + 4;
  float* sr = t + 4 + K;
  const float* cB = t + h2_cmax_off(a.out, a.in, r, 1);
  const float* cA = cB + r;
  auto bounds = [&](int k, float& mL, float& mR) {
    const int half = k / r, step = k - half * r;
    mL = half ? cB[step] : D;
    mR = half ? D : cA[step] + D;
  };
  __shared__ int red[4];
  int emax = -100000;
  for (int k = tid; k < K; k += 256) {
    float mL, mR;
    bounds(k, mL, mR);
    const int sle = min(100, max(-100, 14 - h2_exp(mL)));
    if (mL > 0.f && mR > 0.f && isfinite(mR)) emax = max(emax, h2_exp(mR) - sle);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) emax = max(emax, __shfl_xor(emax, off));
  if ((tid & 63) == 0) red[tid >> 6] = emax;
  __syncthreads();
  emax = max(max(red[0], red[1]), max(red[2], red[3]));
  const int E = emax == -100000 ? 0 : min(120, max(-120, 14 - emax));
  for (int k = tid; k < K; k += 256) {
    float mL, mR;
    bounds(k, mL, mR);
    const int sle = min(100, max(-100, 14 - h2_exp(mL)));
    sl[k] = ldexpf(1.f, sle);
    sr[k] = mL > 0.f ? ldexpf(1.f, min(126, max(-126, E - sle))) : 0.f;
  }
  if (tid == 0) t[0] = ldexpf(1.f, -E);
}

// One thread per 4 factor entries, in the factors' own memory order -- an L thread owns dB[o][4 kq .. 4 kq
// + 3] (consecutive threads: consecutive quads of a row, then the next row), an R thread dA[4 kq .. 4 kq +
// 3][4 cq .. 4 cq + 3] (consecutive threads: consecutive column quads of the same 4 rows) -- so every
// g / m / v / delta / A access is a 16-B piece of a contiguous wave-wide stream, as in K3.  Each thread
// runs Adam on its entries and writes the 8-B halves of the panel granules that depend on them (L half
// 0; R halves 0 and 1).  Per item ap_start[i] threads: out * qr + ceil(in / 4) * qr, qr = ceil(r / 4);
// nseg == 1.
// r % 8 == 0 (every BASELINE config; r05): threads own 8 consecutive k-slots instead -- an L thread dB[o][8 k8 ..
// 8 k8 + 7], an R thread rows 8 k8 .. 8 k8 + 7 of dA at 4 columns -- so each writes WHOLE 16-B panel granules
// (8 k-slots of one half) instead of two scattered 8-B halves, and an R thread both halves of its panel rows
// (A - dA and dA: the full 32-B row per plane, contiguous over consecutive threads)
static inline int64_t h2_ap_threads(int64_t out, int64_t in, int r) {
  if (r % 8 == 0) return out * (r / 8) + (in + 3) / 4 * (r / 8);
  const int64_t qr = (r + 3) / 4;
  return out * qr + (in + 3) / 4 * qr;
}

__global__ __launch_bounds__(256) void k4_h2_adam_pack_kernel(const DeltaArgs* __restrict__ items,
                                                              const int64_t* __restrict__ ap_start, int n,
                                                              AdamPackArgs ap) {
#pragma clang fp contract(off)
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  const int64_t e0 = (int64_t)blockIdx.x * 256;
  int lo = 0, hi = n - 1;  // largest m with ap_start[m] <= e0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ap_start[mid] <= e0) lo = mid;
    else hi = mid - 1;
  }
  const bool refused = adam_refused(ap.err);
  const DeltaArgs& a = items[lo];
  const int r = a.r, K = 2 * r;
  const bool w8 = r % 8 == 0;  // item-uniform: 8 k-slots per thread (h2_ap_threads)
  const int qr = w8 ? r / 8 : (r + 3) / 4;
  int64_t e = e0 - ap_start[lo] + threadIdx.x;
  const int64_t nL = a.out * qr, ncq = (a.in + 3) / 4;
  if (e >= nL + ncq * qr) return;
  const bool left = e < nL;
  if (!left) e -= nL;
  // one 16-B group of 4 entries at element index idx of dA / dB (vec) or element-wise; -> dd, over
  auto adam4 = [&](const float* dbase_elem, int64_t idx, int cnt, bool vec, f32x4& dd) {
    // the items' dA / dB are read-only for K4; the writable pointer comes from the arena base
    const int64_t off = (dbase_elem - ap.dbase) + idx;
    float* dp = ap.dbase + off;
    dd = f32x4{0.f, 0.f, 0.f, 0.f};
    if (vec) {
      HDP_GLOBAL f32x4* G = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.g + off));
      HDP_GLOBAL f32x4* M = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.m + off));
      HDP_GLOBAL f32x4* V = reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.v + off));
      if (!refused) {
        f32x4 gg = *G, mm = *M, vv = *V;
        bool over = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float gq = gg[q], mq = mm[q], vq = vv[q], dq;
          adam1(gq, mq, vq, dq, ap.s);
          mm[q] = mq;
          vv[q] = vq;
          dd[q] = dq;
          over |= !(fabsf(dq) <= ap.D);
        }
        if (over) __hip_atomic_store(ap.gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *M = mm;
        *V = vv;
      }
      *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(dp)) = dd;
      if (ap.zero) *G = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    for (int q = 0; q < cnt; ++q) {
      float* dq_p = dp + q;
      const int64_t o2 = off + q;
      if (refused) {
        *gptr(dq_p) = 0.f;
      } else {
        float gq = *gptr(ap.g + o2), mq = *gptr(ap.m + o2), vq = *gptr(ap.v + o2), dq;
        adam1(gq, mq, vq, dq, ap.s);
        *gptr(ap.m + o2) = mq;
        *gptr(ap.v + o2) = vq;
        *gptr(dq_p) = dq;
        dd[q] = dq;
        if (!(fabsf(dq) <= ap.D)) __hip_atomic_store(ap.gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (ap.zero) *gptr(ap.g + o2) = 0.f;
    }
  };
  // 4 consecutive k-slots 4 kq .. of one panel row x (of block blk): an 8-B half granule
  auto put4 = [&](__bf16* img, int64_t nb, int64_t blk, int x, int kq, int half, const float (&v)[4]) {
    const int k0 = 4 * kq, c = k0 / MX3::kSteps, jo = k0 % MX3::kSteps;
    HDP_GLOBAL _Float16* panel = gptr(reinterpret_cast<_Float16*>(img) + ((int64_t)c * nb + blk) * kPanelH);
    f16x4 hh, ll;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      hh[j] = (_Float16)v[j];
      ll[j] = (_Float16)(v[j] - (float)hh[j]);
    }
    const int g = x * 16 + 8 * MX3::gran(x, half) + jo;
    *reinterpret_cast<HDP_GLOBAL f16x4*>(panel + 0 * kDT * 16 + g) = hh;
    *reinterpret_cast<HDP_GLOBAL f16x4*>(panel + 1 * kDT * 16 + g) = ll;
  };
  // 8 consecutive k-slots 8 k8 .. of one panel row x: a whole 16-B granule of each plane (chunk k8)
  auto put8 = [&](__bf16* img, int64_t nb, int64_t blk, int x, int k8, int half, const float (&v)[8]) {
    HDP_GLOBAL _Float16* panel = gptr(reinterpret_cast<_Float16*>(img) + ((int64_t)k8 * nb + blk) * kPanelH);
    f16x8 hh, ll;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hh[j] = (_Float16)v[j];
      ll[j] = (_Float16)(v[j] - (float)hh[j]);
    }
    const int g = x * 16 + 8 * MX3::gran(x, half);
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 0 * kDT * 16 + g) = hh;
    *reinterpret_cast<HDP_GLOBAL f16x8*>(panel + 1 * kDT * 16 + g) = ll;
  };
  const HDP_GLOBAL float* sc = gptr(a.ktab + 4);  // sl [half][r], then sr [half][r]
  // NJ 16-B groups of 4 entries at element offsets off[j] of the arenas, vectorised: every load of the NJ groups
  // first (g, m, v, and A where `A` is given), then Adam, then every store -- the per-group form (adam4) issues a
  // group's loads only behind the previous group's stores (the arenas may alias as far as the compiler knows),
  // one memory round trip per group (r05: the fused kernel ran at 0.45 of HBM against K3's 0.74)
  auto adam_vec = [&](auto nj, const int64_t* off, const float* A, f32x4* dd, f32x4* av) {
    constexpr int NJ = decltype(nj)::value;
    f32x4 G[NJ], M[NJ], V[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      G[j] = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(ap.g + off[j]));
      M[j] = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(ap.m + off[j]));
      V[j] = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(ap.v + off[j]));
      if (A) av[j] = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(A + (off[j] - (a.dA - ap.dbase))));
    }
    bool over = false;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float gq = G[j][q], mq = M[j][q], vq = V[j][q], dq;
        adam1(gq, mq, vq, dq, ap.s);
        M[j][q] = mq;
        V[j][q] = vq;
        dd[j][q] = dq;
        over |= !(fabsf(dq) <= ap.D);
      }
    if (over) __hip_atomic_store(ap.gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.m + off[j])) = M[j];
      *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.v + off[j])) = V[j];
      *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.dbase + off[j])) = dd[j];
      if (ap.zero) *reinterpret_cast<HDP_GLOBAL f32x4*>(gptr(ap.g + off[j])) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (w8) {
    if (left) {
      const int64_t o = e / qr;
      const int k8 = (int)(e - o * qr);
      f32x4 d0, d1;
      const int64_t idx = o * r + 8 * k8;
      if (a.vec_l && !refused) {
        const int64_t b0 = (a.dB - ap.dbase) + idx;
        const int64_t off[2] = {b0, b0 + 4};
        f32x4 dd[2];
        adam_vec(std::integral_constant<int, 2>{}, off, nullptr, dd, nullptr);
        d0 = dd[0];
        d1 = dd[1];
      } else {
        adam4(a.dB, idx, 4, a.vec_l, d0);
        adam4(a.dB, idx + 4, 4, a.vec_l, d1);
      }
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = d0[j] * sc[8 * k8 + j];
        v[4 + j] = d1[j] * sc[8 * k8 + 4 + j];
      }
      put8(a.limg, (a.out + kDT - 1) / kDT, o / kDT, (int)(o % kDT), k8, 0, v);  // (L half 1 = B: constant)
      return;
    }
    const int k8 = (int)(e / ncq);
    const int64_t c0 = 4 * (e - (int64_t)k8 * ncq);
    const int ccnt = (int)min((int64_t)4, a.in - c0);
    const bool vec = a.vec_r && ccnt == 4;
    float v0[4][8], v1[4][8];  // [column q][k-slot j]
    if (vec && !refused) {  // two halves of 4 rows: all loads of a half in flight together (~130 VGPRs)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
      int64_t off[4];
      const int64_t b0 = (a.dA - ap.dbase) + (int64_t)(8 * k8 + 4 * hh) * a.in + c0;
#pragma unroll
      for (int j = 0; j < 4; ++j) off[j] = b0 + (int64_t)j * a.in;
      f32x4 dd[4], av[4];
      adam_vec(std::integral_constant<int, 4>{}, off, a.A, dd, av);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = 4 * hh + jj;
        const int sk = 8 * k8 + j;
        const float s0v = sc[K + sk], s1v = sc[K + r + sk];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v0[q][j] = (av[jj][q] - dd[jj][q]) * s0v;  // powers of two: exact
          v1[q][j] = dd[jj][q] * s1v;
        }
      }
      }
    }
#pragma unroll
    for (int j = 0; j < ((vec && !refused) ? 0 : 8); ++j) {
      const int sk = 8 * k8 + j;
      const int64_t idx = (int64_t)sk * a.in + c0;
      f32x4 dd, av{0.f, 0.f, 0.f, 0.f};
      adam4(a.dA, idx, ccnt, vec, dd);
      if (vec) {
        av = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(a.A + idx));
      } else {
        for (int q = 0; q < ccnt; ++q) av[q] = a.A[idx + q];
      }
      const float s0v = sc[K + sk], s1v = sc[K + r + sk];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v0[q][j] = (av[q] - dd[q]) * s0v;  // powers of two: exact
        v1[q][j] = dd[q] * s1v;
      }
    }
    const int64_t nCB = (a.in + kDT - 1) / kDT;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= ccnt) break;
      const int64_t col = c0 + q;
      put8(a.rimg, nCB, col / kDT, (int)(col % kDT), k8, 0, v0[q]);
      put8(a.rimg, nCB, col / kDT, (int)(col % kDT), k8, 1, v1[q]);
    }
    return;
  }
  if (left) {
    const int64_t o = e / qr;
    const int kq = (int)(e - o * qr);
    const int cnt = min(4, r - 4 * kq);
    f32x4 dd;
    adam4(a.dB, o * r + 4 * kq, cnt, a.vec_l && cnt == 4, dd);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = j < cnt ? dd[j] * sc[4 * kq + j] : 0.f;
    put4(a.limg, (a.out + kDT - 1) / kDT, o / kDT, (int)(o % kDT), kq, 0, v);  // (L half 1 = B: constant)
    return;
  }
  const int kq = (int)(e / ncq);
  const int64_t c0 = 4 * (e - (int64_t)kq * ncq);
  const int ccnt = (int)min((int64_t)4, a.in - c0);
  const bool vec = a.vec_r && ccnt == 4;
  float v0[4][4], v1[4][4];  // [column q][k-slot j]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int sk = 4 * kq + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) v0[q][j] = v1[q][j] = 0.f;
    if (sk >= r) continue;
    const int64_t idx = (int64_t)sk * a.in + c0;
    f32x4 dd, av{0.f, 0.f, 0.f, 0.f};
    adam4(a.dA, idx, ccnt, vec, dd);
    if (vec) {
      av = *reinterpret_cast<const HDP_GLOBAL f32x4*>(gptr(a.A + idx));
    } else {
      for (int q = 0; q < ccnt; ++q) av[q] = a.A[idx + q];
    }
    const float s0v = sc[K + sk], s1v = sc[K + r + sk];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v0[q][j] = (av[q] - dd[q]) * s0v;  // powers of two: exact
      v1[q][j] = dd[q] * s1v;
    }
  }
  const int64_t nCB = (a.in + kDT - 1) / kDT;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q >= ccnt) break;
    const int64_t col = c0 + q;
    put4(a.rimg, nCB, col / kDT, (int)(col % kDT), kq, 0, v0[q]);
    put4(a.rimg, nCB, col / kDT, (int)(col % kDT), kq, 1, v1[q]);
  }
}

// ---- delta_h2_kernel: the x3w schedule (256 x 128 tiles, 8 waves, XCD-contiguous tile walk,
// direct global->LDS staging) on H2 panels.  A chunk is 32 k = two 16-k sub-images of
// [L block rb | L block rb + 1 | R block] (8 KB each): 48 KB, a 3-chunk ring (144 KB).  Waves
// 0-5 each stage one panel (8 x 1 KB pieces per chunk), waves 6-7 none.  Per chunk and wave: 2
// sub-images x 4 blocks x 3 MFMAs = 24 v_mfma_f32_32x32x16_f16, the x3w count for twice the k.
constexpr int kH2Buf = 12288;  // floats per chunk buffer (48 KB)
// HDP_H2_ABL (measurement builds only, tools/k4abl_build.sh; 0 in the library): bit 0 drops the bf16 W
// read-modify-write of full tiles, bit 1 the MFMAs and their fragment reads, bit 2 the panel staging, bit 3 the
// RND per-segment folds, bit 5 the per-chunk workgroup barrier, bit 6 the ring wait (both: wrong results)
#ifndef HDP_H2_ABL
#define HDP_H2_ABL 0
#endif
constexpr int kH2NB = 3;

__device__ __forceinline__ void h2_mfma(const _Float16* Lb, const _Float16* Rb, int h, int l32, int ow, int cw,
                                        f32x16 (&acc)[2][2]) {
  if constexpr ((HDP_H2_ABL & 2) != 0) return;
  f16x8 fa[2][2], fb[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int xa = ow + 32 * i + l32, xb = cw + 32 * i + l32;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      fa[i][p] = *reinterpret_cast<const f16x8*>(Lb + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
      fb[i][p] = *reinterpret_cast<const f16x8*>(Rb + p * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));
    }
  }
#pragma unroll
  for (int bo = 0; bo < 2; ++bo)
#pragma unroll
    for (int bc = 0; bc < 2; ++bc) {
      f32x16 d = acc[bo][bc];
      d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][1], fb[bc][0], d, 0, 0, 0);  // lo * hi
      d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][0], fb[bc][1], d, 0, 0, 0);  // hi * lo
      d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][0], fb[bc][0], d, 0, 0, 0);  // hi * hi
      acc[bo][bc] = d;
    }
}

// RND chunk (bf16 MERGE of multi-segment plans): the running dW lives in the accumulators themselves, negated
// and in the item's scaled units (r06b): n = -2^E dW.  A segment's MFMA chain starts from C = n, so at its end
// acc = n + sum_seg L R, and the fold is n = f32(bf16(acc)) in place -- the reference's bf16(dW - bracket)
// (hp:389-392) in scaled units (a power-of-two scale commutes with round-to-nearest-even), 3 VALU per pair of
// elements (v_cvt_pk_bf16_f32, then the two halves back to f32 in the accumulator registers), no separate
// running-sum registers and no accumulator zeroing.  The tile's end multiplies by 2^-E once.  (The earlier form
// kept a packed running dW beside the accumulators, dW = bf16(dW - 2^-E acc) and acc = 0 per fold: 56 VALU per
// block; Wn = 8 Mistral / 13B -4 / -2 %, profiles/r06_k4_wn8_ablation.txt.  The f32 sum now rounds onto n at every
// MFMA instead of onto the segment's partial sum: differences at 2^-24 |dW| against the bf16 half-ulp 2^-9.)
__device__ __forceinline__ void h2_fold_block(f32x16& acc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t p = cvt_pk_bf16(acc[2 * j], acc[2 * j + 1]);
    acc[2 * j] = __uint_as_float(p << 16);
    acc[2 * j + 1] = __uint_as_float(p & 0xffff0000u);
  }
}
// `fold` (wave-uniform): the chunk closes a rank segment -- block b's fold is issued right behind block b + 1's
// MFMAs (the fold of blocks 0-2 runs beside MFMAs instead of after all of them)
__device__ __forceinline__ void h2_mfma_rnd(const _Float16* Lb, const _Float16* Rb, int h, int l32, int ow, int cw,
                                            f32x16 (&acc)[2][2], bool fold) {
  if constexpr ((HDP_H2_ABL & 2) != 0) return;
  f16x8 fa[2][2], fb[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int xa = ow + 32 * i + l32, xb = cw + 32 * i + l32;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      fa[i][p] = *reinterpret_cast<const f16x8*>(Lb + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
      fb[i][p] = *reinterpret_cast<const f16x8*>(Rb + p * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));
    }
  }
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int bo = b >> 1, bc = b & 1;
    f32x16 d = acc[bo][bc];
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][1], fb[bc][0], d, 0, 0, 0);  // lo * hi
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][0], fb[bc][1], d, 0, 0, 0);  // hi * lo
    d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[bo][0], fb[bc][0], d, 0, 0, 0);  // hi * hi
    acc[bo][bc] = d;
    if ((HDP_H2_ABL & 8) == 0 && b > 0 && fold) h2_fold_block(acc[(b - 1) >> 1][(b - 1) & 1]);
  }
  if ((HDP_H2_ABL & 8) == 0 && fold) h2_fold_block(acc[1][1]);
}

__device__ __forceinline__ int h2_chunks(const DeltaArgs& a) {
  return (a.nseg * ((a.r + MX3::kSteps - 1) / MX3::kSteps) + 1) >> 1;
}

__device__ __forceinline__ void h2_load_tile(const DeltaGroup& g, X3WLoad& L, int wave) {
  L.m = x3w_module(g.tile_start, L.m, L.t);
  const DeltaArgs& a = g.items[L.m];
  const int out = (int)a.out, in = (int)a.in;
  int o_t, c_t;
  x3w_origin(out, in, (int)(L.t - g.tile_start[L.m]), o_t, c_t);
  const int nRB = (out + kDT - 1) / kDT, nCB = (in + kDT - 1) / kDT;
  L.c = 0;
  L.nch = h2_chunks(a);
  if (wave < 6) {  // wave = 3 sub + kind; rows past the module's last 128 re-read a panel (never stored)
    const int sub = wave / 3, kind = wave % 3;
    const int nb = kind < 2 ? nRB : nCB;
    const int blk = kind == 0 ? o_t / kDT : kind == 1 ? min(o_t / kDT + 1, nRB - 1) : c_t / kDT;
    const __bf16* img = kind < 2 ? a.limg : a.rimg;
    L.src = reinterpret_cast<const char*>(img) + ((int64_t)sub * nb + blk) * kPanelH * 2;
    L.step = (int64_t)2 * nb * kPanelH * 2;
  } else {
    L.src = reinterpret_cast<const char*>(a.limg);
    L.step = 0;
  }
}

// ---- deferred bf16 merge (DEF = 3; bf16 MERGE plans, single segment, >= 4 chunks per tile) ----
// The immediate epilogue reads the W tile behind the LAST chunk's MFMAs only and touches W with 64
// two-byte accesses per lane.  Here a full tile's result becomes 8 lanes' worth of 16-byte pieces of
// whole 128-B rows: d = bf16(-acc) (the merge's rounded dW), transposed within each quad of lanes so
// that lane (q = l32 >> 2, i = l32 & 3) holds row 8 j + 4 h + i, columns 4 q .. 4 q + 3 of block
// (bo, bc), then lanes q and q ^ 1 trade halves: the even one takes block 0's columns 4 q .. 4 q + 7,
// the odd one block 1's columns 4 q - 4 .. 4 q + 3 of the same row, so every wave-instruction moves 8
// rows x 128 contiguous bytes (8 dwordx4 per lane instead of 16 dwordx2: half the W instructions,
// no half-line requests; -19 % K4 time on Mistral-7B shapes).  The NEXT tile's iteration 0 loads those
// W pieces, iteration 2 adds and stores them: the W read-modify-write runs under two chunks of the next
// tile's MFMAs instead of in front of the epilogue.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 4 x 4 transpose of 16-bit values over the 4 lanes of a quad: lane i enters with column i (rows
// 0..3 in P0 = r0 | r1 << 16, P1 = r2 | r3 << 16) and leaves with row i (columns 0..3, same packing).
// Two butterflies: exchange with lane i ^ 1 (v_perm picks the halves: selA = 0x05040100 on even
// lanes, 0x03020706 on odd), then with lane i ^ 2 (whole dwords).
__device__ __forceinline__ void quad_transpose16(uint32_t& P0, uint32_t& P1, uint32_t selA, bool b1) {
  const uint32_t X0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)P0, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  const uint32_t X1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)P1, 0xB1, 0xF, 0xF, false);
  P0 = __builtin_amdgcn_perm(X0, P0, selA);
  P1 = __builtin_amdgcn_perm(X1, P1, selA);
  const uint32_t S = b1 ? P0 : P1;
  const uint32_t R = (uint32_t)__builtin_amdgcn_mov_dpp((int)S, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  if (b1) P0 = R;
  else P1 = R;
}
// piece p = 4 bo + j: soffset of its rows 32 bo + 8 j .. + 7 of the wave's tile (the lane's voffset
// adds its row 4 h + i and its 16 B of the 128-B row)
__device__ __forceinline__ int bpc_soff(int sbase, int rowb, int p) { return sbase + (32 * (p >> 2) + 8 * (p & 3)) * rowb; }
// W pieces of the pending tile: asm loads (invisible to the compiler's wait-count model, which would
// otherwise drain the LDS ring in front of their first use; the consumer waits explicitly)
__device__ __forceinline__ void bpc_load_asm(i32x4 rs4, int voff, int sbase, int rowb, u32x4 (&w)[8]) {
  if constexpr ((HDP_H2_ABL & 1) != 0) {
#pragma unroll
    for (int p = 0; p < 8; ++p) w[p] = u32x4{0u, 0u, 0u, 0u};
    return;
  }
  asm volatile("" : "+s"(sbase), "+s"(rowb));
#pragma unroll
  for (int p = 0; p < 8; ++p)
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(w[p]) : "v"(voff), "s"(rs4), "s"(bpc_soff(sbase, rowb, p)) : "memory");
}
// bf16(W + d) per element, two per dword
__device__ __forceinline__ uint32_t badd2(uint32_t w, uint32_t d) {
  const f32x2v wf{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  const f32x2v df{__uint_as_float(d << 16), __uint_as_float(d & 0xffff0000u)};
  const f32x2v v = wf + df;
  return cvt_pk_bf16(v[0], v[1]);
}
// The stores are asm with the wait states a 16-B store's data VGPRs need before a VALU may overwrite
// them inside the asm: the compiler scheduled such a write right behind the builtin store and the first
// data dword of some lanes was then stored from the NEW value, now and then (tools/dbg_k4_bf16.py)
__device__ __forceinline__ void bpc_store(i32x4 rs4, int voff, int sbase, int rowb, const u32x4 (&w)[8],
                                          const u32x4 (&d)[8]) {
  if constexpr ((HDP_H2_ABL & 1) != 0) {
#pragma unroll
    for (int p = 0; p < 8; ++p) asm volatile("" : : "v"(d[p]), "v"(w[p]));
    return;
  }
  asm volatile("" : "+s"(sbase), "+s"(rowb));
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const u32x4 v{badd2(w[p][0], d[p][0]), badd2(w[p][1], d[p][1]), badd2(w[p][2], d[p][2]), badd2(w[p][3], d[p][3])};
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" : : "v"(v), "v"(voff), "s"(rs4), "s"(bpc_soff(sbase, rowb, p)) : "memory");
  }
}
// lane ^ 4 (the neighbouring quad) by DPP within a 16-lane row: row_ror:4 gives lane i the value of
// lane i - 4 (what an odd quad needs), row_ror:12 that of lane i + 4 (an even quad); VALU only, no
// LDS-unit traffic beside the DMA ring
__device__ __forceinline__ uint32_t xor4_lane(uint32_t v, bool odd) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xF, 0xF, false);
  return odd ? lo : hi;
}

// DEF = 2: the deferred float32 merge of X3WDefer<2> (two pieces per chunk, stored one chunk
// after their loads: with a 3-chunk ring that wait needs no ring chunk the ring wait does not).
// DEF = 3: the deferred bf16 merge above.
// RND (bf16 MERGE of multi-segment plans, Wn > 1): the reference's per-rank rounding (hp:389-392,
// zeros_like(W_res) is bf16): the accumulators hold n = -2^E dW, each segment's MFMA chain adds its bracket to
// it and the fold rounds it to bf16 in place (h2_fold_block; a segment is ceil(r / 8) 16-k groups, an even number
// -- the plan requires r % 16 == 0 -- so segments end on chunk boundaries); at the tile's end acc = 2^-E n = -dW
// feeds the unchanged epilogues (which add bf16(-acc) = dW to W).
template <int MODE, int POL, int DEF = 0, int DT = HDP_F32, bool RND = false>  // DT: W dtype of a MERGE
__global__ __launch_bounds__(512, 1) void delta_h2_kernel(const DeltaArgs* __restrict__ items,
                                                          const int64_t* __restrict__ tile_start, int n,
                                                          int64_t total) {
  static_assert(!RND || (MODE == HDP_DW_MERGE && DT == HDP_BF16), "RND: bf16 MERGE plans only");
  constexpr int NB = kH2NB;
  constexpr bool kDefer = (DEF == 2 || DEF == 4) && MODE == HDP_DW_MERGE && DT == HDP_F32;
  constexpr bool kDeferB = DEF == 3 && MODE == HDP_DW_MERGE && DT == HDP_BF16;
  using DF = X3WDefer<DEF == 4 ? 4 : 2>;
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[NB * kH2Buf];
  const int nx = gridDim.x >= 8 ? 8 : 1;
  const int x = blockIdx.x % nx;
  const int64_t stride = gridDim.x / nx;
  const int64_t t_end = (int64_t)(x + 1) * g.total / nx;
  const int64_t t0 = (int64_t)x * g.total / nx + blockIdx.x / nx;
  if (t0 >= t_end || (int64_t)(blockIdx.x / nx) >= stride) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  int m0 = 0;
  {
    int lo = 0, hi = g.n - 1;  // largest m with tile_start[m] <= t0
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (g.tile_start[mid] <= t0) lo = mid;
      else hi = mid - 1;
    }
    m0 = lo;
  }
  X3WLoad L;
  L.t = t0;
  L.m = m0;
  L.live = true;
  h2_load_tile(g, L, wave);

  auto issue = [&](int buf) {
    if ((HDP_H2_ABL & 4) == 0 && wave < 6) {
      float* dst = smem + buf * kH2Buf + (wave / 3) * 6144 + (wave % 3) * 2048;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const HDP_GLOBAL void*>(gptr(L.src + j * 1024 + lane * 16)),
                                         (__attribute__((address_space(3))) void*)(dst + j * 256), 16, 0, 0);
    }
  };
  auto advance = [&]() {
    if (!L.live) return;
    if (++L.c < L.nch) {
      L.src += L.step;
      return;
    }
    L.t += stride;
    if (L.t >= t_end) {
      L.live = false;  // src stays on the last chunk: later issues repeat it
      return;
    }
    h2_load_tile(g, L, wave);
  };

  int64_t ct = t0;
  int cm = m0, cnch = 0, o_t = 0, c_t = 0;
  int cps = 1;      // RND: chunks per segment
  int segl = 1;     // RND: chunks left in the current segment (a countdown: no runtime modulo per chunk)
  float resc = 0.f;  // RND: 2^-E of the tile's item
  auto compute_tile = [&]() {
    cm = x3w_module(g.tile_start, cm, ct);
    const DeltaArgs& a = g.items[cm];
    cnch = h2_chunks(a);
    x3w_origin((int)a.out, (int)a.in, (int)(ct - g.tile_start[cm]), o_t, c_t);
    if constexpr (RND) {
      cps = ((a.r + MX3::kSteps - 1) / MX3::kSteps) >> 1;
      segl = cps;  // a tile starts a segment (cnch = nseg cps)
      resc = *gptr(a.ktab);
    }
  };
  compute_tile();

  f32x16 acc[2][2];
  zero_tile(acc);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    issue(b);
    advance();
  }
  // chunk i + 1 landed (this wave's pieces): the pieces of chunk i + 2 may stay in flight
  auto ring_wait = [&]() {
    if ((HDP_H2_ABL & 64) == 0 && wave < 6) __builtin_amdgcn_s_waitcnt(vmcnt_imm(8 * (NB - 2)));
  };
  ring_wait();  // chunks 0 and 1
  __builtin_amdgcn_s_barrier();

  constexpr bool kPrefetchW = MODE == HDP_DW_MERGE && !kDefer && !kDeferB;
  // deferred bf16 merge state (kDeferB): the pending tile's rounded dW in quad-transposed 8-B groups,
  // its W groups once loaded, and its address (wave-uniform scalars + this lane's offset)
  u32x4 bpend[kDeferB ? 8 : 1], bw[kDeferB ? 8 : 1];
  int pb_lo = 0, pb_hi = 0, pb_n = 0, pb_sbase = 0, pb_rowb = 0, pb_voff = 0;
  bool ppb = false;
  const uint32_t selA = (l32 & 1) ? 0x03020706u : 0x05040100u;
  const bool qb1 = (l32 & 2) != 0;
  auto pb_rs = [&]() {
    const uint64_t ptr = ((uint64_t)(uint32_t)pb_hi << 32) | (uint32_t)pb_lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), 0, pb_n, 0x00020000);
  };
  // deferred merge state (kDefer): the pending tile's accumulators (already scaled by 2^-E)
  // and address as wave-uniform scalars
  f32x16 pend[2][2];
  float wb[DF::D + 1][8 * DF::PPC];
  int pd_lo = 0, pd_hi = 0, pd_n = 0, pd_sbase = 0, pd_rowb = 0, pd_voff = 0;
  bool pp = false;
  auto pend_rs4 = [&]() {
    i32x4 r;
    r[0] = pd_lo;
    r[1] = pd_hi & 0xffff;
    r[2] = pd_n;
    r[3] = 0x00020000;
    return r;
  };
  auto pend_addr = [&]() {
    TileAddr t;
    const uint64_t ptr = ((uint64_t)(uint32_t)pd_hi << 32) | (uint32_t)pd_lo;
    t.rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), 0, pd_n, 0x00020000);
    t.voff = pd_voff;
    t.sbase = pd_sbase;
    t.rowb = pd_rowb;
    return t;
  };
  int ib = 0;  // i % NB (the ring slot of chunk i), kept as a counter: no modulo per chunk
  auto mfma_chunk = [&]() {
    const _Float16* b = reinterpret_cast<const _Float16*>(smem + ib * kH2Buf);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const _Float16* sb = b + sub * 12288;  // 24 KB sub-image = 12288 fp16
      h2_mfma(sb + (ow >> 7) * 4096, sb + 8192, h, l32, ow & (kDT - 1), cw, acc);
    }
  };
  // RND: chunk k of the tile, the segment fold inside the MFMA sequence (h2_mfma_rnd)
  auto rnd_chunk = [&](bool fold) {
    const _Float16* b = reinterpret_cast<const _Float16*>(smem + ib * kH2Buf);
    h2_mfma_rnd(b + (ow >> 7) * 4096, b + 8192, h, l32, ow & (kDT - 1), cw, acc, false);
    const _Float16* sb = b + 12288;
    h2_mfma_rnd(sb + (ow >> 7) * 4096, sb + 8192, h, l32, ow & (kDT - 1), cw, acc, fold);
  };
  // chunk k of the current tile: plain accumulation, or (RND) closing a rank segment
  auto mfma_step = [&](int k) {
    if constexpr (RND) {
      const bool fold = --segl == 0;  // chunk k closes a segment: (k + 1) % cps == 0
      if (fold) segl = cps;
      rnd_chunk(fold);
    } else {
      mfma_chunk();
    }
  };
  // end of chunk i: every wave done with buffer i % NB -> chunk i + NB into it
  auto next_chunk = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads are done
    if constexpr ((HDP_H2_ABL & 32) == 0) __builtin_amdgcn_s_barrier();
    issue(ib);
    advance();
    ib = ib + 1 == NB ? 0 : ib + 1;
  };
  for (;;) {
    int k = 0;
    bool relax3 = false;  // kDeferB: iteration 3 waits with the predecessor's 16 stores in flight
    if constexpr (kDeferB) {
      if (ppb) {  // iterations 0-2 carry the predecessor's W read-modify-write (the tile has >= 4 chunks)
        const i32x4 rs4{pb_lo, pb_hi & 0xffff, pb_n, 0x00020000};
        bpc_load_asm(rs4, pb_voff, pb_sbase, pb_rowb, bw);
        mfma_step(0);
        if (wave < 6) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk i + 1 (then i + 2 and 8 W loads)
        next_chunk();
        mfma_step(1);
        if (wave < 6) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk i + 2 (then 8 W loads, i + 3)
        next_chunk();
        if (wave < 6) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // the W loads (then chunks i + 3, i + 4)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(bw[q]));
        bpc_store(rs4, pb_voff, pb_sbase, pb_rowb, bw, bpend);
        mfma_step(2);
        if (wave < 6) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk i + 3 (then i + 4, 8 stores)
        next_chunk();
        k = 3;
        relax3 = true;
      }
    }
    if constexpr (kDefer) {
      if (pp) {  // the predecessor's merge on iterations 0 .. span - 1 (cnch >= min_chunks)
        static_for<DF::span>([&](auto kc) {
          constexpr int K = decltype(kc)::value;
          if constexpr (K < DF::G)
            wgroup_load_asm<K * DF::PPC, DF::PPC, POL>(pend_rs4(), pend_addr(), wb[K % (DF::D + 1)]);
          mfma_chunk();
          if constexpr (K >= DF::D) {
            constexpr int J = K - DF::D;
            if (wave < 6) wait_regs<DF::after_load(J, 8)>(wb[J % (DF::D + 1)]);
            else wait_regs<DF::after_load(J, 0)>(wb[J % (DF::D + 1)]);
            wgroup_store<J * DF::PPC, DF::PPC, POL>(pend_addr(), pend, wb[J % (DF::D + 1)]);
          }
          constexpr int w = DF::wops(K - 1) + DF::wops(K) + 8 * (NB - 2);
          if (wave < 6) __builtin_amdgcn_s_waitcnt(vmcnt_imm(w > 63 ? 63 : w));
          next_chunk();
        });
        k = DF::span;
      }
    }
    for (; k + 1 < cnch; ++k) {
      mfma_step(k);
      if (kDeferB && relax3 && k == 3) {
        if (wave < 6) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk i + 4 (then 8 stores, i + 5)
      } else if (kDefer || kDeferB || k != 0) {
        ring_wait();  // (a tile end without deferral drains the counter)
      }
      next_chunk();
    }
    {
      const DeltaArgs& a = g.items[cm];
      const int64_t o_w = o_t + ow, c_w = c_t + cw;
      const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
      const TileAddr taddr = tile_addr<DT == HDP_F32 ? 4 : 2>(a, o_w, c_w, l32, h);
      WPrefetch<MODE, DT> wpf;
      if constexpr (kPrefetchW) {
        if (full) wpf.template load<POL>(taddr);  // covered by the last chunk's MFMAs
      }
      mfma_step(cnch - 1);
      if constexpr (RND) {  // the last segment was folded with its chunk: acc = n = -2^E dW -> -dW
#pragma unroll
        for (int bo = 0; bo < 2; ++bo)
#pragma unroll
          for (int bc = 0; bc < 2; ++bc)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[bo][bc][e] *= resc;
      } else {
        const float esc = *gptr(a.ktab);  // 2^-E: exact
#pragma unroll
        for (int bo = 0; bo < 2; ++bo)
#pragma unroll
          for (int bc = 0; bc < 2; ++bc)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[bo][bc][e] *= esc;
      }
      if constexpr (kDeferB) {
        // (16-B pieces need 16-B aligned rows: other modules' tiles take the element-wise epilogue)
        const bool al16 = (a.in & 7) == 0 && (reinterpret_cast<uintptr_t>(a.dst) & 15) == 0;
        if (full && al16) {  // rounded dW as 16-B pieces of 128-B rows (quad transpose, then a q ^ 1 trade); stored by the next tile
          const bool odd = (l32 & 4) != 0;
#pragma unroll
          for (int bo = 0; bo < 2; ++bo)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              uint32_t P[2][2];
#pragma unroll
              for (int bc = 0; bc < 2; ++bc) {
                const f32x16& A = acc[bo][bc];
                P[bc][0] = cvt_pk_bf16(-A[4 * j], -A[4 * j + 1]);
                P[bc][1] = cvt_pk_bf16(-A[4 * j + 2], -A[4 * j + 3]);
                quad_transpose16(P[bc][0], P[bc][1], selA, qb1);
              }
              // even quad: [own block 0 | partner's block 0]; odd: [partner's block 1 | own block 1]
              const uint32_t r0 = xor4_lane(odd ? P[0][0] : P[1][0], odd);
              const uint32_t r1 = xor4_lane(odd ? P[0][1] : P[1][1], odd);
              bpend[4 * bo + j] = odd ? u32x4{r0, r1, P[1][0], P[1][1]} : u32x4{P[0][0], P[0][1], r0, r1};
            }
          const uint64_t dptr = reinterpret_cast<uint64_t>(a.dst);
          pb_lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)dptr);
          pb_hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(dptr >> 32));
          pb_n = __builtin_amdgcn_readfirstlane((int)(a.out * a.in * 2));
          pb_sbase = __builtin_amdgcn_readfirstlane(taddr.sbase);
          pb_rowb = __builtin_amdgcn_readfirstlane(taddr.rowb);
          pb_voff = (4 * h + (l32 & 3)) * taddr.rowb + (odd ? 64 + 8 * ((l32 >> 2) - 1) : 8 * (l32 >> 2));
          ppb = true;
          if (wave < 6) {
            if (relax3 && k == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // as iteration 3 above
            else ring_wait();
          }
        } else {  // edge (or unaligned) tile: element-wise epilogue (its predecessor's stores were issued at iteration 2)
          ppb = false;
          __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
          epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, false, l32, h);
        }
      } else if constexpr (kDefer) {
        pp = full;  // the predecessor's merge finished by iteration span - 1 <= cnch - 2
        if (full) {
#pragma unroll
          for (int xx = 0; xx < 2; ++xx)
#pragma unroll
            for (int yy = 0; yy < 2; ++yy) pend[xx][yy] = acc[xx][yy];
          const uint64_t dptr = reinterpret_cast<uint64_t>(a.dst);
          pd_lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)dptr);
          pd_hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(dptr >> 32));
          pd_n = __builtin_amdgcn_readfirstlane((int)(a.out * a.in * 4));
          pd_sbase = __builtin_amdgcn_readfirstlane(taddr.sbase);
          pd_rowb = __builtin_amdgcn_readfirstlane(taddr.rowb);
          pd_voff = taddr.voff;
          ring_wait();  // counts no W ops: at most conservative
        } else {
          __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
          epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, false, l32, h);  // edge: element-wise
        }
      } else {
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // W and every chunk in flight have landed
        epilogue<MODE, DT, true, POL>(a, acc, wpf, taddr, o_w, c_w, full, l32, h);
      }
      zero_tile(acc);
    }
    ct += stride;
    if (ct >= t_end) break;
    compute_tile();
    next_chunk();
  }
  if constexpr (kDefer) {
    if (pp) {  // the workgroup's last tile
      float w[64];
      const TileAddr t = pend_addr();
      wgroup_load<0, 8, POL>(t, w);
      wgroup_store<0, 8, POL>(t, pend, w);
    }
  }
  if constexpr (kDeferB) {
    if (ppb) {  // the workgroup's last tile: compiler-tracked loads
      const __amdgpu_buffer_rsrc_t rs = pb_rs();
#pragma unroll
      for (int q = 0; q < 8; ++q) bw[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, pb_voff, bpc_soff(pb_sbase, pb_rowb, q), 0);
      bpc_store(i32x4{pb_lo, pb_hi & 0xffff, pb_n, 0x00020000}, pb_voff, pb_sbase, pb_rowb, bw, bpend);
    }
  }
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // no LDS-DMA outstanding when the workgroup retires
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// validate one module's operands and fill its descriptor (shared by both entry points)
static int make_args(const char* who, int64_t out, int64_t in, int r, int nseg, const float* dA, const float* dB,
                     int64_t delta_seg_stride, const float* A, const float* B, int64_t factor_seg_stride, void* dst,
                     int dst_dtype, int mode, int round_bf16, DeltaArgs& a) {
  HDP_CHECK_ARG(out > 0 && in > 0 && r > 0 && nseg > 0, "%s: bad shape out=%lld in=%lld r=%d nseg=%d", who,
                (long long)out, (long long)in, r, nseg);
  HDP_CHECK_ARG(out * in * (dst_dtype == HDP_BF16 && mode == HDP_DW_MERGE ? 2 : 4) < ((int64_t)1 << 31),
                "%s: matrix too large (%lld x %lld; the kernel addresses one module's dst with 31-bit offsets)", who,
                (long long)out, (long long)in);
  HDP_CHECK_ARG(dA && dB && A && B && dst, "%s: null pointer", who);
  HDP_CHECK_ARG(mode == HDP_DW_STORE || mode == HDP_DW_MERGE, "%s: bad mode %d", who, mode);
  HDP_CHECK_ARG(dst_dtype == HDP_F32 || dst_dtype == HDP_BF16, "%s: bad dtype %d", who, dst_dtype);
  HDP_CHECK_ARG(mode == HDP_DW_MERGE || dst_dtype == HDP_F32, "%s: STORE mode writes float32", who);
  HDP_CHECK_ARG(!(round_bf16 && mode == HDP_DW_MERGE && dst_dtype == HDP_F32),
                "%s: round_bf16 applies to bf16 W_res (or STORE), not to a float32 merge", who);
  HDP_CHECK_ARG(nseg == 1 || (delta_seg_stride > 0 && factor_seg_stride > 0), "%s: segment strides must be positive",
                who);
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
  a.limg = a.rimg = nullptr;
  a.ktab = nullptr;
  return HDP_OK;
}

// algorithmic work of one module: dst written (and W read for MERGE) once + the 4 factor
// operands once; 4 r nseg flop per element
static double args_bytes(const DeltaArgs& a, int mode, int dst_dtype) {
  const double wes = (mode == HDP_DW_MERGE && dst_dtype == HDP_BF16) ? 2.0 : 4.0;
  return (double)a.out * a.in * (mode == HDP_DW_MERGE ? 2.0 * wes : 4.0) + 8.0 * a.r * (a.out + a.in) * a.nseg;
}
static double args_flops(const DeltaArgs& a) { return 4.0 * a.out * a.in * a.r * a.nseg; }
static int64_t args_tiles(const DeltaArgs& a, int tr = kDT) { return ((a.out + tr - 1) / tr) * ((a.in + kDT - 1) / kDT); }

// K4 math selection (hdp_delta_set_math / HDP_K4_MATH=auto|f32|x3): AUTO takes the exact
// f32 MFMA while K4 is HBM-bound (K = 2 r nseg <= 32) and the bf16x3 split above that.
static int g_math = -1;
static int k4_math() {
  if (g_math < 0) {
    const char* e = getenv("HDP_K4_MATH");
    g_math = HDP_MATH_AUTO;
    if (e && (e[0] == 'f' || e[0] == 'F')) g_math = HDP_MATH_F32;
    if (e && (e[0] == 'x' || e[0] == 'X')) g_math = HDP_MATH_X3;
    if (e && (e[0] == 'h' || e[0] == 'H')) g_math = HDP_MATH_H2;
  }
  return g_math;
}
// x3 plan kernel (HDP_K4_X3_STAGE): wide = delta_x3w_kernel (default), glds = delta_x3g_kernel,
// regs = delta_x3p_kernel
enum { X3_REGS = 0, X3_GLDS = 1, X3_WIDE = 2 };
static int g_stage = -1;  // hdp_delta_set_x3_stage overrides the env
static int x3_stage() {
  if (g_stage < 0) {
    const char* e = getenv("HDP_K4_X3_STAGE");
    g_stage = X3_WIDE;
    if (e && e[0] == 'r') g_stage = X3_REGS;
    if (e && e[0] == 'g') g_stage = X3_GLDS;
  }
  return g_stage;
}
static bool use_x3(int r, int nseg) {
  const int m = k4_math();
  return m == HDP_MATH_X3 || m == HDP_MATH_H2 || (m == HDP_MATH_AUTO && 2 * r * nseg > 32);
}

}  // namespace hdp

using namespace hdp;

extern "C" int hdp_delta_set_math(int math) {
  HDP_CHECK_ARG(math == HDP_MATH_AUTO || math == HDP_MATH_F32 || math == HDP_MATH_X3 || math == HDP_MATH_H2,
                "hdp_delta_set_math: bad math %d", math);
  const int prev = k4_math();
  g_math = math;
  return prev;
}

extern "C" int hdp_delta_set_x3_stage(int stage) {
  if (stage != X3_REGS && stage != X3_GLDS && stage != X3_WIDE) {  // -1: the valid returns are 0..2
    set_error("hdp_delta_set_x3_stage: bad stage %d", stage);
    return -1;
  }
  const int prev = x3_stage();
  g_stage = stage;
  return prev;
}

extern "C" int hdp_delta_gemm(int64_t out, int64_t in, int r, int nseg, const float* dA, const float* dB,
                              int64_t delta_seg_stride, const float* A, const float* B,
                              int64_t factor_seg_stride, void* dst, int dst_dtype, int mode, int round_bf16,
                              void* stream) {
  DeltaArgs a;
  const int rc = make_args("hdp_delta_gemm", out, in, r, nseg, dA, dB, delta_seg_stride, A, B, factor_seg_stride, dst,
                           dst_dtype, mode, round_bf16, a);
  if (rc != HDP_OK) return rc;
  const int64_t nwg = args_tiles(a);
  HDP_CHECK_ARG(nwg < (1ll << 31), "hdp_delta_gemm: grid too large");
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)nwg), block(256);
  // fp32: one accumulation chain over all K = 2 r nseg (float32 rounding differs from the
  // reference's rank-by-rank sum only at the 1e-7 level); bf16 with round_bf16: the
  // rank-ordered running sum with bf16 rounding after every segment, as hp:389-392 does.
  const bool rnd = round_bf16 != 0;
  const bool x3 = use_x3(r, nseg);
#define HDP_LAUNCH(M, D, R)                                                                 \
  do {                                                                                      \
    if (x3) hipLaunchKernelGGL((delta_gemm_kernel<M, D, R, MX3>), grid, block, 0, st, a); \
    else hipLaunchKernelGGL((delta_gemm_kernel<M, D, R, MF32>), grid, block, 0, st, a);   \
  } while (0)
  KTimer kt(nseg == 1 ? K_DELTA : K_DELTA_MULTI, st, args_bytes(a, mode, dst_dtype), args_flops(a));
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

// ---- grouped plans ----------------------------------------------------------------------
struct hdp_delta_plan_s {
  DeltaArgs* d_items = nullptr;   // device copies of the descriptors
  int64_t* d_start = nullptr;     // device tile prefix (n + 1)
  int n = 0;
  int64_t total = 0;
  int mode = 0, dtype = 0, round = 0;
  int grid = 0;
  int multiseg = 0;
  int pol = 3;  // float32 MERGE cache policy (HDP_DELTA_POL: bit 0 nt stores, bit 1 nt W loads)
  int x3 = 0;   // bf16x3 split math (decided at creation from the largest K of the items)
  int stage = 0;  // x3: X3_REGS / X3_GLDS / X3_WIDE (fixes the tile geometry of tile_start)
  int def = 0;    // deferred W merge: X3WDefer 1 / 2 (float32 MERGE), 3 = bf16 H2 MERGE (delta_h2_kernel)
  int h2 = 0;     // fp16x2 scaled split (delta_h2_kernel; float32 MERGE / STORE plans)
  float* d_ktab = nullptr;  // h2: per-item scale tables
  int* d_sstart = nullptr;  // h2: k4_h2_scale_kernel workgroup prefix per item
  int sblocks = 0;
  __bf16* d_img = nullptr;         // x3: packed operand panels of every item (MX3P)
  int64_t* d_pack_start = nullptr; // x3: k4_pack_kernel thread-space prefix (256-aligned)
  int64_t* d_ap_start = nullptr;   // fused: k4_h2_adam_pack_kernel thread-space prefix (256-aligned)
  int64_t ap_total = 0;
  int64_t pack_total = 0;
  double bytes = 0.0, flops = 0.0;
  int fused = 0;        // h2 single-segment MERGE: hdp_delta_plan_run_adam applies
  double pack_bytes = 0.0;  // x3 / H2 operand preparation: factors read by the scale pass (H2) and the pack,
                            // panels written (24 B per (row or column, k-slot) for H2, 20 B for x3)
  double adam_bytes = 0.0;  // fused Adam + pack: g, m, v read, m, v, delta, g written (28 B per entry),
                            // + A read and 8 B of R panel per A entry, 4 B of L panel per B entry
  int const_done = 0;   // fused: constant maxima and the constant panel halves written
  int* d_gate = nullptr;
};

template <class K>
static int plan_grid(K kernel, int threads, int64_t total, int& grid) {
  int dev = 0, cus = 0, per_cu = 0;
  HDP_CHECK_HIP(hipGetDevice(&dev));
  HDP_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HDP_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0));
  const int64_t resident = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  grid = (int)std::min<int64_t>(resident, total);
  if (grid >= 8) grid -= grid % 8;  // the XCD-contiguous schedule deals G / 8 workgroups per XCD
  return HDP_OK;
}

extern "C" int hdp_delta_plan_create(const hdp_delta_item* items, int n, int dst_dtype, int mode, int round_bf16,
                                     hdp_delta_plan* plan) {
  HDP_CHECK_ARG(plan && items && n > 0, "hdp_delta_plan_create: need a plan pointer and n > 0 items");
  *plan = nullptr;
  std::vector<DeltaArgs> host(n);
  std::vector<int64_t> start(n + 1, 0);
  double bytes = 0.0, flops = 0.0;
  int multiseg = 0, kmax_r = 0, kmax_seg = 1;
  for (int i = 0; i < n; ++i) {
    const hdp_delta_item& it = items[i];
    const int rc = make_args("hdp_delta_plan_create", it.out, it.in, it.r, it.nseg, it.dA, it.dB, it.delta_seg_stride,
                             it.A, it.B, it.factor_seg_stride, it.dst, dst_dtype, mode, round_bf16, host[i]);
    if (rc != HDP_OK) return rc;
    bytes += args_bytes(host[i], mode, dst_dtype);
    flops += args_flops(host[i]);
    multiseg |= it.nseg > 1;
    if (2 * it.r * it.nseg > 2 * kmax_r * kmax_seg) {
      kmax_r = it.r;
      kmax_seg = it.nseg;
    }
  }
  // float32 STORE plans at K = 32 (Wn = 1, r = 16): the exact f32 MFMA form is MFMA-bound there (half the
  // bytes of a MERGE behind the same 64-cycle f32 MFMAs), so AUTO takes H2 from K = 32 on; env
  // HDP_K4_STORE=f32 keeps the f32 form
  bool store_h2 = mode == HDP_DW_STORE && !round_bf16 && k4_math() == HDP_MATH_AUTO && 2 * kmax_r * kmax_seg >= 32;
  if (const char* e = getenv("HDP_K4_STORE")) store_h2 = store_h2 && e[0] != 'f';
  const bool x3 = use_x3(kmax_r, kmax_seg) || store_h2;
  // a bf16 MERGE of single-segment items (Wn = 1): the ROUND form's dW = bf16(0 - bracket) added as
  // bf16(W + bf16(dW)) is bit-identical to the plain form, whose epilogue adds bf16(-acc) -- so it
  // runs without the running sum (and on the wide x3 kernel, which the ROUND form's registers spill)
  if (round_bf16 && mode == HDP_DW_MERGE && dst_dtype == HDP_BF16 && !multiseg) round_bf16 = 0;
  // the wide x3 kernel's bf16 ROUND merge (running sum + accumulators + bf16 W) spills: X3G there
  int stage = x3 ? x3_stage() : X3_REGS;
  // H2 (AUTO or HDP_MATH_H2) for float32 results and for bf16 merges without per-rank rounding
  // (single-segment plans, see above); bf16 ROUND merges keep bf16x3
  // bf16 ROUND merges (Wn > 1) run on H2 too when every segment ends on a 32-k chunk boundary
  // (ceil(r / 8) even, i.e. r % 16 == 0 for the BASELINE configs): per-segment bf16 folds in the
  // kernel (RND); HDP_K4_RND=x3 keeps them on bf16x3
  bool rnd_h2 = round_bf16 && mode == HDP_DW_MERGE && dst_dtype == HDP_BF16;
  for (int i = 0; i < n && rnd_h2; ++i) rnd_h2 = (((host[i].r + MX3::kSteps - 1) / MX3::kSteps) & 1) == 0;
  if (const char* e = getenv("HDP_K4_RND")) rnd_h2 = rnd_h2 && e[0] != 'x';
  const bool h2 = x3 && (k4_math() == HDP_MATH_AUTO || k4_math() == HDP_MATH_H2) && (!round_bf16 || rnd_h2);
  if (h2) stage = X3_WIDE;  // the same 256 x 128 tile geometry
  else if (stage == X3_WIDE && mode == HDP_DW_MERGE && dst_dtype == HDP_BF16 && round_bf16) stage = X3_GLDS;
  const int tr = (x3 && stage == X3_WIDE) ? 2 * kDT : kDT;
  for (int i = 0; i < n; ++i) start[i + 1] = start[i] + args_tiles(host[i], tr);
  hdp_delta_plan p = new hdp_delta_plan_s;
  p->n = n;
  p->total = start[n];
  p->mode = mode;
  p->dtype = dst_dtype;
  p->round = round_bf16 != 0;
  p->multiseg = multiseg;
  p->bytes = bytes;
  p->flops = flops;
  if (const char* e = getenv("HDP_DELTA_POL")) p->pol = atoi(e) & 15;
  p->x3 = x3;
  p->stage = stage;
  p->h2 = h2;
  if (h2 && mode == HDP_DW_MERGE && dst_dtype == HDP_F32) {  // H2 chunks are 32 k: X3WDefer<2> needs min_chunks
    int64_t nch_min = INT64_MAX;
    for (int i = 0; i < n; ++i)
      nch_min = std::min<int64_t>(nch_min, (host[i].nseg * ((host[i].r + MX3::kSteps - 1) / MX3::kSteps) + 1) / 2);
    // X3WDefer<4> (W loads two chunks ahead) where every tile has >= 7 chunks: LLaMA-2-7B shapes at Wn = 8,
    // 4 layers 2.415 -> 2.341 ms (tools/delta_bench.py --pol 3, r04)
    int want = 4;
    if (const char* e = getenv("HDP_K4_DEFER")) want = atoi(e);
    if (want == 4 && nch_min < x3w_defer_min_chunks<4>()) want = 2;
    p->def = (want != 0 && nch_min >= x3w_defer_min_chunks<2>()) ? (want == 4 ? 4 : 2) : 0;
  }
  if (h2 && mode == HDP_DW_MERGE && dst_dtype == HDP_BF16) {  // deferred bf16 merge: every tile >= 4 chunks
    // (Mistral-7B r = 64, 8 layers: 3.28 -> 3.15 ms per run, tools/delta_bench.py, r03)
    int64_t nch_min = INT64_MAX;
    for (int i = 0; i < n; ++i)
      nch_min = std::min<int64_t>(nch_min, (host[i].nseg * ((host[i].r + MX3::kSteps - 1) / MX3::kSteps) + 1) / 2);
    int want = 3;
    if (const char* e = getenv("HDP_K4_DEFER")) want = atoi(e) == 0 ? 0 : 3;
    p->def = (want == 3 && nch_min >= 4) ? 3 : 0;
  }
  if (x3 && !h2 && stage == X3_WIDE && mode == HDP_DW_MERGE && dst_dtype == HDP_F32 && !round_bf16) {
    // the deferred merge needs every tile's chunk count >= the variant's min_chunks
    int64_t nch_min = host[0].nseg * ((host[0].r + MX3::kSteps - 1) / MX3::kSteps);
    for (int i = 1; i < n; ++i)
      nch_min = std::min<int64_t>(nch_min, host[i].nseg * ((host[i].r + MX3::kSteps - 1) / MX3::kSteps));
    int want = 0;  // measured slower so far (register pressure): opt-in
    if (const char* e = getenv("HDP_K4_DEFER")) want = atoi(e);
    if (want == 1 && nch_min < x3w_defer_min_chunks<1>()) want = 2;
    if (want == 2 && nch_min < x3w_defer_min_chunks<2>()) want = 0;
    p->def = (want == 1 || want == 2) ? want : 0;
  }
  std::vector<int64_t> pstart(n + 1, 0);
  int64_t img_elems = 0;
  std::vector<int64_t> img_off(n, 0);
  // H2: panels of 16 k per (chunk, block), the chunk count padded to even; scale tables
  std::vector<int64_t> ktab_off(n, 0);
  std::vector<int> sstart(n + 1, 0);
  int64_t ktab_floats = 0;
  auto img_chunks = [&](const DeltaArgs& a) {
    const int64_t nch = (int64_t)a.nseg * ((a.r + MX3::kSteps - 1) / MX3::kSteps);
    return h2 ? (nch + 1) / 2 * 2 : nch;
  };
  const int64_t panel = h2 ? kPanelH : kPanel;
  if (p->x3) {
    for (int i = 0; i < n; ++i) {
      const DeltaArgs& a = host[i];
      const int64_t nch = img_chunks(a);
      const int64_t nRB = (a.out + kDT - 1) / kDT, nCB = (a.in + kDT - 1) / kDT;
      img_off[i] = img_elems;
      img_elems += nch * (nRB + nCB) * panel;
      const int64_t th = (h2 ? nch / 2 : nch) * (nRB + nCB) * kDT;  // H2: a thread per pair of chunks
      pstart[i + 1] = pstart[i] + (th + 255) / 256 * 256;
      ktab_off[i] = ktab_floats;
      ktab_floats += (h2_tab_floats(a.out, a.in, a.r, a.nseg) + 63) / 64 * 64;
      sstart[i + 1] = sstart[i] + a.nseg * (int)((a.out + 255) / 256 + (a.in + 255) / 256);
    }
    p->pack_total = pstart[n];
    p->sblocks = sstart[n];
    for (int i = 0; i < n; ++i)
      p->pack_bytes += (h2 ? 24.0 : 20.0) * host[i].r * host[i].nseg * (double)(host[i].out + host[i].in);
  }
  int rc = HDP_OK;
  // every instance of a kernel has the same launch bounds and LDS: the f32 MERGE instance
  // stands for all of them in the occupancy query
  if (h2) rc = plan_grid(delta_h2_kernel<HDP_DW_MERGE, 0>, 512, p->total, p->grid);
  else if (x3 && stage == X3_WIDE) rc = plan_grid(delta_x3w_kernel<HDP_DW_MERGE, HDP_F32, false, 0>, 512, p->total, p->grid);
  else rc = plan_grid(delta_group_kernel<HDP_DW_MERGE, HDP_F32, false>, 256, p->total, p->grid);
  if (rc == HDP_OK && p->x3) {
    if (hipMalloc(&p->d_img, sizeof(__bf16) * img_elems) != hipSuccess ||
        hipMalloc(&p->d_pack_start, sizeof(int64_t) * (n + 1)) != hipSuccess ||
        hipMemcpy(p->d_pack_start, pstart.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) != hipSuccess) {
      set_error("hdp_delta_plan_create: packed-panel workspace allocation failed (%lld bytes)",
                (long long)(sizeof(__bf16) * img_elems));
      rc = HDP_EHIP;
    } else if (h2 && (hipMalloc(&p->d_ktab, sizeof(float) * ktab_floats) != hipSuccess ||
                      hipMemset(p->d_ktab, 0, sizeof(float) * ktab_floats) != hipSuccess ||
                      hipMalloc(&p->d_sstart, sizeof(int) * (n + 1)) != hipSuccess ||
                      hipMemcpy(p->d_sstart, sstart.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice) !=
                          hipSuccess)) {
      set_error("hdp_delta_plan_create: scale-table allocation failed");
      rc = HDP_EHIP;
    } else {
      for (int i = 0; i < n; ++i) {
        const DeltaArgs& a = host[i];
        const int64_t nch = img_chunks(a);
        host[i].limg = p->d_img + img_off[i];
        host[i].rimg = p->d_img + img_off[i] + nch * ((a.out + kDT - 1) / kDT) * panel;
        if (h2) host[i].ktab = p->d_ktab + ktab_off[i];
      }
    }
  }
  p->fused = h2 && !multiseg && mode == HDP_DW_MERGE;
  std::vector<int64_t> apst(n + 1, 0);
  for (int i = 0; i < n && p->fused; ++i) {
    p->adam_bytes += (double)host[i].r * ((28.0 + 4.0) * host[i].out + (28.0 + 4.0 + 8.0) * host[i].in);
    apst[i + 1] = apst[i] + (h2_ap_threads(host[i].out, host[i].in, host[i].r) + 255) / 256 * 256;
  }
  p->ap_total = apst[n];
  if (rc == HDP_OK && p->fused &&
      (hipMalloc(&p->d_ap_start, sizeof(int64_t) * (n + 1)) != hipSuccess ||
       hipMemcpy(p->d_ap_start, apst.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) != hipSuccess)) {
    set_error("hdp_delta_plan_create: fused-Adam table allocation failed");
    rc = HDP_EHIP;
  }
  if (rc == HDP_OK && p->fused && (hipMalloc(&p->d_gate, 256) != hipSuccess || hipMemset(p->d_gate, 0, 256) != hipSuccess)) {
    set_error("hdp_delta_plan_create: gate allocation failed");
    rc = HDP_EHIP;
  }
  if (rc == HDP_OK && (hipMalloc(&p->d_items, sizeof(DeltaArgs) * n) != hipSuccess ||
                       hipMalloc(&p->d_start, sizeof(int64_t) * (n + 1)) != hipSuccess ||
                       hipMemcpy(p->d_items, host.data(), sizeof(DeltaArgs) * n, hipMemcpyHostToDevice) != hipSuccess ||
                       hipMemcpy(p->d_start, start.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) !=
                           hipSuccess)) {
    set_error("hdp_delta_plan_create: device table allocation/copy failed");
    rc = HDP_EHIP;
  }
  if (rc != HDP_OK) {
    hdp_delta_plan_destroy(p);
    return rc;
  }
  *plan = p;
  return HDP_OK;
}

static int plan_launch(hdp_delta_plan p, hipStream_t st, bool pack);

extern "C" int hdp_delta_plan_run(hdp_delta_plan p, void* stream) {
  HDP_CHECK_ARG(p && p->d_items && p->grid > 0, "hdp_delta_plan_run: invalid plan");
  return plan_launch(p, as_stream(stream), true);
}

extern "C" int hdp_delta_plan_fused_adam(hdp_delta_plan p) { return p ? p->fused : 0; }

extern "C" int hdp_delta_plan_invalidate(hdp_delta_plan p) {
  HDP_CHECK_ARG(p, "hdp_delta_plan_invalidate: null plan");
  p->const_done = 0;
  return HDP_OK;
}

extern "C" int hdp_delta_plan_run_adam(hdp_delta_plan p, float* grad, float* m, float* v, float* delta,
                                       float grad_scale, float beta1, float one_minus_beta1, float beta2,
                                       float one_minus_beta2, float bc1, float bc2, float lr, float eps,
                                       float delta_bound, int zero_grad, void* stream) {
  HDP_CHECK_ARG(p && p->d_items && p->grid > 0, "hdp_delta_plan_run_adam: invalid plan");
  HDP_CHECK_ARG(p->fused, "hdp_delta_plan_run_adam: the plan has no fused Adam (single-segment H2 merge plans only)");
  HDP_CHECK_ARG(grad && m && v && delta, "hdp_delta_plan_run_adam: null arena pointer");
  HDP_CHECK_ARG(bc1 != 0.f && bc2 != 0.f, "hdp_delta_plan_run_adam: bias correction is zero (t == 0?)");
  HDP_CHECK_ARG(delta_bound >= 0.f, "hdp_delta_plan_run_adam: negative delta bound");
  hipStream_t st = as_stream(stream);
  {
    KTimer kp(K_DELTA_PACK, st, 0.0);
    if (!p->const_done) {  // once: constant maxima, and every panel (the constant L half 1 = B included)
      hipLaunchKernelGGL(k4_h2_cmax_kernel, dim3((unsigned)p->n, 2), dim3(256), 0, st, p->d_items);
      hipLaunchKernelGGL(k4_h2_scale_kernel, dim3((unsigned)p->sblocks), dim3(256), 0, st, p->d_items, p->d_sstart,
                         p->n, (const int*)nullptr);
      hipLaunchKernelGGL(k4_h2_fin_kernel, dim3((unsigned)p->n), dim3(256), 0, st, p->d_items, (const int*)nullptr);
      hipLaunchKernelGGL(k4_h2_pack_kernel, dim3((unsigned)(p->pack_total / 256)), dim3(256), 0, st, p->d_items,
                         p->d_pack_start, p->n, (const int*)nullptr);
      HDP_CHECK_LAUNCH();
      p->const_done = 1;
    }
    hipLaunchKernelGGL(k4_h2_bound_kernel, dim3((unsigned)p->n), dim3(256), 0, st, p->d_items, delta_bound, p->d_gate);
  }
  HDP_CHECK_LAUNCH();
  {
    KTimer ka(K_ADAM, st, p->adam_bytes);
    AdamPackArgs ap;
    ap.gate = p->d_gate;
    ap.D = delta_bound;
    ap.dbase = delta;
    ap.g = grad;
    ap.m = m;
    ap.v = v;
    ap.err = probe_err_device();
    ap.s = AdamScalars{grad_scale, beta1, one_minus_beta1, beta2, one_minus_beta2, bc1, bc2, lr, eps};
    ap.zero = zero_grad ? 1 : 0;
    hipLaunchKernelGGL(k4_h2_adam_pack_kernel, dim3((unsigned)(p->ap_total / 256)), dim3(256), 0, st, p->d_items,
                       p->d_ap_start, p->n, ap);
  }
  HDP_CHECK_LAUNCH();
  {  // fallback: only if a delta exceeded D (moments not from this Adam sequence) -- then the gated
     // passes rebuild the scales and every panel from the live deltas; otherwise three empty launches
    KTimer kp(K_DELTA_PACK, st, 0.0);
    hipLaunchKernelGGL(k4_h2_scale_kernel, dim3((unsigned)p->sblocks), dim3(256), 0, st, p->d_items, p->d_sstart, p->n,
                       (const int*)p->d_gate);
    hipLaunchKernelGGL(k4_h2_fin_kernel, dim3((unsigned)p->n), dim3(256), 0, st, p->d_items, (const int*)p->d_gate);
    hipLaunchKernelGGL(k4_h2_pack_kernel, dim3((unsigned)(p->pack_total / 256)), dim3(256), 0, st, p->d_items,
                       p->d_pack_start, p->n, (const int*)p->d_gate);
  }
  HDP_CHECK_LAUNCH();
  return plan_launch(p, st, false);
}

extern "C" int hdp_delta_plan_fused_fallback(hdp_delta_plan p, int* taken) {
  HDP_CHECK_ARG(p && taken, "hdp_delta_plan_fused_fallback: null argument");
  *taken = 0;
  if (p->d_gate) HDP_CHECK_HIP(hipMemcpy(taken, p->d_gate, sizeof(int), hipMemcpyDeviceToHost));
  return HDP_OK;
}

static int plan_launch(hdp_delta_plan p, hipStream_t st, bool pack) {
  DeltaGroup g{p->d_items, p->d_start, p->n, p->total};
  dim3 grid((unsigned)p->grid), block(256), wblock(512);
#define HDP_LAUNCH_K(M, D, R, P)                                                                            \
  do {                                                                                                      \
    if (p->x3 && p->stage == X3_WIDE)                                                                       \
      hipLaunchKernelGGL((delta_x3w_kernel<M, D, R, P>), grid, wblock, 0, st, g.items, g.tile_start, g.n,     \
                         g.total);                                                                          \
    else if (p->x3 && p->stage == X3_GLDS)                                                                  \
      hipLaunchKernelGGL((delta_x3g_kernel<M, D, R, P>), grid, block, 0, st, g.items, g.tile_start, g.n,      \
                         g.total);                                                                          \
    else if (p->x3)                                                                                         \
      hipLaunchKernelGGL((delta_x3p_kernel<M, D, R, P>), grid, block, 0, st, g.items, g.tile_start, g.n,      \
                         g.total);                                                                          \
    else                                                                                                    \
      hipLaunchKernelGGL((delta_group_kernel<M, D, R, P, MF32>), grid, block, 0, st, g.items, g.tile_start,     \
                         g.n, g.total);                                                                     \
  } while (0)
#define HDP_LAUNCH(M, D, R) HDP_LAUNCH_K(M, D, R, 0)
#define HDP_LAUNCH_P(M, D, P) HDP_LAUNCH_K(M, D, false, P)
  if (p->x3 && pack) {  // pack the operand panels first (same stream: K4 below reads them)
    KTimer kp(K_DELTA_PACK, st, p->pack_bytes);
    if (p->h2) {  // the scale table from the live factors, then the scaled fp16 panels
      p->const_done = 0;  // (a later fused run re-packs the constant halves with its own scale rule)
      hipLaunchKernelGGL(k4_h2_scale_kernel, dim3((unsigned)p->sblocks), dim3(256), 0, st, p->d_items, p->d_sstart,
                         p->n, (const int*)nullptr);
      hipLaunchKernelGGL(k4_h2_fin_kernel, dim3((unsigned)p->n), dim3(256), 0, st, p->d_items, (const int*)nullptr);
      hipLaunchKernelGGL(k4_h2_pack_kernel, dim3((unsigned)(p->pack_total / 256)), dim3(256), 0, st, p->d_items,
                         p->d_pack_start, p->n, (const int*)nullptr);
    } else {
      hipLaunchKernelGGL(k4_pack_kernel, dim3((unsigned)(p->pack_total / 256)), dim3(256), 0, st, p->d_items,
                         p->d_pack_start, p->n);
    }
  }
  HDP_CHECK_LAUNCH();
  if (p->h2) {
    KTimer kt(p->multiseg ? K_DELTA_MULTI : K_DELTA, st, p->bytes, p->flops);
    if (p->mode == HDP_DW_STORE)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_STORE, 0>), grid, wblock, 0, st, g.items, g.tile_start, g.n, g.total);
    else if (p->dtype == HDP_BF16 && p->round && p->def == 3)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 0, 3, HDP_BF16, true>), grid, wblock, 0, st, g.items,
                         g.tile_start, g.n, g.total);
    else if (p->dtype == HDP_BF16 && p->round)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 0, 0, HDP_BF16, true>), grid, wblock, 0, st, g.items,
                         g.tile_start, g.n, g.total);
    else if (p->dtype == HDP_BF16 && p->def == 3)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 0, 3, HDP_BF16>), grid, wblock, 0, st, g.items, g.tile_start,
                         g.n, g.total);
    else if (p->dtype == HDP_BF16)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 0, 0, HDP_BF16>), grid, wblock, 0, st, g.items, g.tile_start,
                         g.n, g.total);
    else if (p->pol == 3 && p->def == 2)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 3, 2>), grid, wblock, 0, st, g.items, g.tile_start, g.n,
                         g.total);
    else if (p->pol == 3 && p->def == 4)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 3, 4>), grid, wblock, 0, st, g.items, g.tile_start, g.n,
                         g.total);
    else if (p->pol == 3)
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 3>), grid, wblock, 0, st, g.items, g.tile_start, g.n, g.total);
    else
      hipLaunchKernelGGL((delta_h2_kernel<HDP_DW_MERGE, 0>), grid, wblock, 0, st, g.items, g.tile_start, g.n, g.total);
    HDP_CHECK_LAUNCH();
    return HDP_OK;
  }
  KTimer kt(p->multiseg ? K_DELTA_MULTI : K_DELTA, st, p->bytes, p->flops);
  if (p->mode == HDP_DW_STORE) {
    if (p->round) HDP_LAUNCH(HDP_DW_STORE, HDP_F32, true);
    else HDP_LAUNCH(HDP_DW_STORE, HDP_F32, false);
  } else if (p->dtype == HDP_F32) {
    switch (p->pol) {
      case 1: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 1); break;
      case 2: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 2); break;
      case 3:
        if (p->x3 && p->stage == X3_WIDE && p->def == 1)
          hipLaunchKernelGGL((delta_x3w_kernel<HDP_DW_MERGE, HDP_F32, false, 3, 1>), grid, wblock, 0, st, g.items,
                             g.tile_start, g.n, g.total);
        else if (p->x3 && p->stage == X3_WIDE && p->def == 2)
          hipLaunchKernelGGL((delta_x3w_kernel<HDP_DW_MERGE, HDP_F32, false, 3, 2>), grid, wblock, 0, st, g.items,
                             g.tile_start, g.n, g.total);
        else
          HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 3);
        break;
      case 7: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 7); break;
      case 11: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 11); break;
      case 15: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 15); break;
      case 4: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 4); break;
      default: HDP_LAUNCH(HDP_DW_MERGE, HDP_F32, false);
    }
  } else {
    if (p->round) HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, true);
    else HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, false);
  }
#undef HDP_LAUNCH
#undef HDP_LAUNCH_P
#undef HDP_LAUNCH_K
  HDP_CHECK_LAUNCH();
  return HDP_OK;
}

extern "C" int hdp_delta_plan_math(hdp_delta_plan p) {
  if (!p) return -1;
  return p->h2 ? HDP_MATH_H2 : p->x3 ? HDP_MATH_X3 : HDP_MATH_F32;
}

extern "C" int hdp_delta_plan_tiles(hdp_delta_plan p, int64_t* tiles, int* grid) {
  HDP_CHECK_ARG(p, "hdp_delta_plan_tiles: null plan");
  if (tiles) *tiles = p->total;
  if (grid) *grid = p->grid;
  return HDP_OK;
}

extern "C" int hdp_delta_plan_destroy(hdp_delta_plan p) {
  if (!p) return HDP_OK;
  int rc = HDP_OK;
  if (p->d_items && hipFree(p->d_items) != hipSuccess) rc = HDP_EHIP;
  if (p->d_start && hipFree(p->d_start) != hipSuccess) rc = HDP_EHIP;
  if (p->d_img && hipFree(p->d_img) != hipSuccess) rc = HDP_EHIP;
  if (p->d_pack_start && hipFree(p->d_pack_start) != hipSuccess) rc = HDP_EHIP;
  if (p->d_ap_start && hipFree(p->d_ap_start) != hipSuccess) rc = HDP_EHIP;
  if (p->d_ktab && hipFree(p->d_ktab) != hipSuccess) rc = HDP_EHIP;
  if (p->d_sstart && hipFree(p->d_sstart) != hipSuccess) rc = HDP_EHIP;
  if (p->d_gate && hipFree(p->d_gate) != hipSuccess) rc = HDP_EHIP;
  delete p;
  if (rc != HDP_OK) set_error("hdp_delta_plan_destroy: hipFree failed");
  return rc;
}
