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
                __builtin_amdgcn_raw_buffer_load_b32(t.rs, t.voff, reg_soff<4>(t, bo, bc, e), (POL & 2) ? 2 : 0));
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
                                                  (POL & 1) ? 2 : 0);
          } else if constexpr (DT == HDP_F32) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(wpf.w[bo][bc][e] + val), t.rs, t.voff,
                                                  reg_soff<4>(t, bo, bc, e), (POL & 1) ? 2 : 0);
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
          reinterpret_cast<float*>(a.dst)[idx] = val;
        } else if constexpr (DT == HDP_F32) {
          reinterpret_cast<float*>(a.dst)[idx] += val;
        } else {
          uint16_t* p = reinterpret_cast<uint16_t*>(a.dst) + idx;
          *p = f32_to_bf16(bf16_to_f32(*p) + round_bf16(val));
        }
      }
    }
  }
}

template <int MODE, int DT, bool ROUND>
__global__ __launch_bounds__(256, 2) void delta_gemm_kernel(DeltaArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * kLDS];
  const int nC = (int)((a.in + kDT - 1) / kDT);
  const int nO = (int)((a.out + kDT - 1) / kDT);
  const int id = xcd_remap(blockIdx.x, nO * nC);
  const int tO = id / nC, tC = id % nC;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t o_t = (int64_t)tO * kDT, c_t = (int64_t)tC * kDT;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;  // wave offsets inside the tile
  const int64_t o_w = o_t + ow, c_w = c_t + cw;
  const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
  constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
  const TileAddr taddr = tile_addr<ESZ>(a, o_w, c_w, l32, h);
  const int per = (a.r + kSC - 1) / kSC;
  const int nchunks = a.nseg * per;

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only: the bf16-rounded running dW
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;

  Stage st;
  stage_load(a, 0, o_t, c_t, tid, st);
  stage_store(smem, tid, st);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const float* buf = smem + (c & 1) * kLDS;
    if (c + 1 < nchunks) stage_load(a, c + 1, o_t, c_t, tid, st);       // next chunk in flight
    if constexpr (MODE == HDP_DW_MERGE) {
      if (c + 1 == nchunks && full) wpf.load(taddr);                   // W tile in flight
    }
    chunk_mfma(buf, h, l32, ow, cw, acc);
    if (ROUND && (c + 1) % per == 0) fold_segment(run, acc);  // dW = bf16(dW - bracket_i)
    if (c + 1 < nchunks) {
      // the other buffer was last read in chunk c-1, before the previous barrier: free
      stage_store(smem + ((c + 1) & 1) * kLDS, tid, st);
      __syncthreads();
    }
  }
  // the tile's dW: ROUND keeps the bf16 running sum in `run`; otherwise it is -acc
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

__device__ __forceinline__ int chunks_of(const DeltaArgs& a) { return a.nseg * ((a.r + kSC - 1) / kSC); }

__device__ __forceinline__ void tile_origin(const DeltaArgs& a, int64_t l, int64_t& o_t, int64_t& c_t) {
  const int64_t nC = (a.in + kDT - 1) / kDT;
  const int64_t q = l / nC;
  o_t = q * kDT;
  c_t = (l - q * nC) * kDT;
}

template <int MODE, int DT, bool ROUND, int POL = 0>
__global__ __launch_bounds__(256, 2) void delta_group_kernel(const DeltaArgs* __restrict__ items,
                                                             const int64_t* __restrict__ tile_start, int n,
                                                             int64_t total) {
  // (separate __restrict__ parameters: the descriptor loads are provably unclobbered by the
  // kernel's W stores, so they become scalar loads into SGPRs)
  const DeltaGroup g{items, tile_start, n, total};
  __shared__ __attribute__((aligned(16))) float smem[2 * kLDS];
  int64_t t = blockIdx.x;
  if (t >= g.total) return;
  const int64_t stride = gridDim.x;
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
  int c = 0, nch = chunks_of(a), per = (a.r + kSC - 1) / kSC;

  f32x16 acc[2][2];
  f32x16 run[2][2];  // ROUND only: the bf16-rounded running dW
  zero_tile(acc);
  if constexpr (ROUND) zero_tile(run);
  WPrefetch<MODE, (MODE == HDP_DW_STORE ? HDP_F32 : DT)> wpf;

  Stage st;
  stage_load(a, 0, o_t, c_t, tid, st);
  stage_store(smem, tid, st);
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
      if (tn < g.total) {
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
    const bool has_next = tn < g.total;
    const int64_t o_w = o_t + ow, c_w = c_t + cw;
    const bool full = (o_w + 64 <= a.out) && (c_w + 64 <= a.in);
    constexpr int ESZ = (MODE == HDP_DW_MERGE && DT == HDP_BF16) ? 2 : 4;
    const TileAddr taddr = tile_addr<ESZ>(a, o_w, c_w, l32, h);
    if (has_next) stage_load(an, cn, on_t, cn_t, tid, st);             // next factors in flight
    if constexpr (MODE == HDP_DW_MERGE) {
      if (last && full) wpf.template load<POL>(taddr);                  // W tile in flight
    }
    chunk_mfma(smem + buf * kLDS, h, l32, ow, cw, acc);
    if (ROUND && (c + 1) % per == 0) fold_segment(run, acc);
    // the other buffer was last read before the previous barrier: free
    if (has_next) stage_store(smem + (buf ^ 1) * kLDS, tid, st);
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
      nch = chunks_of(a);
      per = (a.r + kSC - 1) / kSC;
    }
    o_t = on_t;
    c_t = cn_t;
  }
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
  return HDP_OK;
}

// algorithmic work of one module: dst written (and W read for MERGE) once + the 4 factor
// operands once; 4 r nseg flop per element
static double args_bytes(const DeltaArgs& a, int mode, int dst_dtype) {
  const double wes = (mode == HDP_DW_MERGE && dst_dtype == HDP_BF16) ? 2.0 : 4.0;
  return (double)a.out * a.in * (mode == HDP_DW_MERGE ? 2.0 * wes : 4.0) + 8.0 * a.r * (a.out + a.in) * a.nseg;
}
static double args_flops(const DeltaArgs& a) { return 4.0 * a.out * a.in * a.r * a.nseg; }
static int64_t args_tiles(const DeltaArgs& a) { return ((a.out + kDT - 1) / kDT) * ((a.in + kDT - 1) / kDT); }

}  // namespace hdp

using namespace hdp;

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
#define HDP_LAUNCH(M, D, R) hipLaunchKernelGGL((delta_gemm_kernel<M, D, R>), grid, block, 0, st, a)
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
  double bytes = 0.0, flops = 0.0;
};

template <int M, int D, bool R>
static int plan_grid(int64_t total, int& grid) {
  int dev = 0, cus = 0, per_cu = 0;
  HDP_CHECK_HIP(hipGetDevice(&dev));
  HDP_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  HDP_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, delta_group_kernel<M, D, R>, 256, 0));
  const int64_t resident = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
  grid = (int)std::min<int64_t>(resident, total);
  return HDP_OK;
}

extern "C" int hdp_delta_plan_create(const hdp_delta_item* items, int n, int dst_dtype, int mode, int round_bf16,
                                     hdp_delta_plan* plan) {
  HDP_CHECK_ARG(plan && items && n > 0, "hdp_delta_plan_create: need a plan pointer and n > 0 items");
  *plan = nullptr;
  std::vector<DeltaArgs> host(n);
  std::vector<int64_t> start(n + 1, 0);
  double bytes = 0.0, flops = 0.0;
  int multiseg = 0;
  for (int i = 0; i < n; ++i) {
    const hdp_delta_item& it = items[i];
    const int rc = make_args("hdp_delta_plan_create", it.out, it.in, it.r, it.nseg, it.dA, it.dB, it.delta_seg_stride,
                             it.A, it.B, it.factor_seg_stride, it.dst, dst_dtype, mode, round_bf16, host[i]);
    if (rc != HDP_OK) return rc;
    start[i + 1] = start[i] + args_tiles(host[i]);
    bytes += args_bytes(host[i], mode, dst_dtype);
    flops += args_flops(host[i]);
    multiseg |= it.nseg > 1;
  }
  hdp_delta_plan p = new hdp_delta_plan_s;
  p->n = n;
  p->total = start[n];
  p->mode = mode;
  p->dtype = dst_dtype;
  p->round = round_bf16 != 0;
  p->multiseg = multiseg;
  p->bytes = bytes;
  p->flops = flops;
  if (const char* e = getenv("HDP_DELTA_POL")) p->pol = atoi(e) & 3;
  int rc = HDP_OK;
  const bool rnd = p->round;
  if (mode == HDP_DW_STORE) rc = rnd ? plan_grid<HDP_DW_STORE, HDP_F32, true>(p->total, p->grid)
                                     : plan_grid<HDP_DW_STORE, HDP_F32, false>(p->total, p->grid);
  else if (dst_dtype == HDP_F32) rc = plan_grid<HDP_DW_MERGE, HDP_F32, false>(p->total, p->grid);
  else rc = rnd ? plan_grid<HDP_DW_MERGE, HDP_BF16, true>(p->total, p->grid)
                : plan_grid<HDP_DW_MERGE, HDP_BF16, false>(p->total, p->grid);
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

extern "C" int hdp_delta_plan_run(hdp_delta_plan p, void* stream) {
  HDP_CHECK_ARG(p && p->d_items && p->grid > 0, "hdp_delta_plan_run: invalid plan");
  hipStream_t st = as_stream(stream);
  DeltaGroup g{p->d_items, p->d_start, p->n, p->total};
  dim3 grid((unsigned)p->grid), block(256);
#define HDP_LAUNCH(M, D, R) hipLaunchKernelGGL((delta_group_kernel<M, D, R>), grid, block, 0, st, g.items, g.tile_start, g.n, g.total)
#define HDP_LAUNCH_P(M, D, P) hipLaunchKernelGGL((delta_group_kernel<M, D, false, P>), grid, block, 0, st, g.items, g.tile_start, g.n, g.total)
  KTimer kt(p->multiseg ? K_DELTA_MULTI : K_DELTA, st, p->bytes, p->flops);
  if (p->mode == HDP_DW_STORE) {
    if (p->round) HDP_LAUNCH(HDP_DW_STORE, HDP_F32, true);
    else HDP_LAUNCH(HDP_DW_STORE, HDP_F32, false);
  } else if (p->dtype == HDP_F32) {
    switch (p->pol) {
      case 1: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 1); break;
      case 2: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 2); break;
      case 3: HDP_LAUNCH_P(HDP_DW_MERGE, HDP_F32, 3); break;
      default: HDP_LAUNCH(HDP_DW_MERGE, HDP_F32, false);
    }
  } else {
    if (p->round) HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, true);
    else HDP_LAUNCH(HDP_DW_MERGE, HDP_BF16, false);
  }
#undef HDP_LAUNCH
#undef HDP_LAUNCH_P
  HDP_CHECK_LAUNCH();
  return HDP_OK;
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
  delete p;
  if (rc != HDP_OK) set_error("hdp_delta_plan_destroy: hipFree failed");
  return rc;
}
