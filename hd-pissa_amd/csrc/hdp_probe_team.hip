// K2 TEAM path: the adapter probe backward reading X and G from HBM exactly once.
//
// Replaces the autograd of hp:139's adapter term (reference: hd_pissa.py:136-140):
//     A.grad += s (G B)^T X        B.grad += s G^T (X A^T),     s = alpha_eff * 1e-16
// Both products need a projection over the FULL row first (J = G B needs every column of G,
// H = X A^T every column of X), then an outer product over the same rows.  The sweep path
// (hdp_probe.hip) streams the smaller operand twice and round-trips stripe partials and pieces
// through HBM (X + G + min(X, G) bytes, six launches).  Here every column stripe of a module --
// X's and G's -- runs at the same time on its own workgroup (the module's TEAM), the team walks
// the rows in lock step, and the per-row projections are exchanged between the team's
// workgroups while each one still holds its rows in registers:
//
//   streaming wave (8 per workgroup, 64 columns each, 16-row steps):
//     LOAD  z(q)            rows 16 s + 4 p + (lane >> 4), 4 consecutive columns per lane
//     PROJ  q               partial 16 x rp of Z F^T over the wave's columns -> LDS, arrive
//     OUTER q - L           acc += Y_other(q - L)^T z(q - L), Y from the other side's granules
//     (z held in a ring of D register sets: loads run D - L steps ahead of PROJ)
//   publisher wave (4 per workgroup, step q handled by publisher q % 4):
//     sum the 8 waves' partials (fixed order) -> write-through store of the stripe partial ->
//     count the arrival on the (side, step) counter; the LAST stripe to arrive sums the nct
//     partials in stripe order (deterministic whoever is last), zeroes rows >= T and publishes
//     the 16 x rp projection as 8-byte {tag, value} granules (the data is the flag).
//   item end: g (+)= s * acc for the wave's 64 columns -- no pieces, no finish pass.
//
// HBM bytes per module: X + G once, the factors once, the gradients (+ the stripe partials,
// 16 rp floats per stripe and step, written through and read back once by the last arriver).
//
// Residency: a team only progresses with all its members running, so the launch is one
// workgroup per CU (grid = CU count; LDS and 12 waves admit exactly one) and the host packs
// the teams into ROUNDS of at most grid-size stripes (first-fit decreasing); workgroup w runs
// item (round k, slot w) for k = 0, 1, ...  All waits are bounded: a broken hand-off sets the
// error word (hdp_probe_team_errors) and the kernel drains with wrong numbers instead of
// hanging the GPU.
//
// Hand-off forms (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement & inter-workgroup
// visibility", valid-forms table row 1 and recipe R2): stripe partials are stored sc1 (buffer
// aux 16) by the one publishing wave, drained (s_waitcnt vmcnt(0)) before its agent-scope
// counter add; only the wave whose add returned last reads them, with sc1 loads; granules are
// single 8-byte sc1 stores / loads tagged with the launch generation (never 0), so no buffer
// needs clearing except the counters (one hipMemsetAsync per launch).
#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <vector>

#include "hdp_probe_int.h"

namespace hdp {

constexpr int kTmStream = kSwWaves;  // streaming waves (64 columns each)
constexpr int kTmPub = 4;            // publisher waves
constexpr int kTmThreads = (kTmStream + kTmPub) * 64;
constexpr int kTmMaxG = 1024;        // item-table width the per-module table budget allows
constexpr unsigned kTmSpinLimit = 1u << 22;  // bounded waits (~seconds): never hang the GPU

typedef unsigned long long u64;

struct alignas(16) TeamSide {
  const void* Z;        // T x N row-major, x dtype
  const float* F;       // f_rk: F[j][n] at j N + n (A, B^T); else F[n][j] at n r + j (B)
  float* g;             // gt = 0: gA [r][N];  gt = 1: gB [N][r]
  float* slab;          // [S][nct][16 rp] stripe partials (write-through)
  u64* yg;              // [S][16 rp] granules {tag, value}: this side's projection
  const u64* yo;        // the other side's
  int* cnt;             // [S] arrival counters (zeroed per launch)
  long long T, N;
  int r, f_rk, gt, nct, S, acc;
  float scale;
  int pad;
};

struct TeamArgs {
  const TeamSide* sides;  // [2 n] (device)
  const int* items;       // [rounds][G]: (side << 6) | stripe, -1 = no item
  int rounds, G;
  unsigned tag;           // launch generation (granule tag, never 0)
  int* err;               // error word (a bounded wait gave up)
  u64* trace;             // diagnosis (HDP_TM_TRACE=1): [G][tq][8] s_memrealtime stamps, else null
  int tq;
  int dbg;                // diagnosis only (HDP_TM_DBG, wrong numbers): 1 = no Y wait, 2 = no global publish,
                          // 4 = no OUTER re-read, 8 = no MFMAs
};

// trace events per (workgroup, step): stream wave 0 / publisher of the step
enum { kTrProj = 0, kTrOuterIn, kTrOuterGo, kTrPubIn, kTrPubStored, kTrPubCounted, kTrLastDone, kTrLastOld };
__device__ __forceinline__ void tm_stamp(const TeamArgs& ta, int w, int q, int ev, int lane, u64 v = 0) {
  if (ta.trace != nullptr && q < ta.tq && lane == 0)
    ta.trace[((size_t)w * ta.tq + q) * 8 + ev] = ev == kTrLastOld ? v : __builtin_amdgcn_s_memrealtime();
}

// a position in a workgroup's step stream: (round k, step s of that round's item)
struct TmCur {
  TeamSide d;  // register copy of the item's side (unused fields are dead per cursor role)
  int k, s, ct, S;
  int live;    // 0: past the end (d, ct, s still name the last step: its loads stay in bounds)
};

// This workgroup's items, copied to LDS at the start: cursors read them with LDS loads (lgkmcnt),
// so moving to the next item issues no vector-memory instruction -- a vector load on only some
// paths makes the compiler's vmcnt accounting fall back to vmcnt(0) and drains the load ring.
constexpr int kTmMaxRounds = 96;
struct TmLocal {
  TeamSide side[kTmMaxRounds];
  int ct[kTmMaxRounds];  // -1: no item in this round
};

__device__ __forceinline__ void tm_side(TeamSide& d, const TeamSide* src) {
  constexpr int NW = sizeof(TeamSide) / 16;
  static_assert(sizeof(TeamSide) % 16 == 0, "TeamSide is read as 16-byte words");
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4* p = reinterpret_cast<const i32x4*>(src);  // LDS
  int wds[4 * NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const i32x4 v = p[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) wds[4 * i + k] = __builtin_amdgcn_readfirstlane(v[k]);
  }
  __builtin_memcpy(&d, wds, sizeof(TeamSide));
}
__device__ __forceinline__ void tm_seek(TmCur& c, const TeamArgs& ta, const TmLocal* loc) {
  for (; c.k < ta.rounds; ++c.k) {
    const int ct = __builtin_amdgcn_readfirstlane(loc->ct[c.k]);
    if (ct >= 0) {
      tm_side(c.d, loc->side + c.k);
      c.ct = ct;
      c.s = 0;
      c.S = c.d.S;
      c.live = 1;
      return;
    }
  }
  c.live = 0;
  c.s = c.S - 1;  // the last step of the last item (valid addresses for the unconditional loads)
}
__device__ __forceinline__ void tm_next(TmCur& c, const TeamArgs& ta, const TmLocal* loc) {
  if (!c.live) return;
  if (++c.s < c.S) return;
  ++c.k;
  tm_seek(c, ta, loc);
}
__device__ __forceinline__ void tm_first(TmCur& c, const TeamArgs& ta, const TmLocal* loc) {
  c.k = 0;
  c.S = 1;
  tm_seek(c, ta, loc);
}

__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void tm_fail(const TeamArgs& ta, bool& broken, int lane) {
  if (!broken && lane == 0) __hip_atomic_store(gptr(ta.err), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  broken = true;
}

// ---------------------------------------------------------------------------------------
// streaming wave
// ---------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void tm_load(f32x4 (&z)[4], const TmCur& c, int wave, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const long long N = c.d.N, T = c.d.T;
  // unconditional (every path issues the same loads): an idle wave of a narrow last stripe and
  // a cursor past the end read clamped, in-bounds addresses
  long long col = (long long)c.ct * kSwC + 64 * wave + 4 * li;
  col = col < N ? col : N - 4;  // N % 4 == 0 (team path precondition)
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    long long row = 16LL * c.s + 4 * p + g;
    row = row < T ? row : T - 1;
    z[p] = load4<DT>(c.d.Z, row * N + col);
  }
}

// this wave's F fragments of the cursor's stripe: f[s][b] = F[j = 16 b + li][c + 16 s + 4 g + q]
template <int RB>
__device__ __forceinline__ void tm_load_f(f32x4 (&f)[4][RB], const TmCur& c, int wave, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const long long N = c.d.N;
  const long long c0 = (long long)c.ct * kSwC + 64 * wave;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      // F[j][n] rows (A, B^T: the team path takes B transposed), clamped in-bounds loads on every
      // lane and a select, so every path issues the same loads
      const int j = 16 * b + li;
      const long long k = c0 + 16 * s + 4 * g;
      const int jc = j < c.d.r ? j : c.d.r - 1;
      const long long kc = k < N ? k : N - 4;
      const f32x4 v = gld4(c.d.F + (long long)jc * N + kc);
      f[s][b] = (j < c.d.r && k < N) ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

// PROJ of step q: the 16 x rp partial of Z F^T over this wave's columns into LDS buffer q % NB
template <int RB, int NB>
__device__ __forceinline__ void tm_proj(const f32x4 (&z)[4], const f32x4 (&f)[4][RB], bool active, int q, float* tile,
                                        float* red, int* arrive, int* done, int wave, int lane, const TeamArgs& ta,
                                        bool& broken) {
  constexpr int rp = 16 * RB;
  const int li = lane & 15, g = lane >> 4;
  f32x4 a0[RB], a1[RB];
#pragma unroll
  for (int b = 0; b < RB; ++b) a0[b] = a1[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (active && !(ta.dbg & 8)) {
    // rows 4 p + g / columns 4 li + q as loaded -> MFMA A-operand fragments (row li) via a
    // wave-private padded tile (conflict-free 16-B writes and reads)
#pragma unroll
    for (int p = 0; p < 4; ++p) *reinterpret_cast<f32x4*>(tile + (4 * p + g) * kTileLd + 4 * li) = z[p];
#pragma unroll
    for (int ss = 0; ss < 4; ++ss) {
      const f32x4 zf = *reinterpret_cast<const f32x4*>(tile + li * kTileLd + 16 * ss + 4 * g);
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (ss & 1) a1[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[qq], f[ss][b][qq], a1[b], 0, 0, 0);
          else a0[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[qq], f[ss][b][qq], a0[b], 0, 0, 0);
        }
    }
  }
  const int b = q % NB, rnd = q / NB;
  if (rnd > 0 && !broken) {  // the publisher has read this buffer's previous round
    for (unsigned it = 0; lds_ld(done + b) < rnd;) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > kTmSpinLimit) {
        tm_fail(ta, broken, lane);
        break;
      }
    }
    asm volatile("" ::: "memory");
  }
  float* rb = red + (b * kTmStream + wave) * 16 * rp;
  // lane holds rows 4 g + reg, column j = 16 bb + li
#pragma unroll
  for (int bb = 0; bb < RB; ++bb)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) rb[(4 * g + reg) * rp + 16 * bb + li] = a0[bb][reg] + a1[bb][reg];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add(arrive + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the other side's projection of step c.s as granules: yv[p][b] = Y[(4 p + g) rp + 16 b + li]
template <int RB>
__device__ __forceinline__ void tm_yload(u64 (&yv)[4][RB], const TmCur& c, int lane) {
  constexpr int rp = 16 * RB;
  const int li = lane & 15, g = lane >> 4;
  const HDP_GLOBAL u64* src = gptr(c.d.yo + (long long)c.s * 16 * rp);
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int b = 0; b < RB; ++b)
      yv[p][b] = __hip_atomic_load(src + (4 * p + g) * rp + 16 * b + li, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int RB>
__device__ __forceinline__ bool tm_yready(const u64 (&yv)[4][RB], unsigned tag) {
  bool ok = true;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int b = 0; b < RB; ++b) ok = ok && (unsigned)(yv[p][b] >> 32) == tag;
  return __all(ok);
}

template <int RB>
__device__ __forceinline__ void tm_outer(const f32x4 (&z)[4], f32x4 (&acc)[RB][4], u64 (&yv)[4][RB], bool active,
                                         const TmCur& c, int lane, const TeamArgs& ta, bool& broken) {
  if (!active) return;
  if (!broken && !(ta.dbg & 1) && !tm_yready<RB>(yv, ta.tag)) {
    for (unsigned it = 0;;) {
      __builtin_amdgcn_s_sleep(2);
      tm_yload<RB>(yv, c, lane);
      if (tm_yready<RB>(yv, ta.tag)) break;
      if (++it > kTmSpinLimit) {
        tm_fail(ta, broken, lane);
        break;
      }
    }
  }
  if (ta.dbg & 8) return;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      const float y = __uint_as_float((unsigned)yv[p][b]);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(y, z[p][q], acc[b][q], 0, 0, 0);
    }
}

// item end: g (+)= s * acc for this wave's 64 columns; lane holds D[j = 16 b + 4 g + reg][n = col + q]
template <int RB>
__device__ __forceinline__ void tm_store_g(f32x4 (&acc)[RB][4], const TmCur& c, int wave, int lane) {
#pragma clang fp contract(off)  // g + s*sum as two roundings, like autograd's mul then add
  const int li = lane & 15, g = lane >> 4;
  const long long N = c.d.N;
  const long long col = (long long)c.ct * kSwC + 64 * wave + 4 * li;
  const float sc = c.d.scale;
  const int r = c.d.r;
  if (col < N) {
    if (c.d.gt == 0) {  // gA [r][N]
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int j = 16 * b + 4 * g + reg;
          if (j < r) {
            float* p = c.d.g + (long long)j * N + col;
            const f32x4 v{sc * acc[b][0][reg], sc * acc[b][1][reg], sc * acc[b][2][reg], sc * acc[b][3][reg]};
            gst4(p, c.d.acc ? gld4(p) + v : v);
          }
        }
    } else {  // gB [N][r]
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j0 = 16 * b + 4 * g;
          float* p = c.d.g + (col + q) * r + j0;
          const f32x4 v = sc * acc[b][q];
          if (r % 4 == 0 && j0 + 3 < r) {
            gst4(p, c.d.acc ? gld4(p) + v : v);
          } else {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg)
              if (j0 + reg < r) gst1(p + reg, c.d.acc ? gld1(p + reg) + v[reg] : v[reg]);
          }
        }
    }
  }
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// The streaming loop.  PROJ reads step q from HBM (loads DP - 1 steps ahead, ring zp); OUTER
// runs L steps behind and RE-READS its 16 rows (ring zo, DO - 1 steps ahead, non-temporal: the
// last use): between the two reads the chip streams about L x 32 KB x CUs (L = 8: 64 MB), so the
// re-read is an Infinity Cache hit and HBM still moves X and G once, while the exchange of a
// step's projection (team skew + publish + last-arriver reduce, ~5-10 us under load) is hidden
// behind L steps without holding L steps of rows in registers.
template <int DT>
__device__ __forceinline__ void tm_load_nt(f32x4 (&z)[4], const TmCur& c, int wave, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const long long N = c.d.N, T = c.d.T;
  long long col = (long long)c.ct * kSwC + 64 * wave + 4 * li;
  col = col < N ? col : N - 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    long long row = 16LL * c.s + 4 * p + g;
    row = row < T ? row : T - 1;
    z[p] = load4_nt<DT>(c.d.Z, row * N + col);
  }
}

template <int DT, int RB, int NB, int DP, int DO, int L>
__device__ __forceinline__ void tm_stream(const TeamArgs& ta, const TmLocal* loc, int wave, int lane, float* tile,
                                          float* red, int* arrive, int* done) {
  static_assert(DP >= 2 && DO >= 2 && L >= DO, "rings: PROJ DP sets, OUTER DO sets, OUTER L >= DO steps behind");
  constexpr int U = DP * DO / (DP % DO == 0 ? DO : DO % DP == 0 ? DP : 1);  // lcm (small rings)
  TmCur cl, cp, co, clo;  // PROJ loads, PROJ, OUTER, OUTER loads
  tm_first(cl, ta, loc);
  if (!cl.live) return;
  cp = cl;
  co = cl;
  clo = cl;
  bool broken = false;
  f32x4 zp[DP][4], zo[DO][4];
  f32x4 f[4][RB];
  f32x4 acc[RB][4];
  u64 yv[4][RB];
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < DP - 1; ++i) {
    tm_load<DT>(zp[i], cl, wave, lane);
    tm_next(cl, ta, loc);
  }
  int qp = 0;
  // Steady state: every iteration issues the same vector loads in the same order (PROJ data,
  // OUTER re-read, the next OUTER's granules) whatever the cursors' states, so the compiler
  // counts them exactly and waits for each with vmcnt(n) instead of draining the rings.
  for (int base = 0;; base += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u;
      tm_load<DT>(zp[(u + DP - 1) % DP], cl, wave, lane);  // PROJ data DP - 1 steps ahead
      tm_next(cl, ta, loc);
      if (cp.live) {
        if (cp.s == 0) tm_load_f<RB>(f, cp, wave, lane);
        const bool act = (long long)cp.ct * kSwC + 64 * wave < cp.d.N;
        tm_proj<RB, NB>(zp[u % DP], f, act, qp, tile, red, arrive, done, wave, lane, ta, broken);
        if (wave == 0) tm_stamp(ta, blockIdx.x, qp, kTrProj, lane);
        tm_next(cp, ta, loc);
        ++qp;
      }
      // OUTER re-reads DO - 1 steps ahead of OUTER (OUTER(q) runs at iteration q + L)
      tm_load_nt<DT>(zo[(u + 2 * DO - 1 - L % DO) % DO], clo, wave, lane);  // (i - L + DO - 1) % DO, base % DO == 0
      if (i >= L - (DO - 1)) tm_next(clo, ta, loc);
      if (i >= L) {
        if (co.live) {
          const bool act = (long long)co.ct * kSwC + 64 * wave < co.d.N;
          const int qo = i - L;
          if (wave == 0) tm_stamp(ta, blockIdx.x, qo, kTrOuterIn, lane);
          tm_outer<RB>(zo[(u + DO - L % DO) % DO], acc, yv, act, co, lane, ta, broken);  // qo % DO
          if (wave == 0) tm_stamp(ta, blockIdx.x, qo, kTrOuterGo, lane);
          if (co.s == co.S - 1) tm_store_g<RB>(acc, co, wave, lane);
          tm_next(co, ta, loc);
        }
        if (!co.live) return;
      }
      if (i >= L - 1) tm_yload<RB>(yv, co, lane);  // the next OUTER's projection
    }
  }
}

// HOLD variant: OUTER uses the rows PROJ loaded, kept in a ring of D register sets (loads D - L
// steps ahead of PROJ, OUTER L steps behind): X and G are delivered to the CUs exactly once, and
// the exchange latency must fit in L steps.
template <int DT, int RB, int NB, int D, int L>
__device__ __forceinline__ void tm_stream_hold(const TeamArgs& ta, const TmLocal* loc, int wave, int lane, float* tile,
                                               float* red, int* arrive, int* done) {
  static_assert(D > L && L >= 1, "ring: D register sets, OUTER L steps behind PROJ");
  TmCur cl, cp, co;
  tm_first(cl, ta, loc);
  if (!cl.live) return;
  cp = cl;
  co = cl;
  bool broken = false;
  f32x4 z[D][4];
  f32x4 f[4][RB];
  f32x4 acc[RB][4];
  u64 yv[4][RB];
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < D - L; ++i) {
    tm_load<DT>(z[i], cl, wave, lane);
    tm_next(cl, ta, loc);
  }
  int qp = 0;
  for (int base = 0;; base += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int i = base + u;
      if (cp.live) {
        if (cp.s == 0) tm_load_f<RB>(f, cp, wave, lane);
        const bool act = (long long)cp.ct * kSwC + 64 * wave < cp.d.N;
        tm_proj<RB, NB>(z[u], f, act, qp, tile, red, arrive, done, wave, lane, ta, broken);
        if (wave == 0) tm_stamp(ta, blockIdx.x, qp, kTrProj, lane);
        tm_next(cp, ta, loc);
        ++qp;
      }
      if (i >= L) {
        if (co.live) {
          const bool act = (long long)co.ct * kSwC + 64 * wave < co.d.N;
          const int qo = i - L;
          if (wave == 0) tm_stamp(ta, blockIdx.x, qo, kTrOuterIn, lane);
          tm_outer<RB>(z[(u - L % D + D) % D], acc, yv, act, co, lane, ta, broken);
          if (wave == 0) tm_stamp(ta, blockIdx.x, qo, kTrOuterGo, lane);
          if (co.s == co.S - 1) tm_store_g<RB>(acc, co, wave, lane);
          tm_next(co, ta, loc);
        }
        if (!co.live) return;
      }
      // the slot OUTER(i - L) freed takes step i - L + D
      tm_load<DT>(z[(u - L % D + D) % D], cl, wave, lane);
      tm_next(cl, ta, loc);
      if (i >= L - 1) tm_yload<RB>(yv, co, lane);  // the next OUTER's projection
    }
  }
}

// ---------------------------------------------------------------------------------------
// publisher wave e: steps q = e, e + kTmPub, ...
// ---------------------------------------------------------------------------------------
template <int RB, int NB>
__device__ __forceinline__ void tm_publish(const TeamArgs& ta, const TmLocal* loc, int e, int lane, const float* red,
                                           int* arrive, int* done) {
  const int w = blockIdx.x;
  constexpr int rp = 16 * RB, E = 16 * rp, V = E / 256;
  TmCur c;
  tm_first(c, ta, loc);
  for (int i = 0; i < e && c.live; ++i) tm_next(c, ta, loc);
  bool broken = false;
  for (int q = e; c.live; q += kTmPub) {
    const int b = q % NB, rnd = q / NB;
    if (!broken) {
      for (unsigned it = 0; lds_ld(arrive + b) < kTmStream * (rnd + 1);) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > kTmSpinLimit) {
          tm_fail(ta, broken, lane);
          break;
        }
      }
      asm volatile("" ::: "memory");
    }
    tm_stamp(ta, w, q, kTrPubIn, lane);
    // the 8 waves' partials in wave order (deterministic)
    f32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ww = 0; ww < kTmStream; ++ww)
        v[i] += *reinterpret_cast<const f32x4*>(red + (b * kTmStream + ww) * E + 256 * i + 4 * lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(done + b, rnd + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (ta.dbg & 2) {
      for (int i = 0; i < kTmPub && c.live; ++i) tm_next(c, ta, loc);
      continue;
    }
    // write-through store of this stripe's partial, drained, then the arrival
    const int nct = c.d.nct;
    float* sbase = c.d.slab + (long long)c.s * nct * E;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(sbase, 0, nct * E * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      u32x4 bits;
#pragma unroll
      for (int k = 0; k < 4; ++k) bits[k] = __float_as_uint(v[i][k]);
      __builtin_amdgcn_raw_buffer_store_b128(bits, rs, (c.ct * E + 256 * i + 4 * lane) * 4, 0, 16 /* sc1 */);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tm_stamp(ta, w, q, kTrPubStored, lane);
    int old = 0;
    if (lane == 0)
      old = __hip_atomic_fetch_add(gptr(c.d.cnt + c.s), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __builtin_amdgcn_readfirstlane(old);
    tm_stamp(ta, w, q, kTrPubCounted, lane);
    tm_stamp(ta, w, q, kTrLastOld, lane, (u64)old);
    if (old == nct - 1) {
      // last stripe of (side, step): sum every stripe's partial in stripe order
      f32x4 sum[V];
#pragma unroll
      for (int i = 0; i < V; ++i) sum[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int c0 = 0; c0 < nct; c0 += 16) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 ld[16][V];
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int i = 0; i < V; ++i)
            ld[u][i] = c0 + u < nct ? __builtin_amdgcn_raw_buffer_load_b128(rs, ((c0 + u) * E + 256 * i + 4 * lane) * 4, 0, 16)
                                    : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int i = 0; i < V; ++i)
            if (c0 + u < nct)
#pragma unroll
              for (int k = 0; k < 4; ++k) sum[i][k] += __uint_as_float(ld[u][i][k]);
      }
      HDP_GLOBAL u64* dst = gptr(c.d.yg + (long long)c.s * E);
      const u64 tg = (u64)ta.tag << 32;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int e0 = 256 * i + 4 * lane;
        const bool live = 16LL * c.s + e0 / rp < c.d.T;  // rows past T contribute nothing
#pragma unroll
        for (int k = 0; k < 4; ++k)
          __hip_atomic_store(dst + e0 + k, tg | (live ? __float_as_uint(sum[i][k]) : 0u), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      tm_stamp(ta, w, q, kTrLastDone, lane);
    }
    for (int i = 0; i < kTmPub && c.live; ++i) tm_next(c, ta, loc);
  }
}

template <int DT, int RB, int NB, int DP, int DO, int L, int HOLD = 0>
__global__ __launch_bounds__(kTmThreads) void probe_team_kernel(TeamArgs ta) {
  // LDS: [tiles 8 x 16 x kTileLd][red NB x 8 x 16 rp][arrive NB][done NB]
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int rp = 16 * RB;
  TmLocal* loc = reinterpret_cast<TmLocal*>(lds);
  float* tiles = lds + sizeof(TmLocal) / sizeof(float);
  float* red = tiles + kTmStream * 16 * kTileLd;
  int* arrive = reinterpret_cast<int*>(red + NB * kTmStream * 16 * rp);
  int* done = arrive + NB;
  const int w = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < 2 * NB) arrive[threadIdx.x] = 0;
  // this workgroup's item of every round: stripe index and side descriptor (host tables, read once)
  for (int k = threadIdx.x; k < ta.rounds; k += kTmThreads) {
    const int it = *gptr(ta.items + k * ta.G + w);
    loc->ct[k] = it < 0 ? -1 : (it & 63);
    if (it >= 0) {
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      const HDP_GLOBAL i32x4* src = reinterpret_cast<const HDP_GLOBAL i32x4*>(gptr(ta.sides + (it >> 6)));
      i32x4* dst = reinterpret_cast<i32x4*>(loc->side + k);
#pragma unroll
      for (int i = 0; i < (int)(sizeof(TeamSide) / 16); ++i) dst[i] = src[i];
    }
  }
  __syncthreads();
  if (wave < kTmStream) {
    if constexpr (HOLD > 0)
      tm_stream_hold<DT, RB, NB, HOLD, L>(ta, loc, wave, lane, tiles + wave * 16 * kTileLd, red, arrive, done);
    else
      tm_stream<DT, RB, NB, DP, DO, L>(ta, loc, wave, lane, tiles + wave * 16 * kTileLd, red, arrive, done);
  }
  if (wave >= kTmStream) tm_publish<RB, NB>(ta, loc, wave - kTmStream, lane, red, arrive, done);
}

// ---------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------
template <int RB>
constexpr int tm_nb() { return RB == 1 ? 8 : 4; }
template <int RB>
constexpr size_t tm_lds() {
  return sizeof(TmLocal) +
         ((size_t)kTmStream * 16 * kTileLd + (size_t)tm_nb<RB>() * kTmStream * 16 * 16 * RB) * sizeof(float) +
         2 * tm_nb<RB>() * sizeof(int);
}

size_t team_table_per_module() { return 2 * sizeof(TeamSide) + kTmMaxG * sizeof(int); }

size_t team_table_bytes(int n) {
  const size_t sides = (2 * (size_t)n * sizeof(TeamSide) + 255) / 256 * 256;
  return sides + (size_t)n * kTmMaxG * sizeof(int);
}

int team_grid() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cached[dev] = cus < kTmMaxG ? cus : kTmMaxG;
  }
  return cached[dev];
}

bool team_fits(const HostGroup& ga) {
  if (ga.RB > 2) return false;
  const int G = team_grid();
  for (const ProbeDesc& d : ga.d) {
    if (d.in % 4 || d.out % 4 || !d.b_t) return false;
    const int nx = (int)((d.in + kSwC - 1) / kSwC), ng = (int)((d.out + kSwC - 1) / kSwC);
    if (nx > 64 || ng > 64 || nx + ng > G) return false;
    if (d.T * (d.in > d.out ? d.in : d.out) >= (1ll << 40)) return false;
  }
  return true;
}

static u64* g_trace = nullptr;
static const int kTraceQ = 2048;
static bool trace_on() {
  static const bool v = [] { const char* e = getenv("HDP_TM_TRACE"); return e && e[0] == '1'; }();
  return v;
}
static int* g_err = nullptr;
static std::mutex g_err_mu;
static std::atomic<unsigned> g_tag{0};

int team_errors(int clear) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  if (!g_err) return 0;
  int v = 0;
  if (hipMemcpy(&v, g_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (clear && v) (void)hipMemset(g_err, 0, sizeof(int));
  return v;
}

static int* err_word() {
  std::lock_guard<std::mutex> lk(g_err_mu);
  if (!g_err) {
    if (hipMalloc(&g_err, sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(g_err, 0, sizeof(int)) != hipSuccess) return nullptr;
  }
  return g_err;
}

template <int DT, int RB>
static int launch_team_t(const HostGroup& ga, char* tab, int* cnt, size_t cnt_bytes, hipStream_t st) {
  constexpr int rp = 16 * RB, NB = tm_nb<RB>();
#ifndef HDP_TM_DP
#define HDP_TM_DP 3
#define HDP_TM_DO 2
#define HDP_TM_L 12
#endif
  constexpr int DP = HDP_TM_DP, DO = HDP_TM_DO, L = HDP_TM_L;
  const int n = ga.n, G = team_grid();
  std::vector<TeamSide> sides(2 * n);
  std::vector<int> team(n);
  int* cnt_at = cnt;
  double xg = 0, fac = 0, grads = 0, slab = 0, flop = 0;
  const double es = DT == HDP_F32 ? 4 : 2;
  for (int i = 0; i < n; ++i) {
    const ProbeDesc& p = ga.d[i];
    const int S = (int)((p.T + 15) / 16);
    const int nx = (int)((p.in + kSwC - 1) / kSwC), ng = (int)((p.out + kSwC - 1) / kSwC);
    u64* gx = reinterpret_cast<u64*>(p.yH);
    u64* gg = reinterpret_cast<u64*>(p.yJ);
    // X side: PROJ with A (r x in) -> H; OUTER with J -> gA.  G side: PROJ with B -> J; OUTER with H -> gB
    sides[2 * i] = TeamSide{p.X, p.A, p.gA, p.slabH, gx, gg, cnt_at, p.T, p.in, p.r, 1, 0, nx, S, p.accumulate, p.scale, 0};
    sides[2 * i + 1] = TeamSide{p.G, p.B, p.gB, p.slabJ, gg, gx, cnt_at + S, p.T, p.out, p.r, p.b_t, 1, ng, S,
                                p.accumulate, p.scale, 0};
    cnt_at += 2 * S;
    team[i] = nx + ng;
    xg += es * p.T * (p.in + p.out);
    fac += 4.0 * p.r * (p.in + p.out);
    grads += 4.0 * p.r * (p.in + p.out) * (p.accumulate ? 2 : 1);
    slab += 2.0 * 4.0 * 16 * rp * (double)S * (nx + ng);
    flop += 4.0 * p.T * p.r * (p.in + p.out);
  }
  HDP_CHECK_ARG((size_t)(cnt_at - cnt) * sizeof(int) <= cnt_bytes, "probe team: counter block too small");
  // rounds: first-fit decreasing of the teams into rounds of G stripes
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return team[a] > team[b]; });
  std::vector<int> used;
  std::vector<std::vector<int>> rmods;
  for (int i : order) {
    size_t k = 0;
    while (k < used.size() && used[k] + team[i] > G) ++k;
    if (k == used.size()) {
      used.push_back(0);
      rmods.emplace_back();
    }
    used[k] += team[i];
    rmods[k].push_back(i);
  }
  const int rounds = (int)used.size();
  HDP_CHECK_ARG(rounds <= n, "probe team: more rounds than modules");
  // table blob: [sides | items[rounds][G]]
  const size_t o_items = (2 * (size_t)n * sizeof(TeamSide) + 255) / 256 * 256;
  std::vector<char> blob(o_items + (size_t)rounds * G * sizeof(int));
  memcpy(blob.data(), sides.data(), 2 * (size_t)n * sizeof(TeamSide));
  int* items = reinterpret_cast<int*>(blob.data() + o_items);
  for (int k = 0; k < rounds; ++k) {
    int slot = 0;
    for (int i : rmods[k]) {
      for (int sd = 0; sd < 2; ++sd)
        for (int ct = 0; ct < sides[2 * i + sd].nct; ++ct) items[k * G + slot++] = ((2 * i + sd) << 6) | ct;
    }
    for (; slot < G; ++slot) items[k * G + slot] = -1;
  }
  int rc = probe_tables_upload(blob, tab, st);
  if (rc) return rc;
  HDP_CHECK_HIP(hipMemsetAsync(cnt, 0, (size_t)(cnt_at - cnt) * sizeof(int), st));
  int* err = err_word();
  HDP_CHECK_ARG(err != nullptr, "probe team: error word allocation failed");
  unsigned tag = ++g_tag;
  if (tag == 0) tag = ++g_tag;
  u64* trace = nullptr;
  if (trace_on()) {
    if (!g_trace) HDP_CHECK_HIP(hipMalloc(&g_trace, (size_t)kTmMaxG * kTraceQ * 8 * sizeof(u64)));
    HDP_CHECK_HIP(hipMemsetAsync(g_trace, 0, (size_t)G * kTraceQ * 8 * sizeof(u64), st));
    trace = g_trace;
  }
  static const int dbg = [] { const char* e = getenv("HDP_TM_DBG"); return e ? atoi(e) : 0; }();
  // OUTER lag (steps): HDP_TM_L = 6 / 8 for experiments (12 measured best of the three)
  static const int lag = [] { const char* e = getenv("HDP_TM_L"); return e ? atoi(e) : L; }();
  // one launch per kTmMaxRounds rounds (a workgroup's item list lives in LDS)
  for (int k0 = 0; k0 < rounds; k0 += kTmMaxRounds) {
    const int nr = rounds - k0 < kTmMaxRounds ? rounds - k0 : kTmMaxRounds;
    TeamArgs ta{reinterpret_cast<const TeamSide*>(tab), reinterpret_cast<const int*>(tab + o_items) + (size_t)k0 * G, nr,
                G, tag, err, trace, kTraceQ, dbg};
    KTimer kt(K_PROBE_TEAM, st, k0 == 0 ? xg + fac + grads : 0.0, k0 == 0 ? flop : 0.0);
    static const int hold = [] { const char* e = getenv("HDP_TM_HOLD"); return e ? atoi(e) : 0; }();
    if (RB == 1 && hold == 64)
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, 4, 6>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
    else if (RB == 1 && hold == 63)
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, 3, 6>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
    else if (RB == 1 && hold == 53)
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, 3, 5>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
    else if (RB == 1 && lag == 6)
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, 6>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
    else if (RB == 1 && lag == 8)
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, 8>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
    else
      hipLaunchKernelGGL((probe_team_kernel<DT, RB, NB, DP, DO, L>), dim3(G), dim3(kTmThreads), tm_lds<RB>(), st, ta);
  }
  HDP_CHECK_LAUNCH();
  (void)slab;
  return HDP_OK;
}

int launch_team(const HostGroup& ga, int x_dtype, char* tab, int* cnt, size_t cnt_bytes, hipStream_t st) {
  if (x_dtype == HDP_F32) return ga.RB == 1 ? launch_team_t<HDP_F32, 1>(ga, tab, cnt, cnt_bytes, st)
                                            : launch_team_t<HDP_F32, 2>(ga, tab, cnt, cnt_bytes, st);
  return ga.RB == 1 ? launch_team_t<HDP_BF16, 1>(ga, tab, cnt, cnt_bytes, st)
                    : launch_team_t<HDP_BF16, 2>(ga, tab, cnt, cnt_bytes, st);
}

}  // namespace hdp

extern "C" int hdp_probe_team_errors(int clear) { return hdp::team_errors(clear); }

extern "C" int64_t hdp_probe_team_trace(void* host, int64_t bytes) {
  if (!hdp::g_trace) return 0;
  const int64_t all = (int64_t)hdp::team_grid() * hdp::kTraceQ * 8 * sizeof(hdp::u64);
  const int64_t n = bytes < all ? bytes : all;
  if (host && n > 0 && hipMemcpy(host, hdp::g_trace, n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return all;
}
