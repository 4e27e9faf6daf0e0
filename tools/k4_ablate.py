"""K4 bf16 H2 ablation builds (measurement tool, not part of the library): variants of
delta_h2_kernel with one part of its work removed, each linked into tools/abl/libhdpissa_<v>.so
(load with HDPISSA_LIB=...; results are WRONG by construction -- timing only).
  nomfma : the 3 MFMAs per block -> one VALU FMA (LDS fragment reads kept)
  nodma  : no global->LDS staging (ring waits and barriers kept)
  now    : the deferred W read-modify-write dropped (loads of one hot line, no stores)
  nobar  : no per-chunk workgroup barrier (ring reuse races: garbage, timing only)
  nolds  : MFMA fragments from registers instead of LDS (the fragment reads dropped)
  w16    : the deferred W read-modify-write as 8 x 16-B per lane over full 128-B rows (8 rows per
           instruction) instead of 16 x 8 B (data placement wrong: timing only)
  f16b   : float32 merges (WPrefetch / epilogue full path) with 16-B W loads and stores over 8 rows x
           128 B per instruction instead of 4 B per lane (data placement wrong: timing only)
  now32  : the float32 deferred merge's W read-modify-write (X3WDefer pieces) dropped: loads of one hot
           line, no stores (timing only)
  stagN  : (a candidate, results exact) workgroup start staggered by (slot % 8) x N x 64 cycles, so
           the persistent workgroups' W read-modify-write bursts do not coincide
usage: python tools/k4_ablate.py [variant ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hd-pissa_amd")
OUT = os.path.join(ROOT, "tools", "abl")


def variant(src, v):
    def rep(old, new, cnt=None):
        nonlocal src
        n = src.count(old)
        assert n >= 1 and (cnt is None or n == cnt), (v, old[:60], n)
        src = src.replace(old, new)
    if v == "nomfma":
        for a, b in (("fa[bo][1], fb[bc][0]", "lo * hi"), ("fa[bo][0], fb[bc][1]", "hi * lo"), ("fa[bo][0], fb[bc][0]", "hi * hi")):
            rep(f"d = __builtin_amdgcn_mfma_f32_32x32x16_f16({a}, d, 0, 0, 0);  // {b}",
                f"d[0] += (float){a.split(', ')[0]}[0] * (float){a.split(', ')[1]}[1];")
    elif v == "nodma":
        rep("""        __builtin_amdgcn_global_load_lds(reinterpret_cast<const HDP_GLOBAL void*>(gptr(L.src + j * 1024 + lane * 16)),
                                         (__attribute__((address_space(3))) void*)(dst + j * 256), 16, 0, 0);""",
            """        asm volatile("" :: "v"(dst + j * 256), "s"(L.src));""")
    elif v == "now":
        rep("""    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(w[g]) : "v"(voff), "s"(rs4), "s"(bgrp_soff(sbase, rowb, g)) : "memory");""",
            """    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(w[g]) : "v"(0), "s"(rs4), "s"(0) : "memory");""")
        rep("""    __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, bgrp_soff(sbase, rowb, g), 0);""",
            """    asm volatile("" :: "v"(v));""")
    elif v == "nobar":
        rep("""    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();
    issue(i % NB);""", """    issue(i % NB);""")
    elif v == "nolds":
        rep("""      fa[i][p] = *reinterpret_cast<const f16x8*>(Lb + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
      fb[i][p] = *reinterpret_cast<const f16x8*>(Rb + p * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));""",
            """      for (int e = 0; e < 8; ++e) {
        fa[i][p][e] = (_Float16)(xa + p + e);
        fb[i][p][e] = (_Float16)(xb - p + e);
      }
      asm volatile("" : "+v"(fa[i][p]), "+v"(fb[i][p]));""")
    elif v == "w16":
        rep("""#pragma unroll
  for (int g = 0; g < 16; ++g)
    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(w[g]) : "v"(voff), "s"(rs4), "s"(bgrp_soff(sbase, rowb, g)) : "memory");""",
            """  const int v16 = (int)((threadIdx.x & 63) >> 3) * rowb + 16 * (int)(threadIdx.x & 7);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    i32x4 t;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(t) : "v"(v16), "s"(rs4), "s"(sbase + 8 * g * rowb) : "memory");
    w[2 * g] = u32x2{(uint32_t)t[0], (uint32_t)t[1]};
    w[2 * g + 1] = u32x2{(uint32_t)t[2], (uint32_t)t[3]};
  }""")
        rep("""#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const u32x2 v{badd2(w[g][0], d[g][0]), badd2(w[g][1], d[g][1])};
    __builtin_amdgcn_raw_buffer_store_b64(v, rs, voff, bgrp_soff(sbase, rowb, g), 0);
  }""", """  const int v16 = (int)((threadIdx.x & 63) >> 3) * rowb + 16 * (int)(threadIdx.x & 7);
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const i32x4 v{(int)badd2(w[2 * g][0], d[2 * g][0]), (int)badd2(w[2 * g][1], d[2 * g][1]),
                  (int)badd2(w[2 * g + 1][0], d[2 * g + 1][0]), (int)badd2(w[2 * g + 1][1], d[2 * g + 1][1])};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, v16, sbase + 8 * g * rowb, 0);
  }""")
        src = src.replace('asm volatile("s_waitcnt vmcnt(24)" ::: "memory");', 'asm volatile("s_waitcnt vmcnt(16)" ::: "memory");')
    elif v == "f16b":
        rep("""            w[bo][bc][e] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(t.rs, t.voff, reg_soff<4>(t, bo, bc, e), w_load_aux(POL)));""",
            """          {
            typedef uint32_t abl_u4 __attribute__((ext_vector_type(4)));
            if ((e & 3) == 0) {
              const int l = (int)(threadIdx.x & 63), v16 = (4 * (l >> 5) + (l & 3)) * t.rowb + 16 * ((l & 31) >> 2);
              const abl_u4 q = __builtin_amdgcn_raw_buffer_load_b128(t.rs, v16, t.sbase + (8 * (e >> 2) + 32 * bo) * t.rowb + 128 * bc, w_load_aux(POL));
              w[bo][bc][e] = __uint_as_float(q[0]);
              w[bo][bc][(e + 1) & 15] = __uint_as_float(q[1]);
              w[bo][bc][(e + 2) & 15] = __uint_as_float(q[2]);
              w[bo][bc][(e + 3) & 15] = __uint_as_float(q[3]);
            }
          }""")
        rep("""            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(wpf.w[bo][bc][e] + val), t.rs, t.voff,
                                                  reg_soff<4>(t, bo, bc, e), w_store_aux(POL));""",
            """            typedef uint32_t abl_u4 __attribute__((ext_vector_type(4)));
            if ((e & 3) == 0) {
              const int v16 = (4 * h + (l32 & 3)) * t.rowb + 16 * (l32 >> 2);
              const float v1 = NEG ? -run[bo][bc][(e + 1) & 15] : run[bo][bc][(e + 1) & 15];
              const float v2 = NEG ? -run[bo][bc][(e + 2) & 15] : run[bo][bc][(e + 2) & 15];
              const float v3 = NEG ? -run[bo][bc][(e + 3) & 15] : run[bo][bc][(e + 3) & 15];
              const abl_u4 q{__float_as_uint(wpf.w[bo][bc][e] + val), __float_as_uint(wpf.w[bo][bc][(e + 1) & 15] + v1),
                             __float_as_uint(wpf.w[bo][bc][(e + 2) & 15] + v2), __float_as_uint(wpf.w[bo][bc][(e + 3) & 15] + v3)};
              __builtin_amdgcn_raw_buffer_store_b128(q, t.rs, v16, t.sbase + (8 * (e >> 2) + 32 * bo) * t.rowb + 128 * bc, w_store_aux(POL));
            }""")
    elif v == "now32":
        rep("""        asm volatile("buffer_load_dword %0, %1, %2, %3 offen nt" : "=v"(w[8 * q + e]) : "v"(t.voff), "s"(rs4), "s"(so) : "memory");
      else
        asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(w[8 * q + e]) : "v"(t.voff), "s"(rs4), "s"(so) : "memory");""",
            """        asm volatile("buffer_load_dword %0, %1, %2, %3 offen nt" : "=v"(w[8 * q + e]) : "v"(0), "s"(rs4), "s"(0) : "memory");
      else
        asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(w[8 * q + e]) : "v"(0), "s"(rs4), "s"(0) : "memory");""")
        rep("""      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w[8 * q + e] + val), t.rs, t.voff,
                                            reg_soff<4>(t, bo, bc, e0 + e), w_store_aux(POL));""",
            """      asm volatile("" :: "v"(w[8 * q + e] + val));""")
    elif v in ("pref", "prio", "prefprio"):
        # candidates (results exact): pref = a chunk's 16 fragments read before its 24 MFMAs (sub-image 1's
        # LDS latency hidden under sub-image 0's MFMAs); prio = s_setprio 1 for waves 4-7 (the second half
        # of every SIMD pair, MI355X_MICROARCH.md "Two waves per SIMD" item 4)
        if v in ("pref", "prefprio"):
            rep("""  auto mfma_chunk = [&]() {
    const _Float16* b = reinterpret_cast<const _Float16*>(smem + (i % NB) * kH2Buf);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const _Float16* sb = b + sub * 12288;  // 24 KB sub-image = 12288 fp16
      h2_mfma(sb + (ow >> 7) * 4096, sb + 8192, h, l32, ow & (kDT - 1), cw, acc);
    }
  };""", """  auto mfma_chunk = [&]() {
    const _Float16* b = reinterpret_cast<const _Float16*>(smem + (i % NB) * kH2Buf);
    f16x8 fa[2][2][2], fb[2][2][2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const _Float16* Lb = b + sub * 12288 + (ow >> 7) * 4096;
      const _Float16* Rb = b + sub * 12288 + 8192;
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        const int xa = (ow & (kDT - 1)) + 32 * i2 + l32, xb = cw + 32 * i2 + l32;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          fa[sub][i2][p] = *reinterpret_cast<const f16x8*>(Lb + p * kDT * 16 + xa * 16 + 8 * MX3::gran(xa, h));
          fb[sub][i2][p] = *reinterpret_cast<const f16x8*>(Rb + p * kDT * 16 + xb * 16 + 8 * MX3::gran(xb, h));
        }
      }
    }
#pragma unroll
    for (int sub = 0; sub < 2; ++sub)
#pragma unroll
      for (int bo = 0; bo < 2; ++bo)
#pragma unroll
        for (int bc = 0; bc < 2; ++bc) {
          f32x16 d = acc[bo][bc];
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[sub][bo][1], fb[sub][bc][0], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[sub][bo][0], fb[sub][bc][1], d, 0, 0, 0);
          d = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[sub][bo][0], fb[sub][bc][0], d, 0, 0, 0);
          acc[bo][bc] = d;
        }
  };""")
        if v in ("prio", "prefprio"):
            rep("""  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  int m0 = 0;""", """  const int l32 = lane & 31, h = lane >> 5;
  const int ow = (wave >> 1) * 64, cw = (wave & 1) * 64;
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  int m0 = 0;""")
    elif v.startswith("stag"):
        n = int(v[4:])
        anchor = """  X3WLoad L;
  L.t = t0;
  L.m = m0;
  L.live = true;
  h2_load_tile(g, L, wave);
"""
        assert src.count(anchor) == 1, "stag anchor"
        src = src.replace(anchor, """  {
    const int slot = (int)((blockIdx.x / nx) % 8);
    for (int q = 0; q < slot; ++q) __builtin_amdgcn_s_sleep(SLEEPN);
  }
""".replace("SLEEPN", str(n)) + anchor)
    else:
        raise SystemExit(f"unknown variant {v}")
    return src


def main():
    os.makedirs(OUT, exist_ok=True)
    base = open(os.path.join(PKG, "csrc", "hdp_delta.hip")).read()
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-function", "-mcode-object-version=5",
             f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(PKG, 'csrc')}", "-I/opt/rocm/include", "-munsafe-fp-atomics"]
    others = [os.path.join(PKG, "build", f"{n}.o") for n in ("hdp_elementwise", "hdp_probe", "hdp_svd", "hdp_api", "hdp_comm")]
    for v in sys.argv[1:] or ["nomfma", "nodma", "now", "nobar", "nolds"]:
        s = os.path.join(OUT, f"hdp_delta_{v}.hip")
        open(s, "w").write(variant(base, v))
        o = os.path.join(OUT, f"hdp_delta_{v}.o")
        subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", s, "-o", o])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-L/opt/rocm/lib",
                               "-Wl,-rpath,/opt/rocm/lib", "-lrccl", "-lrocsolver", "-lrocblas", o, *others, "-o",
                               os.path.join(OUT, f"libhdpissa_{v}.so")])
        print("built", v)


if __name__ == "__main__":
    main()
