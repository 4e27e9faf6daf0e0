"""K2 sweep ablation builds (measurement tool, not part of the library): variants of the float32
sweep with part of its work removed, linked into tools/abl/libhdpissa_<v>.so (HDPISSA_LIB=...;
results WRONG by construction -- timing only).
  halfmfma : every float32 sweep MFMA loop (PROJ and OUTER) issues half its MFMAs -- the phase times
             if the MFMA issue time halved (the ceiling an exact bf16 split of f32 activations targets)
  noreduce : the PROJ step's last-arriving wave skips the sum of the 8 partials and the slab store
  onemfma32: the bf16 16x16x32 PROJ issues one of its three split products
  notile   : the PROJ step skips its LDS tile store (the MFMAs read stale tile data)
  noyload  : the OUTER phases skip the Y (other stream's projection) loads of r-block 4 (stale registers)
  onemfma32o: the bf16 16x16x32 OUTER issues one of its three split products
  ntz      : non-temporal bf16 Z loads in the register-set sweep (float32 Z: the default since r04)
  x6c      : (a candidate) float32 phase C on the X6 OUTER form (pairs of steps; spills at four load sets)
  occb1    : (a candidate, results correct) float32 phase B at one workgroup per CU (three register sets)
usage: python tools/probe_ablate.py [--out DIR] [variant ...]   (default DIR tools/abl)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hd-pissa_amd")
OUT = os.path.join(ROOT, "tools", "abl")


def variant(src, v):
    def rep(old, new):
        nonlocal src
        assert src.count(old) == 1, (v, old[:60], src.count(old))
        src = src.replace(old, new)
    if v == "halfmfma":
        rep("""            for (int q = 0; q < 4; ++q) acc2[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(yv, z[p][q], acc2[b][q], 0, 0, 0);""",
            """            for (int q = 0; q < 2; ++q) acc2[b][q] = __builtin_amdgcn_mfma_f32_16x16x4f32(yv, z[p][q], acc2[b][q], 0, 0, 0);""")
        rep("""            for (int q = 0; q < 4; ++q) {
              if (ss & 1) a1[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[q], f[ss][b][q], a1[b], 0, 0, 0);""",
            """            for (int q = 0; q < 2; ++q) {
              if (ss & 1) a1[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(zf[q], f[ss][b][q], a1[b], 0, 0, 0);""")
    elif v == "noreduce":
        rep("""          for (int e0 = 0; e0 < 16 * r4; e0 += 64) {""", """          for (int e0 = 0; e0 < 0; e0 += 64) {""")
    elif v == "onemfma32":
        rep("""              a = mfma32(zb, fs8[ch][b][2], a);
              a = mfma32(zb, fs8[ch][b][1], a);
              a = mfma32(zb, fs8[ch][b][0], a);""", """              a = mfma32(zb, fs8[ch][b][0], a);""")
    elif v == "notile":
        rep("""      for (int p = 0; p < (DL ? 0 : 4); ++p) *reinterpret_cast<f32x4*>(tile + (4 * p + g) * kTileLd + 4 * li) = z[p];""",
            """      for (int p = 0; p < 0; ++p) *reinterpret_cast<f32x4*>(tile + (4 * p + g) * kTileLd + 4 * li) = z[p];""")
    elif v == "noyload":
        rep("""            const f32x4 v = gld4(d.y_in + yo[p]);
#pragma unroll
            for (int b = 0; b < RB; ++b) y[p][b] = v[b];""", """            const f32x4 v{0.5f, 0.25f, 0.125f, (float)p};
#pragma unroll
            for (int b = 0; b < RB; ++b) y[p][b] = v[b];""")
    elif v == "onemfma32o":
        rep("""          acc2[b][q] = mfma32(yl, zq[q], acc2[b][q]);
          acc2[b][q] = mfma32(ym, zq[q], acc2[b][q]);
          acc2[b][q] = mfma32(yh, zq[q], acc2[b][q]);""", """          acc2[b][q] = mfma32(yh, zq[q], acc2[b][q]);""")
    elif v == "occb1":  # (a candidate, results correct) phase B at one workgroup per CU, three register sets
        rep("""  constexpr int OCC_B = SPLIT_B ? 1 : RB >= 4 ? 3 : VEC ? 2 : 1;""",
            """  constexpr int OCC_B = SPLIT_B ? 1 : RB >= 4 ? 3 : 1;""")
    elif v == "x6c":  # (a candidate) float32 phase C on the X6 OUTER form (pairs of steps, four load sets; spills)
        rep("""      G[2] = k32 ? phase_grid<DT, RBF, kSwOuter, VEC, 1, true, BF>(U[2], 0)""",
            """      G[2] = kf ? phase_grid<DT, RBF, kSwOuter, VEC, 1, true, true>(U[2], 0)""")
        rep("""        if (k32)
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwOuter, VEC, 1, true, BF>), dim3(G[2]), dim3(512), 0, st,""",
            """        if (kf)
          hipLaunchKernelGGL((probe_sweep_kernel<DT, RBF, kSwOuter, VEC, 1, true, true>), dim3(G[2]), dim3(512), 0, st,""")
    elif v == "ntz":
        rep("""            z[p] = load4<DT>(Zb + zo[p], 0);""", """            z[p] = load4_nt<DT>(Zb + zo[p], 0);""")
    else:
        raise SystemExit(f"unknown variant {v}")
    return src


def main():
    global OUT
    args = sys.argv[1:]
    if args[:1] == ["--out"]:
        OUT, args = os.path.abspath(args[1]), args[2:]
    os.makedirs(OUT, exist_ok=True)
    base = open(os.path.join(PKG, "csrc", "hdp_probe.hip")).read()
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-function", "-mcode-object-version=5",
             f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(PKG, 'csrc')}", "-I/opt/rocm/include", "-munsafe-fp-atomics"]
    others = [os.path.join(PKG, "build", f"{n}.o") for n in ("hdp_elementwise", "hdp_delta", "hdp_svd", "hdp_api", "hdp_comm")]
    for v in args or ["halfmfma"]:
        s = os.path.join(OUT, f"hdp_probe_{v}.hip")
        open(s, "w").write(variant(base, v))
        o = os.path.join(OUT, f"hdp_probe_{v}.o")
        subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", s, "-o", o])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-L/opt/rocm/lib",
                               "-Wl,-rpath,/opt/rocm/lib", "-lrccl", "-lrocsolver", "-lrocblas", o, *others, "-o",
                               os.path.join(OUT, f"libhdpissa_{v}.so")])
        print("built", v)


if __name__ == "__main__":
    main()
