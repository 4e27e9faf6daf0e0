"""Summarise tools/pmc_bench.sh (PMC passes over the bench command) into the JSON bench.py reads
for its roofline `traffic` and `mfma_busy` fields.

Per kernel family (the library's kernel-timing names): the LAST N dispatches of the family in the
trace are the bench's instrumented timed steps (N = launches in the bench's --timing-out dump,
which also gives their ALGORITHMIC bytes).  Over those dispatches:
  traffic_over_algorithmic = (2 x FETCH_SIZE + WRITE_SIZE) / algorithmic bytes
      (gfx950 FETCH_SIZE counts half the bytes of a wide streaming read -- MI355X_MICROARCH.md,
      HBM section; WRITE_SIZE is exact for 16-B stores; both reported in KiB)
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
      (GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA busy cycles are summed over SIMDs)
usage: python tools/pmc_bench_summary.py gpurun_out/pmc_bench_<wl> profiles/r04_pmc_bench_<wl>.json
The summary records the kernel-source digest (bench.kernel_source_digest): bench.py uses the
profile only on the same sources.
"""
import collections
import csv
import json
import os
import re
import sys

NAMES = {"fold_bf16": "fold_bf16", "merge_": "merge", "adam_": "adam", "delta_group_kernel": "delta_gemm", "delta_x3w_kernel": "delta_gemm_multiseg",
         "delta_x3p_kernel": "delta_gemm_multiseg", "delta_x3g_kernel": "delta_gemm_multiseg",
         "delta_gemm_kernel": "delta_gemm_multiseg", "delta_h2_kernel": "delta_gemm", "k4_pack_kernel": "delta_pack",
         "k4_h2_adam_pack_kernel": "adam", "k4_h2_": "delta_pack", "probe_proj_kernel": "probe_p1",
         "probe_outer_kernel": "probe_p2", "probe_finish_kernel": "probe_finish",
         "probe_sweep_finish_kernel": "probe_finish", "probe_yreduce_kernel": "probe_reduce"}


def family(sym):
    for k, v in NAMES.items():
        if k in sym:
            return v
    return None


def load(path):
    """dispatch id -> (family, {counter: value}).  The sweep kernels of a group are dispatched in
    the order A, B, C (launch_sweep); their template arguments do not name the phase (the bf16
    r-block-4 phase B is a PROJ-only instance, like A), so the phase comes from the dispatch order."""
    rows = list(csv.DictReader(open(path)))
    sweep = sorted({int(r["Dispatch_Id"]) for r in rows if "probe_sweep_kernel<" in r["Kernel_Name"]})
    phase = {d: ("probe_sweep_a", "probe_sweep_b", "probe_sweep_c")[i % 3] for i, d in enumerate(sweep)}
    out = collections.OrderedDict()
    for r in rows:
        d = int(r["Dispatch_Id"])
        fam = phase.get(d) or family(r["Kernel_Name"])
        if fam is None:
            continue
        out.setdefault(d, (fam, {}))[1][r["Counter_Name"]] = out.get(d, (fam, {}))[1].get(r["Counter_Name"], 0.0) + \
            float(r["Counter_Value"])
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    timing = json.load(open(os.path.join(src, "timing.json")))
    passes = [load(os.path.join(src, f"pass{i}.csv")) for i in (1, 2, 3)]
    fams = collections.defaultdict(lambda: [[], [], []])
    for i, p in enumerate(passes):
        for d, (fam, ctr) in p.items():
            fams[fam][i].append(ctr)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_digest  # noqa: E402
    res = dict(source="tools/pmc_bench.sh: rocprofv3 --pmc over python3 bench.py --steps 2 --warmup 1 --init random "
                      "--no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange",
               source_digest=kernel_source_digest(), args=open(os.path.join(src, "args.txt")).read().strip()
               if os.path.exists(os.path.join(src, "args.txt")) else "",
               traffic_over_algorithmic={}, mfma_busy={}, per_launch={})
    for fam, (p1, p2, p3) in sorted(fams.items()):
        t = timing.get(fam)
        if not t:
            continue
        n = int(t["launches"])
        f1, f2, f3 = p1[-n:], p2[-n:], p3[-n:]
        if len(f1) < n or len(f2) < n:
            continue
        hbm = sum(2 * c["FETCH_SIZE"] * 1024.0 for c in f1) + sum(c["WRITE_SIZE"] * 1024.0 for c in f2)
        alg = t["bytes_per_launch"] * n
        if alg > 0:
            res["traffic_over_algorithmic"][fam] = round(hbm / alg, 4)
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for c in f3)
        simd_cycles = sum(c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 * 1024 for c in f3)
        if simd_cycles > 0:
            res["mfma_busy"][fam] = round(busy / simd_cycles, 4)
        res["per_launch"][fam] = dict(launches=n, hbm_bytes=round(hbm / n), algorithmic_bytes=round(alg / n),
                                      avg_us_live=round(t["avg_us"], 2))
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
