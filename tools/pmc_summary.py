"""Summarise the two PMC passes of tools/pmc.sh into profiles/<name>_pmc_summary.json.

Per hdp kernel launch: HBM bytes = 2 x FETCH_SIZE (gfx950 reports half of a wide streaming
read, MI355X_MICROARCH.md HBM section) + WRITE_SIZE (exact for 16-B stores), both in KiB in
rocprofv3's CSV.  Launches are grouped by the library's kernel-timing names (merge, adam,
delta_gemm, probe_sweep_b, ...); the first (cold) iteration of tools/hotpath_kernels.py is
skipped, exactly as its live timing dump (hotpath_timing.json: launches + ALGORITHMIC bytes
per name) does.  traffic_over_algorithmic[name] = measured HBM bytes / algorithmic bytes,
which bench.py multiplies into its live per-launch algorithmic bytes to fill roofline.traffic.

usage: python tools/pmc_summary.py gpurun_out/pmc profiles/rNN_pmc_summary.json
"""
import collections
import csv
import json
import os
import re
import sys


def family(sym: str, seg_count: dict) -> str:
    """Kernel symbol -> hdp_timing name (see kKernelNames in hdp_api.cpp)."""
    if "merge_" in sym:
        return "merge"
    if "adam_" in sym:
        return "adam"
    if "delta_group_kernel" in sym:  # tools/hotpath_kernels.py: the Wn = 1 plan
        return "delta_gemm"
    if "delta_gemm_kernel" in sym:  # the Wn = 8 per-module launches
        return "delta_gemm_multiseg"
    if "probe_proj_kernel" in sym:
        return "probe_p1"
    if "probe_outer_kernel" in sym:
        return "probe_p2"
    if "probe_finish_kernel" in sym or "probe_sweep_finish_kernel" in sym:
        return "probe_finish"
    if "probe_yreduce_kernel" in sym:
        return "probe_reduce"
    m = re.search(r"probe_sweep_kernel<\d+, \d+, (\d)", sym)
    if m:
        return {"1": "probe_sweep_a", "3": "probe_sweep_b", "2": "probe_sweep_c"}[m.group(1)]
    return sym


def load(src, c):
    out = []
    for r in csv.DictReader(open(os.path.join(src, f"{c}.csv"))):
        if "hdp::" in r["Kernel_Name"]:
            out.append((r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Grid_Size"]),
                        float(r["Counter_Value"]) * 1024.0))
    return out


def main(src, dst):
    timing = json.load(open(os.path.join(src, "hotpath_timing.json")))
    f, w = load(src, "FETCH_SIZE"), load(src, "WRITE_SIZE")
    assert len(f) == len(w)
    fam_f, fam_w = {"n": 0}, {"n": 0}
    per_launch = []
    for (k, g, fv), (k2, g2, wv) in zip(f, w):
        assert k == k2 and g == g2, (k, k2)
        name = family(k, fam_f)
        family(k2, fam_w)
        per_launch.append((name, k, g, 2.0 * fv, wv))
    # drop the cold first iteration: the launches beyond what the warm timing dump counts
    counts = collections.Counter(p[0] for p in per_launch)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    seen = collections.Counter()
    for name, k, g, rd, wr in per_launch:
        seen[name] += 1
        warm = timing.get(name, {}).get("launches", 0)
        if seen[name] <= counts[name] - warm:
            continue
        a = agg[name]
        a[0] += 1
        a[1] += rd
        a[2] += wr
    kern, ratio = [], {}
    for name, (c, rd, wr) in sorted(agg.items()):
        t = timing.get(name)
        alg = t["bytes_per_launch"] if t else None
        kern.append({"kernel": name, "launches": c, "hbm_read_bytes": rd / c, "hbm_write_bytes": wr / c,
                     "hbm_bytes": (rd + wr) / c, "algorithmic_bytes": alg,
                     "avg_us_live": t["avg_us"] if t else None})
        if alg:
            ratio[name] = (rd + wr) / c / alg
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/hotpath_kernels.py",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving); WRITE_SIZE as reported",
           "kernels": kern, "traffic_over_algorithmic": ratio}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(ratio, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
