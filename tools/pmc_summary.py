"""Summarise the two PMC passes of tools/pmc.sh into profiles/<name>_pmc_summary.json.

Per hdp kernel (and grid): HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half of a
wide streaming read, MI355X_MICROARCH.md HBM section) + WRITE_SIZE (exact for 16-B stores),
both in KiB in rocprofv3's CSV; the first of the three iterations (cold) is skipped.
Also records the traffic / algorithmic-bytes ratio per op that bench.py applies to its
live per-launch algorithmic bytes to fill roofline.traffic."""
import collections
import csv
import json
import sys

src, dst = sys.argv[1], sys.argv[2]


def load(c):
    out = []
    for r in csv.DictReader(open(f"{src}/{c}.csv")):
        if "hdp::" in r["Kernel_Name"]:
            out.append((r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Grid_Size"]),
                        float(r["Counter_Value"]) * 1024.0))
    return out


f, w = load("FETCH_SIZE"), load("WRITE_SIZE")
n = len(f) // 3
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
dcount = 0
for (k, g, fv), (k2, g2, wv) in list(zip(f, w))[n:]:
    assert k == k2 and g == g2
    if "delta_gemm" in k:  # hotpath_kernels.py issues nseg = 1 then nseg = 8 per module
        k = k + (" nseg=1" if dcount % 2 == 0 else " nseg=8")
        dcount += 1
    a = agg[(k, g)]
    a[0] += 1
    a[1] += 2.0 * fv
    a[2] += wv
kern = [{"kernel": k, "grid": g, "launches": c, "hbm_read_bytes": fr / c, "hbm_write_bytes": wr / c,
         "hbm_bytes": (fr + wr) / c} for (k, g), (c, fr, wr) in sorted(agg.items())]
# algorithmic bytes of tools/hotpath_kernels.py per op (fp32, T=1024, r=16, one LLaMA layer)
T, r = 1024, 16
shapes = [(4096, 4096)] * 4 + [(11008, 4096)] * 2 + [(4096, 11008)]
probe_alg = sum(4.0 * T * (o + i) + 8.0 * r * (o + i) for o, i in shapes)
probe_hbm_layer = sum(x["hbm_bytes"] * 1 for x in kern if "probe_" in x["kernel"])
delta_alg = sum(8.0 * o * i for o, i in shapes)  # per layer, W read + write (fp32)
delta1_hbm = sum(x["hbm_bytes"] * x["launches"] for x in kern if "nseg=1" in x["kernel"]) / 2.0
delta8_hbm = sum(x["hbm_bytes"] * x["launches"] for x in kern if "nseg=8" in x["kernel"]) / 2.0
res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/hotpath_kernels.py",
       "correction": "FETCH_SIZE x2 (gfx950 wide-read halving); WRITE_SIZE as reported",
       "kernels": kern,
       "traffic_over_algorithmic": {
           "probe_grads_group": probe_hbm_layer / probe_alg,
           "delta_gemm_nseg1": delta1_hbm / delta_alg,
           "delta_gemm_nseg8": delta8_hbm / delta_alg,
       }}
json.dump(res, open(dst, "w"), indent=1)
print(json.dumps(res["traffic_over_algorithmic"]))
