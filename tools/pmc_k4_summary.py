"""Summarise scratch/r06_d.sh-style PMC passes over tools/delta_bench.py (measurement tool): per workload tag,
the delta_h2_kernel counters summed over its dispatches, per wave-tile and per wave-cycle.
usage: python tools/pmc_k4_summary.py DIR TAG TILES_PER_DISPATCH"""
import collections
import csv
import glob
import os
import sys


def main():
    d, tag, tiles = sys.argv[1], sys.argv[2], float(sys.argv[3])
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for p in sorted(glob.glob(os.path.join(d, f"pass*_{tag}.csv"))):
        for r in csv.DictReader(open(p)):
            if "delta_h2_kernel" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((p, r["Dispatch_Id"]))
    for k in sorted(tot):
        n = len(disp[k]) or 1
        v = tot[k] / n  # per dispatch
        wt = tiles * 8  # waves x tiles
        wc = tot.get("SQ_WAVE_CYCLES", 0) / max(len(disp.get("SQ_WAVE_CYCLES", ())), 1) or 1
        print(f"  {k:32s} {v:12.4g} per dispatch  {v / wt:10.1f} per wave-tile  {v / wc:7.3f} per wave-cycle")


if __name__ == "__main__":
    main()
