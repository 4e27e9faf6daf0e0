"""Summarise tools/r03_pmc_sq.sh (measurement tool): per kernel family, counters summed over its dispatches.
usage: python tools/pmc_sq_summary.py gpurun_out/pmc_sq_<tag>"""
import collections
import csv
import os
import re
import sys


def fam(sym):
    m = re.search(r"(probe_\w+_kernel|delta_\w+_kernel|k4_\w+_kernel|adam\w*|merge\w*)(<[^(]*>)?", sym)
    return (m.group(1) + (m.group(2) or "")) if m else None


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for i in (1, 2):
        p = os.path.join(d, f"pass{i}.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            f = fam(r["Kernel_Name"])
            if f is None:
                continue
            tot[f][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[f].add((i, r["Dispatch_Id"]))
    for f, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        gui = c.get("GRBM_GUI_ACTIVE", 0) or 1
        print(f"{f[:110]}")
        print(f"   dispatches {len(disp[f]) // 2}  wait_any/wave {c.get('SQ_WAIT_ANY', 0) / wc:.3f}  wait_inst_any/wave "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}  active_inst_any/wave {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}  "
              f"mfma_busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui / 8 * 1024):.3f}")
        print("   insts: " + "  ".join(f"{k[9:] if k.startswith('SQ_INSTS_') else k[3:]} {c.get(k, 0):.3g}" for k in
                                      ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                                       "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS",
                                       "SQ_LDS_BANK_CONFLICT")))


if __name__ == "__main__":
    main()
