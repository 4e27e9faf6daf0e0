"""Summarise a rocprofv3 --kernel-trace --stats CSV of tools/e2e_train.py (measurement tool): total
time by kernel class (base-model GEMMs, attention, HD-PiSSA K2/K3/K4, elementwise/other) and the top
kernels.  usage: python tools/e2e_prof_summary.py kernel_stats.csv [steps]"""
import csv
import sys


def klass(name):
    n = name.lower()
    if "rocsolver" in n or "_db_" in n or "f64" in n or "syevd" in n or ("rocblas" in n and "double" in n):
        return "SVD-slice init (rocSOLVER + fp64 Gram / projection GEMMs, hp:96-134; once per run)"
    if "hdp::" in n:
        if "probe" in n:
            return "HD-PiSSA K2 probe (hp:139 adapter backward)"
        if "delta" in n or "k4_" in n:
            return "HD-PiSSA K4 delta+merge (hp:389-394)"
        if "adam" in n:
            return "HD-PiSSA K3 Adam (hp:356-373)"
        return "HD-PiSSA other (SVD init, merge)"
    if "cijk" in n or "gemm" in n or "gemv" in n or "matmul" in n or "hipblaslt" in n or "_mt" in n and "mfma" in n:
        return "base-model GEMMs (hipBLASLt / rocBLAS, hp:139 F.linear + autograd dX)"
    if ("attn" in n or "attention" in n or "flash" in n or "softmax" in n or "sdpa" in n
            or n.startswith("bwd_kernel") or n.startswith("bwd_preprocess")):  # AOTriton flash-attention backward
        return "attention / softmax"
    return "elementwise / reductions / other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    tot = {}
    allns = 0.0
    for r in rows:
        ns = float(r["TotalDurationNs"])
        allns += ns
        k = klass(r["Name"])
        tot[k] = tot.get(k, 0.0) + ns
    print(f"total kernel time {allns / 1e9:.3f} s")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {v / 1e9:8.3f} s  {100 * v / allns:5.1f} %  {k}")
    def top(rs, n):
        for r in sorted(rs, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
            print(f"  {float(r['TotalDurationNs']) / 1e9:8.3f} s  calls {r['Calls']:>6s}  avg {float(r['AverageNs']) / 1e3:9.1f} us  "
                  f"{r['Name'][:110]}")
    print("top kernels:")
    top(rows, 15)
    for k in ("attention / softmax", "elementwise / reductions / other"):
        print(f"top kernels of '{k}':")
        top([r for r in rows if klass(r["Name"]) == k], 12)


if __name__ == "__main__":
    main()
