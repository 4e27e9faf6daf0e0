"""Dump the gfx950 disassembly of the kernels of libhdpissa.so whose symbol matches a pattern
(measurement / inspection tool, not part of the library).

  python tools/isa_dump.py PATTERN [--lib path] [--out file] [--stats]
--stats prints per-kernel counts of MFMA / VALU / SALU / LDS / VMEM instructions (static)."""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from isa_scan import disassemble, gfx950_code_objects  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("--lib", default=os.path.join(ROOT, "hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so"))
    ap.add_argument("--out", default=None)
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    pat = re.compile(a.pattern)
    out = open(a.out, "w") if a.out else sys.stdout
    for co in gfx950_code_objects(a.lib):
        lines = disassemble(co)
        cur, keep, body = None, False, []
        for ln in lines + ["<end>:"]:
            if ln.endswith(">:"):
                if keep and body:
                    if a.stats:
                        c = {"mfma": 0, "valu": 0, "salu": 0, "lds": 0, "vmem": 0, "wait": 0, "total": 0}
                        for b in body:
                            m = re.match(r"^\s+([a-z_0-9]+)", b)
                            if not m:
                                continue
                            op = m.group(1)
                            c["total"] += 1
                            if op.startswith("v_mfma"):
                                c["mfma"] += 1
                            elif op.startswith("v_"):
                                c["valu"] += 1
                            elif op.startswith("s_waitcnt") or op == "s_barrier":
                                c["wait"] += 1
                            elif op.startswith("s_"):
                                c["salu"] += 1
                            elif op.startswith("ds_"):
                                c["lds"] += 1
                            elif op.startswith(("buffer_", "global_", "flat_")):
                                c["vmem"] += 1
                        print(cur, c, file=out)
                    else:
                        print(cur, file=out)
                        print("\n".join(body), file=out)
                cur, body = ln, []
                keep = bool(pat.search(ln))
            elif keep:
                body.append(ln)


if __name__ == "__main__":
    main()
