"""Static scan of the gfx950 code objects inside libhdpissa.so (test infrastructure).

The library's .hip_fatbin section holds one clang offload bundle per translation unit; each
bundle's gfx950 entry is an ELF code object that llvm-objdump disassembles.  `wide_store_hazards`
looks for the pattern that made K4's deferred bf16 merge store nondeterministic bytes in r03
(DESIGN §9): a 12- or 16-byte vector-memory store (buffer_/global_/flat_/scratch_store_dwordx3/x4) whose
data VGPRs are overwritten by a vector instruction before two wait states have passed (gfx940+
needs 2; an `s_nop N` supplies N + 1, every other issued instruction 1).  Only the straight-line
successors are scanned: the scan stops at a branch, a label or once the window has passed.
`load_use_hazards` checks hand-issued loads against their vmcnt waits, and `mfma_result_hazards` (r04) the
wait states between an MFMA and the first non-MFMA access of its result on every path, branches included.
"""
from __future__ import annotations

import os
import re
import shutil
import struct
import subprocess
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WAIT_STATES = 2  # VALU write of a >8-byte store's data VGPRs (GCN hazard, gfx940 and later)
OBJDUMP = next((p for p in ("/opt/rocm/llvm/bin/llvm-objdump", "/opt/rocm/lib/llvm/bin/llvm-objdump")
                if os.path.exists(p)), shutil.which("llvm-objdump"))
_WIDE = re.compile(r"^\s*(buffer|global|flat|scratch)_store_dwordx([34])\s+(.*?)(\s+//.*)?$")
_INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*(//.*)?$")
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def gfx950_code_objects(so_path: str) -> list[bytes]:
    """Every gfx950 code object of the shared library's offload bundles."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", so_path, os.path.join(td, "junk.so")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    start = data.find(MAGIC)
    while start >= 0:
        n = struct.unpack_from("<Q", data, start + 24)[0]
        p = start + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                out.append(data[start + off:start + off + size])
        start = data.find(MAGIC, start + 1)
    return out


def disassemble(code_object: bytes) -> list[str]:
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(code_object)
        f.flush()
        r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], check=True, capture_output=True, text=True)
    return r.stdout.splitlines()


def _regs(operand: str) -> set[int]:
    m = _VREG.search(operand)
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _split_operands(ops: str) -> list[str]:
    return [o.strip() for o in re.split(r",\s*(?![^\[]*\])", ops)] if ops else []


def wide_store_hazards(lines: list[str]) -> list[str]:
    """Findings 'function: store ... -> writer ...' for every wide store whose data VGPRs a vector
    instruction writes within the hazard window."""
    found, func = [], "?"
    for i, line in enumerate(lines):
        if line.endswith(">:"):
            func = line.split("<", 1)[-1][:-2]
            continue
        m = _WIDE.match(line)
        if not m:
            continue
        ops = _split_operands(m.group(3))
        # buffer_store: data first; global/flat/scratch_store: address first, data second
        data = _regs(ops[0] if m.group(1) == "buffer" else ops[1] if len(ops) > 1 else "")
        ws = 0
        for nxt in lines[i + 1:]:
            if ws >= WAIT_STATES or not nxt.strip() or nxt.endswith(">:") or nxt.endswith(":"):
                break
            mi = _INSN.match(nxt)
            if not mi:
                break
            op, args = mi.group(1), mi.group(2) or ""
            if op == "s_nop":
                ws += int(args.split()[0], 0) + 1
                continue
            if op.startswith("v_"):
                dst = _split_operands(args)
                if dst and _regs(dst[0]) & data:
                    found.append(f"{func}: {line.strip()} -> {nxt.strip()}")
                    break
            if op.startswith("s_branch") or op.startswith("s_cbranch") or op.startswith("s_setpc") or op == "s_endpgm":
                break
            ws += 1
    return found


_VMEM = re.compile(r"^(buffer|global|flat|scratch)_(load|store|atomic)")
_WAIT = re.compile(r"vmcnt\((\d+)\)")


def load_use_hazards(lines: list[str], limit: int = 4000) -> list[str]:
    """Findings for vector-memory loads whose destination VGPRs an instruction reads or writes before
    an `s_waitcnt vmcnt(k)` covers the load (k <= the VMEM operations issued after it).  Compiler-
    scheduled loads always pass; the check is for hand-issued (asm) loads whose outputs the compiler
    believes ready right after the asm (the deferred merge's W pieces).  The scan follows
    the fall-through path (address order, through conditional branches, up to an unconditional one),
    so a wait on either side of a conditional branch counts."""
    found, func = [], "?"
    for i, line in enumerate(lines):
        if line.endswith(">:"):
            func = line.split("<", 1)[-1][:-2]
            continue
        mi = _INSN.match(line)
        if (not mi or not _VMEM.match(mi.group(1)) or "_load" not in mi.group(1) or "lds" in mi.group(1)
                or " lds" in (mi.group(2) or "")):  # LDS-DMA: no VGPR destination
            continue
        ops = _split_operands(mi.group(2) or "")
        dst = _regs(ops[0]) if ops else set()
        if not dst:
            continue
        after = 0
        for nxt in lines[i + 1:i + 1 + limit]:
            if nxt.endswith(">:"):
                break
            mn = _INSN.match(nxt)
            if not mn:
                continue
            op, args = mn.group(1), mn.group(2) or ""
            if op == "s_waitcnt":
                w = _WAIT.search(args)
                if w and int(w.group(1)) <= after:
                    break
                continue
            if op in ("s_endpgm", "s_branch", "s_setpc_b64"):  # the next address is another path
                break
            opnds = _split_operands(args)
            if _VMEM.match(op) and "_load" in op:
                opnds = opnds[1:]  # another load may rewrite them: vector-memory loads return in order
            if any(_regs(o) & dst for o in opnds):
                found.append(f"{func}: {line.strip()[:80]} -> {nxt.strip()[:80]} ({after} VMEM ops after the load)")
                break
            if _VMEM.match(op):
                after += 1
    return found


_ANYREG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")
_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_BRANCH = re.compile(r"^s_(c?branch\w*)$")


def _regs_va(operand: str) -> set[tuple[str, int]]:
    out = set()
    for m in _ANYREG.finditer(operand):
        if m.group(1):
            out |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def _functions(lines: list[str]):
    """(name, [(addr, op, args, text)]) per function of a disassembly."""
    funcs, cur, name = [], None, "?"
    for line in lines:
        if line.endswith(">:"):
            name = line.split("<", 1)[-1][:-2]
            cur = []
            funcs.append((name, cur))
            continue
        if cur is None:
            continue
        mi, ma = _INSN.match(line), _ADDR.search(line)
        if mi and ma:
            cur.append((int(ma.group(1), 16), mi.group(1), (mi.group(2) or "").strip(), line.strip()))
    return funcs


# wait states a non-MFMA instruction needs after an MFMA issued before it reads (RAW) or writes (WAW)
# the MFMA's destination registers, measured on MI355X (tools/mfma_hazard.hip, profiles/r04_mfma_hazard.txt:
# the last pad that fails -> the first that passes): RAW 16x16x32 bf16 5 -> 6, 16x16x16 bf16 3 -> 5, 16x16x4
# f32 8 -> 9, 32x32x16 bf16 9 -> 10 (its last four registers), 32x32x2 f32 16 -> 18; WAW 16x16x32 3 -> 5,
# 32x32x16 1 -> 3.  WAW of the other forms unmeasured: their RAW figure, except 32x32x2 f32 at hipcc's own
# 17 (its first result registers land first: RAW of registers 0-3 passes at 1).
MFMA_WAIT_STATES = {
    "v_mfma_f32_16x16x32": (6, 5),
    "v_mfma_f32_16x16x16": (5, 5),
    "v_mfma_f32_16x16x4": (9, 9),
    "v_mfma_f32_32x32x16": (10, 3),
    "v_mfma_f32_32x32x2": (18, 17),
}


def mfma_result_hazards(lines: list[str], table: dict | None = None) -> list[str]:
    """Findings for MFMAs whose destination registers a non-MFMA instruction reads or writes fewer wait
    states after the MFMA issued than `table` requires (prefix -> (RAW, WAW)), on any path: the scan
    follows conditional branches both ways and unconditional ones to their targets (every instruction is
    one wait state, `s_nop N` N + 1).  r04: hipcc's own padding misses paths through a taken branch -- the
    r-block-1 K32 probe sweep read a v_mfma_f32_16x16x32_bf16 result 3 wait states after it issued
    (`s_and_b64; s_cbranch_vccnz` to a block whose first VALU read the accumulator) and its projections
    came out wrong (tests/test_gpu_kernels.py::test_probe_k32_all_rblocks); the kernels pad such reads
    explicitly (HDP_MFMA_FENCE in hdp_common.h)."""
    table = MFMA_WAIT_STATES if table is None else table
    found = []
    for name, ins in _functions(lines):
        at = {a: k for k, (a, _, _, _) in enumerate(ins)}
        for k, (addr, op, args, text) in enumerate(ins):
            req = next((v for p, v in table.items() if op.startswith(p)), None)
            if req is None:
                continue
            ops = _split_operands(args)
            dst = _regs_va(ops[0]) if ops else set()
            if not dst:
                continue
            horizon = max(req)
            stack, seen, hit = [(k + 1, 0)], set(), None
            while stack and hit is None:
                j, ws = stack.pop()
                while j < len(ins) and ws < horizon and hit is None:
                    if (j, ws) in seen:
                        break
                    seen.add((j, ws))
                    _, op2, args2, text2 = ins[j]
                    if op2 == "s_nop":
                        ws += int(args2.split()[0], 0) + 1
                        j += 1
                        continue
                    opnds = _split_operands(args2)
                    if op2.startswith("v_mfma"):
                        if opnds and _regs_va(opnds[0]) & dst:
                            break  # rewritten by the next MFMA of the chain: its own hazard from here
                    elif opnds:
                        wr = (op2.startswith("v_") or "_load" in op2) and not op2.startswith("v_cmp")
                        w_regs = _regs_va(opnds[0]) if wr else set()
                        r_regs = set().union(*(_regs_va(o) for o in opnds[1 if wr else 0:]))
                        if r_regs & dst and ws < req[0]:
                            hit = f"{name}: {text[:60]} -> {text2[:60]} reads after {ws} wait states"
                        elif w_regs & dst and ws < req[1]:
                            hit = f"{name}: {text[:60]} -> {text2[:60]} writes after {ws} wait states"
                        if hit:
                            break
                    if op2 in ("s_endpgm", "s_setpc_b64"):
                        break
                    b = _BRANCH.match(op2)
                    if b:
                        off = int(opnds[0], 0) if opnds else 0
                        off = off - 65536 if off >= 32768 else off
                        tgt = at.get(ins[j][0] + 4 + 4 * off)
                        if tgt is not None:
                            stack.append((tgt, ws + 1))
                        if op2 == "s_branch":
                            break
                    ws += 1
                    j += 1
            if hit:
                found.append(hit)
    return found


_SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
VALU_SGPR_VMEM_WAIT_STATES = 5  # CDNA3/4 ISA: a VALU write of an SGPR -> a VMEM instruction reading it


def _sregs(operand: str) -> set[int]:
    out = set()
    for m in _SREG.finditer(operand):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _valu_sgpr_dst(op: str, opnds: list[str]) -> set[int]:
    """SGPRs a vector instruction writes (v_readlane / v_readfirstlane / v_cmp e64 destinations, carry-outs)."""
    if not op.startswith("v_") or not opnds:
        return set()
    if op.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
        return _sregs(opnds[0])
    if "_co_" in op or op.startswith("v_div_scale"):
        return _sregs(opnds[1]) if len(opnds) > 1 else set()
    return set()


def valu_sgpr_vmem_hazards(lines: list[str]) -> list[str]:
    """Findings for vector-memory instructions (loads, stores, atomics, LDS-DMA) reading an SGPR (descriptor,
    soffset) that a vector instruction wrote fewer than 5 wait states before, on the address-order path
    (every instruction one wait state, `s_nop N` N + 1).  hipcc pads this hazard for the instructions it
    schedules, not inside inline asm: r06's deferred bf16 W store (asm) read a descriptor that a v_readlane
    spill reload had written one instruction earlier, and stored through a stale descriptor."""
    found, func = [], "?"
    ins = []
    for line in lines:
        if line.endswith(">:"):
            func = line.split("<", 1)[-1][:-2]
            ins = []
            continue
        mi = _INSN.match(line)
        if not mi:
            continue
        op, args = mi.group(1), mi.group(2) or ""
        opnds = _split_operands(args)
        if _VMEM.match(op) or op.startswith("global_load_lds"):
            reads = set().union(*(_sregs(o) for o in opnds)) if opnds else set()
            ws = 0
            for op2, opnds2 in reversed(ins):
                if ws >= VALU_SGPR_VMEM_WAIT_STATES:
                    break
                if op2 == "s_nop":
                    ws += int(opnds2[0], 0) + 1 if opnds2 else 1
                    continue
                hit = _valu_sgpr_dst(op2, opnds2) & reads
                if hit:
                    found.append(f"{func}: {op} {args[:60]} <- {op2} {', '.join(opnds2)[:40]} ({ws} wait states)")
                    break
                ws += 1
        ins.append((op, opnds))
        if len(ins) > 16:
            ins.pop(0)
    return found
