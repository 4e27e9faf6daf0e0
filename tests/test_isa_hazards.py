"""Static guards on the shipped gfx950 machine code (CPU).

1. No 12/16-byte vector-memory store has its data VGPRs overwritten by a vector instruction inside
   the 2-wait-state window.  In r03 the compiler scheduled exactly that behind K4's deferred bf16
   merge stores and some lanes stored the NEW first dword now and then; the store is now asm with
   its `s_nop 1`.  The scanner finds 13 such sites in the pre-fix source (commit 8b130ea,
   delta_h2_kernel<1,0,3,1>, compiled with this image's hipcc) and none in the current library.
2. No vector-memory load's destination VGPRs are read or written before an `s_waitcnt vmcnt` that
   covers the load.  Compiler-scheduled loads always pass; the check guards the hand-issued (asm)
   W-piece loads of the deferred merge, whose outputs the compiler believes ready right after the asm.
3. (r06) No vector-memory instruction reads an SGPR that a vector instruction (a v_readlane spill reload)
   wrote fewer than 5 wait states before -- the hazard hipcc pads for its own instructions but not inside
   the asm W loads / stores; an unpadded reload in front of the first deferred bf16 W store made it store
   through a stale descriptor (test_delta_plan_h2_bf16_deferred_merge caught it on the GPU).
"""
import os

import pytest

import isa_scan as S

LIB = os.path.join(os.path.dirname(__file__), "..", "hd-pissa_amd", "hdpissa_amd", "_lib", "libhdpissa.so")

BAD_STORE = """\
0000000000000100 <k>:
\tbuffer_store_dwordx4 v[96:99], v104, s[48:51], s10 offen   // 00000007695C: E07C1000 0A0C6068
\tv_lshlrev_b32_e32 v96, 16, v92                             // 000000076964: 24C0B890
\ts_endpgm                                                   // 000000076968: BF810000
"""
GOOD_STORE = BAD_STORE.replace("offen   //", "offen   //", 1).replace(
    "\tv_lshlrev_b32_e32 v96", "\ts_nop 1                                                    // 000000076960: BF800001\n"
    "\tv_lshlrev_b32_e32 v96", 1)
OTHER_REG = BAD_STORE.replace("v_lshlrev_b32_e32 v96, 16, v92", "v_lshlrev_b32_e32 v100, 16, v96")
GLOBAL_BAD = """\
0000000000000100 <k>:
\tglobal_store_dwordx4 v[8:9], v[10:13], off                // 00000001BD68: DC7C9000 007F0A08
\ts_mov_b32 s0, 1                                            // 00000001BD70: BE800081
\tv_mov_b32_e32 v12, 0                                       // 00000001BD74: 7E180280
"""

BAD_LOAD = """\
0000000000000100 <k>:
\tbuffer_load_dwordx4 v[20:23], v4, s[8:11], s12 offen       // 000000000100: E05C1000 0C021404
\tglobal_load_lds_dwordx4 v[2:3], off                        // 000000000108: DDF48000 007F0002
\ts_waitcnt vmcnt(2)                                         // 000000000110: BF8C0F72
\tv_add_u32_e32 v30, v20, v21                                // 000000000114: 683C2914
\ts_endpgm                                                   // 000000000118: BF810000
"""
GOOD_LOAD = BAD_LOAD.replace("s_waitcnt vmcnt(2) ", "s_waitcnt vmcnt(1) ")  # the LDS-DMA may stay in flight


BAD_SGPR = """\
0000000000000100 <k>:
\tv_readlane_b32 s15, v194, 23                               // 000000000100: D2890000 00010000
\tbuffer_store_dwordx4 v[98:101], v106, s[12:15], s5 offen   // 000000000108: E07C1000 05036266
\ts_endpgm                                                   // 000000000110: BF810000
"""
GOOD_SGPR = BAD_SGPR.replace("\tbuffer_store", "\ts_nop 4                                                    // 000000000104: BF800004\n\tbuffer_store", 1)


def test_scanner_finds_valu_sgpr_vmem():
    assert len(S.valu_sgpr_vmem_hazards(BAD_SGPR.splitlines())) == 1
    assert S.valu_sgpr_vmem_hazards(GOOD_SGPR.splitlines()) == []


def test_library_has_no_valu_sgpr_vmem_hazard(library_asm):
    found = [f for lines in library_asm for f in S.valu_sgpr_vmem_hazards(lines)]
    assert found == [], "\n".join(found[:20])


def test_scanner_finds_store_data_overwrite():
    assert len(S.wide_store_hazards(BAD_STORE.splitlines())) == 1
    assert S.wide_store_hazards(GOOD_STORE.splitlines()) == []
    assert S.wide_store_hazards(OTHER_REG.splitlines()) == []  # reads the data: no hazard
    assert len(S.wide_store_hazards(GLOBAL_BAD.splitlines())) == 1  # one wait state is not enough


def test_scanner_finds_use_before_wait():
    assert len(S.load_use_hazards(BAD_LOAD.splitlines())) == 1
    assert S.load_use_hazards(GOOD_LOAD.splitlines()) == []


@pytest.fixture(scope="module")
def library_asm():
    if not os.path.exists(LIB):
        pytest.skip("libhdpissa.so not built (run __graft_entry__.build())")
    if S.OBJDUMP is None:
        pytest.skip("llvm-objdump not found")
    return [S.disassemble(co) for co in S.gfx950_code_objects(LIB)]


def test_library_has_no_store_data_hazard(library_asm):
    stores = sum(1 for lines in library_asm for ln in lines if S._WIDE.match(ln))
    assert stores > 1000, "the scan must see the library's wide stores"
    assert any("delta_h2_kernelILi1ELi0ELi3ELi1E" in ln for lines in library_asm for ln in lines if ln.endswith(">:")), \
        "the deferred bf16 merge kernel must be in the scanned code"
    found = [f for lines in library_asm for f in S.wide_store_hazards(lines)]
    assert found == [], "\n".join(found[:20])


def test_library_has_no_load_use_before_wait(library_asm):
    found = [f for lines in library_asm for f in S.load_use_hazards(lines)]
    assert found == [], "\n".join(found[:20])


# 3. MFMA results (r04).  hipcc pads the reads of an MFMA's result itself but not on every path: the
# r-block-1 K32 probe read a v_mfma_f32_16x16x32_bf16 accumulator 3 wait states after issue behind a taken
# `s_cbranch_vccnz` and its projections came out wrong on some shapes.  The scan follows branches.
BRANCH_READ = """\
0000000000000100 <k>:
\tv_mfma_f32_16x16x32_bf16 v[40:43], v[40:43], v[4:7], v[44:47]// 000000096B00: D3B50028 04B20928
\ts_and_b64 vcc, exec, s[50:51]                              // 000000096B08: 86EA327E
\ts_cbranch_vccnz 2                                          // 000000096B0C: BF870002
\ts_nop 7                                                    // 000000096B10: BF800007
\ts_nop 7                                                    // 000000096B14: BF800007
\ts_or_b64 s[2:3], s[6:7], s[2:3]                            // 000000096B18: 87820206
\tv_add_f32_e32 v3, v8, v40                                  // 000000096B1C: 02065108
\ts_endpgm                                                   // 000000096B20: BF810000
"""
PADDED = BRANCH_READ.replace("\ts_and_b64", "\ts_nop 7                                                    // 000000096B04: BF800007\n\ts_and_b64", 1)
STRAIGHT = BRANCH_READ.replace("s_cbranch_vccnz 2 ", "s_cbranch_vccnz 0 ")  # falls into the pad either way


def test_scanner_finds_mfma_read_behind_branch():
    found = S.mfma_result_hazards(BRANCH_READ.splitlines())
    assert len(found) == 1 and "after 3 wait states" in found[0], found
    assert S.mfma_result_hazards(PADDED.splitlines()) == []
    assert S.mfma_result_hazards(STRAIGHT.splitlines()) == []


def test_library_has_no_mfma_result_hazard(library_asm):
    mfmas = sum(1 for lines in library_asm for ln in lines if "\tv_mfma_" in ln)
    assert mfmas > 1000, "the scan must see the library's MFMAs"
    found = [f for lines in library_asm for f in S.mfma_result_hazards(lines)]
    assert found == [], "\n".join(found[:20])
