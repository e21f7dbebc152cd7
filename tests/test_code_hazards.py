"""The built gfx950 code object has no VALU-writes-SGPR -> vector-memory-reads-SGPR
hazard closer than the 5 wait states the ISA requires (tools/vmem_sgpr_hazards.py).
The compiler's hazard recognizer inserts those wait states for the instructions it
emits, not in front of inline asm: fa_bwd.hip's asm LDS-DMA loads carry an `s_nop 4`
(a spilled descriptor restored by v_readlane right before one gave wrong dQ/dK/dV at
d = 32), and its asm running-sum loads carry none, which this test keeps honest for
whatever the compiler's register allocation does.  CPU only: it reads the library."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "flashattention.jl_amd", "libfa_hip.so")


def test_no_valu_sgpr_vmem_hazards():
    import vmem_sgpr_hazards as H
    if not os.path.exists(LIB):
        pytest.skip("libfa_hip.so not built")
    if shutil.which("objcopy") is None or not os.path.exists(os.path.join(H.LLVM, "llvm-objdump")):
        pytest.skip("binutils / ROCm llvm tools missing")
    lines = H.disassemble(LIB)
    assert sum(1 for l in lines if "offen lds" in l) > 100, "the DMA kernels were not found in the disassembly"
    found = H.scan(lines)
    assert not found, "\n".join(f"{f}: {a} -> {b} ({ws} wait states)" for f, a, b, ws in found[:10])


def test_checker_sees_a_planted_hazard():
    import vmem_sgpr_hazards as H
    lines = ["0000000000001000 <k>:",
             "\tv_readlane_b32 s87, v161, 14  // 0",
             "\tbuffer_load_dwordx4 v50, s[84:87], 0 offen lds  // 0",
             "\tv_readlane_b32 s3, v1, 0",
             "\ts_nop 4",
             "\tbuffer_load_dwordx4 v[0:3], v2, s[0:3], 0 offen offset:16 sc1"]
    found = H.scan(lines)
    assert len(found) == 1 and found[0][1].startswith("v_readlane_b32 s87")


def test_checker_follows_taken_branches_and_back_edges():
    import vmem_sgpr_hazards as H
    # loop head at L0: the back-edge's block ends with a restore 2 wait states before the load
    loop = ["0000000000001000 <k>:",
            "\ts_mov_b32 s0, 0",
            "\ts_nop 7",
            "",
            "0000000000001010 <L0>:",
            "\tbuffer_load_dwordx4 v[0:3], v2, s[0:3], 0 offen sc1",
            "\ts_nop 7",
            "\tv_readlane_b32 s2, v9, 3",
            "\ts_cbranch_scc1 L0",
            "\ts_endpgm"]
    found = H.scan(loop)
    assert len(found) == 1 and found[0][1].startswith("v_readlane_b32 s2") and found[0][3] == 1
    # an unconditional branch ends its block: the instruction above the label does not fall through
    jump = ["0000000000001000 <k>:",
            "\tv_readlane_b32 s2, v9, 3",
            "\ts_branch L1",
            "",
            "0000000000001008 <L0>:",
            "\tbuffer_load_dwordx4 v[0:3], v2, s[0:3], 0 offen sc1",
            "",
            "000000000000100c <L1>:",
            "\ts_endpgm"]
    assert not H.scan(jump)


def test_disassembly_leaves_the_library_untouched():
    """objcopy without an output operand rewrites its input in place; a process that has
    the library mapped then loses its relocated pages (the CPU suite used to segfault in
    the next C++ unwind after this test)."""
    import vmem_sgpr_hazards as H
    if not os.path.exists(LIB) or shutil.which("objcopy") is None:
        pytest.skip("libfa_hip.so or objcopy missing")
    before = os.stat(LIB)
    H.disassemble(LIB)
    after = os.stat(LIB)
    assert (before.st_mtime_ns, before.st_ino, before.st_size) == (after.st_mtime_ns, after.st_ino, after.st_size)


def test_asm_sum_loads_are_not_read_before_their_wait():
    # the compiler does not know the asm loads are in flight: a copy of their destination
    # registers before the kernel's vmcnt wait would take the old contents (a round-6
    # experiment that carried such loads across the loop's back edge got wrong dQ)
    import vmem_sgpr_hazards as H
    if not os.path.exists(LIB):
        pytest.skip("libfa_hip.so not built")
    if shutil.which("objcopy") is None or not os.path.exists(os.path.join(H.LLVM, "llvm-objdump")):
        pytest.skip("binutils / ROCm llvm tools missing")
    lines = H.disassemble(LIB)
    assert sum(1 for l in lines if H.ASM_LOAD.match(l.strip().split("//")[0].strip())) >= 18, \
        "bwd_fused's asm sum loads were not found"
    found = H.scan_asm_loads(lines)
    assert not found, "\n".join(f"{f}: {a} -> {b}" for f, a, b in found[:10])


def test_asm_load_checker_sees_early_reads():
    import vmem_sgpr_hazards as H
    body = ["0000000000001000 <_ZN2fa9bwd_fusedE>:",
            "\tbuffer_load_dwordx4 v[4:7], v2, s[0:3], 0 offen sc1",
            "\tv_mfma_f32_32x32x16_bf16 v[8:23], v[0:3], v[24:27], v[8:23]",
            "\tv_mov_b32_e32 v30, v5",
            "\ts_waitcnt vmcnt(0)"]
    found = H.scan_asm_loads(body)
    assert len(found) == 1 and found[0][2].startswith("v_mov_b32_e32 v30, v5")
    ok = body[:3] + ["\ts_waitcnt vmcnt(0)", "\tv_mov_b32_e32 v30, v5"]
    assert not H.scan_asm_loads(ok)
    clobber = body[:2] + ["\tv_mov_b32_e32 v6, 0", "\ts_waitcnt vmcnt(0)"]
    assert len(H.scan_asm_loads(clobber)) == 1
