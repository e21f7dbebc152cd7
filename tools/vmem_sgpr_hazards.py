"""Scan the gfx950 code object inside libfa_hip.so for one hazard the compiler's
hazard recognizer does not see through inline asm: a VALU instruction that writes an
SGPR (v_readlane_b32 restoring a spilled SGPR, v_readfirstlane_b32, a VOP3 compare
or carry-out) followed, within 5 wait states, by a vector-memory instruction that
reads that SGPR as its buffer descriptor or scalar base/offset.  The ISA requires 5
wait states between the two; the asm buffer loads of fa_bwd.hip carry an `s_nop 4`
only where a spill restore can land in front of them (the LDS-DMA descriptors), so
this check guards the others.

The walk is branch-aware: backwards from each vector-memory instruction along the
fall-through path and, at every basic-block label it reaches (llvm-objdump
`--symbolize-operands`), also into the tail of every block that branches there
(taken `s_cbranch_*` / `s_branch`, including loop back-edges).  Each instruction
counts one wait state, `s_nop N` counts N + 1.

The library is only read: the fat binary is extracted with `objcopy --dump-section`
into a scratch output file.  (Without the output operand objcopy rewrites its input
in place, which truncates the file under any process that has it mapped: the kernel
then drops that process's relocated private pages and its next C++ unwind faults.)

A second check (scan_asm_loads): the destination registers of bwd_fused's asm
running-sum loads are not read, copied or overwritten before a vmcnt wait.

Usage: python tools/vmem_sgpr_hazards.py [libfa_hip.so]   (exit 1 if any is found)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
VMEM = re.compile(r"^(buffer_|global_|scratch_|flat_)\w+")
SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
VALU_SDST = re.compile(r"^(v_readlane_b32|v_readfirstlane_b32)\s+s(\d+)\b|^v_\w+_e64\s+(?:v\[?\d+(?::\d+\])?,\s*)?s\[(\d+):(\d+)\]")
HEADER = re.compile(r"^[0-9a-f]+ <(\S+)>:")
LABEL = re.compile(r"^L\d+$")
BRANCH = re.compile(r"^(s_cbranch_\w+|s_branch)\s+(L\d+)\b")
NO_FALLTHROUGH = re.compile(r"^(s_branch|s_endpgm|s_setpc_b64)\b")


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble(lib):
    """Every translation unit's gfx950 code object (the .hip_fatbin section holds one
    offload bundle per source file), disassembled with symbolized branch targets."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "scratch.so")],
                       check=True)
        blob = open(fat, "rb").read()
        starts, i = [], blob.find(MAGIC)
        while i >= 0:
            starts.append(i)
            i = blob.find(MAGIC, i + 1)
        for n, a in enumerate(starts):
            z = starts[n + 1] if n + 1 < len(starts) else len(blob)
            part, dev = os.path.join(d, f"b{n}.bin"), os.path.join(d, f"b{n}.o")
            open(part, "wb").write(blob[a:z])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            f"--targets={TARGET}", f"--output={dev}"], check=True)
            out += subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--symbolize-operands", dev],
                                  check=True, capture_output=True, text=True).stdout.split("\n")
    return out


def sregs(text):
    r = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            r.add(int(m.group(3)))
        else:
            r.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return r


def _functions(lines):
    """[(name, instructions, {instruction index: [labels starting there]})]."""
    funcs, name, ins, labels = [], None, [], {}
    for line in lines:
        m = HEADER.match(line)
        if m:
            if LABEL.match(m.group(1)):
                labels.setdefault(len(ins), []).append(m.group(1))
                continue
            if name is not None:
                funcs.append((name, ins, labels))
            name, ins, labels = m.group(1), [], {}
            continue
        t = line.strip().split("//")[0].strip()
        if t and not t.endswith(":"):
            ins.append(t)
    if name is not None:
        funcs.append((name, ins, labels))
    return funcs


def _wait_states(t):
    n = re.match(r"^s_nop\s+(?:0x)?([0-9a-f]+)", t)
    return int(n.group(1), 16 if "0x" in t else 10) + 1 if n else 1


def scan(lines):
    found = []
    for func, ins, labels in _functions(lines):
        sources = {}  # label -> indices of the branches that target it
        for i, t in enumerate(ins):
            b = BRANCH.match(t)
            if b:
                sources.setdefault(b.group(2), []).append(i)

        def preds(k):
            # instructions that can execute right before instruction k
            out = [s for lab in labels.get(k, []) for s in sources.get(lab, [])]
            if k - 1 >= 0 and not NO_FALLTHROUGH.match(ins[k - 1]):
                out.append(k - 1)
            return out

        for i, t in enumerate(ins):
            if not VMEM.match(t):
                continue
            srcs = sregs(t.split(None, 1)[1] if " " in t else "")
            if not srcs:
                continue
            # depth-first over predecessors: (instruction index, wait states between it and t)
            stack, seen, hit = [(p, 0) for p in preds(i)], set(), None
            while stack:
                j, ws = stack.pop()
                if ws >= 5 or (j, ws) in seen:
                    continue
                seen.add((j, ws))
                w = VALU_SDST.match(ins[j])
                if w:
                    dst = {int(w.group(2))} if w.group(2) else set(range(int(w.group(3)), int(w.group(4)) + 1))
                    if dst & srcs:
                        hit = (func, ins[j], t, ws)
                        break
                nws = ws + _wait_states(ins[j])
                stack += [(p, nws) for p in preds(j)]
            if hit:
                found.append(hit)
    return found


VGPR = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
ASM_LOAD = re.compile(r"^buffer_load_dwordx4 (v\[\d+:\d+\]), .*\bsc1\b")
STORE = re.compile(r"^(buffer_store|global_store|ds_write|scratch_store|flat_store)")


def vregs(text):
    r = set()
    for m in VGPR.finditer(text):
        if m.group(3) is not None:
            r.add(int(m.group(3)))
        else:
            r.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return r


def scan_asm_loads(lines, func_filter="bwd_fused"):
    """The asm running-sum loads of bwd_fused (`buffer_load_dwordx4 ... sc1`, issued by
    load16_sc1_asm) are hidden from the compiler's waitcnt model: it treats their
    destination registers as written at issue.  A copy, read or overwrite of those
    registers before the kernel's own `s_waitcnt vmcnt` would see the old contents.
    Walks the fall-through path from each such load to the first vmcnt wait (or branch);
    returns [(function, load, offending instruction)]."""
    found = []
    for func, ins, _labels in _functions(lines):
        if func_filter not in func:
            continue
        for i, t in enumerate(ins):
            m = ASM_LOAD.match(t)
            if not m:
                continue
            dst = vregs(m.group(1))
            for u in ins[i + 1:]:
                if (u.startswith("s_waitcnt") and "vmcnt" in u) or u.startswith(("s_branch", "s_cbranch", "s_endpgm")):
                    break
                op, _, rest = u.partition(" ")
                if STORE.match(op):
                    srcs, dsts = vregs(rest), set()
                else:
                    first, _, others = rest.partition(",")
                    srcs, dsts = vregs(others), (set() if op.startswith("buffer_load") else vregs(first))
                if (srcs | dsts) & dst:
                    found.append((func, t, u))
                    break
    return found


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flashattention.jl_amd", "libfa_hip.so")
    lines = disassemble(lib)
    found = scan(lines)
    for f, a, b, ws in found:
        print(f"{f}: {a}  ->  {b}  ({ws} wait states)")
    print(f"{len(found)} VALU-SGPR -> VMEM hazards")
    early = scan_asm_loads(lines)
    for f, a, b in early:
        print(f"{f}: {a}  ->  {b}  (before its vmcnt wait)")
    print(f"{len(early)} asm-load results touched before their wait")
    return 1 if found or early else 0


if __name__ == "__main__":
    sys.exit(main())
