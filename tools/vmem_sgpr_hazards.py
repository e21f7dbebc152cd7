"""Scan the gfx950 code object inside libfa_hip.so for one hazard the compiler's
hazard recognizer does not see through inline asm: a VALU instruction that writes an
SGPR (v_readlane_b32 restoring a spilled SGPR, v_readfirstlane_b32, a VOP3 compare
or carry-out) followed, within 5 wait states, by a vector-memory instruction that
reads that SGPR as its buffer descriptor or scalar base/offset.  The ISA requires 5
wait states between the two; the asm buffer loads of fa_bwd.hip carry an `s_nop 4`
only where a spill restore can land in front of them (the LDS-DMA descriptors), so
this check guards the others.  Linear scan (the fall-through path; each instruction
counts one wait state, `s_nop N` counts N + 1).

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


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble(lib):
    """Every translation unit's gfx950 code object (the .hip_fatbin section holds one
    offload bundle per source file), disassembled."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", lib], check=True)
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
            out += subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", dev], check=True,
                                  capture_output=True, text=True).stdout.split("\n")
    return out


def sregs(text):
    r = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            r.add(int(m.group(3)))
        else:
            r.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return r


def scan(lines):
    found, func = [], "?"
    ins = []
    for line in lines:
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            func, ins = m.group(1), []
            continue
        t = line.strip().split("//")[0].strip()
        if not t or t.endswith(":"):
            continue
        ins.append(t)
        if not VMEM.match(t):
            continue
        ops = t.split(None, 1)[1] if " " in t else ""
        # SGPR operands of the memory instruction (descriptor, saddr, soffset)
        srcs = sregs(ops)
        if not srcs:
            continue
        ws = 0
        for prev in reversed(ins[:-1]):
            if ws >= 5:
                break
            w = VALU_SDST.match(prev)
            if w:
                dst = {int(w.group(2))} if w.group(2) else set(range(int(w.group(3)), int(w.group(4)) + 1))
                if dst & srcs:
                    found.append((func, prev, t, ws))
                    break
            n = re.match(r"^s_nop\s+(?:0x)?([0-9a-f]+)", prev)
            ws += int(n.group(1), 16 if "0x" in prev else 10) + 1 if n else 1
    return found


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flashattention.jl_amd", "libfa_hip.so")
    found = scan(disassemble(lib))
    for f, a, b, ws in found:
        print(f"{f}: {a}  ->  {b}  ({ws} wait states)")
    print(f"{len(found)} VALU-SGPR -> VMEM hazards")
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
