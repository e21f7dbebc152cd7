"""CPU check of the Julia side of the boundary (no Julia in this image, so the
binding is not executed here): every ``ccall`` in
flashattention.jl_amd/julia/FlashAttentionHIP.jl names a symbol declared in
include/fa_hip.h with the same return type and the same argument types, in
order, and every declared entry point has a Julia binding."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "flashattention.jl_amd", "julia", "FlashAttentionHIP.jl")
HDR = os.path.join(ROOT, "include", "fa_hip.h")

C2JL = {"int": "Cint", "int64_t": "Int64", "size_t": "Csize_t", "float": "Cfloat",
        "void*": "Ptr{Cvoid}", "float*": "Ptr{Float32}", "int64_t*": "Ptr{Int64}",
        "char*": "Cstring", "int*": "Ptr{Cint}", "void": "()"}


def _norm_c(t: str) -> str:
    t = t.replace("const", "").strip()
    t = re.sub(r"\s+\w+$", "", t) if re.search(r"[\w\*]\s+\w+$", t) else t   # drop the parameter name
    t = re.sub(r"\s*\*\s*", "*", t).strip()
    return C2JL[t]


def header_prototypes():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for ret, name, args in re.findall(r"^\s*((?:const\s+)?\w+\s*\**)\s*(fa_\w+)\s*\(([^)]*)\)\s*;", src, flags=re.M | re.S):
        args = " ".join(args.split())
        types = [] if args in ("", "void") else [_norm_c(a) for a in args.split(",")]
        out[name] = (_norm_c(ret.replace(" ", "") if "*" in ret else ret.strip()), types)
    return out


def _tuple_after(s: str, i: int) -> str:
    assert s[i] == "("
    depth = 0
    for j in range(i, len(s)):
        depth += s[j] == "("
        depth -= s[j] == ")"
        if depth == 0:
            return s[i + 1:j]
    raise AssertionError("unbalanced")


def julia_ccalls():
    s = open(JL).read()
    out = []
    for mt in re.finditer(r"ccall\(\(:(fa_\w+),\s*libfa_hip\),\s*(\w+),\s*", s):
        name, ret = mt.group(1), mt.group(2)
        inner = _tuple_after(s, mt.end())
        types = [t.strip() for t in re.split(r",(?![^{]*\})", inner) if t.strip()]
        out.append((name, ret, types))
    return out


def test_every_ccall_matches_the_header():
    protos = header_prototypes()
    calls = julia_ccalls()
    assert len(calls) >= 12
    for name, ret, types in calls:
        assert name in protos, f"{name}: not declared in fa_hip.h"
        pret, ptypes = protos[name]
        assert ret == pret, f"{name}: Julia returns {ret}, header {pret}"
        assert types == ptypes, f"{name}: Julia args {types} != header {ptypes}"


def test_every_declared_entry_point_is_bound_in_julia():
    bound = {c[0] for c in julia_ccalls()}
    missing = sorted(set(header_prototypes()) - bound)
    assert not missing, f"no Julia binding for {missing}"
