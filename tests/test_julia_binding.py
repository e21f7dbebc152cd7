"""CPU check of the Julia side of the boundary (no Julia in this image, so the
binding is not executed here): every ``ccall`` in
flashattention.jl_amd/julia/FlashAttentionHIP.jl names a symbol declared in
include/fa_hip.h with the same return type and the same argument types, in
order, and every declared entry point has a Julia binding."""
from __future__ import annotations

import os
import re

import pytest

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


# ---- method coverage: the reference's own calling pattern ----
JL_TYPES = ["Float32", "Float64", "Float16", "AMDGPU.BFloat16"]


def _methods(name: str):
    """(arg types, type vars) of every `function name(...) where {...}` in the binding."""
    s = open(JL).read()
    out = []
    for mt in re.finditer(r"function\s+" + re.escape(name) + r"\(", s):
        inner = _tuple_after(s, mt.end() - 1)
        positional = inner.split(";")[0]
        args = [a.strip() for a in re.split(r",(?![^{]*\})", positional) if a.strip()]
        rest = s[mt.end() - 1 + len(inner) + 2:]
        wh = re.match(r"\s*where\s*\{([^}]*)\}", rest)
        tvars = [t.strip() for t in wh.group(1).split(",")] if wh else []
        out.append(([a.split("::", 1)[1].strip() if "::" in a else "Any" for a in args], tvars))
    return out


def _matches(sig, tvars, actual):
    """Julia-style dispatch check of concrete `ROCArray{X,3}` / `Int` arguments."""
    bind = {}
    for decl, act in zip(sig, actual):
        if decl in ("Any", act):
            continue
        dm = re.fullmatch(r"ROCArray\{(\w+(?:\.\w+)?),\s*(\w+)\}", decl)
        am = re.fullmatch(r"ROCArray\{([\w.]+),(\d+)\}", act)
        if not dm or not am:
            return False
        el, nd = dm.groups()
        if nd != am.group(2) and nd not in tvars:
            return False
        if el in tvars:
            if bind.setdefault(el, am.group(1)) != am.group(1):
                return False
        elif el != am.group(1):
            return False
    return len(sig) == len(actual)


@pytest.mark.parametrize("name,extra", [("dense_fa!", []), ("circulant_fa!", ["Int"])])
def test_inplace_methods_accept_every_lm_eltype(name, extra):
    """dense_fa!(O, l, m, Q, K, V) with `l = similar(Q, N, 1, B)` (src/dense.jl:11-15: l and m
    of Q's element type) and with Float32 l, m must both reach a HIP method for every
    supported element type T."""
    methods = _methods(name)
    assert methods, name
    for T in JL_TYPES:
        for S in sorted({T, "Float32"}):
            A = lambda e: f"ROCArray{{{e},3}}"
            actual = [A(T), A(S), A(S), A(T), A(T), A(T)] + extra
            assert any(_matches(sig, tv, actual) for sig, tv in methods), f"{name}: no method for T={T}, l/m {S}"


def test_backward_accepts_every_lm_eltype():
    methods = _methods("dense_fa_backward")
    for T in JL_TYPES:
        for S in sorted({T, "Float32"}):
            A = lambda e: f"ROCArray{{{e},3}}"
            actual = [A(T)] * 5 + [A(S), A(S)]
            assert any(_matches(sig, tv, actual) for sig, tv in methods), f"no backward method for T={T}, l/m {S}"


def test_no_per_call_device_workspace():
    """Workspaces come from the per-(device, stream) cache; the only device allocation of
    scratch bytes is inside `workspace` itself."""
    s = open(JL).read()
    allocs = [m.start() for m in re.finditer(r"ROCArray\{UInt8\}\(undef", s)]
    fn = s.index("function workspace(")
    end = s.index("\nend", fn)
    assert allocs and all(fn < a < end for a in allocs), "scratch allocated outside workspace()"
    for entry in ("fa_dense_fwd_ws", "fa_dense_bwd,", "fa_windowed_fwd,", "fa_windowed_bwd,", "fa_softmax,"):
        i = s.index("(:" + entry)
        body = s[s.rfind("\nfunction", 0, i):i]
        assert "workspace(nws)" in body, entry
