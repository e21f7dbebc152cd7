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
    """Workspaces come from the per-device cache; the only device allocation of scratch
    bytes is inside `with_workspace` itself, and every entry point with a workspace
    argument makes its call inside `with_workspace(nws) do ws`."""
    s = open(JL).read()
    allocs = [m.start() for m in re.finditer(r"ROCArray\{UInt8\}\(undef", s)]
    fn = s.index("function with_workspace(")
    end = s.index("\nend", fn)
    assert allocs and all(fn < a < end for a in allocs), "scratch allocated outside with_workspace()"
    for entry in ("fa_dense_fwd_ws", "fa_dense_bwd,", "fa_dense_bwd_handoff_status", "fa_windowed_fwd,",
                  "fa_windowed_bwd,", "fa_softmax,"):
        i = s.index("(:" + entry)
        body = s[s.rfind("with_workspace(nws) do ws", 0, i):i]
        assert body and "\n    end\n" not in body and "\nfunction" not in body, entry


def test_workspace_cache_is_per_device_and_stream_ordered():
    """One scratch buffer per device (not per task-local stream), handed
    between streams by an event, and a public way to free it."""
    s = open(JL).read()
    assert "const _WS = Dict{Int,Scratch}()" in s
    fn = s[s.index("function with_workspace("):]
    fn = fn[:fn.index("\nend\n")]
    assert "hipStreamWaitEvent" in fn and "hipEventRecord" in fn
    assert fn.index("r = f(e.buf)") < fn.index("hipEventRecord")
    assert "function free_workspaces!()" in s


# ---- dispatch: every call the reference's own code makes on ROCArrays
# resolves to ONE most specific method, and that method is a HIP one.
# The reference's generic methods, as declared (type variable T shared by every argument):
REFERENCE_GENERICS = {
    # /root/reference/src/dense.jl:21-27
    "dense_fa!": (["AbstractArray{T,3}"] * 6, ["T"]),
    # /root/reference/src/dense.jl:104-111
    "dense_fa_backward": (["AbstractArray{T,3}"] * 7, ["T"]),
    # /root/reference/src/circulant.jl:9-16
    "circulant_fa!": (["AbstractArray{T,3}"] * 6 + ["Int"], ["T"]),
}


def _parse_arg(decl):
    m = re.fullmatch(r"(ROCArray|AbstractArray)\{([\w.]+),\s*(\w+)\}", decl)
    return (m.group(1), m.group(2), m.group(3)) if m else ("Other", decl, None)


def _applies(sig, tvars, actual):
    """Concrete actual types `ROCArray{E,3}` / `Int` against a declared signature."""
    bind = {}
    for decl, act in zip(sig, actual):
        kind, el, nd = _parse_arg(decl)
        if kind == "Other":
            if el != act:
                return False
            continue
        am = re.fullmatch(r"ROCArray\{([\w.]+),(\d+)\}", act)
        if not am or (nd not in tvars and nd != am.group(2)):
            return False
        if el in tvars:
            if bind.setdefault(el, am.group(1)) != am.group(1):
                return False
        elif el != am.group(1):
            return False
    return len(sig) == len(actual)


def _subtype(x, y):
    """Signature x <: signature y (every tuple x admits, y admits) for these forms:
    ROCArray <: AbstractArray; an element type y fixes must be fixed equally in x; the
    positions sharing one of y's type variables must share one of x's, or one type."""
    (sx, tx), (sy, ty) = x, y
    if len(sx) != len(sy):
        return False
    groups = {}
    for a, b in zip(sx, sy):
        ka, ea, na = _parse_arg(a)
        kb, eb, nb = _parse_arg(b)
        if kb == "Other" or ka == "Other":
            if a != b:
                return False
            continue
        if kb == "ROCArray" and ka != "ROCArray":
            return False
        if nb not in ty and na != nb:
            return False
        if eb in ty:
            groups.setdefault(eb, set()).add(("var", ea) if ea in tx else ("type", ea))
        elif ea != eb:
            return False
    return all(len(g) == 1 for g in groups.values())


@pytest.mark.parametrize("name", sorted(REFERENCE_GENERICS))
def test_dispatch_has_a_most_specific_hip_method(name):
    """For T in the supported element types, the reference's own calling pattern (every
    argument of type T: l, m from `similar(Q, N, 1, B)`, src/dense.jl:12-13) and the C
    ABI's (Float32 l, m): among the applicable methods — the HIP ones and the reference's
    generic one — exactly one is a subtype of all the others, and it is a HIP method.
    (Julia's own specificity rules could resolve more; this condition is sufficient
    for no MethodError ambiguity.)"""
    ref = REFERENCE_GENERICS[name]
    hip = _methods(name)
    assert len(hip) >= 4, name
    extra = ["Int"] if name == "circulant_fa!" else []
    n_lm = 5 if name == "dense_fa_backward" else 1
    for T in JL_TYPES:
        for S in sorted({T, "Float32"}):
            A = lambda e: f"ROCArray{{{e},3}}"
            if name == "dense_fa_backward":
                actual = [A(T)] * 5 + [A(S), A(S)]
            else:
                actual = [A(T), A(S), A(S), A(T), A(T), A(T)] + extra
            cands = [("ref", ref)] + [("hip", m) for m in hip]
            app = [(k, m) for k, m in cands if _applies(m[0], m[1], actual)]
            assert any(k == "hip" for k, _ in app), f"{name}: no HIP method for T={T}, l/m {S}"
            best = [(k, m) for k, m in app if all(_subtype(m, o) for _, o in app)]
            assert len(best) == 1 and best[0][0] == "hip", \
                f"{name} T={T} l/m {S}: no unique most specific HIP method among {[m for _, m in app]}"


def test_dispatch_checker_sees_the_round5_ambiguity():
    """The round-5 layout (Float32-l/m method + free-S method, no same-T method) is
    ambiguous with the reference's generic method for an all-Float32 call."""
    ref = REFERENCE_GENERICS["dense_fa!"]
    a = (["ROCArray{T,3}", "ROCArray{Float32,3}", "ROCArray{Float32,3}"] + ["ROCArray{T,3}"] * 3, ["T"])
    b = (["ROCArray{T,3}", "ROCArray{S,3}", "ROCArray{S,3}"] + ["ROCArray{T,3}"] * 3, ["T", "S"])
    actual = ["ROCArray{Float32,3}"] * 6
    app = [m for m in (ref, a, b) if _applies(m[0], m[1], actual)]
    assert len(app) == 3
    assert not [m for m in app if all(_subtype(m, o) for o in app)]
