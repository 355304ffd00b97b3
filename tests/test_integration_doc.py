"""INTEGRATION.md's Julia binding agrees with include/snakehip.h (CPU, no GPU).

Julia is not in this image, so the binding cannot run here. This test reads
it as text instead and checks every `ccall((:sym, lib), Ret, (Types...), args...)`
against the C prototype of `sym`:
  - the symbol is declared in the header and exported by libsnakehip.so;
  - the return type is the header's (Cint for int status, Cstring for char*);
  - the argument count matches, and each Julia type has the C argument's
    width and signedness (pointers: the pointee's);
  - an `Array{T}`/`Vector{T}`/`Matrix{T}` variable passed to a `Ptr{U}`
    argument has T == U (an Int8 board buffer is not read as Float32);
  - the Julia structs TrainerCfg / TrainerStats list the C structs' fields
    in order with the same widths, and their C layout size equals the
    library's own sizeof (snk_abi_sizes; loads without a GPU).
"""
import ctypes as C
import os
import re

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
DOC = os.path.join(REPO, "INTEGRATION.md")
HEADER = os.path.join(REPO, "include", "snakehip.h")
LIB = os.path.join(REPO, "laplace-dqn-snake-game_amd", "libsnakehip.so")

# C scalar -> Julia spellings of the same width and signedness
SCALAR = {
    "int32_t": {"Int32", "Cint"}, "int64_t": {"Int64", "Clonglong"}, "uint32_t": {"UInt32", "Cuint"},
    "uint64_t": {"UInt64", "Culonglong"}, "uint8_t": {"UInt8", "Cuchar"}, "int8_t": {"Int8", "Cchar"},
    "float": {"Float32", "Cfloat"}, "double": {"Float64", "Cdouble"}, "int": {"Int32", "Cint"},
    "void": {"Cvoid", "Nothing"},
}
HANDLES = {"snk_env", "snk_replay", "snk_dqn", "snk_trainer", "snk_comm", "snk_laplace"}
STRUCTS = {"snk_trainer_cfg_t": "TrainerCfg", "snk_trainer_stats_t": "TrainerStats"}
WIDTH = {"Int8": 1, "UInt8": 1, "Int32": 4, "UInt32": 4, "Float32": 4, "Int64": 8, "UInt64": 8, "Float64": 8}


def _balanced(s: str, i: int) -> int:
    """Index just past the bracket group opening at s[i]."""
    pairs = {"(": ")", "{": "}", "[": "]"}
    stack = [pairs[s[i]]]
    j = i + 1
    while stack:
        c = s[j]
        if c in pairs:
            stack.append(pairs[c])
        elif c == stack[-1]:
            stack.pop()
        j += 1
    return j


def _split_top(s: str) -> list[str]:
    """Split on commas outside brackets."""
    out, depth, cur = [], 0, ""
    for c in s:
        if c in "({[":
            depth += 1
        elif c in ")}]":
            depth -= 1
        if c == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += c
    if cur.strip():
        out.append(cur.strip())
    return out


def header_protos() -> dict:
    """name -> (return C type, [param C types]) from snakehip.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    protos = {}
    for m in re.finditer(r"^\s*((?:const\s+)?[\w]+\s*\**)\s*(snk_\w+)\s*\(([^)]*)\)\s*;", txt, re.M):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        ps = [] if params.strip() in ("", "void") else [p.strip() for p in params.split(",")]
        types = []
        for p in ps:
            p = re.sub(r"\b\w+$", "", p).strip() if not p.endswith("*") else p   # drop the parameter name
            types.append(" ".join(p.replace("*", " * ").split()))
        protos[name] = (" ".join(ret.replace("*", " * ").split()), types)
    return protos


def header_struct(cname: str) -> list[tuple[str, str]]:
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    m = re.search(r"typedef struct \{([^}]*)\}\s*" + cname + ";", txt)
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        ctype, names = decl.split(None, 1)
        for n in names.split(","):
            fields.append((n.strip(), ctype))
    return fields


def julia_block() -> str:
    doc = open(DOC).read()
    m = re.search(r"```julia\n(module SnakeHIP.*?)```", doc, re.S)
    assert m, "INTEGRATION.md has no `module SnakeHIP` julia block"
    return m.group(1) + "\n" + "\n".join(re.findall(r"```julia\n(.*?)```", doc, re.S)[1:])


def _jl_ok(ctype: str, jtype: str) -> bool:
    """Does Julia type `jtype` bind C parameter type `ctype`?"""
    t = ctype.replace("const ", "").strip()
    stars = t.count("*")
    base = t.replace("*", "").strip()
    if stars == 0:
        if base in HANDLES:
            return jtype == "Ptr{Cvoid}"
        return jtype in SCALAR.get(base, set())
    m = re.fullmatch(r"(Ptr|Ref)\{(.*)\}", jtype)
    if not m:
        return False
    inner = m.group(2)
    if stars == 1:
        if base in HANDLES:            # snk_env * (out handle)
            return inner == "Ptr{Cvoid}"
        if base in STRUCTS:
            return inner == STRUCTS[base]
        if base == "void":             # untyped buffer (snk_laplace_get, memcpy): any element type
            return inner == "Cvoid" or inner in WIDTH
        return inner in SCALAR[base]
    if stars == 2:                     # float ** / void ** (out pointers)
        m2 = re.fullmatch(r"Ptr\{(.*)\}", inner)
        return bool(m2) and (m2.group(1) in SCALAR[base] or (base == "void" and m2.group(1) == "Cvoid"))
    return False


def ccalls(src: str):
    """Yield (name, ret, [types], [args], position) of every ccall in src."""
    for m in re.finditer(r"ccall\(", src):
        i = m.end() - 1
        j = _balanced(src, i)
        parts = _split_top(src[i + 1:j - 1])
        sym = re.fullmatch(r"\(:(\w+),\s*lib\)", parts[0])
        assert sym, f"ccall without (:sym, lib): {parts[0]}"
        tup = parts[2]
        assert tup.startswith("(") and tup.endswith(")"), tup
        types = _split_top(tup[1:-1])
        yield sym.group(1), parts[1], types, parts[3:], m.start()


def test_every_ccall_matches_the_header():
    protos = header_protos()
    src = julia_block()
    lib = C.CDLL(LIB)
    seen = 0
    for name, ret, types, args, _ in ccalls(src):
        assert name in protos, f"{name}: not declared in snakehip.h"
        assert hasattr(lib, name), f"{name}: not exported by libsnakehip.so"
        cret, cparams = protos[name]
        assert (ret == "Cstring") if cret == "const char *" else ret in ("Cint", "Int32"), (name, ret, cret)
        assert len(types) == len(cparams), f"{name}: {len(types)} Julia types for {len(cparams)} C parameters"
        assert len(args) == len(cparams), f"{name}: {len(args)} arguments for {len(cparams)} parameters"
        for k, (jt, ct) in enumerate(zip(types, cparams)):
            assert _jl_ok(ct, jt), f"{name} argument {k + 1}: Julia {jt} does not bind C `{ct}`"
        seen += 1
    assert seen >= 35, seen


def test_arrays_passed_to_pointers_have_the_pointee_type():
    """`out = Array{Float32}(...)` handed to a Ptr{Int8} argument is the
    round-2 defect this guards against."""
    src = julia_block()
    decl = [(m.start(), m.group(1), m.group(2))
            for m in re.finditer(r"\b(\w+)\s*=\s*(?:Array|Vector|Matrix)\{(\w+)\}\(", src)]
    checked = 0
    for name, _, types, args, pos in ccalls(src):
        for jt, a in zip(types, args):
            m = re.fullmatch(r"Ptr\{(\w+)\}", jt)
            if not m or not re.fullmatch(r"\w+", a):
                continue
            prior = [d for d in decl if d[1] == a and d[0] < pos]
            if not prior:
                continue
            elt = prior[-1][2]
            assert m.group(1) in (elt, "Cvoid"), f"{name}: Array{{{elt}}} `{a}` passed as {jt}"
            checked += 1
    assert checked >= 8, checked


def _julia_struct(src: str, name: str) -> list[tuple[str, str]]:
    m = re.search(r"struct " + name + r"\b[^\n]*\n(.*?)\nend", src, re.S)
    assert m, name
    return re.findall(r"(\w+)::(\w+)", m.group(1))


def _c_layout(widths: list[int]) -> int:
    off, align = 0, 1
    for w in widths:
        off = (off + w - 1) // w * w + w
        align = max(align, w)
    return (off + align - 1) // align * align


@pytest.mark.parametrize("cname", sorted(STRUCTS))
def test_julia_structs_match_the_c_structs(cname):
    src = julia_block()
    jfields = _julia_struct(src, STRUCTS[cname])
    cfields = header_struct(cname)
    assert [f for f, _ in jfields] == [f for f, _ in cfields], (jfields, cfields)
    for (f, jt), (_, ct) in zip(jfields, cfields):
        assert jt in SCALAR[ct], f"{cname}.{f}: Julia {jt} vs C {ct}"
    lib = C.CDLL(LIB)
    cfg, st = C.c_int64(0), C.c_int64(0)
    assert lib.snk_abi_sizes(C.byref(cfg), C.byref(st)) == 0
    size = {"snk_trainer_cfg_t": cfg.value, "snk_trainer_stats_t": st.value}[cname]
    assert _c_layout([WIDTH[jt if jt in WIDTH else {"Cint": "Int32"}[jt]] for _, jt in jfields]) == size
    assert f"Int32({size})" in src, f"the Julia {STRUCTS[cname]} constructor must set struct_size = {size}"


def test_python_structs_match_the_library():
    import snake_amd._lib as L
    lib = C.CDLL(LIB)
    cfg, st = C.c_int64(0), C.c_int64(0)
    assert lib.snk_abi_sizes(C.byref(cfg), C.byref(st)) == 0
    assert C.sizeof(L.TrainerCfg) == cfg.value and C.sizeof(L.TrainerStats) == st.value
    assert L.TrainerCfg().struct_size == cfg.value and L.TrainerStats().struct_size == st.value
    assert [f for f, _ in L.TrainerCfg._fields_] == [f for f, _ in header_struct("snk_trainer_cfg_t")]
    assert [f for f, _ in L.TrainerStats._fields_] == [f for f, _ in header_struct("snk_trainer_stats_t")]
