"""Source lint of the HIP sources (CPU, no GPU).

Round 4 shipped a wrong-result regression (55737c8): `__shared__ float
a3red[8][4][4]` was declared inside a lambda of conv_h3f_kernel. The lambda
was instantiated once per row-tile count, so waves with 3 and 4 row tiles
reduced into DIFFERENT arrays and dense_h3_kernel's per-sample scale read
uninitialised LDS; one call could pass and the next fail. A `__shared__`
array inside a lambda or a device helper is one array per instantiation of
that function, never the kernel's. This test fails on any `__shared__`
declared outside the body of a `__global__` function itself (nested plain
blocks of the kernel are fine): always inside a lambda, and inside a device
helper unless its line carries the marker `lds: one per kernel` (a comment
stating that the helper is instantiated once per kernel, or that its
instantiations never share the array, e.g. the two bodies of a paired launch).

It also keeps kernel-selection environment variables out of the shipping
library: `getenv` may appear only inside `#ifdef SNK_*_MEASURE` /
`SNK_ENV_CLOCKS` blocks (a stray variable must not
change the production arithmetic).
"""
import glob
import os
import re

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CSRC = os.path.join(REPO, "laplace-dqn-snake-game_amd", "csrc")
CONTROL = {"if", "for", "while", "switch", "else", "do", "catch", "try", "return"}


def strip_comments(src: str) -> str:
    """Comments and string/char literals -> spaces (newlines kept, so line numbers hold)."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            out.append(" " * (j - i))
            i = j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append(re.sub(r"[^\n]", " ", src[i:j]))
            i = j
        elif c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(c + " " * (min(j, n) - i - 1) + (c if j < n else ""))
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def scope_kind(header: str, enclosing: list) -> str:
    """Kind of the scope a '{' opens, from the statement text before it."""
    h = " ".join(header.split())
    if re.search(r"\[[\s&=\w,*]*\]\s*(\([^()]*(\([^()]*\)[^()]*)*\))?\s*(mutable\s*)?"
                 r"(__attribute__\s*\(\(.*\)\)\s*)?(->\s*[\w:<>,\s]+)?$", h):
        return "lambda"
    first = re.match(r"[A-Za-z_]\w*", h)
    if first and first.group(0) in CONTROL:
        return "block"
    in_func = any(k in ("kernel", "function", "lambda") for k in enclosing)
    if not in_func and re.search(r"\)\s*(const\s*)?(noexcept\s*)?(->\s*[\w:<>,\s]+)?$", h):
        return "kernel" if "__global__" in h else "function"
    if re.search(r"\b(namespace|struct|class|union|enum)\b", h) or h.startswith('extern "C"') or h == "extern":
        return "ns"
    return "block"


MARK = "lds: one per kernel"


def shared_outside_kernels(path: str):
    raw = open(path).read().split("\n")
    src = strip_comments("\n".join(raw))
    stack, bad, last = [], [], 0
    i = 0
    while i < len(src):
        c = src[i]
        if c == "#":   # preprocessor line: not a statement boundary
            j = src.find("\n", i)
            i = len(src) if j < 0 else j
            last = i
            continue
        if c == "{":
            stack.append(scope_kind(src[last:i], stack))
            last = i + 1
        elif c == "}":
            if stack:
                stack.pop()
            last = i + 1
        elif c == ";":
            last = i + 1
        elif src.startswith("__shared__", i) and not re.match(r"\w", src[i - 1] if i else " "):
            owner = next((k for k in reversed(stack) if k in ("kernel", "function", "lambda")), None)
            line = src.count("\n", 0, i) + 1
            if owner != "kernel" and not (owner == "function" and MARK in raw[line - 1]):
                bad.append(f"{os.path.basename(path)}:{line}: __shared__ inside a {owner or 'namespace scope'}")
        i += 1
    return bad


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp")))


def test_lint_sees_the_sources():
    assert len(sources()) >= 15


def test_lint_catches_shared_in_lambda(tmp_path):
    f = tmp_path / "x.hip"
    f.write_text("""
template <int N> __device__ float helper() { __shared__ float h[4]; return h[0]; }
__device__ float helper2() { __shared__ float h[4]; return h[0]; }   // lds: one per kernel
__global__ void k(float *p) {
    __shared__ float ok[4];
    if (p) { __shared__ float ok2[2]; }
    auto lam = [&](int t) __attribute__((always_inline)) { __shared__ float bad[8]; return bad[t]; };
    auto tile = [&](auto ic) { __shared__ int bad2; };
}
""")
    bad = shared_outside_kernels(str(f))
    assert len(bad) == 3, bad
    assert "function" in bad[0] and "lambda" in bad[1] and "lambda" in bad[2]


def test_no_shared_outside_kernel_bodies():
    bad = [b for p in sources() for b in shared_outside_kernels(p)]
    assert not bad, "__shared__ must be declared in the __global__ body itself:\n" + "\n".join(bad)


def test_no_getenv_in_shipping_library():
    bad = []
    for p in sources():
        depth_meas = []
        for ln, line in enumerate(strip_comments(open(p).read()).split("\n"), 1):
            s = line.strip()
            if s.startswith("#if"):
                depth_meas.append(bool(re.search(r"SNK_\w*MEASURE|SNK_ENV_CLOCKS|SNK_\w*CLOCKS", s)))
            elif s.startswith("#else") and depth_meas:
                depth_meas[-1] = False
            elif s.startswith("#endif") and depth_meas:
                depth_meas.pop()
            elif "getenv" in s and not any(depth_meas):
                bad.append(f"{os.path.basename(p)}:{ln}: {s}")
    assert not bad, "getenv outside measurement builds:\n" + "\n".join(bad)
