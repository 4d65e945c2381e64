"""The Go cgo shim (go/bk/krum_bk.go) checked against include/bk.h without a Go
toolchain.  Test infrastructure only.

The shim replaces getTopKRUMIndex / initialize (DistSys/krum.go:31-44,
100-166).  No Go compiler is in the image, so two checks stand in for
`go build`:

1. Names and arity: every `C.bk_*(...)` call in the shim names a function
   that bk.h declares, with as many arguments as its prototype; every
   `C.BK_*` constant and `C.bk_*` type it names is defined there.
2. Types: the shim's calls are rewritten mechanically into C (cgo's
   conversions `C.int64_t(x)`, `(*C.T)(p)`, `unsafe.Pointer(p)`, `nil`, and
   the shim's own variable declarations mapped to their C types) and compiled
   against bk.h with `gcc -fsyntax-only -Werror`, so an argument whose type no
   longer matches the prototype fails as cgo would.
"""
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(REPO, "go", "bk", "krum_bk.go")
HEADER = os.path.join(REPO, "include", "bk.h")


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _split_args(s):
    """Top-level comma split of an argument list (parentheses / brackets nest)."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    last = "".join(cur).strip()
    if last:
        out.append(last)
    return out


def _call_args(src, start):
    """The argument text of the call whose '(' is at src[start]."""
    depth = 0
    for i in range(start, len(src)):
        if src[i] == "(":
            depth += 1
        elif src[i] == ")":
            depth -= 1
            if depth == 0:
                return src[start + 1:i]
    raise ValueError("unbalanced call at %d" % start)


def header_decls(header_text):
    """bk.h -> ({function: [param, ...]}, {constant names}, {type names})."""
    h = _strip_c_comments(header_text)
    funcs = {}
    for mt in re.finditer(r"(?:^|;|\})[ \t]*([A-Za-z_][\w \t\*]*?)\b(bk_\w+)\s*\(([^;{]*?)\)\s*;", h,
                          re.S | re.M):
        params = [p for p in _split_args(" ".join(mt.group(3).split()))]
        if params == ["void"]:
            params = []
        funcs[mt.group(2)] = params
    consts = set(re.findall(r"#define\s+(BK_\w+)", h))
    for body in re.findall(r"enum\s+\w*\s*\{(.*?)\}", h, re.S):
        consts |= set(re.findall(r"\b(BK_\w+)\b\s*(?:=|,|$)", body, re.M))
    types = set(re.findall(r"typedef\s+struct\s+\w+\s+(bk_\w+)\s*;", h))
    return funcs, consts, types


def shim_calls(go_text):
    """Every C.bk_* call in the shim: [(function name, [argument text], line)]."""
    calls = []
    for mt in re.finditer(r"\bC\.(bk_\w+)\s*\(", go_text):
        args = _split_args(" ".join(_call_args(go_text, mt.end() - 1).split()))
        calls.append((mt.group(1), args, go_text.count("\n", 0, mt.start()) + 1))
    return calls


def shim_names(go_text):
    consts = set(re.findall(r"\bC\.(BK_\w+)", go_text))
    types = set(re.findall(r"\*C\.(bk_\w+)\b(?!\s*\()", go_text))
    return consts, types


def check_names(go_text, header_text):
    """Problems with the shim's names and arities against the header."""
    funcs, consts, types = header_decls(header_text)
    probs = []
    for name, args, line in shim_calls(go_text):
        if name not in funcs:
            probs.append("krum_bk.go:%d: C.%s is not declared in bk.h" % (line, name))
        elif len(args) != len(funcs[name]):
            probs.append("krum_bk.go:%d: C.%s takes %d arguments in bk.h, the shim passes %d"
                         % (line, name, len(funcs[name]), len(args)))
    c_used, t_used = shim_names(go_text)
    for k in sorted(c_used - consts):
        probs.append("C.%s is not defined in bk.h" % k)
    for t in sorted(t_used - types):
        probs.append("C.%s is not a type in bk.h" % t)
    return probs


# ---- the type check: the shim's calls as C ---------------------------------

def _go_type_to_c(t, name):
    t = t.strip()
    if t.startswith("[]C."):
        return "%s %s[1]" % (t[4:], name)
    if t.startswith("*C."):
        return "%s *%s" % (t[3:], name)
    if t.startswith("C."):
        return "%s %s" % (t[2:], name)
    if t == "unsafe.Pointer":
        return "void *%s" % name
    if t in ("int", "int64", "int32"):
        return "long long %s" % name
    raise ValueError("unmapped Go type %r" % t)


def _functions(go_text):
    """(name, parameter list, body) of each top-level func."""
    out = []
    for mt in re.finditer(r"^func\s+(?:\([^)]*\)\s*)?(\w+)\(([^)]*)\)[^{]*\{", go_text, re.M):
        depth, i = 0, mt.end() - 1
        for j in range(i, len(go_text)):
            if go_text[j] == "{":
                depth += 1
            elif go_text[j] == "}":
                depth -= 1
                if depth == 0:
                    out.append((mt.group(1), mt.group(2), go_text[i + 1:j]))
                    break
    return out


def _param_decls(params):
    """Go parameters ("n, d, f int, sel []C.int64_t, mOut *C.int64_t") ->
    {name: C declaration} for the types _go_type_to_c maps."""
    d, pending = {}, []
    for p in [x.strip() for x in params.split(",") if x.strip()]:
        parts = p.split(None, 1)
        pending.append(parts[0])
        if len(parts) == 2:  # a type closes the names collected so far
            for nm in pending:
                try:
                    d[nm] = _go_type_to_c(parts[1], nm)
                except ValueError:
                    pass
            pending = []
    return d


def _decls(text):
    """Go declarations -> {name: C declaration}."""
    d = {}
    for mt in re.finditer(r"^\s*(?:var\s+)?([A-Za-z_]\w*(?:\s*,\s*[A-Za-z_]\w*)*)\s+"
                          r"(\*C\.\w+|C\.\w+|unsafe\.Pointer|int64|int)\s*(?://.*)?$", text, re.M):
        for nm in mt.group(1).split(","):
            nm = nm.strip()
            if nm not in ("var", "return"):
                d[nm] = _go_type_to_c(mt.group(2), nm)
    for mt in re.finditer(r"\b(\w+)\s*:=\s*make\(\s*(\[\]C\.\w+)", text):
        d[mt.group(1)] = _go_type_to_c(mt.group(2), mt.group(1))
    return d


def _to_c(expr):
    e = expr
    # (*unsafe.Pointer)(p): cgo's Go view of a `const void *const *` (or `void **`)
    # parameter -- cgo drops the qualifiers, so the C view is the prototype's
    e = re.sub(r"\(\*unsafe\.Pointer\)", "(const void *const *)", e)
    e = re.sub(r"\(\*C\.(\w+)\)", r"(\1 *)", e)                              # (*C.T)(p)
    e = re.sub(r"\bC\.(int64_t|int32_t|int|double|size_t|uint32_t)\(", r"(\1)(", e)  # C.int64_t(x)
    e = re.sub(r"\bunsafe\.Pointer\(", "(void *)(", e)
    e = re.sub(r"\bC\.(\w+)", r"\1", e)
    e = re.sub(r"\bnil\b", "NULL", e)
    return e


def shim_as_c(go_text):
    """A C translation unit making the shim's calls with the shim's types."""
    # package-level variables: the `var ( ... )` blocks and `var x T` lines
    # outside any func
    head = "\n".join(re.findall(r"^var\s*\((.*?)^\)", go_text, re.S | re.M) +
                     re.findall(r"^var\s+([^(\n].*)$", go_text, re.M))
    pkg = _decls(head)
    lines = ["#include <stddef.h>", "#include <stdint.h>", '#include "bk.h"', ""]
    for nm, decl in pkg.items():
        lines.append("static %s;" % decl)
    for fname, params, body in _functions(go_text):
        calls = [(m.group(1), _call_args(body, m.end() - 1))
                 for m in re.finditer(r"\bC\.(bk_\w+)\s*\(", body)]
        if not calls:
            continue
        loc = dict(_param_decls(params), **_decls(body))
        used = set()
        for _, a in calls:
            used |= set(re.findall(r"(?<![\w.])([A-Za-z_]\w*)\b(?!\s*\()", _to_c(a)))
        lines.append("void shim_%s(void) {" % fname)
        for nm in sorted(used):
            if nm in loc:
                lines.append("    %s;" % loc[nm])
            elif nm in pkg or nm.startswith("BK_") or nm == "NULL" or re.match(
                    r"^(int64_t|int32_t|int|double|void|const|size_t|uint32_t|bk_\w+)$", nm):
                continue
            else:  # a Go int local (n, d, f, k, need, g, m ...)
                lines.append("    long long %s = 1;" % nm)
        for name, a in calls:
            args = ", ".join(_to_c(x) for x in _split_args(" ".join(a.split())))
            lines.append("    (void)%s(%s);" % (name, args))
        lines.append("}")
    # every constant the shim names (also those it only compares with, e.g. BK_OK)
    lines.append("int shim_constants(void) {")
    lines.append("    return 0" + "".join(" + (int)(%s)" % k for k in sorted(shim_names(go_text)[0])) + ";")
    lines.append("}")
    return "\n".join(lines) + "\n"


def compile_check(go_text, include_dir):
    """gcc -fsyntax-only -Werror of the shim's calls: (ok, diagnostics, C source)."""
    src = shim_as_c(go_text)
    with tempfile.NamedTemporaryFile("w", suffix=".c", delete=False) as fp:
        fp.write(src)
        path = fp.name
    try:
        r = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", "-Werror",
                            "-Wno-unused-variable", "-Wno-unused-function",
                            "-Wno-unused-but-set-variable", "-I" + include_dir, path],
                           capture_output=True, text=True)
    finally:
        os.unlink(path)
    return r.returncode == 0, r.stderr, src
