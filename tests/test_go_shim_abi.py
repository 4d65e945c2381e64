"""CPU: the Go cgo shim (go/bk/krum_bk.go, the drop-in for
DistSys/krum.go:31-44,100-166) against the C ABI it binds (include/bk.h),
without a Go toolchain: every C.bk_* call names a
declared function with the prototype's arity, every C.BK_* constant is
defined, and the calls -- rewritten into C with the shim's own types --
compile against bk.h under -Werror.  Renaming or re-arity-ing any entry the
shim uses, or dropping a constant it names, must fail both checks."""
import os
import re

import pytest

import go_shim_check as G

GO = open(G.SHIM).read()
HDR = open(G.HEADER).read()
USED = sorted({name for name, _, _ in G.shim_calls(GO)})
CONSTS = sorted(G.shim_names(GO)[0])


def _write_header(tmp_path, text):
    d = tmp_path / "inc"
    d.mkdir(exist_ok=True)
    (d / "bk.h").write_text(text)
    return str(d)


def _proto_span(text, name):
    """(start, open paren, close paren) of name's declaration in bk.h."""
    mt = re.search(r"^[A-Za-z_][\w \t\*]*?\b%s\s*\(" % re.escape(name), text, re.M)
    assert mt, name
    op = mt.end() - 1
    depth = 0
    for i in range(op, len(text)):
        if text[i] == "(":
            depth += 1
        elif text[i] == ")":
            depth -= 1
            if depth == 0:
                return mt.start(), op, i
    raise AssertionError(name)


def test_shim_uses_the_abi_entries():
    # the drop-in's own entry points must be among them
    # (r6: the verifier's rows go through bk_multikrum_rows -- VERDICT r5 item 1)
    for name in ("bk_create", "bk_multikrum_rows", "bk_stage_alloc", "bk_last_error",
                 "bk_selection_margin", "bk_multikrum_noised", "bk_group_multikrum"):
        assert name in USED, name
    assert {"BK_OK", "BK_HOST_PINNED", "BK_F64"} <= set(CONSTS)


def test_shim_names_and_arity_match_the_header():
    assert G.check_names(GO, HDR) == []


def test_shim_calls_compile_against_the_header():
    ok, err, src = G.compile_check(GO, os.path.dirname(G.HEADER))
    assert ok, err + "\n" + src
    # every call of the shim is in the translation unit
    assert src.count("(void)bk_") == len(G.shim_calls(GO))


@pytest.mark.parametrize("name", USED)
def test_renaming_an_entry_fails(tmp_path, name):
    s, op, cp = _proto_span(HDR, name)
    bad = HDR[:op] + "_renamed" + HDR[op:]
    assert any(name in p for p in G.check_names(GO, bad))
    ok, err, _ = G.compile_check(GO, _write_header(tmp_path, bad))
    assert not ok and name in err


@pytest.mark.parametrize("name", [n for n in USED
                                  if G.header_decls(HDR)[0][n]])  # entries with parameters
def test_dropping_a_parameter_fails(tmp_path, name):
    s, op, cp = _proto_span(HDR, name)
    params = G._split_args(HDR[op + 1:cp])
    bad = HDR[:op + 1] + ", ".join(params[:-1] or ["void"]) + HDR[cp:]
    assert any("arguments" in p and name in p for p in G.check_names(GO, bad))
    ok, err, _ = G.compile_check(GO, _write_header(tmp_path, bad))
    assert not ok and name in err


@pytest.mark.parametrize("name", [n for n in USED if G.header_decls(HDR)[0][n]])
def test_adding_a_parameter_fails(tmp_path, name):
    s, op, cp = _proto_span(HDR, name)
    bad = HDR[:cp] + ", int64_t extra" + HDR[cp:]
    assert any("arguments" in p and name in p for p in G.check_names(GO, bad))
    ok, err, _ = G.compile_check(GO, _write_header(tmp_path, bad))
    assert not ok


@pytest.mark.parametrize("name,old,new", [
    # sel_idx as int32_t*: the shim's (*C.int64_t) no longer fits
    ("bk_multikrum_rows", "int64_t *sel_idx", "int32_t *sel_idx"),
    ("bk_multikrum_noised", "int64_t *sel_idx", "int32_t *sel_idx"),
    # the row-pointer array as a flat batch: the shim's (*unsafe.Pointer) no longer fits
    ("bk_multikrum_rows", "const void *const *rows", "const double *rows")])
def test_a_pointer_parameter_changing_type_fails(tmp_path, name, old, new):
    s, op, cp = _proto_span(HDR, name)
    proto = HDR[op:cp].replace(old, new)
    assert proto != HDR[op:cp]
    bad = HDR[:op] + proto + HDR[cp:]
    ok, err, _ = G.compile_check(GO, _write_header(tmp_path, bad))
    assert not ok and name in err


@pytest.mark.parametrize("const", CONSTS)
def test_dropping_a_constant_fails(tmp_path, const):
    bad = re.sub(r"\b%s\b" % const, const + "_GONE", HDR)
    assert any(const in p for p in G.check_names(GO, bad))
    ok, _, _ = G.compile_check(GO, _write_header(tmp_path, bad))
    assert not ok
