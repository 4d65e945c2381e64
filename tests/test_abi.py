"""libbk.so: loads, exports every symbol include/bk.h declares, validates
arguments without a GPU, and fails loudly (an error status, never a CPU
fallback) when no GPU is present."""
import ctypes
import os
import re

import pytest

from biscotti_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(REPO, "include", "bk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(bk_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("bk_create", "bk_destroy", "bk_multikrum", "bk_multikrum_device",
                 "bk_last_error", "bk_multikrum_sharded_device", "bk_comm_init"):
        assert must in names
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"amdgcn-amd-amdhsa" in data


def test_abi_version_and_names():
    L = _lib.lib()
    assert L.bk_abi_version() == _lib.BK_ABI_VERSION == 14
    assert L.bk_kernel_name(0) == b"k_gram"
    assert L.bk_kernel_name(99) == b"?"
    assert len(_lib.KERNELS) == 19
    for i, name in enumerate(_lib.KERNELS):
        assert L.bk_kernel_name(i) == name.encode()


@pytest.mark.parametrize("n,d,f,status", [
    (10, 25, 2, 0), (10, 25, 0, -1), (10, 25, 10, -1), (10, 25, -1, -1), (0, 25, 1, -1),
    (10, 0, 2, -1), (2, 1, 1, 0), (16385, 8, 3, -5), (16384, 8, 3, 0)])
def test_check_args(n, d, f, status):
    assert _lib.lib().bk_check_args(n, d, f) == status
    if status:
        assert _lib.last_error()


def test_upper_elems():
    """64x64 upper sub-tiles + the trailing record {column count, fp32-MFMA
    columns, int8 Gram error bound, 0}."""
    from biscotti_amd import dist as D
    L = _lib.lib()
    assert L.bk_upper_elems(1) == 4096 + 4
    assert L.bk_upper_elems(64) == 4096 + 4
    assert L.bk_upper_elems(65) == 3 * 4096 + 4
    assert L.bk_upper_elems(512) == 36 * 4096 + 4
    for n in (1, 63, 64, 65, 512, 4097):
        assert D.upper_elems(n) == L.bk_upper_elems(n)


def test_plan_fills_the_chip():
    """The K1 v3 plan (host planner, bk_plan.hip): whole workgroups on every CU
    of every XCD, and the whole upper triangle covered."""
    L = _lib.lib()
    v = [ctypes.c_int64() for _ in range(4)]
    for n, d in [(512, 1 << 20), (1024, 131072), (4096, 262144), (100, 7850), (512, 131072)]:
        assert L.bk_plan(None, n, d, *[ctypes.byref(x) for x in v]) == 0
        S, kc, ntile, nwg = (x.value for x in v)
        T = (n + 63) // 64
        assert ntile == T * (T + 1) // 2 and kc == 16
        assert S >= 1 and nwg % 8 == 0 and nwg >= 248  # b = 8j + x slots, ~every CU busy
    assert L.bk_plan(None, 512, 1 << 20, *[ctypes.byref(x) for x in v]) == 0
    assert v[0].value == 4  # two band quads + two off-diagonal pairs of super-tiles


@pytest.mark.parametrize("mode,rounds", [("2", ""), ("1", ""), ("0", ""), ("3", ""), ("3", "4"),
                                         ("2", "8")])
def test_plan_covers_every_kblock_once(mode, rounds):
    """The planner's own check (bk_plan.hip): every (group, k-block) pair is
    owned by exactly one workgroup and every group has one ragged-tail
    workgroup -- for McNaughton pieces (default), the v8 round-aligned strides,
    the v7 interleave and the aligned pieces (bk_plan_mode), over shapes from
    tiny to BK_MAX_N."""
    L = _lib.lib()
    v = [ctypes.c_int64() for _ in range(2)]
    for n, d in [(1, 1), (2, 16), (65, 100), (100, 7850), (300, 1000003), (512, 1 << 20),
                 (512, 131072), (1000, 12345), (4096, 32768), (16384, 4096)]:
        assert L.bk_plan_mode(None, n, d, int(mode), int(rounds or 0),
                              *[ctypes.byref(x) for x in v]) == 0, (n, d, _lib.last_error())


def test_probe_knobs_are_not_in_the_product():
    """The timing-only ablations and planner overrides (BK_GRAM_MODE,
    BK_K2_MODE, BK_PLAN_*, ...) are compiled only into -DBK_PROBES builds:
    the product library does not even contain their names."""
    blob = open(_lib.LIB_PATH, "rb").read()
    for knob in (b"BK_GRAM_MODE", b"BK_K2_MODE", b"BK_PLAN_MODE", b"BK_PLAN_ROUNDS",
                 b"BK_PLAN_NB_COST", b"BK_PLAN_WGOH", b"BK_QUAD_BAL", b"BK_K2_KPT",
                 b"BK_K2_TRANSPOSE_MIN_N", b"BK_SCHED", b"BK_SCORES", b"BK_RONI_VALU",
                 b"BK_RONI_TILES", b"BK_TRACE_FILE", b"BK_SMALL_TRACE"):
        assert knob not in blob, knob


def test_null_and_bad_arguments_do_not_crash():
    L = _lib.lib()
    assert L.bk_create(None, 0) == _lib.BK_EINVAL
    assert L.bk_multikrum(None, None, 0, 0, 10, 10, 10, 2, None, None, None, None) == _lib.BK_EINVAL
    assert L.bk_set_stream(None, None) == _lib.BK_EINVAL
    assert L.bk_timing_read(None, 0, None, None) == _lib.BK_EINVAL
    assert L.bk_group_create(None, 1, None, 0) == _lib.BK_EINVAL
    g = ctypes.c_void_p()
    assert L.bk_group_create(ctypes.byref(g), 0, None, 0) == _lib.BK_EINVAL
    assert L.bk_group_create(ctypes.byref(g), 2, None, 7) == _lib.BK_EINVAL
    dup = (ctypes.c_int * 2)(0, 0)  # RCCL modes need distinct devices
    assert L.bk_group_create(ctypes.byref(g), 2, dup, _lib.BK_GROUP_ALLREDUCE) == _lib.BK_EINVAL
    assert L.bk_group_multikrum(None, None, 0, 0, 10, 10, 10, 2, None, None, None,
                                None) == _lib.BK_EINVAL
    assert L.bk_group_size(None) == 0 and L.bk_group_ctx(None, 0) is None
    L.bk_group_destroy(None)
    assert L.bk_set_f32_mode(None, _lib.BK_F32_MFMA) == _lib.BK_EINVAL
    assert L.bk_multikrum_noised(None, None, 10, None, 1, 10, _lib.BK_HOST, 10, 10, 2, None, None,
                                 None, None, None, 10) == _lib.BK_EINVAL
    assert L.bk_set_f32_mode(None, _lib.BK_F32_CERTIFIED) == _lib.BK_EINVAL
    assert L.bk_selection_margin(None, None, None, None) == _lib.BK_EINVAL
    assert L.bk_selection_margin_record(None, None) == _lib.BK_EINVAL
    assert L.bk_certified_reruns(None) == 0
    assert L.bk_comm_size(None, None, None) == _lib.BK_EINVAL
    assert L.bk_comm_stats(None, None, None) == _lib.BK_EINVAL
    assert L.bk_set_small_path(None, 1) == _lib.BK_EINVAL
    assert L.bk_timing_stride(None, 2) == _lib.BK_EINVAL
    assert L.bk_multikrum_sharded_device(None, None, 0, 10, 0, 0, 2, None, None,
                                         None) == _lib.BK_EINVAL


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = ctypes.c_void_p()
    st = _lib.lib().bk_create(ctypes.byref(ctx), 0)
    assert st in (_lib.BK_EHIP, _lib.BK_EINVAL)
    assert _lib.last_error()
    from biscotti_amd.krum import Engine
    with pytest.raises((RuntimeError, ValueError)):
        Engine(0)


def test_code_object_hash_is_the_fatbin(tmp_path):
    """PMC records are matched on the hash of libbk.so's .hip_fatbin (the
    kernels' code), which bench.py recomputes; a non-ELF file is refused"""
    import re
    from biscotti_amd import _lib
    h = _lib.code_object_sha16()
    assert re.fullmatch(r"[0-9a-f]{16}", h)
    assert bench_lib_sha16() == h
    bad = tmp_path / "x.so"
    bad.write_bytes(b"not an elf")
    with pytest.raises(ValueError):
        _lib.code_object_sha16(str(bad))


def bench_lib_sha16():
    import importlib
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return importlib.import_module("bench").lib_sha16()
