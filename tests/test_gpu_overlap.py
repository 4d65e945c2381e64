"""The exchange overlapped with the Gram (bk_comm_set_mode 2; VERDICT r5 item
3): the packed upper in k pieces by rows, computed by ONE Gram
launch in piece order, each piece reduced and all-reduced on a communication
stream (behind a device signal the piece's last workgroup raises) while the
later pieces compute.  Through libbk's sharded entry on a 1-rank RCCL communicator (one
GPU): every output -- selection, scores, mean, the margin record -- bitwise
the serial exchange's (mode 0), in the exact, fp32 MFMA and int8 modes, for
2..5 pieces, on K1 v3 plans that split (n >= ~2048) and on one that does not
(n = 512: mode 0 runs instead).  At N ranks each exchanged element is the sum
of the ranks' bitwise-identical pieces, so the equality holds there too; both
column shards of a 2-way split are checked here.  A piece that fails poisons
the record and still joins every remaining all-reduce."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from biscotti_amd import _lib  # noqa: E402

MODES = {"exact": _lib.BK_F32_EXACT, "mfma": _lib.BK_F32_MFMA,
         "i8x2_certified": _lib.BK_F32_I8X2_CERTIFIED, "i8": _lib.BK_F32_I8}


def _engine(pieces=None, fail_piece=None):
    from biscotti_amd.dist import bootstrap_rccl
    from biscotti_amd.krum import Engine
    if fail_piece is not None:
        os.environ["BK_TEST_FAIL_PIECE"] = str(fail_piece)
    try:
        eng = Engine(0)
    finally:
        os.environ.pop("BK_TEST_FAIL_PIECE", None)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    bootstrap_rccl(eng, 0, 1, lambda b, src: b)
    return eng


def _run(eng, X, f, xmode, pieces=None, f32_mode=None, c0=0, dl=None):
    n = X.shape[0]
    dl = X.shape[1] if dl is None else dl
    dt = _lib.BK_F32 if X.dtype == torch.float32 else _lib.BK_F64
    if pieces is not None:
        os.environ["BK_OVERLAP_PIECES"] = str(pieces)
    try:
        eng.comm_set_mode(xmode)
    finally:
        os.environ.pop("BK_OVERLAP_PIECES", None)
    if f32_mode is not None:
        eng.set_f32_mode(f32_mode)
    sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
    sc = torch.empty(n, dtype=torch.float64, device="cuda")
    mean = torch.empty(dl, dtype=torch.float64, device="cuda")
    Xs = X[:, c0:c0 + dl]
    eng.timing_select(["exchange_exposed", "allreduce", "k_gram"])
    eng.multikrum_sharded_ptr(Xs.data_ptr(), dt, n, dl, X.stride(0), f, sel.data_ptr(),
                              sc.data_ptr(), mean.data_ptr())
    eng.synchronize()
    rec = np.zeros(8)
    _lib.check(_lib.lib().bk_selection_margin_record(eng.ctx, rec.ctypes.data_as(
        __import__("ctypes").POINTER(__import__("ctypes").c_double))))
    kt = eng.timing_read()
    eng.timing_select([])
    if f32_mode is not None:
        eng.set_f32_mode(_lib.BK_F32_EXACT)
    return sel.cpu().numpy(), sc.cpu().numpy(), mean.cpu().numpy(), rec, kt


def _same(a, b):
    return all(np.array_equal(np.asarray(x).view(np.int64), np.asarray(y).view(np.int64))
               for x, y in zip(a[:4], b[:4]))


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("pieces", [2, 3, 5])
def test_overlapped_exchange_bitwise_serial(oracle, mode, pieces):
    n, d, f = 2500, 8192, 750
    X = torch.from_numpy(oracle.synth(n, d, 31337, f, dtype=np.float32)).cuda()
    eng = _engine()
    try:
        ser = _run(eng, X, f, 0, f32_mode=MODES[mode])
        ovl = _run(eng, X, f, 2, pieces=pieces, f32_mode=MODES[mode])
    finally:
        eng.close()
    assert _same(ser, ovl), mode
    # the overlapped call evented its exposed exchange (the pieces ran)
    assert "exchange_exposed" in ovl[4] and "exchange_exposed" not in ser[4]
    if mode in ("exact", "i8x2_certified"):
        assert np.array_equal(ser[0], oracle.krum(X.cpu().numpy(), f)[0])


def test_overlap_both_shards_of_a_two_way_split(oracle):
    """each column shard of a 2-rank job, overlapped vs serial: bitwise"""
    from biscotti_amd.dist import shard_bounds
    n, d, f = 2200, 6000, 600
    X = torch.from_numpy(oracle.synth(n, d, 4242, f)).cuda()
    eng = _engine()
    try:
        for r in (0, 1):
            c0, dl = shard_bounds(d, 2, r)
            ser = _run(eng, X, f, 0, c0=c0, dl=dl)
            ovl = _run(eng, X, f, 2, pieces=2, c0=c0, dl=dl)
            assert _same(ser, ovl), r
            assert ser[3][6] == dl  # the record's column count: this shard's
    finally:
        eng.close()


def test_overlap_falls_back_where_the_plan_does_not_split(oracle):
    """n = 512's McNaughton plan (workgroups span groups): mode 2 runs the
    serial exchange -- same bits, no exposed-exchange events"""
    n, d, f = 512, 20000, 153
    X = torch.from_numpy(oracle.synth(n, d, 99, f)).cuda()
    eng = _engine()
    try:
        ser = _run(eng, X, f, 0)
        ovl = _run(eng, X, f, 2)
    finally:
        eng.close()
    assert _same(ser, ovl)
    assert "exchange_exposed" not in ovl[4]


@pytest.mark.parametrize("fail_piece", [1, 2])
def test_failed_piece_poisons_and_joins(oracle, fail_piece):
    n, d, f = 2500, 4096, 750
    X = torch.from_numpy(oracle.synth(n, d, 7, f)).cuda()
    eng = _engine(fail_piece=fail_piece)
    try:
        os.environ["BK_OVERLAP_PIECES"] = "2"
        eng.comm_set_mode(2)
        os.environ.pop("BK_OVERLAP_PIECES", None)
        sel = torch.empty(n - f, dtype=torch.int64, device="cuda")
        with pytest.raises(_lib.BKError) as ei:
            eng.multikrum_sharded_ptr(X.data_ptr(), _lib.BK_F64, n, d, d, f, sel.data_ptr())
        assert ei.value.status == _lib.BK_EHIP and "BK_TEST_FAIL_PIECE" in str(ei.value)
        # the rank joined both all-reduces with a poisoned record: the call is invalid
        with pytest.raises(_lib.BKError) as e2:
            eng.synchronize()
        assert e2.value.status == _lib.BK_ERCCL
        ex, _ = eng.comm_stats()
        assert ex >= 1
    finally:
        eng.close()


@pytest.mark.parametrize("disagree", [0, 1])
def test_piece_layout_agreed_across_ranks(oracle, disagree):
    """the ranks agree on the piece layout at a signature's first call (one
    max-all-reduce of {status, layout, -layout}, run here on 1 rank through
    BK_TEST_FAIL_BEFORE_EXCHANGE=3, which agrees without failing): equal
    layouts keep the overlapped exchange; a peer that cut differently
    (BK_TEST_PIECES_DISAGREE=1) turns it off, and the call exchanges whole --
    bitwise the same either way"""
    n, d, f = 2500, 4096, 750
    X = torch.from_numpy(oracle.synth(n, d, 2024, f)).cuda()
    os.environ["BK_TEST_FAIL_BEFORE_EXCHANGE"] = "3"
    if disagree:
        os.environ["BK_TEST_PIECES_DISAGREE"] = "1"
    try:
        eng = _engine()
    finally:
        os.environ.pop("BK_TEST_FAIL_BEFORE_EXCHANGE", None)
        os.environ.pop("BK_TEST_PIECES_DISAGREE", None)
    try:
        ser = _run(eng, X, f, 0)
        ovl = _run(eng, X, f, 2, pieces=2)
        ovl2 = _run(eng, X, f, 2, pieces=2)  # the agreed signature: no new agreement
    finally:
        eng.close()
    assert _same(ser, ovl) and _same(ser, ovl2)
    for o in (ovl, ovl2):
        assert ("exchange_exposed" in o[4]) == (not disagree)
