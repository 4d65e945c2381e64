"""ctypes binding of libbk.so (include/bk.h).

The HIP library is the product path: if it is missing this module raises on
import-time use -- there is no CPU fallback anywhere in biscotti_amd.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbk.so")

BK_OK, BK_EINVAL, BK_ENOMEM, BK_EHIP, BK_ERCCL, BK_ENOTSUP = 0, -1, -2, -3, -4, -5
BK_F64, BK_F32 = 0, 1
BK_HOST, BK_HOST_PINNED, BK_DEVICE = 0, 1, 2
BK_MAX_N = 16384
BK_UNIQUE_ID_BYTES = 128
BK_SYNTH_FP32ROUND = 1
BK_GROUP_ALLREDUCE, BK_GROUP_DETERMINISTIC, BK_GROUP_HOST_EXCHANGE = 0, 1, 2
BK_ABI_VERSION = 14
BK_F32_EXACT, BK_F32_MFMA, BK_F32_CERTIFIED, BK_F32_I8, BK_F32_I8_CERTIFIED = 0, 1, 2, 3, 4
BK_F32_I8X2, BK_F32_I8X2_CERTIFIED = 5, 6  # two digit planes, three products (bk.h)
BK_F64_EXACT, BK_F64_I8, BK_F64_I8_CERTIFIED, BK_F64_I8X2, BK_F64_I8X2_CERTIFIED = 0, 3, 4, 5, 6
KERNELS = ["k_gram", "k_reduce", "k_transpose", "k_scores", "k_rank", "k_compact", "k_mean",
           "allreduce", "k_synth", "h2d", "d2h", "k_aggregate", "k_qsum", "k_noise", "k_roni",
           "k_small", "k_slice", "score_gather", "exchange_exposed"]
K = {name: i for i, name in enumerate(KERNELS)}

# every symbol include/bk.h declares: name -> (restype, argtypes)
_i = ctypes.c_int
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_p = ctypes.c_void_p
_d = ctypes.c_double
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pd = ctypes.POINTER(ctypes.c_double)
SIGNATURES = {
    "bk_abi_version": (_i, []),
    "bk_last_error": (ctypes.c_char_p, []),
    "bk_check_args": (_i, [_i64, _i64, _i64]),
    "bk_create": (_i, [ctypes.POINTER(_p), _i]),
    "bk_destroy": (None, [_p]),
    "bk_set_stream": (_i, [_p, _p]),
    "bk_get_stream": (_p, [_p]),
    "bk_synchronize": (_i, [_p]),
    "bk_stage_alloc": (_i, [_p, _i64, ctypes.POINTER(_p)]),
    "bk_stage_free": (_i, [_p, _p]),
    "bk_multikrum": (_i, [_p, _p, _i, _i, _i64, _i64, _i64, _i64, _p, _p, _p, _p]),
    "bk_multikrum_rows": (_i, [_p, _p, _i, _i64, _i64, _i64, _p, _p, _p, _p]),
    "bk_set_host_threads": (_i, [_p, _i]),
    "bk_multikrum_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "bk_upper_elems": (_i64, [_i64]),
    "bk_gram_upper_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _p]),
    "bk_finish_device": (_i, [_p, _p, _p, _i, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "bk_comm_unique_id": (_i, [_p]),
    "bk_comm_init": (_i, [_p, _i, _i, _p]),
    "bk_comm_set_mode": (_i, [_p, _i]),
    "bk_multikrum_sharded_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _i64, _p, _p, _p]),
    "bk_synth_fill_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _i64, _i64, _u64, _i64, _d, _d,
                                  _d, _i]),
    "bk_timing_enable": (_i, [_p, _i]),
    "bk_graph_enable": (_i, [_p, _i]),
    "bk_set_f32_mode": (_i, [_p, _i]),
    "bk_set_f64_mode": (_i, [_p, _i]),
    "bk_timing_select": (_i, [_p, ctypes.c_uint32]),
    "bk_timing_stride": (_i, [_p, ctypes.c_int]),
    "bk_timing_read": (_i, [_p, _i, _pd, _pi64]),
    "bk_kernel_name": (ctypes.c_char_p, [_i]),
    "bk_plan": (_i, [_p, _i64, _i64, _pi64, _pi64, _pi64, _pi64]),
    "bk_plan_mode": (_i, [_p, _i64, _i64, _i, _i, _pi64, _pi64]),
    "bk_aggregate_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _p, _i64, _p]),
    "bk_aggregate": (_i, [_p, _p, _i, _i, _i64, _i64, _i64, _p, _i64, _p]),
    "bk_quantized_sum_device": (_i, [_p, _p, _i, _i64, _i64, _i64, _p, _i64, _i, _p, _p]),
    "bk_noise_apply_device": (_i, [_p, _p, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64]),
    "bk_multikrum_noised": (_i, [_p, _p, _i64, _p, _i64, _i64, _i, _i64, _i64, _i64, _p, _p,
                                 _p, _p, _p, _i64]),
    "bk_roni_device": (_i, [_p, _p, _i64, _i64, _i64, _p, _p, _p, _i64, _i64, _p]),
    "bk_roni_set_validation": (_i, [_p, _p, _i64, _i64, _i64, _p]),
    "bk_roni": (_i, [_p, _p, _p, _i64, _i64, _i64, _p]),
    "bk_roni_softmax_device": (_i, [_p, _p, _i64, _i64, _i64, _p, _i64, _p, _p, _i64, _i64, _p,
                                    _p]),
    "bk_roni_softmax_batches_device": (_i, [_p, _p, _i64, _i64, _i64, _p, _i64, _p, _p, _i64,
                                            _i64, _p, _i64, _p, _p]),
    "bk_roni_softmax_set_validation": (_i, [_p, _p, _i64, _i64, _i64, _p, _i64]),
    "bk_roni_softmax": (_i, [_p, _p, _p, _i64, _i64, _p, _p]),
    "bk_roni_softmax_batches": (_i, [_p, _p, _p, _i64, _i64, _p, _i64, _p, _p]),
    "bk_group_create": (_i, [ctypes.POINTER(_p), _i, _p, _i]),
    "bk_group_destroy": (None, [_p]),
    "bk_group_size": (_i, [_p]),
    "bk_group_multikrum": (_i, [_p, _p, _i, _i, _i64, _i64, _i64, _i64, _p, _p, _p, _p]),
    "bk_group_ctx": (_p, [_p, _i]),
    "bk_selection_margin": (_i, [_p, _pd, _pd, ctypes.POINTER(_i)]),
    "bk_selection_margin_record": (_i, [_p, _pd]),
    "bk_certified_reruns": (_i64, [_p]),
    "bk_comm_size": (_i, [_p, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "bk_comm_stats": (_i, [_p, _pi64, _pd]),
    "bk_set_small_path": (_i, [_p, _i]),
}

_lib = None


class BKError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("libbk status %d: %s" % (status, msg))
        self.status = status


def code_object_sha16(path=None):
    """sha256 (16 hex digits) of libbk.so's device code: its .hip_fatbin
    section, i.e. the gfx950 code objects of every kernel.  PMC records
    (profiles/pmc_*.json) are stamped with it, so a record stays valid across
    host-only rebuilds and goes stale when any kernel's code changes."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as fh:
        data = fh.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError("not an ELF64 file: %s" % (path or LIB_PATH))
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def section(i):
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)

    stroff = section(shstrndx)[4]
    for i in range(shnum):
        name, _, _, _, off, size = section(i)
        end = data.index(b"\0", stroff + name)
        if data[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    raise ValueError("no .hip_fatbin section in %s" % (path or LIB_PATH))


def lib():
    """Load libbk.so; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libbk.so not found at %s -- build it with "
                              "`python -m biscotti_amd.build` (HIP/gfx950); there is no CPU "
                              "fallback" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error():
    e = lib().bk_last_error()
    return e.decode() if e else ""


def check(status):
    if status != BK_OK:
        if status == BK_EINVAL:
            raise ValueError(last_error())
        raise BKError(status, last_error())
    return status
