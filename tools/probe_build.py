"""The probe build of libbk.so (-DBK_PROBES): the only build that reads the
timing-only ablations (BK_GRAM_MODE, BK_K2_MODE), planner overrides
(BK_PLAN_*), kernel-shape knobs and debug traces (BK_TRACE_FILE,
BK_SMALL_TRACE).  The product library ignores them (bk_internal.h probe_env).

    python tools/probe_build.py          # builds tools/ab/libbk_probes.so (CPU, in-tree)

Tools that set probe knobs call use(_lib) before creating an Engine: it points
biscotti_amd._lib at $LIB if set, else at the probe build.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PROBE_LIB = os.path.join(HERE, "ab", "libbk_probes.so")


def build(extra=()):
    sys.path.insert(0, REPO)
    from biscotti_amd import build as B
    os.makedirs(os.path.dirname(PROBE_LIB), exist_ok=True)
    return B.build(force=True, extra=["-DBK_PROBES"] + list(extra), out=PROBE_LIB)


def use(_lib):
    path = os.environ.get("LIB") or PROBE_LIB
    if not os.path.exists(path):
        raise SystemExit("%s missing: run `python tools/probe_build.py` first" % path)
    _lib.LIB_PATH = os.path.abspath(path)
    return _lib.LIB_PATH


if __name__ == "__main__":
    print(build(sys.argv[1:]))
