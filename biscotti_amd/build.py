"""Build recipe for libbk.so (the HIP engine + C ABI), gfx950 only.

    python -m biscotti_amd.build            # or __graft_entry__.build()

hipcc cross-compiles without a GPU.  The .so lands in-tree
(biscotti_amd/libbk.so) so it travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libbk.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

SOURCES = ["bk_kernels.hip", "bk_small.hip", "bk_aggregate.hip", "bk_roni.hip", "bk_plan.hip",
           "bk_i8.hip", "bk_api.hip"]
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # the synthetic generator and the distance / mean arithmetic must round
    # exactly like numpy (no implicit FMA); MFMA is explicit
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-function",
    "-I" + os.path.join(REPO, "include"),
    "-I" + CSRC,
]
LIBS = ["-L" + os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib")]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(REPO, "include", "bk.h"),
                                                                 __file__]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force=False, verbose=True, extra=(), out=LIB, jobs=None):
    """extra/out: debug variants (e.g. -DBK_PROBES, -DBK_K1_PROBE into tools/ab/),
    never the product: the probe knobs (BK_GRAM_MODE, BK_PLAN_*, ...) exist
    only in a -DBK_PROBES build (bk_internal.h probe_env).
    Each source compiles to its own object in parallel (every kernel is launched
    from its own translation unit, so no relocatable device code is needed),
    then one link."""
    if not force and out == LIB and not needs_build():
        return LIB
    import fcntl
    import hashlib
    import tempfile
    # a fixed object directory per (output, flags): the object paths end up in
    # the linked library, and a random temp name made every build's sha256
    # differ (the PMC records are matched to the library by that hash).  Two
    # processes building the same output would delete each other's objects,
    # so the whole build holds an exclusive lock on that directory's lock file.
    key = hashlib.sha1(("\0".join([out] + list(extra))).encode()).hexdigest()[:12]
    tmp = os.path.join(tempfile.gettempdir(), "bk_build_" + key)
    with open(tmp + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(tmp, out, extra, verbose, jobs)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(tmp, out, extra, verbose, jobs):
    import concurrent.futures as cf
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    cflags = [f for f in FLAGS if f != "-shared"] + list(extra)
    objs = [os.path.join(tmp, os.path.splitext(s)[0] + ".o") for s in SOURCES]

    def compile_one(i):
        cmd = [HIPCC] + cflags + ["-c", os.path.join(CSRC, SOURCES[i]), "-o", objs[i]]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, range(len(SOURCES))))
    arch = [f for f in FLAGS if f.startswith("--offload-arch=")]
    cmd = [HIPCC] + arch + ["-shared", "-fPIC"] + objs + ["-o", out + ".tmp"] + LIBS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    shutil.rmtree(tmp, ignore_errors=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
