"""The synchronous host entry (bench.py host_entry_variant) for one build of
libbk.so, in a process of its own (the clock state of one build must not
blend into the next's):

    LIB=build_ab/libbk_x.so WL=B_mnist python tools/host_entry_ab.py <label>

Prints one JSON line: steady-state ms per call, the single calls after idle,
the H2D alone and the kernel's evented time.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402

if os.environ.get("LIB"):
    _lib.LIB_PATH = os.path.abspath(os.environ["LIB"])
import bench  # noqa: E402
from biscotti_amd.krum import Engine  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "host"
# torch's HIP runtime first: torch ships its own libamdhip64, and when libbk's
# (/opt/rocm) initialises the device first, torch's init then finds no GPU
import torch  # noqa: E402
torch.zeros(1, device="cuda")
eng = Engine(0)
r = bench.host_entry_variant(eng, "cuda:0", os.environ.get("WL", "B_mnist"),
                             single_calls=int(os.environ.get("SINGLE", 15)),
                             idle_s=float(os.environ.get("IDLE", 0.2)))
keep = ("ms_per_call", "single_call_ms_median", "single_calls_ms", "h2d_alone_ms",
        "overhead_over_h2d_ms", "kernel_avg_ms", "h2d_evented_ms", "d2h_evented_ms")
print(json.dumps({"label": label, **{k: r[k] for k in keep if k in r},
                  "parity": r["parity"].get("selected_set")}), flush=True)
eng.close()
