"""k_small (config B / A, device-resident) for one build of libbk.so, in a
process of its own:

    LIB=tools/ab/libbk_x.so WL=B_mnist python tools/small_ab.py <label>

Prints one JSON line: the one-launch step (bench.small_variant: 500 steps),
its parity against the golden, and the host entry's call time."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biscotti_amd import _lib  # noqa: E402

if os.environ.get("LIB"):
    _lib.LIB_PATH = os.path.abspath(os.environ["LIB"])
import bench  # noqa: E402
from biscotti_amd.krum import Engine  # noqa: E402

label = sys.argv[1] if len(sys.argv) > 1 else "small"
import torch  # noqa: E402
torch.zeros(1, device="cuda")
eng = Engine(0)
wl = os.environ.get("WL", "B_mnist")
r = bench.small_variant(eng, "cuda:0", wl)
h = bench.host_entry_variant(eng, "cuda:0", wl)
print(json.dumps({"label": label, "workload": wl, "ms_per_step": r["one_launch"]["ms_per_step"],
                  "parity": r["one_launch"]["parity"].get("selected_set"),
                  "mean": r["one_launch"]["parity"].get("mean"),
                  "host_ms_per_call": h["ms_per_call"]}), flush=True)
eng.close()
