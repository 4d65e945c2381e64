"""SURVEY §8(f) row 4's kernels (bench.py roni_cases: K7 logistic RONI, K8 over
the whole set, K8 with the reference's last-mini-batch semantics), each run
`reps` times back to back, plus the launch floor of the box: a 1-workgroup
torch kernel launched back to back, timed with events.  Under rocprofv3
(tools/profile_roni.sh) its dispatches give each kernel's duration and
counters.

    python tools/roni_probe.py [reps] [--probe]   (--probe: the -DBK_PROBES
        build, e.g. BK_RONI_LDS=1 for r5's LDS-staged K7 kernel)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    import bench
    if "--probe" in sys.argv:
        sys.argv.remove("--probe")
        import probe_build
        from biscotti_amd import _lib
        probe_build.use(_lib)
    from biscotti_amd.krum import Engine
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    runs = bench.roni_cases(eng, dev)
    out = {}
    for name, spec in runs.items():
        fn = spec[0]
        fn()
        torch.cuda.synchronize()
        eng.timing_enable(True)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        t = eng.timing_read().get("k_roni")
        eng.timing_enable(False)
        out[name] = {"ms": t["avg_ms"], "launches": t["count"], **(spec[3] if len(spec) > 3 else {})}
    out["launch_floor_ms"] = bench.launch_floor_ms(dev)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
