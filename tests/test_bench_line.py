"""CPU: bench.py's printed line: the contract's keys, and
as the LAST key a per-config summary small enough for the driver's stored
tail; the full record goes to the detail file."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record():
    roof = {"bound": "mfma", "achieved": 68.0, "peak": 78.6, "unit": "TFLOP/s", "frac": 0.865,
            "traffic": 1.07e10, "traffic_source": "x", "kernel": "k_gram", "kernel_avg_ms": 4.05,
            "traffic_ratio_to_unique_bytes": 2.5}
    par = {"selected_set": "match", "mean": "match",
           "margin": {"near_tie": False, "gap": 5e5, "err_bound": 1e-3}}
    dv = {"value": 1.0, "ms_per_step": 2.0, "roofline": roof, "parity": par, "steps": 20,
          "step_roofline": {"t_floor_ms": 1.0, "frac": 0.5}, "filler": "x" * 4000}
    sm = {"one_launch": {"ms_per_step": 0.02, "GB_per_s": 290.0, "parity": par}, "value": 290.0,
          "ms_per_step": 0.02, "roofline": dict(roof, unit="GB/s"),
          "host_entry": {"ms_per_call": 0.15, "overhead_over_h2d_ms": 0.02, "parity": par}}
    variants = {k: dict(dv) for k in ("D_512x1M_f256", "C_1024x131072", "E_4096x262144_fp32",
                                      "E_4096x262144_fp32_mfma", "E_4096x262144_fp32_certified",
                                      "E_4096x262144_fp32_i8", "E_4096x262144_fp32_i8_certified",
                                      "D_512x1M_f153_i8_certified")}
    variants["E_4096x262144_fp32_i8_certified"]["certified_reruns"] = 0
    variants["B_mnist"] = sm
    variants["A_creditcard"] = sm
    return {"metric": "m", "value": 940.0, "unit": "GB/s", "n_gpus": 1, "steps": 40, "warmup": 10,
            "ms_per_step": 4.57, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic", "config": {"workload": "D_512x1M_f153"},
            "roofline": roof, "roofline_hbm_k4": {"frac": 0.8}, "step_roofline": {"frac": 0.76},
            "kernels_ms_avg": {"k_gram": 4.05}, "parity": par, "variants": variants,
            "single_call": {"ms": 5.7, "k_gram_frac": 0.68},
            "next_rows": {"k_noise": {"ms": 0.74, "roofline": {"frac": 0.72}}},
            "e2e_pinned_h2d_d2h": {"GB_per_s": 56.0, "ms": 76.7},
            "cpu_baseline": {"value": 2.4, "unit": "GB/s", "cores": 16, "kind": "port",
                             "sample": "s", "value_1core": 0.18}}


def test_compact_line_keeps_every_config_and_fits(tmp_path):
    sys.path.insert(0, REPO)
    import bench
    rec = _record()
    path = str(tmp_path / "detail.json")
    line = bench.compact_line(rec, path)
    s = json.dumps(line)
    assert len(s) < 6000, len(s)
    assert list(line)[-1] == "summary"
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in line, k
    summ = line["summary"]
    for k in list(rec["variants"]) + ["D_512x1M_f153"]:
        assert k in summ and summ[k]["sel"] == "match", k
        assert summ[k]["value"] is not None and summ[k]["ms"] is not None, k
    assert summ["B_mnist"]["host_over_h2d_ms"] == 0.02
    assert summ["E_4096x262144_fp32_i8_certified"]["reruns"] == 0
    assert json.load(open(path))["variants"]["C_1024x131072"]["filler"]  # the full record


def test_launcher_refuses_fewer_gpus_than_rccl_ranks():
    """`bench.py --gpus N` without WORLD_SIZE starts its own
    ranks; with the RCCL exchange and fewer visible GPUs than N it returns a
    non-zero status and launches nothing."""
    sys.path.insert(0, REPO)
    import argparse
    import bench
    a = argparse.Namespace(gpus=8, exchange="rccl")
    assert bench.launch_ranks(a, argv=["--gpus", "8"], gpus_fn=lambda: 1) != 0
    a = argparse.Namespace(gpus=2, exchange="host")
    assert bench.launch_ranks(a, argv=["--gpus", "2"], gpus_fn=lambda: 0) != 0


def test_launcher_relays_the_ranks_failure(capfd):
    """The launcher's child torch.distributed.run: here (no GPU) the ranks
    fail, and the parent must return their non-zero status with nothing on
    stdout -- never a 1-GPU line in place of the N-rank one."""
    import argparse
    sys.path.insert(0, REPO)
    import bench
    a = argparse.Namespace(gpus=2, exchange="host")
    rc = bench.launch_ranks(a, argv=["--gpus", "2", "--exchange", "host", "--steps", "1",
                                     "--warmup", "0", "--workload", "A_creditcard",
                                     "--no-cpu-baseline"], gpus_fn=lambda: 1)
    out = capfd.readouterr().out
    assert rc != 0 and not out.strip()


def test_visible_gpus_needs_no_gpu_runtime(tmp_path):
    """the launcher counts GPUs from the environment or the
    KFD topology (sysfs), never through torch / HIP: a fresh interpreter that
    runs it has imported no torch and opened no /dev/kfd."""
    import subprocess
    topo = tmp_path / "nodes"
    dri = tmp_path / "dri"
    dri.mkdir()
    # 2 CPU nodes, 4 GPU nodes (one without a render minor), one CPU node; the
    # GPU of minor 131 has no render node here (not exposed to this process)
    for i, (gid, minor) in enumerate([(0, 0), (0, 0), (12345, 128), (0, 0), (777, 129),
                                      (999, None), (555, 131)]):
        (topo / str(i)).mkdir(parents=True)
        (topo / str(i) / "gpu_id").write_text("%d\n" % gid)
        if minor is not None:
            (topo / str(i) / "properties").write_text("cpu_cores_count 0\ndrm_render_minor %d\n"
                                                      % minor)
        if minor in (128, 129):
            (dri / ("renderD%d" % minor)).write_text("")
    code = r"""
import builtins, os, sys
sys.path.insert(0, %r)
opened = []
real_open, real_os_open = builtins.open, os.open
def spy(path, *a, **k):
    opened.append(str(path))
    return real_open(path, *a, **k)
def spy_os(path, *a, **k):
    opened.append(str(path))
    return real_os_open(path, *a, **k)
builtins.open, os.open = spy, spy_os
import bench
env = {k: v for k, v in os.environ.items() if not k.endswith("VISIBLE_DEVICES")}
n_topo = bench.visible_gpus(environ=env, topology=%r, dri=%r)
n_env = bench.visible_gpus(environ=dict(env, HIP_VISIBLE_DEVICES="0,3"))
n_rocr = bench.visible_gpus(environ=dict(env, ROCR_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="1"))
n_none = bench.visible_gpus(environ=env, topology=%r)
print(n_topo, n_env, n_rocr, n_none, "torch" in sys.modules,
      any("kfd" in p and p.startswith("/dev") for p in opened))
""" % (REPO, str(topo), str(dri), str(tmp_path / "missing"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["3", "2", "0", "0", "False", "False"], r.stdout


def test_launcher_parent_touches_no_gpu_runtime(tmp_path):
    """`bench.py --gpus 2` as the launcher parent, its child replaced by a
    stand-in: the parent counts GPUs, starts one child and relays its line,
    and has imported no torch (so no torch.cuda) and opened no /dev/kfd."""
    import subprocess
    code = r"""
import builtins, json, os, subprocess, sys
sys.path.insert(0, %r)
opened = []
real_open = builtins.open
def spy(path, *a, **k):
    opened.append(str(path))
    return real_open(path, *a, **k)
builtins.open = spy
started = []
class FakeChild:
    def __init__(self, cmd, **kw):
        started.append(cmd)
        self.stdout = iter(['{"n_gpus": 2}' + chr(10)])
    def wait(self):
        return 0
    def send_signal(self, s):
        pass
subprocess.Popen = FakeChild
import bench
os.environ["HIP_VISIBLE_DEVICES"] = "0,1"
sys.argv = ["bench.py", "--gpus", "2"]
try:
    bench.main()
except SystemExit as e:
    rc = e.code
sys.stderr.write(json.dumps({"rc": rc, "children": len(started),
                             "torch": "torch" in sys.modules,
                             "kfd": any(p.startswith("/dev/kfd") for p in opened),
                             "runs_torchrun": "torch.distributed.run" in " ".join(started[0])}))
""" % REPO
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=env)
    res = json.loads(r.stderr.strip().splitlines()[-1])
    assert res == {"rc": 0, "children": 1, "torch": False, "kfd": False, "runs_torchrun": True}, r
    assert json.loads(r.stdout.strip()) == {"n_gpus": 2}
