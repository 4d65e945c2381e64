"""The trace summarisers behind DESIGN's r6 claims, on synthetic rocprofv3
CSVs: tools/trace_fills.py (where the rocclr fill / copy dispatches of a run
come from, relative to the Gram dispatches) and tools/pmc_summary.py's
timed-window selection (dispatches in time order, whatever the CSV's row
order)."""
import csv
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

KT = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id",
      "Kernel_Name", "Correlation_Id", "Start_Timestamp", "End_Timestamp"]


def _write(path, header, rows):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=header)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _k(name, cid, t0, t1):
    return {"Kind": "KERNEL_DISPATCH", "Agent_Id": "Agent 2", "Queue_Id": 1, "Stream_Id": 1,
            "Thread_Id": 1, "Dispatch_Id": cid, "Kernel_Id": 1, "Kernel_Name": name,
            "Correlation_Id": cid, "Start_Timestamp": t0, "End_Timestamp": t1}


def test_trace_fills_places_each_blit(tmp_path):
    import trace_fills
    gram = "void bk::k_gram3<0, double>(double const*, long)"
    rows = [_k("__amd_rocclr_fillBufferAligned", 1, 10, 11),   # setup, before the Gram
            _k("__amd_rocclr_copyBuffer", 2, 12, 13),
            _k(gram, 3, 100, 200),
            _k("__amd_rocclr_fillBufferAligned", 4, 210, 211),  # between two Gram dispatches
            _k(gram, 5, 300, 400),
            _k("__amd_rocclr_copyBuffer", 6, 500, 501)]         # after the last
    # the CSV's rows deliberately out of time order
    _write(str(tmp_path / "run_kernel_trace.csv"), KT, rows[::-1])
    _write(str(tmp_path / "run_hip_api_trace.csv"),
           ["Domain", "Function", "Process_Id", "Thread_Id", "Correlation_Id", "Start_Timestamp",
            "End_Timestamp"],
           [{"Domain": "HIP_RUNTIME_API_EXT", "Function": f, "Process_Id": 1, "Thread_Id": 1,
             "Correlation_Id": c, "Start_Timestamp": 0, "End_Timestamp": 1}
            for f, c in (("hipMemsetAsync", 1), ("hipMemcpyAsync", 2), ("hipMemsetAsync", 4),
                         ("hipMemcpy", 6))])
    out = tmp_path / "fills.md"
    trace_fills.main(str(tmp_path), str(out))
    text = out.read_text()
    assert "k_gram dispatches: 2" in text
    assert "| __amd_rocclr_fillBufferAligned | hipMemsetAsync | before the first k_gram | 1 |" in text
    assert "| __amd_rocclr_copyBuffer | hipMemcpyAsync | before the first k_gram | 1 |" in text
    assert ("| __amd_rocclr_fillBufferAligned | hipMemsetAsync | between k_gram dispatches "
            "(inside the steps) | 1 |") in text
    assert "| __amd_rocclr_copyBuffer | hipMemcpy | after the last k_gram | 1 |" in text


def test_pmc_summary_short_names():
    import pmc_summary
    assert pmc_summary.short("void bk::k_gram_i8<2, 4, 4>(signed char const*, long)") == \
        "k_gram_i8<2, 4, 4>"
    assert pmc_summary.short("bk::k_roni_sign_reg<1>(double const*)") == "k_roni_sign_reg<1>"
