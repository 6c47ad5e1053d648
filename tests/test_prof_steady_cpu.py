"""tools/prof_steady.py: the steady-state window of a rocprofv3 kernel trace starts after the
side-stream probes, and the queue map shows which streams shared a hardware queue (VERDICT r05
item 5)."""

import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import prof_steady  # noqa: E402


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Stream_Id"])
        w.writerows(rows)


def test_window_excludes_probes_and_maps_queues(tmp_path):
    p = str(tmp_path / "kernel_trace.csv")
    _trace(p, [
        ("warm_gemm", 0, 10, 1, 1),
        ("adamw_kernel", 10, 20, 1, 1),                  # --skip 1 ends here
        ("spin_kernel", 21, 30, 1, 1),                   # the post-warm-up probe pair
        ("spin_kernel", 21, 30, 2, 7),
        ("gemm", 31, 40, 1, 1),
        ("wgrad", 32, 38, 2, 7),                         # side stream on its own queue
        ("reduce", 39, 45, 1, 9),                        # a stream sharing the compute queue
        ("adamw_kernel", 46, 50, 1, 1),
    ])
    out, summ = prof_steady.steady(p, "adamw_kernel", 1)
    names = {d["name"] for d in out}
    assert "spin_kernel" not in names and "warm_gemm" not in names
    assert names == {"gemm", "wgrad", "reduce", "adamw_kernel"}
    assert summ["probes_in_window"] == 0 and summ["markers_skipped_for_probes"] == 0
    q = summ["queues"]
    assert set(q["1"]) == {"1", "9"} and set(q["2"]) == {"7"}
    # keeping the probes (--probe '') puts them back in the window
    out, summ = prof_steady.steady(p, "adamw_kernel", 1, probe="")
    assert "spin_kernel" in {d["name"] for d in out}
