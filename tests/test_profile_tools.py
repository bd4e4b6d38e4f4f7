"""The profile summarisers keep the steady state: tools/pmc_traffic.py --tail and
tools/kstats_tail.py take each kernel's LAST dispatches (the step workloads' burn-in
runs in the profiled process).  CPU only, synthetic rocprofv3-format CSVs."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pmc_traffic  # noqa: E402


def _counter_csv(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for did, name, val in rows:
            # two TCC instances per dispatch: per_dispatch sums them
            for half in (val / 2, val / 2):
                w.writerow({"Dispatch_Id": did, "Kernel_Name": name, "Counter_Name": counter, "Counter_Value": half})


def test_pmc_tail_takes_last_dispatches(tmp_path):
    # 30 burn-in dispatches at 2000 KB, then 10 steady ones at 10 KB, interleaved with another kernel
    rows = []
    for i in range(40):
        rows.append((2 * i, "void choco::topk_finish_kernel<0, true>(...)", 2000.0 if i < 30 else 10.0))
        rows.append((2 * i + 1, "void other(...)", 5.0))
    d = tmp_path / "f"
    d.mkdir()
    _counter_csv(d / "x_counter_collection.csv", "FETCH_SIZE", rows)
    allv, n = pmc_traffic.per_dispatch(str(d), "FETCH_SIZE", "topk_finish_kernel")
    assert n == 40 and allv[len(allv) // 2] == 2000.0  # the whole-run median is the burn-in's
    tail, n = pmc_traffic.per_dispatch(str(d), "FETCH_SIZE", "topk_finish_kernel", tail=10)
    assert n == 40 and tail == [10.0] * 10


def test_kstats_tail(tmp_path):
    p = tmp_path / "k_kernel_trace.csv"
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 0
        for i in range(30):
            dur = 260000 if i < 25 else 16000  # burn-in calls slow, the last 5 steady
            w.writerow({"Dispatch_Id": i, "Kernel_Name": "K34", "Start_Timestamp": t, "End_Timestamp": t + dur})
            t += dur + 100
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kstats_tail.py"), str(p), "5"],
                         capture_output=True, text=True, check=True).stdout
    rows = list(csv.DictReader(out.splitlines()))
    assert len(rows) == 1 and rows[0]["Name"] == "K34"
    assert int(float(rows[0]["Calls"])) == 5 and float(rows[0]["AverageNs"]) == 16000.0
