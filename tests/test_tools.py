"""The measurement tools' parsing (no GPU): tools/window_stats.py keeps only
the dispatches between bench.py's spin-kernel markers, and
tools/gat_bwd_split.py names kernels past their (anonymous) namespaces and
counts only the calls after its marker."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)


def test_window_stats_keeps_the_timed_region(tmp_path):
    rows = [("setup_sort", 0, 5), ("void at::cuda::spin_kernel(long)", 10, 12),
            ("gspmm_sum_kernel<2>", 20, 30), ("gspmm_sum_kernel<2>", 31, 45),
            ("void at::cuda::spin_kernel(long)", 50, 51), ("after", 60, 70),
            ("void at::cuda::spin_kernel(long)", 80, 81), ("leg2", 90, 99),
            ("void at::cuda::spin_kernel(long)", 100, 101)]
    p = tmp_path / "trace.csv"
    _trace(p, rows)
    out = tmp_path / "stats.csv"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "window_stats.py"),
                           str(p), "--out", str(out)])
    got = list(csv.DictReader(open(out)))
    assert [r["Name"] for r in got] == ["gspmm_sum_kernel<2>"]
    assert int(got[0]["Calls"]) == 2 and float(got[0]["TotalDurationNs"]) == 24
    assert float(got[0]["Percentage"]) == 100.0
    ws = _tool("window_stats").windows(list(csv.DictReader(open(p))))
    assert ws == [(12, 50), (81, 100)]


def test_gat_split_names_and_window(tmp_path):
    g = _tool("gat_bwd_split")
    assert g.kernel_key("void dglhip::(anonymous namespace)::gat_backward_t_kernel<true, "
                        "false, 0, 5, true>(long, int const*)") == "gat_backward_t_kernel"
    assert g.kernel_key("dglhip::rowsum_heads8_kernel(long)") == "rowsum_heads8_kernel"
    plan = tmp_path / "plan.json"
    json.dump({"nodes": 1, "edges": 1, "calls": 2,
               "blocks": [{"items": 1, "slots": 4, "suffix": False}]}, open(plan, "w"))
    csvp = tmp_path / "c.csv"
    with open(csvp, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writerow([1, "dglhip::(anonymous namespace)::gat_backward_t_kernel<1>()",
                     "TCC_HIT_sum", 1000])  # the plan-building call: not counted
        w.writerow([2, "at::cuda::spin_kernel(long)", "TCC_HIT_sum", 0])
        for d in (3, 4):
            w.writerow([d, "dglhip::(anonymous namespace)::gat_backward_t_kernel<1>()",
                         "TCC_HIT_sum", 10])
            w.writerow([d, "dglhip::(anonymous namespace)::gat_backward_t_kernel<1>()",
                         "TCC_MISS_sum", 30])
    out = tmp_path / "split.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "gat_bwd_split.py"),
                           "parse", str(plan), str(csvp), "--out", str(out)],
                          stdout=subprocess.DEVNULL)
    res = json.load(open(out))
    k = res["kernels"]["gat_backward_t_kernel"]
    assert res["calls_counted"] == 2 and k["dispatches_per_call"] == 1.0
    assert k["per_call"]["TCC_HIT_sum"] == 10 and abs(k["per_call"]["miss_rate"] - 0.75) < 1e-12
