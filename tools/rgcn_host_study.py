"""Where the R-GCN step's host time goes (configs[4], tools/rgcn_step.py's step).

Per BLAS library (torch.backends.cuda.preferred_blas_library): host enqueue
ms per step (no sync inside the steps), ms to completion, and the top ops by
self CPU time (torch.profiler, CPU activity only).

  python tools/rgcn_host_study.py --blas hipblaslt rocblas --out gpurun_out/rgcn_host.json
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
import tools.rgcn_step as rs  # noqa: E402


def measure(blas, steps, top):
    if blas != "default":
        rs.lp.select_blas(blas)  # "rocblas" / "hipblaslt"
    args = rs.lp.parser().parse_args([])
    dev = torch.device("cuda", 0)
    raw = rs.make_samples(args, 5 + 3 * steps)
    samples = [rs.to_dev(s, dev) for s in raw]
    model, opt = rs.build_model(args, dev)
    model.train()
    for s in samples[:5]:
        rs.one_step(model, opt, s, args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in samples[5:5 + steps]:
        rs.one_step(model, opt, s, args)
    t_enq = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / steps * 1e3
    # phases, each bracketed by a sync (graph build, forward + loss, backward + Adam)
    ph = []
    for s in samples[5 + steps:5 + 2 * steps]:
        _, t = rs.one_step(model, opt, s, args, torch.cuda.synchronize)
        ph.append([b - a for a, b in zip(t[:-1], t[1:])])
    phases = [sum(p[i] for p in ph) / len(ph) * 1e3 for i in range(3)]
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for s in samples[5 + 2 * steps:]:
            rs.one_step(model, opt, s, args)
        torch.cuda.synchronize()
    rows = sorted(prof.key_averages(), key=lambda e: -e.self_cpu_time_total)[:top]
    # host syncs torch sees (set_sync_debug_mode), one step
    import warnings
    syncs = []
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            rs.one_step(model, opt, samples[5], args)
        for w in caught:
            syncs.append(str(w.message)[:120])
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    # Python-level host time by function (cProfile, tottime)
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for s in samples[5:5 + steps]:
        rs.one_step(model, opt, s, args)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    funcs = sorted(st.stats.items(), key=lambda kv: -kv[1][2])[:top]
    py = [{"func": "%s:%d(%s)" % (os.path.basename(k[0]), k[1], k[2]),
           "tottime_us_per_step": v[2] / steps * 1e6, "cumtime_us_per_step": v[3] / steps * 1e6,
           "calls_per_step": v[1] / steps} for k, v in funcs]
    ops = [{"name": e.key, "self_us_per_step": e.self_cpu_time_total / steps,
            "total_us_per_step": e.cpu_time_total / steps, "calls_per_step": e.count / steps}
           for e in rows]
    return {"blas": blas, "host_enqueue_ms": t_enq, "to_completion_ms": t_all,
            "phase_ms": {"graph": phases[0], "forward": phases[1], "backward": phases[2]},
            "top_self_cpu": ops, "syncs_one_step": syncs, "cprofile_top": py}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blas", nargs="+", default=["default"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = []
    for b in a.blas:
        r = measure(b, a.steps, a.top)
        print("%s: enqueue %.3f ms/step, completion %.3f, phases %s" % (
            b, r["host_enqueue_ms"], r["to_completion_ms"],
            {k: round(v, 3) for k, v in r["phase_ms"].items()}), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
