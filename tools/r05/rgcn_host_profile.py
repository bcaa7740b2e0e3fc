"""r05: where the R-GCN step's host time goes (torch.profiler, CPU activity
only): per-step host ms and the top ops by self CPU time."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
import tools.rgcn_step as rs  # noqa: E402


def main():
    args = rs.lp.parser().parse_args([])
    dev = torch.device("cuda", 0)
    raw = rs.make_samples(args, 25)
    samples = [rs.to_dev(s, dev) for s in raw]
    model, opt = rs.build_model(args, dev)
    model.train()
    for s in samples[:5]:
        rs.one_step(model, opt, s, args)
    torch.cuda.synchronize()
    # host time per step when the GPU never makes the host wait: enqueue only
    t0 = time.perf_counter()
    for s in samples[5:15]:
        rs.one_step(model, opt, s, args)
    t_enq = (time.perf_counter() - t0) / 10 * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / 10 * 1e3
    print("host enqueue ms/step %.3f, to completion %.3f" % (t_enq, t_all), flush=True)
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for s in samples[15:25]:
            rs.one_step(model, opt, s, args)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30))


if __name__ == "__main__":
    main()
