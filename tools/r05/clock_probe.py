"""r05 probe: the headline call's time round by round (20 calls a round)
from a cold start, to see whether a slow headline is a phase of the run
(clocks, a lazy build, another process) or of the schedule."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dgl-1_amd")]
import dgl  # noqa: E402
import dgl.function as fn  # noqa: E402
from dgl import data, kernel  # noqa: E402


_GC = []


def _gc_cb(phase, info):
    _GC.append((phase, info.get("generation"), time.perf_counter()))


def main():
    import gc
    gc.callbacks.append(_gc_cb)
    if os.environ.get("PROBE_SAVEALL"):
        gc.set_debug(gc.DEBUG_SAVEALL)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    src, dst, n = data.reddit_like(device=dev)
    g = dgl.DGLGraph((src.cpu(), dst.cpu()))
    del src, dst
    gen = torch.Generator(device=dev).manual_seed(1)
    h = torch.rand(n, 128, generator=gen, device=dev) * 2 - 1
    g.ndata["h"] = h
    adj = g.sparse_adjacency(dev)
    torch.cuda.synchronize()
    res = []
    if os.environ.get("PROBE_SCHEDULE_FIRST"):
        print("blocks", kernel.blocked_schedule(adj, h), flush=True)
        torch.cuda.synchronize()
    if os.environ.get("PROBE_PER_CALL"):
        # each of the first calls alone: wall and GPU span
        for c in range(int(os.environ["PROBE_PER_CALL"])):
            kernel.timing_enable(True, per_call=True)
            t = time.perf_counter()
            g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h_out"))
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t) * 1e3
            ms, calls = kernel.timing_read()
            kernel.timing_enable(False)
            print(json.dumps(["call", c, round(wall, 3), round(ms, 3)]), flush=True)
    t0 = time.perf_counter()
    for r in range(rounds):
        kernel.timing_enable(True, per_call=True)
        t = time.perf_counter()
        for _ in range(20):
            g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h_out"))
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / 20 * 1e3
        ms, calls = kernel.timing_read()
        kernel.timing_enable(False)
        pauses = []
        for i in range(0, len(_GC) - 1):
            if _GC[i][0] == "start" and _GC[i + 1][0] == "stop":
                pauses.append((_GC[i][1], round((_GC[i + 1][2] - _GC[i][2]) * 1e3, 2)))
        _GC.clear()
        if os.environ.get("PROBE_SAVEALL") and gc.garbage:
            import collections
            cnt = collections.Counter(type(o).__name__ for o in gc.garbage)
            print("garbage", len(gc.garbage), cnt.most_common(12), flush=True)
            gc.garbage.clear()
        res.append((round(time.perf_counter() - t0, 3), round(wall, 3), round(ms / calls, 3),
                    [p for p in pauses if p[1] > 1.0], len(pauses)))
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
