"""Benchmark: edges/s of update_all g-SpMM (copy_u + sum, feat = 128).

BASELINE.json metric: "edges/sec on update_all g-SpMM (copy_u+sum, feat=128)
at 1/2/4/8 GPUs". Workload (config.workload):

* N = 1: the Reddit-shaped graph of BASELINE.json configs[1] (232,965 nodes,
  114,615,892 edges + self-loops, fp32 features of width 128), synthetic
  (dgl.data.reddit_like) — the real dataset cannot be downloaded here; when
  DGL's Reddit release files are under $DGL_DATA_DIR/reddit, that graph is
  used instead and `data` says so. One
  step = ``g.update_all(fn.copy_src('h','m'), fn.sum('m','h_out'))`` through
  the DGLGraph API (scheduler -> cached CSR -> HIP g-SpMM), inputs resident in
  HBM.
* N > 1 (weak scaling): the same generator at N x the nodes and edges, dst
  rows 1-D partitioned over the ranks (dgl.distributed.PartitionedGraph); one
  step = RCCL all-gather of the node-feature halo + the local g-SpMM.

Ranks: ``python bench.py --gpus N`` with N > 1 and no WORLD_SIZE in the
environment starts ``python -m torch.distributed.run --nproc-per-node N
bench.py ...`` as a CHILD process (before this process loads the HIP library
or touches the GPU), relays its output and exits with its return code. Under
an outer torchrun (WORLD_SIZE set) the script runs as one rank and refuses a
WORLD_SIZE that disagrees with --gpus.

Timing: W warm-up steps, then K steps bracketed by barrier + synchronize;
the max over ranks is reported; value = all edges processed / that time.
roofline: algorithmic bytes of one g-SpMM launch (SURVEY.md §8d:
E*(4F+4) + R*(4F+8)) / the kernel's mean duration, measured with hipEvents
recorded around every launch on its own stream inside the timed region
(rank 0's; ``per_rank`` lists every rank's).
cpu_baseline: the reference's own CPU arithmetic (torch.sparse.mm on the
uncoalesced COO, python/dgl/backend/pytorch/tensor.py:145-146) on a bounded
sample of the same graph, timed on rank 0 after the timed region, at every N.

rmat26 (secondary block of the same JSON line, keyed rmat<scale>;
--no-rmat-leg skips it): the
north star also asks for absolute edges/s on RMAT-26 at 1/2/4/8 GPUs next to
the CPU baseline. After the headline timing (and with its memory released)
the same ranks time one fixed Graph500 R-MAT graph (scale --rmat-scale, edge
factor 16, 1.07B edges at 26): strong scaling, dst rows partitioned as above,
heavy rows chunked. Its CPU baseline is the reference product on a sample of
that graph (rank 0, after the timed region).

Run: python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import absolute_import

import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dgl-1_amd"))
sys.path.insert(0, ROOT)

# bound by _load_dgl() once the launcher decision is made (loading
# libdgl_hip.so is the first thing that may touch the GPU)
dgl = fn = data = kernel = None

FEAT = 128
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# the guide's highest measured rate for uniformly random rows gathered from a
# table past L2 and resident in the 256 MiB Infinity Cache (38 MB table, 8.6
# TB/s; 7.4-7.9 at 151 MB): the ceiling of a gather whose table the Infinity
# Cache holds (MI355X_MICROARCH.md "Indexed rows: gather into LDS")
IC_GATHER_PEAK_GBS = 8600.0
INFINITY_CACHE_BYTES = 256 << 20
# the guide's measured rate for indexed rows gathered from an XCD's L2 (rows
# shared by every workgroup: 16.8-18.8 TB/s chip-wide): the ceiling of the
# source-blocked schedule, whose blocks of ~7.5 MiB the 4 MiB L2s serve
L2_GATHER_PEAK_GBS = 18800.0


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def _load_dgl():
    global dgl, fn, data, kernel
    import dgl as _dgl
    import dgl.function as _fn
    from dgl import data as _data, kernel as _kernel
    dgl, fn, data, kernel = _dgl, _fn, _data, _kernel


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-edges", type=int, default=10_000_000)
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 PMC passes that fill roofline.traffic")
    ap.add_argument("--graph-scale", type=float, default=1.0,
                    help="per-GPU graph size as a fraction of Reddit (testing only)")
    ap.add_argument("--workload", default="reddit", choices=["reddit", "rmat"],
                    help="reddit: weak-scaled Reddit-shaped graph (default, the driver's line); "
                         "rmat: one fixed Graph500 R-MAT graph partitioned over the ranks "
                         "(strong scaling, heavy rows chunked)")
    ap.add_argument("--rmat-scale", type=int, default=26)
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="single-GPU study: build the x N graph, keep rank 0's partition and "
                         "time its local g-SpMM against the full (all-gathered) feature matrix "
                         "(no communication; not a driver line)")
    ap.add_argument("--pipeline-chunks", type=int, default=4,
                    help="N>1: halo all-gather chunks overlapped with the local g-SpMM "
                         "(0 = one all-gather, then the kernel; bit-exact rows)")
    ap.add_argument("--halo-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="N>1: wire type of the exchanged remote rows (bf16 halves the "
                         "exchange; rows then carry bf16 rounding of remote inputs)")
    ap.add_argument("--no-bf16-leg", action="store_true",
                    help="N>1: skip the secondary timing of the same step with the bf16 halo")
    ap.add_argument("--no-train-leg", action="store_true",
                    help="skip the secondary timing of a training step (forward + backward)")
    ap.add_argument("--no-rmat-leg", action="store_true",
                    help="skip the secondary RMAT strong-scaling block (rmat26)")
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="run the multi-rank code path (RCCL group, partition, collectives) "
                         "on a world of one rank (single-GPU rehearsal; not a driver line)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL) for runs; gloo lets several ranks share one GPU "
                         "to rehearse the multi-rank path")
    ap.add_argument("--no-model-legs", action="store_true",
                    help="N=1: skip the model legs (gcn_reddit, gat, sage, gat_pubmed, rgcn)")
    ap.add_argument("--model-legs", default=None,
                    help="N=1: run only these model legs (comma list; a profiling aid)")
    ap.add_argument("--no-strong-leg", action="store_true",
                    help="N>1: skip the fixed-graph (strong scaling) Reddit block")
    ap.add_argument("--emulate-strong", action="store_true",
                    help="with --emulate-world W: rank 0 of the fixed N=1 graph partitioned W "
                         "ways (strong scaling) instead of the x W graph")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="N>1: collective timeout (s) of the process groups; a dead or hung "
                         "peer then ends the job in bounded time")
    ap.add_argument("--no-one-launch-leg", action="store_true",
                    help="skip the one_launch block (the headline step with the source-blocked "
                         "schedule off)")
    ap.add_argument("--no-sage-rmat-leg", action="store_true",
                    help="skip configs[3]'s GraphSAGE-mean epochs on the rmat leg's graph")
    ap.add_argument("--leg-deadline", type=float, default=None,
                    help="seconds a secondary leg may run before rank 0 prints the line built "
                         "so far (with the leg's error) and exits; default: the collective "
                         "timeout less 60 s at N>1, 900 s at N=1")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: run every leg through the library's host kernels with gloo "
                         "(tests of the launcher and the multi-rank plumbing; not a driver line)")
    return ap


# ---------------------------------------------------------------------------
# launcher: --gpus N > 1 without an outer torchrun
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
    finally:
        s.close()


def launch_command(args, argv, env, port=None):
    """The child command that runs this script as ``args.gpus`` ranks, or None
    when this process is to run as a rank itself (one GPU, or WORLD_SIZE
    already set by an outer launcher). Decided from argv and the environment
    only: nothing here loads the HIP library or touches a device."""
    if args.gpus <= 1 or "WORLD_SIZE" in env:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
            "--master-port", str(port if port is not None else _free_port()),
            os.path.abspath(__file__)] + list(argv)


class _Terminated(Exception):
    def __init__(self, signum):
        Exception.__init__(self, "signal %d" % signum)
        self.signum = signum


def relay(cmd, env=None):
    """Run ``cmd`` as a child in its own session, pass rank 0's JSON line
    through to stdout (every other line of the child's stdout to stderr),
    return its exit code. SIGTERM,
    SIGINT and SIGHUP to this process, or any exception here, kill the
    child's whole process group (the torchrun agent and every rank) before
    this process exits (128 + the signal's number for a signal). This
    process never touches the GPU."""
    import signal
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")

    def on_signal(signum, frame):
        raise _Terminated(signum)
    old = {sig: signal.signal(sig, on_signal)
           for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    proc = None
    try:
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, start_new_session=True,
                                bufsize=1, universal_newlines=True)
        for line in proc.stdout:
            # the JSON line to stdout, anything a library printed there to stderr
            out = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            out.write(line)
            out.flush()
        return proc.wait()
    except _Terminated as t:
        log("relay: %s, killing the ranks' process group" % t)
        _kill_group(proc)
        return 128 + t.signum
    except BaseException:
        _kill_group(proc)
        raise
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)


def _descendants(pid):
    """Every live descendant pid of ``pid`` (from /proc's parent links)."""
    kids = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open("/proc/%s/stat" % d) as f:
                st = f.read()
            ppid = int(st[st.rindex(")") + 2:].split()[1])
        except (OSError, ValueError, IndexError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    out, todo = [], [pid]
    while todo:
        for c in kids.get(todo.pop(), []):
            out.append(c)
            todo.append(c)
    return out


def _kill_group(proc):
    """End the child and everything under it: torchrun starts its ranks in
    sessions of their own, so the child's process group alone does not reach
    them. SIGTERM first (torchrun stops its workers), then SIGKILL to every
    descendant still there."""
    if proc is None:
        return
    tree = set(_descendants(proc.pid))
    for sig in (15, 9):
        for pid in [proc.pid] + sorted(tree):
            try:
                os.kill(pid, sig)
            except OSError:
                pass
        try:
            os.killpg(proc.pid, sig)
        except OSError:
            pass
        deadline = time.time() + (10 if sig == 15 else 30)
        while time.time() < deadline:
            tree |= set(_descendants(proc.pid)) if proc.poll() is None else set()
            alive = [p for p in tree if os.path.exists("/proc/%d" % p) and
                     not _zombie(p)]
            if proc.poll() is not None and not alive:
                return
            time.sleep(0.2)


def _zombie(pid):
    try:
        with open("/proc/%d/stat" % pid) as f:
            st = f.read()
        return st[st.rindex(")") + 2] == "Z"
    except (OSError, ValueError, IndexError):
        return True


def world_mismatch(args, env):
    """Error text when an outer launcher's WORLD_SIZE disagrees with --gpus."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world != args.gpus and not (world == 1 and args.dist_rehearsal):
        return "--gpus %d but WORLD_SIZE %d" % (args.gpus, world)
    return None


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def algorithmic_bytes(num_edges, num_rows, feat):
    """Gather model: each edge reads one int32 column id and one fp32 source
    row; each row reads its int64 indptr entry and writes one fp32 row."""
    return num_edges * (4 * feat + 4) + num_rows * (4 * feat + 8)


def cpu_sample(src, dst, n, target_edges):
    """The CPU baseline's bounded sample: the in-edges (edge-id order) of the
    first rows of the graph, ``target_edges`` of them, as host tensors
    (rows, d, s). Taken before the edge lists are released; timed after the
    timed region."""
    deg = torch.bincount(dst, minlength=n)
    cum = torch.cumsum(deg, 0)
    rows = int(torch.searchsorted(cum, torch.tensor(target_edges, device=cum.device))) + 1
    rows = min(rows, n)
    sel = dst < rows
    return rows, dst[sel].cpu(), src[sel].cpu()


def cpu_baseline(sample, n, h_cpu, seconds_budget=16.0):
    """The reference path on host cores: torch.sparse.mm(COO(dst, src), H) on
    the sample, timed at one thread and at torch's default thread count (the
    setting the reference runs with); ``value`` is the faster of the two.
    ``h_cpu`` None: a full-size (n, F) table whose pages are touched only for
    the sample's source rows (random features there): the gathers spread over
    the whole table's address range, as on the GPU, without allocating it
    (RMAT-26: 34 GB of address space, the sample's rows resident)."""
    rows, d, s = sample
    threads = torch.get_num_threads()
    e = int(s.numel())
    ncols = n
    touched = None
    if h_cpu is None:
        uniq = torch.unique(s)
        touched = int(uniq.numel())
        h_cpu = torch.empty(n, FEAT)  # untouched pages are never materialised
        h_cpu[uniq] = torch.rand(touched, FEAT) * 2 - 1
    A = torch.sparse_coo_tensor(torch.stack([d, s]), torch.ones(e), (rows, ncols))
    runs = {}
    try:
        for nt in sorted({1, threads}):
            torch.set_num_threads(nt)
            # at least 2 calls, then calls until about half the budget is spent
            # (10-30 s of CPU work in all; a fast host runs the 10M-edge sample
            # in ~0.25 s a call)
            reps, t_total = 0, 0.0
            while reps < 2 or (t_total < seconds_budget / 2 and reps < 40):
                t0 = time.perf_counter()
                ref = torch.sparse.mm(A, h_cpu)
                t_total += time.perf_counter() - t0
                reps += 1
            runs[nt] = (e * reps / t_total, reps)
    finally:
        torch.set_num_threads(threads)
    best = max(runs, key=lambda k: runs[k][0])
    build = build_cpu_baseline(rows, ncols, d, s, h_cpu, ref)
    return {"value": runs[best][0], "unit": "edges/s", "cores": best, "kind": "reference",
            "by_threads": {str(k): v[0] for k, v in sorted(runs.items())},
            "build_kernel": build,
            "sample": "torch.sparse.mm on the reference's uncoalesced COO (fp32 ones, "
                      "edge-id order) over the in-edges of the first %d rows: %d edges x "
                      "F=%d%s, %s call(s), torch %s, timed at %s thread(s) (torch default %d, "
                      "the job's host-core share; value = the faster, at %d: the product "
                      "is single-threaded in practice); host has %d cpus"
                      % (rows, e, h_cpu.shape[1],
                         "" if touched is None else
                         " (the full %d-row table's address range; its %d referenced rows "
                         "resident)" % (n, touched),
                         "/".join(str(v[1]) for _, v in sorted(runs.items())),
                         torch.__version__, " and ".join(str(k) for k in sorted(runs)),
                         threads, best, os.cpu_count() or 0)}


def build_cpu_baseline(rows, ncols, d, s, h_cpu, ref):
    """the build's own host g-SpMM (libdgl_hip's
    dglhip_gspmm_host over a CSR, std::thread-parallel) on the same sample, at
    the host-core share the job has ($OMP_NUM_THREADS / $DGL_NUM_THREADS, else
    every hardware thread), and whether it reproduces (i) bit for bit."""
    adj = kernel.from_coo(rows, ncols, d, s, kernel.ORDER_EID, "cpu")
    out = kernel.gspmm(adj, "copy_u", "sum", h_cpu)  # warm: builds the host CSR once
    reps, t_total = 0, 0.0
    while reps < 3:
        t0 = time.perf_counter()
        out = kernel.gspmm(adj, "copy_u", "sum", h_cpu)
        t_total += time.perf_counter() - t0
        reps += 1
    threads = int(os.environ.get("DGL_NUM_THREADS") or os.environ.get("OMP_NUM_THREADS")
                  or (os.cpu_count() or 1))
    return {"value": int(s.numel()) * reps / t_total, "unit": "edges/s",
            "cores": min(threads, 64), "kind": "build",
            "bit_identical_to_reference": bool(torch.equal(out, ref.to_dense()
                                                           if ref.is_sparse else ref))}


def pmc_traffic(child_args, per_call_calls=None):
    """HBM bytes of the g-SpMM from two rocprofv3 --pmc passes (FETCH_SIZE,
    WRITE_SIZE) of a short child run of this script, corrected as
    MI355X_MICROARCH.md §HBM prescribes (tools/pmc_traffic.py): mean per
    gspmm_sum_kernel launch, or (``per_call_calls``) every g-SpMM kernel of a
    call (light rows + chunks + combine) summed and divided by the number of
    calls. Runs before this process touches the GPU; None if the profiler is
    unavailable."""
    import shutil
    import tempfile
    from tools.pmc_traffic import traffic, traffic_per_call
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    env = dict(os.environ, TMPDIR="/tmp")
    out = tempfile.mkdtemp(prefix="dglhip_pmc_", dir="/tmp")
    csvs = []
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, counter)
        cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__)] + child_args
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, timeout=300, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except (subprocess.SubprocessError, OSError) as err:
            log("pmc pass %s failed: %s" % (counter, err))
            return None
        csvs.append(os.path.join(d, "run_counter_collection.csv"))
    try:
        if per_call_calls:
            return traffic_per_call(csvs[0], csvs[1], per_call_calls)
        return traffic(csvs[0], csvs[1])
    except (OSError, ValueError, KeyError) as err:
        log("pmc parse failed: %s" % err)
        return None
    finally:
        shutil.rmtree(out, ignore_errors=True)


HALO_DTYPE = {"fp32": None, "bf16": torch.bfloat16}


def describe_partition(pg, world, args):
    backend = "RCCL" if args.dist_backend == "nccl" else args.dist_backend
    if pg.halo_mode == "alltoall":
        halo = "%s all-to-allv halo (%d referenced remote rows on this rank)%s" % (
            backend, pg.num_halo, " in %d chunks, the own-source segment and each landed "
            "chunk overlapped with the rest of the exchange" % args.pipeline_chunks
            if args.pipeline_chunks > 0 else "")
    else:
        halo = "%s all-gather halo%s" % (
            backend, " in %d chunks overlapped with the local g-SpMM" % args.pipeline_chunks
            if args.pipeline_chunks > 0 else "")
    if pg.halo_dtype is not None:
        halo += ", remote rows on the wire as bf16 (fp32 reduction)"
    return "%d-way 1-D dst-row partition, %s" % (world, halo)


def _window_marker(dev):
    """A one-wave spin kernel on the current stream, outside the timed
    region, on each side of it: in a rocprofv3 kernel trace the dispatches
    between two markers are exactly the timed steps' (tools/window_stats.py
    turns them into a stats table without the graph setup's kernels)."""
    if dev.type == "cuda":
        torch.cuda._sleep(1)


def timed_steps(step, steps, warmup, world, dev):
    """W warm-up steps, then K steps bracketed by barrier + synchronize; returns
    (max-over-ranks seconds, this rank's g-SpMM kernel ms per step). On the
    host path (no device launches to time) the kernel ms is the rank's own
    wall time per step.

    Kernel ms: the GPU span of every g-SpMM call of the step between two
    events on the stream the library launches on (kernel.timing_enable
    per_call: the call's launches and its output's zero fill; at N > 1 the
    waits on the exchange precede a segment's first event, so they stay out).
    An event pair around every launch instead (r01-r03) put 38 markers into
    each blocked call of the timed region: 0.18 ms per N = 1 step (3.84 ms per
    call without them, tools/items_policy_ab.py)."""
    for _ in range(warmup):
        step()
    _sync(dev)
    # the setup's garbage collected now, and no collection inside the timed
    # region (as timeit does): a collection there once freed the setup's
    # 0.9-GB host edge arrays in the middle of a step (r05, a 170-ms stall)
    gc.collect()
    gc_was = gc.isenabled()
    gc.disable()
    try:
        if dist.is_initialized():
            dist.barrier()
        kernel.timing_enable(True, per_call=dev.type == "cuda")
        _window_marker(dev)  # tools/window_stats.py: the timed region's kernels
        _sync(dev)
        t_start = time.perf_counter()
        for _ in range(steps):
            step()
        _sync(dev)
        own = time.perf_counter() - t_start
        if dist.is_initialized():
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        _window_marker(dev)
    finally:
        if gc_was:
            gc.enable()
    kms, launches = kernel.timing_read()
    kernel.timing_enable(False)
    if launches == 0:
        kms = own * 1e3
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, kms / steps


def per_rank(values, world, dev):
    """Every rank's tuple of floats, gathered to all ranks (a SUM all-reduce
    over a rank-slotted tensor: works on every backend)."""
    k = len(values)
    t = torch.zeros(world * k, dtype=torch.float64, device=dev)
    r = dist.get_rank() if dist.is_initialized() else 0
    t[r * k:(r + 1) * k] = torch.tensor(values, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(t)
    t = t.cpu().tolist()
    return [t[i * k:(i + 1) * k] for i in range(world)]


def pipelined_blocks(pg):
    """Source-blocked launches of a pipelined partition's segments per step
    (0: every segment one launch): the own rows in fp32, the halo's at its
    wire type."""
    if pg.chunks <= 0:
        return kernel.blocked_schedule(pg.adj, torch.empty(2, FEAT, device=pg.device))
    halo = torch.float32 if pg.halo_dtype is None else pg.halo_dtype
    return kernel.segment_blocks(pg.seg_csrs, FEAT,
                                 [torch.float32] + [halo] * (len(pg.seg_csrs) - 1))


def sweep_segments(pg):
    """Segments of a pipelined partition the plan runs on the accumulating
    source sweep (DESIGN.md §4.1 "Source sweep"; the N = 8 halo chunks)."""
    if pg.chunks <= 0 or pg.device.type != "cuda":
        return 0
    n = 0
    for csr in pg.seg_csrs:
        if csr.nnz:
            path, _ = csr.plan.schedule(kernel.MSG_COPY_U, kernel.RED_SUM_ACCUM, FEAT, 0,
                                        csr.num_cols)
            n += path == kernel.PLAN_PATH_SWEEP
    return n


def gather_peak(table_bytes, blocks=0):
    """(peak GB/s, source) of a row gather from a ``table_bytes`` table: with
    the source-blocked schedule (``blocks`` > 0) the guide's L2 indexed-row
    rate; else the Infinity-Cache random-row rate while the table fits the
    cache, else the HBM spec peak."""
    if blocks:
        return L2_GATHER_PEAK_GBS, (
            "source-blocked gather (%d launches of ~%.1f MB slices of the %.0f MB table, "
            "each continuing every row's chain): the slices are served by the XCDs' 4 MiB "
            "L2s; the guide's measured rate for indexed rows from L2, 16.8-18.8 TB/s "
            "chip-wide (MI355X_MICROARCH.md 'Indexed rows'), upper end"
            % (blocks, table_bytes / blocks / 1e6, table_bytes / 1e6))
    if table_bytes < INFINITY_CACHE_BYTES:
        return IC_GATHER_PEAK_GBS, (
            "Infinity-Cache-resident gather (table %.0f MB < 256 MiB): the guide's measured "
            "random-row rate from the Infinity Cache, 8.6 TB/s (MI355X_MICROARCH.md 'Indexed "
            "rows'); no counter on this part separates Infinity-Cache hits from DRAM reads"
            % (table_bytes / 1e6))
    return HBM_PEAK_GBS, "HBM3E spec peak (MI355X_MICROARCH.md)"


def roofline_block(num_edges, num_rows, kms, world, dev, table_bytes, blocks=0, **extra):
    """The g-SpMM roofline of this rank (algorithmic bytes of its launch(es)
    per step over its kernel ms per step) against the gather's ceiling for a
    table of ``table_bytes`` (gather_peak), with every rank's figures in
    ``per_rank`` when N > 1. ``effective_gather_frac`` is the same rate over
    the 8 TB/s HBM spec: a figure of effective gather bandwidth, not of DRAM
    bytes (FETCH_SIZE / TCC_EA0_RDREQ_DRAM count Infinity-Cache hits)."""
    peak, source = gather_peak(table_bytes, blocks)
    b = algorithmic_bytes(num_edges, num_rows, FEAT)
    ach = b / (kms * 1e-3) / 1e9 if kms > 0 else None
    roof = {"bound": "hbm", "achieved": ach, "peak": peak, "unit": "GB/s",
            "frac": None if ach is None else ach / peak,
            "effective_gather_frac": None if ach is None else ach / HBM_PEAK_GBS,
            "peak_source": source, "kernel_ms": kms, "bytes_per_launch": b}
    roof.update(extra)
    if world > 1:
        rows = per_rank([float(b), float(kms)], world, dev)
        roof["per_rank"] = [{"rank": i, "bytes_per_step": r[0], "kernel_ms": r[1],
                             "achieved": r[0] / (r[1] * 1e-3) / 1e9 if r[1] > 0 else None,
                             "frac": r[0] / (r[1] * 1e-3) / 1e9 / peak
                             if r[1] > 0 else None} for i, r in enumerate(rows)]
    return roof


def compulsory_bytes(num_edges, num_rows, num_sources, feat):
    """Bytes a g-SpMM launch must move to or from DRAM at least: every
    referenced source row once, the column ids and indptr once, the output
    once (any cache re-use only lowers the rest)."""
    return num_sources * 4 * feat + num_edges * 4 + num_rows * (4 * feat + 8)


def exchange_block(pg, h_local, steps, world, dev):
    """N > 1: the halo exchange of one step alone (the pack, then RCCL's
    all_gather_into_tensor or all_to_all_single, as the step issues it, in
    one piece), timed like the step; with the step's own time it shows how
    much of the exchange the pipelined segments hide."""
    from dgl.distributed import _AllGatherRows, _AllToAllRows
    if pg.halo_mode == "alltoall":
        def step():
            _AllToAllRows.apply(h_local, pg.send_idx, pg.send_splits, pg.recv_splits, pg.group,
                                pg.halo_dtype)
        recv_rows = sum(pg.recv_splits)
    else:
        def step():
            _AllGatherRows.apply(h_local, pg.max_rows, pg.group, pg.halo_dtype)
        recv_rows = (world - 1) * pg.max_rows
    el, _ = timed_steps(step, steps, 1, world, dev)
    per = el / steps
    nbytes = recv_rows * FEAT * (2 if pg.halo_dtype is not None else 4)
    return {"ms_per_step": per * 1e3, "mode": pg.halo_mode, "recv_bytes_rank0": nbytes,
            "recv_GBs_rank0": nbytes / per / 1e9,
            "note": "the step's halo exchange alone (max over ranks); rank 0's received "
                    "bytes over that time"}


# exit code of a run that printed its line but lost a leg (a failed or hung
# peer, a hung kernel): the relay and the driver see a failure
EXIT_LEG_FAILED = 3
_LINE_LOCK = threading.Lock()
_LINE_DONE = [False]


def emit_line(result):
    """Print the JSON line once per process: the leg-deadline timer's thread
    and the main thread can both reach here; the first one prints."""
    with _LINE_LOCK:
        if _LINE_DONE[0]:
            return False
        text = json.dumps(result)
        sys.stdout.write(text + "\n")
        sys.stdout.flush()
        _LINE_DONE[0] = True
        return True


class LegRunner(object):
    """Runs the secondary legs after the headline on every rank so that one
    leg's failure cannot lose the line (r03 verdict, Weak 6).

    * Each leg is ``setup`` (rank-local work: graph generation, buffers)
      then ``run`` (timing, collectives). Every rank catches its own
      exception; after each phase the ranks exchange their errors over a
      separate gloo group (``agree``), so a rank that failed in setup makes
      every rank skip the leg together, with no collective left waiting.
    * A failed leg is recorded as ``{"error": ...}`` (every failing rank's
      message) and, at N > 1, the later legs are skipped: a collective may
      have been left half-done.
    * Rank 0 arms a deadline per leg (``--leg-deadline``, shorter than the
      collectives' timeout): a leg still running then (a hung peer, a hung
      kernel) makes rank 0 print the line built so far, with the leg's
      error, and exit, before the process group's timeout (with
      TORCH_NCCL_ASYNC_ERROR_HANDLING=1) tears the ranks down.
    * ``DGLHIP_BENCH_FAIL=<leg>:<rank>[:run]`` injects a failure into one
      rank's setup (or run) phase of one leg (tests)."""

    def __init__(self, result, world, rank, deadline, group=None):
        self.result, self.world, self.rank = result, world, rank
        self.deadline = deadline
        self.group = group
        self.failed = None
        inject = os.environ.get("DGLHIP_BENCH_FAIL", "")
        parts = inject.split(":") if inject else []
        self.inject = (parts[0], int(parts[1]), parts[2] if len(parts) > 2 else "setup") \
            if len(parts) >= 2 else None

    def _maybe_fail(self, name, phase):
        if self.inject and self.inject[0] == name and self.inject[1] == self.rank and \
                self.inject[2] == phase:
            raise RuntimeError("injected failure (DGLHIP_BENCH_FAIL) in leg %s, %s phase"
                               % (name, phase))

    def agree(self, err):
        """Every rank's error string (None: ok), on every rank."""
        if self.world == 1 or not dist.is_initialized():
            return [err]
        out = [None] * self.world
        dist.all_gather_object(out, err, group=self.group)
        return out

    def _arm(self, name):
        if self.rank != 0 or not self.deadline:
            return None
        import threading

        def fire():
            line = dict(self.result)
            line[name] = {"error": "leg still running after %.0f s (a peer failed or hung, "
                                   "or a kernel hung): rank 0 printed the line and exited"
                                   % self.deadline}
            try:
                emit_line(line)
            finally:
                # a hung peer or kernel is a failed run: the line is printed
                # (the headline is intact) but the exit code says so
                os._exit(EXIT_LEG_FAILED)
        t = threading.Timer(self.deadline, fire)
        t.daemon = True
        t.start()
        return t

    def run(self, name, setup, run=None, collective=True):
        """Run one leg; its dict (or error) goes to result[name]. ``run``
        gets setup's return value. Returns True when the leg succeeded."""
        if self.failed is not None and collective and self.world > 1:
            self.result[name] = {"skipped": "after the failure of leg %r" % self.failed}
            return False
        timer = self._arm(name)
        t0 = time.time()
        try:
            err = state = None
            try:
                self._maybe_fail(name, "setup")
                state = setup()
            except Exception as e:  # noqa: BLE001 - any failure of the leg is recorded
                err = "rank %d (setup): %r" % (self.rank, e)
            errs = self.agree(err)
            if all(x is None for x in errs) and run is not None:
                try:
                    self._maybe_fail(name, "run")
                    state = run(state)
                except Exception as e:  # noqa: BLE001
                    err = "rank %d: %r" % (self.rank, e)
                errs = self.agree(err)
        finally:
            if timer is not None:
                timer.cancel()
        bad = [x for x in errs if x is not None]
        if bad:
            self.result[name] = {"error": "; ".join(bad)}
            if collective:
                self.failed = name
            log("leg %s failed: %s" % (name, "; ".join(bad)))
            return False
        self.result[name] = state
        log("leg %s done in %.1fs" % (name, time.time() - t0))
        return True


def rmat_setup(args, rank, dev):
    """The rmat leg's rank-local part: the graph (every rank generates the
    same one), its CPU sample on rank 0, its distinct-source count."""
    t0 = time.time()
    src, dst, n = data.rmat(args.rmat_scale, 16, seed=0, device=dev)
    n_src = int((torch.bincount(src, minlength=n) > 0).sum())  # distinct sources
    sample = None
    if rank == 0 and not args.no_cpu_baseline:
        sample = cpu_sample(src, dst, n, 2_000_000)
    log("rmat leg: scale %d, %d edges, generated in %.1fs" % (args.rmat_scale, int(src.numel()),
                                                              time.time() - t0))
    return {"src": src, "dst": dst, "n": n, "n_src": n_src, "sample": sample}


def rmat_run(args, world, rank, dev, st, pmc=None):
    """RMAT strong scaling on the same ranks: one fixed graph, 1-D dst-row
    partition, heavy rows chunked (kernel.set_row_split("auto"))."""
    from dgl.distributed import PartitionedGraph, balanced_bounds
    old = kernel.set_row_split("auto")
    try:
        t0 = time.time()
        src, dst, n, n_src, sample = st["src"], st["dst"], st["n"], st["n_src"], st["sample"]
        st.clear()
        E = int(src.numel())
        gen = torch.Generator(device=dev)
        gen.manual_seed(1)
        if not dist.is_initialized():
            adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
            del src, dst
            h = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1
            local_edges, local_rows = E, n

            def step():
                kernel.gspmm(adj, "copy_u", "sum", h)
            par = "single GPU"
        else:
            bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
            lo, hi = int(bounds[rank]), int(bounds[rank + 1])
            sel = (dst >= lo) & (dst < hi)
            pg = PartitionedGraph(n, src[sel], dst[sel], bounds, dev,
                                  pipeline_chunks=args.pipeline_chunks,
                                  halo_dtype=HALO_DTYPE[args.halo_dtype])
            del src, dst, sel
            h_local = torch.rand(hi - lo, FEAT, generator=gen, device=dev) * 2 - 1
            local_edges, local_rows = pg.num_edges, pg.num_local

            def step():
                pg.update_all(h_local)
            par = describe_partition(pg, world, args)
        _sync(dev)
        log("rmat leg: setup %.1fs" % (time.time() - t0))
        steps = min(args.steps, 5)
        elapsed, kms = timed_steps(step, steps, 2, world, dev)
        exch = exchange_block(pg, h_local, steps, world, dev) if dist.is_initialized() else None
        # HBM-honest roofline: H (34 GB at scale 26) cannot stay in the caches
        roof = roofline_block(
            local_edges, local_rows, kms, world, dev, n * FEAT * 4,
            traffic=None if pmc is None else pmc["bytes"],
            kernel="g-SpMM copy_u+sum, heavy rows chunked (light-row, chunk and combine "
                   "kernels of one call%s)" % (", every segment of the pipelined partition"
                                               if dist.is_initialized() else ""),
            traffic_source=None if pmc is None else
            "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes (bench.py --workload "
            "rmat), every g-SpMM kernel of a call summed, mean per call, read x2 (gfx950)",
            regime="HBM-bound random row gather (H = %.0f GB >> 256 MB Infinity Cache)"
                   % (n * FEAT * 4 / 1e9))
        # frac here is an effective-gather fraction (algorithmic gather bytes
        # over the HBM spec), not DRAM utilisation: most gathers hit a small
        # hot set that the Infinity Cache serves (dram_traffic bounds below)
        roof["frac_kind"] = ("effective gather: algorithmic bytes (every edge's source row "
                             "read in full) / kernel time / HBM spec peak; not DRAM "
                             "utilisation (see dram_traffic)")
        if dist.is_initialized():
            roof["note"] = ("rank 0's local algorithmic bytes (its edges and rows) over rank "
                            "0's g-SpMM kernel ms per step; per_rank: every rank")
        else:
            # DRAM bytes per call lie between the compulsory bytes (every
            # referenced row once) and the fabric bytes (which include
            # Infinity-Cache hits): no counter separates the two on gfx950
            roof["dram_traffic"] = {
                "lower_bound": compulsory_bytes(E, n, n_src, FEAT),
                "upper_bound": None if pmc is None else pmc["bytes"],
                "note": "compulsory bytes (%d distinct source rows once, ids, indptr, output) "
                        "<= DRAM bytes <= fabric bytes (FETCH_SIZE x2 + WRITE_SIZE, which "
                        "count Infinity-Cache hits)" % n_src}
        cpu = None
        if sample is not None:
            t2 = time.time()
            cpu = cpu_baseline(sample, n, None, seconds_budget=10.0)
            log("rmat cpu baseline took %.1fs" % (time.time() - t2))
        if not dist.is_initialized() and not args.no_sage_rmat_leg:
            # configs[3]'s model on this same graph next (sage_rmat leg)
            del h
            _RMAT_KEEP.update(adj=adj, n=n, sample=sample)
        return {"value": E * steps / elapsed, "unit": "edges/s", "n_gpus": world,
                "steps": steps, "warmup": 2, "ms_per_step": elapsed / steps * 1e3,
                "scaling": "strong",
                "config": "rmat-%d (Graph500 0.57/0.19/0.19/0.05, ids permuted, seed 0): "
                          "%d nodes, %d edges, feat=%d, heavy rows chunked"
                          % (args.rmat_scale, n, E, FEAT),
                "parallelism": par, "kernel_ms_rank0": kms, "roofline": roof,
                "halo_exchange": exch, "cpu_baseline": cpu}
    finally:
        kernel.set_row_split(old)


# the rmat leg's graph, handed to the sage_rmat leg at N = 1 (one graph of
# 1.07B edges in memory, built once)
_RMAT_KEEP = {}


def reddit_graph(args, scale, dev):
    """The synthetic Reddit-shaped graph at ``scale`` x its size (times
    --graph-scale, a testing knob)."""
    if args.graph_scale == 1.0:
        return data.reddit_like(scale=scale, seed=0, device=dev)
    return data.chung_lu(int(data.REDDIT_NODES * scale * args.graph_scale),
                         int(data.REDDIT_EDGES * scale * args.graph_scale),
                         data.REDDIT_MAX_OVER_MEAN, seed=0, device=dev)


def strong_setup(args, world, rank, dev):
    """The fixed-graph block's rank-local part: the N = 1 Reddit-shaped graph
    (every rank generates it) and this rank's rows of it."""
    from dgl.distributed import balanced_bounds
    src, dst, n = reddit_graph(args, 1, dev)
    bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    sel = (dst >= lo) & (dst < hi)
    return {"n": n, "E": int(src.numel()), "bounds": bounds, "lo": lo, "hi": hi,
            "src": src[sel], "dst": dst[sel]}


def strong_run(args, world, rank, dev, st):
    """N > 1: the headline step on the FIXED N = 1 graph (114.8M edges at every
    N), 1-D partitioned like the weak-scaled line: value = all its edges per
    step over the max-over-ranks step time (scaling "strong")."""
    from dgl.distributed import PartitionedGraph
    n, E, lo, hi = st["n"], st["E"], st["lo"], st["hi"]
    pg2 = PartitionedGraph(n, st.pop("src"), st.pop("dst"), st["bounds"], dev,
                           pipeline_chunks=args.pipeline_chunks,
                           halo_dtype=HALO_DTYPE[args.halo_dtype])
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    h2 = torch.rand(hi - lo, FEAT, generator=gen, device=dev) * 2 - 1

    def step2():
        pg2.update_all(h2)
    el, kms = timed_steps(step2, args.steps, args.warmup, world, dev)
    roof = roofline_block(pg2.num_edges, pg2.num_local, kms, world, dev, n * FEAT * 4,
                          pipelined_blocks(pg2),
                          kernel="gspmm_sum_kernel<copy_u> (rank 0, every segment of the "
                                 "pipelined partition)")
    return {"value": E * args.steps / el, "unit": "edges/s", "n_gpus": world,
            "ms_per_step": el / args.steps * 1e3, "kernel_ms_rank0": kms, "scaling": "strong",
            "config": "reddit-shaped x1%s (the N = 1 graph): %d nodes, %d edges, feat=%d, "
                      "1-D partitioned over %d ranks"
                      % ("" if args.graph_scale == 1.0 else " (graph-scale %g)" % args.graph_scale,
                         n, E, FEAT, world),
            "parallelism": describe_partition(pg2, world, args), "roofline": roof,
            "halo_exchange": exchange_block(pg2, h2, args.steps, world, dev)}


def _claim_stdout():
    """Keep the process's stdout for the one JSON line. Libraries write to
    file descriptor 1 themselves (gloo's "[Gloo] Rank r is connected to ..."
    for every group it builds, RCCL and ROCm notices): point descriptor 1 at
    stderr and give Python a stream on a duplicate of the original stdout."""
    sys.stdout.flush()
    keep = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(keep, "w", buffering=1)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = build_parser().parse_args(argv)
    cmd = launch_command(args, argv, os.environ)
    if cmd is not None:
        # N ranks, one process per GPU: the child torchrun starts them; this
        # process never loads the HIP library nor touches a device
        log("starting %d ranks: %s" % (args.gpus, " ".join(cmd)))
        return relay(cmd)
    err = world_mismatch(args, os.environ)
    if err is not None:
        log("error: " + err)
        return 2
    _claim_stdout()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    on_cpu = args.device == "cpu"
    if on_cpu:
        args.no_traffic = True
        if args.dist_backend == "nccl":
            args.dist_backend = "gloo"
    pmc = None
    rmat_pmc = None
    side_group = None
    if world == 1 and not args.no_traffic and args.workload == "reddit" and not args.dist_rehearsal:
        t0 = time.time()  # before this process initialises the GPU
        # every g-SpMM kernel of the 3 calls (warm-up + 2 steps), per call
        # (no other leg: every g-SpMM kernel of the child run is summed)
        pmc = pmc_traffic(["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-traffic",
                           "--no-rmat-leg", "--no-train-leg", "--no-model-legs",
                           "--no-one-launch-leg", "--no-sage-rmat-leg"],
                          per_call_calls=3)
        if not args.no_rmat_leg and args.emulate_world <= 1:
            # the rmat leg's kernels: every g-SpMM kernel of a call, per call
            rmat_pmc = pmc_traffic(["--workload", "rmat", "--rmat-scale", str(args.rmat_scale),
                                    "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                                    "--no-traffic"], per_call_calls=3)
        log("pmc traffic passes took %.1fs" % (time.time() - t0))
    _load_dgl()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if on_cpu:
        dev = torch.device("cpu")
    else:
        dev_index = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    if world > 1 or args.dist_rehearsal:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29631")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        # a dead or hung peer ends the job in bounded time (r03 verdict, Weak 6)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        from datetime import timedelta
        tmo = timedelta(seconds=args.dist_timeout)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(args.dist_backend, timeout=tmo)
        # the legs' error exchange (LegRunner.agree) on its own gloo group
        side_group = dist.new_group(backend="gloo", timeout=tmo)

    t0 = time.time()
    real_reddit = None
    blocks = 0
    nsw = 0  # pipelined segments on the accumulating source sweep
    if args.workload == "rmat":
        src, dst, n = data.rmat(args.rmat_scale, 16, seed=0, device=dev)
        kernel.set_row_split("auto")
        args.no_cpu_baseline = True
    elif (not dist.is_initialized() and args.graph_scale == 1.0 and args.emulate_world <= 1
          and data._on_disk("reddit", os.environ.get("DGL_DATA_DIR"))):
        # the real graph when its release files are on the box
        root = os.environ["DGL_DATA_DIR"]
        ds = data.RedditDataset(root)
        s0, d0 = ds.graph
        loops = torch.arange(ds.num_nodes)
        src = torch.cat([s0, loops]).to(dev)
        dst = torch.cat([d0, loops]).to(dev)
        n = ds.num_nodes
        real_reddit = "Reddit release files under %s (self-loops added)" % root
        del ds, s0, d0, loops
    else:
        src, dst, n = reddit_graph(args, world, dev)
    num_edges_total = int(src.numel())
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    log("rank %d: graph %d nodes %d edges generated in %.1fs" % (rank, n, num_edges_total,
                                                                  time.time() - t0))
    sample = h_cpu = None
    want_cpu = (rank == 0 and not args.no_cpu_baseline and args.workload == "reddit"
                and args.emulate_world <= 1)
    if want_cpu:  # taken now, timed after the timed region
        sample = cpu_sample(src, dst, n, args.cpu_sample_edges)

    if not dist.is_initialized() and args.workload == "rmat" and args.emulate_world <= 1:
        # 1.07B edges: build the device CSR directly (no host copy of the edge list)
        adj = kernel.from_coo(n, n, dst, src, kernel.ORDER_EID, dev)
        del src, dst
        src = dst = None
        h = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1
        num_local_edges, num_rows = num_edges_total, n

        def step():
            kernel.gspmm(adj, "copy_u", "sum", h)
        parallelism = "single GPU (kernel API; heavy rows chunked)"
    elif not dist.is_initialized() and args.emulate_world > 1:
        from dgl.distributed import balanced_bounds
        W = args.emulate_world
        if args.workload == "reddit" and not args.emulate_strong:  # weak: the x W graph
            del src, dst
            src, dst, n = data.reddit_like(scale=W, seed=0, device=dev)
        num_edges_total = int(src.numel())
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), W)
        lo, hi = int(bounds[0]), int(bounds[1])
        sel = (dst >= lo) & (dst < hi)
        num_local_edges, num_rows = int(sel.sum()), hi - lo
        num_edges_total = num_local_edges  # value = this rank's edges / its time
        if args.pipeline_chunks > 0:
            from dgl.distributed import PartitionedGraph
            pg = PartitionedGraph(n, src[sel], dst[sel], bounds, dev,
                                  pipeline_chunks=args.pipeline_chunks,
                                  halo_dtype=HALO_DTYPE[args.halo_dtype], rank=0, world=W)
            h_local = torch.rand(hi - lo, FEAT, generator=gen, device=dev) * 2 - 1
            pg.update_all(h_local)  # allocates the halo buffer
            bufs = pg.halo if isinstance(pg.halo, list) else [pg.halo]
            for buf in bufs:
                if buf.dtype == torch.float16:  # bf16 rows in their wire view
                    buf = buf.view(torch.bfloat16)
                buf.uniform_(-1, 1)

            def step():
                pg.update_all(h_local)
            blocks = pipelined_blocks(pg)
            mode = ("pipelined segments (own + all-to-allv halo of %d rows in %d chunks)"
                    % (pg.num_halo, args.pipeline_chunks)
                    if pg.halo_mode == "alltoall" else
                    "pipelined segments (own + %d halo chunks)" % args.pipeline_chunks)
        else:
            adj = kernel.from_coo(hi - lo, n, dst[sel] - lo, src[sel], kernel.ORDER_EID, dev)
            h = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1

            def step():
                kernel.gspmm(adj, "copy_u", "sum", h)
            blocks = kernel.blocked_schedule(adj, h)
            mode = "one g-SpMM"
        del sel
        parallelism = "emulated rank 0 of %d%s, %s, no communication (H = %.0f MB)" % (
            W, " (fixed N = 1 graph: strong scaling)" if args.emulate_strong else "", mode,
            n * FEAT * 4 / 1e6)
        args.no_cpu_baseline = True
    elif not dist.is_initialized():
        g = dgl.DGLGraph((src.cpu(), dst.cpu()))
        h = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1
        g.ndata["h"] = h
        if want_cpu:
            h_cpu = h.cpu()
        num_local_edges, num_rows = num_edges_total, n
        t1 = time.time()
        g.sparse_adjacency(dev)  # build + cache the device CSR (graph ingestion)
        _sync(dev)
        log("device CSR built in %.1fs" % (time.time() - t1))

        def step():
            g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h_out"))
        parallelism = "single GPU" if not on_cpu else "host (library host kernels)"
        blocks = kernel.blocked_schedule(g.sparse_adjacency(dev), h)
        if blocks:
            parallelism += (", source-blocked schedule: %d launches over contiguous source "
                            "blocks, every row's chain continued block by block. Precondition: "
                            "the edges are numbered source-major, so along every row's slots "
                            "the source blocks never decrease and the blocked chains are the "
                            "edge-id chains (bit-identical); a mutable graph in arbitrary edge "
                            "order fails that check and runs the one-launch schedule instead "
                            "(same bits, about 2x the time on this graph: the one_launch "
                            "block), while a readonly graph's slots are (dst, src)-sorted as "
                            "the reference's ImmutableGraph, so it is blocked in any edge order"
                            % blocks)
    else:
        from dgl.distributed import PartitionedGraph, balanced_bounds
        bounds = balanced_bounds(torch.bincount(dst, minlength=n), world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        sel = (dst >= lo) & (dst < hi)
        pg = PartitionedGraph(n, src[sel], dst[sel], bounds, dev,
                              pipeline_chunks=args.pipeline_chunks,
                              halo_dtype=HALO_DTYPE[args.halo_dtype])
        h_full = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1
        h_local = h_full[lo:hi].contiguous()
        if want_cpu:
            h_cpu = h_full.cpu()
        del h_full, sel
        num_local_edges, num_rows = pg.num_edges, pg.num_local

        def step():
            pg.update_all(h_local)
        parallelism = describe_partition(pg, world, args)
        blocks = pipelined_blocks(pg)
        nsw = sweep_segments(pg) if pg.halo_dtype is None else 0
        if nsw:
            parallelism += ("; %d of the %d segments on the accumulating source sweep (running "
                            "sums in LDS, DESIGN.md 4.1), the rest as listed"
                            % (nsw, len(pg.seg_csrs)))
    del src, dst
    _sync(dev)
    if dev.type == "cuda":
        log("setup done in %.1fs; peak HBM %.1f GB" % (
            time.time() - t0, torch.cuda.max_memory_allocated(dev) / 1e9))

    elapsed, kernel_ms = timed_steps(step, args.steps, args.warmup, world, dev)
    value = num_edges_total * args.steps / elapsed
    roof = roofline_block(
        num_local_edges, num_rows, kernel_ms, world, dev, n * FEAT * 4, blocks,
        traffic=None if pmc is None else pmc["bytes"],
        kernel_timing=("GPU span of each g-SpMM call between two events on the launch stream "
                       "(every launch of the call and its output's zero fill), summed per step"
                       if dev.type == "cuda" else "host wall time per step"),
        kernel="gspmm_sum_kernel<copy_u>%s (rank 0%s)" % (
            " + gspmm_sweep_stream_kernel" if nsw else "",
            ", every segment of the pipelined partition" if dist.is_initialized() else
            ", every block launch and short-row tier of one call" if blocks else ""),
        traffic_source=None if pmc is None else
        "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes, every g-SpMM kernel of a "
        "call summed, mean per call, read x2 (gfx950); EA requests: bytes the L2s did "
        "not serve",
        regime=("L2-served gather: H = %.0f MB in %d source blocks of %.1f MB; traffic "
                "(EA requests) = the bytes the L2s did not serve, from the Infinity Cache "
                "(H and out fit it) or DRAM" % (n * FEAT * 4 / 1e6, blocks,
                                                n * FEAT * 4 / blocks / 1e6)) if blocks else
        ("Infinity-Cache-resident gather: H = %.0f MB fits the 256 MiB Infinity "
                "Cache, whose hits FETCH_SIZE counts as fetches (traffic = fabric bytes, not "
                "DRAM bytes); the DRAM-bound figure is the rmat%d block's roofline"
                % (n * FEAT * 4 / 1e6, args.rmat_scale))
        if n * FEAT * 4 < INFINITY_CACHE_BYTES else
        "HBM-bound gather (H exceeds the Infinity Cache)")
    if blocks:
        roof["launches_per_call"] = blocks  # bytes_per_launch / kernel_ms: per call
        if pmc is not None and kernel_ms > 0:
            # the bytes the L2s did not serve, against the rate the fabric
            # serves random rows at (the Infinity-Cache row rate)
            rate = pmc["bytes"] / (kernel_ms * 1e-3) / 1e9
            roof["l2_miss_traffic_GBs"] = rate
            roof["l2_miss_traffic_frac"] = rate / IC_GATHER_PEAK_GBS
    result = {
        "metric": "edges/sec on update_all g-SpMM (copy_u+sum, feat=128)",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.workload == "reddit" else "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": (real_reddit + "; random U(-1,1) features") if real_reddit else
                ("synthetic (seeded Chung-Lu power-law graph of Reddit's shape; random "
                 "U(-1,1) features)") if args.workload == "reddit" else
                "synthetic (seeded Graph500 R-MAT 0.57/0.19/0.19/0.05, ids permuted)",
        "config": {
            "workload": ("%s x%d%s: %d nodes, %d edges (incl. self-loops), feat=%d"
                         % ("reddit" if real_reddit else "reddit-shaped", world,
                            "" if args.graph_scale == 1.0 else
                            " (graph-scale %g)" % args.graph_scale, n, num_edges_total, FEAT))
                        if args.workload == "reddit" else
                        ("rmat-%d: %d nodes, %d edges, feat=%d, row split %s"
                         % (args.rmat_scale, n, num_edges_total, FEAT, kernel.get_row_split())),
            "global_batch": n,
            "feat": FEAT,
            "parallelism": parallelism,
        },
        "roofline": roof,
        "cpu_baseline": None,
    }
    if on_cpu:
        result["device"] = "cpu (host kernels; plumbing test, not a measurement)"
    deadline = args.leg_deadline
    if deadline is None:
        deadline = max(args.dist_timeout - 60.0, 30.0) if world > 1 else 900.0
    legs = LegRunner(result, world, rank, deadline, group=side_group)
    distributed = dist.is_initialized()

    if distributed:
        legs.run("halo_exchange", lambda: None,
                 lambda _: exchange_block(pg, h_local, args.steps, world, dev))
    if distributed and args.halo_dtype == "fp32" and not args.no_bf16_leg:
        # the opt-in bf16 halo on the same partition (not the headline: remote
        # rows are rounded to bf16, so rows are no longer bit-exact)
        def bf16_run(_):
            pg.set_halo_dtype(torch.bfloat16)
            try:
                el16, k16 = timed_steps(step, args.steps, args.warmup, world, dev)
            finally:
                pg.set_halo_dtype(None)
            return {"value": num_edges_total * args.steps / el16, "unit": "edges/s",
                    "ms_per_step": el16 / args.steps * 1e3, "kernel_ms_rank0": k16,
                    "note": "same partition and step with halo_dtype=bf16: remote rows travel "
                            "and are read as bf16, summed in fp32; own rows exact. Opt-in, not "
                            "the headline (results carry bf16 rounding of remote inputs)"}
        legs.run("halo_bf16", lambda: None, bf16_run)
    if (not distributed and blocks and args.workload == "reddit" and args.emulate_world <= 1
            and not args.no_one_launch_leg):
        # the same step with the source-blocked schedule off: what a graph in
        # arbitrary edge order (which fails the monotone check) runs instead
        def one_launch_run(_):
            old = kernel.set_blocked("off")
            try:
                el1, k1 = timed_steps(step, args.steps, args.warmup, world, dev)
            finally:
                kernel.set_blocked(old)
            return {"value": num_edges_total * args.steps / el1, "unit": "edges/s",
                    "ms_per_step": el1 / args.steps * 1e3, "kernel_ms": k1,
                    "note": "the headline step on the one-launch schedule (source-blocked "
                            "schedule off): the schedule of a graph whose edges are not "
                            "numbered source-major; same bits"}
        legs.run("one_launch", lambda: None, one_launch_run, collective=False)
    if args.workload == "reddit" and args.emulate_world <= 1 and not args.no_train_leg:
        # training step of the same layer: forward + backward (the transposed
        # g-SpMM; at N > 1 the pipelined halo's reverse exchange overlapped with
        # the transposed segments), inputs requiring grad, a fixed upstream grad
        def train_setup():
            if distributed:
                h_tr = h_local.detach().clone().requires_grad_(True)
                d_out = torch.rand(pg.num_local, FEAT, generator=gen, device=dev) * 2 - 1
            else:
                h_tr = h.detach().clone().requires_grad_(True)
                d_out = torch.rand(n, FEAT, generator=gen, device=dev) * 2 - 1
            return h_tr, d_out

        def train_run(st):
            h_tr, d_out = st
            if distributed:
                def train_step():
                    pg.update_all(h_tr).backward(d_out)
            else:
                def train_step():
                    g.ndata["h"] = h_tr
                    g.update_all(fn.copy_src("h", "m"), fn.sum("m", "h_out"))
                    g.ndata["h_out"].backward(d_out)
            try:
                el_tr, k_tr = timed_steps(train_step, args.steps, args.warmup, world, dev)
            finally:
                if not distributed:
                    g.ndata["h"] = h
            return {"value": num_edges_total * args.steps / el_tr, "unit": "edges/s (fwd+bwd)",
                    "ms_per_step": el_tr / args.steps * 1e3, "kernel_ms_rank0": k_tr,
                    "note": "update_all(copy_src, sum) forward + backward (dH = A^T dC through "
                            "the transposed CSR%s) per step, same graph and partition"
                            % ("; halo exchange and its reverse pipelined in %d chunks"
                               % args.pipeline_chunks if distributed and
                               args.pipeline_chunks > 0 else "")}
        legs.run("train_step", train_setup, train_run)
    if distributed and args.workload == "reddit" and not args.no_strong_leg:
        legs.run("strong", lambda: strong_setup(args, world, rank, dev),
                 lambda st: strong_run(args, world, rank, dev, st))
    if sample is not None or world > 1:
        # rank 0, after the timed region (the other ranks wait in agree)
        def cpu_run(_):
            if sample is None:
                return None
            t2 = time.time()
            out = cpu_baseline(sample, n, h_cpu)
            log("cpu baseline took %.1fs" % (time.time() - t2))
            return out
        legs.run("cpu_baseline", lambda: None, cpu_run, collective=False)
    if (world == 1 and args.workload == "reddit" and args.emulate_world <= 1 and
            not args.no_model_legs and not on_cpu and not args.dist_rehearsal):
        import bench_models as bm
        want = not args.no_cpu_baseline
        only = set(args.model_legs.split(",")) if args.model_legs else None
        if only is not None:
            legs_run = legs.run

            def run_selected(name, *a, **k):
                return legs_run(name, *a, **k) if name in only else None
            legs.run = run_selected
        legs.run("gcn_reddit", lambda: None, lambda _: bm.gcn_reddit_leg(
            g, dev, kernel, gather_peak, algorithmic_bytes, sample, cpu=want),
            collective=False)
        _release(dev)
        legs.run("gat", lambda: None, lambda _: bm.gat_layer_leg(
            g, dev, kernel, gather_peak, sample, cpu=want), collective=False)
        legs.run("sage", lambda: None, lambda _: bm.sage_leg(
            g, dev, kernel, gather_peak, algorithmic_bytes, sample, cpu=want),
            collective=False)
        _release(dev)
        legs.run("gat_pubmed", lambda: None, lambda _: bm.gat_pubmed_leg(
            dev, kernel, gather_peak, cpu=want), collective=False)
        legs.run("rgcn", lambda: None, lambda _: bm.rgcn_leg(
            dev, kernel, gather_peak, cpu=want), collective=False)
    sample = h_cpu = None
    if not args.no_rmat_leg and args.workload == "reddit" and args.emulate_world <= 1:
        # release the headline leg before the 1.07B-edge graph
        step = g = h = adj = pg = h_local = None  # noqa: F841
        _release(dev)
        legs.run("rmat%d" % args.rmat_scale, lambda: rmat_setup(args, rank, dev),
                 lambda st: rmat_run(args, world, rank, dev, st, rmat_pmc))
        if _RMAT_KEEP:
            # configs[3] at its own size: GraphSAGE-mean epochs on the same graph
            st = dict(_RMAT_KEEP)
            _RMAT_KEEP.clear()
            import bench_models as bm
            legs.run("sage_rmat%d" % args.rmat_scale, lambda: st, lambda s_: bm.sage_rmat_leg(
                s_, dev, kernel, gather_peak, algorithmic_bytes,
                cpu=not args.no_cpu_baseline), collective=False)
            st = None
            _release(dev)
    if rank == 0:
        emit_line(result)
    if distributed:
        if legs.failed is not None:
            # a collective may be half-done: leave without the group's
            # teardown, with a failing exit code (the line, printed above,
            # carries the leg's error)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(EXIT_LEG_FAILED)
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _release(dev):
    import gc
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
