#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that faults / aborts / times out (exit >= 2 or 124/134/137/139).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc ;;
    seltests)
      # a chosen subset, verbose, each test bounded: SEL="tests/x.py tests/y.py::z" [KEXPR=...]
      timeout -k 10 1100 python -u -m pytest $SEL -m gpu -x -v -s --timeout ${TEST_TIMEOUT:-300} \
        --timeout-method thread -p no:cacheprovider ${KEXPR:+-k "$KEXPR"} > gpurun_out/pytest_sel.log 2>&1
      rc=$?; tail -5 gpurun_out/pytest_sel.log; ok $rc || exit $rc ;;
    sage)
      # GraphSAGE-mean full-graph epochs on RMAT-$RMAT_SCALE, one GPU, heavy-row policy both ways
      for rs in ${ROW_SPLITS:-off auto}; do
        timeout -k 10 600 python -u examples/graphsage/train.py --graph rmat --rmat-scale ${RMAT_SCALE:-26} \
          --gpu 0 --n-epochs ${EPOCHS:-5} --row-split $rs > gpurun_out/sage_rmat_$rs.log 2>&1
        rc=$?; tail -2 gpurun_out/sage_rmat_$rs.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    sagedist)
      # GraphSAGE-mean --dist on a world-1 RCCL group (pipelined halo fwd + bwd), RMAT-$RMAT_SCALE
      for pc in ${PIPE_CHUNKS:-0 4}; do
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 29613 examples/graphsage/train.py --dist \
          --graph rmat --rmat-scale ${RMAT_SCALE:-24} --gpu 0 --n-epochs ${EPOCHS:-5} \
          --pipeline-chunks $pc > gpurun_out/sagedist_$pc.log 2>&1
        rc=$?; tail -2 gpurun_out/sagedist_$pc.log; [ $rc -eq 0 ] || exit $rc
      done ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    benchquick)
      # the default line's legs without the PMC passes and the RMAT leg
      timeout -k 10 600 python bench.py --no-traffic --no-rmat-leg ${BENCH_ARGS:-} > gpurun_out/benchquick.json 2> gpurun_out/benchquick.err
      rc=$?; tail -12 gpurun_out/benchquick.err; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      # the bench line and the kernel statistics of the SAME process (headline leg only)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run \
        --output-format csv -- python bench.py --no-traffic --no-rmat-leg --no-train-leg --no-cpu-baseline --no-model-legs \
        > gpurun_out/prof.json 2> gpurun_out/prof.log
      rc=$?; tail -1 gpurun_out/prof.log; cat gpurun_out/prof.json; [ $rc -eq 0 ] || exit $rc
      # the same trace over the timed steps alone (bench.py's spin-kernel markers)
      python tools/window_stats.py gpurun_out/prof/run_kernel_trace.csv --window 0 \
        --out gpurun_out/prof/timed_kernel_stats.csv || exit $? ;;
    dist)
      # rehearse the multi-rank bench path: 2 ranks sharing the one GPU over gloo
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 1 --rmat-scale 18 \
        --graph-scale 0.05 --dist-backend gloo > gpurun_out/dist.json 2> gpurun_out/dist.err
      rc=$?; tail -3 gpurun_out/dist.err; cat gpurun_out/dist.json; [ $rc -eq 0 ] || exit $rc ;;
    rehearsal)
      # the N>1 bench path (RCCL group, partition, collectives, max-over-ranks timing) on one rank
      timeout -k 10 600 python bench.py --dist-rehearsal --no-traffic --steps 5 --warmup 2 \
        > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err
      rc=$?; tail -4 gpurun_out/rehearsal.err; cat gpurun_out/rehearsal.json; [ $rc -eq 0 ] || exit $rc ;;
    examples)
      ( timeout -k 10 600 python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 --n-hidden 128 --n-epochs 20 &&
        timeout -k 10 300 python examples/gcn/gcn_spmv.py --dataset cora --gpu 0 --n-epochs 50 &&
        timeout -k 10 300 python examples/gcn/gcn_spmv.py --dataset cora --gpu 0 --n-epochs 50 --hip-graph &&
        timeout -k 10 300 python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 --n-hidden 128 --n-epochs 20 --hip-graph &&
        timeout -k 10 300 python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 30 &&
        timeout -k 10 300 python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 30 --udf &&
        timeout -k 10 300 python examples/gat/train.py --dataset pubmed --gpu 0 --epochs 30 --hip-graph &&
        timeout -k 10 300 python examples/graphsage/train.py --dataset reddit --gpu 0 --n-epochs 10 &&
        timeout -k 10 300 python examples/rgcn/link_predict.py --gpu 0 --n-epochs 20 &&
        timeout -k 10 300 python examples/rgcn/link_predict.py --gpu 0 --n-epochs 20 --udf ) \
        > gpurun_out/examples.log 2>&1
      rc=$?; tail -4 gpurun_out/examples.log; [ $rc -eq 0 ] || exit $rc ;;
    emul)
      wl=${WORKLOAD:-reddit}
      for w in ${EMUL_WORLDS:-2 8}; do for c in ${CHUNKS:-0 4}; do
        tag=${wl}_${w}_$c${HALO_DTYPE:+_$HALO_DTYPE}${STRONG:+_strong}
        timeout -k 10 600 python bench.py --workload $wl --emulate-world $w --pipeline-chunks $c \
          --steps 10 --warmup 3 --no-traffic ${HALO_DTYPE:+--halo-dtype $HALO_DTYPE} \
          ${STRONG:+--emulate-strong} \
          > gpurun_out/emul_$tag.json 2> gpurun_out/emul_$tag.err
        rc=$?; tail -1 gpurun_out/emul_$tag.err; [ $rc -eq 0 ] || exit $rc
        python -c "import json; d=json.load(open('gpurun_out/emul_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
      done; done ;;
    rgcn)
      # configs[4] step phase by phase + each typed-block kernel alone (fused; then the UDF formulation)
      timeout -k 10 300 python -u tools/rgcn_step.py --kernels --out gpurun_out/rgcn_step.json > gpurun_out/rgcn.log 2>&1 &&
      timeout -k 10 300 python -u tools/rgcn_step.py --udf --steps 5 --out gpurun_out/rgcn_step_udf.json >> gpurun_out/rgcn.log 2>&1
      rc=$?; tail -2 gpurun_out/rgcn.log; [ $rc -eq 0 ] || exit $rc ;;
    rgcnprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rgcnprof -o run \
        --output-format csv -- python tools/rgcn_step.py --steps 20 > gpurun_out/rgcnprof.log 2>&1
      rc=$?; tail -2 gpurun_out/rgcnprof.log; [ $rc -eq 0 ] || exit $rc ;;
    l2split)
      # the headline's L2 hits / misses and EA requests per block launch (tools/l2_split.py)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/l2a -o run \
        --output-format csv -- python tools/l2_split.py run --out gpurun_out/l2_plan.json > gpurun_out/l2a.log 2>&1 &&
      timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/l2b -o run \
        --output-format csv -- python tools/l2_split.py run --out gpurun_out/l2_plan.json > gpurun_out/l2b.log 2>&1 &&
      python tools/l2_split.py parse gpurun_out/l2_plan.json gpurun_out/l2a/run_counter_collection.csv \
        --out gpurun_out/l2_split_hits.json > /dev/null &&
      python tools/l2_split.py parse gpurun_out/l2_plan.json gpurun_out/l2b/run_counter_collection.csv \
        --out gpurun_out/l2_split_ea.json > /dev/null
      rc=$?; tail -2 gpurun_out/l2b.log; [ $rc -eq 0 ] || exit $rc ;;
    gatprof)
      # GAT 8 x 16 forward + backward on the Reddit-shaped graph: kernel statistics
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gatprof -o run \
        --output-format csv -- python tools/gat_bench.py --fwd-bwd-only --iters 10 > gpurun_out/gatprof.log 2>&1
      rc=$?; tail -2 gpurun_out/gatprof.log; [ $rc -eq 0 ] || exit $rc ;;
    sageprof)
      # kernel statistics of GraphSAGE-mean full-graph epochs on RMAT-$RMAT_SCALE (configs[3])
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/sageprof -o run \
        --output-format csv -- python examples/graphsage/train.py --graph rmat \
        --rmat-scale ${RMAT_SCALE:-26} --gpu 0 --n-epochs ${EPOCHS:-4} > gpurun_out/sageprof.log 2>&1
      rc=$?; tail -2 gpurun_out/sageprof.log; [ $rc -eq 0 ] || exit $rc ;;
    gcnprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gcnprof -o run \
        --output-format csv -- python examples/gcn/gcn_spmv.py --dataset reddit --gpu 0 \
        --n-hidden 128 --n-epochs 8 > gpurun_out/gcnprof.log 2>&1
      rc=$?; tail -2 gpurun_out/gcnprof.log; [ $rc -eq 0 ] || exit $rc ;;
    sweep)
      timeout -k 10 600 python tools/kernel_sweep.py > gpurun_out/sweep_reddit.json 2> gpurun_out/sweep.err &&
      timeout -k 10 600 python tools/kernel_sweep.py --workload rmat --rmat-scale 25 > gpurun_out/sweep_rmat.json 2>> gpurun_out/sweep.err
      rc=$?; cat gpurun_out/sweep_reddit.json gpurun_out/sweep_rmat.json; [ $rc -eq 0 ] || exit $rc ;;
    featsweep)
      timeout -k 10 600 python tools/feat_sweep.py ${FEATS:+--feats $FEATS} > gpurun_out/feat_sweep.json 2> gpurun_out/feat_sweep.err
      rc=$?; tail -12 gpurun_out/feat_sweep.err; [ $rc -eq 0 ] || exit $rc ;;
    disttest)
      timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 240 \
        --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
      rc=$?; tail -3 gpurun_out/pytest_dist.log; ok $rc || exit $rc ;;
    relabel)
      timeout -k 10 300 python tools/relabel_study.py > gpurun_out/relabel_reddit.json 2> gpurun_out/relabel.err &&
      timeout -k 10 600 python tools/relabel_study.py --workload rmat --rmat-scale ${RMAT_SCALE:-26} \
        --feats ${RMAT_FEATS:-128} > gpurun_out/relabel_rmat.json 2>> gpurun_out/relabel.err
      rc=$?; cat gpurun_out/relabel.err | tail -8; [ $rc -eq 0 ] || exit $rc ;;
    reducers)
      timeout -k 10 600 python tools/reducer_bench.py > gpurun_out/reducers.json 2> gpurun_out/reducers.err
      rc=$?; cat gpurun_out/reducers.json; tail -3 gpurun_out/reducers.err; [ $rc -eq 0 ] || exit $rc ;;
    rmat)
      timeout -k 10 900 python bench.py --workload rmat --rmat-scale ${RMAT_SCALE:-26} --steps 5 \
        --warmup 2 > gpurun_out/rmat.json 2> gpurun_out/rmat.err
      rc=$?; tail -4 gpurun_out/rmat.err; cat gpurun_out/rmat.json; [ $rc -eq 0 ] || exit $rc ;;
    legprof)
      # one model leg under the kernel trace (LEG=gcn_reddit): its timed epochs' kernels alone
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/legprof -o run \
        --output-format csv -- python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg \
        --no-train-leg --no-one-launch-leg --no-cpu-baseline --model-legs ${LEG:-gcn_reddit} \
        > gpurun_out/legprof.json 2> gpurun_out/legprof.log
      rc=$?; tail -1 gpurun_out/legprof.log; [ $rc -eq 0 ] || exit $rc
      python tools/window_stats.py gpurun_out/legprof/run_kernel_trace.csv --window 1 \
        --out gpurun_out/legprof/leg_timed_kernel_stats.csv || exit $? ;;
    rgcnlegs)
      # the R-GCN leg alone, REPEAT times (process-to-process spread), then its host study
      for i in $(seq ${REPEAT:-3}); do
        timeout -k 10 300 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-train-leg \
          --no-one-launch-leg --no-cpu-baseline --model-legs rgcn > gpurun_out/rgcn_leg_$i.json 2> gpurun_out/rgcn_leg_$i.err
        rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/rgcn_leg_$i.err; exit $rc; }
        python -c "import json; d=json.load(open('gpurun_out/rgcn_leg_$i.json'))['rgcn']; print('rgcn', d['ms_per_step'], d['kernel_ms'], d['launches_per_step'])"
      done
      timeout -k 10 400 python -u tools/rgcn_host_study.py --blas rocblas --out gpurun_out/rgcn_host.json > gpurun_out/rgcn_host.log 2>&1
      rc=$?; tail -1 gpurun_out/rgcn_host.log; [ $rc -eq 0 ] || exit $rc ;;
    gatsplit)
      # the GAT backward's L2 hits / misses and EA requests over the timed calls (tools/gat_bwd_split.py)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/gsa -o run \
        --output-format csv -- python tools/gat_bwd_split.py run --out gpurun_out/gat_plan.json > gpurun_out/gsa.log 2>&1 &&
      timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/gsb -o run \
        --output-format csv -- python tools/gat_bwd_split.py run --out gpurun_out/gat_plan.json > gpurun_out/gsb.log 2>&1 &&
      python tools/gat_bwd_split.py parse gpurun_out/gat_plan.json gpurun_out/gsa/run_counter_collection.csv \
        gpurun_out/gsb/run_counter_collection.csv --out gpurun_out/gat_bwd_l2_split.json > /dev/null
      rc=$?; tail -2 gpurun_out/gsb.log; [ $rc -eq 0 ] || exit $rc ;;
    gatvariants)
      # GAT 8 x 16 fwd + bwd per backward variant (VARIANTS="0 3"), interleaved rounds
      timeout -k 10 400 python -u tools/gat_bwd_variants.py --variants ${VARIANTS:-0} --rounds ${ROUNDS:-3} \
        --out gpurun_out/gat_bwd_variants.json > gpurun_out/gat_bwd_variants.log 2>&1
      rc=$?; tail -3 gpurun_out/gat_bwd_variants.log; [ $rc -eq 0 ] || exit $rc ;;
    benchlegs)
      # the N = 1 line without the PMC passes, the RMAT legs and the CPU baselines (model legs timed)
      timeout -k 10 600 python bench.py --no-traffic --no-rmat-leg --no-sage-rmat-leg --no-cpu-baseline \
        ${BENCH_ARGS:-} > gpurun_out/benchlegs.json 2> gpurun_out/benchlegs.err
      rc=$?; tail -3 gpurun_out/benchlegs.err; [ $rc -eq 0 ] || exit $rc
      python tools/bench_summary.py gpurun_out/benchlegs.json ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv \
          -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-rmat-leg --no-train-leg --no-model-legs > gpurun_out/pmc_$c.log 2>&1
        rc=$?; tail -2 gpurun_out/pmc_$c.log; [ $rc -eq 0 ] || exit $rc
      done ;;
  esac
done
echo "gpu_check done"
