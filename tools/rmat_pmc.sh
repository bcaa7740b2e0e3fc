cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d gpurun_out/rmatpmc_$c -o run --output-format csv \
    -- python bench.py --workload rmat --rmat-scale 26 --steps 2 --warmup 1 --no-traffic --no-rmat-leg --no-cpu-baseline > gpurun_out/rmatpmc_$c.log 2>&1
  rc=$?; tail -1 gpurun_out/rmatpmc_$c.log; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import csv, glob, collections, json
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob("gpurun_out/rmatpmc_%s/**/*counter_collection.csv" % c, recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gspmm" in r["Kernel_Name"] and r["Counter_Name"] == c:
            agg[r["Kernel_Name"][:90]].append(float(r["Counter_Value"]))
    res[c] = {k: (len(v), sum(v) / len(v)) for k, v in agg.items()}
print(json.dumps(res, indent=1))
PY
