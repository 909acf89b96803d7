# Quick check: GPU tests, the default bench line twice (no PMC, no CPU
# baseline), then optional PMC counter sets (one rocprofv3 pass each).
#   bash tools/gpu/run_quick.sh "<bench args>" ["COUNTERS ..."] ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $ARGS > gpurun_out/quick_$i.json 2> gpurun_out/quick_$i.err || { tail -20 gpurun_out/quick_$i.err; exit 1; }
  python - "$i" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/quick_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"].get("stage_ms",{})
print(f"{d['config']['config_name']:>10} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f}  {st}")
PY
done
i=0
for set in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/qpmc/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-pmc $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/qpmc_$i.log" 2>&1) \
    || { echo "pmc pass $i ($set) failed"; tail -20 gpurun_out/qpmc_$i.log; exit 1; }
  python - gpurun_out/qpmc/p$i <<'PY'
import csv,collections,glob,sys
f=glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True)[0]
acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].split('(')[0].split('::')[-1]
    acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
    n[(k,r['Counter_Name'])]+=1
for k,d in acc.items():
    print(k, {c:f"{v/n[(k,c)]:.4g}/disp" for c,v in d.items()})
PY
done
