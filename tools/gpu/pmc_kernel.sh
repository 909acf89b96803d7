# PMC passes (one counter set per rocprofv3 run) over an arbitrary python
# command; per-kernel averages per dispatch.
#   bash tools/gpu/pmc_kernel.sh "<python args>" "SET1" "SET2" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
i=0
for set in "$@"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kpmc/p$i" -o run -- python3 $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/kpmc_$i.log" 2>&1) \
    || { echo "pmc pass $i ($set) failed"; tail -20 gpurun_out/kpmc_$i.log; exit 1; }
  python - gpurun_out/kpmc/p$i <<'PY'
import csv,collections,glob,sys
f=glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True)[0]
acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'].replace('(anonymous namespace)::','').split('(')[0]
    acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
    n[(k,r['Counter_Name'])]+=1
for k,d in acc.items():
    if 'rocclr' in k: continue
    print(k, {c:f"{v/n[(k,c)]:.4g}" for c,v in d.items()})
PY
done
