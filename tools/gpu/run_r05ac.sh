# Round 5: two-rank rehearsal of the N>1 bench path on one MI355X (gloo; the
# driver's N>1 runs use RCCL on separate GPUs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --extras none --no-pmc --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench2.json')); print(json.dumps({k: d.get(k) for k in ('value','n_gpus','placement','ms_per_step','parity')})[:800])"
