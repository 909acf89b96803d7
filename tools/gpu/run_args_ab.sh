# A/B of bench.py argument sets on the in-tree library (GPU tests first):
#   bash tools/gpu/run_args_ab.sh "<args 1>" "<args 2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for pass in $(seq ${PASSES:-2}); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $a > gpurun_out/args_$i.json 2> gpurun_out/args_$i.err || { tail -20 gpurun_out/args_$i.err; exit 1; }
    python - "$i" "$a" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/args_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"]["stage_ms"]
print(f"{sys.argv[2]:>28} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  kernel {r['kernel_ms']:.4f} ms frac {r['frac']:.4f}  parse {st['parse_ms']:.3f} recon {st['reconstruct_ms']:.3f} score {st['score_ms']:.3f} total {st['total_ms']:.3f}")
PY
  done
done
