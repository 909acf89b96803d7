# A/B of environment settings on the in-tree library (GPU tests first):
#   bash tools/gpu/run_env_ab.sh "<bench args>" "VAR=a" "VAR=b" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARGS=$1; shift
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for pass in $(seq ${PASSES:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc $ARGS > gpurun_out/env_$i.json 2> gpurun_out/env_$i.err || { tail -20 gpurun_out/env_$i.err; exit 1; }
    python - "$i" "$e" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/env_{sys.argv[1]}.json"))
r=d["roofline"]; st=d["config"]["stage_ms"]
print(f"{sys.argv[2]:>22} {d['value']:>11.0f} fps {d['ms_per_step']:7.3f} ms  kernel {r['kernel_ms']:.4f} ms/launch  launches {d['config']['recon_launches']}  parse {st['parse_ms']:.3f} recon {st['reconstruct_ms']:.3f}")
PY
  done
done
