# A/B of VTS_GENERAL_GROUPS on the full-syntax benches (GPU tests first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
B="--config 720p-10min --coding full --steps 3 --warmup 1 --no-pmc --no-parity --no-cpu-baseline"
for pass in 1 2; do
  for g in 1 2 3 4; do
    for b in "" "--bframes"; do
      VTS_GENERAL_GROUPS=$g timeout -k 10 240 python bench.py $B $b > gpurun_out/gg.json 2> gpurun_out/gg.err || { tail -20 gpurun_out/gg.err; exit 1; }
      python - "$g" "$b" <<'PY'
import json,sys
d=json.load(open("gpurun_out/gg.json")); st=d["config"]["stage_ms"]
print(f"groups {sys.argv[1]} {sys.argv[2]:>9} {d['value']:>9.0f} fps {d['ms_per_step']:8.2f} ms parse {st['parse_ms']:.1f} recon {st['reconstruct_ms']:.1f}")
PY
    done
  done
done
