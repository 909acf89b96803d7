# General-decoder GPU tests on the new tree, then a same-box A/B of the
# full-syntax bench (new vs tools/exp/old), I/P and B streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -30 gpurun_out/pytest_full.log; exit 1; }
tail -1 gpurun_out/pytest_full.log
for pass in 1 2; do
  for v in new old; do
    for b in "" "--bframes"; do
      if [ $v = new ]; then B=bench.py; else B=tools/exp/old/bench.py; fi
      timeout -k 10 600 python $B --config 720p-10min --coding full $b --steps 2 --warmup 1 --no-pmc --no-parity --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python - "$v $b" <<'PY'
import json,sys
d=json.load(open("gpurun_out/ab.json")); st=d["config"]["stage_ms"]
print(f"{sys.argv[1]:>14} {d['value']:>9.0f} fps {d['ms_per_step']:8.1f} ms parse {st['parse_ms']:7.1f} recon {st['reconstruct_ms']:7.1f}")
PY
    done
  done
done
