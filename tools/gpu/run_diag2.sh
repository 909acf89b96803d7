set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu/score_diag.py > gpurun_out/diag2.log 2>&1 || { tail -30 gpurun_out/diag2.log; exit 1; }
cat gpurun_out/diag2.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
