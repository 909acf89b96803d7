set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu/score_diag.py > gpurun_out/diag.log 2>&1 || { tail -30 gpurun_out/diag.log; exit 1; }
timeout -k 10 300 python bench.py --workload score --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_score.log 2>&1 || { tail -30 gpurun_out/bench_score.log; exit 1; }
cat gpurun_out/bench_score.log
