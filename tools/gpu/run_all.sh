# Round GPU session: tests, bench (decode+score and score-only), rocprof.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
step bench_decode_score
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step bench_score
timeout -k 10 300 python bench.py --workload score --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_score.json 2> gpurun_out/bench_score.err \
  || { tail -30 gpurun_out/bench_score.err; exit 1; }
cat gpurun_out/bench_score.json
step rocprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name '*stats*' | head
echo done
