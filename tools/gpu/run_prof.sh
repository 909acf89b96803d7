# GPU tests, then rocprofv3 kernel-trace/stats of the decode+score bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures: still profile
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name '*kernel_stats.csv' -exec cat {} \;
