# Round 2 check: GPU tests, then the default bench line (720p-2h, parity,
# rocprofv3 trace/PMC passes kept under gpurun_out/r02_prof).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 900 python -u bench.py --profile-dir gpurun_out/r02_prof > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cat gpurun_out/r02_prof/kernel_busy.txt | head -8
