# General decoder: parity tests, then a bench line + rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_full_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -60 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 600 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
