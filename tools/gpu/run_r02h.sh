# Full-syntax bench after the parser scratch fix (non-B, then B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_full_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -30 gpurun_out/pytest_full.log; exit 1; }
tail -2 gpurun_out/pytest_full.log
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --no-pmc --no-parity --no-cpu-baseline > gpurun_out/bench_full3.json 2> gpurun_out/bench_full3.err || { tail -30 gpurun_out/bench_full3.err; exit 1; }
cat gpurun_out/bench_full3.json
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --bframes --steps 3 --warmup 1 --no-pmc --no-parity --no-cpu-baseline > gpurun_out/bench_fullb3.json 2> gpurun_out/bench_fullb3.err || { tail -30 gpurun_out/bench_fullb3.err; exit 1; }
cat gpurun_out/bench_fullb3.json
