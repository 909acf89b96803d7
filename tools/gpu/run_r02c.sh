# General decoder: GPU parity tests + a bench line on a full-syntax 10-min 720p
# stream (intra/residual/quarter-pel/3 refs/deblocking) with rocprofv3 passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -2 gpurun_out/pytest_full.log
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --profile-dir gpurun_out/r02_full_prof > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
