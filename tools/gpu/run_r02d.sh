# Round-2 check of HEAD: every GPU parity test (incl. the CABAC/High-profile
# real clip on the device), smoke, and the general-decoder bench line with
# its rocprofv3 kernel trace kept.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -30 gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --profile-dir gpurun_out/r02_full_prof > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
