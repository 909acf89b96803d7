# Round-2 check of HEAD: every GPU parity test, smoke, the default bench line
# (720p-2h, parity + roofline + PMC + CPU baseline), its rocprofv3 kernel
# stats, and the full 216 000-frame 1080p-2h config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/pytest_gpu.log | tail -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { tail -30 gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
timeout -k 10 900 python -u bench.py --profile-dir gpurun_out/r02_final_prof > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-parity > "$GRAFT_REPO_ROOT/gpurun_out/prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof -name '*kernel_stats.csv' -exec head -6 {} \;
timeout -k 10 900 python -u bench.py --config 1080p-2h --steps 3 --warmup 1 --no-pmc > gpurun_out/b1080.json 2> gpurun_out/b1080.err || { tail -20 gpurun_out/b1080.err; exit 1; }
cat gpurun_out/b1080.json
