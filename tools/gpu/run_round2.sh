# Round check + every BASELINE config (one MI355X): GPU tests, default bench
# line, rocprofv3 kernel trace/stats of the same bench, 720p-2h streamed,
# 1080p 30-min sample, 480p-60s.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
cat gpurun_out/prof.json
find gpurun_out/prof -name '*kernel_stats.csv' -exec head -4 {} \;
timeout -k 10 400 python bench.py --config 720p-2h --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/b2h.json 2> gpurun_out/b2h.err || { tail -20 gpurun_out/b2h.err; exit 1; }
cat gpurun_out/b2h.json
timeout -k 10 400 python bench.py --config 1080p-2h --frames 54000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b1080.json 2> gpurun_out/b1080.err || { tail -20 gpurun_out/b1080.err; exit 1; }
cat gpurun_out/b1080.json
timeout -k 10 300 python bench.py --config 480p-60s --no-cpu-baseline > gpurun_out/b480.json 2> gpurun_out/b480.err || { tail -20 gpurun_out/b480.err; exit 1; }
cat gpurun_out/b480.json
