# Round-2 late check: smoke, the default bench line (720p-2h with parity,
# cpu_baseline, PMC passes), and the full 216 000-frame 1080p-2h config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 500 python bench.py --config 1080p-2h --steps 3 --warmup 1 --no-pmc > gpurun_out/b1080.json 2> gpurun_out/b1080.err || { tail -20 gpurun_out/b1080.err; exit 1; }
cat gpurun_out/b1080.json
