# 1080p (k = 6) bench line with live PMC traffic, and the rocprofv3 kernel stats of the same config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config 1080p-2h --frames 54000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b1080.json 2> gpurun_out/b1080.err || { tail -20 gpurun_out/b1080.err; exit 1; }
cat gpurun_out/b1080.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof1080" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 1080p-2h --frames 54000 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof1080.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof1080.err" \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof1080.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
head -4 gpurun_out/prof1080/run_kernel_stats.csv
