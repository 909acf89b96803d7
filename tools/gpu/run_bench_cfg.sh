# One bench line (with its PMC traffic passes) per argument set, plus the
# rocprofv3 kernel stats of the same command.  bash tools/gpu/run_bench_cfg.sh TAG "<args>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; ARGS=$2
timeout -k 10 600 python bench.py --no-cpu-baseline $ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-pmc --steps 5 --warmup 1 $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit 1; }
cat "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/run_kernel_stats.csv"
