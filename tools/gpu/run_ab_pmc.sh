# A/B of libvtseg variants, then the default bench (with its PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
PASSES=${PASSES:-2} bash tools/gpu/run_variants.sh "$1" ${@:2} || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_pmc.json 2> gpurun_out/bench_pmc.err || { tail -30 gpurun_out/bench_pmc.err; exit 1; }
cat gpurun_out/bench_pmc.json
