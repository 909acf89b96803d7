# Full-syntax benches on the general decoder: 10-min 720p with B pictures
# (x264-like) and without, each with oracle parity and its rocprofv3 trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --bframes --steps 3 --warmup 1 --profile-dir gpurun_out/r02_fullb_prof > gpurun_out/bench_fullb.json 2> gpurun_out/bench_fullb.err || { tail -30 gpurun_out/bench_fullb.err; exit 1; }
cat gpurun_out/bench_fullb.json
timeout -k 10 900 python -u bench.py --config 720p-10min --coding full --steps 3 --warmup 1 --profile-dir gpurun_out/r02_full2_prof > gpurun_out/bench_full2.json 2> gpurun_out/bench_full2.err || { tail -30 gpurun_out/bench_full2.err; exit 1; }
cat gpurun_out/bench_full2.json
