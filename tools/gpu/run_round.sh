# Round check: GPU tests, default bench line (with CPU baseline), rocprofv3
# kernel stats of the same bench, then a 2-rank torchrun rehearsal (both ranks
# on the one GPU of the box, gloo for the count exchange).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err" \
  || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.err"; exit 1; }
cat "$GRAFT_REPO_ROOT/gpurun_out/prof.json"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name '*kernel_stats.csv' -exec cat {} \;
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --dist-backend gloo > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { tail -20 gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
