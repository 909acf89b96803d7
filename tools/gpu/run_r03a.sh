# Round 3, first GPU check: GPU tests (incl. the ADVICE fixes), smoke, the new
# default bench line (720p-batch via plan_batch + extras) with its profiles,
# and the 2-rank gloo rehearsal of the batch config on one GPU (full parity).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03a
O=gpurun_out/r03a
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
t0=$SECONDS
timeout -k 10 720 python bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall s: $((SECONDS - t0))" | tee $O/bench.time
cut -c1-600 $O/bench.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --parity-frames all > $O/rehearsal_batch_2rank.json 2> $O/rehearsal_batch_2rank.err || { tail -20 $O/rehearsal_batch_2rank.err; exit 1; }
cut -c1-400 $O/rehearsal_batch_2rank.json
