# Transcode tests on general-decoder inputs + a 2-rank gloo rehearsal of the
# multi-GPU bench path on the one GPU (10-min 720p per rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_transcode_gpu.py -v --timeout 240 --timeout-method thread -k general > gpurun_out/pytest_tc.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_tc.log | tail -30; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_tc.log
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -v --timeout 240 --timeout-method thread -k fhd_crop > gpurun_out/pytest_fhd.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_fhd.log | tail -30; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_fhd.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 720p-10min --steps 3 --warmup 1 --dist-backend gloo --no-pmc > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err || { tail -30 gpurun_out/bench_2rank.err; exit 1; }
cat gpurun_out/bench_2rank.json
