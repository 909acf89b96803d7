#!/bin/bash
# round 6 (g): native batch GPU tests; single-wave issue latencies; 4 content
# sessions through plan_batch on 4 / 16 hardware queues, plain vs CU-masked streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batch_native.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest_batch_native.log 2>&1
rc=$?; tail -4 $O/pytest_batch_native.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/micro/issue_lat > $O/issue_lat.jsonl 2>&1 || exit $?
cat $O/issue_lat.jsonl
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 /tmp/c1.mp4 /tmp/c2.mp4 /tmp/c3.mp4 || exit $?
for q in 4 16; do
  for sq in plain own; do
    GPU_MAX_HW_QUEUES=$q VTS_STREAM_QUEUES=$sq timeout -k 10 120 python -u tools/gpu/batch_probe.py \
      /tmp/c0.mp4 /tmp/c1.mp4 /tmp/c2.mp4 /tmp/c3.mp4 > $O/batch_q${q}_${sq}.json 2> $O/batch_q${q}_${sq}.err || { tail -5 $O/batch_q${q}_${sq}.err; exit 1; }
    echo "q=$q streams=$sq $(cat $O/batch_q${q}_${sq}.json)"
  done
done
