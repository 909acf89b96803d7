#!/bin/bash
# round 6 (i): single-wave issue latencies (SCC declared clobbered); 4 content
# sessions through plan_batch on 4 hardware queues with each stream-set policy
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06i
mkdir -p $O
for t in 0 1 2 3 4 5 6 7 8 9 10 12 13 14 11; do
  timeout -k 5 20 ./tools/micro/issue_lat $t >> $O/issue_lat.jsonl 2>&1 || { echo "test $t rc=$?"; break; }
done
cat $O/issue_lat.jsonl
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 /tmp/c1.mp4 /tmp/c2.mp4 /tmp/c3.mp4 || exit $?
for sq in plain auto prio own; do
  GPU_MAX_HW_QUEUES=4 VTS_STREAM_QUEUES=$sq timeout -k 10 120 python -u tools/gpu/batch_probe.py \
    /tmp/c0.mp4 /tmp/c1.mp4 /tmp/c2.mp4 /tmp/c3.mp4 > $O/batch_q4_${sq}.json 2> $O/batch_q4_${sq}.err || { tail -5 $O/batch_q4_${sq}.err; exit 1; }
  echo "q=4 streams=$sq $(cat $O/batch_q4_${sq}.json)"
done
