#!/bin/bash
# round 6 (c): CABAC bin micro-benchmark; stream concurrency on 4 / 16 HW queues
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06c
timeout -k 10 120 ./tools/micro/cabac_bins 200000 > gpurun_out/r06c/cabac_bins.jsonl 2>&1 || exit $?
cat gpurun_out/r06c/cabac_bins.jsonl
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 60 ./tools/micro/qprobe 8 20 >> gpurun_out/r06c/qprobe.jsonl 2>&1 || exit $?
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 60 ./tools/micro/qprobe 24 20 >> gpurun_out/r06c/qprobe.jsonl 2>&1 || exit $?
cat gpurun_out/r06c/qprobe.jsonl
