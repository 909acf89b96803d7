#!/bin/bash
# round 6 (e): CABAC engine variants on one lone wave
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06e
timeout -k 10 120 ./tools/micro/cabac_engine 200000 > gpurun_out/r06e/cabac_engine.jsonl 2>&1
rc=$?
cat gpurun_out/r06e/cabac_engine.jsonl
exit $rc
