#!/bin/bash
# round 6 (r): dword context tables fail on the device (all-intra stream):
# engine micro-benchmark (device engines agree?) and the CABAC GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 120 ./tools/micro/cabac_engine 20000 > $O/cabac_engine.jsonl 2>&1; cat $O/cabac_engine.jsonl
timeout -k 10 400 python -u -m pytest tests/test_full_gpu.py -x -q -k "cabac" --timeout 200 --timeout-method thread > $O/pytest_cabac.log 2>&1
tail -30 $O/pytest_cabac.log
