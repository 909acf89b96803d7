#!/bin/bash
# round 6 (k): CABAC residual decisions on a fixed lane table (+ rare bit-reader
# paths off the common path): same-box A/B against the base library on the
# 10-min 720p content stream and an 80-frame all-intra content stream; the
# engine micro-benchmark with unrolled decisions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 120 ./tools/micro/cabac_engine 200000 > $O/cabac_engine.jsonl 2>&1 || exit $?
cat $O/cabac_engine.jsonl
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > /dev/null 2>&1 || exit $?
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/allintra.mp4 3 $O/allintra base cur || exit $?
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content base cur || exit $?
