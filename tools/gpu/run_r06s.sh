#!/bin/bash
# round 6 (s): GPU suite, then the default bench line with its profiler passes
# kept (kernel-trace stats and PMC summaries of the same bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err
rc=$?
tail -14 $O/bench.err
find $O/prof -name "*kernel_stats.csv" | head -5
exit $rc
