#!/bin/bash
# round 6 (p): the default bench line on the current tree (content batch +
# mixed batch record), then the rocprofv3 kernel-trace summary of the same
# bench at a reduced step count
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -14 $O/bench.err
exit $rc
