#!/bin/bash
# round 6 (ag): the default bench line with its profiler passes on the tree
# with the split CABAC parse and the exact intra levels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ag
mkdir -p $O
timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err
rc=$?
tail -14 $O/bench.err
exit $rc
