#!/bin/bash
# round 6 (aq): the final tree's default bench line with its profiler passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aq
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
