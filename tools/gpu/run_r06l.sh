#!/bin/bash
# round 6 (l): section timing of the CABAC parse (experiment library) on the
# all-intra and 10-min content streams; then the default bench line on the
# capped stream policy
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > /dev/null 2>&1 || exit $?
timeout -k 10 120 python -u tools/gpu/parse_trace.py tools/exp/lib_trace.so /tmp/allintra.mp4 > $O/trace_allintra.json 2> $O/trace_allintra.err || { tail -5 $O/trace_allintra.err; exit 1; }
head -60 $O/trace_allintra.json
timeout -k 10 800 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
