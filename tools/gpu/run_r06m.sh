#!/bin/bash
# round 6 (m): section timing of the CABAC parse (experiment library); A/B of
# the parse changes (base = round start, slot = fixed-table decisions, cur =
# + one-trip significance map and level prefix); then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > /dev/null 2>&1 || exit $?
timeout -k 10 120 python -u tools/gpu/parse_trace.py tools/exp/lib_trace.so /tmp/allintra.mp4 > $O/trace_allintra.json 2> $O/trace_allintra.err
rc=$?; tail -3 $O/trace_allintra.err; head -70 $O/trace_allintra.json
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/allintra.mp4 3 $O/allintra base slot cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content base cur || exit $?
timeout -k 10 800 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -12 $O/bench.err
exit $rc
