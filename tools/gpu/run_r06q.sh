#!/bin/bash
# round 6 (q): one context state per dword (six lane tables) against the
# packed tables: all-intra, content and noise streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > $O/parse_hot.log 2>&1 || { tail -5 $O/parse_hot.log; exit 1; }
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/allintra.mp4 3 $O/allintra packed cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content packed cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/n0.mp4 2 $O/noise packed cur || exit $?
