#!/bin/bash
# round 6 (o): CABAC decision bit from the compare's lane mask (no readback)
# + plain context slots: A/B against the VGPR-lane build on the all-intra,
# content and noise streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > /dev/null 2>&1 || exit $?
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/allintra.mp4 3 $O/allintra lanes cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content lanes cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/n0.mp4 2 $O/noise lanes cur || exit $?
