#!/bin/bash
# round 6 (ar): deblocking workgroups of 512 / 256 threads (32 / 16 rows in
# flight: a 720p plane in two / three passes, but a workgroup that fits beside
# the other group's inter waves sooner) against the in-tree 1024, on the noise
# and content streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ar
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/n0.mp4 2 $O/noise cur t512 t256 || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content cur t512 t256 || exit $?
