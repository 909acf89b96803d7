#!/bin/bash
# round 6 (an): intra coefficient rows prefetched with the header (i2_prefetch) — the GPU suite,
# then A/B against the previous build (tools/exp/lib_base.so) on the content and noise streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06an
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content base cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/n0.mp4 2 $O/noise base cur || exit $?
