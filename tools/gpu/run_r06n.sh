#!/bin/bash
# round 6 (n): CABAC coefficients in VGPR lanes (no LDS block buffer on the
# device): GPU suite, then same-box A/B against the fixed-table library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/gpu/parse_hot.py /tmp/allintra.mp4 80 1 > /dev/null 2>&1 || exit $?
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/allintra.mp4 3 $O/allintra slot cur || exit $?
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/c0.mp4 3 $O/content slot cur || exit $?
