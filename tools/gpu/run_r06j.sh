#!/bin/bash
# round 6 (j): GPU suite, then the default bench line (box default hardware
# queues; new records general_long / general_hd, mixed content + noise batch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 800 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -14 $O/bench.err
exit $rc
