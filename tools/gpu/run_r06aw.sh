#!/bin/bash
# round 6 (aw): the stream-release test and its neighbours on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aw
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_full_gpu.py -k "stream_pool or released_stream or async_runs" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
