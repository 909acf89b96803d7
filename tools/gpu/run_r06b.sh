#!/bin/bash
# round 6 (b): GPU suite, then the default bench line, on the re-entered tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06b
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06b/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r06b/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
rc=$?
tail -3 gpurun_out/r06b/bench.err
exit $rc
