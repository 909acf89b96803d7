#!/bin/bash
# round 6 (a): the GPU suite on the chunked CABAC arena
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06a/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/r06a/pytest_gpu.log
exit $rc
