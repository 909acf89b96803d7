# General decoder GPU tests only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_full.log
exit $rc
