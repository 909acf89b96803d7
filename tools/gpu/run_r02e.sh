# B pictures on the device: the general decoder's GPU parity tests (incl. the
# new B-stream cases), then the remaining GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { tail -60 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread --deselect tests/test_full_gpu.py > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
