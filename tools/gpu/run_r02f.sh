# General decoder GPU parity tests only (B / CABAC B iteration).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/pytest_full.log | tail -40; exit 1; }
tail -3 gpurun_out/pytest_full.log
