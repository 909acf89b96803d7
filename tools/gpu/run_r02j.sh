# Transcode tests on general-decoder inputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_transcode_gpu.py -v --timeout 240 --timeout-method thread -k general > gpurun_out/pytest_tc.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_tc.log | tail -30; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_tc.log
