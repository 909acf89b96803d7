# Round 4: the bS-schedule parity test (VTS_BS 0 / 1 / 2 x 1 / 2 GOP groups,
# one window and several) and the rest of the general-decoder GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04ab}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_full_gpu.py tests/test_recon_groups_gpu.py > $O/pytest_general.log 2>&1 || { tail -30 $O/pytest_general.log; exit 1; }
grep -c PASSED $O/pytest_general.log
grep bs_schedules $O/pytest_general.log
tail -1 $O/pytest_general.log
