#!/bin/bash
# round 6 (ai): the short parse on the own-queue group stream of CU-masked sets, a CU-masked stream for plain sets
# queue of its own) — the split-parse tests, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ai
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parse_split_gpu.py tests/test_batch_native.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --no-pmc > $O/bench.json 2> $O/bench.err
rc=$?
tail -9 $O/bench.err
exit $rc
