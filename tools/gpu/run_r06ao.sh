#!/bin/bash
# round 6 (ao): the default bench line after the e2e record's page-cache read
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ao
mkdir -p $O
timeout -k 10 900 python -u bench.py --no-pmc > $O/bench.json 2> $O/bench.err
rc=$?
tail -10 $O/bench.err
exit $rc
