#!/bin/bash
# round 6 (t): the writelane -> readlane hazard probe; the headline bench with
# its profiler passes after the pooled streams are released at exit (the
# --pmc passes crashed in __cxa_finalize since the CU-masked stream sets)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
timeout -k 5 60 ./tools/micro/lane_hazard > $O/lane_hazard.json 2>&1
rc=$?; cat $O/lane_hazard.json; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --extras none --no-cpu-baseline --profile-dir $O/prof > $O/bench.json 2> $O/bench.err
rc=$?
tail -8 $O/bench.err
cat $O/prof/profile_passes.json | python -c "import json,sys; d=json.load(sys.stdin); print({k: {kk: v[kk] for kk in ('FETCH_SIZE','WRITE_SIZE','hbm_bytes') if kk in v} if isinstance(v, dict) else v for k, v in d.items()})"
exit $rc
