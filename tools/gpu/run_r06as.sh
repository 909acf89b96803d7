#!/bin/bash
# round 6 (as): the long CABAC parse launch on N compute units of its own, the
# short one on the rest (VTS_PARSE_ISOLATE), same process, content stream;
# the split-parse tests with isolation on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06as
mkdir -p $O
VTS_PARSE_ISOLATE=32 timeout -k 10 300 python -u -m pytest tests/test_parse_split_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 500 python -u tools/gpu/env_ab.py /tmp/c0.mp4 2 off=VTS_PARSE_ISOLATE=0 i32=VTS_PARSE_ISOLATE=32 i64=VTS_PARSE_ISOLATE=64 i16=VTS_PARSE_ISOLATE=16 > $O/ab_content.json 2> $O/ab_content.err || { tail -5 $O/ab_content.err; exit 1; }
cat $O/ab_content.json
