#!/bin/bash
# round 6 (af): CABAC long slices in a parse launch of their own, the rest and
# the early pictures' derivation beside it — parity (forced / by size / off,
# one and several windows) + the GPU suite, then a same-process A/B of
# VTS_PARSE_SPLIT on the 10-min content and noise streams and the 30-min
# content stream in windows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06af
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 400 python -u tools/gpu/env_ab.py /tmp/c0.mp4 3 split=VTS_PARSE_SPLIT=1 one=VTS_PARSE_SPLIT=0 > $O/ab_content.json 2> $O/ab_content.err || { tail -5 $O/ab_content.err; exit 1; }
cat $O/ab_content.json
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
timeout -k 10 400 python -u tools/gpu/env_ab.py /tmp/n0.mp4 1 split=VTS_PARSE_SPLIT=1 one=VTS_PARSE_SPLIT=0 > $O/ab_noise.json 2> $O/ab_noise.err || { tail -5 $O/ab_noise.err; exit 1; }
cat $O/ab_noise.json
