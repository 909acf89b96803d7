#!/bin/bash
# round 6 (au): intra + deblocking in one launch per level (h264_intra_deblock)
# — the GPU suite on it, then a same-process A/B of VTS_INTRA_DBK on the
# content and noise streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06au
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 400 python -u tools/gpu/env_ab.py /tmp/c0.mp4 3 fused=VTS_INTRA_DBK=1 two=VTS_INTRA_DBK=0 > $O/ab_content.json 2> $O/ab_content.err || { tail -5 $O/ab_content.err; exit 1; }
cat $O/ab_content.json
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
timeout -k 10 400 python -u tools/gpu/env_ab.py /tmp/n0.mp4 1 fused=VTS_INTRA_DBK=1 two=VTS_INTRA_DBK=0 > $O/ab_noise.json 2> $O/ab_noise.err || { tail -5 $O/ab_noise.err; exit 1; }
cat $O/ab_noise.json
