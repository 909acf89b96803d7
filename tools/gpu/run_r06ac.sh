#!/bin/bash
# round 6 (ac): per-workgroup start / end of the deblocking and intra
# launches (tools/exp/wg_trace.h variant) on the 10-min content and noise
# streams: start skew vs slowest plane per level launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 200 python -u tools/gpu/wg_trace.py tools/exp/lib_wg.so /tmp/c0.mp4 > $O/content.json 2> $O/content.err || { tail -5 $O/content.err; exit 1; }
cat $O/content.json
timeout -k 10 300 python -u tools/gpu/write_streams.py noise 18000 /tmp/n0.mp4 || exit $?
timeout -k 10 200 python -u tools/gpu/wg_trace.py tools/exp/lib_wg.so /tmp/n0.mp4 > $O/noise.json 2> $O/noise.err || { tail -5 $O/noise.err; exit 1; }
cat $O/noise.json
