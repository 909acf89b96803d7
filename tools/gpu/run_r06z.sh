#!/bin/bash
# round 6 (z): GOP groups 1..4 on the 10-min content and noise streams
# (same process, alternating), to see how much of the reconstruction is the
# groups contending for compute units
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 300 python -u tools/gpu/write_streams.py content 18000 /tmp/c0.mp4 || exit $?
timeout -k 10 400 python -u tools/gpu/env_ab.py /tmp/c0.mp4 2 g1=VTS_GENERAL_GROUPS=1 g2=VTS_GENERAL_GROUPS=2 g3=VTS_GENERAL_GROUPS=3 g4=VTS_GENERAL_GROUPS=4 > $O/ab_content.json 2> $O/ab_content.err || { tail -5 $O/ab_content.err; exit 1; }
cat $O/ab_content.json
