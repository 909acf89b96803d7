#!/bin/bash
# round 6 (ap): the e2e record (plan_batch over 4 subset streams) with the
# build before the split parse's own-queue stream (tools/exp/lib_base.so,
# commit 2633b5c) and the current one, alternating, fresh processes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ap
mkdir -p $O
timeout -k 10 300 python -u - <<'PY' || exit $?
import sys; sys.path.insert(0, "."); sys.path.insert(0, "video-transformer_amd")
from pathlib import Path
import bench
bench.synth_videos([(Path(f"/tmp/e{i}.mp4"), 100 + i) for i in range(4)], 1280, 720, 18000)
print("written")
PY
for pass in 1 2; do
  for lib in tools/exp/lib_base.so video-transformer_amd/vtseg/libvtseg.so; do
    timeout -k 10 200 python -u tools/gpu/e2e_probe.py $lib /tmp/e0.mp4 /tmp/e1.mp4 /tmp/e2.mp4 /tmp/e3.mp4 >> $O/e2e.jsonl 2>> $O/e2e.err || { tail -5 $O/e2e.err; exit 1; }
  done
done
cat $O/e2e.jsonl
