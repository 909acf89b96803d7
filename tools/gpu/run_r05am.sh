# Round 5: thumb_pics row bands sized for 1 / 2 / 4 / 8 chunks per thread
# (VTS_THUMB_CHUNKS; static per process, so one process per setting), and the
# pool off for reference; 10-min 720p content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05am
mkdir -p $O
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    fs = [ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=18000, **kw),
          ex.submit(scene.synth_write, "/tmp/gcontent.mp4", n_frames=18000, content=True, gop_max_s=8.0, **kw)]
    for f in fs: f.result()
print("streams written", flush=True)
PY
for V in gcontent gcab; do
  for C in 4 2 1 8 nopool 8 1 2 4; do
    if [ $C = nopool ]; then spec="nopool=VTS_SURF_POOL=0"; else spec="c$C="; fi
    VTS_THUMB_CHUNKS=${C/nopool/4} timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 3 $spec >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
done
