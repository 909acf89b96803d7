# Round 5: CABAC arena tightened after the first run (VTS_ARENA_TIGHT=1, the
# default) vs kept at the estimate (0); same box, 10-min 720p content / noise.
# The knob is read once per process: one process per setting, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ar
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
  for T in 1 0 0 1 1 0; do
    VTS_ARENA_TIGHT=$T timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 4 tight$T= >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
done
