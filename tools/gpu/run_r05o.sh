# Round 5: config [3]'s batch step after other sessions (the bench's order)
# against a fresh process, 16 and 32 hardware queues.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, n_frames=18000, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(6) as ex:
    fs = [ex.submit(scene.synth_write, f"/tmp/gc{i}.mp4", content=True, gop_max_s=8.0, **dict(kw, seed=0x5EED + i)) for i in range(4)]
    fs.append(ex.submit(scene.synth_write, "/tmp/gnoise.mp4", **dict(kw, seed=0x5EED)))
    fs.append(ex.submit(scene.synth_write, "/tmp/sub.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=7))
    for f in fs: f.result()
print("streams written", flush=True)
PY
V="/tmp/gc0.mp4 /tmp/gc1.mp4 /tmp/gc2.mp4 /tmp/gc3.mp4"
for Q in 16 32; do
  for PRE in "" "/tmp/sub.mp4,/tmp/sub.mp4,/tmp/gnoise.mp4,/tmp/gc0.mp4"; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python tools/gpu/batch_ctx_probe.py "$PRE" $V > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    cat $O/b.json
  done
done
