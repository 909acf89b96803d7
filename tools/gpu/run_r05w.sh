# Round 5: GOP groups 2 / 3 / 4 now that sessions get six streams on six
# hardware queues (16 queues, the bench's setting): content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
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
  GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python tools/gpu/env_ab.py /tmp/$V.mp4 3 g2=VTS_GENERAL_GROUPS=2 g3=VTS_GENERAL_GROUPS=3 g4=VTS_GENERAL_GROUPS=4 > $O/ab_$V.json 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  cat $O/ab_$V.json
done
