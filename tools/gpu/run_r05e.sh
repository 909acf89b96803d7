# Round 5: long CABAC slices' wave priority (s_setprio 3 for the first n_long
# workgroups) A/B against no priority, on the content and noise streams; and
# the parse time of an all-I content stream of 80 pictures (its waves nearly
# alone on their compute units: the long slices' uncontended time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(3) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=18000, **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcontent.mp4", n_frames=18000, content=True, gop_max_s=8.0, **kw)
    c = ex.submit(scene.synth_write, "/tmp/gintra.mp4", n_frames=80, content=True, gop_max_s=0.01, **kw)
    a.result(); b.result(); c.result()
print("streams written", flush=True)
PY
timeout -k 10 200 python tools/gpu/env_ab.py /tmp/gintra.mp4 5 x= > $O/ab_gintra.json 2> $O/ab_gintra.err || { tail -20 $O/ab_gintra.err; exit 1; }
cat $O/ab_gintra.json
for V in gcontent gcab; do
  PASSES=2 timeout -k 10 500 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/ab_$V cur noprio || exit 1
done
