# Round 4: kernel trace of the general decoder's reconstruction on the content
# and noise streams (one warm-up + one decode each), for the per-stream
# timeline: busy time, gaps between a group's level launches, group overlap.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04p}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcontent.mp4", content=True, gop_max_s=8.0, **kw)
    a.result(); b.result()
print("streams written", flush=True)
PY
for V in gcontent gcab; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/kt_$V" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/env_ab.py" /tmp/$V.mp4 1 x= > "$GRAFT_REPO_ROOT/$O/kt_$V.log" 2>&1) || { tail -30 $O/kt_$V.log; exit 1; }
  tail -1 $O/kt_$V.log
done
find $O -name '*.csv' | head
