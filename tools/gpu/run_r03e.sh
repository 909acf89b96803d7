# Round 3: parse section profile (VTS_EXP_PROF build) on the x264-like 10-min
# 720p streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03e
mkdir -p $O
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
from concurrent.futures import ThreadPoolExecutor
kw = dict(width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full", slices_per_row=0,
          max_motion=4, bframes=True, weighted="implicit")
with ThreadPoolExecutor(2) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", cabac=True, transform_8x8=True, **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcavlc.mp4", **kw)
    a.result(); b.result()
print("streams written")
PY
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
cp tools/exp/lib_prof.so video-transformer_amd/vtseg/libvtseg.so
for v in gcab gcavlc; do
timeout -k 10 300 python tools/gpu/parse_prof.py /tmp/$v.mp4 > $O/prof_$v.json 2> $O/prof_$v.err || { tail -20 $O/prof_$v.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
cat $O/prof_$v.json
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
