# Round 5: deblocking step sections (VTS_EXP_RPROF build) on the content and
# noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    fs = [ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=3000, **kw),
          ex.submit(scene.synth_write, "/tmp/gcontent.mp4", n_frames=3000, content=True, gop_max_s=8.0, **kw)]
    for f in fs: f.result()
print("streams written", flush=True)
PY
cp video-transformer_amd/vtseg/libvtseg.so /tmp/lib_intree.so
cp tools/exp/lib_rprof.so video-transformer_amd/vtseg/libvtseg.so
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/$V.mp4 > $O/rprof_$V.json 2> $O/rprof_$V.err || { tail -20 $O/rprof_$V.err; cp /tmp/lib_intree.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
  cat $O/rprof_$V.json
done
cp /tmp/lib_intree.so video-transformer_amd/vtseg/libvtseg.so
