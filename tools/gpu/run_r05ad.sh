# Round 5: inter kernel with packed predictions (VTS_EXP_INTER_PK, 133 VGPRs)
# and packed + occupancy 4 (128 VGPRs, 2 spilled) against the in-tree build,
# alternating libraries in separate processes on the content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ad
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
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
for V in gcontent gcab; do
  for L in cur pk pk4 pk4 pk cur; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    timeout -k 10 200 python tools/gpu/env_ab.py /tmp/$V.mp4 3 $L= >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
