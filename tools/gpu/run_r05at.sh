# Round 5: the CABAC parse kernel with the per-slice stored-block output
# (in-tree, arena tightened) vs without it (lib_nouse, VTS_ARENA_TIGHT=0):
# same box, processes alternated, 10-min 720p content / noise.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05at}
mkdir -p $O
if [ -n "$SUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
fi
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
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
for V in gcontent gcab; do
  for L in cur nouse nouse cur cur nouse; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    T=1; [ $L = nouse ] && T=0
    VTS_ARENA_TIGHT=$T timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 4 $L= >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
