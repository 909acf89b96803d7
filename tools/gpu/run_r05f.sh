# Round 5: (1) the scalar CABAC engine (VTS_EXP_SENGINE) against the VGPR
# engine on the all-I content stream (single-wave latency) and the content /
# noise streams; (2) four content sessions through plan_batch with 4 (HIP's
# default) vs 16 hardware queues per process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(6) as ex:
    fs = [ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=18000, **kw),
          ex.submit(scene.synth_write, "/tmp/gintra.mp4", n_frames=80, content=True, gop_max_s=0.01, **kw)]
    fs += [ex.submit(scene.synth_write, f"/tmp/gcontent{i}.mp4", n_frames=18000, content=True, gop_max_s=8.0,
                     **dict(kw, seed=0x5EED + i)) for i in range(4)]
    for f in fs: f.result()
print("streams written", flush=True)
PY
for V in gintra gcontent0 gcab; do
  PASSES=2 timeout -k 10 500 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/ab_$V cur seng || exit 1
done
for Q in 4 16; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python tools/gpu/batch_probe.py /tmp/gcontent0.mp4 /tmp/gcontent1.mp4 /tmp/gcontent2.mp4 /tmp/gcontent3.mp4 > $O/batch_q$Q.json 2> $O/batch_q$Q.err || { tail -20 $O/batch_q$Q.err; exit 1; }
  cat $O/batch_q$Q.json
done
