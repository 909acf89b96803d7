# Round 5: GPU parity suite (with the opt-in per-picture scheduler test), then
# same-box A/B of the deblocking wavefront's prefetch depth (VTS_EXP_DBK_PF2:
# the macroblock after next in flight too) on the content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05i}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_full_gpu.py tests/test_decode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
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
  PASSES=2 timeout -k 10 500 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/ab_$V cur ${VARS:-pf2} || exit 1
done
