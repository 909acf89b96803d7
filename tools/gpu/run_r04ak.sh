# Round 4: deblocking by plane, a still macroblock skips the rows-above stores under a clean
# ring line (tools/exp/lib_dirty.so) vs the in-tree library: the general GPU suite on
# dirty, then a same-box A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04ak}
mkdir -p $O
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB /tmp/lib_intree.so
cp tools/exp/lib_dirty.so $LIB
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_full_gpu.py tests/test_recon_groups_gpu.py > $O/pytest_dirty.log 2>&1 || { tail -30 $O/pytest_dirty.log; cp /tmp/lib_intree.so $LIB; exit 1; }
cp /tmp/lib_intree.so $LIB
tail -1 $O/pytest_dirty.log
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
  PASSES=2 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/$V cur dirty || exit 1
done
