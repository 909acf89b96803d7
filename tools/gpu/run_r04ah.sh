# Round 4: deblocking by plane, still macroblocks store only a filtered left neighbour's columns.
# General parity suite with the in-tree library, then a same-box A/B against
# the previous deblocking kernel (tools/exp/lib_prev.so) on the content and
# noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04ah}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_full_gpu.py tests/test_recon_groups_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
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
  PASSES=2 bash tools/gpu/lib_ab.sh /tmp/$V.mp4 3 $O/$V cur prev || exit 1
done
