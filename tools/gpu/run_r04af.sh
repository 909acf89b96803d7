# Round 4: deblocking by plane with a one-macroblock lag (VTS_DBK=4) vs without (3) vs
# h264_deblock_lds (2): the general GPU suite with VTS_DBK=4 and with the default (3),
# then a same-box A/B and a kernel trace of VTS_DBK=4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04af}
mkdir -p $O
VTS_DBK=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_full_gpu.py tests/test_recon_groups_gpu.py > $O/pytest_plane.log 2>&1 || { tail -30 $O/pytest_plane.log; exit 1; }
tail -1 $O/pytest_plane.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_full_gpu.py tests/test_recon_groups_gpu.py > $O/pytest_default.log 2>&1 || { tail -30 $O/pytest_default.log; exit 1; }
tail -1 $O/pytest_default.log
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
  timeout -k 10 400 python tools/gpu/env_ab.py /tmp/$V.mp4 3 lds=VTS_DBK=2 plane=VTS_DBK=3 lag1=VTS_DBK=4 > $O/ab_$V.json 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  cat $O/ab_$V.json
done
(cd /tmp && export TMPDIR=/tmp && VTS_DBK=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/kt_gcontent" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/env_ab.py" /tmp/gcontent.mp4 1 x= > "$GRAFT_REPO_ROOT/$O/kt_gcontent.log" 2>&1) || { tail -30 $O/kt_gcontent.log; exit 1; }
echo traced
