# Round 5: transcode GPU tests (+ the unwritable-output test); the general
# decoder's paced bS on its own stream in multi-window runs:
# content stream in 3 windows, VTS_BS_STREAM 0 (score stream) vs 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_transcode_gpu.py tests/test_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
scene.synth_write("/tmp/gcontent.mp4", n_frames=18000, content=True, gop_max_s=8.0, **kw)
print("streams written", flush=True)
PY
AB_WINDOW_FRAMES=6000 timeout -k 10 300 python tools/gpu/env_ab.py /tmp/gcontent.mp4 3 score=VTS_BS_STREAM=0 own=VTS_BS_STREAM=1 > $O/ab_w6000.json 2> $O/ab_w6000.err || { tail -20 $O/ab_w6000.err; exit 1; }
cat $O/ab_w6000.json
timeout -k 10 300 python tools/gpu/env_ab.py /tmp/gcontent.mp4 3 score=VTS_BS_STREAM=0 own=VTS_BS_STREAM=1 > $O/ab_w0.json 2> $O/ab_w0.err || { tail -20 $O/ab_w0.err; exit 1; }
cat $O/ab_w0.json
