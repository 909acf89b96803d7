# Round 5: GPU tests after the mapped-file open (subset decoder), then the
# 2-h 720p open stages: mapped (default) and the host-copy path (VTS_OPEN_COPY).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_full_gpu.py tests/test_transcode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'video-transformer_amd')
from vtseg import scene
scene.synth_write('/tmp/long.mp4', width=1280, height=720, fps=30, n_frames=216000, seed=0x5EED)
print('long written', flush=True)
" || exit 1
timeout -k 10 300 python tools/gpu/open_probe.py 3 /tmp/long.mp4 > $O/open_map.json 2> $O/open_map.err || { tail -5 $O/open_map.err; exit 1; }
cat $O/open_map.json
VTS_OPEN_COPY=1 timeout -k 10 300 python tools/gpu/open_probe.py 3 /tmp/long.mp4 > $O/open_copy.json 2> $O/open_copy.err || { tail -5 $O/open_copy.err; exit 1; }
cat $O/open_copy.json
