# Round 5: subset + general GPU tests after the reading threads took over the
# NAL walk, then the 2-h 720p open stages with 8 and 16 reading threads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_full_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'video-transformer_amd')
from vtseg import scene
scene.synth_write('/tmp/long.mp4', width=1280, height=720, fps=30, n_frames=216000, seed=0x5EED)
print('long written', flush=True)
" || exit 1
for T in 8; do
  VTS_READ_THREADS=$T timeout -k 10 300 python tools/gpu/open_probe.py 3 /tmp/long.mp4 > $O/open_t$T.json 2> $O/open_t$T.err || { tail -5 $O/open_t$T.err; exit 1; }
  cat $O/open_t$T.json
done
