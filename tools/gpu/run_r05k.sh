# Round 5: subset-decoder GPU tests (threaded NAL walk), the hipMalloc probe,
# the 2-h 720p open stages (vts_open_timings, 3 opens in one process), and the
# deblocking store-ordering A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/gpu/alloc_probe.py > $O/alloc.json 2> $O/alloc.err || { tail -5 $O/alloc.err; exit 1; }
cat $O/alloc.json
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'video-transformer_amd')
from vtseg import scene
scene.synth_write('/tmp/long.mp4', width=1280, height=720, fps=30, n_frames=216000, seed=0x5EED)
print('long written', flush=True)
" || exit 1
timeout -k 10 300 python tools/gpu/open_probe.py 3 /tmp/long.mp4 > $O/open.json 2> $O/open.err || { tail -5 $O/open.err; exit 1; }
cat $O/open.json
rm -f /tmp/long.mp4
TAG=r05k VARS="buf bufpf2" bash tools/gpu/run_r05i.sh
