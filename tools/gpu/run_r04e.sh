# Round 4: lane-parallel intra (h264_intra_v2) parity and same-box A/B against
# h264_intra_full, its section profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04e}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_full_gpu.py tests/test_transcode_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED,
                  coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                  transform_8x8=True)
print("stream written")
PY
timeout -k 10 400 python tools/gpu/env_ab.py /tmp/gcab.mp4 3 intra1=VTS_INTRA=1 intra2=VTS_INTRA=2 > $O/ab_intra.json 2> $O/ab_intra.err || { tail -20 $O/ab_intra.err; exit 1; }
cat $O/ab_intra.json
cp video-transformer_amd/vtseg/libvtseg.so /tmp/lib_cur.so
cp tools/exp/lib_rprof.so video-transformer_amd/vtseg/libvtseg.so
timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/gcab.mp4 > $O/rprof.json 2> $O/rprof.err || { tail -20 $O/rprof.err; cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
cat $O/rprof.json
cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
