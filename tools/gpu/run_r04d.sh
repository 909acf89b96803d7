# Round 4: open stages with the caching device allocator, decoder + transcode
# parity on it, intra section profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04d}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(2) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED,
                  coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                  transform_8x8=True)
    b = ex.submit(scene.synth_write, "/tmp/sub.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED)
    a.result(); b.result()
print("streams written")
PY
timeout -k 10 300 python tools/gpu/open_probe.py 3 /tmp/sub.mp4 /tmp/gcab.mp4 /tmp/sub.mp4 > $O/open.json 2> $O/open.err || { tail -20 $O/open.err; exit 1; }
cat $O/open.json
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_full_gpu.py tests/test_transcode_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp video-transformer_amd/vtseg/libvtseg.so /tmp/lib_cur.so
cp tools/exp/lib_rprof.so video-transformer_amd/vtseg/libvtseg.so
timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/gcab.mp4 > $O/rprof.json 2> $O/rprof.err || { tail -20 $O/rprof.err; cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
cat $O/rprof.json
cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
