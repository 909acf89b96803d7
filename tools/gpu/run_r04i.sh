# Round 4: parity of the deblocking kernel after the single-read horizontal
# pass; parse sections (VTS_EXP_PROF) and reconstruction sections
# (VTS_EXP_RPROF) on the content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_full_gpu.py tests/test_transcode_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python tools/gpu/content_probe.py /tmp/gcontent.mp4 3 > $O/content.json 2> $O/content.err || { tail -20 $O/content.err; exit 1; }
cat $O/content.json
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED,
                  coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                  transform_8x8=True)
print("noise stream written")
PY
cp video-transformer_amd/vtseg/libvtseg.so /tmp/lib_cur.so
for V in gcontent gcab; do
  cp tools/exp/lib_prof.so video-transformer_amd/vtseg/libvtseg.so
  timeout -k 10 300 python tools/gpu/parse_prof.py /tmp/$V.mp4 > $O/pprof_$V.json 2> $O/pprof_$V.err || { tail -20 $O/pprof_$V.err; cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
  cat $O/pprof_$V.json
  cp tools/exp/lib_rprof.so video-transformer_amd/vtseg/libvtseg.so
  timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/$V.mp4 > $O/rprof_$V.json 2> $O/rprof_$V.err || { tail -20 $O/rprof_$V.err; cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
  cat $O/rprof_$V.json
done
cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
