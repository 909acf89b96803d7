# Round 4: where the general decoder's deblocking / intra waves spend their
# time (s_memtime sections, VTS_EXP_RPROF build) on the bench's general stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04b}
mkdir -p $O
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=int(__import__("os").environ.get("NF", "18000")),
                  seed=0x5EED, coding="full", slices_per_row=0, max_motion=4, bframes=True,
                  weighted="implicit", cabac=True, transform_8x8=True)
print("stream written")
PY
cp video-transformer_amd/vtseg/libvtseg.so /tmp/lib_cur.so
for lib in ${LIBS:-rprof}; do
cp tools/exp/lib_$lib.so video-transformer_amd/vtseg/libvtseg.so
timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/gcab.mp4 > $O/rprof_$lib.json 2> $O/rprof_$lib.err || { tail -20 $O/rprof_$lib.err; cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
cat $O/rprof_$lib.json
done
cp /tmp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
