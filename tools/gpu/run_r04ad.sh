# Round 4: s_memtime section times (VTS_EXP_RPROF build, tools/exp/lib_rprof.so)
# of h264_deblock_lds and h264_intra_v2 on the content and noise streams after
# the round's reconstruction work.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04ad}
mkdir -p $O
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
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB /tmp/lib_intree.so
cp tools/exp/lib_rprof.so $LIB
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/recon_prof.py /tmp/$V.mp4 > $O/sections_$V.json 2> $O/sections_$V.err || { tail -20 $O/sections_$V.err; cp /tmp/lib_intree.so $LIB; exit 1; }
  cat $O/sections_$V.json
done
cp /tmp/lib_intree.so $LIB
