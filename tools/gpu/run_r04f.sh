set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 200 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/qvga.mp4", n_frames=8, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7, coding="full", seed=31, width=320, height=240, max_motion=3)
scene.synth_write("/tmp/tiny.mp4", n_frames=8, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7, coding="full", seed=31, width=48, height=32, max_motion=2)
PY
for v in qvga tiny; do
timeout -k 10 200 python tools/gpu/intra_diff.py /tmp/$v.mp4 VTS_INTRA=1 VTS_INTRA=2 > $O/diff_$v.txt 2>&1 || { tail -20 $O/diff_$v.txt; exit 1; }
head -120 $O/diff_$v.txt
done
