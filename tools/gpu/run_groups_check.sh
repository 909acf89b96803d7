# General decoder reconstruction with 1 vs 2 GOP groups on the x264-like
# 10-min 720p CABAC B stream (is the bench line's general record running its
# two groups serialised?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-groups}
mkdir -p $O
[ -f /tmp/gcab.mp4 ] || timeout -k 10 300 python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                  slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
PY
for g in 2 1 2 1; do
  VTS_GENERAL_GROUPS=$g timeout -k 10 300 python bench.py --video /tmp/gcab.mp4 --config 720p-10min --coding full --bframes --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-parity --extras none > $O/g$g.json 2> $O/g$g.err || { tail -20 $O/g$g.err; exit 1; }
  python -c "import json; d=json.load(open('$O/g$g.json')); print('groups $g', d['value'], d['config']['stage_ms'])" | tee -a $O/groups.txt
done
