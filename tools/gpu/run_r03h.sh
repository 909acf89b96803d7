# Round 3: merged parse launch (B slices wait on per-picture completion
# counters instead of one launch per colocated level): general-decoder GPU
# parity (merged is the default), then same-box A/B by VTS_PARSE_MERGE.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_full_gpu.py tests/test_transcode_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1 || { tail -30 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
python - <<'PY'
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
from concurrent.futures import ThreadPoolExecutor
kw = dict(width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full", slices_per_row=0,
          max_motion=4, bframes=True, weighted="implicit")
with ThreadPoolExecutor(2) as ex:
    a = ex.submit(scene.synth_write, "/tmp/gcab.mp4", cabac=True, transform_8x8=True, **kw)
    b = ex.submit(scene.synth_write, "/tmp/gcavlc.mp4", **kw)
    a.result(); b.result()
print("streams written")
PY
for v in gcab gcavlc; do
for m in 0 1 0 1; do
  VTS_PARSE_MERGE=$m timeout -k 10 300 python bench.py --video /tmp/$v.mp4 --config 720p-10min --coding full --bframes --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-parity --extras none > $O/ab_${v}_$m.json 2> $O/ab_${v}_$m.err || { tail -20 $O/ab_${v}_$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/ab_${v}_$m.json')); print('$v merge=$m', d['value'], d['config']['stage_ms'])" | tee -a $O/ab.txt
done
done
