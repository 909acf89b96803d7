# Round 4: general parser at 5 (in-tree) / 6 / 8 waves per SIMD on the content
# stream (latency-bound parse) and the noise stream (issue-bound).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04m}
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
PASSES=2 bash tools/gpu/lib_ab.sh /tmp/gcontent.mp4 3 $O/ab_content cur w6 w8 || exit 1
PASSES=1 bash tools/gpu/lib_ab.sh /tmp/gcab.mp4 3 $O/ab_noise cur w6 w8 || exit 1
timeout -k 10 800 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['e2e']['value'])
for k in ('general', 'general_content', 'long_video'):
    r = d.get(k, {}); print(k, r.get('value'), r.get('stage_ms'), r.get('open_s'), r.get('windows'), r.get('cuts'), r.get('bits_per_frame'), (r.get('parity') or {}).get('all_equal'))
"
