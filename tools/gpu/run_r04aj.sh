# Round 4 final check (deblocking by plane, still-macroblock stores skipped): full GPU parity suite, smoke, the default bench line with
# its rocprofv3 summaries, and a kernel trace of the content stream (tools/kt_timeline.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r04aj}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 800 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['e2e']['value'])
for k in ('general', 'general_content', 'long_video'):
    r = d.get(k, {}); print(k, r.get('value'), r.get('stage_ms'), r.get('open_s'), r.get('windows'), r.get('cuts'), r.get('bits_per_frame'), (r.get('parity') or {}).get('all_equal'))
"
timeout -k 10 300 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from vtseg import scene
scene.synth_write("/tmp/gcontent.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                  slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True,
                  content=True, gop_max_s=8.0)
print("content stream written", flush=True)
PY
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/kt_gcontent" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/env_ab.py" /tmp/gcontent.mp4 1 x= > "$GRAFT_REPO_ROOT/$O/kt_gcontent.log" 2>&1) || { tail -30 $O/kt_gcontent.log; exit 1; }
echo traced
