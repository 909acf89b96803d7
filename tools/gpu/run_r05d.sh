# Round 5: DbkInfo level ring, CABAC arena estimate + overflow re-run, async
# runs (plan_batch submits every session first), derive prefetch.  GPU parity
# suite; parse wave timeline + section profile (VTS_EXP_PROF build) of the
# content and noise streams; then the default bench line (with general_batch).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
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
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/env_ab.py /tmp/$V.mp4 3 x= > $O/ab_$V.json 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  cat $O/ab_$V.json
done
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB /tmp/lib_intree.so
cp tools/exp/lib_prof.so $LIB
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/parse_waves.py /tmp/$V.mp4 > $O/waves_$V.json 2> $O/waves_$V.err || { tail -20 $O/waves_$V.err; cp /tmp/lib_intree.so $LIB; exit 1; }
  timeout -k 10 300 python tools/gpu/parse_prof.py /tmp/$V.mp4 > $O/sections_$V.json 2> $O/sections_$V.err || { tail -20 $O/sections_$V.err; cp /tmp/lib_intree.so $LIB; exit 1; }
  head -c 1500 $O/waves_$V.json; echo; cat $O/sections_$V.json
done
cp /tmp/lib_intree.so $LIB
timeout -k 10 900 python -u bench.py --profile-dir $O/prof > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['frac'], d['parity']['all_equal'], d['e2e'].get('value'), d['cpu_baseline']['value'])
for k in ('general_batch', 'general', 'general_content', 'long_video', 'hd_1080p'):
    r = d.get(k, {}); print(k, r.get('value'), r.get('ms_per_step'), r.get('single_video_ms'), r.get('batch_over_single'), r.get('hbm_gb_per_session'), r.get('stage_ms'), r.get('open_s'), r.get('cuts'), (r.get('parity') or {}).get('all_equal'), r.get('error'))
"
