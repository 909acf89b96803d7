# Round 3: same-box A/B of parser builds (tools/exp/lib_<name>.so) after the
# GPU parity of the general decoder and the transcode on general inputs, on
# the x264-like 10-min 720p streams (LIBS names the builds, cur = in-tree).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
# an earlier GPU step of the same call failed or was killed: start nothing more
[ -f gpurun_out/gpu_step_failed ] && { echo "earlier GPU step failed; not starting"; exit 1; }
O=gpurun_out/${OUT:-r03i}
mkdir -p $O
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
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
for lib in ${LIBS:-lane cur lane cur}; do
  cp tools/exp/lib_$lib.so video-transformer_amd/vtseg/libvtseg.so
  timeout -k 10 300 python bench.py --video /tmp/$v.mp4 --config 720p-10min --coding full --bframes --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-parity --extras none > $O/ab_${v}_$lib.json 2> $O/ab_${v}_$lib.err || { tail -20 $O/ab_${v}_$lib.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/ab_${v}_$lib.json')); print('$v $lib', d['value'], d['config']['stage_ms'])" | tee -a $O/ab.txt
done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
if [ -n "$PROF" ]; then
cp tools/exp/lib_prof.so video-transformer_amd/vtseg/libvtseg.so
for v in gcab gcavlc; do
timeout -k 10 300 python tools/gpu/parse_prof.py /tmp/$v.mp4 > $O/prof_$v.json 2> $O/prof_$v.err || { tail -20 $O/prof_$v.err; exit 1; }
cat $O/prof_$v.json
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
fi
