# Round 5: split CABAC parse (VTS_PARSE_SPLIT: the intra pictures' long slices
# on their own stream, the other pictures' h264_derive launches beside them):
# general-decoder GPU tests, then same-box A/B on 10-min 720p content / noise.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_full_gpu.py tests/test_decode_gpu.py tests/test_devmem_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -n "FAILED" $O/pytest.txt | head
if [ $rc -ne 0 ]; then exit 1; fi
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python - <<'PY' || exit 1
import sys; sys.path.insert(0, "video-transformer_amd")
from concurrent.futures import ThreadPoolExecutor
from vtseg import scene
kw = dict(width=1280, height=720, fps=30, seed=0x5EED, coding="full", slices_per_row=0, max_motion=4,
          bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
with ThreadPoolExecutor(2) as ex:
    fs = [ex.submit(scene.synth_write, "/tmp/gcab.mp4", n_frames=18000, **kw),
          ex.submit(scene.synth_write, "/tmp/gcontent.mp4", n_frames=18000, content=True, gop_max_s=8.0, **kw)]
    for f in fs: f.result()
print("streams written", flush=True)
PY
for V in gcontent gcab; do
  timeout -k 10 300 python tools/gpu/env_ab.py /tmp/$V.mp4 4 split=VTS_PARSE_SPLIT=1 one=VTS_PARSE_SPLIT=0 >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  tail -1 $O/ab_$V.jsonl
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python tools/gpu/env_ab.py /tmp/gcontent.mp4 4 split4q=VTS_PARSE_SPLIT=1 one4q=VTS_PARSE_SPLIT=0 >> $O/ab_gcontent_4queues.jsonl 2> $O/ab_4q.err || { tail -20 $O/ab_4q.err; exit 1; }
tail -1 $O/ab_gcontent_4queues.jsonl
