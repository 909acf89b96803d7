# Round 5: the defaults after r05af (recycled surfaces with thumbnails inline
# in bands of rows, packed inter prediction at occupancy 4): GPU suite, then
# same-box A/B of the pool modes with the bench's 16 hardware queues on 10-min
# 720p content and noise streams, and the sessions' device bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu.txt
grep -n "FAILED\|ERROR" $O/pytest_gpu.txt | head -20
if [ $rc -gt 1 ] || grep -q "Memory access fault\|HSA_STATUS_ERROR\|hipErrorLaunchFailure" $O/pytest_gpu.txt; then exit 1; fi
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
timeout -k 10 300 python - <<'PY' > $O/device_bytes.json || exit 1
import json, os, sys; sys.path.insert(0, "video-transformer_amd")
import torch
from vtseg import _lib, scene
L = _lib.lib()
out = {}
for V in ("gcontent", "gcab"):
    for pool in ("1", "0"):
        os.environ["VTS_SURF_POOL"] = pool
        b0 = int(L.vts_device_bytes(0))
        with scene.VideoScorer(f"/tmp/{V}.mp4") as v:
            v.run(); torch.cuda.synchronize()
            out[f"{V}_pool{pool}"] = {"session_gb": round((int(L.vts_device_bytes(0)) - b0) / 1e9, 2),
                                      "surfaces": int(L.vts_schedule_info(v._ctx, 11))}
print(json.dumps(out))
PY
cat $O/device_bytes.json
for V in gcontent gcab; do
  timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 4 nopool=VTS_SURF_POOL=0 inline=VTS_SURF_POOL=1 side3=VTS_SURF_THUMB=side,VTS_SURF_LAG=3 >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$V.jsonl').read().splitlines()[-1]); print('$V', {k: (v['parse_ms'], v['reconstruct_ms'], v['score_ms'], v['total_ms'], v['digest']) for k, v in d.items()})"
done
