# Round 5: CABAC arena cut to each slice's stored blocks after the first clean
# run: general-decoder GPU tests, then the sessions' device bytes before and
# after the first run and same-box step times on 10-min 720p content / noise.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05aq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
tail -2 $O/pytest_gpu.txt
grep -n "FAILED" $O/pytest_gpu.txt | head
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
timeout -k 10 400 python - <<'PY' > $O/device_bytes.json || exit 1
import json, sys, time; sys.path.insert(0, "video-transformer_amd")
import torch
from vtseg import _lib, scene
L = _lib.lib()
out = {}
for V in ("gcontent", "gcab"):
    b0 = int(L.vts_device_bytes(0))
    with scene.VideoScorer(f"/tmp/{V}.mp4") as v:
        opened = int(L.vts_device_bytes(0)) - b0
        a0 = int(L.vts_schedule_info(v._ctx, 10))
        v.run(); torch.cuda.synchronize()
        after = int(L.vts_device_bytes(0)) - b0
        a1 = int(L.vts_schedule_info(v._ctx, 10))
        ts = []
        for _ in range(3):
            t = time.perf_counter(); v.run(); torch.cuda.synchronize(); ts.append((time.perf_counter() - t) * 1e3)
        out[V] = {"session_gb_open": round(opened / 1e9, 2), "session_gb_after_first_run": round(after / 1e9, 2),
                  "arena_blocks_open": a0, "arena_blocks_after": a1, "step_ms": [round(x, 1) for x in ts],
                  "timings": v.timings()}
print(json.dumps(out))
PY
cat $O/device_bytes.json
