# Round 5: recycled surfaces in the general decoder (VTS_SURF_POOL) and the
# packed inter prediction (VTS_EXP_INTER_PK, pk4 = + occupancy 4): the GPU
# suite, then same-box A/B on 10-min 720p content and noise streams (each
# library with the pool on and off), and the session's device bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu.txt
grep -n "FAILED\|ERROR" $O/pytest_gpu.txt | head -20
# assertion failures (rc 1) still leave the GPU usable; anything else (a crash,
# a time limit) or a device fault message ends the call here
if [ $rc -gt 1 ] || grep -q "Memory access fault\|HSA_STATUS_ERROR\|hipErrorLaunchFailure" $O/pytest_gpu.txt; then exit 1; fi
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
                                      "surfaces": int(L.vts_schedule_info(v._ctx, 11)),
                                      "ring_frames": int(L.vts_schedule_info(v._ctx, 3))}
print(json.dumps(out))
PY
cat $O/device_bytes.json
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
for V in gcontent gcab; do
  for L in cur pk pk4 pk4 pk cur; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    timeout -k 10 200 python tools/gpu/env_ab.py /tmp/$V.mp4 3 ${L}_pool=VTS_SURF_POOL=1 ${L}_nopool=VTS_SURF_POOL=0 >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    tail -1 $O/ab_$V.jsonl
  done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
