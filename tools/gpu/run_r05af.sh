# Round 5: recycled surfaces, thumbnails inline on the group stream vs on a
# side stream (lag 3 / 12), with the bench's 16 hardware queues; packed inter
# prediction at occupancy 4 (pk4); 10-min 720p content and noise streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05af
mkdir -p $O
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
    for name, env in (("inline", {}), ("side3", {"VTS_SURF_THUMB": "side", "VTS_SURF_LAG": "3"}),
                      ("side12", {"VTS_SURF_THUMB": "side", "VTS_SURF_LAG": "12"})):
        for k in ("VTS_SURF_THUMB", "VTS_SURF_LAG"): os.environ.pop(k, None)
        os.environ.update(env)
        b0 = int(L.vts_device_bytes(0))
        with scene.VideoScorer(f"/tmp/{V}.mp4") as v:
            v.run(); torch.cuda.synchronize()
            out[f"{V}_{name}"] = {"session_gb": round((int(L.vts_device_bytes(0)) - b0) / 1e9, 2),
                                  "surfaces": int(L.vts_schedule_info(v._ctx, 11))}
print(json.dumps(out))
PY
cat $O/device_bytes.json
cp video-transformer_amd/vtseg/libvtseg.so tools/exp/lib_cur.so
for V in gcontent gcab; do
  for L in cur pk4 pk4 cur; do
    cp tools/exp/lib_$L.so video-transformer_amd/vtseg/libvtseg.so
    timeout -k 10 240 python tools/gpu/env_ab.py /tmp/$V.mp4 3 ${L}_nopool=VTS_SURF_POOL=0 ${L}_inline=VTS_SURF_POOL=1 ${L}_side3=VTS_SURF_THUMB=side,VTS_SURF_LAG=3 ${L}_side12=VTS_SURF_THUMB=side,VTS_SURF_LAG=12 >> $O/ab_$V.jsonl 2> $O/ab_$V.err || { tail -20 $O/ab_$V.err; cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/ab_$V.jsonl').read().splitlines()[-1]); print('$V', {k: (v['reconstruct_ms'], v['score_ms'], v['digest']) for k, v in d.items()})"
  done
done
cp tools/exp/lib_cur.so video-transformer_amd/vtseg/libvtseg.so
