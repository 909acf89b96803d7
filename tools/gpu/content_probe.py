"""Write a 10-min 720p content stream (synth_content.h) and report its rate,
the device decode's stage times over RUNS runs and planted vs detected cuts:
    python tools/gpu/content_probe.py OUT.mp4 RUNS"""
import json
import sys
import time

sys.path.insert(0, "video-transformer_amd")
import torch
from vtseg import scene

path, runs = sys.argv[1], int(sys.argv[2])
t0 = time.perf_counter()
info = scene.synth_write(path, width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                         slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                         transform_8x8=True, content=True, gop_max_s=8.0)
write_s = time.perf_counter() - t0
print(f"written in {write_s:.1f} s", file=sys.stderr, flush=True)
t0 = time.perf_counter()
v = scene.VideoScorer(path, device=0)
open_s = time.perf_counter() - t0
v.run()
torch.cuda.synchronize()
st = []
for _ in range(runs):
    t0 = time.perf_counter()
    v.run()
    torch.cuda.synchronize()
    st.append((time.perf_counter() - t0, v.timings()))
det = v.scene_cuts()
v.close()
planted = info["cuts"]
wall = sum(s for s, _ in st) / runs
keys = st[0][1].keys()
print(json.dumps({"write_s": round(write_s, 1), "open_s": round(open_s, 3), "bytes": info["bytes"],
                  "kbit_per_frame": round(info["bytes"] * 8 / 18000 / 1000, 1), "n_idr": info["n_idr"],
                  "wall_ms": round(wall * 1e3, 2), "frames_per_s": round(18000 / wall, 1),
                  "stage_ms": {k: round(sum(t[k] for _, t in st) / runs, 2) for k in keys},
                  "planted_cuts": len(planted), "detected_cuts": len(det),
                  "detected_at_planted": len(set(det) & set(planted))}))
