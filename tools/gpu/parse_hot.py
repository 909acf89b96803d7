"""The CABAC parse of long I slices alone: an all-intra 720p content stream
(every picture an IDR, one slice each) through the general decoder, `runs`
times, with its parse / reconstruction times.  Target of the PC-sampling and
per-bin cost measurements (tools/gpu/run_r06d.sh).
  python tools/gpu/parse_hot.py OUT.mp4 [frames] [runs]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
import torch  # noqa: E402,F401  (HIP runtime first, as bench.py)
from vtseg import scene  # noqa: E402

path = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 80
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
if not Path(path).exists():
    scene.synth_write(path, width=1280, height=720, fps=30, n_frames=frames, seed=0x5EED, coding="full",
                      slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                      transform_8x8=True, content=True, gop_max_s=1.0 / 30, cut_min_s=0.5, cut_max_s=1.0)
v = scene.VideoScorer(path, device=0)
assert v.general()
out = []
for _ in range(runs):
    t0 = time.perf_counter()
    v.run()
    torch.cuda.synchronize()
    out.append({"wall_ms": round((time.perf_counter() - t0) * 1e3, 2),
                **{k: round(x, 2) for k, x in v.timings().items()}})
v.close()
print(json.dumps({"bytes": Path(path).stat().st_size, "frames": frames, "runs": out}), flush=True)
