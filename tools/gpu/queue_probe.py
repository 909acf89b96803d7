"""General decoder timing in a fresh process vs after other sessions were
opened, run and closed in the same process (bench.py's general record runs
after the batch's and the 2-h video's sessions)."""
import sys
import time

sys.path.insert(0, "video-transformer_amd")
import torch  # noqa: E402
from vtseg import scene  # noqa: E402


def timeit(path):
    v = scene.VideoScorer(path, device=0)
    v.run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(2):
        v.run()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t) / 2
    r = (round(el * 1e3, 1), {k: round(x, 1) for k, x in v.timings().items()})
    v.close()
    return r


import os  # noqa: E402
if not os.path.exists("/tmp/gcab.mp4"):
    scene.synth_write("/tmp/gcab.mp4", width=1280, height=720, fps=30, n_frames=18000, seed=0x5EED, coding="full",
                      slices_per_row=0, max_motion=4, bframes=True, weighted="implicit", cabac=True,
                      transform_8x8=True)
scene.synth_write("/tmp/small.mp4", width=1280, height=720, fps=30, n_frames=1800, seed=7)
print("fresh", timeit("/tmp/gcab.mp4"), flush=True)
vs = [scene.VideoScorer("/tmp/small.mp4", device=0) for _ in range(5)]
for v in vs:
    v.run()
torch.cuda.synchronize()
for v in vs:
    v.close()
print("after 5 sessions closed", timeit("/tmp/gcab.mp4"), flush=True)
vs = [scene.VideoScorer("/tmp/small.mp4", device=0) for _ in range(3)]
for v in vs:
    v.run()
torch.cuda.synchronize()
print("with 3 sessions open", timeit("/tmp/gcab.mp4"), flush=True)
for v in vs:
    v.close()
