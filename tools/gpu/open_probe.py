"""vts_open stage times (vts_open_timings) on the given MP4s, each opened
`reps` times in this process (sessions closed in between)."""
import json
import sys
import time

sys.path.insert(0, "video-transformer_amd")
import torch  # noqa: F401  (libvtseg binds to torch's HIP runtime)
from vtseg import scene

reps = int(sys.argv[1])
out = {}
torch.zeros(1, device="cuda")
for p in sys.argv[2:]:
    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        v = scene.VideoScorer(p, device=0)
        dt = time.perf_counter() - t0
        rows.append({"wall_ms": round(dt * 1e3, 1), "general": v.general(),
                     **{k: round(x, 1) for k, x in v.open_timings().items()}})
        v.close()
    out[p] = rows
print(json.dumps(out))
