"""config [3]'s batch after other sessions came and went (the bench's order):
open, run and close PRE sessions of the given pre-videos, then four resident
content sessions through plan_batch against one alone.
    python tools/gpu/batch_ctx_probe.py PRE1,PRE2,... VIDEO ..."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "video-transformer_amd"))
import torch
from vtseg import batch, scene

pre = [p for p in sys.argv[1].split(",") if p]
paths = sys.argv[2:]
for p in pre:
    with scene.VideoScorer(p, device=0) as v:
        v.run()
torch.cuda.synchronize()
cfg = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                    "long_video": {"enabled": True, "default_segment_seconds": 480, "overlap_seconds": 20,
                                   "min_segment_seconds": 90, "hard_max_api_calls": 50, "consolidate": True,
                                   "budget_strategy": "compress_segments"}}}
ses = {i: scene.VideoScorer(p, device=0) for i, p in enumerate(paths)}
v0 = ses[0]
v0.run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    v0.run()
torch.cuda.synchronize()
single = (time.perf_counter() - t0) / 3 * 1e3
batch.plan_batch(paths, cfg, score=True, sessions=ses)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    batch.plan_batch(paths, cfg, score=True, sessions=ses)
torch.cuda.synchronize()
bms = (time.perf_counter() - t0) / 3 * 1e3
print(json.dumps({"queues": os.environ.get("GPU_MAX_HW_QUEUES"), "pre": len(pre), "single_ms": round(single, 2),
                  "batch_ms": round(bms, 2), "batch_over_single": round(bms / single, 3)}))
for v in ses.values():
    v.close()
