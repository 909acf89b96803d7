"""Several resident sessions through vtseg.batch.plan_batch (every run
submitted before any wait) against one session's run alone: step times and
the result digests.
    python tools/gpu/batch_probe.py VIDEO ..."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "video-transformer_amd"))
import torch
from vtseg import batch, scene

paths = sys.argv[1:]
cfg = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                    "long_video": {"enabled": True, "default_segment_seconds": 480, "overlap_seconds": 20,
                                   "min_segment_seconds": 90, "hard_max_api_calls": 50, "consolidate": True,
                                   "budget_strategy": "compress_segments"}}}  # bench.REF_CONFIG
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
    items = batch.plan_batch(paths, cfg, score=True, sessions=ses)
torch.cuda.synchronize()
bms = (time.perf_counter() - t0) / 3 * 1e3
dig = hashlib.sha1(b"".join(v.score().scores.tobytes() for v in ses.values())).hexdigest()[:16]
print(json.dumps({"queues": os.environ.get("GPU_MAX_HW_QUEUES"), "videos": len(paths), "single_ms": round(single, 2),
                  "batch_ms": round(bms, 2), "batch_over_single": round(bms / single, 3),
                  "cuts": [it.n_cuts for it in items], "digest": dig}))
for v in ses.values():
    v.close()
