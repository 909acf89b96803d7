"""vts_open of the 2-h video after the bench's earlier sessions (held open
together, then closed, in the bench's order), with VTS_DEVMEM_LOG=1 on stderr.
    python tools/gpu/open_order_probe.py LONG SUB1,SUB2,.. NOISE CONTENT"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "video-transformer_amd"))
import torch
from vtseg import scene

long_p, subs, noise, content = sys.argv[1], sys.argv[2].split(","), sys.argv[3], sys.argv[4]
torch.zeros(1, device="cuda")
out = {}
ses = [scene.VideoScorer(p, device=0) for p in subs]
for v in ses:
    v.run()
torch.cuda.synchronize()
for v in ses:
    v.close()
print("[probe] headline-like sessions closed", file=sys.stderr, flush=True)
for name, p in (("noise", noise), ("content", content)):
    t0 = time.perf_counter()
    v = scene.VideoScorer(p, device=0)
    out[name + "_open_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    out[name + "_stages"] = {k: round(x, 1) for k, x in v.open_timings().items()}
    v.run()
    torch.cuda.synchronize()
    v.close()
    print(f"[probe] {name} closed", file=sys.stderr, flush=True)
t0 = time.perf_counter()
v = scene.VideoScorer(long_p, device=0)
out["long_open_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
out["long_stages"] = {k: round(x, 1) for k, x in v.open_timings().items()}
v.close()
print(json.dumps(out))
