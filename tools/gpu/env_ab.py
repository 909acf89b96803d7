"""Same-process A/B of vts_open-time environment switches on one video:
    python tools/gpu/env_ab.py VIDEO RUNS NAME=VAR=VAL[,VAR=VAL] ...
Each variant (in the given order, then again in reverse) opens a session with
its variables set, runs RUNS timed decodes after one warm-up and reports the
mean stage times and the result's checksum (scores / histograms must agree)."""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "video-transformer_amd"))
import numpy as np
import torch
from vtseg import scene

path, runs = sys.argv[1], int(sys.argv[2])
variants = []
for spec in sys.argv[3:]:
    name, _, kv = spec.partition("=")
    env = dict(x.split("=", 1) for x in kv.split(",") if x)
    variants.append((name, env))
res = {n: [] for n, _ in variants}
digest = {}
for order in (variants, variants[::-1]):
    for name, env in order:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        v = scene.VideoScorer(path, device=0, window_frames=int(os.environ.get("AB_WINDOW_FRAMES", "0")))
        for k, x in old.items():
            if x is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = x
        v.run()
        torch.cuda.synchronize()
        for _ in range(runs):
            t0 = time.perf_counter()
            v.run()
            torch.cuda.synchronize()
            res[name].append({"wall_ms": (time.perf_counter() - t0) * 1e3, **v.timings()})
        r = v.score()
        digest[name] = hashlib.sha1(r.scores.tobytes() + r.hist.tobytes() + r.sad.tobytes()).hexdigest()[:16]
        v.close()
out = {}
for name, rows in res.items():
    out[name] = {k: round(float(np.mean([r[k] for r in rows])), 2) for k in rows[0]}
    out[name]["digest"] = digest[name]
print(json.dumps(out))
