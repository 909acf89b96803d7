"""Per-slice wave times of the CABAC parse (VTS_EXP_PROF build copied over
vtseg/libvtseg.so): one decode of the given video, then for the last parse
launch each workgroup's start / end s_memtime, the slice it parsed and its
NAL size; prints the launch span, the busy sum, the longest slices' times
and a size-binned summary (is the launch bound by its longest slices?)."""
import ctypes as C
import json
import sys

import numpy as np

sys.path.insert(0, "video-transformer_amd")
sys.path.insert(0, "oracle")
import torch  # noqa: F401  (libvtseg binds to torch's HIP runtime)
import oracle
from vtseg import _lib, scene

path = sys.argv[1]
v = scene.VideoScorer(path, device=0, decoder="general")
v.run()
torch.cuda.synchronize()
v.run()
torch.cuda.synchronize()
n = v.n_frames  # one slice per picture in these streams
fn = _lib.lib().vts_debug_parse_waves
fn.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(3 * n, np.uint64)
fn(buf.ctypes.data, n)
t = buf.reshape(n, 3)
start, end = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
sl = (t[:, 2] & 0xffffffff).astype(np.int64)
hw = (t[:, 2] >> 32).astype(np.int64)
m = oracle.read_mp4(path)
# window slice index -> sample size (one window, slices in parse-level order: map by the scheduler's order is
# not exported; use durations vs rank of size instead)
dur = end - start
t0 = start.min()
span = end.max() - t0
order = np.argsort(-dur)
res = {"video": path, "timings": v.timings(), "span_ticks": int(span), "busy_sum_ticks": int(dur.sum()),
       "mean_concurrency": round(float(dur.sum() / span), 1),
       "longest": [[int(dur[k]), int(start[k] - t0), int(end[k] - t0), int(sl[k]), int(hw[k])] for k in order[:12]],
       "dur_pct": {p: int(np.percentile(dur, p)) for p in (50, 90, 99, 100)},
       "sizes_pct": {p: int(np.percentile(m["sizes"], p)) for p in (50, 90, 99, 100)},
       "end_pct_of_span": {p: round(float((np.percentile(end, p) - t0) / span), 3) for p in (50, 90, 99, 99.9)}}
# concurrency over time (20 bins)
bins = np.linspace(t0, t0 + span, 21)
conc = []
for b0, b1 in zip(bins[:-1], bins[1:]):
    ov = np.clip(np.minimum(end, b1) - np.maximum(start, b0), 0, None)
    conc.append(round(float(ov.sum() / (b1 - b0)), 1))
res["concurrency_by_twentieth"] = conc
print(json.dumps(res))
v.close()
