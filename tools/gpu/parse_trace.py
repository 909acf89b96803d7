"""Section timing of the CABAC slice parser (experiment library built with
tools/exp/trace_dev.h): one run of VIDEO, then every parse wave's buckets;
prints the longest wave's cycles per trace section and the whole launch's.
    python tools/gpu/parse_trace.py tools/exp/lib_trace.so VIDEO"""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from vtseg import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
from vtseg import scene  # noqa: E402

NAMES = {0: "begin_mb..", 1: "dec", 2: "bypass", 3: "term", 4: "skip(B)..", 5: "skip(P)..", 6: "b_direct..",
         7: "store_block..", 8: "end_mb..", 9: "init_mb..", 10: "after dec", 11: "after bypass",
         12: "residual setup..", 13: "residual_t entry..", 14: "level loop..", 15: "slice start..", 16: "slice end"}
K = 20
v = scene.VideoScorer(sys.argv[2], device=0)
v.run()
v.run()
nsl = int(v._lib.vts_schedule_info(v._ctx, 2))
L = _lib.lib()
buf = np.zeros(4096 * 2 * K, np.uint64)
n = L.vts_trace_dump(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), max(1, min(nsl, 4096)))
print("slices", nsl, "dumped", n, file=sys.stderr, flush=True)
t = buf[: n * 2 * K].reshape(n, 2, K)
tot = t[:, 0, :].sum(1)
w = int(tot.argmax())
out = {"slices": nsl, "waves_read": n, "longest_wave": w, "longest_cycles": int(tot[w]),
       "timings": {k: round(x, 2) for k, x in v.timings().items()},
       "longest": {NAMES.get(i, str(i)): {"cycles": int(t[w, 0, i]), "visits": int(t[w, 1, i]),
                                          "per_visit": round(float(t[w, 0, i]) / max(1, int(t[w, 1, i])), 1)}
                   for i in range(K) if t[w, 1, i]},
       "all_waves": {NAMES.get(i, str(i)): {"cycles": int(t[:, 0, i].sum()), "visits": int(t[:, 1, i].sum())}
                     for i in range(K) if t[:, 1, i].sum()}}
v.close()
print(json.dumps(out, indent=1), flush=True)
