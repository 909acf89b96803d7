"""Per-workgroup start / end of h264_deblock_plane and h264_intra_v2 on one
run of VIDEO (experiment library built with tools/exp/wg_trace.h): per level
launch, how late its last workgroup started after its first (start skew),
its slowest and median workgroup, and the launch's span.
    python tools/gpu/wg_trace.py LIB VIDEO"""
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

REC = np.dtype([("key", "<u8"), ("t0", "<u8"), ("t1", "<u8"), ("block", "<u4"), ("grid", "<u4")])
L = _lib.lib()
fn = L.vts_wg_dump
fn.restype = C.c_int
fn.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(1 << 18, REC)
with scene.VideoScorer(sys.argv[2], device=0) as v:
    v.run()
    fn(buf.ctypes.data, len(buf))
    v.run()
    n = fn(buf.ctypes.data, len(buf))
    t = v.timings()
r = buf[:n]
out = {"timings": {k: round(x, 2) for k, x in t.items()}, "records": int(n)}
for kern, name in ((0, "deblock"), (1, "intra")):
    s = r[(r["key"] & 1) == kern]
    keys = np.unique(s["key"])
    skew, mx, med, span, grid = [], [], [], [], []
    for k in keys:
        g = s[s["key"] == k]
        d = (g["t1"].astype(np.int64) - g["t0"].astype(np.int64)) / 100.0  # us (100 MHz)
        skew.append((int(g["t0"].max()) - int(g["t0"].min())) / 100.0)
        span.append((int(g["t1"].max()) - int(g["t0"].min())) / 100.0)
        mx.append(float(d.max()))
        med.append(float(np.median(d)))
        grid.append(int(g["grid"][0]))
    q = lambda a: [round(float(np.percentile(a, p)), 1) for p in (10, 50, 90, 100)]  # noqa: E731
    out[name] = {"launches": len(keys), "workgroups": int(len(s)), "grid_p10_50_90_100": q(grid),
                 "start_skew_us": q(skew), "slowest_wg_us": q(mx), "median_wg_us": q(med), "span_us": q(span),
                 "sum_span_ms": round(sum(span) / 1e3, 2), "sum_slowest_ms": round(sum(mx) / 1e3, 2),
                 "sum_skew_ms": round(sum(skew) / 1e3, 2)}
print(json.dumps(out, indent=1), flush=True)
