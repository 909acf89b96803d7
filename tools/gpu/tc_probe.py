"""Transcode timing probe: synthetic video -> vts_transcode, stage times."""
import sys, time, json, tempfile
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
from vtseg import scene
W, H, F = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1280, 720, 18000)))
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
d = Path(tempfile.mkdtemp(prefix="tc_", dir="/tmp"))
src = d / "in.mp4"
info = scene.synth_write(src, width=W, height=H, n_frames=F)
with scene.VideoScorer(src) as v:
    for r in range(reps):
        t = time.perf_counter()
        f = v.transcode(d / "out.mp4")
        f["wall_ms"] = (time.perf_counter() - t) * 1e3
        f["in_bytes"] = src.stat().st_size
        f["fps"] = F / f["wall_ms"] * 1e3
        print(json.dumps(f), flush=True)
