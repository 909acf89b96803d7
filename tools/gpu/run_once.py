"""Open VIDEO (general decoder), run it twice (the first warms up): a short
program for profiler runs.  python tools/gpu/run_once.py VIDEO"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
import torch  # noqa: E402,F401
from vtseg import scene  # noqa: E402

with scene.VideoScorer(sys.argv[1], device=0) as v:
    v.run()
    v.run()
    print({k: round(x, 2) for k, x in v.timings().items()}, flush=True)
