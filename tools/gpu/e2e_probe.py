"""plan_batch (score) over 4 synthetic 10-min 720p subset streams in a fresh
process: the bench's e2e record alone, for same-box A/B of library builds.
    python tools/gpu/e2e_probe.py LIB VIDEO..."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "video-transformer_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch  # noqa: E402
from vtseg import _lib  # noqa: E402

_lib.LIB_PATH = Path(sys.argv[1]).resolve()
from vtseg import batch  # noqa: E402
import bench  # noqa: E402

paths = sys.argv[2:]
for p in paths:
    with open(p, "rb") as fh:
        while fh.read(1 << 24):
            pass
torch.cuda.synchronize()
out = []
for _ in range(3):
    t0 = time.perf_counter()
    batch.plan_batch(paths, bench.REF_CONFIG, score=True, device=0)
    out.append(round(time.perf_counter() - t0, 3))
print(json.dumps({"lib": sys.argv[1], "seconds": out}), flush=True)
