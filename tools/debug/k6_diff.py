"""Locate macroblocks where the device decode differs from the oracle."""
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "video-transformer_amd"), str(ROOT / "oracle")]
import oracle  # noqa: E402
from vtseg import scene  # noqa: E402

d = Path(tempfile.mkdtemp())
p = d / "h.mp4"
kw = dict(width=480, height=270, max_motion=7, odd_motion=True)
scene.synth_write(p, n_frames=50, cut_min_s=0.5, cut_max_s=1.0, gop_max_s=0.6, hash_frames=True, **kw)
frames, info = oracle.decode_file(p)
W, H = 480, 270
for k, fused in ((6, 1), (6, -1)):
    with scene.VideoScorer(p, k=k, fused=fused) as v:
        v.score()
        bad = []
        for i in range(50):
            g = v.frame_nv12(i).reshape(frames[i].shape)
            if not np.array_equal(g, frames[i]):
                diff = np.argwhere(g != frames[i])
                ys, xs = diff[:, 0], diff[:, 1]
                mbs = sorted({(int(y) // 16 if y < H else (int(y) - H) // 8, int(x) // 16, int(y) >= H)
                              for y, x in diff[:2000]})
                bad.append((i, len(diff), mbs[:12]))
        print(f"k={k} fused={fused}: {len(bad)} bad frames")
        for b in bad[:4]:
            print("  frame", b[0], "ndiff", b[1], "(mby, mbx, chroma):", b[2])
