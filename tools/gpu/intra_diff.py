"""Debug: decode a small full-syntax stream with two environment variants and
print where the frames differ (first frame, macroblock list, the first bad
macroblocks' luma / chroma differences)."""
import json
import os
import sys

sys.path.insert(0, "video-transformer_amd")
sys.path.insert(0, "oracle")
import numpy as np
import torch  # noqa: F401
from vtseg import scene
import oracle

path = sys.argv[1]
envs = [dict(x.split("=", 1) for x in spec.split(",")) for spec in sys.argv[2:4]]
want, _ = oracle.decode_full(path)
outs = []
for env in envs:
    os.environ.update(env)
    with scene.VideoScorer(path, keep_frames=True) as v:
        v.score()
        outs.append(np.stack([v.frame_nv12(i).reshape(want[i].shape) for i in range(want.shape[0])]))
H = want.shape[1] * 2 // 3
W = want.shape[2]
for name, got in zip(["A", "B"], outs):
    bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
    print(name, "frames differing from the oracle:", bad[:10].tolist())
got = outs[1]
bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
if len(bad):
    f = int(bad[0])
    g, w = got[f].astype(int), want[f].astype(int)
    mbs = []
    for my in range(H // 16):
        for mx in range(W // 16):
            dy = g[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16] != w[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16]
            dc = g[H + my * 8:H + my * 8 + 8, mx * 16:mx * 16 + 16] != w[H + my * 8:H + my * 8 + 8, mx * 16:mx * 16 + 16]
            if dy.any() or dc.any():
                mbs.append((mx, my, int(dy.sum()), int(dc.sum())))
    print("frame", f, "bad MBs (x, y, luma px, chroma px):", mbs[:40], "of", len(mbs))
    for (mx, my, _, _) in mbs[:3]:
        print("MB", mx, my, "luma diff mask:")
        print((g[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16] - w[my * 16:my * 16 + 16, mx * 16:mx * 16 + 16]))
        print("chroma diff:")
        print((g[H + my * 8:H + my * 8 + 8, mx * 16:mx * 16 + 16] - w[H + my * 8:H + my * 8 + 8, mx * 16:mx * 16 + 16]))
