"""Debug: the tiny general-decoder stream through h264_recon_sched (kernel
printf variant), checked against the oracle.  python rs_tiny.py OUT.mp4"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "video-transformer_amd"))
import numpy as np
import oracle
from vtseg import scene
path = sys.argv[1]
n = int(os.environ.get("N", "48"))
kw = dict(width=int(os.environ.get("W", "48")), height=int(os.environ.get("H", "32")), max_motion=2)
scene.synth_write(path, n_frames=n, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7, coding="full", seed=31, **kw)
frames, _ = oracle.decode_full(path)
print("oracle done", flush=True)
with scene.VideoScorer(path, keep_frames=True, k=4) as v:
    assert v.general()
    res = v.score()
    got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
    bad = np.nonzero((got != frames).reshape(n, -1).any(1))[0]
    print("bad frames", bad[:10].tolist(), flush=True)
