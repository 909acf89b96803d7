"""Compare every score-kernel output with the oracle per case; print a summary
and dump mismatching cases for offline analysis (no asserts)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "oracle"), str(ROOT / "video-transformer_amd")]
import torch  # noqa: E402

import oracle  # noqa: E402
from test_score_gpu import CASES, smooth_nv12  # noqa: E402
from vtseg import scene  # noqa: E402

out_dir = ROOT / "gpurun_out"
out_dir.mkdir(exist_ok=True)
for (W, H, P, coded, k, n) in CASES:
    rng = np.random.default_rng(1234 + W + k)
    host, stride = smooth_nv12(rng, n, W, H, P, coded + H // 2, coded)
    dev = torch.from_numpy(host).cuda()
    o = scene.score_nv12(dev, width=W, height=H, pitch=P, uv_row_offset=coded,
                         frame_stride=stride, n_frames=n, k=k)
    torch.cuda.synchronize()
    ref = oracle.score_frames(host, stride, n, W, H, P, coded, k)
    g = {"rgb": o["rgb"].cpu().numpy().reshape(-1), "hist": o["hist"].cpu().numpy().view(np.uint32),
         "sad": o["sad"].cpu().numpy().view(np.uint64), "score": o["score"].cpu().numpy(),
         "last_luma": o["last_luma"].cpu().numpy()}
    res = {key: bool(np.array_equal(g[key], ref[key])) for key in g}
    print(W, H, k, n, res, flush=True)
    if not all(res.values()):
        np.savez_compressed(out_dir / f"diag_{W}x{H}_k{k}.npz", **{"gpu_" + a: b for a, b in g.items()})
