"""Dump score-kernel outputs for offline comparison with the oracle."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "oracle"), str(ROOT / "video-transformer_amd")]
import torch  # noqa: E402

from test_score_gpu import smooth_nv12  # noqa: E402
from vtseg import scene  # noqa: E402

out_dir = ROOT / "gpurun_out"
out_dir.mkdir(exist_ok=True)
for (W, H, P, coded, k, n) in [(640, 480, 640, 480, 4, 37), (160, 96, 160, 96, 4, 1100)]:
    rng = np.random.default_rng(1234 + W + k)
    host, stride = smooth_nv12(rng, n, W, H, P, coded + H // 2, coded)
    dev = torch.from_numpy(host).cuda()
    o = scene.score_nv12(dev, width=W, height=H, pitch=P, uv_row_offset=coded,
                         frame_stride=stride, n_frames=n, k=k)
    torch.cuda.synchronize()
    np.savez_compressed(out_dir / f"score_diag_{W}x{H}_{n}.npz",
                        rgb=o["rgb"].cpu().numpy(), hist=o["hist"].cpu().numpy(),
                        sad=o["sad"].cpu().numpy(), score=o["score"].cpu().numpy(),
                        last=o["last_luma"].cpu().numpy())
print("dumped")
