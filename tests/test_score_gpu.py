"""Score kernel (vts_score_nv12_dev, HIP/gfx950) vs the scalar C oracle.

Bit-exact on every output: RGB thumbnails, 256-bin histograms, SAD (uint64)
and the fp32 score (north_star tolerance is |d| <= 1e-4; integer accumulation
makes it exact, and the test asserts exact equality).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X (torch.cuda.is_available() is False)")
    return torch


def smooth_nv12(rng, n, width, height, pitch, rows_total, uv_row_offset):
    """Frames of smooth random content + noise, with pitch/crop padding filled
    with garbage so out-of-window reads would show up."""
    stride = pitch * rows_total
    stride = (stride + 15) // 16 * 16
    buf = rng.integers(0, 256, size=n * stride, dtype=np.uint8)
    for f in range(n):
        base = f * stride
        gy = rng.integers(0, 256, size=(height // 16 + 2, width // 16 + 2)).astype(np.float32)
        yy = np.kron(gy, np.ones((16, 16), np.float32))[:height, :width]
        yy = np.clip(yy + rng.normal(0, 6, size=yy.shape), 0, 255).astype(np.uint8)
        plane = buf[base: base + pitch * height].reshape(height, pitch)
        plane[:, :width] = yy
        uv = buf[base + pitch * uv_row_offset: base + pitch * (uv_row_offset + height // 2)]
        uv = uv.reshape(height // 2, pitch)
        uv[:, :width] = rng.integers(0, 256, size=(height // 2, width), dtype=np.uint8)
    return buf, stride


CASES = [
    # width, height, pitch, coded rows (uv offset), k, n_frames
    (640, 480, 640, 480, 4, 37),
    (1280, 720, 1280, 720, 4, 9),
    (1920, 1080, 2048, 1088, 6, 5),
    (320, 240, 384, 256, 2, 7),
    (320, 240, 320, 240, 8, 6),
    (160, 96, 160, 96, 4, 1100),  # > 512 frames: multi-frame runs + seam kernel
]


@pytest.mark.parametrize("width,height,pitch,coded,k,n", CASES)
def test_score_kernel_bit_exact_vs_oracle(width, height, pitch, coded, k, n):
    torch = _torch()
    from vtseg import scene
    rng = np.random.default_rng(1234 + width + k)
    host, stride = smooth_nv12(rng, n, width, height, pitch, coded + height // 2, coded)
    dev = torch.from_numpy(host).cuda()
    out = scene.score_nv12(dev, width=width, height=height, pitch=pitch, uv_row_offset=coded,
                           frame_stride=stride, n_frames=n, k=k)
    torch.cuda.synchronize()
    ref = oracle.score_frames(host, stride, n, width, height, pitch, coded, k)
    w, h = width // k, height // k
    assert np.array_equal(out["rgb"].cpu().numpy().reshape(-1), ref["rgb"])
    assert np.array_equal(out["hist"].cpu().numpy().view(np.uint32), ref["hist"])
    assert np.array_equal(out["sad"].cpu().numpy().view(np.uint64), ref["sad"])
    assert np.array_equal(out["score"].cpu().numpy(), ref["score"])
    assert np.array_equal(out["last_luma"].cpu().numpy(), ref["last_luma"])
    assert int(out["hist"].sum()) == n * w * h


def test_score_kernel_prev_luma_continuity():
    """Scoring a batch in two halves with prev_luma = first half's last_luma
    equals scoring it whole (the streaming window contract)."""
    torch = _torch()
    from vtseg import scene
    rng = np.random.default_rng(7)
    width, height, k, n = 640, 360, 4, 600
    host, stride = smooth_nv12(rng, n, width, height, width, height + height // 2, height)
    dev = torch.from_numpy(host).cuda()
    kw = dict(width=width, height=height, pitch=width, uv_row_offset=height,
              frame_stride=stride, k=k, want_rgb=False)
    whole = scene.score_nv12(dev, n_frames=n, **kw)
    a = scene.score_nv12(dev[: 250 * stride], n_frames=250, **kw)
    b = scene.score_nv12(dev[250 * stride:], n_frames=n - 250, prev_luma=a["last_luma"], **kw)
    torch.cuda.synchronize()
    joined = torch.cat([a["sad"], b["sad"]]).cpu().numpy()
    assert np.array_equal(joined, whole["sad"].cpu().numpy())
    assert np.array_equal(torch.cat([a["hist"], b["hist"]]).cpu().numpy(),
                          whole["hist"].cpu().numpy())


def test_score_kernel_rejects_bad_geometry():
    torch = _torch()
    from vtseg import VtsegError, scene
    dev = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    with pytest.raises(VtsegError):
        scene.score_nv12(dev, width=100, height=64, pitch=128, uv_row_offset=64,
                         frame_stride=128 * 96, n_frames=1, k=4)  # width % 16 != 0
    with pytest.raises(VtsegError):
        scene.score_nv12(dev, width=128, height=64, pitch=128, uv_row_offset=64,
                         frame_stride=128 * 96, n_frames=1, k=3)
