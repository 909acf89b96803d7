"""Interleaved GOP groups: the GOPs of a window split into
G groups whose level launches run on G HIP streams.  The schedule changes
only which launch (and stream) reconstructs a frame, never what it computes,
so every group count must give the oracle's frames, scores, histograms, SADs
and RGB thumbnails bit for bit — short and long GOPs (groups with different
level counts), k = 4 (h264_recon_score<4>) and k = 6 with a cropped bottom
row (h264_recon_score6b).  The count is read from VTS_RECON_GROUPS at open.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import scene

pytestmark = pytest.mark.gpu


def _require_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")


@pytest.mark.parametrize("groups", [1, 2, 3, 4])
@pytest.mark.parametrize("k,W,H", [(4, 320, 240), (6, 480, 270)])
def test_group_counts_equal_oracle(tmp_path, monkeypatch, groups, k, W, H):
    _require_gpu()
    n = 120
    path = tmp_path / "g.mp4"
    # uneven GOPs: cuts every 0.3-1.2 s, at most 0.9 s per GOP -> 5..27 levels
    scene.synth_write(path, width=W, height=H, n_frames=n, max_motion=4, odd_motion=True,
                      cut_min_s=0.3, cut_max_s=1.2, gop_max_s=0.9)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, k)
    monkeypatch.setenv("VTS_RECON_GROUPS", str(groups))
    with scene.VideoScorer(path, k=k) as v:
        assert v.fused()
        res = v.score()
        res2 = v.score()  # a second run over the same schedule (command epochs)
        for i in range(n):
            assert np.array_equal(v.frame_nv12(i).reshape(frames[i].shape), frames[i]), i
        rgb = np.stack([v.thumbnail_rgb(i, k) for i in range(n)]).reshape(-1)
    for r in (res, res2):
        assert np.array_equal(r.hist, ref["hist"])
        assert np.array_equal(r.sad, ref["sad"])
        assert np.array_equal(r.scores, ref["score"])
    assert np.array_equal(rgb, ref["rgb"])
