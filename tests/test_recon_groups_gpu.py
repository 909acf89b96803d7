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


@pytest.mark.parametrize("group_parse", ["0", "1"])
@pytest.mark.parametrize("k,W,H", [(4, 320, 240), (6, 480, 270)])
def test_groups_over_pipelined_windows(tmp_path, monkeypatch, group_parse, k, W, H):
    """Two groups, per-group parse chunks on or off, many small windows over
    two rings: a group's stream must not add to a window's histograms / SADs
    before clear_accum (on the decode stream) has zeroed them."""
    _require_gpu()
    n = 240
    path = tmp_path / "w.mp4"
    scene.synth_write(path, width=W, height=H, n_frames=n, max_motion=4, cut_min_s=0.4,
                      cut_max_s=1.5, gop_max_s=0.3)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, k)
    monkeypatch.setenv("VTS_RECON_GROUPS", "2")
    monkeypatch.setenv("VTS_GROUP_PARSE", group_parse)
    with scene.VideoScorer(path, k=k, window_frames=40, n_streams=2) as v:
        assert v._lib.vts_schedule_info(v._ctx, 1) > 4  # several windows
        for _ in range(3):
            res = v.score()
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])


@pytest.mark.parametrize("window", [0, 24])
def test_nonreference_i_pictures_keep_groups_and_windows_correct(tmp_path, monkeypatch, window):
    """Refresh pictures written as non-reference I pictures: the next P
    picture predicts from the reference before the I picture.  Windows and
    interleaved groups may start only where no later picture predicts
    across, so the schedule stays correct (and deterministic)."""
    _require_gpu()
    n = 150
    path = tmp_path / "nr.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=n, max_motion=4, cut_min_s=2,
                      cut_max_s=3, gop_max_s=0.3, nonref_refresh=True)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 320, 240, 320, 240, 4)
    monkeypatch.setenv("VTS_RECON_GROUPS", "2")
    with scene.VideoScorer(path, window_frames=window) as v:
        for _ in range(2):
            res = v.score()
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])
