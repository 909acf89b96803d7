"""Level-blocked reconstruction (h264_recon_score_tb) vs the C
oracle.

The kernel decodes L consecutive GOP levels of a macroblock row per
workgroup, keeping the levels between the first and the last in LDS.  Its
scores, histograms, SADs and RGB thumbnails must equal the oracle's bit for
bit whatever the block depth; the frames it keeps in HBM (each block's last
level) must equal the oracle's frames; the frames it does not keep must fail
loudly when asked for; motion beyond the one-group halo per level must fall
back to per-level launches with identical results.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import VtsegError, scene

pytestmark = pytest.mark.gpu


def _require_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")


def _tb_launches(v) -> int:
    return int(v._lib.vts_schedule_info(v._ctx, 5))


def _check(res, rgb, ref):
    assert np.array_equal(rgb, ref["rgb"])
    assert np.array_equal(res.hist, ref["hist"])
    assert np.array_equal(res.sad, ref["sad"])
    assert np.array_equal(res.scores, ref["score"])


def _stream(tmp_path, name, n, **kw):
    path = tmp_path / f"{name}.mp4"
    scene.synth_write(path, n_frames=n, **kw)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, kw["width"], kw["height"],
                              kw["width"], kw["height"], 4, want_rgb=True)
    return path, frames, ref


@pytest.mark.parametrize("level_block", [2, 3, 4, 5, 8])
def test_block_depths_equal_oracle(tmp_path, level_block):
    """Every block depth (short and long GOPs, chains ending inside a block,
    half-pel chroma from LDS rows, edge clamping) gives the oracle's results;
    kept frames equal the oracle's frames."""
    _require_gpu()
    n = 150
    path, frames, ref = _stream(tmp_path, "d", n, width=320, height=240, max_motion=4,
                                odd_motion=True, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=0.9,
                                slices_per_row=2)
    with scene.VideoScorer(path, level_block=level_block) as v:
        res = v.score()
        assert _tb_launches(v) > 0
        rgb = np.stack([v.thumbnail_rgb(i) for i in range(n)]).reshape(-1)
        kept = 0
        for i in range(n):
            try:
                got = v.frame_nv12(i)
            except VtsegError as e:
                assert "LDS only" in str(e)
                continue
            kept += 1
            assert np.array_equal(got.reshape(frames[i].shape), frames[i]), i
        assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])
    _check(res, rgb, ref)
    assert 0 < kept < n


def test_keep_frames_stores_every_level(tmp_path):
    _require_gpu()
    n = 90
    path, frames, ref = _stream(tmp_path, "k", n, width=256, height=144, max_motion=4,
                                cut_min_s=0.6, cut_max_s=1.2, gop_max_s=0.8)
    with scene.VideoScorer(path, level_block=4, keep_frames=True) as v:
        res = v.score()
        assert _tb_launches(v) > 0
        for i in range(n):
            assert np.array_equal(v.frame_nv12(i).reshape(frames[i].shape), frames[i]), i
        rgb = np.stack([v.thumbnail_rgb(i) for i in range(n)]).reshape(-1)
    _check(res, rgb, ref)


@pytest.mark.parametrize("motion", [8, 24])
def test_motion_beyond_halo_falls_back(tmp_path, motion):
    """Vertical motion beyond 4 rows per level: the launch flags it and the
    host re-runs the video with one launch per level; same results."""
    _require_gpu()
    n = 90
    path, frames, ref = _stream(tmp_path, "m", n, width=320, height=240, max_motion=motion,
                                cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.8)
    with scene.VideoScorer(path, level_block=4) as v:
        assert _tb_launches(v) > 0
        res = v.score()
        if motion > 16:  # pans of more than 4 rows per frame certainly occur
            assert _tb_launches(v) == 0  # fell back
        keep_all = _tb_launches(v) == 0
        rgb = np.stack([v.thumbnail_rgb(i) for i in range(n)]).reshape(-1)
        for i in range(n if keep_all else 0):  # the per-level schedule stores every frame
            assert np.array_equal(v.frame_nv12(i).reshape(frames[i].shape), frames[i]), i
    _check(res, rgb, ref)


def test_level_blocked_windows_and_repeat(tmp_path):
    """Small windows over two rings (chains restart at each window) and a
    second run on the same session."""
    _require_gpu()
    n = 400
    path, frames, ref = _stream(tmp_path, "w", n, width=480, height=272, max_motion=2,
                                cut_min_s=1, cut_max_s=4, gop_max_s=0.5)
    with scene.VideoScorer(path, window_frames=40, n_streams=2, level_block=4) as v:
        a = v.score()
        assert _tb_launches(v) > 0
        v.run()
        b = v.score()
    for r in (a, b):
        assert np.array_equal(r.hist, ref["hist"])
        assert np.array_equal(r.sad, ref["sad"])
        assert np.array_equal(r.scores, ref["score"])


def test_hd720_level_blocked(tmp_path):
    """The benchmark's shape (1280x720, motion <= 4): level-blocked launches
    equal the oracle; the default (auto) schedule stays per-level."""
    _require_gpu()
    n = 70
    path, frames, ref = _stream(tmp_path, "hd", n, width=1280, height=720, max_motion=4,
                                cut_min_s=0.5, cut_max_s=1.5, gop_max_s=1.0)
    with scene.VideoScorer(path) as v:
        assert _tb_launches(v) == 0
    with scene.VideoScorer(path, level_block=4) as v:
        res = v.score()
        assert _tb_launches(v) > 0
        rgb = np.stack([v.thumbnail_rgb(i) for i in range(n)]).reshape(-1)
    _check(res, rgb, ref)
