"""CABAC windows whose longest slices (x264's intra pictures) parse in a
launch of their own, beside the others and the derivation of every picture
that needs none of them (session_full.hip, Window::plong / dlv_early).  The
split changes only when work runs: every frame, histogram, SAD and score must
equal the oracle's with the split forced onto the longest eighth of each
window's slices (VTS_PARSE_SPLIT=2: B pictures whose colocated picture is
early and late both occur), chosen by size (default) and off (0); one window
and several on two rings."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import scene

pytestmark = pytest.mark.gpu

STREAMS = [
    ("content_qvga", dict(width=320, height=240, content=True), 90),
    ("cabac_b_temporal", dict(width=176, height=144, temporal_direct=True), 60),
    ("cabac_b_spatial_slices", dict(width=176, height=144, slices_per_row=2), 60),
]


@pytest.mark.parametrize("mode", ["2", "1", "0"], ids=["forced", "by_size", "off"])
@pytest.mark.parametrize("name,kw,n", STREAMS, ids=[s[0] for s in STREAMS])
def test_split_parse_equals_the_oracle(tmp_path, monkeypatch, name, kw, n, mode):
    import torch
    assert torch.cuda.is_available()
    kw = dict(kw)
    path = tmp_path / f"{name}.mp4"
    if kw.pop("content", False):
        scene.synth_write(path, n_frames=n, coding="full", max_motion=4, bframes=True, weighted="implicit",
                          cabac=True, transform_8x8=True, content=True, cut_min_s=0.5, cut_max_s=1.5,
                          gop_max_s=1.0, seed=41, **kw)
    else:
        src = tmp_path / "src.mp4"
        scene.synth_write(src, n_frames=n, coding="full", bframes=True, weighted="implicit", cut_min_s=0.5,
                          cut_max_s=1.2, gop_max_s=0.8, seed=3, chunks=1, **kw)
        oracle.cabac_convert(src, path, seed=5, t8=True)
    frames, _ = oracle.decode_full(path)
    W, H = frames.shape[2], frames.shape[1] * 2 // 3
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
    monkeypatch.setenv("VTS_PARSE_SPLIT", mode)
    for wf in (0, n // 3):
        with scene.VideoScorer(path, keep_frames=wf == 0, window_frames=wf) as v:
            assert v.general()
            split = v._lib.vts_schedule_info(v._ctx, 13)
            if mode == "2":
                assert split > 0
            if mode == "0":
                assert split == 0
            res = v.score()
            if wf == 0:
                got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
                bad = np.nonzero((got != frames).reshape(n, -1).any(1))[0]
                assert bad.tolist() == []
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])
