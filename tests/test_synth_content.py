"""The content mode of the full-syntax writer (synth_content.h; VERDICT r03
"make the full-syntax bench stream look like video").  CPU only.

The writer codes textured moving scenes in closed loop: it reconstructs
every macroblock as a decoder does (including the deblocking filter) and
hashes its reconstruction (vts_synth_info.recon_hash).  That hash must equal
the hash of the independent C oracle's decode (oracle/h264_full_oracle.c
fo_decode) of the stream it wrote: the writer's mode decisions, quantisation
and CABAC syntax, and the oracle's decoding, agree picture for picture.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import scene

X264ISH = dict(coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit",
               cabac=True, transform_8x8=True, content=True)


@pytest.mark.parametrize("w,h,n,seed,kw", [
    (320, 240, 72, 7, {}),
    (320, 180, 60, 3, {}),                           # cropped bottom rows
    (176, 144, 60, 11, dict(transform_8x8=False)),   # CABAC Main profile
    (176, 144, 48, 5, dict(cabac=False, transform_8x8=False, weighted=None)),  # CAVLC, default bi-pred
    (352, 288, 40, 13, dict(slices_per_row=2)),      # two slices per row
])
def test_writer_reconstruction_equals_the_oracle_decode(tmp_path, w, h, n, seed, kw):
    path = tmp_path / "c.mp4"
    args = dict(X264ISH, **kw)
    info = scene.synth_write(path, width=w, height=h, fps=30, n_frames=n, seed=seed, cut_min_s=0.6,
                             cut_max_s=1.5, gop_max_s=1.2, hash_frames=True, **args)
    frames, _ = oracle.decode_full(path)
    assert frames.shape[0] == n
    assert info["recon_hash"] == oracle.recon_hash(frames)
    assert info["n_cuts"] >= 1


def test_content_stream_looks_like_video(tmp_path):
    """Consecutive pictures differ little except at the planted cuts, where
    the luma histogram changes; the rate is far below the noise stream's."""
    n, w, h = 150, 320, 240
    path, noise = tmp_path / "c.mp4", tmp_path / "n.mp4"
    info = scene.synth_write(path, width=w, height=h, fps=30, n_frames=n, seed=9, cut_min_s=1.0,
                             cut_max_s=2.0, gop_max_s=8.0, **X264ISH)
    ninfo = scene.synth_write(noise, width=w, height=h, fps=30, n_frames=n, seed=9, cut_min_s=1.0,
                              cut_max_s=2.0, gop_max_s=8.0, **dict(X264ISH, content=False))
    assert info["bytes"] * 2 < ninfo["bytes"]
    frames, _ = oracle.decode_full(path)
    y = frames[:, :h].astype(np.int32)
    diff = np.abs(y[1:] - y[:-1]).mean(axis=(1, 2))
    cuts = set(info["cuts"])
    assert cuts
    at_cut = [diff[c - 1] for c in cuts]
    within = [diff[i - 1] for i in range(1, n) if i not in cuts]
    assert min(at_cut) > 2 * np.percentile(within, 90)
    # the scorer (oracle restatement) finds exactly the planted cuts
    r = oracle.score_frames(frames.reshape(-1), frames[0].size, n, w, h, w, h, 4)
    assert np.nonzero(r["score"] > scene.DEFAULT_CUT_THRESHOLD)[0].tolist() == sorted(cuts)


def test_content_mode_argument_checks(tmp_path):
    with pytest.raises(ValueError):
        scene.synth_write(tmp_path / "x.mp4", n_frames=4, coding="full", content=True)
    with pytest.raises(Exception):
        scene.synth_write(tmp_path / "y.mp4", width=64, height=64, n_frames=4, coding="full", bframes=True,
                          weighted="explicit", content=True)
