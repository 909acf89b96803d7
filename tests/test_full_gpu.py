"""General device decoder (decode_full.hip) vs the oracle (h264_full_oracle.c).

Full-syntax streams (coding="full": intra 4x4 / 16x16 / chroma modes,
residual blocks, quarter-sample partitions over up to 3 references, list
modification, non-reference pictures, QP changes, the deblocking filter with
idc 0/1/2 and offsets): every decoded frame, histogram, SAD, score and RGB
thumbnail must equal the oracle's bit for bit.  The subset streams must also
decode identically on the general path (decoder="general").  Parity of the
pictures themselves against a third-party decoder is unpinned (none in the
image); the product's decoding code is the same as the CPU harness checked in
tests/test_full_host.py.
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


def _first_diff(a, b):
    bad = np.nonzero((a != b).reshape(a.shape[0], -1).any(1))[0]
    return bad[:8].tolist()


def _recycled_equal(path, ref, k=4):
    """The same stream opened without keep_frames: decoded surfaces recycled
    (thumb_pics per level launch, thumb_sad per window), so only the scoring
    outputs can be compared, and they must equal the oracle's."""
    with scene.VideoScorer(path, k=k) as v:
        assert v.general() and v._lib.vts_schedule_info(v._ctx, 11) > 0
        res = v.score()
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        n = res.scores.shape[0]
        rgb = np.stack([v.thumbnail_rgb(i, k) for i in range(n)]).reshape(-1)
        assert np.array_equal(rgb, ref["rgb"])


FULL = [
    ("tiny", dict(width=48, height=32, max_motion=2)),
    ("qvga", dict(width=320, height=240, max_motion=3)),
    ("ragged", dict(width=336, height=200, slices_per_row=3, max_motion=6)),
    ("oneslice", dict(width=320, height=240, slices_per_row=0, max_motion=8)),
    ("cip", dict(width=320, height=240, max_motion=3, constrained_intra=True)),
    ("crop", dict(width=480, height=270, slices_per_row=2, max_motion=4)),
    ("hd720", dict(width=1280, height=720, slices_per_row=0, max_motion=6)),
]


@pytest.mark.parametrize("name,kw", FULL, ids=[f[0] for f in FULL])
def test_general_decoder_bit_exact(tmp_path, name, kw):
    _require_gpu()
    n = 24 if kw["height"] >= 720 else 48
    path = tmp_path / f"{name}.mp4"
    scene.synth_write(path, n_frames=n, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7,
                      coding="full", seed=31, **kw)
    frames, _ = oracle.decode_full(path)
    W, H = kw["width"], kw["height"]
    k = 4 if H <= 720 and H % 4 == 0 else 6
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, k)
    with scene.VideoScorer(path, keep_frames=True, k=k) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        rgb = np.stack([v.thumbnail_rgb(i, k) for i in range(n)]).reshape(-1)
        assert np.array_equal(rgb, ref["rgb"])
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        res2 = v.score()   # a second run over the same rings (record epochs)
        assert np.array_equal(res2.scores, res.scores)
    _recycled_equal(path, ref, k)


def test_general_decoder_windows_and_rings(tmp_path):
    """Many small windows on two rings / two streams equal one window."""
    _require_gpu()
    n = 150
    path = tmp_path / "w.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=n, cut_min_s=0.5, cut_max_s=1.5,
                      gop_max_s=0.5, coding="full", seed=5)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 320, 240, 320, 240, 4)
    with scene.VideoScorer(path, window_frames=30, n_streams=2, keep_frames=True) as v:
        assert v.general() and v.windows() >= 4
        res = v.score()
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])


@pytest.mark.parametrize("kw", [dict(width=320, height=240, max_motion=4),
                                dict(width=336, height=200, slices_per_row=3, max_motion=6,
                                     odd_motion=True),
                                dict(width=160, height=96, max_motion=4, gop_max_s=0.3,
                                     nonref_refresh=True)])
def test_subset_streams_on_the_general_path(tmp_path, kw):
    _require_gpu()
    kw = dict(kw)
    gop = kw.pop("gop_max_s", 0.8)
    path = tmp_path / "s.mp4"
    scene.synth_write(path, n_frames=60, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=gop, **kw)
    with scene.VideoScorer(path) as a:
        assert not a.general()
        want = a.score()
    with scene.VideoScorer(path, decoder="general", keep_frames=True) as b:
        assert b.general()
        got = b.score()
        frames, _ = oracle.decode_full(path)
        assert np.array_equal(b.frame_nv12(59).reshape(frames[-1].shape), frames[-1])
    assert np.array_equal(got.hist, want.hist)
    assert np.array_equal(got.sad, want.sad)
    assert np.array_equal(got.scores, want.scores)


def test_subset_only_decoder_refuses_full_syntax(tmp_path):
    _require_gpu()
    path = tmp_path / "f.mp4"
    scene.synth_write(path, width=64, height=48, n_frames=10, coding="full")
    with scene.VideoScorer(path, decoder="subset") as v:
        with pytest.raises(VtsegError):
            v.score()


def test_real_cabac_high_profile_stream():
    """A real High-profile CABAC clip (tests/golden/real/realshort.mp4: CABAC
    I/P slices, 8x8 transform, Intra 8x8/4x4/16x16, deblocking) decodes and
    scores on the device bit for bit like the oracle (auto-selected general
    decoder)."""
    _require_gpu()
    from pathlib import Path
    path = Path(__file__).resolve().parent / "golden" / "real" / "realshort.mp4"
    frames, _ = oracle.decode_full(path)
    n = frames.shape[0]
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 320, 240, 320, 240, 4)
    with scene.VideoScorer(path, keep_frames=True) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])


def test_real_cabac_subset_decoder_refuses():
    _require_gpu()
    from pathlib import Path
    path = Path(__file__).resolve().parent / "golden" / "real" / "realshort.mp4"
    with pytest.raises(VtsegError):
        with scene.VideoScorer(path, decoder="subset") as v:
            v.score()


B_STREAMS = [
    ("spatial", dict(width=176, height=144)),
    ("explicit", dict(width=176, height=144, weighted="explicit")),
    ("implicit", dict(width=176, height=144, weighted="implicit")),
    ("temporal", dict(width=176, height=144, temporal_direct=True)),
    ("slices", dict(width=176, height=144, slices_per_row=2, weighted="implicit", temporal_direct=True)),
    ("hd720", dict(width=1280, height=720, slices_per_row=0, weighted="explicit", temporal_direct=True)),
    ("fhd_crop", dict(width=1920, height=1080, slices_per_row=0, weighted="implicit")),
]


@pytest.mark.parametrize("name,kw", B_STREAMS, ids=[b[0] for b in B_STREAMS])
def test_b_pictures_bit_exact(tmp_path, name, kw):
    """Main-profile B streams (reordered mini-GOPs with B reference pictures,
    spatial / temporal direct, every B partition shape, explicit / implicit
    weighted prediction, explicitly weighted P slices): frames in presentation
    order, thumbnails, histograms, SADs and scores equal the oracle; the
    parse runs B pictures one launch after their colocated pictures."""
    _require_gpu()
    n = 16 if kw["height"] > 720 else (30 if kw["height"] >= 720 else 45)
    path = tmp_path / f"b_{name}.mp4"
    scene.synth_write(path, n_frames=n, coding="full", bframes=True, cut_min_s=0.5, cut_max_s=1.2,
                      gop_max_s=0.8, seed=11, chunks=1, **kw)
    frames, _ = oracle.decode_full(path)
    W, H = kw["width"], kw["height"]
    k = 4 if H <= 720 else 6
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, k)
    with scene.VideoScorer(path, keep_frames=True, k=k) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        rgb = np.stack([v.thumbnail_rgb(i, k) for i in range(n)]).reshape(-1)
        assert np.array_equal(rgb, ref["rgb"])
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
    _recycled_equal(path, ref, k)


def test_b_pictures_windows_and_rings(tmp_path):
    """A B stream in many windows (closed mini-GOP runs: the same frames in
    decode and presentation order) on two rings equals the oracle."""
    _require_gpu()
    n = 120
    path = tmp_path / "bw.mp4"
    scene.synth_write(path, width=160, height=96, n_frames=n, coding="full", bframes=True,
                      weighted="explicit", chunks=4, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=0.6, seed=9)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 160, 96, 160, 96, 4)
    with scene.VideoScorer(path, window_frames=30, n_streams=2, keep_frames=True) as v:
        assert v.general() and v.windows() >= 3
        res = v.score()
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])


def test_b_stream_refused_by_the_subset_decoder(tmp_path):
    _require_gpu()
    path = tmp_path / "b.mp4"
    scene.synth_write(path, width=64, height=48, n_frames=20, coding="full", bframes=True)
    with pytest.raises(VtsegError):
        with scene.VideoScorer(path, decoder="subset") as v:
            v.score()


CABAC_B = [
    ("p_t8", dict(width=176, height=144), True),
    ("b_spatial", dict(width=176, height=144, bframes=True), False),
    ("b_explicit_t8", dict(width=176, height=144, bframes=True, weighted="explicit"), True),
    ("b_temporal_implicit", dict(width=176, height=144, bframes=True, temporal_direct=True, weighted="implicit"), False),
    ("b_slices_t8", dict(width=176, height=144, bframes=True, slices_per_row=2), True),
    ("b_hd720_t8", dict(width=1280, height=720, bframes=True, slices_per_row=0, weighted="explicit"), True),
]


@pytest.mark.parametrize("name,kw,t8", CABAC_B, ids=[c[0] for c in CABAC_B])
def test_cabac_b_streams_bit_exact(tmp_path, name, kw, t8):
    """CABAC P / B streams (oracle.cabac_convert: the writer's headers with a
    synthesised CABAC macroblock layer covering every B mb_type /
    sub_mb_type, both lists' contexts, direct quadrants and 8x8 transforms)
    decode and score on the device exactly like the oracle."""
    _require_gpu()
    n = 16 if kw["height"] >= 720 else 30
    src, path = tmp_path / "src.mp4", tmp_path / f"{name}.mp4"
    scene.synth_write(src, n_frames=n, coding="full", cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.8, seed=3,
                      chunks=1, **kw)
    oracle.cabac_convert(src, path, seed=5, t8=t8)
    frames, _ = oracle.decode_full(path)
    W, H = kw["width"], kw["height"]
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
    with scene.VideoScorer(path, keep_frames=True) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
    _recycled_equal(path, ref)


@pytest.mark.parametrize("groups", [1, 2, 3, 4])
@pytest.mark.parametrize("bframes", [False, True], ids=["ip", "b"])
def test_gop_groups_on_streams_equal_the_oracle(tmp_path, monkeypatch, groups, bframes):
    """The window's GOPs dealt to 1-4 groups that reconstruct on their own
    streams (VTS_GENERAL_GROUPS): every frame, histogram, SAD and score still
    equals the oracle, in one window and in several windows on two rings."""
    _require_gpu()
    monkeypatch.setenv("VTS_GENERAL_GROUPS", str(groups))
    n = 120
    path = tmp_path / "g.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=bframes,
                      weighted="implicit" if bframes else None, cut_min_s=0.5, cut_max_s=1.5,
                      gop_max_s=0.4, seed=17)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    for wf in (0, 60):
        with scene.VideoScorer(path, keep_frames=wf == 0, window_frames=wf, n_streams=2) as v:
            assert v.general()
            res = v.score()
            if wf == 0:
                got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
                assert _first_diff(got, frames) == []
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])


@pytest.mark.parametrize("groups", [1, 2])
def test_recycled_surfaces_equal_the_oracle(tmp_path, monkeypatch, groups):
    """Without keep_frames the general decoder recycles decoded-picture
    surfaces: a per-GOP-group liveness plan maps window slots to surfaces,
    each level launch is thumbnailed right after it and the window's SADs
    come from the thumbnail ring.  Histograms, SADs, scores and RGB
    thumbnails equal the oracle in one window and in several windows on two
    rings, on a second run too; the session holds fewer surfaces than window
    frames and refuses to hand a frame back."""
    _require_gpu()
    monkeypatch.setenv("VTS_GENERAL_GROUPS", str(groups))
    n = 240
    path = tmp_path / "pool.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=n, coding="full", bframes=True, weighted="implicit",
                      cabac=True, transform_8x8=True, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=0.5, seed=41)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 320, 240, 320, 240, 4)
    for wf in (0, 80):
        with scene.VideoScorer(path, window_frames=wf, n_streams=2) as v:
            assert v.general()
            surfs = v._lib.vts_schedule_info(v._ctx, 11)
            ring = v._lib.vts_schedule_info(v._ctx, 3)
            assert 0 < surfs < ring, (surfs, ring)
            for _ in range(2):
                res = v.score()
                assert np.array_equal(res.hist, ref["hist"])
                assert np.array_equal(res.sad, ref["sad"])
                assert np.array_equal(res.scores, ref["score"])
            rgb = np.stack([v.thumbnail_rgb(i, 4) for i in range(n)]).reshape(-1)
            assert np.array_equal(rgb, ref["rgb"])
            with pytest.raises(VtsegError, match="not kept"):
                v.frame_nv12(n - 1)
    monkeypatch.setenv("VTS_SURF_POOL", "0")  # the knob: one surface per window slot again
    with scene.VideoScorer(path, window_frames=80, n_streams=2) as v:
        assert v._lib.vts_schedule_info(v._ctx, 11) == 0
        res = v.score()
        assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])


@pytest.mark.parametrize("groups", [1, 2])
def test_paced_bs_equals_the_oracle(tmp_path, monkeypatch, groups):
    """The deblocking descriptors are derived one level launch at a time on
    the score stream, paced by the reconstruction chain: every frame,
    histogram, SAD and score equals the oracle, with one and two GOP groups,
    in one window and in several windows (where the score stream also scores
    the window before)."""
    _require_gpu()
    monkeypatch.setenv("VTS_GENERAL_GROUPS", str(groups))
    n = 120
    path = tmp_path / "bs.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=True, weighted="implicit",
                      cabac=True, transform_8x8=True, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=0.4, seed=23)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    for wf in (0, 60):
        with scene.VideoScorer(path, keep_frames=wf == 0, window_frames=wf, n_streams=2) as v:
            assert v.general()
            res = v.score()
            if wf == 0:
                got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
                assert _first_diff(got, frames) == []
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])


def test_chroma_only_deblocking_goes_to_the_general_decoder(tmp_path):
    """A subset-syntax stream whose deblocking filter is active on chroma
    edges only (QPY 3, chroma_qp_index_offset 12, filter offsets +12: luma
    indexA <= 15, chroma indexA 24 on I_PCM edges) must not run on the subset kernels, which do not filter: auto mode
    picks the general decoder and matches the general oracle; subset-only
    mode refuses it (8.7.2.2: an edge filters where indexA >= 16)."""
    _require_gpu()
    path = tmp_path / "cdbk.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=40, cut_min_s=0.5, cut_max_s=1.2,
                      gop_max_s=0.6, seed=77, chroma_deblock=True)
    frames, _ = oracle.decode_full(path)
    unfiltered, _ = oracle.decode_full(path, flags=1)
    assert not np.array_equal(frames, unfiltered)   # the filter changes chroma
    H = 240
    assert np.array_equal(frames[:, :H], unfiltered[:, :H])  # and only chroma
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, 40, 320, 240, 320, 240, 4)
    with scene.VideoScorer(path, keep_frames=True) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(40)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.scores, ref["score"])
    with scene.VideoScorer(path, decoder="subset") as v:
        with pytest.raises(VtsegError):
            v.score()


def test_window_without_clean_picture_in_slot_range_is_refused(tmp_path, monkeypatch):
    """a window always extends to the next clean intra picture;
    when clean pictures are further apart than the int16 ring-slot range the
    open must fail cleanly (VTS_E_UNSUPPORTED) instead of wrapping slots.  The
    cap is lowered with VTS_WINDOW_SLOT_CAP so the stream stays small: one
    IDR, then 39 P pictures."""
    _require_gpu()
    path = tmp_path / "onegop.mp4"
    scene.synth_write(path, width=64, height=48, n_frames=40, cut_min_s=100, cut_max_s=100,
                      gop_max_s=100, coding="full", seed=3)
    monkeypatch.setenv("VTS_WINDOW_SLOT_CAP", "16")
    with pytest.raises(VtsegError, match="clean intra picture"):
        scene.VideoScorer(path, decoder="general")
    monkeypatch.setenv("VTS_WINDOW_SLOT_CAP", "40")
    frames, _ = oracle.decode_full(path)
    with scene.VideoScorer(path, decoder="general", keep_frames=True) as v:
        v.score()
        assert np.array_equal(v.frame_nv12(39).reshape(frames[-1].shape), frames[-1])


WRITER_CABAC = [
    ("ip_t8", dict(width=320, height=240, transform_8x8=True)),
    ("b_t8_implicit", dict(width=320, height=240, bframes=True, transform_8x8=True, weighted="implicit")),
    ("b_t8_explicit_temporal_rows", dict(width=336, height=200, bframes=True, transform_8x8=True,
                                         weighted="explicit", temporal_direct=True, slices_per_row=1)),
    ("hd720_x264like", dict(width=1280, height=720, bframes=True, transform_8x8=True, weighted="implicit")),
]


@pytest.mark.parametrize("name,kw", WRITER_CABAC, ids=[c[0] for c in WRITER_CABAC])
def test_writer_cabac_streams_bit_exact(tmp_path, name, kw):
    """The writer's own CABAC streams (synth_full.cpp, cabac=True; High
    profile with transform_8x8): x264's structure (CABAC, B pyramid, 8x8
    transform, weighted bi-prediction, one slice per picture) decoded and
    scored on the device equal the oracle frame for frame."""
    _require_gpu()
    kw = dict(kw)
    spr = kw.pop("slices_per_row", 0)
    n = 24 if kw["height"] >= 720 else 45
    path = tmp_path / f"{name}.mp4"
    scene.synth_write(path, n_frames=n, coding="full", cabac=True, slices_per_row=spr, cut_min_s=0.4,
                      cut_max_s=1.0, gop_max_s=0.6, seed=29, max_motion=4, **kw)
    frames, _ = oracle.decode_full(path)
    W, H = kw["width"], kw["height"]
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
    with scene.VideoScorer(path, keep_frames=True) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
    _recycled_equal(path, ref)


SCALING = [
    ("cavlc_sps", dict(scaling="sps")),
    ("cavlc_both_b", dict(scaling="both", bframes=True)),
    ("cabac_pps_t8", dict(scaling="pps", cabac=True, transform_8x8=True)),
    ("cabac_both_t8_b", dict(scaling="both", cabac=True, transform_8x8=True, bframes=True, weighted="implicit")),
    ("cabac_pps_no_t8", dict(scaling="pps", cabac=True)),
]


@pytest.mark.parametrize("name,kw", SCALING, ids=[s[0] for s in SCALING])
def test_scaling_matrix_streams_bit_exact(tmp_path, name, kw):
    """Scaling matrices (8.5.9, the writer's seeded SPS / PPS lists with the
    fall-back rules, defaults, early-ended and full lists): the device's
    LevelScale dequantisation (4x4 / 8x8, intra / inter, luma / chroma, the
    DC transforms) equals the oracle's on every frame, thumbnail, histogram,
    SAD and score."""
    _require_gpu()
    n, W, H = 30, 320, 240
    path = tmp_path / f"sc_{name}.mp4"
    scene.synth_write(path, width=W, height=H, n_frames=n, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7,
                      coding="full", slices_per_row=0, max_motion=4, seed=7, **kw)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
    with scene.VideoScorer(path, keep_frames=True, k=4) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
    _recycled_equal(path, ref)


@pytest.mark.parametrize("merge", ["0", "1"])
def test_cavlc_b_parse_merged_and_per_level(tmp_path, monkeypatch, merge):
    """the CAVLC parser's merged launch (default; B slices wait on
    their colocated picture's completion counter) and the per-level fallback
    (VTS_PARSE_MERGE=0: one launch per colocated level) both equal the oracle
    on a B stream with temporal direct in several windows.  (The CABAC parser
    has no such wait: h264_derive reads the colocated records, by parse
    level, test_cabac_temporal_direct_windows_and_arena_rerun.)"""
    _require_gpu()
    monkeypatch.setenv("VTS_PARSE_MERGE", merge)
    n = 60
    path = tmp_path / "mb.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=True,
                      temporal_direct=True, weighted="implicit", cut_min_s=0.5, cut_max_s=1.2,
                      gop_max_s=0.6, seed=21, chunks=1)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    for wf in (0, 24):
        with scene.VideoScorer(path, keep_frames=wf == 0, window_frames=wf, n_streams=2) as v:
            assert v.general()
            res = v.score()
            if wf == 0:
                got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
                assert _first_diff(got, frames) == []
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.scores, ref["score"])


@pytest.mark.parametrize("per_byte", ["4", "0"], ids=["estimate", "overflow_rerun"])
def test_cabac_temporal_direct_windows_and_arena_rerun(tmp_path, monkeypatch, per_byte):
    """The CABAC syntax parse + h264_derive (colocated records read by parse
    level) on a B stream with temporal direct, in one window and in several
    windows on two rings; with VTS_ARENA_PER_BYTE=0 the windows' arenas (one
    256-block chunk) overflow, the run reports DEC_E_ARENA to
    the host, which grows the arena from what the windows asked for and runs
    again: every frame, histogram and score equals the oracle either way."""
    _require_gpu()
    monkeypatch.setenv("VTS_ARENA_PER_BYTE", per_byte)
    n = 60
    src, path = tmp_path / "src.mp4", tmp_path / "td.mp4"
    scene.synth_write(src, width=176, height=144, n_frames=n, coding="full", bframes=True,
                      temporal_direct=True, weighted="implicit", cut_min_s=0.5, cut_max_s=1.2,
                      gop_max_s=0.6, seed=21, chunks=1)
    oracle.cabac_convert(src, path, seed=7, t8=True)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    for wf in (0, 24):
        with scene.VideoScorer(path, keep_frames=wf == 0, window_frames=wf, n_streams=2) as v:
            assert v.general()
            res = v.score()
            res2 = v.score()  # a second run on the re-sized arena
            if wf == 0:
                got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
                assert _first_diff(got, frames) == []
            for r in (res, res2):
                assert np.array_equal(r.hist, ref["hist"])
                assert np.array_equal(r.scores, ref["score"])
            assert (v.arena_reruns() >= 1) if per_byte == "0" else (v.arena_reruns() == 0)


def test_cabac_arena_growth_and_reruns_after_another_session(tmp_path, monkeypatch):
    """the bench line whose 10-min 720p content stream
    differed from the oracle ran a noise-stream session first and re-mapped
    the content session's arena after its first run.  Here, at 720p: a noise
    stream's session whose arena overflows and grows (re-mapped HBM) is run
    three times and closed; then a content stream's session on the recycled
    HBM overflows and grows too, and every one of its three runs — the first
    after the growth, then two on the grown arena — equals the oracle in
    histograms, SADs and scores (the chunk counters give every run a
    different block layout)."""
    _require_gpu()
    W, H = 1280, 720
    x264ish = dict(coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit",
                   cabac=True, transform_8x8=True)
    noise, content = tmp_path / "noise.mp4", tmp_path / "content.mp4"
    scene.synth_write(noise, width=W, height=H, fps=30, n_frames=240, seed=5, cut_min_s=1.0,
                      cut_max_s=3.0, gop_max_s=4.0, **x264ish)
    scene.synth_write(content, width=W, height=H, fps=30, n_frames=900, seed=3, cut_min_s=2.0,
                      cut_max_s=6.0, gop_max_s=8.0, content=True, **x264ish)
    monkeypatch.setenv("VTS_ARENA_PER_BYTE", "0")
    for path, n in ((noise, 240), (content, 900)):
        frames, _ = oracle.decode_full(path)
        ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
        del frames
        with scene.VideoScorer(path, k=4) as v:
            assert v.general()
            for run in range(3):
                res = v.score()
                assert np.array_equal(res.hist, ref["hist"]), (path.name, run)
                assert np.array_equal(res.sad, ref["sad"]), (path.name, run)
                assert np.array_equal(res.scores, ref["score"]), (path.name, run)
            assert v.arena_reruns() >= 1


def test_async_runs_of_several_sessions_equal_the_oracle(tmp_path):
    """vts_run_async on three sessions (a CABAC B, a CAVLC B and a subset
    stream) before any vts_wait: the device overlaps them and every result
    equals the oracle; results read without an explicit wait complete the
    run first; a session closed with a run still pending waits for it."""
    _require_gpu()
    n = 48
    paths = [tmp_path / f"a{i}.mp4" for i in range(3)]
    src = tmp_path / "src.mp4"
    scene.synth_write(src, width=176, height=144, n_frames=n, coding="full", bframes=True, weighted="implicit",
                      cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.5, seed=29, chunks=1)
    oracle.cabac_convert(src, paths[0], seed=9, t8=True)
    scene.synth_write(paths[1], width=176, height=144, n_frames=n, coding="full", bframes=True,
                      weighted="implicit", cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.5, seed=31)
    scene.synth_write(paths[2], width=176, height=144, n_frames=n, cut_min_s=0.5, cut_max_s=1.2, seed=37)
    refs = []
    for i, p in enumerate(paths):
        frames, _ = (oracle.decode_full(p) if i < 2 else oracle.decode_file(p))
        refs.append(oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4))
    vs = [scene.VideoScorer(p) for p in paths]
    try:
        for _ in range(2):
            for v in vs:
                v.run_async()
            for i, v in enumerate(vs):
                if i != 1:
                    v.wait()      # session 1: scene_cuts() below waits itself
                cuts = v.scene_cuts()
                assert cuts == np.nonzero(refs[i]["score"] > 0.08)[0].tolist()
                res = v.score()
                assert np.array_equal(res.scores, refs[i]["score"])
                assert np.array_equal(res.hist, refs[i]["hist"])
        vs[0].run_async()  # left pending: close waits
    finally:
        for v in vs:
            v.close()


def test_sessions_reopened_in_sequence_reuse_the_stream_pool(tmp_path):
    """sessions take their HIP streams from a process-wide pool and
    give them back on close; open / run / close several sessions in sequence
    (and two at once) on the same B stream: every run equals the oracle."""
    _require_gpu()
    n = 48
    path = tmp_path / "pool.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=True,
                      weighted="implicit", cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.5, seed=23)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    for _ in range(4):
        with scene.VideoScorer(path) as v:
            res = v.score()
            assert np.array_equal(res.scores, ref["score"]) and np.array_equal(res.hist, ref["hist"])
    with scene.VideoScorer(path) as a, scene.VideoScorer(path) as b:
        ra, rb = a.score(), b.score()
        assert np.array_equal(ra.scores, ref["score"]) and np.array_equal(rb.sad, ref["sad"])
    with scene.VideoScorer(path) as v:
        assert np.array_equal(v.score().scores, ref["score"])


def test_released_stream_sets_are_made_again(tmp_path):
    """vts_release_streams destroys the idle pooled stream sets (a session's
    stays while it is open); sessions opened afterwards make new sets and
    still equal the oracle (the loader calls it at interpreter exit)."""
    _require_gpu()
    from vtseg import _lib
    n = 36
    path = tmp_path / "rel.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=True, cabac=True,
                      weighted="implicit", cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.5, seed=29)
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    L = _lib.lib()
    with scene.VideoScorer(path) as a, scene.VideoScorer(path) as b:
        assert np.array_equal(a.score().scores, ref["score"]) and np.array_equal(b.score().sad, ref["sad"])
        assert L.vts_release_streams(0) >= 0  # the open sessions' sets are not idle: kept
        assert np.array_equal(a.score().hist, ref["hist"])
    assert L.vts_release_streams(-1) >= 2  # both sets idle now
    assert L.vts_release_streams(-1) == 0
    for _ in range(2):
        with scene.VideoScorer(path) as v:
            assert np.array_equal(v.score().scores, ref["score"])


CONTENT = [
    ("qvga", dict(width=320, height=240), 90),
    ("crop_rows", dict(width=320, height=180, slices_per_row=2), 60),
    ("hd720", dict(width=1280, height=720), 36),
]


@pytest.mark.parametrize("name,kw,n", CONTENT, ids=[c[0] for c in CONTENT])
def test_content_streams_equal_the_writer_and_the_oracle(tmp_path, name, kw, n):
    """Content-mode streams (synth_content.h: textured moving scenes coded
    with skip / direct / 16x16 motion / intra decisions and quantised
    residuals, x264's structure): the device's frames equal the oracle's and
    the writer's own closed-loop reconstruction (recon_hash), and the device
    scorer finds the planted cuts."""
    _require_gpu()
    kw = dict(kw)
    spr = kw.pop("slices_per_row", 0)
    path = tmp_path / f"content_{name}.mp4"
    info = scene.synth_write(path, n_frames=n, coding="full", slices_per_row=spr, max_motion=4, bframes=True,
                             weighted="implicit", cabac=True, transform_8x8=True, content=True, hash_frames=True,
                             cut_min_s=0.5, cut_max_s=1.5, gop_max_s=1.0, seed=41, **kw)
    frames, _ = oracle.decode_full(path)
    assert info["recon_hash"] == oracle.recon_hash(frames)
    W, H = kw["width"], kw["height"]
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 4)
    with scene.VideoScorer(path, keep_frames=True) as v:
        assert v.general()
        res = v.score()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(n)])
        assert _first_diff(got, frames) == []
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        assert v.scene_cuts() == sorted(info["cuts"])
    _recycled_equal(path, ref)
