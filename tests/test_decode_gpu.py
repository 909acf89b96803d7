"""Device decode + score (vts_open/vts_score, HIP on gfx950) vs the C oracle.

For each synthetic stream: every decoded NV12 frame, every 256-bin histogram
and SAD, and every fp32 score must equal the scalar oracle's bit for bit
(north_star allows |d score| <= 1e-4; integer accumulation makes it exact and
the test asserts exact equality).  Segment boundary frame indices must match
the exact rational oracle.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import VtsegError, scene
from vtseg import video_segmenter as vs

pytestmark = pytest.mark.gpu

STREAMS = [
    ("qvga", dict(width=320, height=240)),
    ("median", dict(width=320, height=240, slices_per_row=0, max_motion=8)),
    ("ragged", dict(width=336, height=200, slices_per_row=3, max_motion=6)),
    ("nhd", dict(width=640, height=360, slices_per_row=2, max_motion=2)),
    ("static", dict(width=96, height=64, max_motion=0)),
    ("bigpan", dict(width=320, height=240, max_motion=24)),    # edge MBs: partial fill
    ("hugepan", dict(width=256, height=160, max_motion=40)),   # edge MBs: all fill
    ("halfpel", dict(width=320, height=240, max_motion=5, odd_motion=True)),   # chroma bilinear
    ("hd720", dict(width=1280, height=720, max_motion=4)),
    ("fhd", dict(width=1920, height=1080, max_motion=8)),
]


def _require_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")


def _oracle_scores(frames, w, h):
    k = 4 if h <= 720 else 6
    return oracle.score_frames(frames.reshape(-1), frames[0].size, frames.shape[0], w, h, w, h, k,
                               want_rgb=True)


@pytest.mark.parametrize("level_block", [1, 4], ids=["per_level", "level_blocked"])
@pytest.mark.parametrize("name,kw", STREAMS, ids=[s[0] for s in STREAMS])
def test_decode_and_score_bit_exact(tmp_path, name, kw, level_block):
    """level_block 1: one reconstruct launch per GOP level; 4: the
    level-blocked kernel where it applies (k = 4), storing every frame here
    (keep_frames) so each one is compared."""
    _require_gpu()
    n = 90 if kw["height"] < 720 else 40
    path = tmp_path / f"{name}.mp4"
    r = scene.synth_write(path, n_frames=n, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.8,
                          hash_frames=True, **kw)
    frames, info = oracle.decode_file(path)
    assert oracle.recon_hash(frames) == r["recon_hash"]
    ref = _oracle_scores(frames, kw["width"], kw["height"])
    with scene.VideoScorer(path, level_block=level_block, keep_frames=True) as vsr:
        res = vsr.score()
        for i in range(n):
            got = vsr.frame_nv12(i).reshape(frames[i].shape)
            assert np.array_equal(got, frames[i]), f"frame {i} differs"
        rgb = np.stack([vsr.thumbnail_rgb(i) for i in range(n)]).reshape(-1)
        assert np.array_equal(rgb, ref["rgb"])
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        assert res.pts.tolist() == info["pts"]
        cuts = vsr.scene_cuts()
        assert cuts == np.nonzero(ref["score"] > scene.DEFAULT_CUT_THRESHOLD)[0].tolist()
        assert set(r["cuts"]) <= set(cuts)


def test_windowed_two_stream_pipeline_equals_single_window(tmp_path):
    """Many small windows over two HIP streams / two rings give exactly the
    single-window results (score continuity across window seams)."""
    _require_gpu()
    path = tmp_path / "w.mp4"
    scene.synth_write(path, width=640, height=360, n_frames=400, cut_min_s=1, cut_max_s=4,
                      gop_max_s=0.5)
    with scene.VideoScorer(path) as a:
        whole = a.score()
    for n_streams in (1, 2):
        with scene.VideoScorer(path, window_frames=40, n_streams=n_streams) as b:
            part = b.score()
            assert np.array_equal(part.scores, whole.scores)
            assert np.array_equal(part.hist, whole.hist)
            assert np.array_equal(part.sad, whole.sad)
            with pytest.raises(VtsegError):
                b.frame_nv12(0)  # evicted from the ring


def test_repeated_runs_are_deterministic(tmp_path):
    _require_gpu()
    path = tmp_path / "d.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=120)
    with scene.VideoScorer(path) as v:
        a = v.score()
        v.run()
        b = v.score()
    assert np.array_equal(a.scores, b.scores) and np.array_equal(a.hist, b.hist)


def test_boundary_frames_for_planned_segments(tmp_path):
    _require_gpu()
    path = tmp_path / "b.mp4"
    scene.synth_write(path, width=128, height=96, n_frames=1800, max_motion=2)  # 60 s
    segs = vs.plan_segments(60.0, 25.0, 2.5)
    times = [t for s in segs for t in (s.start, s.end, s.effective_start, s.effective_end)]
    with scene.VideoScorer(path) as v:
        got = v.boundary_frames(times)
        pts = v.score().pts.tolist()
    assert got == oracle.boundary_frames(pts, 30000, times)
    assert got[:4] == [0, 825, 0, 750]


def test_emulation_prevention_inside_pcm_fails_loudly(tmp_path):
    """Outside the subset kernels: an EPB inside I_PCM samples.  The subset-only
    decoder must refuse with the reason, never return wrong pixels; the default
    (auto) decoder hands the stream to the general decoder, which reads the
    samples through the RBSP and equals the general oracle."""
    _require_gpu()
    path = tmp_path / "z.mp4"
    scene.synth_write(path, width=160, height=96, n_frames=30, gop_max_s=0.5,
                      pcm_zero_runs=True)
    with scene.VideoScorer(path, decoder="subset") as v:
        with pytest.raises(VtsegError, match="emulation prevention inside I_PCM"):
            v.score()
    frames, _ = oracle.decode_full(path)
    with scene.VideoScorer(path, keep_frames=True) as v:
        v.score()
        assert v.general()
        got = np.stack([v.frame_nv12(i).reshape(frames[i].shape) for i in range(30)])
    assert np.array_equal(got, frames)


@pytest.mark.parametrize("coding", ["cabac", "cavlc"])
def test_corrupted_slice_data_fails_loudly(tmp_path, coding):
    """a stream whose slice data was damaged after its
    headers (so vts_open accepts it) fails its run with VTS_E_DECODE — the
    parse ends away from the RBSP stop bit or meets impossible syntax — and
    the session stays usable: closing it and decoding the intact stream
    again equals the oracle."""
    _require_gpu()
    from vtseg import _lib
    n = 24
    path, bad = tmp_path / "ok.mp4", tmp_path / "bad.mp4"
    extra = dict(cabac=True, transform_8x8=True) if coding == "cabac" else {}
    # one slice per picture: the damage (past the first third of the sample)
    # lands in slice data, never in another slice's header, which vts_open
    # would refuse instead
    scene.synth_write(path, width=176, height=144, n_frames=n, coding="full", bframes=True, weighted="implicit",
                      cut_min_s=0.5, cut_max_s=1.0, gop_max_s=0.5, seed=17, slices_per_row=0, **extra)
    m = oracle.read_mp4(path)
    data = bytearray(path.read_bytes())
    rng = np.random.default_rng(5)
    for i in range(0, n, 3):  # every third picture: a few bytes past its slice header
        off, size = int(m["offsets"][i]), int(m["sizes"][i])
        for _ in range(3):
            j = off + int(rng.integers(size // 3, size))
            data[j] ^= 0xA5
    bad.write_bytes(bytes(data))
    with scene.VideoScorer(bad) as v:
        with pytest.raises(VtsegError) as ei:
            v.score()
        assert ei.value.code == _lib.VTS_E_DECODE, ei.value
    frames, _ = oracle.decode_full(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 176, 144, 176, 144, 4)
    with scene.VideoScorer(path) as v:
        assert np.array_equal(v.score().scores, ref["score"])


def test_open_rejects_non_mp4(tmp_path):
    _require_gpu()
    bad = tmp_path / "x.mp4"
    bad.write_bytes(b"\x00" * 4096)
    with pytest.raises(VtsegError):
        scene.VideoScorer(bad)


@pytest.mark.parametrize("k", [2, 4, 8])
def test_fused_and_unfused_paths_agree_with_oracle(tmp_path, k):
    """Scoring fused into reconstruction (one pass) equals the two-kernel path
    and the oracle, for every k that divides a macroblock."""
    _require_gpu()
    path = tmp_path / "f.mp4"
    n = 75
    scene.synth_write(path, width=480, height=272, n_frames=n, cut_min_s=0.6, cut_max_s=1.2,
                      gop_max_s=0.7, max_motion=6, slices_per_row=2)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, 480, 272, 480, 272, k)
    results = []
    for fused in (1, -1):
        with scene.VideoScorer(path, k=k, fused=fused) as v:
            assert v._lib.vts_schedule_info(v._ctx, 4) == (1 if fused == 1 else 0)
            res = v.score()
            rgb = np.stack([v.thumbnail_rgb(i, k) for i in range(n)]).reshape(-1)
            results.append((res, rgb))
            assert np.array_equal(v.frame_nv12(n - 1).reshape(frames[-1].shape), frames[-1])
        assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(rgb, ref["rgb"])


K6_STREAMS = [
    ("q270", dict(width=480, height=270, max_motion=6, slices_per_row=2)),     # crop 2 rows
    ("q540", dict(width=960, height=540, max_motion=24, slices_per_row=1)),    # crop 4, edge fills
    ("nocrop", dict(width=384, height=192, max_motion=4, slices_per_row=0)),   # one slice/picture
    ("halfpel6", dict(width=480, height=270, max_motion=7, odd_motion=True)),  # general path
]


@pytest.mark.parametrize("name,kw", K6_STREAMS, ids=[s[0] for s in K6_STREAMS])
def test_k6_band_kernel_agrees_with_unfused_and_oracle(tmp_path, name, kw):
    """k = 6 (1080p's thumbnail factor) fused into reconstruction: six-row
    bands across macroblock rows, pixels straddling lanes, cropped rows
    reconstructed but not scored."""
    _require_gpu()
    path = tmp_path / f"{name}.mp4"
    n = 50
    scene.synth_write(path, n_frames=n, cut_min_s=0.5, cut_max_s=1.0, gop_max_s=0.6,
                      hash_frames=True, **kw)
    frames, _ = oracle.decode_file(path)
    W, H = kw["width"], kw["height"]
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, 6)
    for fused in (1, -1):
        with scene.VideoScorer(path, k=6, fused=fused) as v:
            assert v.fused() == (fused == 1)
            res = v.score()
            for i in range(n):
                assert np.array_equal(v.frame_nv12(i).reshape(frames[i].shape), frames[i]), i
            rgb = np.stack([v.thumbnail_rgb(i, 6) for i in range(n)]).reshape(-1)
        assert np.array_equal(res.hist, ref["hist"])
        assert np.array_equal(res.sad, ref["sad"])
        assert np.array_equal(res.scores, ref["score"])
        assert np.array_equal(rgb, ref["rgb"])


def test_fused_windowed_pipeline(tmp_path):
    _require_gpu()
    path = tmp_path / "fw.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=300, cut_min_s=1, cut_max_s=3,
                      gop_max_s=0.5)
    with scene.VideoScorer(path, fused=-1) as a:
        whole = a.score()
    with scene.VideoScorer(path, window_frames=32, n_streams=2, fused=1) as b:
        part = b.score()
    assert np.array_equal(part.scores, whole.scores)
    assert np.array_equal(part.hist, whole.hist)


@pytest.mark.parametrize("gops", [1, 3, -1])
def test_gop_grouped_schedule_equals_all_at_once(tmp_path, gops):
    _require_gpu()
    path = tmp_path / "g.mp4"
    scene.synth_write(path, width=320, height=240, n_frames=240, cut_min_s=0.8, cut_max_s=2,
                      gop_max_s=0.4)
    frames, _ = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, 240, 320, 240, 320, 240, 4)
    with scene.VideoScorer(path, gops_per_launch=gops) as v:
        res = v.score()
        assert np.array_equal(v.frame_nv12(239).reshape(frames[-1].shape), frames[-1])
    assert np.array_equal(res.scores, ref["score"]) and np.array_equal(res.hist, ref["hist"])


def test_missing_slice_fails_loudly_even_over_stale_commands(tmp_path):
    """The last picture lacks a slice.  With small windows the two command
    rings are reused, so the missing macroblocks' slots hold valid commands
    of an earlier window (another epoch): they must still read as absent and
    the run must fail with the reason, on every run."""
    _require_gpu()
    path = tmp_path / "m.mp4"
    n = 185  # the last picture is a P picture (IDR every 30)
    scene.synth_write(path, width=160, height=96, n_frames=n, cut_min_s=20, cut_max_s=30,
                      gop_max_s=1.0, drop_last_slice=True)
    for window in (0, 31):
        with scene.VideoScorer(path, window_frames=window) as v:
            for _ in range(2):
                with pytest.raises(VtsegError, match="not covered by any slice"):
                    v.score()


@pytest.mark.parametrize("W,H,k", [(1280, 720, 4), (1920, 1080, 6)], ids=["720p", "1080p"])
def test_streamed_hd_windows_bit_exact(tmp_path, monkeypatch, W, H, k):
    """BASELINE configs [2] / [4] in miniature: 720p (h264_recon_score<4>) and
    1080p (h264_recon_score6b, cropped 1088 -> 1080) decoded in the streamed
    schedule — many whole-GOP windows over two rings and two HIP streams
    (decode of window i+1 overlapping scoring of window i), two interleaved GOP
    groups per window — every histogram, SAD, score, scene cut and the frames
    still in the ring equal the oracle's over 600 frames."""
    _require_gpu()
    n = 600
    path = tmp_path / f"s{H}.mp4"
    scene.synth_write(path, width=W, height=H, n_frames=n, max_motion=8, cut_min_s=2,
                      cut_max_s=8, gop_max_s=2.0, seed=0x5EED + H)
    ref = oracle.decode_score_gops(path, k, threads=8)
    monkeypatch.setenv("VTS_RECON_GROUPS", "2")
    with scene.VideoScorer(path, k=k, window_frames=150, n_streams=2) as v:
        assert v.fused()
        assert v.windows() >= 4
        for _ in range(2):
            res = v.score()
            assert np.array_equal(res.hist, ref["hist"])
            assert np.array_equal(res.sad, ref["sad"])
            assert np.array_equal(res.scores, ref["score"])
        assert v.scene_cuts() == np.nonzero(ref["score"] > scene.DEFAULT_CUT_THRESHOLD)[0].tolist()
        m = oracle.read_mp4(path)
        nls = m["nal_length_size"]
        last_idr = max(i for i in range(n) if m["data"][m["offsets"][i] + nls] & 0x1F == 5)
        samples = [m["data"][o:o + z] for o, z in zip(m["offsets"][last_idr:], m["sizes"][last_idr:])]
        tail = oracle.decode_samples(m["sps"][0], m["pps"][0], samples, nls)[-3:]
        for j in range(3):
            assert np.array_equal(v.frame_nv12(n - 3 + j).reshape(tail[j].shape), tail[j])
