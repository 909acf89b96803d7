"""CPU tests: synthetic stream writer, container probe, oracle decoder, boundaries.

No reference test covers decoded pixels (the reference never decodes); the
decoder/scorer oracle is pinned to the generator's own reconstruction
(vts_synth_info.recon_hash): two independent implementations of the same
H.264 clauses must agree bit for bit.  Parity vs a third-party decoder is
unpinned (no ffmpeg/libavcodec in the image).
"""
from __future__ import annotations

import math

import numpy as np
import pytest

import oracle
from vtseg import _lib, scene, video_utils
from vtseg import video_segmenter as vs

STREAMS = [
    dict(width=320, height=240),
    dict(width=320, height=240, slices_per_row=0, max_motion=8),   # median MV prediction
    dict(width=336, height=200, slices_per_row=3, max_motion=6),   # ragged slices, crop
    dict(width=640, height=360, slices_per_row=2, max_motion=2),   # 360 = 22.5 MB rows: crop 8
    dict(width=96, height=64, max_motion=0),                       # static: P_Skip runs only
    dict(width=320, height=240, max_motion=5, odd_motion=True),     # half-pel chroma bilinear
    dict(width=160, height=96, max_motion=4, gop_max_s=0.3, nonref_refresh=True),  # non-ref I
]


@pytest.mark.parametrize("kw", STREAMS)
def test_generator_reconstruction_equals_oracle_decode(tmp_path, kw):
    path = tmp_path / "s.mp4"
    kw = dict(kw)
    gop = kw.pop("gop_max_s", 1.0)
    r = scene.synth_write(path, n_frames=120, cut_min_s=0.7, cut_max_s=1.6, gop_max_s=gop,
                          hash_frames=True, **kw)
    frames, info = oracle.decode_file(path)
    assert frames.shape == (120, kw["height"] * 3 // 2, kw["width"])
    assert oracle.recon_hash(frames) == r["recon_hash"]
    assert info["pts"] == [1000 * i for i in range(120)]


def test_pcm_with_emulation_prevention_decodes_in_oracle(tmp_path):
    """Zero runs in I_PCM samples force emulation-prevention bytes inside the
    PCM span; the oracle's EPB-aware PCM read still matches the generator."""
    path = tmp_path / "z.mp4"
    r = scene.synth_write(path, width=160, height=96, n_frames=30, gop_max_s=0.5,
                          hash_frames=True, pcm_zero_runs=True)
    m = oracle.read_mp4(path)
    assert any(b"\x00\x00\x03" in m["data"][o:o + n] for o, n in zip(m["offsets"], m["sizes"]))
    frames, _ = oracle.decode_file(path)
    assert oracle.recon_hash(frames) == r["recon_hash"]
    assert (frames[0, :96, :] == 0).sum() > 0


def test_scene_cuts_are_the_top_scores(tmp_path):
    path = tmp_path / "c.mp4"
    r = scene.synth_write(path, width=320, height=240, n_frames=300, cut_min_s=1, cut_max_s=3,
                          gop_max_s=1.0)
    frames, _ = oracle.decode_file(path)
    s = oracle.score_frames(frames.reshape(-1), frames[0].size, 300, 320, 240, 320, 240, 4)
    cuts = set(np.nonzero(s["score"] > scene.DEFAULT_CUT_THRESHOLD)[0].tolist())
    assert set(r["cuts"]) <= cuts
    assert len(cuts - set(r["cuts"])) <= 2  # pan + sparkle rarely crosses the threshold


def test_probe_duration_matches_container(tmp_path):
    path = tmp_path / "p.mp4"
    scene.synth_write(path, width=128, height=96, n_frames=45)  # 1.5 s at 30 fps
    assert video_utils.probe_duration(path) == 1.5
    assert video_utils.probe_duration(str(path)) == 1.5


def test_probe_duration_never_raises(tmp_path):
    assert video_utils.probe_duration(tmp_path / "missing.mp4") == 0.0
    junk = tmp_path / "junk.mp4"
    junk.write_bytes(b"\x00\x00\x00\x10ftypisom" + b"\x00" * 64)
    assert video_utils.probe_duration(junk) == 0.0  # no moov
    dummy = tmp_path / "dummy.mp4"
    dummy.write_bytes(b"\x00" * 1024)  # reference tests' zero-byte "videos"
    assert video_utils.probe_duration(dummy) == 0.0


def test_probe_duration_falls_back_to_ffprobe_without_a_native_answer(tmp_path, monkeypatch):
    """An ISO-BMFF file the native parser cannot time (no moov / fragmented)
    gets ffprobe's answer, as in the reference; a timed file never runs it."""
    calls = []

    def fake(path):
        calls.append(str(path))
        return 12.5

    monkeypatch.setattr(video_utils, "_ffprobe_duration", fake)
    junk = tmp_path / "frag.mp4"
    junk.write_bytes(b"\x00\x00\x00\x10ftypisom" + b"\x00" * 64)
    assert video_utils.probe_duration(junk) == 12.5
    assert calls == [str(junk)]
    good = tmp_path / "g.mp4"
    scene.synth_write(good, width=64, height=48, n_frames=30)
    assert video_utils.probe_duration(good) == 1.0
    assert calls == [str(junk)]


def test_probe_info_fields(tmp_path):
    import ctypes as C
    path = tmp_path / "i.mp4"
    scene.synth_write(path, width=1920, height=1080, n_frames=4)
    info = _lib.VideoInfo()
    _lib.check(_lib.lib().vts_probe_info(str(path).encode(), C.byref(info)))
    assert (info.width, info.height) == (1920, 1080)
    assert (info.coded_width, info.coded_height) == (1920, 1088)
    assert info.n_frames == 4 and info.track_timescale == 30000 and info.codec == 1
    assert info.profile_idc == 66 and info.duration_us == 133000  # mvhd is in ms


def test_boundary_frames_native_equals_exact_rational():
    import ctypes as C
    rng = np.random.default_rng(3)
    for ts, delta in [(30000, 1001), (30000, 1000), (90000, 3003), (1000, 33)]:
        pts = [i * delta for i in range(500)]
        times = [0.0, -0.0, -5.0, 1e-300, float("nan"), float("inf"), float("-inf"), 1e300]
        times += list(rng.uniform(0, 500 * delta / ts, 200))
        times += [i * delta / ts for i in range(0, 500, 7)]
        times += [math.nextafter(i * delta / ts, -1.0) for i in range(1, 500, 11)]
        times += [math.nextafter(i * delta / ts, 2.0 ** 40) for i in range(1, 500, 13)]
        pa = (C.c_int64 * len(pts))(*pts)
        ta = (C.c_double * len(times))(*times)
        out = (C.c_int64 * len(times))()
        _lib.check(_lib.lib().vts_boundary_frames_pts(pa, len(pts), ts, ta, len(times), out))
        assert list(out) == oracle.boundary_frames(pts, ts, times)


def test_segment_boundaries_to_frames_for_planned_segments():
    """Each planned segment time maps to a frame index (first frame at or after
    it), consistent with the exact rational definition."""
    import ctypes as C
    fps_pts = [1000 * i for i in range(18000)]
    segs = vs.plan_segments(600.0, 480, 20)
    times = [t for s in segs for t in (s.start, s.end, s.effective_start, s.effective_end)]
    pa = (C.c_int64 * len(fps_pts))(*fps_pts)
    ta = (C.c_double * len(times))(*times)
    out = (C.c_int64 * len(times))()
    _lib.check(_lib.lib().vts_boundary_frames_pts(pa, len(fps_pts), 30000, ta, len(times), out))
    assert list(out) == [0, 15000, 0, 14400, 13800, 18000, 14400, 18000]


def test_synth_rejects_bad_parameters(tmp_path):
    with pytest.raises(_lib.VtsegError):
        scene.synth_write(tmp_path / "x.mp4", width=15, height=16, n_frames=1)
    with pytest.raises(_lib.VtsegError):
        scene.synth_write(tmp_path / "x.mp4", width=64, height=64, n_frames=1, max_motion=3)


@pytest.mark.parametrize("k", [4, 6])
def test_gop_parallel_oracle_equals_sequential(tmp_path, k):
    """oracle.decode_score_gops (the bench's parity leg): GOP-parallel decode
    + score with the GOP-start SADs completed afterwards equals one sequential
    pass over the whole stream."""
    path = tmp_path / "g.mp4"
    W, H = (320, 240) if k == 4 else (480, 270)
    scene.synth_write(path, width=W, height=H, n_frames=200, cut_min_s=0.5, cut_max_s=2.0,
                      gop_max_s=0.4, max_motion=6)
    frames, info = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, 200, W, H, W, H, k,
                              want_rgb=False)
    got = oracle.decode_score_gops(path, k, threads=4)
    assert got["frames"] == 200 and got["gops"] > 10
    assert np.array_equal(got["hist"], ref["hist"])
    assert np.array_equal(got["sad"], ref["sad"])
    assert np.array_equal(got["score"], ref["score"])
    assert got["pts"] == info["pts"]
    part = oracle.decode_score_gops(path, k, threads=2, max_frames=50)
    assert 50 <= part["frames"] < 80
    assert np.array_equal(part["score"], ref["score"][:part["frames"]])
