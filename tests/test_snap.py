"""Opt-in keyframe / scene-aware boundaries (vtseg.snap).

The reference's snap_to_keyframe (video_segmenter.py:157-159) is an identity
stub and nothing in it snaps, so there is no reference output to match: the
default paths must stay the reference's (identity, fixed plan; pinned by the
golden tests), and the opt-in paths are checked against their definition
here.  Keyframe times are checked against the oracle's own MP4 reader (IDR
access units); scene-cut anchors against the oracle scorer (GPU test)."""
from __future__ import annotations

import json
from fractions import Fraction
from pathlib import Path

import pytest

import oracle
from vtseg import scene, snap
from vtseg import video_segmenter as vs
from vtseg.driver import APICounter, SegmentationDriver


def test_snap_time_rules():
    a = [0.0, 9.5, 10.5, 20.0]
    assert snap.snap_time(10.25, a, 1.0) == 10.5           # nearest
    assert snap.snap_time(10.0, a, 1.0) == 9.5             # tie (0.5 / 0.5): the earlier
    assert snap.snap_time(10.25, a, 1.0, "floor") == 9.5
    assert snap.snap_time(15.0, a, 0.3) == 15.0            # nothing within reach
    assert snap.snap_time(10.0, [], 5.0) == 10.0
    assert snap.snap_time(14.0, a, float("inf")) == 10.5
    with pytest.raises(ValueError):
        snap.snap_time(1.0, a, 1.0, "ceil")


def test_default_snap_to_keyframe_is_the_reference_identity(tmp_path):
    assert vs.snap_to_keyframe(tmp_path / "missing.mp4", 12.5) == 12.5
    assert vs.snap_to_keyframe("x.mp4", -3) == 0.0
    with pytest.raises(ValueError):
        vs.snap_to_keyframe("x.mp4", 1.0, mode="anchors")


def test_snapped_plan_without_reachable_anchors_is_the_fixed_plan():
    base = vs.plan_segments(600.0, 480, 20)
    assert snap.plan_segments_snapped(600.0, 480, 20, [], max_shift=30) == base
    assert snap.plan_segments_snapped(600.0, 480, 20, [100.0], max_shift=30) == base
    assert snap.plan_segments_snapped(60.0, 480, 20, [10.0], max_shift=30) == \
        vs.plan_segments(60.0, 480, 20)                     # one segment: nothing to move


def test_snapped_plan_moves_inner_boundaries_and_keeps_overlap_rules():
    segs = snap.plan_segments_snapped(100.0, 30.0, 5.0, [28.0, 61.5, 95.0], max_shift=3.0)
    assert [(s.effective_start, s.effective_end) for s in segs] == \
        [(0.0, 28.0), (28.0, 61.5), (61.5, 90.0), (90.0, 100.0)]
    assert [(s.start, s.end) for s in segs] == \
        [(0.0, 33.0), (23.0, 66.5), (56.5, 95.0), (85.0, 100.0)]
    assert [s.segment_id for s in segs] == [0, 1, 2, 3]
    # a move past the next fixed boundary is not made
    segs = snap.plan_segments_snapped(100.0, 30.0, 0.0, [61.0], max_shift=40.0)
    assert [s.effective_end for s in segs] == [30.0, 61.0, 90.0, 100.0]
    segs = snap.plan_segments_snapped(100.0, 30.0, 0.0, [95.0], max_shift=40.0)
    assert [s.effective_end for s in segs] == [30.0, 60.0, 95.0, 100.0]


def _idr_times(path):
    m = oracle.read_mp4(path)
    data, nls = m["data"], m["nal_length_size"]
    return [float(Fraction(int(m["dts"][i]), m["timescale"])) for i, off in enumerate(m["offsets"])
            if data[off + nls] & 0x1F == 5]


def test_keyframe_times_are_the_idr_access_units(tmp_path):
    path = tmp_path / "k.mp4"
    info = scene.synth_write(path, width=160, height=96, n_frames=300, cut_min_s=0.7,
                             cut_max_s=2.0, gop_max_s=1.0)
    kf = snap.keyframe_times(path)
    assert len(kf) == info["n_idr"]
    assert kf == _idr_times(path)
    assert vs.snap_to_keyframe(path, 4.2, mode="keyframe", direction="floor") == \
        max(t for t in kf if t <= 4.2)


def test_driver_snap_keyframe_is_opt_in(tmp_path):
    path = tmp_path / "clip.mp4"
    scene.synth_write(path, width=160, height=96, n_frames=1800, cut_min_s=3, cut_max_s=9,
                      gop_max_s=2.0)  # 60 s
    kf = snap.keyframe_times(path)
    base = {"enabled": True, "default_segment_seconds": 20, "overlap_seconds": 2,
            "min_segment_seconds": 5, "hard_max_api_calls": 50,
            "duration_threshold_seconds": 30}

    def boundaries(tag, long_video):
        tmp = tmp_path / tag
        cfg = {"system": {"temp_dir": str(tmp)},
               "analyzer": {"max_continuations": 3, "retry_times": 5, "long_video": long_video}}

        def extract(**kw):
            Path(kw["output_path"]).write_bytes(b"x")
            return True

        drv = SegmentationDriver(cfg, APICounter(max_calls=50), lambda p, parts: {"ok": 1},
                                 extract=extract)
        drv.run(path)
        man = json.loads((tmp / "segments" / "clip" / "manifest.json").read_text())
        return [s["effective_end"] for s in man["segments"]][:-1]

    fixed = boundaries("fixed", dict(base))
    snapped = boundaries("snap", dict(base, snap="keyframe", snap_max_shift_seconds=2.5))
    assert fixed == [20.0, 40.0]
    for f, b in zip(fixed, snapped):
        near = [t for t in kf if abs(t - f) <= 2.5]
        assert b == (min(near, key=lambda t: (abs(t - f), t)) if near else f)
    assert snapped != fixed or not any(abs(t - f) <= 2.5 for t in kf for f in fixed)
    with pytest.raises(ValueError):
        boundaries("scene", dict(base, snap="scene"))  # needs a scene_anchors callable


@pytest.mark.gpu
def test_scene_cut_anchors_from_the_device_scorer(tmp_path):
    path = tmp_path / "s.mp4"
    info = scene.synth_write(path, width=320, height=240, n_frames=900, cut_min_s=2,
                             cut_max_s=6, gop_max_s=2.0)
    times = scene.scene_cut_times(path)
    frames, meta = oracle.decode_file(path)
    ref = oracle.score_frames(frames.reshape(-1), frames[0].size, frames.shape[0], 320, 240,
                              320, 240, 4, want_rgb=False)
    want = [float(Fraction(meta["pts"][i], meta["timescale"]))
            for i in range(len(ref["score"])) if ref["score"][i] > scene.DEFAULT_CUT_THRESHOLD]
    assert times == want
    assert len(times) >= len(info["cuts"]) > 0
    segs = snap.plan_segments_snapped(30.0, 10, 1, times, max_shift=2.0)
    for s, f in zip(segs[:-1], (10.0, 20.0)):
        near = [t for t in times if abs(t - f) <= 2.0]
        assert s.effective_end == (min(near, key=lambda t: (abs(t - f), t)) if near else f)
