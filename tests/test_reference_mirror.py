"""The reference's own hot-path tests, re-run against the drop-in.

Mirrors /reference/tests/test_video_segmenter.py:89-178 and
tests/test_budget_planner.py:25-61 (same inputs, same assertions), importing
the build's modules instead of utils.video_segmenter / utils.budget_planner.
"""
from __future__ import annotations

import math
import shutil
from pathlib import Path
from typing import cast

import pytest

from vtseg import budget_planner
from vtseg import video_segmenter


def _assert_close(value: float, expected: float) -> None:
    assert math.isclose(value, expected, rel_tol=0.0, abs_tol=1e-6)


def test_plan_segments_with_overlap() -> None:
    segments = video_segmenter.plan_segments(duration=100.0, segment_seconds=30.0,
                                             overlap_seconds=5.0)
    assert len(segments) == 4
    _assert_close(segments[0].start, 0.0)
    _assert_close(segments[0].end, 35.0)
    _assert_close(segments[0].effective_start, 0.0)
    _assert_close(segments[0].effective_end, 30.0)
    _assert_close(segments[1].start, 25.0)
    _assert_close(segments[1].end, 65.0)
    _assert_close(segments[1].effective_start, 30.0)
    _assert_close(segments[1].effective_end, 60.0)
    _assert_close(segments[3].start, 85.0)
    _assert_close(segments[3].end, 100.0)
    _assert_close(segments[3].effective_start, 90.0)
    _assert_close(segments[3].effective_end, 100.0)


def test_plan_segments_no_overlap() -> None:
    segments = video_segmenter.plan_segments(duration=50.0, segment_seconds=20.0,
                                             overlap_seconds=-3.0)
    assert len(segments) == 3
    _assert_close(segments[1].start, 20.0)
    _assert_close(segments[1].end, 40.0)


def test_manifest_create_and_resume(tmp_path: Path) -> None:
    manifest = video_segmenter.create_manifest(video_id="video123", duration=65.0,
                                               segment_seconds=30.0, overlap_seconds=5.0,
                                               temp_dir=tmp_path)
    manifest_path = video_segmenter.get_manifest_path("video123", tmp_path)
    assert manifest_path.exists()
    assert manifest["segments"][0]["status"] == "pending"
    manifest["segments"][0]["status"] = "completed"
    video_segmenter.save_manifest(manifest_path, manifest)
    loaded = video_segmenter.load_or_create_manifest(video_id="video123", duration=65.0,
                                                     segment_seconds=30.0, overlap_seconds=5.0,
                                                     temp_dir=tmp_path)
    assert loaded["segments"][0]["status"] == "completed"
    pending = video_segmenter.pending_segments(loaded)
    assert all(segment["id"] != 0 for segment in pending)


@pytest.mark.skipif(shutil.which("ffmpeg") is None, reason="ffmpeg not available")
def test_extract_segment_integration(tmp_path: Path) -> None:
    import subprocess
    input_path = tmp_path / "input.mp4"
    output_path = tmp_path / "segment.mp4"
    subprocess.run(["ffmpeg", "-y", "-hide_banner", "-loglevel", "error", "-f", "lavfi", "-i",
                    "color=c=black:s=320x240:d=1", "-c:v", "libx264", str(input_path)],
                   capture_output=True, text=True, timeout=30, check=True)
    assert video_segmenter.extract_segment(input_path=input_path, start=0.0, end=0.5,
                                           output_path=output_path, stream_copy=True)
    assert output_path.exists() and output_path.stat().st_size > 0


def test_extract_segment_without_ffmpeg_returns_false(tmp_path: Path, monkeypatch) -> None:
    monkeypatch.setenv("PATH", str(tmp_path))  # no ffmpeg on PATH
    out = tmp_path / "o" / "seg.mp4"
    assert video_segmenter.extract_segment(tmp_path / "in.mp4", 0.0, 1.0, out) is False
    assert not out.exists() and out.parent.exists()
    assert video_segmenter.extract_segment(tmp_path / "in.mp4", 1.0, 1.0, out) is False


def _base_config() -> dict[str, object]:
    return {"analyzer": {"max_continuations": 3, "retry_times": 5,
                         "long_video": {"enabled": True, "default_segment_seconds": 480,
                                        "overlap_seconds": 20, "min_segment_seconds": 90,
                                        "hard_max_api_calls": 50, "consolidate": True}}}


def test_long_video_caps_calls() -> None:
    plan = budget_planner.plan_segments_with_budget(3 * 60 * 60, _base_config(),
                                                    current_api_count=0)
    assert plan.num_segments >= 1
    assert plan.estimated_calls <= plan.hard_max_calls


def test_short_video_under_threshold_single_segment() -> None:
    config = _base_config()
    analyzer_config = cast(dict[str, object], config["analyzer"])
    long_video_config = cast(dict[str, object], analyzer_config["long_video"])
    long_video_config["duration_threshold_seconds"] = 600
    plan = budget_planner.plan_segments_with_budget(9 * 60, config, current_api_count=0)
    assert plan.num_segments == 1
    assert plan.overlap == 0


def test_budget_exact_limit() -> None:
    config: dict[str, object] = {
        "analyzer": {"max_continuations": 2, "retry_times": 0,
                     "long_video": {"enabled": True, "default_segment_seconds": 400,
                                    "overlap_seconds": 0, "min_segment_seconds": 90,
                                    "hard_max_api_calls": 8, "consolidate": True}}}
    plan = budget_planner.plan_segments_with_budget(1200, config, current_api_count=0)
    assert plan.estimated_calls == plan.hard_max_calls


def test_snap_to_keyframe_is_identity_clamp() -> None:
    assert video_segmenter.snap_to_keyframe("x.mp4", 12.5) == 12.5
    assert video_segmenter.snap_to_keyframe("x.mp4", -3) == 0.0
