"""Manifest files written by vtseg.video_segmenter are byte-identical to the
reference's (video_segmenter.py:170-218), created_at and temp dir excepted."""
from __future__ import annotations

from conftest import fhex, load_golden
from vtseg import video_segmenter as vs


def _arg(v, is_int):
    return v if is_int else fhex(v)


def test_manifest_bytes_match_reference(tmp_path):
    for i, c in enumerate(load_golden("manifests.json")):
        td = tmp_path / f"t{i}"
        m = vs.create_manifest(video_id=c["video_id"], duration=fhex(c["duration"]),
                               segment_seconds=_arg(c["segment_seconds"], c["segment_is_int"]),
                               overlap_seconds=_arg(c["overlap_seconds"], c["overlap_is_int"]),
                               temp_dir=td)
        raw = vs.get_manifest_path(c["video_id"], td).read_text(encoding="utf-8")
        raw = raw.replace(str(td), "@TEMP@").replace(m["created_at"], "@CREATED@")
        assert raw == c["json"], c["video_id"]


def test_existing_manifest_is_reused_verbatim(tmp_path):
    m = vs.create_manifest(video_id="v", duration=100.0, segment_seconds=30.0,
                           overlap_seconds=5.0, temp_dir=tmp_path)
    m["segments"][1]["status"] = "failed"
    m["segments"][1]["error"] = "x"
    vs.save_manifest(vs.get_manifest_path("v", tmp_path), m)
    again = vs.load_or_create_manifest(video_id="v", duration=999.0, segment_seconds=1.0,
                                       overlap_seconds=0.0, temp_dir=tmp_path)
    assert again == m


def test_update_unknown_segment_logs_warning(tmp_path, caplog):
    m = vs.create_manifest(video_id="v", duration=10.0, segment_seconds=5.0,
                           overlap_seconds=0.0, temp_dir=tmp_path)
    vs.update_segment_status(m, 99, "completed")
    assert "not found" in caplog.text
    vs.update_segment_status(m, 0, "processing", increment_attempts=True, error="e")
    assert m["segments"][0]["attempts"] == 1 and m["segments"][0]["error"] == "e"
