"""Native manifest writer (vts_manifest_json, csrc/manifest.cpp)
against the reference's create_manifest bytes (tests/golden/manifests.json,
generated from /root/reference by tests/golden/make_golden.py) and, for the
formatting rules, against Python's own json.dumps(indent=2, ensure_ascii=True)
on random inputs (float repr, int objects, unicode and control characters)."""
from __future__ import annotations

import json
import math
import random
import struct

import pytest

from vtseg import video_segmenter as vs

GOLDEN = json.load(open(__import__("pathlib").Path(__file__).parent / "golden" / "manifests.json"))


def _num(v, is_int):
    return int(v) if is_int else float.fromhex(v)


@pytest.mark.parametrize("case", GOLDEN, ids=[c["video_id"] for c in GOLDEN])
def test_native_manifest_matches_reference_bytes(case):
    text = vs.manifest_json(
        video_id=case["video_id"], duration=float.fromhex(case["duration"]),
        segment_seconds=_num(case["segment_seconds"], case["segment_is_int"]),
        overlap_seconds=_num(case["overlap_seconds"], case["overlap_is_int"]),
        segment_dir="@TEMP@/segments/" + case["video_id"], created_at="@CREATED@")
    assert text == case["json"]


def _python_text(video_id, duration, seg, ovl, segment_dir, created_at):
    """The reference's formatting, restated with the build's planner."""
    entries = []
    for s in vs.plan_segments(duration, seg, ovl):
        entries.append({"id": s.segment_id, "start": s.start, "end": s.end,
                        "effective_start": s.effective_start,
                        "effective_end": s.effective_end,
                        "file_path": str(__import__("pathlib").Path(segment_dir)
                                         / f"segment_{s.segment_id:04d}.mp4"),
                        "status": "pending", "attempts": 0, "error": None})
    m = {"version": 1, "video_id": video_id, "created_at": created_at,
         "segment_seconds": seg, "overlap_seconds": ovl, "segments": entries}
    return json.dumps(m, indent=2, ensure_ascii=True)


def _rand_double(rng):
    while True:
        x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        if math.isfinite(x) and x > 0:
            return x


def test_native_manifest_fuzz_against_python_json():
    rng = random.Random(5)
    ids = ["a", "vid eo", "quote\"back\\slash", "tab\tnl\nesc\x1b del\x7f", "é中文",
           "emoji 😀 astral", " sep", "x" * 300]
    for trial in range(400):
        kind = trial % 4
        if kind == 0:      # random doubles of every magnitude, few segments
            seg = _rand_double(rng)
            dur = seg * rng.choice([0.5, 1.0, 2.5, 3.0])
            ovl = rng.choice([0, 0.0, seg / 7, -1.5])
        elif kind == 1:    # ints, as SegmentPlan hands them over
            seg = rng.randint(1, 2000)
            ovl = rng.randint(0, 50)
            dur = rng.choice([rng.randint(0, 20000), rng.uniform(0, 20000)])
        elif kind == 2:    # fractional seconds
            seg = round(rng.uniform(0.05, 900), rng.randint(0, 6))
            ovl = round(rng.uniform(0, 30), rng.randint(0, 4))
            dur = rng.uniform(0, 5000)
        else:              # tiny / huge
            seg = rng.choice([1e-5, 3e-7, 1e15, 1e16, 123456789012345678.0])
            dur = seg * rng.randint(0, 9)
            ovl = rng.choice([0, seg / 3])
        vid = rng.choice(ids)
        sdir = rng.choice(["/tmp/t/segments/" + vid, "rel/segments/" + vid, "/"])
        created = "2026-10-16T08:00:00.123456+00:00"
        want = _python_text(vid, dur, seg, ovl, sdir, created)
        got = vs.manifest_json(video_id=vid, duration=dur, segment_seconds=seg,
                               overlap_seconds=ovl, segment_dir=sdir, created_at=created)
        assert got == want, (trial, dur, seg, ovl)


def test_native_manifest_defers_to_python_for_other_objects():
    # bool prints as `true`, numpy ints are refused by json: both stay with Python
    assert vs.manifest_json(video_id="v", duration=10.0, segment_seconds=True,
                            overlap_seconds=0, segment_dir="d", created_at="c") is None
    assert vs.manifest_json(video_id="bad\udcff", duration=10.0, segment_seconds=5,
                            overlap_seconds=0, segment_dir="d", created_at="c") is None


def test_create_manifest_file_is_native_text(tmp_path):
    m = vs.create_manifest(video_id="vid", duration=600.0, segment_seconds=480,
                           overlap_seconds=20, temp_dir=tmp_path)
    raw = vs.get_manifest_path("vid", tmp_path).read_text(encoding="utf-8")
    assert raw == json.dumps(m, indent=2, ensure_ascii=True)
    assert vs.load_or_create_manifest(video_id="vid", duration=1.0, segment_seconds=1,
                                      overlap_seconds=0, temp_dir=tmp_path) == m
