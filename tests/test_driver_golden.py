"""vtseg.driver vs the reference ContentAnalyzer's segmentation call sequences.

tests/golden/driver_sequences.json was captured by running the reference's
analyze_video (content_analyzer.py:560-964) with the LLM calls replaced
(make_golden.py).  The same scenarios run through vtseg.driver must produce the
identical extract/analyze call sequence, gap notes, API-counter state and
persisted manifest.  Mirrors the reference tests test_long_video_edge_cases.py,
test_long_video_integration.py and test_segment_analysis.py.
"""
from __future__ import annotations

import json
from pathlib import Path

import pytest

from conftest import fhex, load_golden
from vtseg import driver as drv
from vtseg import video_segmenter as vs

OVERFLOW_MSG = "400 INVALID_ARGUMENT: input token count exceeds maximum of 1048576"
CASES = load_golden("driver_sequences.json")


def run_scenario(s: dict, tmp: Path) -> dict:
    config = {"system": {"temp_dir": str(tmp / "temp")},
              "proxy": {"base_url": "http://localhost:8000", "timeout": 60},
              "analyzer": json.loads(json.dumps(s["analyzer"]))}
    counter = drv.APICounter(max_calls=s["max_calls"], current_count=s["current"])
    video = tmp / f"video{s['suffix']}"
    video.write_bytes(b"\x00" * 16)
    duration = fhex(s["duration"])
    if s["premanifest"]:
        vs.load_or_create_manifest(video_id=video.stem, duration=duration,
                                   segment_seconds=s["premanifest"]["segment_seconds"],
                                   overlap_seconds=s["premanifest"]["overlap_seconds"],
                                   temp_dir=str(tmp / "temp"))
    events: list = []
    seg_ranges: dict = {}
    state = {"n": 0}

    def extract(*, input_path, start, end, output_path, stream_copy=True):
        events.append(["extract", Path(input_path).name, float(start).hex(), float(end).hex(),
                       Path(output_path).name, bool(stream_copy)])
        Path(output_path).parent.mkdir(parents=True, exist_ok=True)
        Path(output_path).write_bytes(b"segment")
        return True

    def analyze(segment_path: Path, parts: list):
        events.append(["analyze", segment_path.name, parts[0]])
        state["n"] += 1
        info = seg_ranges.get(segment_path.name)
        if s["overflow_over"] is not None and info is not None and \
                info[1] - info[0] > s["overflow_over"]:
            raise Exception(OVERFLOW_MSG)
        if info is not None and info[2] in s["fail_ids"]:
            raise RuntimeError(f"boom {info[2]}")
        counter.increment("Gemini")  # _call_analysis_json counts after the call returns
        return {"n": state["n"]}

    d = drv.SegmentationDriver(config, counter, analyze, probe=lambda p: duration,
                               extract=extract)
    orig = d.analyze_segment_range

    def wrapper(**kw):
        sp = kw["segment_path"]
        if sp is None:
            sp = kw["segment_dir"] / (f"segment_{kw['segment_id']:04d}_{int(kw['start'] * 1000):010d}_"
                                      f"{int(kw['end'] * 1000):010d}.mp4")
        seg_ranges[Path(sp).name] = (kw["start"], kw["end"], kw["segment_id"])
        if kw["segment_id"] in s["empty_ids"] and kw["segment_path"] is not None:
            events.append(["empty", kw["segment_id"]])
            return []
        return orig(**kw)

    d.analyze_segment_range = wrapper
    md = None
    try:
        res = d.run(video)
        outcome = "ok" if res.outcome == "segmented" else "single_pass"
        if res.outcome == "segmented":
            md = res.metadata
    except Exception as exc:  # compare exception type with the reference
        outcome = f"raise:{type(exc).__name__}"
    mpath = tmp / "temp" / "segments" / video.stem / "manifest.json"
    manifest = None
    if mpath.exists():
        manifest = json.loads(mpath.read_text())
        manifest.pop("created_at", None)
        for e in manifest["segments"]:
            e["file_path"] = Path(e["file_path"]).name
    return {"outcome": outcome, "events": events,
            "metadata": None if md is None else {"duration": float(md["duration"]).hex(),
                                                 "segments": md["segments"],
                                                 "segment_gaps": md["segment_gaps"]},
            "final_count": counter.current_count, "final_max_calls": counter.max_calls,
            "manifest": manifest}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_driver_matches_reference_sequence(case, tmp_path):
    got = run_scenario(case, tmp_path)
    for key in ("outcome", "events", "metadata", "final_count", "final_max_calls", "manifest"):
        assert got[key] == case[key], key


def test_timecodes_match_reference():
    for hexval, expected in load_golden("timecodes.json"):
        assert drv.format_timecode(fhex(hexval)) == expected


def test_overflow_detection():
    assert drv.is_input_token_overflow_error(Exception(OVERFLOW_MSG))
    assert not drv.is_input_token_overflow_error(Exception("400 INVALID_ARGUMENT"))
