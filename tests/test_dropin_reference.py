"""The drop-in inside the real reference (build container only).

Imports the reference's own ``ContentAnalyzer`` from /root/reference (google
genai stubbed exactly as tests/golden/make_golden.py does), installs
``vtseg.dropin`` (the reference's segmenter modules and the names
content_analyzer.py:27-34 imported are rebound to vtseg's), and replays the
25 recorded segmentation scenarios (make_golden.gen_driver): the analyzer's
call sequence, segment files, gap notes, API counter and manifest must equal
driver_sequences.json, which the unmodified reference produced.  Skipped where
the reference is absent (the GPU box); nothing from the reference is copied.
"""
from __future__ import annotations

import importlib
import json
import sys
from pathlib import Path

import pytest

REF_SRC = Path("/root/reference/src")
GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.mark.skipif(not REF_SRC.is_dir(), reason="reference checkout not present")
def test_reference_content_analyzer_with_vtseg_dropin(monkeypatch):
    sys.path.insert(0, str(GOLDEN))
    try:
        import make_golden
    finally:
        sys.path.remove(str(GOLDEN))
    saved = {k: v for k, v in sys.modules.items()
             if k == "utils" or k.startswith(("utils.", "analyzer", "google"))}
    monkeypatch.syspath_prepend(str(REF_SRC))
    try:
        for k in list(saved):
            del sys.modules[k]
        make_golden._stub_genai()
        import vtseg.dropin
        from vtseg import budget_planner, video_segmenter, video_utils

        ca = importlib.import_module("analyzer.content_analyzer")
        bound = vtseg.dropin.install()
        assert "analyzer.content_analyzer.plan_segments_with_budget" in bound
        # the analyzer now resolves the segmenter names to vtseg
        assert ca.plan_segments_with_budget is budget_planner.plan_segments_with_budget
        assert ca.load_or_create_manifest is video_segmenter.load_or_create_manifest
        assert ca.probe_duration is video_utils.probe_duration
        assert sys.modules["utils.video_segmenter"] is video_segmenter
        counter = importlib.import_module("utils.counter")
        throttle = importlib.import_module("utils.gemini_throttle")
        got = make_golden.gen_driver(ca, counter, throttle)
    finally:
        for k in [k for k in sys.modules if k == "utils" or k.startswith(("utils.", "analyzer", "google"))]:
            del sys.modules[k]
        sys.modules.update(saved)
    want = json.loads((GOLDEN / "driver_sequences.json").read_text())
    assert [s["name"] for s in got] == [s["name"] for s in want]
    for g, w in zip(got, want):
        # JSON round trip: tuples -> lists, as the fixture was written
        assert json.loads(json.dumps(g)) == w, g["name"]
