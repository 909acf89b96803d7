"""vtseg.dropin binds the build under the reference's module names.

Uses a stand-in package with the reference's import structure
(src/utils/__init__.py:5 re-exports video_segmenter; content_analyzer.py:27-34
imports the segmenter names at module level); no reference code is run.
"""
from __future__ import annotations

import importlib
import sys
import textwrap


def test_install_rebinds_reference_names(tmp_path, monkeypatch):
    (tmp_path / "utils").mkdir()
    (tmp_path / "utils" / "__init__.py").write_text("from . import video_segmenter\n")
    for m in ("video_segmenter", "video_utils", "budget_planner"):
        (tmp_path / "utils" / f"{m}.py").write_text("ORIGINAL = True\n"
                                                     "def probe_duration(p): return -1.0\n"
                                                     "def extract_segment(*a, **k): return None\n"
                                                     "def load_or_create_manifest(**k): return None\n"
                                                     "def save_manifest(*a): return None\n"
                                                     "def update_segment_status(*a, **k): return None\n"
                                                     "def plan_segments_with_budget(*a): return None\n"
                                                     "class SegmentPlan: pass\n")
    (tmp_path / "analyzer").mkdir()
    (tmp_path / "analyzer" / "__init__.py").write_text("")
    (tmp_path / "analyzer" / "content_analyzer.py").write_text(textwrap.dedent("""
        from utils.budget_planner import SegmentPlan, plan_segments_with_budget
        from utils.video_segmenter import (
            extract_segment, load_or_create_manifest, save_manifest, update_segment_status)
        from utils.video_utils import probe_duration
    """))
    saved = {k: v for k, v in sys.modules.items() if k == "utils" or k.startswith(("utils.", "analyzer"))}
    for k in list(saved):
        del sys.modules[k]
    monkeypatch.syspath_prepend(str(tmp_path))
    try:
        ca = importlib.import_module("analyzer.content_analyzer")
        assert ca.probe_duration("x") == -1.0
        import vtseg.dropin as dropin
        from vtseg import video_segmenter, video_utils
        bound = dropin.install()
        assert "analyzer.content_analyzer.probe_duration" in bound
        assert ca.probe_duration is video_utils.probe_duration
        assert ca.extract_segment is video_segmenter.extract_segment
        assert sys.modules["utils.video_segmenter"] is video_segmenter
        assert sys.modules["utils"].video_segmenter is video_segmenter
        from utils.video_segmenter import plan_segments  # resolves to the build
        assert plan_segments is video_segmenter.plan_segments
    finally:
        for k in [k for k in sys.modules if k == "utils" or k.startswith(("utils.", "analyzer"))]:
            del sys.modules[k]
        sys.modules.update(saved)


def test_install_upload_transcode_is_opt_in(tmp_path, monkeypatch):
    """install(upload_transcode=True) replaces ContentAnalyzer's
    _compress_video_for_upload (content_analyzer.py:167-236) with
    vtseg.upload's; the default leaves it alone."""
    (tmp_path / "analyzer").mkdir()
    (tmp_path / "analyzer" / "__init__.py").write_text("")
    (tmp_path / "analyzer" / "content_analyzer.py").write_text(textwrap.dedent("""
        class ContentAnalyzer:
            logger = None
            def _compress_video_for_upload(self, video_path):
                return "reference"
    """))
    saved = {k: v for k, v in sys.modules.items() if k == "utils" or k.startswith(("utils.", "analyzer"))}
    for k in list(saved):
        del sys.modules[k]
    monkeypatch.syspath_prepend(str(tmp_path))
    try:
        ca = importlib.import_module("analyzer.content_analyzer")
        import vtseg.dropin as dropin
        from vtseg import upload
        dropin.install()
        assert ca.ContentAnalyzer()._compress_video_for_upload("x") == "reference"
        seen = {}
        monkeypatch.setattr(upload, "compress_video_for_upload",
                            lambda p, logger=None: seen.setdefault("p", p))
        bound = dropin.install(upload_transcode=True)
        assert "analyzer.content_analyzer.ContentAnalyzer._compress_video_for_upload" in bound
        assert ca.ContentAnalyzer()._compress_video_for_upload("v.mp4") == "v.mp4"
    finally:
        for k in [k for k in sys.modules if k == "utils" or k.startswith(("utils.", "analyzer"))]:
            del sys.modules[k]
        sys.modules.update(saved)
