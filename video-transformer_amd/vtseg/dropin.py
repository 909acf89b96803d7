"""Install vtseg as the segmenter of a reference (shizhenneko/Video-Transformer)
checkout, without editing its sources.

    import sys; sys.path.insert(0, "<ref>/src"); sys.path.insert(0, "<repo>/video-transformer_amd")
    import vtseg.dropin; vtseg.dropin.install()
    from analyzer.content_analyzer import ContentAnalyzer   # now uses vtseg

install() binds this package's modules under the reference's module names
(``utils.video_segmenter``, ``utils.video_utils``, ``utils.budget_planner``)
and, if ``analyzer.content_analyzer`` is already imported, rebinds the names it
imported at module level (content_analyzer.py:27-34) — the same names the
reference's own tests patch.
"""
from __future__ import annotations

import sys

from . import budget_planner, video_segmenter, video_utils

MODULES = {
    "utils.video_segmenter": video_segmenter,
    "utils.video_utils": video_utils,
    "utils.budget_planner": budget_planner,
}
# names content_analyzer.py:27-34 imports from the segmenter modules
ANALYZER_NAMES = {
    "SegmentPlan": budget_planner.SegmentPlan,
    "plan_segments_with_budget": budget_planner.plan_segments_with_budget,
    "extract_segment": video_segmenter.extract_segment,
    "load_or_create_manifest": video_segmenter.load_or_create_manifest,
    "save_manifest": video_segmenter.save_manifest,
    "update_segment_status": video_segmenter.update_segment_status,
    "probe_duration": video_utils.probe_duration,
}


def install(upload_transcode: bool = False) -> list[str]:
    """Bind vtseg under the reference's names; returns what was bound.

    upload_transcode: also replace ContentAnalyzer._compress_video_for_upload
    (content_analyzer.py:167-236) with the GPU transcode (vtseg.upload;
    opt-in: its bytes differ from x264's)."""
    done = []
    for name, mod in MODULES.items():
        sys.modules[name] = mod
        done.append(name)
    pkg = sys.modules.get("utils")
    if pkg is not None:
        for name, mod in MODULES.items():
            setattr(pkg, name.split(".", 1)[1], mod)
    ca = sys.modules.get("analyzer.content_analyzer")
    if ca is not None:
        for attr, obj in ANALYZER_NAMES.items():
            if hasattr(ca, attr):
                setattr(ca, attr, obj)
                done.append(f"analyzer.content_analyzer.{attr}")
        if upload_transcode and hasattr(ca, "ContentAnalyzer"):
            from . import upload

            def _compress_video_for_upload(self, video_path):
                return upload.compress_video_for_upload(video_path, logger=self.logger)

            ca.ContentAnalyzer._compress_video_for_upload = _compress_video_for_upload
            done.append("analyzer.content_analyzer.ContentAnalyzer._compress_video_for_upload")
    return done
