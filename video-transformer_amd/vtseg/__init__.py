"""vtseg — MI355X-native long-video segmenter (drop-in for the segmenter path of
shizhenneko/Video-Transformer).

Drop-in modules (same names/signatures as the reference's ``src/utils``):
    vtseg.video_segmenter   utils/video_segmenter.py
    vtseg.video_utils       utils/video_utils.py
    vtseg.budget_planner    utils/budget_planner.py
Analyzer-slice mirror (segmentation-facing control flow of
``ContentAnalyzer``, content_analyzer.py:494-964):
    vtseg.driver
GPU scene scoring (decode + NV12 scoring on gfx950):
    vtseg.scene
Installing the drop-in into a reference checkout:
    vtseg.dropin.install()
"""
from ._lib import (NonTerminatingError, VtsegError, VtsegLibraryError,  # noqa: F401
                   lib)

__all__ = ["NonTerminatingError", "VtsegError", "VtsegLibraryError", "lib"]
