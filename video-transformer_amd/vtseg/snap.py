"""Opt-in keyframe / scene-aware segment boundaries.

The reference's ``snap_to_keyframe`` (src/utils/video_segmenter.py:157-159)
is an unused identity stub, and ``plan_segments`` (:42-83) cuts at fixed
times; ``extract_segment``'s stream copy then starts each file at the
keyframe at or before the cut (:118-136), so a segment's file holds up to a
GOP of video from the previous segment.  This module is where that stub's
intent is realised, strictly opt-in: nothing here runs unless a caller asks
(``video_segmenter.snap_to_keyframe(..., mode=...)``, ``create_manifest(...,
anchors=...)``, or ``long_video.snap`` in the driver config), so default
segment lists stay bit-identical to the reference's.

Anchors are either keyframes (the MP4 sync samples, ``vts_keyframe_pts``,
exact integer timestamps) or scene cuts (frames whose device-computed score
exceeds the threshold, ``scene.VideoScorer.scene_cut_times``).  A boundary
moves to the nearest anchor within ``max_shift`` seconds; boundaries stay
strictly increasing, otherwise the fixed-time boundary is kept.
"""
from __future__ import annotations

import ctypes as C
from bisect import bisect_left, bisect_right
from fractions import Fraction
from pathlib import Path
from typing import Iterable, Sequence

from . import _lib


def keyframe_times(video_path: str | Path) -> list[float]:
    """Presentation times (seconds, correctly rounded from the exact
    timestamp / timescale) of the first video track's keyframes."""
    lib = _lib.lib()
    n, ts = C.c_int64(0), C.c_int64(0)
    path = str(video_path).encode()
    rc = lib.vts_keyframe_pts(path, None, 0, C.byref(n), C.byref(ts))
    if rc != _lib.VTS_E_CAPACITY:
        _lib.check(rc)
    buf = (C.c_int64 * max(1, n.value))()
    _lib.check(lib.vts_keyframe_pts(path, buf, n.value, C.byref(n), C.byref(ts)))
    if ts.value <= 0:
        raise _lib.VtsegError(_lib.VTS_E_FORMAT, "track timescale <= 0")
    return [float(Fraction(int(buf[i]), ts.value)) for i in range(n.value)]


def snap_time(t: float, anchors: Sequence[float], max_shift: float,
              direction: str = "nearest") -> float:
    """The anchor nearest to ``t`` (ties: the earlier) within ``max_shift``
    seconds, or ``t``.  ``direction="floor"``: the latest anchor <= t (where
    a stream copy would start a file cut at t).  ``anchors`` sorted."""
    if direction not in ("nearest", "floor"):
        raise ValueError(f"direction must be 'nearest' or 'floor', not {direction!r}")
    if not anchors or max_shift < 0:
        return t
    if direction == "floor":
        i = bisect_right(anchors, t) - 1
        return anchors[i] if i >= 0 and t - anchors[i] <= max_shift else t
    i = bisect_left(anchors, t)
    best = None
    for j in (i - 1, i):
        if 0 <= j < len(anchors):
            d = abs(anchors[j] - t)
            if d <= max_shift and (best is None or d < abs(best - t)):
                best = anchors[j]
    return t if best is None else best


def plan_segments_snapped(duration: float, segment_seconds: float, overlap_seconds: float,
                          anchors: Iterable[float], *, max_shift: float,
                          direction: str = "nearest"):
    """``plan_segments`` (the reference's fixed windows), then every inner core
    boundary moved to an anchor per ``snap_time``; extract windows are
    recomputed from the moved cores with the reference's overlap rules
    (video_segmenter.py:57-68).  Same segment count as the fixed plan; a move
    that would not keep the boundaries strictly increasing is not made."""
    from .video_segmenter import SegmentInfo, plan_segments
    base = plan_segments(duration, segment_seconds, overlap_seconds)
    if len(base) < 2:
        return base
    a = sorted(float(x) for x in anchors)
    cores = [base[0].effective_start]
    for i, seg in enumerate(base[:-1]):
        b = seg.effective_end
        s = snap_time(b, a, max_shift, direction)
        # stay above the previous boundary and below the next fixed one
        cores.append(s if cores[-1] < s < base[i + 1].effective_end else b)
    cores.append(base[-1].effective_end)
    overlap = max(0.0, overlap_seconds)
    out = []
    for i in range(len(base)):
        cs, ce = cores[i], cores[i + 1]
        start = 0.0 if cs == 0 else max(0.0, cs - overlap)
        end = duration if ce >= duration else min(duration, ce + overlap)
        out.append(SegmentInfo(segment_id=i, start=start, end=end, effective_start=cs,
                               effective_end=ce))
    return out
