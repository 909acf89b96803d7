"""Drop-in for the reference ``utils.video_utils`` (src/utils/video_utils.py).

``probe_duration`` reads the ISO-BMFF ``moov`` box natively (libvtseg
``vts_probe_duration``) and returns the value ffprobe prints for
``-show_entries format=duration`` on such files:
``av_rescale(mvhd.duration, 1_000_000, mvhd.timescale) / 1e6`` (a fragmented
MP4 whose mvhd says 0: the longest track's fragment samples, same rounding).
For any other container it keeps the reference behaviour exactly: run ffprobe
with the reference's arguments and 15 s timeout.  Where the native parser has
no answer for an ISO-BMFF file (no ``mvhd``, a parse error, a zero duration)
it also falls back to that ffprobe command, so such files get ffprobe's value
as in the reference.  Like the reference it never raises and
returns 0.0 on any failure (video_utils.py:28-38).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

from . import _lib


def _ffprobe_duration(path: Path) -> float:
    # video_utils.py:9-38, for containers the native parser does not read
    cmd = ["ffprobe", "-v", "error", "-select_streams", "v:0", "-show_entries",
           "format=duration", "-of", "default=noprint_wrappers=1:nokey=1", str(path)]
    try:
        result = subprocess.run(cmd, capture_output=True, text=True, timeout=15)
    except (subprocess.TimeoutExpired, FileNotFoundError, OSError):
        return 0.0
    if result.returncode != 0:
        return 0.0
    try:
        return float((result.stdout or "").strip())
    except ValueError:
        return 0.0


def _is_isobmff(path: Path) -> bool:
    try:
        with open(path, "rb") as f:
            head = f.read(12)
    except OSError:
        return False
    return len(head) >= 8 and head[4:8] in (b"ftyp", b"moov", b"mdat", b"free",
                                             b"skip", b"wide", b"pnot")


def probe_duration(video_path: str | Path) -> float:
    path = Path(video_path)
    if not _is_isobmff(path):
        return _ffprobe_duration(path)
    seconds = C.c_double(0.0)
    _lib.lib().vts_probe_duration(str(path).encode(), C.byref(seconds))
    if seconds.value > 0.0:
        return float(seconds.value)
    # no native answer (the reason is in vts_last_error()): ffprobe decides
    return _ffprobe_duration(path)
