"""Upload compression: drop-in for ContentAnalyzer._compress_video_for_upload
(reference src/analyzer/content_analyzer.py:167-236).

The reference shrinks a video larger than 30 MB before uploading it with
``ffmpeg -y -i IN -vf scale=-2:360 -c:v libx264 -crf 28 -preset fast -c:a aac
-b:a 64k compressed_<name>`` and falls back to the original path when ffmpeg
is missing, fails or times out.  Here the pixel work runs on the MI355X
(``VideoScorer.transcode`` -> ``vts_transcode``: device decode, area
downscale to scale=-2:360, device H.264 encode).  Streams
outside the device decoder's subset, or a GPU failure, take the reference's
own ffmpeg command when ffmpeg exists, and otherwise the reference's
fallback: the original path.  The source's audio (every non-video track)
is stream-copied into the output (``vts_add_tracks``): the reference
re-encodes it to AAC 64k, here it keeps its original coding (no AAC encoder in
the image), so the uploaded file still has the sound track.
"""
from __future__ import annotations

import logging
import shutil
import subprocess
from pathlib import Path

from ._lib import VtsegError, VtsegLibraryError

MAX_SIZE_MB = 30  # content_analyzer.py:174


def compressed_path_for(video_path: Path) -> Path:
    """content_analyzer.py:185 naming."""
    return video_path.parent / f"compressed_{video_path.name}"


def _ffmpeg(video_path: Path, out: Path, logger: logging.Logger) -> Path:
    """The reference's command and fallbacks (content_analyzer.py:191-236)."""
    cmd = ["ffmpeg", "-y", "-i", str(video_path), "-vf", "scale=-2:360", "-c:v", "libx264",
           "-crf", "28", "-preset", "fast", "-c:a", "aac", "-b:a", "64k", str(out)]
    try:
        result = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    except FileNotFoundError:
        logger.warning("ffmpeg not installed; skipping compression")
        return video_path
    except subprocess.TimeoutExpired:
        logger.warning("ffmpeg compression timed out (5 min); skipping compression")
        if out.exists():
            out.unlink()
        return video_path
    if result.returncode != 0:
        logger.warning(f"ffmpeg compression failed: {(result.stderr or '')[:200]}")
        return video_path
    return out


def compress_video_for_upload(video_path: Path, *, logger: logging.Logger | None = None,
                              device: int = 0, max_size_mb: float = MAX_SIZE_MB) -> Path:
    """Same decisions and return values as the reference method: the input
    path when it is <= 30 MB, an existing non-empty compressed_<name> as is,
    otherwise the new compressed file, or the input path when compression
    is impossible."""
    log = logger or logging.getLogger(__name__)
    video_path = Path(video_path)
    file_size_mb = video_path.stat().st_size / (1024 * 1024)
    if file_size_mb <= max_size_mb:
        log.info(f"video {file_size_mb:.1f}MB <= {max_size_mb}MB, skipping compression")
        return video_path
    log.info(f"video {file_size_mb:.1f}MB > {max_size_mb}MB, compressing on the GPU...")
    out = compressed_path_for(video_path)
    if out.exists() and out.stat().st_size > 0:
        log.info(f"found existing compressed file {out.name}, skipping compression")
        return out
    video_only = out.with_name(out.name + ".video.tmp")
    try:
        from . import _lib
        from .scene import VideoScorer
        with VideoScorer(video_path, device=device) as v:
            facts = v.transcode(video_only)
        # the source's audio / other tracks, stream-copied beside the new video
        _lib.check(_lib.lib().vts_add_tracks(str(video_only).encode(),
                                             str(video_path).encode(), str(out).encode()))
        video_only.unlink()
        facts["bytes_written"] = out.stat().st_size
    except (VtsegError, VtsegLibraryError, OSError) as exc:
        for p in (out, video_only):
            if p.exists():
                p.unlink()
        log.warning(f"GPU transcode unavailable ({exc}); using ffmpeg")
        if shutil.which("ffmpeg") is None:
            log.warning("ffmpeg not installed; skipping compression")
            return video_path
        return _ffmpeg(video_path, out, log)
    new_size_mb = facts["bytes_written"] / (1024 * 1024)
    log.info(f"compressed: {file_size_mb:.1f}MB -> {new_size_mb:.1f}MB "
             f"({new_size_mb / file_size_mb * 100:.0f}%)")
    return out
