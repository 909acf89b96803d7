"""Drop-in for the reference ``utils.video_segmenter`` (src/utils/video_segmenter.py).

Same public names, signatures, types and error conventions as the reference
module; the planning arithmetic runs in libvtseg (C++, bit-exact) through
``vtseg._lib``.  Manifest persistence stays plain JSON with the reference's
exact formatting (``indent=2, ensure_ascii=True``) so an existing manifest is
resumable by either implementation.

Reference map:
    SegmentInfo / SegmentEntry / SegmentManifest   video_segmenter.py:12-39
    plan_segments                                  video_segmenter.py:42-83
    extract_segment                                video_segmenter.py:86-154
    snap_to_keyframe                               video_segmenter.py:157-159
    get_segment_dir / get_manifest_path            video_segmenter.py:162-167
    create_manifest / load_manifest / save_manifest / load_or_create_manifest
                                                   video_segmenter.py:170-238
    pending_segments / update_segment_status       video_segmenter.py:241-266
"""
from __future__ import annotations

import ctypes as C
import json
import logging
import numbers
import subprocess
from dataclasses import dataclass
from datetime import datetime, timezone
from pathlib import Path
from typing import TypedDict, cast

from . import _lib
from .video_utils import _is_isobmff


@dataclass(frozen=True)
class SegmentInfo:
    segment_id: int
    start: float
    end: float
    effective_start: float
    effective_end: float


class SegmentEntry(TypedDict):
    id: int
    start: float
    end: float
    effective_start: float
    effective_end: float
    file_path: str
    status: str
    attempts: int
    error: str | None


class SegmentManifest(TypedDict):
    version: int
    video_id: str
    created_at: str
    segment_seconds: float
    overlap_seconds: float
    segments: list[SegmentEntry]


def _as_real(name: str, value: object) -> float:
    """float(value) for the real-number types the reference accepts.

    The reference compares its arguments with ``<=``/``<`` and adds them to
    floats, so non-numbers raise TypeError there; they do here too.
    """
    if isinstance(value, numbers.Real):
        return float(value)
    raise TypeError(
        f"'<=' not supported between instances of '{type(value).__name__}' and 'int'"
        f" ({name})")


def plan_segments(
    duration: float, segment_seconds: float, overlap_seconds: float
) -> list[SegmentInfo]:
    """Fixed windows with overlap on the inner sides (video_segmenter.py:42-83).

    Runs ``vts_plan_segments`` in libvtseg.  Raises ``vtseg.NonTerminatingError``
    where the reference loop would never end (e.g. duration = +inf).
    """
    d = _as_real("duration", duration)
    s = _as_real("segment_seconds", segment_seconds)
    o = _as_real("overlap_seconds", overlap_seconds)
    lib = _lib.lib()
    n = C.c_int64(0)
    cap = 64
    while True:
        buf = (_lib.Segment * cap)()
        rc = lib.vts_plan_segments(d, s, o, buf, cap, C.byref(n))
        if rc == _lib.VTS_E_CAPACITY:
            cap = int(n.value)
            continue
        _lib.check(rc)
        break
    # The reference returns the caller's own `duration` object in two places
    # (min()/ternary picks it); keep that for int durations.
    keep = isinstance(duration, int)
    out: list[SegmentInfo] = []
    for i in range(int(n.value)):
        g = buf[i]
        out.append(SegmentInfo(
            segment_id=int(g.segment_id),
            start=g.start,
            end=duration if keep and (g.flags & 1) else g.end,
            effective_start=g.effective_start,
            effective_end=duration if keep and (g.flags & 2) else g.effective_end,
        ))
    return out


def extract_segment(
    input_path: str | Path,
    start: float,
    end: float,
    output_path: str | Path,
    stream_copy: bool = True,
) -> bool:
    """Cut [start, end] into output_path (video_segmenter.py:86-154).

    Same contract as the reference: never raises, False on any failure, a
    failed copy's partial output is unlinked, copy first then re-encode.  The
    stream copy of ISO-BMFF input is native (``vts_extract_segment``: from
    the keyframe at or before ``start``, moov first, like ``ffmpeg -ss S -i IN
    -t D -movflags +faststart -c copy``); other containers, a failed native
    copy and the re-encode fallback run the reference's ffmpeg commands
    (``%.3f`` timestamps, 120 s timeout).
    """
    duration = end - start
    if duration <= 0:
        return False

    input_path = Path(input_path)
    output_path = Path(output_path)
    output_path.parent.mkdir(parents=True, exist_ok=True)

    def run(args: list[str]) -> bool:
        try:
            proc = subprocess.run(args, capture_output=True, text=True, timeout=120)
        except (FileNotFoundError, OSError, subprocess.TimeoutExpired):
            return False
        return (proc.returncode == 0 and output_path.exists()
                and output_path.stat().st_size > 0)

    if stream_copy:
        if _is_isobmff(input_path):
            try:
                rc = _lib.lib().vts_extract_segment(str(input_path).encode(), float(start),
                                                    float(end), str(output_path).encode())
            except (TypeError, ValueError):
                rc = -1
            if rc == 0 and output_path.exists() and output_path.stat().st_size > 0:
                return True
            if output_path.exists():
                output_path.unlink()

    head = ["ffmpeg", "-y", "-hide_banner", "-loglevel", "error",
            "-ss", f"{start:.3f}", "-i", str(input_path),
            "-t", f"{duration:.3f}", "-movflags", "+faststart"]
    if stream_copy:
        if run(head + ["-c", "copy", str(output_path)]):
            return True
        if output_path.exists():
            output_path.unlink()
    return run(head + ["-c:v", "libx264", "-preset", "veryfast", "-crf", "23",
                       "-c:a", "aac", "-b:a", "128k", str(output_path)])


def snap_to_keyframe(video_path: str | Path, timestamp: float, *, mode: str = "identity",
                     anchors: list[float] | None = None, max_shift: float = float("inf"),
                     direction: str = "nearest") -> float:
    """Identity clamp by default, exactly as the reference stub
    (video_segmenter.py:157-159), so segment lists stay bit-identical.

    Opt-in (vtseg.snap): ``mode="keyframe"`` snaps to the file's keyframes
    (MP4 sync samples), ``mode="anchors"`` to caller-given times (e.g. scene
    cuts from ``scene.VideoScorer``), the nearest within ``max_shift``
    seconds (``direction="floor"``: the latest at or before).
    """
    t = max(0.0, float(timestamp))
    if mode == "identity":
        return t
    from . import snap
    if mode == "keyframe":
        anchors = snap.keyframe_times(video_path)
    elif mode != "anchors" or anchors is None:
        raise ValueError("mode must be 'identity', 'keyframe' or 'anchors' (with anchors)")
    return max(0.0, snap.snap_time(t, sorted(anchors), max_shift, direction))


def get_segment_dir(video_id: str, temp_dir: str | Path) -> Path:
    return Path(temp_dir) / "segments" / video_id


def get_manifest_path(video_id: str, temp_dir: str | Path) -> Path:
    return get_segment_dir(video_id, temp_dir) / "manifest.json"


def create_manifest(
    *,
    video_id: str,
    duration: float,
    segment_seconds: float,
    overlap_seconds: float,
    temp_dir: str | Path,
    anchors: list[float] | None = None,
    max_shift: float = 0.0,
) -> SegmentManifest:
    """The reference's create_manifest (video_segmenter.py:170-205).  Opt-in:
    ``anchors`` (keyframe or scene-cut times) move the inner boundaries by up
    to ``max_shift`` seconds (vtseg.snap.plan_segments_snapped)."""
    segment_dir = get_segment_dir(video_id, temp_dir)
    segment_dir.mkdir(parents=True, exist_ok=True)
    entries: list[SegmentEntry] = []
    if anchors is None:
        plan = plan_segments(duration, segment_seconds, overlap_seconds)
    else:
        from .snap import plan_segments_snapped
        plan = plan_segments_snapped(duration, segment_seconds, overlap_seconds, anchors,
                                     max_shift=max_shift)
    for seg in plan:
        entries.append({
            "id": seg.segment_id,
            "start": seg.start,
            "end": seg.end,
            "effective_start": seg.effective_start,
            "effective_end": seg.effective_end,
            "file_path": str(segment_dir / f"segment_{seg.segment_id:04d}.mp4"),
            "status": "pending",
            "attempts": 0,
            "error": None,
        })
    manifest: SegmentManifest = {
        "version": 1,
        "video_id": video_id,
        "created_at": datetime.now(timezone.utc).isoformat(),
        "segment_seconds": segment_seconds,
        "overlap_seconds": overlap_seconds,
        "segments": entries,
    }
    path = get_manifest_path(video_id, temp_dir)
    text = None if anchors is not None else manifest_json(
        video_id=video_id, duration=duration, segment_seconds=segment_seconds,
        overlap_seconds=overlap_seconds, segment_dir=segment_dir,
        created_at=manifest["created_at"])
    if text is None:  # objects only Python's json knows how to print (or refuse)
        save_manifest(path, manifest)
    else:
        path.parent.mkdir(parents=True, exist_ok=True)
        _ = path.write_text(text, encoding="utf-8")
    return manifest


def _num_arg(value: object) -> tuple[float, bytes | None] | None:
    """(double, int repr) for the number types the native writer prints the
    way json.dumps does: int (not bool) and float; None for anything else."""
    if isinstance(value, bool):
        return None
    if type(value) is int:
        return float(value) if abs(value) < 2 ** 1023 else float("inf"), str(value).encode()
    if isinstance(value, float):
        return float(value), None
    return None


def manifest_json(*, video_id: str, duration: float, segment_seconds: float,
                  overlap_seconds: float, segment_dir: str | Path,
                  created_at: str) -> str | None:
    """The text create_manifest + save_manifest write
    (video_segmenter.py:170-218: ``json.dumps(manifest, indent=2,
    ensure_ascii=True)``), produced natively by ``vts_manifest_json``.
    None when an argument is not a plain int/float/str the native writer
    prints exactly like json (the caller then uses Python's json)."""
    nums = [_num_arg(v) for v in (duration, segment_seconds, overlap_seconds)]
    if any(n is None for n in nums) or not all(
            isinstance(x, str) for x in (video_id, created_at)):
        return None
    try:
        sid, sdir, sca = (x.encode("utf-8") for x in (video_id, str(segment_dir), created_at))
    except UnicodeEncodeError:  # lone surrogates (undecodable file names)
        return None
    (d, di), (sg, sgi), (ov, ovi) = nums  # type: ignore[misc]
    args = _lib.ManifestArgs(sid, sdir, sca, d, di, sg, sgi, ov, ovi)
    lib = _lib.lib()
    n = C.c_int64(0)
    rc = lib.vts_manifest_json(C.byref(args), None, 0, C.byref(n))
    if rc != _lib.VTS_E_CAPACITY:
        _lib.check(rc)
    buf = C.create_string_buffer(int(n.value) + 1)
    _lib.check(lib.vts_manifest_json(C.byref(args), buf, n.value + 1, C.byref(n)))
    return buf.raw[: n.value].decode("ascii")


def load_manifest(manifest_path: str | Path) -> SegmentManifest:
    return cast(SegmentManifest,
                json.loads(Path(manifest_path).read_text(encoding="utf-8")))


def save_manifest(manifest_path: str | Path, manifest: SegmentManifest) -> None:
    path = Path(manifest_path)
    path.parent.mkdir(parents=True, exist_ok=True)
    _ = path.write_text(json.dumps(manifest, indent=2, ensure_ascii=True),
                        encoding="utf-8")


def load_or_create_manifest(
    *,
    video_id: str,
    duration: float,
    segment_seconds: float,
    overlap_seconds: float,
    temp_dir: str | Path,
    anchors: list[float] | None = None,
    max_shift: float = 0.0,
) -> SegmentManifest:
    manifest_path = get_manifest_path(video_id, temp_dir)
    if manifest_path.exists():  # resume: reuse the persisted plan verbatim
        return load_manifest(manifest_path)
    return create_manifest(video_id=video_id, duration=duration,
                           segment_seconds=segment_seconds,
                           overlap_seconds=overlap_seconds, temp_dir=temp_dir,
                           anchors=anchors, max_shift=max_shift)


def pending_segments(manifest: SegmentManifest) -> list[SegmentEntry]:
    return [seg for seg in manifest["segments"] if seg["status"] != "completed"]


def update_segment_status(
    manifest: SegmentManifest,
    segment_id: int,
    status: str,
    *,
    error: str | None = None,
    increment_attempts: bool = False,
) -> None:
    for seg in manifest["segments"]:
        if seg["id"] == segment_id:
            seg["status"] = status
            if error is not None:
                seg["error"] = error
            if increment_attempts:
                seg["attempts"] = seg["attempts"] + 1
            return
    logging.getLogger(__name__).warning("Segment id %s not found in manifest", segment_id)
