"""Segmentation driver: the segmentation-facing slice of the reference's
``ContentAnalyzer`` (src/analyzer/content_analyzer.py), with the LLM I/O left
to a caller-supplied callback.

It reproduces, call for call, what the reference does around the segmenter:
    analyze_video             :560-581   probe -> budget plan -> gate
    _should_use_segmentation  :494-506
    _analyze_video_segments   :822-964   manifest loop, resume, gap notes
    _analyze_segment_range    :721-820   extract + recursive binary split on
                                         input-token overflow
    _format_timecode          :308-314
    _build_segment_prompt_parts :444-455
    _is_input_token_overflow_error :1367-1383
so the (start, end, prompt_start, prompt_end, file name) sequence the LLM layer
sees is identical to the reference's (tests/golden/driver_sequences.json).
Everything it calls is this package's drop-in: ``probe_duration``,
``plan_segments_with_budget``, ``load_or_create_manifest`` / ``save_manifest``
/ ``update_segment_status`` and ``extract_segment``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable

from .budget_planner import SegmentPlan, plan_segments_with_budget
from .video_segmenter import (extract_segment, load_or_create_manifest, save_manifest,
                              update_segment_status)
from .video_utils import probe_duration


class APILimitExceeded(RuntimeError):
    """Same role as the reference's utils.counter.APILimitExceeded."""


@dataclass
class APICounter:
    """Behaviour-compatible with the reference's utils/counter.py:10-73."""
    max_calls: int = 20
    current_count: int = 0
    hard_max_calls: int | None = None
    limit_exc: type = field(default=APILimitExceeded, repr=False)

    def _effective_max_calls(self) -> int:
        if self.hard_max_calls is None:
            return self.max_calls
        return min(self.max_calls, self.hard_max_calls)

    def set_max_calls(self, max_calls: int, hard_max_calls: int | None = None) -> int:
        if hard_max_calls is not None:
            self.hard_max_calls = hard_max_calls
        effective_hard = self.hard_max_calls if self.hard_max_calls is not None else max_calls
        self.max_calls = min(max_calls, effective_hard)
        return self.max_calls

    def increment(self, service: str) -> bool:
        if service.lower() == "gemini":
            limit = self._effective_max_calls()
            if self.current_count >= limit:
                raise self.limit_exc(f"Gemini API call limit reached: {self.current_count}/{limit}")
            self.current_count += 1
        return True

    def can_call(self) -> bool:
        return self.current_count < self._effective_max_calls()

    def remaining(self) -> int:
        return max(self._effective_max_calls() - self.current_count, 0)


def format_timecode(seconds: float) -> str:
    total = max(int(seconds), 0)
    return f"{total // 3600:02d}:{(total % 3600) // 60:02d}:{total % 60:02d}"


def build_segment_prompt_parts(segment_index: int, total_segments: int, start: float,
                               end: float) -> list[str]:
    return [
        f"This is segment {segment_index} of {total_segments}, "
        f"covering time range {format_timecode(start)} to {format_timecode(end)}. "
        "Output timestamps as absolute video time (HH:MM:SS or milliseconds). "
        "Structure deep_dive as a single chapter with chapter_title indicating the time range."
    ]


def is_input_token_overflow_error(exc: Exception) -> bool:
    msg = str(exc).lower()
    return ("400" in msg and "invalid_argument" in msg
            and "input token count exceeds" in msg and "1048576" in msg)


def _coerce_float(value: object) -> float | None:
    if isinstance(value, (int, float, str)):
        try:
            return float(value)
        except ValueError:
            return None
    return None


# analyze(segment_path, extra_text_parts) -> response data; it is the LLM call
# (the reference's _upload_video + _call_analysis_json, which also counts the
# call on the APICounter).
AnalyzeFn = Callable[[Path, list], Any]


@dataclass
class SegmentationResult:
    outcome: str                      # "segmented" | "single_pass"
    duration: float
    plan: SegmentPlan
    segment_outputs: list[dict] = field(default_factory=list)
    gap_notes: list[str] = field(default_factory=list)
    total_segments: int = 0

    @property
    def metadata(self) -> dict:
        return {"duration": self.duration, "segments": self.total_segments,
                "segment_gaps": self.gap_notes}


class SegmentationDriver:
    def __init__(self, config: dict, api_counter, analyze: AnalyzeFn, *,
                 probe: Callable = probe_duration, extract: Callable = extract_segment,
                 limit_exc: type | tuple = APILimitExceeded,
                 scene_anchors: Callable[[Path], list[float]] | None = None):
        self.scene_anchors = scene_anchors  # opt-in `snap: scene` (e.g. scene.scene_cut_times)
        self.config = config
        self.analyzer_config = config.get("analyzer", {})
        self.api_counter = api_counter
        self.analyze = analyze
        self.probe = probe
        self.extract = extract
        self.limit_exc = limit_exc

    # content_analyzer.py:494-506
    def should_use_segmentation(self, duration: float, plan: SegmentPlan,
                                long_video_config: dict) -> bool:
        if duration <= 0:
            return False
        if not long_video_config.get("enabled", True):
            return False
        threshold = _coerce_float(long_video_config.get("duration_threshold_seconds"))
        if threshold is not None and duration >= threshold:
            return True
        return plan.num_segments > 1

    # content_analyzer.py:560-581
    def run(self, video_path: str | Path) -> SegmentationResult:
        video_path = Path(video_path)
        if not video_path.exists():
            raise FileNotFoundError(f"视频文件不存在: {video_path}")
        duration = self.probe(video_path)
        long_video_config = self.analyzer_config.get("long_video", {})
        plan = plan_segments_with_budget(duration, self.config, self.api_counter.current_count)
        if self.should_use_segmentation(duration, plan, long_video_config):
            return self.analyze_video_segments(video_path, duration, plan)
        return SegmentationResult("single_pass", duration, plan)

    # content_analyzer.py:721-820
    def analyze_segment_range(self, *, video_path: Path, segment_id: int, segment_index: int,
                              total_segments: int, start: float, end: float,
                              prompt_start: float, prompt_end: float, segment_dir: Path,
                              segment_path: Path | None,
                              min_segment_seconds: float) -> list[dict]:
        duration = end - start
        if duration <= 0:
            return []
        if not self.api_counter.can_call():
            raise self._limit("API 调用次数不足，停止分段分析")
        if segment_path is None:
            segment_path = segment_dir / (
                f"segment_{segment_id:04d}_{int(start * 1000):010d}_{int(end * 1000):010d}.mp4")
        if not segment_path.exists() or segment_path.stat().st_size <= 0:
            if not self.extract(input_path=video_path, start=start, end=end,
                                output_path=segment_path, stream_copy=True):
                raise RuntimeError("分段视频切割失败")
        try:
            parts = build_segment_prompt_parts(segment_index, total_segments, prompt_start,
                                               prompt_end)
            data = self.analyze(segment_path, parts)
            return [{"start": prompt_start, "end": prompt_end, "data": data}]
        except Exception as exc:
            if is_input_token_overflow_error(exc):
                if duration / 2 < min_segment_seconds:
                    raise
                mid = (start + end) / 2
                common = dict(video_path=video_path, segment_id=segment_id,
                              segment_index=segment_index, total_segments=total_segments,
                              segment_dir=segment_dir, segment_path=None,
                              min_segment_seconds=min_segment_seconds)
                left = self.analyze_segment_range(start=start, end=mid, prompt_start=start,
                                                  prompt_end=mid, **common)
                right = self.analyze_segment_range(start=mid, end=end, prompt_start=mid,
                                                   prompt_end=end, **common)
                return left + right
            raise

    def _snap_args(self, video_path: Path, long_video_config: dict,
                   segment_seconds: float) -> dict:
        """Opt-in segment boundaries on keyframes / scene cuts (vtseg.snap;
        SURVEY §8f-3): ``long_video.snap`` = "keyframe" | "scene", moving each
        boundary by at most ``snap_max_shift_seconds`` (default a tenth of a
        segment).  Absent (the reference config): no extra arguments, so the
        manifest call and the segment list are the reference's."""
        mode = long_video_config.get("snap")
        if not mode:
            return {}
        shift = _coerce_float(long_video_config.get("snap_max_shift_seconds"))
        if shift is None:
            shift = 0.1 * float(segment_seconds)
        if mode == "keyframe":
            from .snap import keyframe_times
            anchors = keyframe_times(video_path)
        elif mode == "scene":
            if self.scene_anchors is None:
                raise ValueError("long_video.snap = 'scene' needs a scene_anchors callable "
                                 "(e.g. vtseg.scene.scene_cut_times)")
            anchors = self.scene_anchors(video_path)
        else:
            raise ValueError(f"long_video.snap must be 'keyframe' or 'scene', not {mode!r}")
        return {"anchors": anchors, "max_shift": shift}

    def _limit(self, msg: str) -> Exception:
        exc = self.limit_exc[0] if isinstance(self.limit_exc, tuple) else self.limit_exc
        return exc(msg)

    # content_analyzer.py:822-964 (merge/consolidation of LLM output excluded)
    def analyze_video_segments(self, video_path: Path, duration: float,
                               plan: SegmentPlan) -> SegmentationResult:
        if duration <= 0:
            raise RuntimeError("无法获取视频时长，无法分段分析")
        long_video_config = self.analyzer_config.get("long_video", {})
        segment_seconds = plan.segment_duration
        overlap_seconds = plan.overlap
        if segment_seconds <= 0:
            segment_seconds = int(long_video_config.get("min_segment_seconds") or 90)
            overlap_seconds = 0
        min_segment_seconds = float(long_video_config.get("min_segment_seconds") or 90)
        if plan.hard_max_calls:
            self.api_counter.set_max_calls(self.api_counter.max_calls, plan.hard_max_calls)
        if not self.api_counter.can_call():
            raise self._limit("API 调用次数不足以执行分段分析")

        temp_dir = self.config.get("system", {}).get("temp_dir", "./data/temp")
        video_id = video_path.stem
        manifest = load_or_create_manifest(video_id=video_id, duration=duration,
                                           segment_seconds=segment_seconds,
                                           overlap_seconds=overlap_seconds, temp_dir=temp_dir,
                                           **self._snap_args(video_path, long_video_config,
                                                             segment_seconds))
        segment_dir = Path(temp_dir) / "segments" / video_id
        manifest_path = segment_dir / "manifest.json"
        segments = sorted(manifest["segments"], key=lambda item: item["id"])
        total = len(segments)
        if total == 0:
            raise RuntimeError("无法生成分段计划，缺少可分析的片段")

        def span(item) -> str:
            s = float(item.get("effective_start", item["start"]))
            e = float(item.get("effective_end", item["end"]))
            return f"{format_timecode(s)}-{format_timecode(e)}"

        outputs: list[dict] = []
        gaps: list[str] = []
        for entry in segments:
            sid = entry["id"]
            eff_start = float(entry.get("effective_start", entry["start"]))
            eff_end = float(entry.get("effective_end", entry["end"]))
            if not self.api_counter.can_call():
                gaps.append(f"{format_timecode(eff_start)}-{format_timecode(eff_end)}")
                gaps.extend(span(it) for it in segments if it["id"] > sid)
                break
            update_segment_status(manifest, sid, "processing", increment_attempts=True)
            save_manifest(manifest_path, manifest)
            try:
                results = self.analyze_segment_range(
                    video_path=video_path, segment_id=sid, segment_index=sid + 1,
                    total_segments=total, start=float(entry["start"]), end=float(entry["end"]),
                    prompt_start=eff_start, prompt_end=eff_end, segment_dir=segment_dir,
                    segment_path=Path(entry["file_path"]),
                    min_segment_seconds=min_segment_seconds)
                if results:
                    outputs.extend(results)
                    update_segment_status(manifest, sid, "completed")
                else:
                    update_segment_status(manifest, sid, "failed", error="segment returned empty")
                    gaps.append(f"{format_timecode(eff_start)}-{format_timecode(eff_end)}")
            except self.limit_exc:
                update_segment_status(manifest, sid, "skipped", error="api budget exhausted")
                gaps.append(f"{format_timecode(eff_start)}-{format_timecode(eff_end)}")
                gaps.extend(span(it) for it in segments if it["id"] > sid)
                break
            except Exception as exc:
                update_segment_status(manifest, sid, "failed", error=str(exc))
                gaps.append(f"{format_timecode(eff_start)}-{format_timecode(eff_end)}")
            finally:
                save_manifest(manifest_path, manifest)
        if not outputs:
            raise RuntimeError("分段分析失败，未获得任何有效结果")
        return SegmentationResult("segmented", duration, plan, outputs, gaps, total)
