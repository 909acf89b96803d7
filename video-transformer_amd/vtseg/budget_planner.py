"""Drop-in for the reference ``utils.budget_planner`` (src/utils/budget_planner.py).

Config lookup and the Python-object coercions (``_coerce_int``,
``_coerce_bool``, ``float(threshold)``; budget_planner.py:20-40, 82-103) stay
on the Python side because they are defined by Python's ``int()``/``float()``
on arbitrary objects; the arithmetic of plan_segments_with_budget
(budget_planner.py:104-194, including ``_estimate_segments`` /
``_estimate_calls`` at :43-70) runs in libvtseg (``vts_plan_with_budget``).
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Mapping
from dataclasses import dataclass
from typing import cast

from . import _lib


@dataclass(frozen=True)
class SegmentPlan:
    segment_duration: int
    overlap: int
    num_segments: int
    estimated_calls: int
    available_calls: int
    hard_max_calls: int
    fits_budget: bool


def _coerce_int(value: object, default: int) -> int:
    if isinstance(value, (int, float, str)):
        try:
            return int(value)
        except ValueError:
            return default
    return default


def _coerce_bool(value: object, default: bool) -> bool:
    if isinstance(value, bool):
        return value
    if isinstance(value, (int, float)):
        return bool(value)
    if isinstance(value, str):
        normalized = value.strip().lower()
        if normalized in {"true", "1", "yes", "y", "on"}:
            return True
        if normalized in {"false", "0", "no", "n", "off"}:
            return False
    return default


_INT64_MIN, _INT64_MAX = -(1 << 63), (1 << 63) - 1


def _i64(name: str, v: int) -> int:
    if not (_INT64_MIN <= v <= _INT64_MAX):
        raise OverflowError(f"{name}={v} outside the int64 range of the native planner")
    return v


_ERRORS = {
    _lib.VTS_E_VALUE: ValueError,
    _lib.VTS_E_OVERFLOW: OverflowError,
    _lib.VTS_E_ZERODIV: ZeroDivisionError,
    _lib.VTS_E_RANGE: OverflowError,
}


def budget_cfg(config: Mapping[str, object]) -> "_lib.BudgetCfg":
    """The reference's config coercion (budget_planner.py:95-103) as the C
    ABI's vts_budget_cfg (also vts_batch_run's planning input)."""
    analyzer_raw = config.get("analyzer")
    analyzer = cast(dict[str, object], analyzer_raw) if isinstance(analyzer_raw, dict) else {}
    lv_raw = analyzer.get("long_video")
    lv = cast(dict[str, object], lv_raw) if isinstance(lv_raw, dict) else {}

    cfg = _lib.BudgetCfg()
    cfg.default_segment_seconds = _i64("default_segment_seconds",
                                       _coerce_int(lv.get("default_segment_seconds"), 480))
    cfg.overlap_seconds = _i64("overlap_seconds", _coerce_int(lv.get("overlap_seconds"), 20))
    cfg.min_segment_seconds = _i64("min_segment_seconds",
                                   _coerce_int(lv.get("min_segment_seconds"), 90))
    cfg.hard_max_api_calls = _i64("hard_max_api_calls",
                                  _coerce_int(lv.get("hard_max_api_calls"), 50))
    cfg.max_continuations = _i64("max_continuations",
                                 _coerce_int(analyzer.get("max_continuations"), 3))
    cfg.retry_times = _i64("retry_times", _coerce_int(analyzer.get("retry_times"), 0))
    threshold_raw = lv.get("duration_threshold_seconds")
    cfg.consolidate = 1 if _coerce_bool(lv.get("consolidate"), True) else 0

    threshold = None
    if isinstance(threshold_raw, (int, float, str)):
        try:
            threshold = float(threshold_raw)
        except ValueError:
            threshold = None
    cfg.has_threshold = 0 if threshold is None else 1
    cfg.duration_threshold_seconds = 0.0 if threshold is None else threshold
    return cfg


def plan_segments_with_budget(
    duration: float,
    config: Mapping[str, object],
    current_api_count: int,
) -> SegmentPlan:
    cfg = budget_cfg(config)
    duration_f = float(duration)  # reference: max(float(duration), 0.0) at :104
    count = _i64("current_api_count", int(current_api_count))

    out = _lib.Plan()
    rc = _lib.lib().vts_plan_with_budget(duration_f, C.byref(cfg), count, C.byref(out))
    if rc in _ERRORS:
        raise _ERRORS[rc](_lib.last_error())
    _lib.check(rc)
    return SegmentPlan(
        segment_duration=int(out.segment_duration),
        overlap=int(out.overlap),
        num_segments=int(out.num_segments),
        estimated_calls=int(out.estimated_calls),
        available_calls=int(out.available_calls),
        hard_max_calls=int(out.hard_max_calls),
        fits_budget=bool(out.fits_budget),
    )


__all__ = ["SegmentPlan", "plan_segments_with_budget", "budget_cfg", "_coerce_int", "_coerce_bool"]
