"""Product planner (vtseg -> libvtseg C++) vs the reference's golden vectors.

Bit-exact: every float is compared through float.hex (tests/golden/*.json were
captured from the reference by tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import pytest

from conftest import fhex, load_golden, same_float
from vtseg import NonTerminatingError, VtsegError
from vtseg import budget_planner as bp
from vtseg import video_segmenter as vs


def _arg(hexval: str, is_int: bool):
    v = fhex(hexval)
    return int(v) if is_int else v


def test_plan_segments_bit_exact_vs_reference():
    cases = load_golden("plan_segments.json")
    for c in cases:
        d = fhex(c["duration"])
        s = _arg(c["segment_seconds"], c["segment_is_int"])
        o = _arg(c["overlap_seconds"], c["overlap_is_int"])
        got = vs.plan_segments(d, s, o)
        exp = c["segments"]
        assert len(got) == len(exp), c
        for g, e in zip(got, exp):
            assert g.segment_id == e[0]
            for gv, ev in zip((g.start, g.end, g.effective_start, g.effective_end), e[1:]):
                assert isinstance(gv, float)
                assert same_float(gv, fhex(ev)), (c, g, e)


def test_plan_segments_returns_callers_int_duration_like_reference():
    # reference: min(cursor + seg, duration) / `extract_end = duration` hand back
    # the caller's object (video_segmenter.py:55, 63)
    segs = vs.plan_segments(100, 30, 5)
    assert segs[-1].end == 100 and type(segs[-1].end) is int
    assert type(segs[-1].effective_end) is int
    assert type(segs[0].end) is float


def test_plan_segments_fp_accumulation_case():
    segs = vs.plan_segments(1.0, 0.1, 0)
    assert len(segs) == 11
    assert segs[-1].start == 0.9999999999999999 and segs[-1].end == 1.0


def test_plan_segments_nonterminating_inputs_raise():
    with pytest.raises(NonTerminatingError):
        vs.plan_segments(float("inf"), 30.0, 0.0)
    # the reference would build a 2^55-element list; the native planner refuses
    with pytest.raises(VtsegError):
        vs.plan_segments(2.0 ** 60, 2.0 ** 5, 0.0)


def test_plan_segments_type_errors_like_reference():
    with pytest.raises(TypeError):
        vs.plan_segments("600", 30.0, 0.0)


def test_budget_plans_match_reference():
    g = load_golden("budget_plans.json")
    configs = g["configs"]
    for row in g["cases"]:
        name, dur, kind, count, plan, err = row
        duration = dur if kind == "str" else (int(fhex(dur)) if kind == "int" else fhex(dur))
        if err is not None:
            with pytest.raises(Exception) as ei:
                bp.plan_segments_with_budget(duration, configs[name], count)
            assert type(ei.value).__name__ == err, row
            continue
        p = bp.plan_segments_with_budget(duration, configs[name], count)
        got = [p.segment_duration, p.overlap, p.num_segments, p.estimated_calls,
               p.available_calls, p.hard_max_calls, p.fits_budget]
        assert got == plan, (row, got)
        assert isinstance(p.fits_budget, bool)


def test_budget_nan_and_inf_raise_like_reference():
    with pytest.raises(ValueError):
        bp.plan_segments_with_budget(float("nan"), {}, 0)
    with pytest.raises(OverflowError):
        bp.plan_segments_with_budget(float("inf"), {}, 0)


def test_budget_zero_division_like_reference():
    cfg = {"analyzer": {"max_continuations": -1, "long_video": {"hard_max_api_calls": 1}}}
    with pytest.raises(ZeroDivisionError):
        bp.plan_segments_with_budget(100000.0, cfg, 0)


def test_known_answers_from_survey():
    # SURVEY.md §8(a) a2 (config.yaml values)
    cfg = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                        "long_video": {"enabled": True, "default_segment_seconds": 480,
                                       "overlap_seconds": 20, "min_segment_seconds": 90,
                                       "hard_max_api_calls": 50, "consolidate": True,
                                       "duration_threshold_seconds": None}}}
    exp = {60.0: (480, 20, 1), 600.0: (480, 20, 2), 7200.0: (720, 0, 10),
           7200.5: (721, 0, 10), 10800.0: (1080, 0, 10)}
    for d, (sd, ov, ns) in exp.items():
        p = bp.plan_segments_with_budget(d, cfg, 0)
        assert (p.segment_duration, p.overlap, p.num_segments) == (sd, ov, ns), d
    assert math.isclose(vs.plan_segments(600.0, 480, 20)[1].start, 460.0)
