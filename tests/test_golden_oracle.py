"""Pin the CPU oracle against the reference's golden vectors (tests/golden/).

The planning oracle (oracle/vtseg_oracle.c) is trusted only because it
reproduces every vector captured from the reference implementation
(tests/golden/make_golden.py imports src/utils/{video_segmenter,budget_planner}.py).
"""
from __future__ import annotations

import math

import oracle
from conftest import fhex, load_golden, same_float


def test_oracle_plan_segments_matches_reference_goldens():
    cases = load_golden("plan_segments.json")
    assert len(cases) > 5000
    for c in cases:
        d, s, o = fhex(c["duration"]), fhex(c["segment_seconds"]), fhex(c["overlap_seconds"])
        got = oracle.plan_segments(d, s, o)
        exp = c["segments"]
        assert len(got) == len(exp), (c, got)
        for g, e in zip(got, exp):
            assert g[0] == e[0]
            for gv, ev in zip(g[1:], e[1:]):
                assert same_float(gv, fhex(ev)), (c, g, e)


def _coerce_int(value, default):
    if isinstance(value, (int, float, str)):
        try:
            return int(value)
        except ValueError:
            return default
    return default


def _coerce_bool(value, default):
    if isinstance(value, bool):
        return value
    if isinstance(value, (int, float)):
        return bool(value)
    if isinstance(value, str):
        n = value.strip().lower()
        if n in {"true", "1", "yes", "y", "on"}:
            return True
        if n in {"false", "0", "no", "n", "off"}:
            return False
    return default


def oracle_cfg(config: dict) -> oracle.BudgetCfg:
    an = config.get("analyzer")
    an = an if isinstance(an, dict) else {}
    lv = an.get("long_video")
    lv = lv if isinstance(lv, dict) else {}
    cfg = oracle.BudgetCfg()
    cfg.default_segment_seconds = _coerce_int(lv.get("default_segment_seconds"), 480)
    cfg.overlap_seconds = _coerce_int(lv.get("overlap_seconds"), 20)
    cfg.min_segment_seconds = _coerce_int(lv.get("min_segment_seconds"), 90)
    cfg.hard_max_api_calls = _coerce_int(lv.get("hard_max_api_calls"), 50)
    cfg.max_continuations = _coerce_int(an.get("max_continuations"), 3)
    cfg.retry_times = _coerce_int(an.get("retry_times"), 0)
    cfg.consolidate = 1 if _coerce_bool(lv.get("consolidate"), True) else 0
    thr = lv.get("duration_threshold_seconds")
    val = None
    if isinstance(thr, (int, float, str)):
        try:
            val = float(thr)
        except ValueError:
            val = None
    cfg.has_threshold = 0 if val is None else 1
    cfg.duration_threshold_seconds = 0.0 if val is None else val
    return cfg


def golden_duration(row) -> float:
    d, kind = row[1], row[2]
    return float(d) if kind == "str" else fhex(d)


def test_oracle_budget_matches_reference_goldens():
    g = load_golden("budget_plans.json")
    configs = g["configs"]
    n = 0
    for row in g["cases"]:
        name, _, _, count, plan, err = row
        cfg = oracle_cfg(configs[name])
        got = oracle.plan_with_budget(golden_duration(row), cfg, count)
        if err is not None:
            assert isinstance(got, int) and got < 0, (row, got)
        else:
            assert got == tuple(plan), (row, got)
        n += 1
    assert n > 10000


def test_oracle_boundary_frames_exact():
    pts = [i * 1001 for i in range(100)]  # 30000/1001 fps
    ts = 30000
    times = [0.0, -1.0, 1e-300, 1001 / 30000, math.nextafter(1001 / 30000, 0), 2.0,
             3.3033, 1e300, float("nan"), float("inf"), float("-inf")]
    got = oracle.boundary_frames(pts, ts, times)
    assert got[0] == 0 and got[1] == 0 and got[2] == 1
    assert got[-3:] == [100, 100, 0]
    # frame i has t_i = i*1001/30000 exactly; a time a hair below t_i maps to i
    assert got[4] == 1
