"""Generate the golden planning / manifest / driver fixtures from the reference.

This script is the ONLY place that touches the reference implementation, and it
runs only in the build container (``/root/reference`` does not exist on the GPU
box).  It imports the reference's pure-Python segmenter modules
(``src/utils/video_segmenter.py``, ``src/utils/budget_planner.py``) and the
segmentation slice of ``src/analyzer/content_analyzer.py`` (with the absent
``google.genai`` SDK stubbed in-process; the SDK is never exercised because
``_upload_video`` / ``_generate_content`` are replaced), runs them over a grid
of inputs, and writes plain-data JSON fixtures next to this file.  Floats are
stored as ``float.hex`` strings so parity can be checked bit-exactly.

Usage (from the repo root, in the build container)::

    python tests/golden/make_golden.py

Fixtures written:
    plan_segments.json     reference ``plan_segments`` (video_segmenter.py:42-83)
    budget_plans.json      reference ``plan_segments_with_budget`` (budget_planner.py:73-194)
    manifests.json         reference ``create_manifest`` bytes minus ``created_at``
                           (video_segmenter.py:170-218)
    driver_sequences.json  reference ``ContentAnalyzer.analyze_video`` segmentation
                           call sequences (content_analyzer.py:560-964)
    timecodes.json         reference ``ContentAnalyzer._format_timecode`` (:308-314)
"""
from __future__ import annotations

import copy
import json
import math
import sys
import tempfile
import types
from pathlib import Path
from types import SimpleNamespace
from unittest.mock import MagicMock, Mock, patch

REF_SRC = Path("/root/reference/src")
OUT = Path(__file__).resolve().parent


def _hex(x: float) -> str:
    return float(x).hex()


def _stub_genai() -> None:
    """Stub the missing google-genai SDK (names only) so the analyzer imports."""
    google = types.ModuleType("google")
    genai = types.ModuleType("google.genai")
    gtypes = types.ModuleType("google.genai.types")

    class _Any:  # accepts any constructor call / attribute
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return _Any

    genai.Client = _Any  # type: ignore[attr-defined]
    for name in ("GenerateContentConfig", "Part", "Content", "ThinkingConfig",
                 "FileData", "HttpOptions", "SafetySetting"):
        setattr(gtypes, name, _Any)
    gtypes.__getattr__ = lambda name: _Any  # type: ignore[attr-defined]
    genai.types = gtypes  # type: ignore[attr-defined]
    google.genai = genai  # type: ignore[attr-defined]
    sys.modules.setdefault("google", google)
    sys.modules["google.genai"] = genai
    sys.modules["google.genai.types"] = gtypes


# --------------------------------------------------------------------------
# (a) plan_segments grid
# --------------------------------------------------------------------------
def gen_plan_segments(vs) -> list[dict]:
    durations = [0.0, -1.0, -0.0, 1e-9, 0.3, 0.5, 1.0, 1.5, 10.0, 50.0, 59.999,
                 60.0, 61.0, 65.0, 100.0, 120.0, 180.0, 599.9, 600.0, 950.0,
                 1200.0, 1900.0, 3599.5, 3600.0, 7200.0, 7200.5, 10800.0,
                 123456.789, 0.1 + 0.2, 1e16, 1e300, float("nan")]
    segs = [0.0, -5.0, 0.1, 1.0, 7.3, 20.0, 30.0, 59.5, 60.0, 90.0, 200.0,
            400.0, 480.0, 601.0, 720.0, 721.0, 1080.0, 3600.0, 1e15, 1e299,
            float("nan"), 480, 90, 3600]
    overlaps = [0.0, -3.0, -0.0, 5.0, 20.0, 0.25, 100.0, 1e300,
                float("nan"), 20]
    cases = []
    for d in durations:
        for s in segs:
            # skip inputs on which the reference itself never terminates or
            # produces an unreasonably long list
            if isinstance(s, float) and math.isnan(s):
                pass
            elif d > 0 and s > 0 and not math.isnan(d):
                if d / s > 60:
                    continue
            for o in overlaps:
                out = vs.plan_segments(d, s, o)
                cases.append({
                    "duration": _hex(d),
                    "segment_seconds": _hex(s),
                    "segment_is_int": isinstance(s, int),
                    "overlap_seconds": _hex(o),
                    "overlap_is_int": isinstance(o, int),
                    "segments": [[seg.segment_id, _hex(seg.start), _hex(seg.end),
                                  _hex(seg.effective_start), _hex(seg.effective_end)]
                                 for seg in out],
                })
    return cases


# --------------------------------------------------------------------------
# (b) plan_segments_with_budget grid
# --------------------------------------------------------------------------
def _yaml_config() -> dict:
    import yaml
    return yaml.safe_load((REF_SRC.parent / "config" / "config.yaml").read_text())


def _budget_configs() -> list[tuple[str, dict]]:
    base_yaml = _yaml_config()
    test_base = {
        "analyzer": {"max_continuations": 3, "retry_times": 5,
                     "long_video": {"enabled": True, "default_segment_seconds": 480,
                                    "overlap_seconds": 20, "min_segment_seconds": 90,
                                    "hard_max_api_calls": 50, "consolidate": True}}}
    exact = {"analyzer": {"max_continuations": 2, "retry_times": 0,
                          "long_video": {"enabled": True, "default_segment_seconds": 400,
                                         "overlap_seconds": 0, "min_segment_seconds": 90,
                                         "hard_max_api_calls": 8, "consolidate": True}}}
    edge = {"analyzer": {"retry_times": 1, "max_continuations": 1,
                         "long_video": {"enabled": True, "default_segment_seconds": 60,
                                        "overlap_seconds": 0, "min_segment_seconds": 30,
                                        "hard_max_api_calls": 50,
                                        "duration_threshold_seconds": 120}}}
    out: list[tuple[str, dict]] = [
        ("config_yaml", {"analyzer": base_yaml["analyzer"]}),
        ("test_base", test_base),
        ("test_exact", exact),
        ("test_edge", edge),
        ("empty", {}),
        ("analyzer_not_dict", {"analyzer": "nope"}),
        ("long_video_not_dict", {"analyzer": {"long_video": [1, 2]}}),
    ]

    def variant(name: str, **lv) -> None:
        cfg = copy.deepcopy(test_base)
        for k, v in lv.items():
            if k in ("max_continuations", "retry_times"):
                cfg["analyzer"][k] = v
            else:
                cfg["analyzer"]["long_video"][k] = v
        out.append((name, cfg))

    variant("thr_600", duration_threshold_seconds=600)
    variant("thr_str", duration_threshold_seconds="600")
    variant("thr_bad_str", duration_threshold_seconds="abc")
    variant("thr_zero", duration_threshold_seconds=0)
    variant("thr_float", duration_threshold_seconds=59.5)
    variant("thr_bool", duration_threshold_seconds=True)
    variant("thr_list", duration_threshold_seconds=[600])
    variant("seg_str", default_segment_seconds="720")
    variant("seg_bad_str", default_segment_seconds="480.5")
    variant("seg_float", default_segment_seconds=480.9)
    variant("seg_bool", default_segment_seconds=True)
    variant("seg_none", default_segment_seconds=None)
    variant("seg_small", default_segment_seconds=10)
    variant("seg_ws_str", default_segment_seconds="  300 ")
    variant("ovl_big", overlap_seconds=1000)
    variant("ovl_neg", overlap_seconds=-5)
    variant("ovl_str", overlap_seconds="30")
    variant("min_big", min_segment_seconds=1000)
    variant("min_neg", min_segment_seconds=-10)
    variant("hard_8", hard_max_api_calls=8)
    variant("hard_3", hard_max_api_calls=3)
    variant("hard_0", hard_max_api_calls=0)
    variant("hard_12", hard_max_api_calls=12)
    variant("hard_20", hard_max_api_calls=20)
    variant("hard_str", hard_max_api_calls="15")
    variant("cons_false", consolidate=False)
    variant("cons_str_off", consolidate="off")
    variant("cons_str_yes", consolidate=" YES ")
    variant("cons_str_bad", consolidate="maybe")
    variant("cons_zero", consolidate=0)
    variant("cons_float", consolidate=0.5)
    variant("cont_0", max_continuations=0)
    variant("cont_10", max_continuations=10)
    variant("retry_0", retry_times=0)
    variant("retry_str", retry_times="2")
    variant("retry_neg", retry_times=-3)
    return out


def gen_budget(bp) -> list[dict]:
    durations = [0, -5, 0.4, 1, 59.9, 60, 61, 90, 100, 119.9, 120, 121, 180, 479,
                 480, 481, 540, 600, 601, 950, 1200, 1900, 3600, 7200, 7200.5,
                 10800, 3 * 3600, 36000, 86400, 1e7, 123.456, "600", "7200.25"]
    counts = [0, 1, 10, 25, 40, 45, 49, 50, 60, -5]
    cases = []
    for name, cfg in _budget_configs():
        for d in durations:
            for c in counts:
                try:
                    p = bp.plan_segments_with_budget(d, cfg, c)
                    res = [p.segment_duration, p.overlap, p.num_segments,
                           p.estimated_calls, p.available_calls, p.hard_max_calls,
                           p.fits_budget]
                    err = None
                except Exception as exc:  # record the reference's exception type
                    res, err = None, type(exc).__name__
                # compact row: config, duration (hex or str), kind, count, plan, error
                kind = "str" if isinstance(d, str) else ("int" if isinstance(d, int) else "float")
                cases.append([name, d if isinstance(d, str) else _hex(d), kind, c, res, err])
    return {"fields": ["config_name", "duration", "duration_kind", "current_api_count",
                       "plan", "error"],
            "plan_fields": ["segment_duration", "overlap", "num_segments",
                            "estimated_calls", "available_calls", "hard_max_calls",
                            "fits_budget"],
            "configs": {n: c for n, c in _budget_configs()}, "cases": cases}


# --------------------------------------------------------------------------
# (d) manifests
# --------------------------------------------------------------------------
def gen_manifests(vs) -> list[dict]:
    cases = []
    grid = [("video123", 65.0, 30.0, 5.0), ("vid", 600.0, 480, 20),
            ("long", 7200.0, 720, 0), ("long5", 7200.5, 721, 0),
            ("tiny", 1.0, 0.1, 0), ("zero", 0.0, 480, 20),
            ("frac", 123456.789, 1000.5, 12.25), ("big", 1e16, 1e15, 3.0),
            ("unié中", 100.0, 30.0, 5.0), ("ovl_float", 100.0, 30, 5.5)]
    for vid, dur, seg, ovl in grid:
        with tempfile.TemporaryDirectory() as td:
            m = vs.create_manifest(video_id=vid, duration=dur, segment_seconds=seg,
                                   overlap_seconds=ovl, temp_dir=td)
            raw = vs.get_manifest_path(vid, td).read_text(encoding="utf-8")
            created = m["created_at"]
            raw = raw.replace(td, "@TEMP@").replace(created, "@CREATED@")
        cases.append({"video_id": vid, "duration": _hex(dur),
                      "segment_seconds": seg if isinstance(seg, int) else _hex(seg),
                      "segment_is_int": isinstance(seg, int),
                      "overlap_seconds": ovl if isinstance(ovl, int) else _hex(ovl),
                      "overlap_is_int": isinstance(ovl, int),
                      "json": raw})
    return cases


# --------------------------------------------------------------------------
# (c) analyzer segmentation call sequences
# --------------------------------------------------------------------------
def _response(i: int) -> dict:
    return {"title": f"S{i}", "one_sentence_summary": "s", "key_takeaways": [f"k{i}"],
            "deep_dive": [{"chapter_title": "c", "chapter_summary": "",
                           "sections": [{"topic": f"t{i}", "explanation": "e",
                                         "timestamp": "00:00:01-00:00:02"}]}],
            "glossary": {}}


OVERFLOW_MSG = "400 INVALID_ARGUMENT: input token count exceeds maximum of 1048576"


def gen_driver(ca_mod, counter_mod, throttle_mod) -> list[dict]:
    ContentAnalyzer = ca_mod.ContentAnalyzer
    APICounter = counter_mod.APICounter
    GeminiThrottle = throttle_mod.GeminiThrottle
    base_analyzer = _yaml_config()["analyzer"]

    scenarios = []

    def sc(name, duration, analyzer_cfg, max_calls, *, current=0, suffix=".mp4",
           overflow_over=None, fail_ids=(), empty_ids=(), premanifest=None):
        scenarios.append(dict(name=name, duration=duration, analyzer=analyzer_cfg,
                              max_calls=max_calls, current=current, suffix=suffix,
                              overflow_over=overflow_over, fail_ids=list(fail_ids),
                              empty_ids=list(empty_ids), premanifest=premanifest))

    yaml_an = copy.deepcopy(base_analyzer)
    for d in (0.0, 60.0, 61.0, 600.0, 950.0, 1900.0, 7200.0, 7200.5, 10800.0):
        sc(f"yaml_{d}", d, yaml_an, 20)
    sc("yaml_7200_budget3", 7200.0, yaml_an, 3)
    sc("yaml_7200_current45", 7200.0, yaml_an, 60, current=45)
    test_an = {"max_continuations": 1, "retry_times": 1,
               "long_video": {"enabled": True, "default_segment_seconds": 60,
                              "overlap_seconds": 0, "min_segment_seconds": 30,
                              "hard_max_api_calls": 50, "consolidate": True,
                              "duration_threshold_seconds": None}}
    sc("test_180", 180.0, test_an, 10)
    sc("test_180_budget2", 180.0, test_an, 2)
    t61 = copy.deepcopy(test_an)
    t61["long_video"]["duration_threshold_seconds"] = 60
    sc("test_61_thr60", 61.0, t61, 5)
    sc("test_59_thr60", 59.0, t61, 5)
    t3600 = copy.deepcopy(test_an)
    t3600["long_video"].update(duration_threshold_seconds=3600,
                               default_segment_seconds=3600, min_segment_seconds=3600)
    sc("test_7200_seg3600", 7200.0, t3600, 10)
    split = copy.deepcopy(test_an)
    split["long_video"].update(duration_threshold_seconds=0, default_segment_seconds=200)
    sc("split_120", 120.0, split, 10, overflow_over=61.0)
    sc("split_400", 400.0, split, 20, overflow_over=55.0)
    sc("split_400_floor", 400.0, split, 20, overflow_over=1.0)
    ovl = copy.deepcopy(test_an)
    ovl["long_video"].update(overlap_seconds=7, default_segment_seconds=50)
    sc("ovl_170", 170.0, ovl, 20)
    sc("ovl_170_fail1", 170.0, ovl, 20, fail_ids=[1])
    sc("ovl_170_empty2", 170.0, ovl, 20, empty_ids=[2])
    sc("mkv_180", 180.0, test_an, 10, suffix=".mkv")
    disabled = copy.deepcopy(test_an)
    disabled["long_video"]["enabled"] = False
    sc("disabled_600", 600.0, disabled, 10)
    sc("resume_180", 180.0, test_an, 10,
       premanifest={"segment_seconds": 90, "overlap_seconds": 0})

    results = []
    for s in scenarios:
        with tempfile.TemporaryDirectory() as td:
            tdp = Path(td)
            config = {"system": {"temp_dir": str(tdp / "temp")},
                      "proxy": {"base_url": "http://localhost:8000", "timeout": 60},
                      "analyzer": copy.deepcopy(s["analyzer"])}
            counter = APICounter(max_calls=s["max_calls"], current_count=s["current"])
            throttle = Mock(spec=GeminiThrottle)
            throttle.call_with_retry = Mock(side_effect=lambda f, *a, **k: f(*a))
            throttle.wait_before_call = Mock()
            with patch.object(ca_mod.genai, "Client") as mc:
                mc.return_value = MagicMock()
                an = ContentAnalyzer(config=config, api_counter=counter,
                                     logger=MagicMock(), throttle=throttle,
                                     api_key="k")
            an._delete_remote_file = Mock()
            video = tdp / f"video{s['suffix']}"
            video.write_bytes(b"\x00" * 16)
            if s["premanifest"]:
                ca_mod.load_or_create_manifest(
                    video_id=video.stem, duration=s["duration"],
                    segment_seconds=s["premanifest"]["segment_seconds"],
                    overlap_seconds=s["premanifest"]["overlap_seconds"],
                    temp_dir=str(tdp / "temp"))
            events: list = []
            uploads: list = []

            class _SinglePass(Exception):
                pass

            def upload(path):
                if Path(path) == video:
                    raise _SinglePass()
                uploads.append(Path(path).name)
                return SimpleNamespace(uri="gs://x", mime_type="video/mp4", name="files/1")

            def extract(*, input_path, start, end, output_path, stream_copy=True):
                events.append(["extract", Path(input_path).name, _hex(start), _hex(end),
                               Path(output_path).name, bool(stream_copy)])
                Path(output_path).parent.mkdir(parents=True, exist_ok=True)
                Path(output_path).write_bytes(b"segment")
                return True

            state = {"n": 0}

            def generate(video_file, system_role, main_prompt, extra_text_parts=None):
                seg_name = uploads[-1]
                text = (extra_text_parts or [""])[0]
                events.append(["analyze", seg_name, text])
                state["n"] += 1
                # decode this segment's range from its file name or manifest order
                return _scripted(seg_name, text)

            def _scripted(seg_name, text):
                info = seg_ranges.get(seg_name)
                if s["overflow_over"] is not None and info is not None:
                    if info[1] - info[0] > s["overflow_over"]:
                        raise Exception(OVERFLOW_MSG)
                if info is not None and info[2] in s["fail_ids"]:
                    raise RuntimeError(f"boom {info[2]}")
                return _response(state["n"])

            seg_ranges: dict = {}
            orig_range = an._analyze_segment_range

            def range_wrapper(**kw):
                sp = kw["segment_path"]
                if sp is None:
                    sp = kw["segment_dir"] / (
                        f"segment_{kw['segment_id']:04d}_{int(kw['start'] * 1000):010d}_"
                        f"{int(kw['end'] * 1000):010d}.mp4")
                seg_ranges[Path(sp).name] = (kw["start"], kw["end"], kw["segment_id"])
                if kw["segment_id"] in s["empty_ids"] and kw["segment_path"] is not None:
                    events.append(["empty", kw["segment_id"]])
                    return []
                return orig_range(**kw)

            an._analyze_segment_range = range_wrapper
            an._upload_video = upload
            an._generate_content = generate
            an._maybe_consolidate_note = lambda note, context: note
            captured = {}

            def from_api(*, video_path, response_data, metadata):
                captured["metadata"] = metadata
                return SimpleNamespace(metadata=metadata)

            outcome = "ok"
            with patch.object(ca_mod, "probe_duration", return_value=s["duration"]), \
                 patch.object(ca_mod, "extract_segment", side_effect=extract), \
                 patch.object(ca_mod.AnalysisResult, "from_api_response",
                              side_effect=from_api):
                try:
                    an.analyze_video(video)
                except _SinglePass:
                    outcome = "single_pass"
                except Exception as exc:
                    outcome = f"raise:{type(exc).__name__}"
            plan = ca_mod.plan_segments_with_budget(
                s["duration"], config, s["current"])
            md = captured.get("metadata")
            mpath = tdp / "temp" / "segments" / video.stem / "manifest.json"
            manifest = None
            if mpath.exists():
                manifest = json.loads(mpath.read_text())
                manifest.pop("created_at", None)
                for e in manifest["segments"]:
                    e["file_path"] = Path(e["file_path"]).name
            results.append({
                "name": s["name"], "duration": _hex(s["duration"]),
                "analyzer": s["analyzer"], "max_calls": s["max_calls"],
                "current": s["current"], "suffix": s["suffix"],
                "overflow_over": s["overflow_over"], "fail_ids": s["fail_ids"],
                "empty_ids": s["empty_ids"], "premanifest": s["premanifest"],
                "plan_num_segments": plan.num_segments,
                "outcome": outcome, "events": events,
                "metadata": None if md is None else {
                    "duration": _hex(md["duration"]), "segments": md["segments"],
                    "segment_gaps": md["segment_gaps"]},
                "final_count": counter.current_count,
                "final_max_calls": counter.max_calls,
                "manifest": manifest,
            })
    return results


def gen_timecodes(ca_mod) -> list:
    vals = [0.0, 0.9, 1.0, 59.99, 60.0, 3599.999, 3600.0, 7200.5, 86399.0, 360000.0,
            -5.0, 1e7, 480.0, 500.0, 123456.789]
    return [[_hex(v), ca_mod.ContentAnalyzer._format_timecode(v)] for v in vals]


def main() -> None:
    sys.path.insert(0, str(REF_SRC))
    _stub_genai()
    import importlib
    vs = importlib.import_module("utils.video_segmenter")
    bp = importlib.import_module("utils.budget_planner")
    ca = importlib.import_module("analyzer.content_analyzer")
    counter = importlib.import_module("utils.counter")
    throttle = importlib.import_module("utils.gemini_throttle")

    def dump(name, obj):
        (OUT / name).write_text(json.dumps(obj, separators=(",", ":"),
                                           ensure_ascii=True) + "\n")
        print(f"wrote {name}: {len(obj)} cases")

    dump("plan_segments.json", gen_plan_segments(vs))
    dump("budget_plans.json", gen_budget(bp))
    dump("manifests.json", gen_manifests(vs))
    dump("driver_sequences.json", gen_driver(ca, counter, throttle))
    dump("timecodes.json", gen_timecodes(ca))


if __name__ == "__main__":
    main()
