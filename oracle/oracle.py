"""Python access to the CPU oracle (liboracle.so) plus small pure-Python oracles.

TEST INFRASTRUCTURE — only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.  The product never does.

    plan_segments / plan_with_budget   restate src/utils/video_segmenter.py:42-83
                                       and src/utils/budget_planner.py:73-194
    boundary_frames                    exact rational pts/timescale >= t (Fraction)
    score_frames                       DESIGN.md §Scoring, scalar C
    decode_file                        DESIGN.md §Decoder subset, scalar C
"""
from __future__ import annotations

import ctypes as C
import subprocess
from bisect import bisect_left
from fractions import Fraction
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


def build() -> Path:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


class _Seg(C.Structure):
    _fields_ = [("segment_id", C.c_int64), ("start", C.c_double), ("end", C.c_double),
                ("effective_start", C.c_double), ("effective_end", C.c_double),
                ("flags", C.c_int64)]


class BudgetCfg(C.Structure):
    _fields_ = [("default_segment_seconds", C.c_int64), ("overlap_seconds", C.c_int64),
                ("min_segment_seconds", C.c_int64), ("hard_max_api_calls", C.c_int64),
                ("max_continuations", C.c_int64), ("retry_times", C.c_int64),
                ("has_threshold", C.c_int32), ("consolidate", C.c_int32),
                ("duration_threshold_seconds", C.c_double)]


class _Plan(C.Structure):
    _fields_ = [("segment_duration", C.c_int64), ("overlap", C.c_int64),
                ("num_segments", C.c_int64), ("estimated_calls", C.c_int64),
                ("available_calls", C.c_int64), ("hard_max_calls", C.c_int64),
                ("fits_budget", C.c_int32), ("_pad", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _lib.or_plan_segments.argtypes = [C.c_double, C.c_double, C.c_double,
                                          C.POINTER(_Seg), C.c_int64, C.POINTER(C.c_int64)]
        _lib.or_plan_with_budget.argtypes = [C.c_double, C.POINTER(BudgetCfg), C.c_int64,
                                             C.POINTER(_Plan)]
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        _lib.or_score_frames.argtypes = [
            u8p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    return _lib


def plan_segments(duration: float, seg: float, ovl: float) -> list[tuple]:
    n = C.c_int64(0)
    cap = 4096
    buf = (_Seg * cap)()
    rc = lib().or_plan_segments(float(duration), float(seg), float(ovl), buf, cap,
                                C.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle plan_segments rc={rc}")
    return [(buf[i].segment_id, buf[i].start, buf[i].end, buf[i].effective_start,
             buf[i].effective_end) for i in range(n.value)]


def plan_with_budget(duration: float, cfg: BudgetCfg, count: int):
    p = _Plan()
    rc = lib().or_plan_with_budget(float(duration), C.byref(cfg), int(count), C.byref(p))
    if rc != 0:
        return rc
    return (p.segment_duration, p.overlap, p.num_segments, p.estimated_calls,
            p.available_calls, p.hard_max_calls, bool(p.fits_budget))


def boundary_frames(pts: list[int], timescale: int, times: list[float]) -> list[int]:
    """Index of the first frame with pts/timescale >= t, in exact rationals."""
    out = []
    for t in times:
        if t != t or t == float("inf"):
            out.append(len(pts))
            continue
        if t == float("-inf"):
            out.append(0)
            continue
        thr = Fraction(t) * timescale  # exact
        # first integer pts >= thr  <=>  pts >= ceil(thr)
        c = -((-thr.numerator) // thr.denominator)
        out.append(bisect_left(pts, c))
    return out


def score_frames(nv12: np.ndarray, frame_stride: int, n_frames: int, width: int,
                 height: int, pitch: int, uv_row_offset: int, k: int,
                 prev_luma: np.ndarray | None = None, want_rgb: bool = True):
    """Scalar scorer. nv12 is a flat uint8 array holding n_frames frames."""
    w, h = width // k, height // k
    rgb = np.zeros(n_frames * w * h * 3, np.uint8) if want_rgb else None
    hist = np.zeros(n_frames * 256, np.uint32)
    sad = np.zeros(n_frames, np.uint64)
    score = np.zeros(n_frames, np.float32)
    last = np.zeros(w * h, np.uint8)
    prev = None if prev_luma is None else np.ascontiguousarray(prev_luma, np.uint8)

    def ptr(a):
        return None if a is None else a.ctypes.data

    rc = lib().or_score_frames(np.ascontiguousarray(nv12).reshape(-1), frame_stride,
                               n_frames, width, height, pitch, uv_row_offset, k, ptr(prev),
                               ptr(rgb), ptr(hist), ptr(sad), ptr(score), ptr(last))
    if rc != 0:
        raise RuntimeError(f"oracle score_frames rc={rc}")
    return {"rgb": rgb, "hist": hist.reshape(n_frames, 256), "sad": sad, "score": score,
            "last_luma": last}
