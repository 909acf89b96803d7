"""ctypes binding of libvtseg.so (the C ABI declared in include/vtseg.h).

The library is built in-tree (``__graft_entry__.build()`` or
``python video-transformer_amd/build.py``) and loaded from
``video-transformer_amd/vtseg/libvtseg.so``.  There is no fallback: if the
library is missing or stale every entry point raises ``VtsegLibraryError``.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libvtseg.so"
ABI_VERSION = 8

VTS_OK = 0
VTS_E_INVALID = -1
VTS_E_CAPACITY = -2
VTS_E_NONTERMINATING = -3
VTS_E_RANGE = -4
VTS_E_VALUE = -5
VTS_E_OVERFLOW = -6
VTS_E_IO = -7
VTS_E_FORMAT = -8
VTS_E_UNSUPPORTED = -9
VTS_E_HIP = -10
VTS_E_NODEVICE = -11
VTS_E_DECODE = -12
VTS_E_ZERODIV = -13


class VtsegLibraryError(RuntimeError):
    """libvtseg.so is missing, stale or failed to load."""


class VtsegError(RuntimeError):
    """A libvtseg call returned an error status."""

    def __init__(self, code: int, message: str):
        super().__init__(f"vtseg error {code}: {message}")
        self.code = code
        self.message = message


class NonTerminatingError(VtsegError):
    """The reference loop would never terminate on these inputs."""


class Segment(C.Structure):
    _fields_ = [("segment_id", C.c_int64), ("start", C.c_double), ("end", C.c_double),
                ("effective_start", C.c_double), ("effective_end", C.c_double),
                ("flags", C.c_int64)]


class BudgetCfg(C.Structure):
    _fields_ = [("default_segment_seconds", C.c_int64), ("overlap_seconds", C.c_int64),
                ("min_segment_seconds", C.c_int64), ("hard_max_api_calls", C.c_int64),
                ("max_continuations", C.c_int64), ("retry_times", C.c_int64),
                ("has_threshold", C.c_int32), ("consolidate", C.c_int32),
                ("duration_threshold_seconds", C.c_double)]


class Plan(C.Structure):
    _fields_ = [("segment_duration", C.c_int64), ("overlap", C.c_int64),
                ("num_segments", C.c_int64), ("estimated_calls", C.c_int64),
                ("available_calls", C.c_int64), ("hard_max_calls", C.c_int64),
                ("fits_budget", C.c_int32), ("_pad", C.c_int32)]


class VideoInfo(C.Structure):
    _fields_ = [("duration", C.c_double), ("duration_us", C.c_int64),
                ("movie_timescale", C.c_int64), ("movie_duration", C.c_int64),
                ("track_timescale", C.c_int64), ("n_frames", C.c_int64),
                ("n_sync", C.c_int64), ("width", C.c_int32), ("height", C.c_int32),
                ("coded_width", C.c_int32), ("coded_height", C.c_int32),
                ("profile_idc", C.c_int32), ("level_idc", C.c_int32),
                ("codec", C.c_int32), ("_pad", C.c_int32)]


class ScoreDesc(C.Structure):
    _fields_ = [("nv12", C.c_void_p), ("frame_stride", C.c_int64), ("n_frames", C.c_int64),
                ("width", C.c_int32), ("height", C.c_int32), ("pitch", C.c_int32),
                ("uv_row_offset", C.c_int32), ("k", C.c_int32), ("_pad", C.c_int32),
                ("rgb", C.c_void_p), ("hist", C.c_void_p), ("sad", C.c_void_p),
                ("score", C.c_void_p), ("prev_luma", C.c_void_p), ("last_luma", C.c_void_p),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_int64)]


class Params(C.Structure):
    _fields_ = [("k", C.c_int32), ("window_frames", C.c_int32), ("keep_rgb", C.c_int32),
                ("n_streams", C.c_int32), ("cut_threshold", C.c_float), ("fused", C.c_int32),
                ("gops_per_launch", C.c_int32), ("parse_chunks", C.c_int32),
                ("level_block", C.c_int32), ("keep_frames", C.c_int32), ("decoder", C.c_int32),
                ("_pad", C.c_int32)]


class SynthParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("fps_num", C.c_int32),
                ("fps_den", C.c_int32), ("n_frames", C.c_int64), ("seed", C.c_uint64),
                ("cut_min_s", C.c_double), ("cut_max_s", C.c_double),
                ("gop_max_s", C.c_double), ("max_motion", C.c_int32),
                ("slices_per_row", C.c_int32), ("hash_frames", C.c_int32),
                ("edge_cases", C.c_int32), ("chunks", C.c_int32), ("coding", C.c_int32)]


class SynthInfo(C.Structure):
    _fields_ = [("bytes_written", C.c_int64), ("n_idr", C.c_int64), ("n_cuts", C.c_int64),
                ("timescale", C.c_int64), ("recon_hash", C.c_uint64)]


class TranscodeParams(C.Structure):
    _fields_ = [("height", C.c_int32), ("search_range", C.c_int32), ("max_mb_sad", C.c_int32),
                ("keyint", C.c_int32), ("cut_threshold", C.c_float), ("idr_at_cuts", C.c_int32),
                ("qp", C.c_int32)]


class TranscodeInfo(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("n_frames", C.c_int64),
                ("n_idr", C.c_int64), ("pcm_mbs", C.c_int64), ("inter_mbs", C.c_int64),
                ("skip_mbs", C.c_int64), ("bytes_written", C.c_int64), ("ms", C.c_double * 4)]


class ManifestArgs(C.Structure):
    _fields_ = [("video_id", C.c_char_p), ("segment_dir", C.c_char_p),
                ("created_at", C.c_char_p), ("duration", C.c_double),
                ("duration_int", C.c_char_p), ("segment_seconds", C.c_double),
                ("segment_seconds_int", C.c_char_p), ("overlap_seconds", C.c_double),
                ("overlap_seconds_int", C.c_char_p)]


class BatchParams(C.Structure):
    _fields_ = [("score", C.c_int32), ("device", C.c_int32), ("max_in_flight", C.c_int32),
                ("_pad", C.c_int32), ("current_api_count", C.c_int64), ("rccl_comm", C.c_void_p)]


class BatchRecord(C.Structure):
    _fields_ = [("duration", C.c_double), ("n_segments", C.c_int64), ("n_cuts", C.c_int64),
                ("rank", C.c_int32), ("score_failed", C.c_int32)]


# name -> (restype, argtypes); every symbol declared in include/vtseg.h
_P = C.POINTER
SIGNATURES: dict[str, tuple] = {
    "vts_plan_segments": (C.c_int, [C.c_double, C.c_double, C.c_double, _P(Segment),
                                    C.c_int64, _P(C.c_int64)]),
    "vts_plan_with_budget": (C.c_int, [C.c_double, _P(BudgetCfg), C.c_int64, _P(Plan)]),
    "vts_boundary_frames_pts": (C.c_int, [_P(C.c_int64), C.c_int64, C.c_int64,
                                          _P(C.c_double), C.c_int64, _P(C.c_int64)]),
    "vts_manifest_json": (C.c_int, [_P(ManifestArgs), C.c_char_p, C.c_int64, _P(C.c_int64)]),
    "vts_probe_duration": (C.c_int, [C.c_char_p, _P(C.c_double)]),
    "vts_keyframe_pts": (C.c_int, [C.c_char_p, _P(C.c_int64), C.c_int64, _P(C.c_int64),
                                   _P(C.c_int64)]),
    "vts_probe_info": (C.c_int, [C.c_char_p, _P(VideoInfo)]),
    "vts_extract_segment": (C.c_int, [C.c_char_p, C.c_double, C.c_double, C.c_char_p]),
    "vts_add_tracks": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p]),
    "vts_score_workspace_bytes": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int64]),
    "vts_score_nv12_dev": (C.c_int, [_P(ScoreDesc), C.c_void_p]),
    "vts_open": (C.c_int, [C.c_int, C.c_char_p, _P(Params), _P(C.c_void_p)]),
    "vts_open_memory": (C.c_int, [C.c_int, C.c_void_p, C.c_int64, _P(Params),
                                  _P(C.c_void_p)]),
    "vts_info": (C.c_int, [C.c_void_p, _P(VideoInfo)]),
    "vts_score": (C.c_int, [C.c_void_p, _P(C.c_float), _P(C.c_uint32), _P(C.c_uint64),
                            _P(C.c_int64), C.c_int64, _P(C.c_int64)]),
    "vts_run": (C.c_int, [C.c_void_p]),
    "vts_run_async": (C.c_int, [C.c_void_p]),
    "vts_wait": (C.c_int, [C.c_void_p]),
    "vts_scene_cuts": (C.c_int, [C.c_void_p, _P(C.c_int64), C.c_int64, _P(C.c_int64)]),
    "vts_frame_pts": (C.c_int, [C.c_void_p, _P(C.c_int64), C.c_int64, _P(C.c_int64)]),
    "vts_boundary_frames": (C.c_int, [C.c_void_p, _P(C.c_double), C.c_int64,
                                      _P(C.c_int64)]),
    "vts_get_frame_nv12": (C.c_int, [C.c_void_p, C.c_int64, _P(C.c_uint8), C.c_int64]),
    "vts_get_thumbnail_rgb": (C.c_int, [C.c_void_p, C.c_int64, _P(C.c_uint8), C.c_int64]),
    "vts_last_timings": (C.c_int, [C.c_void_p, _P(C.c_double)]),
    "vts_open_timings": (C.c_int, [C.c_void_p, _P(C.c_double), C.c_int32]),
    "vts_empty_cache": (C.c_int, [C.c_int]),
    "vts_release_streams": (C.c_int, [C.c_int]),
    "vts_device_bytes": (C.c_int64, [C.c_int]),
    "vts_schedule_info": (C.c_int64, [C.c_void_p, C.c_int32]),
    "vts_close": (C.c_int, [C.c_void_p]),
    "vts_transcode": (C.c_int, [C.c_void_p, C.c_char_p, _P(TranscodeParams),
                                _P(TranscodeInfo)]),
    "vts_synth_write": (C.c_int, [C.c_char_p, _P(SynthParams), _P(SynthInfo),
                                  _P(C.c_int64), C.c_int64]),
    "vts_rccl_unique_id": (C.c_int, [_P(C.c_uint8)]),
    "vts_rccl_comm_init": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _P(C.c_uint8), _P(C.c_void_p)]),
    "vts_rccl_comm_destroy": (C.c_int, [C.c_void_p]),
    "vts_batch_run": (C.c_int, [_P(C.c_char_p), C.c_int64, _P(BudgetCfg), _P(BatchParams),
                                _P(C.c_void_p)]),
    "vts_batch_get": (C.c_int, [C.c_void_p, C.c_int64, _P(BatchRecord)]),
    "vts_batch_arrays": (C.c_int, [C.c_void_p, C.c_int64, _P(C.c_int64), _P(C.c_int64),
                                   _P(C.c_double)]),
    "vts_batch_error": (C.c_int, [C.c_void_p, C.c_int64, C.c_char_p, C.c_int64, _P(C.c_int64)]),
    "vts_batch_free": (None, [C.c_void_p]),
    "vts_last_error": (C.c_char_p, []),
    "vts_abi_version": (C.c_int, []),
    "vts_device_count": (C.c_int, []),
}

_lib: C.CDLL | None = None


def lib() -> C.CDLL:
    """Load libvtseg.so once; raise VtsegLibraryError when unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise VtsegLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (no CPU fallback exists)")
    try:
        handle = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | C.RTLD_LOCAL)
    except OSError as exc:
        raise VtsegLibraryError(f"cannot load {LIB_PATH}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(handle, name)
        except AttributeError as exc:
            raise VtsegLibraryError(f"{LIB_PATH} lacks symbol {name} (stale build?)") from exc
        fn.restype = res
        fn.argtypes = args
    if handle.vts_abi_version() != ABI_VERSION:
        raise VtsegLibraryError("libvtseg ABI version mismatch; rebuild")
    _lib = handle
    # pooled stream sets go before the HIP runtime's own teardown (rocprofv3
    # --pmc runs crashed at exit otherwise; session.hip vts_release_streams)
    atexit.register(handle.vts_release_streams, -1)
    return handle


def last_error() -> str:
    msg = lib().vts_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int) -> int:
    """Raise VtsegError for a negative status."""
    if rc < 0:
        msg = last_error()
        if rc == VTS_E_NONTERMINATING:
            raise NonTerminatingError(rc, msg)
        raise VtsegError(rc, msg)
    return rc
