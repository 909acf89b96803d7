"""GPU scene scoring: decode + NV12 scoring on MI355X through libvtseg.

Two levels:

* ``score_nv12(...)`` — the scoring kernel on NV12 frames already in device
  memory (torch tensors are used only as device-memory plumbing; the work is
  ``vts_score_nv12_dev``, hand-written HIP for gfx950, enqueued on torch's
  current HIP stream).
* ``VideoScorer`` — a session over one MP4 file: host demux, device H.264
  subset decode, device scoring (``vts_open`` / ``vts_score`` / ``vts_run``).

There is no CPU fallback: without libvtseg.so or without a GPU these raise.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from . import _lib

DEFAULT_CUT_THRESHOLD = 0.08


def _torch():
    import torch  # plumbing only: device allocations and the current stream
    return torch


def _stream_handle(device) -> int:
    torch = _torch()
    return int(torch.cuda.current_stream(device).cuda_stream)


def thumb_size(width: int, height: int, k: int) -> tuple[int, int]:
    return width // k, height // k


def score_nv12(nv12, *, width: int, height: int, pitch: int, uv_row_offset: int,
               frame_stride: int, n_frames: int, k: int, prev_luma=None,
               want_rgb: bool = True, want_hist: bool = True, out: dict | None = None,
               workspace=None) -> dict:
    """Score n_frames NV12 frames resident on the GPU (uint8 tensor, any shape,
    contiguous, 16-byte aligned).  Returns device tensors
    {rgb [F,h,w,3] u8, hist [F,256] i32(u32 bits), sad [F] i64(u64 bits),
    score [F] f32, last_luma [h*w] u8}."""
    torch = _torch()
    if not nv12.is_cuda:
        raise ValueError("nv12 must be a device tensor")
    if nv12.dtype != torch.uint8 or not nv12.is_contiguous():
        raise ValueError("nv12 must be a contiguous uint8 tensor")
    dev = nv12.device
    w, h = thumb_size(width, height, k)
    if out is None:
        out = {
            "rgb": torch.empty((n_frames, h, w, 3), dtype=torch.uint8, device=dev)
            if want_rgb else None,
            "hist": torch.empty((n_frames, 256), dtype=torch.int32, device=dev)
            if want_hist else None,
            "sad": torch.empty(n_frames, dtype=torch.int64, device=dev),
            "score": torch.empty(n_frames, dtype=torch.float32, device=dev),
            "last_luma": torch.empty(h * w, dtype=torch.uint8, device=dev),
        }
    ws_bytes = int(_lib.lib().vts_score_workspace_bytes(width, height, k, n_frames))
    if workspace is None or workspace.numel() < ws_bytes:
        workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    d = _lib.ScoreDesc()
    d.nv12 = nv12.data_ptr()
    d.frame_stride = frame_stride
    d.n_frames = n_frames
    d.width, d.height, d.pitch, d.uv_row_offset, d.k = width, height, pitch, uv_row_offset, k

    def p(t):
        return None if t is None else t.data_ptr()

    d.rgb = p(out["rgb"])
    d.hist = p(out["hist"])
    d.sad = p(out["sad"])
    d.score = p(out["score"])
    d.prev_luma = p(prev_luma)
    d.last_luma = p(out["last_luma"])
    d.workspace = workspace.data_ptr()
    d.workspace_bytes = workspace.numel()
    _lib.check(_lib.lib().vts_score_nv12_dev(C.byref(d), C.c_void_p(_stream_handle(dev))))
    out["_workspace"] = workspace
    return out


@dataclass
class SceneResult:
    scores: np.ndarray       # float32 [F]
    hist: np.ndarray         # uint32 [F, 256]
    sad: np.ndarray          # uint64 [F]
    pts: np.ndarray          # int64 [F], track timescale, presentation order
    timescale: int

    def cuts(self, threshold: float = DEFAULT_CUT_THRESHOLD) -> np.ndarray:
        return np.nonzero(self.scores > threshold)[0]


class VideoScorer:
    """Decode + score one MP4 file on GPU `device` (vts_open ... vts_close)."""

    def __init__(self, path: str | Path, device: int = 0, *, k: int = 0,
                 window_frames: int = 0, n_streams: int = 2,
                 cut_threshold: float = DEFAULT_CUT_THRESHOLD, fused: int = 0,
                 gops_per_launch: int = 0, parse_chunks: int = 0, level_block: int = 0,
                 keep_frames: bool = False, decoder: str = "auto"):
        self._lib = _lib.lib()
        prm = _lib.Params()
        prm.k = k
        prm.window_frames = window_frames
        prm.keep_rgb = 0
        prm.n_streams = n_streams
        prm.cut_threshold = cut_threshold
        prm.fused = fused
        prm.gops_per_launch = gops_per_launch
        prm.parse_chunks = parse_chunks
        prm.level_block = level_block
        prm.keep_frames = 1 if keep_frames else 0
        prm.decoder = {"auto": 0, "subset": 1, "general": 2}[decoder]
        self._threshold = cut_threshold
        ctx = C.c_void_p()
        _lib.check(self._lib.vts_open(int(device), str(path).encode(), C.byref(prm),
                                      C.byref(ctx)))
        self._ctx = ctx
        info = _lib.VideoInfo()
        _lib.check(self._lib.vts_info(self._ctx, C.byref(info)))
        self.info = info

    @property
    def n_frames(self) -> int:
        return int(self.info.n_frames)

    def score(self) -> SceneResult:
        n = self.n_frames
        scores = np.zeros(n, np.float32)
        hist = np.zeros((n, 256), np.uint32)
        sad = np.zeros(n, np.uint64)
        pts = np.zeros(n, np.int64)
        got = C.c_int64(0)
        f32 = C.POINTER(C.c_float)
        _lib.check(self._lib.vts_score(
            self._ctx, scores.ctypes.data_as(f32),
            hist.ctypes.data_as(C.POINTER(C.c_uint32)),
            sad.ctypes.data_as(C.POINTER(C.c_uint64)),
            pts.ctypes.data_as(C.POINTER(C.c_int64)), n, C.byref(got)))
        return SceneResult(scores, hist, sad, pts, int(self.info.track_timescale))

    def run(self) -> None:
        """Decode + score with results left on the device (benchmark step)."""
        _lib.check(self._lib.vts_run(self._ctx))

    def run_async(self) -> None:
        """Enqueue a run (decode + score) and return; wait() (or any call that
        reads results) completes it.  Runs of several sessions submitted
        before any wait share the device."""
        _lib.check(self._lib.vts_run_async(self._ctx))

    def wait(self) -> None:
        """Complete a run_async() (errors and re-runs as in run())."""
        _lib.check(self._lib.vts_wait(self._ctx))

    def arena_reruns(self) -> int:
        """Runs repeated because a CABAC window's slices asked for more
        coefficient blocks than its arena held (the session keeps the grown
        arena)."""
        return int(self._lib.vts_schedule_info(self._ctx, 9))

    def timings(self) -> dict:
        t = (C.c_double * 4)()
        _lib.check(self._lib.vts_last_timings(self._ctx, t))
        return {"total_ms": t[0], "parse_ms": t[1], "reconstruct_ms": t[2],
                "score_ms": t[3]}

    def open_timings(self) -> dict:
        """Host time of this session's vts_open by stage (ms)."""
        t = (C.c_double * 8)()
        n = self._lib.vts_open_timings(self._ctx, t, 8)
        if n < 0:
            _lib.check(n)
        return {"demux_ms": t[0], "read_ms": t[2], "schedule_ms": t[3], "alloc_ms": t[4],
                "upload_wait_ms": t[5], "rest_ms": t[6], "total_ms": t[7]}

    def recon_launches(self) -> int:
        """Reconstruct launches per run (one per GOP level per window)."""
        return int(self._lib.vts_schedule_info(self._ctx, 0))

    def general(self) -> bool:
        """The general CAVLC decoder runs (not the I_PCM / integer-motion
        subset kernels)."""
        return bool(self._lib.vts_schedule_info(self._ctx, 8))

    def own_queues(self) -> bool:
        """The session's HIP streams have hardware queues of their own (it was
        opened beside other sessions; session.hip streams_take)."""
        return int(self._lib.vts_schedule_info(self._ctx, 12)) == 1

    def windows(self) -> int:
        """Decode windows per run (1 = the whole video at once; more = the
        streamed two-ring schedule)."""
        return int(self._lib.vts_schedule_info(self._ctx, 1))

    def level_blocks(self) -> tuple[int, int]:
        """(launches, chains) of the level-blocked schedule per run; (0, 0)
        when the per-level schedule runs."""
        return (int(self._lib.vts_schedule_info(self._ctx, 5)),
                int(self._lib.vts_schedule_info(self._ctx, 6)))

    def fused(self) -> bool:
        """Scoring runs fused into reconstruction (k in {2,4,8}, no crop)."""
        return bool(self._lib.vts_schedule_info(self._ctx, 4))

    def boundary_frames(self, times) -> list[int]:
        arr = (C.c_double * len(times))(*[float(t) for t in times])
        out = (C.c_int64 * len(times))()
        _lib.check(self._lib.vts_boundary_frames(self._ctx, arr, len(times), out))
        return list(out)

    def scene_cuts(self) -> list[int]:
        n = C.c_int64(0)
        cap = self.n_frames
        buf = (C.c_int64 * max(cap, 1))()
        _lib.check(self._lib.vts_scene_cuts(self._ctx, buf, cap, C.byref(n)))
        return list(buf[: n.value])

    def frame_pts(self) -> np.ndarray:
        """Presentation timestamps of every frame (int64, track timescale,
        presentation order; host data, no device work)."""
        n = self.n_frames
        pts = np.zeros(max(n, 1), np.int64)
        got = C.c_int64(0)
        _lib.check(self._lib.vts_frame_pts(self._ctx, pts.ctypes.data_as(C.POINTER(C.c_int64)),
                                           n, C.byref(got)))
        return pts[:n]

    def scene_cut_times(self) -> list[float]:
        """Presentation times (s) of the scene-cut frames (decodes + scores):
        anchors for the opt-in scene-aware segment boundaries (vtseg.snap)."""
        from fractions import Fraction
        res = self.score()
        return [float(Fraction(int(res.pts[i]), res.timescale))
                for i in res.cuts(self._threshold)]

    def frame_nv12(self, i: int) -> np.ndarray:
        w, h = int(self.info.width), int(self.info.height)
        out = np.zeros(w * h * 3 // 2, np.uint8)
        _lib.check(self._lib.vts_get_frame_nv12(
            self._ctx, i, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size))
        return out

    def thumbnail_rgb(self, i: int, k: int | None = None) -> np.ndarray:
        kk = k or (4 if int(self.info.height) <= 720 else 6)
        w, h = int(self.info.width) // kk, int(self.info.height) // kk
        out = np.zeros((h, w, 3), np.uint8)
        _lib.check(self._lib.vts_get_thumbnail_rgb(
            self._ctx, i, out.ctypes.data_as(C.POINTER(C.c_uint8)), out.size))
        return out

    def transcode(self, out_path: str | Path, *, height: int = 360, search_range: int = 8,
                  max_mb_sad: int = 1536, keyint: int = 250, idr_at_cuts: bool = False,
                  cut_threshold: float = 0.0, qp: int = 28) -> dict:
        """360p upload transcode of this video into `out_path` (vts_transcode,
        DESIGN.md §11): decode + score + area downscale + device H.264
        encode with a quantised residual at `qp` (<= 0: none, the round-2
        encoder).  Returns the facts and per-stage milliseconds."""
        prm = _lib.TranscodeParams()
        prm.height = height
        prm.search_range = search_range if search_range != 0 else -1
        prm.max_mb_sad = max_mb_sad
        prm.keyint = keyint
        prm.cut_threshold = cut_threshold
        prm.idr_at_cuts = 1 if idr_at_cuts else 0
        prm.qp = qp if qp > 0 else -1
        info = _lib.TranscodeInfo()
        _lib.check(self._lib.vts_transcode(self._ctx, str(out_path).encode(), C.byref(prm),
                                           C.byref(info)))
        return {"width": info.width, "height": info.height, "n_frames": info.n_frames,
                "n_idr": info.n_idr, "pcm_mbs": info.pcm_mbs, "inter_mbs": info.inter_mbs,
                "skip_mbs": info.skip_mbs, "bytes_written": info.bytes_written,
                "decode_ms": info.ms[0], "search_ms": info.ms[1], "write_ms": info.ms[2],
                "mux_ms": info.ms[3]}

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.vts_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_write(path: str | Path, *, width: int = 1280, height: int = 720,
                fps: int = 30, n_frames: int = 300, seed: int = 0x5EED,
                cut_min_s: float = 2.0, cut_max_s: float = 20.0, gop_max_s: float = 2.0,
                max_motion: int = 4, slices_per_row: int = 1,
                hash_frames: bool = False, pcm_zero_runs: bool = False,
                odd_motion: bool = False, drop_last_slice: bool = False,
                nonref_refresh: bool = False, chunks: int = 0, coding: str = "subset",
                constrained_intra: bool = False, bframes: bool = False,
                weighted: str | None = None, temporal_direct: bool = False,
                chroma_deblock: bool = False, cabac: bool = False,
                transform_8x8: bool = False, scaling: str | None = None,
                content: bool = False) -> dict:
    """Write a synthetic H.264/MP4 clip (see vts_synth_write); returns its facts
    and the ground-truth scene-cut frames.  coding="full" only: ``bframes`` codes
    B pictures (Main profile, POC type 0, composition offsets in the MP4),
    ``weighted`` = "explicit" (pred_weight_table in P and B slices) or
    "implicit" (weighted_bipred_idc 2), ``temporal_direct`` mixes temporal with
    spatial direct prediction.  coding="subset" only: ``chroma_deblock``
    turns the deblocking filter on at QPY 3 with chroma_qp_index_offset 12 and
    filter offsets +12, so only chroma edges filter (a stream the subset
    kernels must refuse).  coding="full" only: ``cabac`` writes the same syntax
    decisions with CABAC (cabac_init_idc 0, Main profile; x264's default entropy
    coder) and ``transform_8x8`` (with cabac, High profile) adds Intra_8x8 and
    8x8-transform inter macroblocks.  coding="full" only: ``scaling`` =
    "sps", "pps" or "both" writes seeded scaling matrices (High profile; lists
    absent, default, ending early or full, exercising fall-back rules A / B).
    coding="full" with ``bframes`` only: ``content`` codes pictures instead of
    random syntax (textured scenes cut at the planted frames, a panning
    background and moving sprites; skip / direct / 16x16 motion / intra
    decisions by SAD, residuals quantised from the source's prediction error;
    synth_content.h)."""
    p = _lib.SynthParams()
    p.width, p.height, p.fps_num, p.fps_den = width, height, fps, 1
    p.n_frames, p.seed = n_frames, seed
    p.cut_min_s, p.cut_max_s, p.gop_max_s = cut_min_s, cut_max_s, gop_max_s
    p.max_motion, p.slices_per_row = max_motion, slices_per_row
    p.hash_frames = 1 if hash_frames else 0
    p.edge_cases = (1 if pcm_zero_runs else 0) | (2 if odd_motion else 0) | \
        (4 if drop_last_slice else 0) | (8 if nonref_refresh else 0)
    p.chunks = chunks
    p.coding = {"subset": 0, "full": 1}[coding]
    if constrained_intra:
        p.edge_cases |= 16
    if cabac or transform_8x8:
        if coding != "full":
            raise ValueError("cabac / transform_8x8 need coding='full'")
        if transform_8x8 and not cabac:
            raise ValueError("transform_8x8 needs cabac (8x8 CAVLC streams are refused)")
        p.edge_cases |= 1024 | (2048 if transform_8x8 else 0)
    if scaling:
        if coding != "full":
            raise ValueError("scaling matrices need coding='full'")
        p.edge_cases |= {"sps": 4096, "pps": 8192, "both": 4096 | 8192}[scaling]
    if chroma_deblock:
        if coding != "subset":
            raise ValueError("chroma_deblock is a subset-stream edge case")
        p.edge_cases |= 512
    if bframes or weighted or temporal_direct:
        if coding != "full":
            raise ValueError("B pictures / weighted prediction need coding='full'")
        p.edge_cases |= 32 | {None: 0, "explicit": 64, "implicit": 128}[weighted] | \
            (256 if temporal_direct else 0)
    if content:
        if coding != "full" or not bframes:
            raise ValueError("content mode needs coding='full' and bframes")
        p.edge_cases |= 16384
    info = _lib.SynthInfo()
    cuts = (C.c_int64 * max(n_frames, 1))()
    _lib.check(_lib.lib().vts_synth_write(str(path).encode(), C.byref(p), C.byref(info),
                                          cuts, n_frames))
    return {"bytes": int(info.bytes_written), "n_idr": int(info.n_idr),
            "n_cuts": int(info.n_cuts), "timescale": int(info.timescale),
            "recon_hash": int(info.recon_hash),
            "cuts": list(cuts[: int(info.n_cuts)])}


def scene_cut_times(path: str | Path, device: int = 0) -> list[float]:
    """Decode + score `path` on the GPU and return its scene-cut times."""
    with VideoScorer(path, device=device) as v:
        return v.scene_cut_times()
