"""Batch segmentation across GPUs: one process per GPU, video i on rank i % N.

The reference processes a batch with a sequential loop
(src/pipeline.py:376-393 -> analyze_video per URL).  Here every rank probes,
plans and (optionally) decodes+scores its own videos on its own GPU; the only
exchange is one all-gather of a small per-video record (segment count, scene
cut count, duration in microseconds) so every rank ends with the whole batch's
plan — RCCL over xGMI when the group is NCCL, gloo on CPU.  When scene
scoring is requested a second all-gather carries the per-video boundary
arrays, padded to the batch maximum: the segment windows as
frame indices [start, end) of every planned segment (int64) and the scene-cut
frame indices (int64) with their presentation times (f64).  No pixel data
crosses GPUs.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path

from .budget_planner import plan_segments_with_budget
from .video_segmenter import plan_segments
from .video_utils import probe_duration

REC = 4  # int64 fields per video: n_segments, n_cuts, duration_us, scoring failed (0/1)


@dataclass(frozen=True)
class BatchItem:
    index: int
    path: str
    duration: float
    n_segments: int
    n_cuts: int          # -1 when scene scoring was not requested
    rank: int
    # with score=True: frame index range [start, end) of every planned
    # segment's extract window, scene-cut frame indices and their times (s)
    segment_frames: tuple[tuple[int, int], ...] = ()
    cut_frames: tuple[int, ...] = ()
    cut_times: tuple[float, ...] = ()
    # scene scoring of this video failed on its rank (e.g. a stream outside
    # the device decoder's subset); n_cuts is -1 and the arrays are empty.
    # score_error holds the message on the rank that owns the video only.
    score_failed: bool = False
    score_error: str | None = None


def _segments(duration: float, config: dict, current_api_count: int):
    plan = plan_segments_with_budget(duration, config, current_api_count)
    if plan.segment_duration <= 0:
        return []
    return plan_segments(duration, plan.segment_duration, plan.overlap)


def plan_batch(paths: list[str | Path], config: dict, *, current_api_count: int = 0,
               score: bool = False, device: int | None = None, group=None,
               sessions: dict | None = None, max_in_flight: int = 4,
               always_gather: bool = False) -> list[BatchItem]:
    """Plan (and with score=True decode + score) a batch of videos, video i on
    rank i % world, and all-gather the results (module docstring).

    sessions: optional {video index: open scene.VideoScorer} for this rank's
    videos, kept open by the caller (their elementary streams stay resident in
    HBM across calls; the benchmark's timed step).  Videos without one are
    opened from their file and closed again (demux + upload included); at
    most `max_in_flight` of those are open at once (a general-decoder session
    holds tens of GB of HBM), the oldest finished and closed before the next
    opens, and an open that fails while others are in flight is retried once
    after they are drained.

    always_gather: run the all-gathers through the initialised process group
    even at world size 1 (the RCCL path of an N=1 run; otherwise a single
    rank keeps its own records without a collective)."""
    import torch
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    rank = dist.get_rank(group) if distributed else 0
    force = always_gather and distributed
    n = len(paths)
    per = (n + world - 1) // world
    backend = dist.get_backend(group) if distributed else "none"
    on_gpu = backend == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")

    local = torch.zeros((per, REC), dtype=torch.int64)
    seg_frames: list[list[int]] = [[] for _ in range(per)]
    cut_frames: list[list[int]] = [[] for _ in range(per)]
    cut_times: list[list[float]] = [[] for _ in range(per)]
    errors: dict[int, str] = {}
    mine = list(enumerate(range(rank, n, world)))
    segs_of: dict[int, list] = {}
    durations: dict[int, float] = {}
    for j, i in mine:
        p = str(paths[i])
        durations[i] = probe_duration(p)
        segs_of[i] = _segments(durations[i], config, current_api_count)
    if score:
        # Local sessions' runs are submitted before earlier ones are waited
        # for, so the device overlaps them (one video's serial parse tail or
        # reconstruction chain leaves compute units another's fills).  A
        # failure on one video must not keep this rank from the collectives
        # below (the other ranks would wait forever): it is recorded in the
        # video's record.
        from collections import deque

        from .scene import VideoScorer
        running: deque = deque()  # (j, i, session, opened here), in submission order

        def fail(j, i, exc):
            errors[i] = f"{type(exc).__name__}: {exc}"
            local[j, 3] = 1
            local[j, 1] = -1

        def finish_oldest():
            j, i, v, own = running.popleft()
            try:
                v.wait()
                cuts = v.scene_cuts()    # only the scores come back to find the cuts
                pts = v.frame_pts()
                times = [t for sg in segs_of[i] for t in (sg.start, sg.end)]
                sf = v.boundary_frames(times) if times else []
                ts = int(v.info.track_timescale)
                seg_frames[j] = sf
                cut_frames[j] = list(cuts)
                cut_times[j] = [float(pts[c]) / ts for c in cuts]
                local[j, 1] = len(cuts)
            except Exception as exc:  # noqa: BLE001 - reported per video
                fail(j, i, exc)
            finally:
                if own:
                    v.close()

        dev_id = device
        for j, i in mine:
            v, own = (sessions or {}).get(i), False
            try:
                if v is None:
                    own = True
                    while sum(1 for x in running if x[3]) >= max(1, max_in_flight):
                        finish_oldest()
                    if dev_id is None:
                        dev_id = torch.cuda.current_device()
                    try:
                        v = VideoScorer(str(paths[i]), device=dev_id)
                    except Exception:  # noqa: BLE001 - HBM held by the runs in flight: drain, retry once
                        if not running:
                            raise
                        while running:
                            finish_oldest()
                        v = VideoScorer(str(paths[i]), device=dev_id)
                v.run_async()            # decode + score; per-frame results stay on the device
                running.append((j, i, v, own))
            except Exception as exc:  # noqa: BLE001 - reported per video
                fail(j, i, exc)
                if own and v is not None:
                    v.close()
        while running:
            finish_oldest()
    for j, i in mine:
        local[j, 0] = len(segs_of[i])
        if not score or i in errors:
            local[j, 1] = -1
        local[j, 2] = round(durations[i] * 1_000_000)
    g = _all_gather(local, world, group, dev, force).view(world, per, REC)
    arrays = (exchange_boundaries(g, seg_frames, cut_frames, cut_times, group=group, device=dev,
                                  always_gather=force)
              if score else None)
    items = []
    for i in range(n):
        r, j = i % world, i // world
        extra = {}
        if arrays is not None:
            sf, cf, ct = arrays[r][j]
            extra = {"segment_frames": sf, "cut_frames": cf, "cut_times": ct}
        items.append(BatchItem(index=i, path=str(paths[i]), duration=int(g[r, j, 2]) / 1e6,
                               n_segments=int(g[r, j, 0]), n_cuts=int(g[r, j, 1]), rank=r,
                               score_failed=bool(g[r, j, 3]), score_error=errors.get(i),
                               **extra))
    return items


def exchange_boundaries(records, seg_frames, cut_frames, cut_times, *, group=None,
                        device=None, always_gather: bool = False):
    """Second all-gather of the batch: per-video boundary arrays.

    records: the gathered [world, per, REC] int64 (n_segments, n_cuts, ...) of
    the first exchange, identical on every rank, so every rank pads to the
    same widths.  seg_frames[j] (2 per segment), cut_frames[j], cut_times[j]:
    this rank's j-th video.  Returns [world][per] of (segment_frames pairs,
    cut_frames, cut_times) tuples.  always_gather: through the process group
    even at world size 1 (plan_batch).
    """
    import torch
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    dev = device if device is not None else torch.device("cpu")
    per = records.shape[1]
    nseg, ncut = records[:, :, 0], records[:, :, 1].clamp(min=0)
    width_i = max(1, int((2 * nseg + ncut).max()))
    width_f = max(1, int(ncut.max()))
    li = torch.full((per, width_i), -1, dtype=torch.int64)
    lf = torch.zeros((per, width_f), dtype=torch.float64)
    for j in range(per):
        row = list(seg_frames[j]) + list(cut_frames[j])
        if row:
            li[j, :len(row)] = torch.tensor(row, dtype=torch.int64)
        if len(cut_times[j]):
            lf[j, :len(cut_times[j])] = torch.tensor(list(cut_times[j]), dtype=torch.float64)
    force = always_gather and distributed
    gi = _all_gather(li, world, group, dev, force).view(world, per, width_i)
    gf = _all_gather(lf, world, group, dev, force).view(world, per, width_f)
    out = []
    for r in range(world):
        row_r = []
        for j in range(per):
            ns, nc = int(records[r, j, 0]), int(ncut[r, j])
            if records.shape[2] > 3 and int(records[r, j, 3]):
                row_r.append(((), (), ()))  # scoring failed: no boundary arrays
                continue
            vals = gi[r, j].tolist()
            row_r.append((tuple((vals[2 * s], vals[2 * s + 1]) for s in range(ns)),
                          tuple(vals[2 * ns:2 * ns + nc]), tuple(gf[r, j, :nc].tolist())))
        out.append(row_r)
    return out


def _all_gather(local, world: int, group, dev, force: bool = False):
    """[per, ...] on every rank -> [world * per, ...] on the CPU (at world
    size 1 the rank's own tensor, unless `force`: then through the group)."""
    import torch
    import torch.distributed as dist

    if world == 1 and not force:
        return local
    t = local.to(dev)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.cpu()


class RcclComm:
    """An RCCL communicator made by libvtseg (vts_rccl_comm_init) for
    plan_batch_native: the id from `unique_id()` on one rank, sent to the
    others by the caller's own means."""

    def __init__(self, device: int, world: int, rank: int, uid: bytes):
        import ctypes as C

        from . import _lib
        if len(uid) != 128:
            raise ValueError("an RCCL unique id is 128 bytes")
        self._lib = _lib.lib()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        _lib.check(self._lib.vts_rccl_comm_init(device, world, rank, buf, C.byref(h)))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C

        from . import _lib
        buf = (C.c_uint8 * 128)()
        _lib.check(_lib.lib().vts_rccl_unique_id(buf))
        return bytes(buf)

    def close(self) -> None:
        if self.handle:
            self._lib.vts_rccl_comm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def plan_batch_native(paths: list[str | Path], config: dict, *, current_api_count: int = 0,
                      score: bool = False, device: int = 0, max_in_flight: int = 4,
                      comm: RcclComm | None = None) -> list[BatchItem]:
    """plan_batch through the C ABI's vts_batch_run (one native call: probe,
    plan, decode + score, and the two all-gathers over RCCL when `comm` is
    given) — what a host without torch.distributed calls; the same BatchItems."""
    import ctypes as C

    from . import _lib
    from .budget_planner import _i64, budget_cfg
    L = _lib.lib()
    n = len(paths)
    arr = (C.c_char_p * max(n, 1))(*[str(p).encode() for p in paths])
    prm = _lib.BatchParams()
    prm.score = 1 if score else 0
    prm.device = int(device)
    prm.max_in_flight = int(max_in_flight)
    prm.current_api_count = _i64("current_api_count", int(current_api_count))
    prm.rccl_comm = comm.handle if comm is not None else None
    cfg = budget_cfg(config)
    h = C.c_void_p()
    _lib.check(L.vts_batch_run(arr, n, C.byref(cfg), C.byref(prm), C.byref(h)))
    try:
        items = []
        for i in range(n):
            rec = _lib.BatchRecord()
            _lib.check(L.vts_batch_get(h, i, C.byref(rec)))
            extra = {}
            if score and not rec.score_failed:
                ns, nc = int(rec.n_segments), max(0, int(rec.n_cuts))
                sf = (C.c_int64 * max(1, 2 * ns))()
                cf = (C.c_int64 * max(1, nc))()
                ct = (C.c_double * max(1, nc))()
                _lib.check(L.vts_batch_arrays(h, i, sf, cf, ct))
                extra = {"segment_frames": tuple((sf[2 * s], sf[2 * s + 1]) for s in range(ns)),
                         "cut_frames": tuple(cf[:nc]), "cut_times": tuple(ct[:nc])}
            err = None
            if rec.score_failed:
                ln = C.c_int64(0)
                L.vts_batch_error(h, i, None, 0, C.byref(ln))
                if ln.value:
                    buf = C.create_string_buffer(ln.value + 1)
                    L.vts_batch_error(h, i, buf, ln.value + 1, C.byref(ln))
                    err = buf.value.decode("utf-8", "replace")
            items.append(BatchItem(index=i, path=str(paths[i]), duration=float(rec.duration),
                                   n_segments=int(rec.n_segments), n_cuts=int(rec.n_cuts),
                                   rank=int(rec.rank), score_failed=bool(rec.score_failed),
                                   score_error=err, **extra))
        return items
    finally:
        L.vts_batch_free(h)
