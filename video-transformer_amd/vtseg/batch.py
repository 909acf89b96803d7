"""Batch segmentation across GPUs: one process per GPU, video i on rank i % N.

The reference processes a batch with a sequential loop
(src/pipeline.py:376-393 -> analyze_video per URL).  Here every rank probes,
plans and (optionally) decodes+scores its own videos on its own GPU; the only
exchange is one all-gather of a small per-video record (segment count, scene
cut count, duration in microseconds) so every rank ends with the whole batch's
plan — RCCL over xGMI when the group is NCCL, gloo on CPU.  No pixel data
crosses GPUs.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path

from .budget_planner import plan_segments_with_budget
from .video_segmenter import plan_segments
from .video_utils import probe_duration

REC = 3  # int64 fields per video: n_segments, n_cuts, duration_us


@dataclass(frozen=True)
class BatchItem:
    index: int
    path: str
    duration: float
    n_segments: int
    n_cuts: int          # -1 when scene scoring was not requested
    rank: int


def _segment_count(duration: float, config: dict, current_api_count: int) -> int:
    plan = plan_segments_with_budget(duration, config, current_api_count)
    if plan.segment_duration <= 0:
        return 0
    return len(plan_segments(duration, plan.segment_duration, plan.overlap))


def plan_batch(paths: list[str | Path], config: dict, *, current_api_count: int = 0,
               score: bool = False, device: int | None = None, group=None) -> list[BatchItem]:
    import torch
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if distributed else 1
    rank = dist.get_rank(group) if distributed else 0
    n = len(paths)
    per = (n + world - 1) // world
    backend = dist.get_backend(group) if distributed else "none"
    on_gpu = backend == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")

    local = torch.zeros((per, REC), dtype=torch.int64)
    for j, i in enumerate(range(rank, n, world)):
        p = str(paths[i])
        duration = probe_duration(p)
        n_cuts = -1
        if score:
            from .scene import VideoScorer
            with VideoScorer(p, device=torch.cuda.current_device() if device is None else device) as v:
                v.score()
                n_cuts = len(v.scene_cuts())
        local[j, 0] = _segment_count(duration, config, current_api_count)
        local[j, 1] = n_cuts
        local[j, 2] = round(duration * 1_000_000)
    local = local.to(dev)
    if distributed:
        gathered = torch.empty((world * per, REC), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(gathered, local, group=group)
    else:
        gathered = local
    g = gathered.cpu().view(world, per, REC)
    items = []
    for i in range(n):
        r, j = i % world, i // world
        items.append(BatchItem(index=i, path=str(paths[i]), duration=int(g[r, j, 2]) / 1e6,
                               n_segments=int(g[r, j, 0]), n_cuts=int(g[r, j, 1]), rank=r))
    return items
