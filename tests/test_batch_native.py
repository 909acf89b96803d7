"""The C ABI's batch entry point (vts_batch_run, vtseg.batch.plan_batch_native)
against vtseg.batch.plan_batch: the same BatchItems (records and boundary
arrays) for the same videos — planning only on the CPU, decode + score and an
RCCL communicator of one rank on the GPU."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import pytest

from vtseg import _lib, scene
from vtseg.batch import RcclComm, plan_batch, plan_batch_native

ROOT = Path(__file__).resolve().parents[1]
CONFIG = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                       "long_video": {"enabled": True, "default_segment_seconds": 20,
                                      "overlap_seconds": 2, "min_segment_seconds": 5,
                                      "hard_max_api_calls": 50, "consolidate": True}}}


def _rows(items):
    # score_error: Python's "Type: message" vs the library's message
    return [tuple(v for k, v in vars(i).items() if k != "score_error") for i in items]


def _videos(tmp_path, n, frames=(300, 900, 1500, 60, 2400), **kw):
    paths = []
    for i in range(n):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=64, height=48, n_frames=frames[i % len(frames)], seed=i, **kw)
        paths.append(str(p))
    return paths


def test_batch_symbols_and_struct_sizes():
    L = _lib.lib()
    for name in ("vts_batch_run", "vts_batch_get", "vts_batch_arrays", "vts_batch_error", "vts_batch_free",
                 "vts_rccl_unique_id", "vts_rccl_comm_init", "vts_rccl_comm_destroy"):
        assert hasattr(L, name), name
    assert C.sizeof(_lib.BatchParams) == 32
    assert C.sizeof(_lib.BatchRecord) == 32


@pytest.mark.parametrize("api_count", [0, 40])
def test_native_plan_only_batch_equals_plan_batch(tmp_path, api_count):
    """score=False (no device work): probe + budget plan + segments per video,
    a file that is not a video (duration 0.0, no segments) among them."""
    paths = _videos(tmp_path, 5)
    bad = tmp_path / "not_a_video.mp4"
    bad.write_bytes(b"\0" * 64)
    paths.insert(2, str(bad))
    want = plan_batch(paths, CONFIG, current_api_count=api_count)
    got = plan_batch_native(paths, CONFIG, current_api_count=api_count)
    assert _rows(got) == _rows(want)
    assert got[2].duration == 0.0 and got[2].n_segments == 0
    assert all(i.n_cuts == -1 and not i.score_failed for i in got)


def test_native_batch_of_nothing():
    assert plan_batch_native([], CONFIG) == []


def test_native_scoring_without_a_device_marks_every_video(tmp_path):
    """score=True with no GPU (the CPU suite): every open fails, every video
    is flagged with its message, the call itself succeeds."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("scoring succeeds with a GPU")
    paths = _videos(tmp_path, 3)
    got = plan_batch_native(paths, CONFIG, score=True)
    assert all(i.score_failed and i.n_cuts == -1 and i.score_error for i in got)
    assert [i.n_segments for i in got] == [i.n_segments for i in plan_batch(paths, CONFIG)]


@pytest.mark.gpu
@pytest.mark.parametrize("max_in_flight", [4, 1])
def test_native_scored_batch_equals_plan_batch(tmp_path, max_in_flight):
    """Decode + score on the device: cuts, cut times and segment frames of
    every video equal plan_batch's (subset streams and a CABAC B stream of
    the general decoder), with all sessions or one at a time in flight."""
    import torch
    assert torch.cuda.is_available()
    paths = _videos(tmp_path, 4)
    g = tmp_path / "general.mp4"
    scene.synth_write(g, width=320, height=240, fps=30, n_frames=240, seed=4, coding="full", slices_per_row=0,
                      max_motion=4, bframes=True, weighted="implicit", cabac=True, transform_8x8=True,
                      cut_min_s=1.0, cut_max_s=3.0)
    paths.append(str(g))
    want = plan_batch(paths, CONFIG, score=True, device=0)
    got = plan_batch_native(paths, CONFIG, score=True, device=0, max_in_flight=max_in_flight)
    assert _rows(got) == _rows(want)
    assert not any(i.score_failed for i in got)
    assert sum(i.n_cuts for i in got) > 0


@pytest.mark.gpu
def test_native_batch_over_a_one_rank_rccl_communicator(tmp_path):
    """The RCCL exchange inside the library (vts_rccl_comm_init, two
    ncclAllGather rounds) at world size 1 on the box's GPU: equal to the
    exchange-free call and to plan_batch."""
    import torch
    assert torch.cuda.is_available()
    paths = _videos(tmp_path, 3)
    want = plan_batch(paths, CONFIG, score=True, device=0)
    with RcclComm(0, 1, 0, RcclComm.unique_id()) as comm:
        got = plan_batch_native(paths, CONFIG, score=True, device=0, comm=comm)
        got2 = plan_batch_native(paths, CONFIG, score=False, device=0, comm=comm)
    assert _rows(got) == _rows(want)
    assert _rows(got2) == _rows(plan_batch(paths, CONFIG))
    assert all(i.rank == 0 for i in got)


@pytest.mark.gpu
def test_concurrent_sessions_take_their_own_hardware_queues(tmp_path):
    """The stream-set policy (session.hip streams_take): the first of several
    open sessions on plain streams, the next three on CU-masked streams with
    hardware queues of their own, any further one on plain streams again (at
    most 3 such sets per device); every session's scores equal a lone
    session's, runs submitted together or one by one; a session opened after
    all closed is plain again."""
    import numpy as np
    import torch
    assert torch.cuda.is_available()
    paths = _videos(tmp_path, 5, frames=(600,))
    with scene.VideoScorer(paths[0], device=0) as v:
        assert not v.own_queues()
        ref = v.score().scores.copy()
    vs = [scene.VideoScorer(p, device=0) for p in paths]
    try:
        assert [v.own_queues() for v in vs] == [False, True, True, True, False]
        for v in vs:
            v.run_async()
        for v in vs:
            v.wait()
        for i, v in enumerate(vs):
            want = ref if i == 0 else None
            got = v.score().scores
            if want is not None:
                assert np.array_equal(got, want)
        alone = []
        for p in paths:
            with scene.VideoScorer(p, device=0) as w:
                alone.append(w.score().scores.copy())
        for v, a in zip(vs, alone):
            assert np.array_equal(v.score().scores, a)
    finally:
        for v in vs:
            v.close()
    with scene.VideoScorer(paths[1], device=0) as v:
        assert not v.own_queues()
