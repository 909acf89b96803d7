"""Multi-process batch path (world_size 2, gloo on CPU): sharding + all-gather.

Each rank plans its own videos (i % 2 == rank); after the all-gather every
rank holds the same batch plan, equal to a single-process run.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CONFIG = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                       "long_video": {"enabled": True, "default_segment_seconds": 20,
                                      "overlap_seconds": 2, "min_segment_seconds": 5,
                                      "hard_max_api_calls": 50, "consolidate": True}}}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, paths, out_dir, score=False):
    sys.path[:0] = [str(ROOT / "video-transformer_amd")]
    import torch.distributed as dist
    from vtseg.batch import plan_batch
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    items = plan_batch(paths, CONFIG, score=score, device=0 if score else None)
    # score_error (the message) stays on the rank that owns the video
    rows = [tuple(vars(i).values())[:-1] for i in items]
    (Path(out_dir) / f"r{rank}.txt").write_text(repr(rows))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_scoring_failure_still_reaches_the_collectives(tmp_path):
    """score=True where scoring fails on every rank (no GPU in the CPU
    suite: VideoScorer raises): each rank must still take part in both
    all-gathers, so the batch completes with every video flagged."""
    import torch
    import torch.multiprocessing as mp
    if torch.cuda.is_available():
        pytest.skip("scoring succeeds with a GPU; covered by the gpu variant")
    from vtseg import scene
    paths = []
    for i in range(3):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=64, height=48, n_frames=300, seed=i)
        paths.append(str(p))
    mp.start_processes(_worker, args=(2, _free_port(), paths, str(tmp_path), True), nprocs=2,
                       join=True, start_method="spawn")
    r0 = eval((tmp_path / "r0.txt").read_text())
    r1 = eval((tmp_path / "r1.txt").read_text())
    assert r0 == r1
    assert [t[4] for t in r0] == [-1, -1, -1]          # n_cuts
    assert [t[9] for t in r0] == [True, True, True]    # score_failed
    assert all(t[6] == () and t[7] == () for t in r0)  # no boundary arrays


@pytest.mark.gpu
def test_two_rank_scored_batch_on_one_gpu_equals_serial(tmp_path):
    """The scoring + boundary-exchange path with two processes (gloo, both
    ranks on GPU 0): every rank ends with the serial run's plan, scene cuts,
    segment frame ranges and cut times."""
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")
    from vtseg import scene
    from vtseg.batch import plan_batch
    paths = []
    for i in range(3):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=320, height=240, n_frames=900 + 300 * i, seed=7 + i,
                          cut_min_s=2, cut_max_s=6)
        paths.append(str(p))
    serial = [tuple(vars(i).values())[:-1] for i in plan_batch(paths, CONFIG, score=True,
                                                                device=0)]
    assert all(t[4] > 0 and not t[9] for t in serial)
    mp.start_processes(_worker, args=(2, _free_port(), paths, str(tmp_path), True), nprocs=2,
                       join=True, start_method="spawn")
    r0 = eval((tmp_path / "r0.txt").read_text())
    r1 = eval((tmp_path / "r1.txt").read_text())
    assert r0 == r1
    strip = [t[:5] + t[6:] for t in serial]             # rank differs from the serial run
    assert [t[:5] + t[6:] for t in r0] == strip
    assert [t[5] for t in r0] == [0, 1, 0]


@pytest.mark.parametrize("n_videos", [5, 2, 1])
def test_two_rank_batch_equals_serial(tmp_path, n_videos):
    import torch.multiprocessing as mp
    from vtseg import scene
    from vtseg.batch import plan_batch
    paths = []
    for i in range(n_videos):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=64, height=48, n_frames=300 + 150 * i, seed=i)
        paths.append(str(p))
    serial = [tuple(vars(i).values())[:5] for i in plan_batch(paths, CONFIG)]
    assert all(not i.score_failed for i in plan_batch(paths, CONFIG))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    mp.start_processes(_worker, args=(2, _free_port(), paths, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    r0 = eval((tmp_path / "r0.txt").read_text())
    r1 = eval((tmp_path / "r1.txt").read_text())
    assert r0 == r1
    assert [t[:5] for t in r0] == serial
    assert [t[5] for t in r0] == [i % 2 for i in range(n_videos)]
    assert [t[2] for t in r0] == [(300 + 150 * i) / 30 for i in range(n_videos)]


def _exchange_worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT / "video-transformer_amd")]
    import torch
    import torch.distributed as dist
    from vtseg.batch import exchange_boundaries
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    # 3 videos per rank; rank r video j has j+1 segments and (r + 2j) % 4 cuts
    per = 3
    recs = torch.zeros((world, per, 4), dtype=torch.int64)
    for r in range(world):
        for j in range(per):
            recs[r, j, 0] = j + 1
            recs[r, j, 1] = (r + 2 * j) % 4
    seg, cut, tim = [], [], []
    for j in range(per):
        ns, nc = j + 1, (rank + 2 * j) % 4
        seg.append([100 * rank + 10 * j + t for t in range(2 * ns)])
        cut.append([1000 * rank + 7 * j + t for t in range(nc)])
        tim.append([0.5 * rank + j + t / 3 for t in range(nc)])
    out = exchange_boundaries(recs, seg, cut, tim)
    (Path(out_dir) / f"x{rank}.txt").write_text(repr(out))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_boundary_exchange(tmp_path):
    """Second all-gather: ragged per-video boundary arrays,
    padded to the batch maximum, arrive intact on every rank."""
    import torch.multiprocessing as mp
    mp.start_processes(_exchange_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    x0 = eval((tmp_path / "x0.txt").read_text())
    x1 = eval((tmp_path / "x1.txt").read_text())
    assert x0 == x1
    for r in range(2):
        for j in range(3):
            ns, nc = j + 1, (r + 2 * j) % 4
            seg = [100 * r + 10 * j + t for t in range(2 * ns)]
            sf, cf, ct = x0[r][j]
            assert sf == tuple((seg[2 * s], seg[2 * s + 1]) for s in range(ns))
            assert cf == tuple(1000 * r + 7 * j + t for t in range(nc))
            assert ct == tuple(0.5 * r + j + t / 3 for t in range(nc))


def _one_rank_group(backend: str):
    import torch
    import torch.distributed as dist
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, **kw)


def test_world_one_forced_gather_equals_plain_run(tmp_path):
    """always_gather=True at world size 1 (gloo on CPU): the records and the
    boundary arrays go through dist.all_gather_into_tensor and come back equal
    to the collective-free run."""
    import torch.distributed as dist
    from vtseg import scene
    from vtseg.batch import exchange_boundaries, plan_batch
    paths = []
    for i in range(3):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=64, height=48, n_frames=300 + 150 * i, seed=i)
        paths.append(str(p))
    plain = plan_batch(paths, CONFIG)
    _one_rank_group("gloo")
    try:
        forced = plan_batch(paths, CONFIG, always_gather=True)
        import torch
        recs = torch.tensor([[[2, 3, 0, 0], [1, 0, 0, 0]]], dtype=torch.int64)
        x = exchange_boundaries(recs, [[0, 10, 8, 20], [0, 5]], [[3, 9, 15], []],
                                [[0.1, 0.3, 0.5], []], always_gather=True)
    finally:
        dist.destroy_process_group()
    assert forced == plain
    assert x == [[(((0, 10), (8, 20)), (3, 9, 15), (0.1, 0.3, 0.5)), (((0, 5),), (), ())]]


@pytest.mark.gpu
def test_rccl_world_one_batch_equals_serial(tmp_path):
    """the RCCL branch of plan_batch on an MI355X.  A
    world-size-1 NCCL (= RCCL) process group; plan_batch with
    always_gather=True sends the per-video records and the padded boundary
    arrays through dist.all_gather_into_tensor on the GPU, and every item
    (segments, scene cuts, segment frame ranges, cut times) equals the
    collective-free serial run; exchange_boundaries alone too."""
    import torch
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")
    from vtseg import scene
    from vtseg.batch import exchange_boundaries, plan_batch
    paths = []
    for i in range(3):
        p = tmp_path / f"v{i}.mp4"
        scene.synth_write(p, width=320, height=240, n_frames=600 + 300 * i, seed=7 + i,
                          cut_min_s=2, cut_max_s=6)
        paths.append(str(p))
    serial = plan_batch(paths, CONFIG, score=True, device=0)
    assert all(it.n_cuts > 0 and not it.score_failed for it in serial)
    torch.cuda.set_device(0)
    _one_rank_group("nccl")
    try:
        assert dist.get_backend() == "nccl"
        got = plan_batch(paths, CONFIG, score=True, device=0, always_gather=True)
        recs = torch.tensor([[[2, 3, 0, 0], [1, 0, 0, 0]]], dtype=torch.int64)
        x = exchange_boundaries(recs, [[0, 10, 8, 20], [0, 5]], [[3, 9, 15], []],
                                [[0.1, 0.3, 0.5], []], device=torch.device("cuda", 0),
                                always_gather=True)
    finally:
        dist.destroy_process_group()
    assert got == serial
    assert x == [[(((0, 10), (8, 20)), (3, 9, 15), (0.1, 0.3, 0.5)), (((0, 5),), (), ())]]


@pytest.mark.gpu
def test_bounded_in_flight_sessions_equal_serial(tmp_path):
    """plan_batch opens at most max_in_flight sessions at once
    (finishing and closing the oldest first): with more videos than that —
    five CABAC B videos, one or two in flight — every record succeeds and
    equals the default run's."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")
    from vtseg import scene
    from vtseg.batch import plan_batch
    paths = []
    for i in range(5):
        p = tmp_path / f"c{i}.mp4"
        scene.synth_write(p, width=320, height=240, n_frames=240 + 60 * i, seed=11 + i, coding="full",
                          slices_per_row=0, bframes=True, weighted="implicit", cabac=True,
                          transform_8x8=True, cut_min_s=1, cut_max_s=3, gop_max_s=2)
        paths.append(str(p))
    ref = plan_batch(paths, CONFIG, score=True, device=0)
    assert all(not it.score_failed and it.n_cuts >= 0 for it in ref)
    for k in (1, 2):
        got = plan_batch(paths, CONFIG, score=True, device=0, max_in_flight=k)
        assert got == ref
