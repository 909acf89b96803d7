"""The sessions' device allocator (csrc/devmem.cpp): requests of >= 256 MiB are
physical chunks mapped into fresh virtual ranges and kept on release, smaller
ones come from cached hipMalloc segments.  Sessions of different shapes opened
one after another (and two at once) decode bit-exactly, every byte handed out
comes back at close, and vts_empty_cache returns the idle memory to HIP."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import _lib, scene

pytestmark = pytest.mark.gpu


def _require_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")


def test_sessions_of_different_shapes_reuse_mapped_chunks(tmp_path):
    _require_gpu()
    import torch
    L = _lib.lib()
    small = tmp_path / "small.mp4"
    big = tmp_path / "big.mp4"
    scene.synth_write(small, width=320, height=240, n_frames=90, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.8)
    # several hundred MB of surfaces: the mapped path
    scene.synth_write(big, width=1280, height=720, n_frames=300, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.8)
    refs = {}
    for p in (small, big):
        frames, _ = oracle.decode_file(p)
        refs[p] = frames
    base = int(L.vts_device_bytes(0))
    order = [big, small, big, small, big]
    scores = {}
    for p in order:
        with scene.VideoScorer(p, keep_frames=True) as v:
            r = v.score()
            n = r.scores.shape[0]
            got = np.stack([v.frame_nv12(i).reshape(refs[p][i].shape) for i in range(n)])
            assert np.array_equal(got, refs[p]), p.name
            if p in scores:
                assert np.array_equal(scores[p], r.scores)
            scores[p] = r.scores
            assert int(L.vts_device_bytes(0)) > base
        torch.cuda.synchronize()
        assert int(L.vts_device_bytes(0)) == base, "bytes still handed out after close"
    with scene.VideoScorer(big) as a, scene.VideoScorer(small) as b:
        assert np.array_equal(a.score().scores, scores[big])
        assert np.array_equal(b.score().scores, scores[small])
    assert int(L.vts_device_bytes(0)) == base
    assert L.vts_empty_cache(0) == 0
    with scene.VideoScorer(big) as v:  # fresh chunks after the cache went back to HIP
        assert np.array_equal(v.score().scores, scores[big])
