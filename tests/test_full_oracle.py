"""CPU tests of the general H.264 oracle (oracle/h264_full_oracle.c) and the
full-syntax stream writer (vts_synth_params.coding = 1).

* On the round-1 subset streams (I_PCM, P_Skip / integer-motion P_L0_16x16,
  deblocking off) the general decoder equals the subset oracle, which the
  writer's own reconstruction hash pins (test_synth_oracle.py).
* On full-syntax streams (intra 4x4 / 16x16 / chroma modes, residual blocks,
  quarter-sample partitions, 3 references, list modification, non-reference
  pictures, QP changes, deblocking) the writer and the oracle must agree on
  every syntax element: the oracle fails unless each slice's data ends exactly
  at its rbsp_stop_one_bit, with every macroblock covered once.
Decoded pixels of full-syntax streams are pinned by no third-party decoder
(none in the image): "parity unpinned"; the GPU decoder must equal them.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import scene

SUBSET = [
    dict(width=320, height=240),
    dict(width=336, height=200, slices_per_row=3, max_motion=6),
    dict(width=320, height=240, max_motion=5, odd_motion=True),
    dict(width=160, height=96, max_motion=4, gop_max_s=0.3, nonref_refresh=True),
]


@pytest.mark.parametrize("kw", SUBSET)
def test_general_decoder_equals_subset_oracle(tmp_path, kw):
    kw = dict(kw)
    gop = kw.pop("gop_max_s", 1.0)
    path = tmp_path / "s.mp4"
    r = scene.synth_write(path, n_frames=90, cut_min_s=0.7, cut_max_s=1.6, gop_max_s=gop,
                          hash_frames=True, **kw)
    a, _ = oracle.decode_file(path)
    b, info = oracle.decode_full(path)
    assert np.array_equal(a, b)
    assert oracle.recon_hash(b) == r["recon_hash"]


FULL = [
    ("tiny", dict(width=48, height=32, max_motion=2)),
    ("qvga", dict(width=320, height=240, max_motion=3)),
    ("ragged", dict(width=336, height=200, slices_per_row=3, max_motion=6)),
    ("oneslice", dict(width=320, height=240, slices_per_row=0, max_motion=8)),
    ("cip", dict(width=320, height=240, max_motion=3, constrained_intra=True)),
    ("crop", dict(width=480, height=270, slices_per_row=2, max_motion=4)),
]


@pytest.mark.parametrize("name,kw", FULL, ids=[f[0] for f in FULL])
def test_full_syntax_streams_decode_exactly(tmp_path, name, kw):
    path = tmp_path / f"{name}.mp4"
    r = scene.synth_write(path, n_frames=48, cut_min_s=0.5, cut_max_s=1.2, gop_max_s=0.7,
                          coding="full", seed=11, **kw)
    frames, info = oracle.decode_full(path)
    assert frames.shape == (48, kw["height"] * 3 // 2, kw["width"])
    assert info["pts"] == [1000 * i for i in range(48)]
    again, _ = oracle.decode_full(path)
    assert np.array_equal(frames, again)
    unfiltered, _ = oracle.decode_full(path, flags=1)
    assert not np.array_equal(frames, unfiltered)   # the deblocking filter is active
    assert r["n_idr"] >= 2


def test_full_syntax_is_deterministic_and_seeded(tmp_path):
    a, b, c = tmp_path / "a.mp4", tmp_path / "b.mp4", tmp_path / "c.mp4"
    for p, seed in ((a, 5), (b, 5), (c, 6)):
        scene.synth_write(p, width=96, height=64, n_frames=30, coding="full", seed=seed)
    assert a.read_bytes() == b.read_bytes()
    assert a.read_bytes() != c.read_bytes()


def test_full_syntax_chunks_concatenate(tmp_path):
    """Chunked (parallel) writing: each chunk starts with an IDR, the whole
    stream still decodes."""
    p = tmp_path / "k.mp4"
    scene.synth_write(p, width=64, height=48, n_frames=90, coding="full", chunks=3,
                      cut_min_s=5, cut_max_s=9, gop_max_s=2.0)
    frames, _ = oracle.decode_full(p)
    assert frames.shape[0] == 90


def test_chroma_only_deblocking_is_outside_the_subset(tmp_path):
    """deblocking active on chroma edges only (luma indexA < 16,
    chroma QPc(QPY + chroma_qp_index_offset) pushing indexA to 24).  The
    subset oracle refuses the stream like the subset device parser, and the
    general oracle's filter changes chroma samples only."""
    path = tmp_path / "cdbk.mp4"
    scene.synth_write(path, width=160, height=96, n_frames=12, cut_min_s=0.2, cut_max_s=0.4,
                      gop_max_s=0.2, seed=77, chroma_deblock=True)
    m = oracle.read_mp4(path)
    samples = [m["data"][o:o + z] for o, z in zip(m["offsets"], m["sizes"])]
    with pytest.raises(RuntimeError, match="rc=-9"):
        oracle.decode_samples(m["sps"][0], m["pps"][0], samples, m["nal_length_size"])
    frames, _ = oracle.decode_full(path)
    unfiltered, _ = oracle.decode_full(path, flags=1)
    assert np.array_equal(frames[:, :96], unfiltered[:, :96])
    assert not np.array_equal(frames[:, 96:], unfiltered[:, 96:])
