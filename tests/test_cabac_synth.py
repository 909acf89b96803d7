"""CABAC stream synthesis (oracle.cabac_convert, h264_full_oracle.c
fo_cabac_convert) — test infrastructure for the CABAC B paths, for which no
real stream exists in the image (the one real CABAC clip,
tests/golden/real/realshort.mp4, has I / P slices only).

The writer's CAVLC streams keep their slice headers (cabac_init_idc 0 added)
and get a CABAC macroblock layer the oracle's own parser generates in
synthesis mode: each bin is a seeded random choice, arithmetic-coded per
9.3.4.  Checks here: the converted stream decodes with the ordinary oracle to
exactly the pictures the synthesis produced, every slice ending at its stop
bit (the decoder refuses otherwise), and the syntax really covers B
macroblocks.  What this pins: the arithmetic coder / parser round trip and
the device's agreement with the oracle (test_full_host / test_full_gpu).
What it does not pin: the B-slice CABAC binarizations and context rules
against a third-party encoder — parity unpinned (none in the image).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle
from vtseg import scene

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("kw,t8", [({}, False), ({"bframes": True}, True),
                                   ({"bframes": True, "weighted": "explicit", "slices_per_row": 2}, False),
                                   ({"bframes": True, "temporal_direct": True}, True)])
def test_synthesised_cabac_round_trip(tmp_path, kw, t8):
    src, dst = tmp_path / "src.mp4", tmp_path / "cabac.mp4"
    scene.synth_write(src, width=96, height=64, n_frames=24, coding="full", cut_min_s=0.4, cut_max_s=1.0,
                      gop_max_s=0.6, seed=7, chunks=1, **kw)
    syn = oracle.cabac_convert(src, dst, seed=11, t8=t8)
    m = oracle.read_mp4(dst)
    frames, info = oracle.decode_full(dst)
    order = sorted(range(len(m["pts"])), key=lambda i: m["pts"][i])
    assert np.array_equal(frames, syn[order])
    assert m["pts"] == oracle.read_mp4(src)["pts"]


def test_synthesised_b_syntax_covers_the_b_macroblock_types(tmp_path):
    """The motion dump of a converted B stream has list-1 and bi-predicted
    blocks and direct-derived ones (refIdx from both lists on B pictures)."""
    src, dst, dump = tmp_path / "src.mp4", tmp_path / "cabac.mp4", tmp_path / "mv.txt"
    scene.synth_write(src, width=96, height=64, n_frames=24, coding="full", bframes=True, cut_min_s=0.4,
                      cut_max_s=1.0, gop_max_s=0.6, seed=7, chunks=1)
    oracle.cabac_convert(src, dst, seed=3)
    env = dict(os.environ, FO_MVDUMP=str(dump),
               PYTHONPATH=os.pathsep.join([str(ROOT / "video-transformer_amd"), str(ROOT / "oracle")]))
    subprocess.run([sys.executable, "-c", f"import oracle; oracle.decode_full({str(dst)!r})"], check=True, env=env)
    rows = np.array([list(map(int, x.split())) for x in dump.read_text().splitlines()])
    l1 = rows[(rows[:, 3] == 1) & (rows[:, 4] >= 0)]
    assert len(l1) > 100
    both = set(map(tuple, rows[(rows[:, 3] == 0) & (rows[:, 4] >= 0)][:, :3].tolist())) & \
        set(map(tuple, l1[:, :3].tolist()))
    assert len(both) > 50
