"""B pictures and weighted prediction in the general oracle (h264_full_oracle.c).

The synthetic writer (synth_full.cpp, edge_cases bit 5) codes Main-profile
streams with B pictures: mini-GOPs coded anchor first, B reference pictures
(colocated for the others), POC type 0 with a wrapping lsb, spatial and
temporal direct prediction (B_Skip, B_Direct_16x16, B_Direct_8x8), every B
partition / sub-partition shape with L0 / L1 / Bi prediction, explicit and
implicit weighted prediction, and composition offsets in the MP4.

Checks (no third-party decoder exists in the image: parity of the pictures is
unpinned against one): every slice parses to its stop bit; the motion field
of every 4x4 block (refIdxL0/L1, mvL0/L1) the oracle derives equals the one
the writer derived independently while choosing syntax (direct prediction
8.4.1.2, motion vector prediction 8.4.1.3); frames come out in presentation
order.
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

MODES = [
    ("spatial", {}),
    ("explicit", {"weighted": "explicit"}),
    ("implicit", {"weighted": "implicit"}),
    ("temporal", {"temporal_direct": True}),
    ("slices", {"slices_per_row": 2, "weighted": "implicit", "temporal_direct": True}),
]


def _run(code: str, env: dict) -> None:
    e = dict(os.environ)
    e.update(env)
    e["PYTHONPATH"] = os.pathsep.join([str(ROOT / "video-transformer_amd"), str(ROOT / "oracle")])
    subprocess.run([sys.executable, "-c", code], check=True, env=e, cwd=ROOT)


@pytest.mark.parametrize("name,kw", MODES, ids=[m[0] for m in MODES])
def test_writer_and_oracle_derive_the_same_motion(tmp_path, name, kw):
    path = tmp_path / "b.mp4"
    wdump, odump = tmp_path / "w.txt", tmp_path / "o.txt"
    args = dict(width=176, height=144, n_frames=45, coding="full", bframes=True, cut_min_s=0.5,
                cut_max_s=1.2, gop_max_s=0.8, seed=11, chunks=1, **kw)
    _run(f"from vtseg import scene; scene.synth_write({str(path)!r}, **{args!r})",
         {"VTS_SYNTH_MVDUMP": str(wdump)})
    _run(f"import oracle; oracle.decode_full({str(path)!r})", {"FO_MVDUMP": str(odump)})
    w = wdump.read_text().splitlines()
    o = odump.read_text().splitlines()
    assert len(w) == len(o) == 45 * 99 * 32
    bad = [i for i, (a, b) in enumerate(zip(w, o)) if a != b]
    assert not bad, (w[bad[0]], o[bad[0]])
    # both lists and bi-prediction really occur
    lines = np.array([list(map(int, x.split())) for x in o[::7]])
    assert (lines[:, 3] == 1).any() and ((lines[:, 3] == 1) & (lines[:, 4] >= 0)).any()


def test_presentation_order_and_cuts(tmp_path):
    path = tmp_path / "b.mp4"
    info = scene.synth_write(path, width=96, height=64, n_frames=90, coding="full", bframes=True,
                             cut_min_s=0.4, cut_max_s=1.0, gop_max_s=0.6, seed=5)
    m = oracle.read_mp4(path)
    assert any(c != m["cts"][0] for c in m["cts"]), "no reordering"
    frames, inf = oracle.decode_full(path)
    assert inf["pts"] == sorted(inf["pts"]) and len(set(inf["pts"])) == 90
    assert frames.shape[0] == 90
    assert info["n_cuts"] >= 3


def test_b_streams_decode_in_several_chunks(tmp_path):
    """Chunks are closed GOP runs: each starts with an IDR and reorders only
    inside itself."""
    path = tmp_path / "c.mp4"
    scene.synth_write(path, width=64, height=48, n_frames=120, coding="full", bframes=True,
                      weighted="explicit", chunks=4, cut_min_s=0.5, cut_max_s=2.0, seed=9)
    frames, inf = oracle.decode_full(path)
    assert frames.shape[0] == 120 and inf["pts"] == sorted(inf["pts"])
