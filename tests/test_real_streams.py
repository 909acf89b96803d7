"""Real (third-party encoded) H.264 streams: the CPU oracle.

tests/golden/real/realshort.mp4 is a real High-profile CABAC clip (see the
README there).  The oracle must decode every one of its slices with the CABAC
parse ending exactly at the RBSP stop bit (it raises otherwise), and its output
must equal the pinned hash (regenerate with the snippet in _regenerate()).
The GPU decoder is compared with the oracle in tests/test_full_gpu.py.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import pytest

import oracle

REAL = Path(__file__).resolve().parent / "golden" / "real"


def _regenerate() -> dict:  # pragma: no cover - documentation of the fixture
    fr, _ = oracle.decode_full(REAL / "realshort.mp4")
    return {"frames": int(fr.shape[0]), "sha256_nv12": hashlib.sha256(fr.tobytes()).hexdigest(),
            "frame_sha256_16": [hashlib.sha256(f.tobytes()).hexdigest()[:16] for f in fr]}


def test_realshort_cabac_high_profile_oracle():
    pin = json.loads((REAL / "realshort_oracle.json").read_text())
    fr, info = oracle.decode_full(REAL / "realshort.mp4")
    assert fr.shape == (36, 240 * 3 // 2, 320)
    assert (info["width"], info["height"]) == (320, 240)
    got = [hashlib.sha256(f.tobytes()).hexdigest()[:16] for f in fr]
    assert got == pin["frame_sha256_16"]
    assert hashlib.sha256(fr.tobytes()).hexdigest() == pin["sha256_nv12"]


def test_realshort_is_what_the_readme_says():
    m = oracle.read_mp4(REAL / "realshort.mp4")
    sps, pps = m["sps"][0], m["pps"][0]
    assert sps[1] == 100              # profile_idc: High
    assert pps[1] & 0x20              # pic_parameter_set_id ue '1', seq ue '1', entropy_coding_mode_flag 1
