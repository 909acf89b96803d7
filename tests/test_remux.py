"""Native stream-copy extract_segment (vts_extract_segment) on ISO-BMFF.

The reference cuts with `ffmpeg -ss S -i IN -t D -movflags +faststart -c copy`
(video_segmenter.py:118-136); its only real-ffmpeg test checks that a non-empty
file appears (test_video_segmenter.py:147-178).  Here the cut is checked
exactly: decoding the output gives the source frames from the keyframe at or
before S through the last frame presented before S + D.  Byte parity with
ffmpeg's output is unpinned (no ffmpeg in the image).
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np
import pytest

import oracle
from vtseg import scene, video_utils
from vtseg import video_segmenter as vs


@pytest.fixture(scope="module")
def clip(tmp_path_factory):
    path = tmp_path_factory.mktemp("remux") / "src.mp4"
    info = scene.synth_write(path, width=160, height=96, n_frames=300, cut_min_s=2.2,
                             cut_max_s=3.1, gop_max_s=1.0, max_motion=4)
    frames, meta = oracle.decode_file(path)
    sync = [i for i in range(300) if i % 1 == 0]
    return path, frames, info, sync


def _idr_frames(path):
    m = oracle.read_mp4(path)
    data = m["data"]
    idr = []
    for i, (off, size) in enumerate(zip(m["offsets"], m["sizes"])):
        nal_type = data[off + 4] & 0x1F
        if nal_type == 5:
            idr.append(i)
    return idr


@pytest.mark.parametrize("start,end", [(2.5, 6.0), (0.0, 1.0), (0.2, 9.99), (4.0, 4.4),
                                       (7.0, 100.0), (1.0, 2.0)])
def test_cut_decodes_to_the_source_frames(clip, tmp_path, start, end):
    path, frames, _, _ = clip
    out = tmp_path / "seg" / "cut.mp4"
    assert vs.extract_segment(path, start, end, out, stream_copy=True)
    idr = _idr_frames(path)
    pts = [1000 * i for i in range(300)]  # exact rational comparison with the doubles
    first = max(i for i in idr if Fraction(pts[i], 30000) <= Fraction(start))
    last = oracle.boundary_frames(pts, 30000, [end])[0] - 1
    got, meta = oracle.decode_file(out)
    assert got.shape[0] == last - first + 1
    assert np.array_equal(got, frames[first:last + 1])
    # presentation starts at `start`: the edit list hides the pre-roll
    span = min(end, 10.0) - start
    assert video_utils.probe_duration(out) == round(span * 1000) / 1000


def test_cut_is_moov_first_and_reopens(clip, tmp_path):
    path, _, _, _ = clip
    out = tmp_path / "c.mp4"
    assert vs.extract_segment(path, 3.0, 5.0, out)
    head = out.read_bytes()[:64]
    assert head[4:8] == b"ftyp" and b"moov" in head
    assert oracle.read_mp4(out)["timescale"] == 30000


def test_extract_failure_modes(clip, tmp_path, monkeypatch):
    path, _, _, _ = clip
    out = tmp_path / "x" / "y.mp4"
    assert not vs.extract_segment(path, 5.0, 5.0, out)          # empty range
    assert not vs.extract_segment(path, 50.0, 60.0, out)        # past the end
    assert not out.exists()
    monkeypatch.setenv("PATH", str(tmp_path))                    # no ffmpeg
    assert not vs.extract_segment(path, 1.0, 2.0, out, stream_copy=False)
    junk = tmp_path / "junk.mkv"
    junk.write_bytes(b"\x1aE\xdf\xa3" + b"\x00" * 100)
    assert not vs.extract_segment(junk, 0.0, 1.0, out)
