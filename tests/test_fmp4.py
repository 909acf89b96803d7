"""Fragmented MP4 (ISO/IEC 14496-12 §8.8: moov with empty sample tables +
mvex, then moof/mdat pairs): the demuxer appends every movie fragment's
samples (tfhd / tfdt / trun, trex defaults) to the track's table, so probing,
keyframe anchors, the stream-copy cutter, the batch path and the device
decoder read a fragmented file exactly as the progressive file it was made
from (tests/fmp4.py rewrites one as the other).  The reference hands such
files to ffprobe / ffmpeg (src/utils/video_utils.py:9-38,
video_segmenter.py:118-136); ffprobe's value for a fragmented file whose
mvhd says 0 is unpinned here (no ffprobe in the image): the longest track's
sample span is used."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np
import pytest

import fmp4
import oracle
from vtseg import _lib, scene, snap, video_utils
from vtseg import video_segmenter as vs
from vtseg.batch import plan_batch_native

CONFIG = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                       "long_video": {"enabled": True, "default_segment_seconds": 20,
                                      "overlap_seconds": 2, "min_segment_seconds": 5,
                                      "hard_max_api_calls": 50, "consolidate": True}}}


def _info(path):
    vi = _lib.VideoInfo()
    _lib.check(_lib.lib().vts_probe_info(str(path).encode(), C.byref(vi)))
    return {k: getattr(vi, k) for k, _ in _lib.VideoInfo._fields_ if not k.startswith("_")}


VARIANTS = [
    ("runs30", dict(per_fragment=30)),
    ("runs7_zero_mvhd", dict(per_fragment=7, zero_mvhd=True, mehd=False)),
    ("runs1_durations_per_sample", dict(per_fragment=1, trex_defaults=False)),
]


@pytest.fixture(scope="module")
def streams(tmp_path_factory):
    d = tmp_path_factory.mktemp("fmp4")
    prog = d / "prog.mp4"
    scene.synth_write(prog, width=160, height=96, n_frames=300, cut_min_s=2.2, cut_max_s=3.1, gop_max_s=1.0,
                      max_motion=4)
    bprog = d / "bprog.mp4"  # B pictures: composition offsets in the runs
    scene.synth_write(bprog, width=64, height=48, fps=30, n_frames=90, seed=3, coding="full", slices_per_row=0,
                      bframes=True, weighted="implicit", cabac=True, transform_8x8=True)
    return d, prog, bprog


@pytest.mark.parametrize("name,kw", VARIANTS, ids=[v[0] for v in VARIANTS])
def test_probe_and_keyframes_equal_the_progressive_file(streams, name, kw):
    d, prog, bprog = streams
    for src in (prog, bprog):
        frag = d / f"{src.stem}_{name}.mp4"
        fmp4.fragment(src, frag, **kw)
        a, b = _info(frag), _info(src)
        if kw.get("zero_mvhd"):  # the raw mvhd field says 0; duration / duration_us still equal
            assert a.pop("movie_duration") == 0
            b.pop("movie_duration")
        assert a == b
        assert video_utils.probe_duration(frag) == video_utils.probe_duration(src) > 0
        assert snap.keyframe_times(frag) == snap.keyframe_times(src)


def test_fragment_samples_decode_to_the_same_frames(streams):
    """The oracle's own MP4 reader only knows progressive files: the
    fragmented file's samples, cut back out with the native stream-copy
    remuxer (a progressive MP4), decode to the source's frames."""
    d, prog, _ = streams
    frag = d / "prog_whole.mp4"
    fmp4.fragment(prog, frag, per_fragment=30)
    out = d / "back.mp4"
    assert vs.extract_segment(frag, 0.0, 100.0, out, stream_copy=True)
    want, _ = oracle.decode_file(prog)
    got, _ = oracle.decode_file(out)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("start,end", [(2.5, 6.0), (0.0, 1.0), (4.0, 4.4)])
def test_cut_from_a_fragmented_file_equals_the_progressive_cut(streams, tmp_path, start, end):
    d, prog, _ = streams
    frag = d / "prog_cut.mp4"
    if not frag.exists():
        fmp4.fragment(prog, frag, per_fragment=30)
    a, b = tmp_path / "a.mp4", tmp_path / "b.mp4"
    assert vs.extract_segment(prog, start, end, a, stream_copy=True)
    assert vs.extract_segment(frag, start, end, b, stream_copy=True)
    assert a.read_bytes() == b.read_bytes()


def test_batch_plan_of_fragmented_files(streams):
    d, prog, bprog = streams
    fa, fb = d / "batch_a.mp4", d / "batch_b.mp4"
    fmp4.fragment(prog, fa, per_fragment=30)
    fmp4.fragment(bprog, fb, per_fragment=7, zero_mvhd=True, mehd=False)
    want = plan_batch_native([str(prog), str(bprog)], CONFIG)
    got = plan_batch_native([str(fa), str(fb)], CONFIG)
    assert [(i.duration, i.n_segments) for i in got] == [(i.duration, i.n_segments) for i in want]


def test_corrupt_fragments_fail_cleanly(streams, tmp_path):
    """A trun that runs past its box, or points outside the file, is a
    format error (probe answers 0.0), never a crash."""
    d, prog, _ = streams
    frag = d / "prog_corrupt_src.mp4"
    fmp4.fragment(prog, frag, per_fragment=30)
    data = bytearray(frag.read_bytes())
    i = data.find(b"trun")
    bad = tmp_path / "bad_count.mp4"
    cnt = bytearray(data)
    cnt[i + 8:i + 12] = (10 ** 6).to_bytes(4, "big")  # sample_count far past the box
    bad.write_bytes(bytes(cnt))
    assert video_utils.probe_duration(bad) == 0.0  # (ffprobe, the fallback, is absent here)
    vi = _lib.VideoInfo()
    assert _lib.lib().vts_probe_info(str(bad).encode(), C.byref(vi)) == _lib.VTS_E_FORMAT
    off = tmp_path / "bad_offset.mp4"
    o = bytearray(data)
    o[i + 12:i + 16] = (2 ** 31 - 1).to_bytes(4, "big")  # data_offset beyond the file
    off.write_bytes(bytes(o))
    assert _lib.lib().vts_probe_info(str(off).encode(), C.byref(vi)) == _lib.VTS_E_FORMAT


@pytest.mark.gpu
def test_device_decoder_reads_fragmented_files(streams):
    """vts_open on a fragmented file: every score, histogram and SAD equals
    the progressive file's (subset decoder and the general decoder's CABAC B
    stream)."""
    import torch
    assert torch.cuda.is_available()
    d, prog, bprog = streams
    for src, kw in ((prog, dict(per_fragment=30)), (bprog, dict(per_fragment=7, zero_mvhd=True, mehd=False))):
        frag = d / f"{src.stem}_dev.mp4"
        fmp4.fragment(src, frag, **kw)
        with scene.VideoScorer(src, device=0) as a, scene.VideoScorer(frag, device=0) as b:
            ra, rb = a.score(), b.score()
            assert np.array_equal(ra.scores, rb.scores)
            assert np.array_equal(ra.hist, rb.hist)
            assert np.array_equal(ra.sad, rb.sad)
            assert a.scene_cuts() == b.scene_cuts()
            assert list(a.frame_pts()) == list(b.frame_pts())
