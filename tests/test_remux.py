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
from pathlib import Path

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


def _box(typ: bytes, payload: bytes) -> bytes:
    import struct
    return struct.pack(">I", 8 + len(payload)) + typ + payload


def _audio_mp4(path, n_samples: int, timescale: int = 48000, delta: int = 1024) -> list[bytes]:
    """A minimal audio-only ISO-BMFF file: one 'soun' track whose sample entry
    and payloads are opaque bytes (the remuxer is codec-agnostic)."""
    import struct
    samples = [bytes([(7 * i + j) & 0xFF for j in range(40 + (i % 5))]) for i in range(n_samples)]
    mdat_payload = b"".join(samples)
    ftyp = _box(b"ftyp", b"isom" + struct.pack(">I", 0x200) + b"isomiso2mp41")
    stsd = _box(b"stsd", struct.pack(">II", 0, 1) + _box(b"mp4a", bytes(28)))
    stts = _box(b"stts", struct.pack(">III", 0, 1, n_samples) + struct.pack(">I", delta))
    stsc = _box(b"stsc", struct.pack(">IIIII", 0, 1, 1, n_samples, 1))
    stsz = _box(b"stsz", struct.pack(">III", 0, 0, n_samples) +
                b"".join(struct.pack(">I", len(s)) for s in samples))

    def moov(off):
        stco = _box(b"stco", struct.pack(">II", 0, 1) + struct.pack(">I", off))
        stbl = _box(b"stbl", stsd + stts + stsc + stsz + stco)
        minf = _box(b"minf", _box(b"smhd", bytes(8)) + stbl)
        hdlr = _box(b"hdlr", bytes(8) + b"soun" + bytes(12) + b"audio\x00")
        mdhd = _box(b"mdhd", struct.pack(">IIIIIHH", 0, 0, 0, timescale, n_samples * delta,
                                         0x55C4, 0))
        tkhd = _box(b"tkhd", struct.pack(">IIIII", 3, 0, 0, 1, 0) +
                    struct.pack(">IIIIHHHH", n_samples * delta * 1000 // timescale, 0, 0, 0,
                                0, 0, 0x0100, 0) + bytes(36 + 8))
        trak = _box(b"trak", tkhd + _box(b"mdia", mdhd + hdlr + minf))
        mvhd = _box(b"mvhd", struct.pack(">IIIII", 0, 0, 0, 1000,
                                         n_samples * delta * 1000 // timescale) + bytes(80))
        return _box(b"moov", mvhd + trak)

    off = len(ftyp) + len(moov(0)) + 8
    Path(path).write_bytes(ftyp + moov(off) + _box(b"mdat", mdat_payload))
    return samples


def _tracks(path):
    """(handler, [sample bytes]) of every track, via an independent box walk."""
    import struct
    data = Path(path).read_bytes()
    top = {t: (a, b) for t, a, b in oracle._boxes(data, 0, len(data))}
    out = []
    for t, ta, tb in oracle._boxes(data, *top["moov"]):
        if t != "trak":
            continue
        kids = lambda a, b: {n: (x, y) for n, x, y in oracle._boxes(data, a, b)}  # noqa: E731
        mdia = kids(ta, tb)["mdia"]
        hd = kids(*mdia)["hdlr"]
        handler = data[hd[0] + 8:hd[0] + 12]
        stbl = kids(*kids(*mdia)["minf"])["stbl"]
        sb = kids(*stbl)
        sa = sb["stsz"][0]
        cnt = struct.unpack(">I", data[sa + 8:sa + 12])[0]
        sizes = struct.unpack(f">{cnt}I", data[sa + 12:sa + 12 + 4 * cnt])
        co = sb["co64"][0] if "co64" in sb else sb["stco"][0]
        nch = struct.unpack(">I", data[co + 4:co + 8])[0]
        fmt = "Q" if "co64" in sb else "I"
        offs = struct.unpack(f">{nch}{fmt}", data[co + 8:co + 8 + nch * (8 if fmt == "Q" else 4)])
        if nch == cnt:
            starts = list(offs)
        else:  # one chunk holding everything (the test's own audio file)
            starts, p = [], offs[0]
            for z in sizes:
                starts.append(p)
                p += z
        out.append((handler, [data[s:s + z] for s, z in zip(starts, sizes)]))
    return out


def test_add_tracks_keeps_the_sources_audio(tmp_path):
    """vts_add_tracks: the new video plus the source's audio track, both
    stream-copied byte for byte (the upload transcode keeps the sound)."""
    from vtseg import _lib
    video = tmp_path / "v.mp4"
    scene.synth_write(video, width=64, height=48, n_frames=60)
    audio = tmp_path / "a.mp4"
    samples = _audio_mp4(audio, 94)
    src = tmp_path / "src.mp4"      # "downloaded" file: video + audio
    _lib.check(_lib.lib().vts_add_tracks(str(video).encode(), str(audio).encode(),
                                         str(src).encode()))
    got = _tracks(src)
    assert [h for h, _ in got] == [b"vide", b"soun"]
    assert got[1][1] == samples
    frames, _ = oracle.decode_file(video)
    assert np.array_equal(oracle.decode_file(src)[0], frames)
    # the source's video track is replaced, its audio kept
    new_video = tmp_path / "n.mp4"
    scene.synth_write(new_video, width=32, height=32, n_frames=30, seed=9)
    out = tmp_path / "out.mp4"
    _lib.check(_lib.lib().vts_add_tracks(str(new_video).encode(), str(src).encode(),
                                         str(out).encode()))
    got = _tracks(out)
    assert [h for h, _ in got] == [b"vide", b"soun"]
    assert got[1][1] == samples
    assert np.array_equal(oracle.decode_file(out)[0], oracle.decode_file(new_video)[0])
    assert video_utils.probe_duration(out) == 2.005  # the audio's 94 x 1024 / 48000 s
