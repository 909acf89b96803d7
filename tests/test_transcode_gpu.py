"""Device upload transcode (vts_transcode) vs the C oracle.

The reference's _compress_video_for_upload (content_analyzer.py:167-236)
runs x264, which is absent here: byte parity with its output is unpinned.
Pinned instead: every output sample byte, the SPS/PPS and the macroblock
statistics of the device encoder equal transcode_oracle.c's on the same
decoded frames and scene scores, and the device decoder reads the output
back to exactly the encoder's reconstruction.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from vtseg import scene

pytestmark = pytest.mark.gpu

CASES = [
    # name, synth kwargs, transcode kwargs
    ("qvga_half", dict(width=320, height=192, n_frames=90), dict(height=96)),
    ("hd720_360", dict(width=1280, height=720, n_frames=75, max_motion=4), dict()),
    ("vga_4to3", dict(width=640, height=480, n_frames=60, max_motion=6), dict()),
    ("fhd_360", dict(width=1920, height=1080, n_frames=40, max_motion=8), dict()),
    ("halfpel", dict(width=320, height=240, n_frames=60, max_motion=5, odd_motion=True),
     dict(height=120, search_range=4)),
    ("allpcm", dict(width=320, height=192, n_frames=30), dict(height=96, max_mb_sad=-1)),
    ("keyint", dict(width=320, height=192, n_frames=70, cut_min_s=30, cut_max_s=40,
                    gop_max_s=10), dict(height=96, keyint=16, search_range=16)),
    ("idr_at_cuts", dict(width=320, height=192, n_frames=90), dict(height=96, idr_at_cuts=True)),
    ("bigpan_edges", dict(width=320, height=192, n_frames=60, max_motion=24), dict(height=96)),
    ("qp36", dict(width=640, height=480, n_frames=45, max_motion=6), dict(qp=36)),
    ("qp20_pan", dict(width=320, height=192, n_frames=60, max_motion=8), dict(height=96, qp=20)),
    # EPB inside I_PCM: the subset kernels refuse mid-transcode and auto mode
    # reruns the decode + downscale on the general decoder
    ("auto_switch", dict(width=320, height=192, n_frames=60, pcm_zero_runs=True), dict(height=96, qp=20)),
    ("no_residual", dict(width=320, height=192, n_frames=60), dict(height=96, qp=0)),
]


def _require_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test requires an MI355X")


def _oracle_run(path, tk):
    frames, info = oracle.decode_file(path)
    F, W, H = frames.shape[0], info["width"], info["height"]
    k = 4 if H <= 720 else 6
    sc = oracle.score_frames(frames.reshape(-1), frames[0].size, F, W, H, W, H, k,
                             want_rgb=False)["score"]
    kw = dict(out_height=tk.get("height", 360), search_range=tk.get("search_range", 8),
              max_mb_sad=tk.get("max_mb_sad", 1536), keyint=tk.get("keyint", 250),
              idr_at_cuts=tk.get("idr_at_cuts", False), qp=tk.get("qp", 28))
    return oracle.transcode(frames, W, H, sc, want_recon=True, **kw), info


@pytest.mark.parametrize("name,sk,tk", CASES, ids=[c[0] for c in CASES])
def test_transcode_bytes_match_oracle(tmp_path, name, sk, tk):
    _require_gpu()
    src, out = tmp_path / "in.mp4", tmp_path / "out.mp4"
    synth = dict(cut_min_s=0.7, cut_max_s=1.5, gop_max_s=0.5)
    synth.update(sk)
    scene.synth_write(src, **synth)
    ref, info = _oracle_run(src, tk)
    with scene.VideoScorer(src) as v:
        facts = v.transcode(out, **tk)
    assert (facts["width"], facts["height"]) == (ref["width"], ref["height"])
    assert facts["n_idr"] == ref["n_idr"]
    assert (facts["pcm_mbs"], facts["inter_mbs"], facts["skip_mbs"]) == \
        (ref["pcm_mbs"], ref["inter_mbs"], ref["skip_mbs"])
    m = oracle.read_mp4(out)
    data = m["data"]
    got = [data[o:o + s] for o, s in zip(m["offsets"], m["sizes"])]
    assert len(got) == len(ref["samples"])
    for i, (a, b) in enumerate(zip(got, ref["samples"])):
        assert a == b, f"sample {i} differs"
    mbw, mbh = ref["coded_width"] // 16, ref["coded_height"] // 16
    fps = info["timescale"] / (info["pts"][1] - info["pts"][0])
    sps, pps = oracle.sps_pps(mbw, mbh, ref["coded_width"] - ref["width"],
                              ref["coded_height"] - ref["height"], fps)
    assert m["sps"][0] == sps and m["pps"][0] == pps
    assert m["dts"] == list(info["pts"])  # same timing as the source
    # the device decoder reads it back to the encoder's reconstruction
    sw, sh, ch = ref["width"], ref["height"], ref["coded_height"]
    rec = ref["recon"]
    with scene.VideoScorer(out, keep_frames=True) as d:
        d.score()
        last = d.frame_nv12(d.n_frames - 1).reshape(sh * 3 // 2, sw)
    want = np.concatenate([rec[-1, :sh, :sw], rec[-1, ch:ch + sh // 2, :sw]])
    assert np.array_equal(last, want)


def test_transcode_residual_coding_compresses(tmp_path):
    """Residual coding (qp 28, the reference's CRF) against the round-2
    encoder on a 720p synthetic: the output is below 0.3x the input (the
    reference expects 1/5 .. 1/10 from x264, content_analyzer.py:170), smaller
    than without a residual, and byte-equal to the oracle's."""
    _require_gpu()
    src = tmp_path / "in.mp4"
    scene.synth_write(src, width=1280, height=720, n_frames=120, max_motion=4, cut_min_s=2, cut_max_s=4,
                      gop_max_s=2)
    sizes = {}
    for qp in (28, 0):
        out = tmp_path / f"o{qp}.mp4"
        with scene.VideoScorer(src) as v:
            facts = v.transcode(out, qp=qp)
        ref, _ = _oracle_run(src, dict(qp=qp))
        m = oracle.read_mp4(out)
        got = [m["data"][o:o + z] for o, z in zip(m["offsets"], m["sizes"])]
        assert got == ref["samples"]
        sizes[qp] = sum(map(len, got))
        assert facts["pcm_mbs"] == ref["pcm_mbs"]
    assert sizes[28] < sizes[0]
    assert sizes[28] < 0.3 * src.stat().st_size


def test_transcode_windowed_equals_one_window(tmp_path):
    """Streamed decode (two rings of small windows) downscales every window
    into the same store: identical output file."""
    _require_gpu()
    src = tmp_path / "in.mp4"
    scene.synth_write(src, width=320, height=192, n_frames=150, cut_min_s=0.7, cut_max_s=1.5,
                      gop_max_s=0.5)
    outs = []
    for window in (0, 31):
        out = tmp_path / f"o{window}.mp4"
        with scene.VideoScorer(src, window_frames=window) as v:
            v.transcode(out, height=96)
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]


def test_transcode_twice_and_after_score(tmp_path):
    """The session stays usable: scoring, transcoding twice (store reused)."""
    _require_gpu()
    src = tmp_path / "in.mp4"
    scene.synth_write(src, width=320, height=192, n_frames=60, cut_min_s=0.7, cut_max_s=1.5,
                      gop_max_s=0.5)
    with scene.VideoScorer(src) as v:
        r0 = v.score()
        a = v.transcode(tmp_path / "a.mp4", height=96)
        b = v.transcode(tmp_path / "b.mp4", height=96)
        r1 = v.score()
    assert a["bytes_written"] == b["bytes_written"]
    assert (tmp_path / "a.mp4").read_bytes() == (tmp_path / "b.mp4").read_bytes()
    assert np.array_equal(r0.scores, r1.scores)


def test_transcode_to_unwritable_path_then_normal(tmp_path):
    """a transcode whose output cannot be opened fails (after the
    encoder's device work was queued) with its streams drained before the
    buffers go back to the allocator; the next transcode in the same session
    — whose buffers come from that same cache — writes the same bytes as a
    fresh session."""
    _require_gpu()
    from vtseg import VtsegError
    src = tmp_path / "in.mp4"
    scene.synth_write(src, width=320, height=192, n_frames=60, cut_min_s=0.7, cut_max_s=1.5,
                      gop_max_s=0.5)
    with scene.VideoScorer(src) as v:
        ref = v.transcode(tmp_path / "ref.mp4", height=96)
    with scene.VideoScorer(src) as v:
        with pytest.raises(VtsegError):
            v.transcode(tmp_path / "no_such_dir" / "x.mp4", height=96)
        got = v.transcode(tmp_path / "ok.mp4", height=96)
    assert got["bytes_written"] == ref["bytes_written"]
    assert (tmp_path / "ok.mp4").read_bytes() == (tmp_path / "ref.mp4").read_bytes()


def test_compress_video_for_upload_gpu(tmp_path):
    """The drop-in method: > max size -> compressed_<name> next to the input,
    a valid H.264 MP4 at 360 lines; a second call reuses it."""
    _require_gpu()
    from vtseg import upload
    src = tmp_path / "clip.mp4"
    scene.synth_write(src, width=1280, height=720, n_frames=60, cut_min_s=0.7, cut_max_s=1.5,
                      gop_max_s=0.5)
    out = upload.compress_video_for_upload(src, max_size_mb=1)
    assert out == tmp_path / "compressed_clip.mp4" and out.stat().st_size > 0
    assert out.stat().st_size < src.stat().st_size
    m = oracle.read_mp4(out)
    assert len(m["sizes"]) == 60
    assert upload.compress_video_for_upload(src, max_size_mb=1) == out


def test_compress_video_for_upload_keeps_audio(tmp_path):
    """A source with a sound track: the compressed upload copy carries the new
    360p video and the source's audio samples unchanged (the reference keeps
    audio with -c:a aac, content_analyzer.py:206-209)."""
    _require_gpu()
    from test_remux import _audio_mp4, _tracks
    from vtseg import _lib, upload
    video = tmp_path / "v.mp4"
    scene.synth_write(video, width=1280, height=720, n_frames=60, gop_max_s=0.5)
    audio = tmp_path / "a.mp4"
    samples = _audio_mp4(audio, 90)
    src = tmp_path / "clip.mp4"
    _lib.check(_lib.lib().vts_add_tracks(str(video).encode(), str(audio).encode(),
                                         str(src).encode()))
    out = upload.compress_video_for_upload(src, max_size_mb=1)
    assert out == tmp_path / "compressed_clip.mp4"
    got = _tracks(out)
    assert [h for h, _ in got] == [b"vide", b"soun"]
    assert got[1][1] == samples
    m = oracle.read_mp4(out)
    assert len(m["sizes"]) == 60
    assert not list(tmp_path.glob("*.tmp"))


def _oracle_run_full(path, tk):
    """The oracle side for any stream the general decoder takes: frames in
    presentation order from h264_full_oracle.c, then the same transcode."""
    frames, info = oracle.decode_full(path)
    F, W, H = frames.shape[0], info["width"], info["height"]
    k = 4 if H <= 720 else 6
    sc = oracle.score_frames(frames.reshape(-1), frames[0].size, F, W, H, W, H, k,
                             want_rgb=False)["score"]
    kw = dict(out_height=tk.get("height", 360), search_range=tk.get("search_range", 8),
              max_mb_sad=tk.get("max_mb_sad", 1536), keyint=tk.get("keyint", 250),
              idr_at_cuts=tk.get("idr_at_cuts", False), qp=tk.get("qp", 28))
    return oracle.transcode(frames, W, H, sc, want_recon=True, **kw), info


FULL_CASES = [
    ("full_ip", dict(width=320, height=240, n_frames=60, coding="full"), None),
    ("b_frames", dict(width=320, height=240, n_frames=60, coding="full", bframes=True, weighted="implicit"),
     None),
    ("cabac_b", dict(width=320, height=240, n_frames=45, coding="full", bframes=True, chunks=1), "cabac"),
    ("real_cabac_clip", None, "real"),
]


@pytest.mark.parametrize("name,sk,mode", FULL_CASES, ids=[c[0] for c in FULL_CASES])
def test_transcode_of_general_decoder_inputs(tmp_path, name, sk, mode):
    """The upload transcode on inputs only the general decoder takes
    (residuals + deblocking, B pictures reordered to presentation order,
    CABAC B, the real High-profile CABAC clip): every output byte equals the
    oracle's transcode of the oracle's decode, timing follows the source's
    presentation times, and the device decoder reads the output back to the
    encoder's reconstruction."""
    _require_gpu()
    from pathlib import Path
    src, out = tmp_path / "in.mp4", tmp_path / "out.mp4"
    if mode == "real":
        src = Path(__file__).resolve().parent / "golden" / "real" / "realshort.mp4"
    elif mode == "cabac":
        cav = tmp_path / "cavlc.mp4"
        scene.synth_write(cav, cut_min_s=0.7, cut_max_s=1.5, gop_max_s=0.8, seed=3, **sk)
        oracle.cabac_convert(cav, src, seed=5, t8=True)
    else:
        scene.synth_write(src, cut_min_s=0.7, cut_max_s=1.5, gop_max_s=0.8, seed=3, **sk)
    tk = dict(height=120)
    ref, info = _oracle_run_full(src, tk)
    with scene.VideoScorer(src) as v:
        assert v.general()
        facts = v.transcode(out, **tk)
    assert (facts["width"], facts["height"]) == (ref["width"], ref["height"])
    assert (facts["pcm_mbs"], facts["inter_mbs"], facts["skip_mbs"]) == \
        (ref["pcm_mbs"], ref["inter_mbs"], ref["skip_mbs"])
    m = oracle.read_mp4(out)
    data = m["data"]
    got = [data[o:o + s] for o, s in zip(m["offsets"], m["sizes"])]
    assert len(got) == len(ref["samples"])
    for i, (a, b) in enumerate(zip(got, ref["samples"])):
        assert a == b, f"sample {i} differs"
    assert m["dts"] == [p - info["pts"][0] for p in info["pts"]] or m["dts"] == list(info["pts"])
    sw, sh, ch = ref["width"], ref["height"], ref["coded_height"]
    rec = ref["recon"]
    with scene.VideoScorer(out, keep_frames=True) as d:
        d.score()
        last = d.frame_nv12(d.n_frames - 1).reshape(sh * 3 // 2, sw)
    want = np.concatenate([rec[-1, :sh, :sw], rec[-1, ch:ch + sh // 2, :sw]])
    assert np.array_equal(last, want)
