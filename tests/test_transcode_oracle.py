"""Upload transcode on the CPU side: the oracle's definition
checked for self-consistency, the output-size rule against ffmpeg's
scale=-2:H formula, and the drop-in's decision flow against the reference's
_compress_video_for_upload (content_analyzer.py:167-236)."""
from __future__ import annotations

import logging

import numpy as np
import pytest

import oracle
from vtseg import scene, upload


def _ffmpeg_minus2_width(W, H, h):
    """libavfilter scale_eval: w = av_rescale(h, W, H * 2) * 2, av_rescale
    rounding to nearest with ties away from zero."""
    from fractions import Fraction
    q = Fraction(h * W, H * 2)
    return int(q + Fraction(1, 2)) * 2


@pytest.mark.parametrize("W,H", [(1280, 720), (1920, 1080), (640, 480), (320, 240), (1366, 768),
                                 (720, 576), (3840, 2160), (854, 480), (426, 240)])
def test_small_width_is_ffmpeg_scale_minus2(W, H):
    assert oracle.small_width(W, H, 360) == _ffmpeg_minus2_width(W, H, 360)


def _box(frame, W, H, k):
    """Integer-ratio area filter = box mean, rounded half up, min 1."""
    y = frame[:H].astype(np.int64)
    uv = frame[H:].astype(np.int64)
    by = (y.reshape(H // k, k, W // k, k).sum(axis=(1, 3)) + k * k // 2) // (k * k)
    u = uv[:, 0::2].reshape(H // 2 // k, k, W // 2 // k, k).sum(axis=(1, 3))
    v = uv[:, 1::2].reshape(H // 2 // k, k, W // 2 // k, k).sum(axis=(1, 3))
    bu, bv = (u + k * k // 2) // (k * k), (v + k * k // 2) // (k * k)
    return np.maximum(by, 1), np.maximum(bu, 1), np.maximum(bv, 1)


@pytest.mark.parametrize("k", [2, 3])
def test_area_downscale_integer_ratio_is_box_mean(k):
    rng = np.random.default_rng(k)
    W, H = 96 * k, 64 * k
    fr = rng.integers(0, 256, (H * 3 // 2, W), dtype=np.uint8)
    fr[:8, :8] = 0  # zeros clamp to 1
    out = oracle.downscale_nv12(fr, W, H, 64)
    by, bu, bv = _box(fr, W, H, k)
    assert np.array_equal(out[:64, :96], by)
    assert np.array_equal(out[64:96, 0:96:2], bu)
    assert np.array_equal(out[64:96, 1:96:2], bv)
    assert out.min() >= 1


def test_area_downscale_fractional_ratio_matches_exact_weights():
    """640x480 -> 480x360: weights (3,1) (2,2) (1,3) per axis, total 16."""
    rng = np.random.default_rng(7)
    fr = rng.integers(1, 256, (720, 640), dtype=np.uint8)
    out = oracle.downscale_nv12(fr, 640, 480, 360)
    y = fr[:480].astype(np.int64)
    wts = [(0, (3, 1)), (1, (2, 2)), (2, (1, 3))]

    def ax(n_out):
        m = np.zeros((n_out, n_out * 4 // 3), np.int64)
        for o in range(n_out):
            base, (a, b) = (o // 3) * 4 + o % 3, wts[o % 3][1]
            m[o, base], m[o, base + 1] = a, b
        return m
    Mx, My = ax(480), ax(360)
    want = (My @ y @ Mx.T + 8) // 16
    assert np.array_equal(out[:360, :480], np.maximum(want, 1))
    assert np.array_equal(out[360, :480], out[359, :480])  # replicated padding rows


@pytest.fixture(scope="module")
def clip(tmp_path_factory):
    p = tmp_path_factory.mktemp("tc") / "clip.mp4"
    scene.synth_write(p, width=320, height=192, n_frames=90, cut_min_s=0.7, cut_max_s=1.5,
                      gop_max_s=0.5)
    frames, info = oracle.decode_file(p)
    sc = oracle.score_frames(frames.reshape(-1), frames[0].size, 90, 320, 192, 320, 192, 4,
                             want_rgb=False)["score"]
    return frames, sc, info


@pytest.mark.parametrize("T,R", [(768, 8), (0, 8), (768, 0), (-1, 8), (5000, 16)])
def test_oracle_round_trip_and_error_bound(clip, T, R):
    """The round-2 encoder (qp 0: no residual): I_PCM where the motion
    misses by more than T, every output decodes (subset decoder) to the
    encoder's reconstruction."""
    frames, sc, info = clip
    r = oracle.transcode(frames, 320, 192, sc, out_height=96, search_range=R, max_mb_sad=T,
                         want_recon=True, qp=0)
    cw, ch, sw, sh = r["coded_width"], r["coded_height"], r["width"], r["height"]
    sps, pps = oracle.sps_pps(cw // 16, ch // 16, cw - sw, ch - sh, 30.0)
    dec = oracle.decode_samples(sps, pps, r["samples"])
    rec = r["recon"]
    assert np.array_equal(dec, np.concatenate([rec[:, :sh, :sw], rec[:, ch:ch + sh // 2, :sw]], 1))
    ds = np.stack([oracle.downscale_nv12(f, 320, 192, 96) for f in frames])
    err = np.abs(ds.astype(np.int64) - rec.astype(np.int64))
    # per macroblock luma+chroma SAD <= T (T < 0: everything I_PCM, exact)
    for f in range(len(frames)):
        for my in range(ch // 16):
            for mx in range(cw // 16):
                s = err[f, my * 16:my * 16 + 16, mx * 16:mx * 16 + 16].sum() + \
                    err[f, ch + my * 8:ch + my * 8 + 8, mx * 16:mx * 16 + 16].sum()
                assert s <= max(T, 0)
    n_mb = len(frames) * (cw // 16) * (ch // 16)
    assert r["pcm_mbs"] + r["inter_mbs"] + r["skip_mbs"] == n_mb
    assert r["sync"][0] and r["sync"].sum() == r["n_idr"]
    if T < 0:
        assert r["pcm_mbs"] == n_mb


def _decode_full_samples(tmp_path, r, name="o.mp4"):
    cw, ch, sw, sh = r["coded_width"], r["coded_height"], r["width"], r["height"]
    sps, pps = oracle.sps_pps(cw // 16, ch // 16, cw - sw, ch - sh, 30.0)
    n = len(r["samples"])
    path = tmp_path / name
    oracle.write_mp4(path, sps, pps, r["samples"], [i * 1000 for i in range(n)], [0] * n, 30000, sw, sh)
    dec, _ = oracle.decode_full(path)
    return dec


@pytest.mark.parametrize("qp,R,T", [(28, 8, 1536), (20, 8, 1536), (36, 4, 1536), (28, 0, 1536),
                                    (28, 8, -1)])
def test_oracle_residual_coding_round_trip(tmp_path, clip, qp, R, T):
    """Residual coding (P_L0_16x16 + quantised 4x4 residual, CAVLC
    residual_block with nC from the left macroblock): the general oracle
    decoder reads the output back to exactly the encoder's reconstruction,
    every inter macroblock's residual bound stays within the I_PCM payload,
    and the result is smaller than the residual-free encoder's."""
    frames, sc, _ = clip
    r = oracle.transcode(frames, 320, 192, sc, out_height=96, search_range=R, max_mb_sad=T,
                         want_recon=True, qp=qp)
    cw, ch, sw, sh = r["coded_width"], r["coded_height"], r["width"], r["height"]
    rec = r["recon"]
    dec = _decode_full_samples(tmp_path, r)
    assert np.array_equal(dec, np.concatenate([rec[:, :sh, :sw], rec[:, ch:ch + sh // 2, :sw]], 1))
    n_mb = len(frames) * (cw // 16) * (ch // 16)
    assert r["pcm_mbs"] + r["inter_mbs"] + r["skip_mbs"] == n_mb
    if T < 0:
        assert r["pcm_mbs"] == n_mb
        return
    old = oracle.transcode(frames, 320, 192, sc, out_height=96, search_range=R, max_mb_sad=T, qp=0)
    assert sum(map(len, r["samples"])) < sum(map(len, old["samples"]))
    assert r["pcm_mbs"] <= old["pcm_mbs"]
    ds = np.stack([oracle.downscale_nv12(f, 320, 192, 96) for f in frames]).astype(np.float64)
    mse = np.mean((ds[:, :sh, :sw] - rec[:, :sh, :sw].astype(np.float64)) ** 2)
    assert 10 * np.log10(255.0 ** 2 / max(mse, 1e-9)) > 30.0


@pytest.mark.parametrize("at_cuts", [False, True])
def test_oracle_idr_at_keyint_and_optionally_cuts(clip, at_cuts):
    frames, sc, _ = clip
    r = oracle.transcode(frames, 320, 192, sc, out_height=96, keyint=7, idr_at_cuts=at_cuts)
    idr = np.nonzero(r["sync"])[0]
    last = 0
    for f in range(len(frames)):
        is_idr = f == 0 or (at_cuts and sc[f] > 0.08) or f - last >= 7
        last = f if is_idr else last
        assert bool(r["sync"][f]) == is_idr
    assert len(idr) == r["n_idr"]


# ------------------------------------------------ drop-in decision flow

def test_upload_small_file_is_returned(tmp_path):
    p = tmp_path / "v.mp4"
    p.write_bytes(b"x" * 1000)
    assert upload.compress_video_for_upload(p) == p
    assert not (tmp_path / "compressed_v.mp4").exists()


def test_upload_existing_compressed_is_reused(tmp_path):
    p = tmp_path / "v.mp4"
    p.write_bytes(b"x" * (2 << 20))
    c = tmp_path / "compressed_v.mp4"
    c.write_bytes(b"y")
    assert upload.compress_video_for_upload(p, max_size_mb=1) == c


def test_upload_without_gpu_or_ffmpeg_returns_input(tmp_path, monkeypatch, caplog):
    """No usable device (or a stream outside the decoder subset) and no
    ffmpeg: the reference's FileNotFoundError branch -> the input path, and
    no partial output left behind."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    p = tmp_path / "v.mp4"
    scene.synth_write(p, width=320, height=192, n_frames=30)
    monkeypatch.setattr(upload.shutil, "which", lambda name: None)
    with caplog.at_level(logging.WARNING):
        assert upload.compress_video_for_upload(p, max_size_mb=0.01) == p
    assert not (tmp_path / "compressed_v.mp4").exists()
    assert "ffmpeg not installed" in caplog.text
