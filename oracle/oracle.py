"""Python access to the CPU oracle (liboracle.so) plus small pure-Python oracles.

TEST INFRASTRUCTURE — only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.  The product never does.

    plan_segments / plan_with_budget   restate src/utils/video_segmenter.py:42-83
                                       and src/utils/budget_planner.py:73-194
    boundary_frames                    exact rational pts/timescale >= t (Fraction)
    score_frames                       DESIGN.md §Scoring, scalar C
    decode_file                        DESIGN.md §Decoder subset, scalar C
    decode_full                        ITU-T H.264 CAVLC I/P decoding, scalar C
                                       (h264_full_oracle.c)
    transcode / downscale_nv12         DESIGN.md §11 upload transcode, scalar C
                                       (transcode_oracle.c)
"""
from __future__ import annotations

import ctypes as C
import subprocess
from bisect import bisect_left
from fractions import Fraction
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


def build() -> Path:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


class _Seg(C.Structure):
    _fields_ = [("segment_id", C.c_int64), ("start", C.c_double), ("end", C.c_double),
                ("effective_start", C.c_double), ("effective_end", C.c_double),
                ("flags", C.c_int64)]


class BudgetCfg(C.Structure):
    _fields_ = [("default_segment_seconds", C.c_int64), ("overlap_seconds", C.c_int64),
                ("min_segment_seconds", C.c_int64), ("hard_max_api_calls", C.c_int64),
                ("max_continuations", C.c_int64), ("retry_times", C.c_int64),
                ("has_threshold", C.c_int32), ("consolidate", C.c_int32),
                ("duration_threshold_seconds", C.c_double)]


class _Plan(C.Structure):
    _fields_ = [("segment_duration", C.c_int64), ("overlap", C.c_int64),
                ("num_segments", C.c_int64), ("estimated_calls", C.c_int64),
                ("available_calls", C.c_int64), ("hard_max_calls", C.c_int64),
                ("fits_budget", C.c_int32), ("_pad", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _lib.or_plan_segments.argtypes = [C.c_double, C.c_double, C.c_double,
                                          C.POINTER(_Seg), C.c_int64, C.POINTER(C.c_int64)]
        _lib.or_plan_with_budget.argtypes = [C.c_double, C.POINTER(BudgetCfg), C.c_int64,
                                             C.POINTER(_Plan)]
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        _lib.or_parse_sps_pps.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64,
                                          C.c_int, C.c_void_p]
        _lib.or_decode_samples.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_int64, C.c_void_p, C.c_void_p]
        _lib.or_score_frames.argtypes = [
            u8p, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.or_small_width.argtypes = [C.c_int, C.c_int, C.c_int]
        _lib.or_downscale_nv12.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int]
        _lib.or_sps_pps.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p]
        _lib.or_pick_level.argtypes = [C.c_int, C.c_double]
        _lib.or_transcode.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p,
                                      C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_void_p]
    return _lib


def plan_segments(duration: float, seg: float, ovl: float) -> list[tuple]:
    n = C.c_int64(0)
    cap = 4096
    buf = (_Seg * cap)()
    rc = lib().or_plan_segments(float(duration), float(seg), float(ovl), buf, cap,
                                C.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle plan_segments rc={rc}")
    return [(buf[i].segment_id, buf[i].start, buf[i].end, buf[i].effective_start,
             buf[i].effective_end) for i in range(n.value)]


def plan_with_budget(duration: float, cfg: BudgetCfg, count: int):
    p = _Plan()
    rc = lib().or_plan_with_budget(float(duration), C.byref(cfg), int(count), C.byref(p))
    if rc != 0:
        return rc
    return (p.segment_duration, p.overlap, p.num_segments, p.estimated_calls,
            p.available_calls, p.hard_max_calls, bool(p.fits_budget))


def boundary_frames(pts: list[int], timescale: int, times: list[float]) -> list[int]:
    """Index of the first frame with pts/timescale >= t, in exact rationals."""
    out = []
    for t in times:
        if t != t or t == float("inf"):
            out.append(len(pts))
            continue
        if t == float("-inf"):
            out.append(0)
            continue
        thr = Fraction(t) * timescale  # exact
        # first integer pts >= thr  <=>  pts >= ceil(thr)
        c = -((-thr.numerator) // thr.denominator)
        out.append(bisect_left(pts, c))
    return out


def score_frames(nv12: np.ndarray, frame_stride: int, n_frames: int, width: int,
                 height: int, pitch: int, uv_row_offset: int, k: int,
                 prev_luma: np.ndarray | None = None, want_rgb: bool = True):
    """Scalar scorer. nv12 is a flat uint8 array holding n_frames frames."""
    w, h = width // k, height // k
    rgb = np.zeros(n_frames * w * h * 3, np.uint8) if want_rgb else None
    hist = np.zeros(n_frames * 256, np.uint32)
    sad = np.zeros(n_frames, np.uint64)
    score = np.zeros(n_frames, np.float32)
    last = np.zeros(w * h, np.uint8)
    prev = None if prev_luma is None else np.ascontiguousarray(prev_luma, np.uint8)

    def ptr(a):
        return None if a is None else a.ctypes.data

    rc = lib().or_score_frames(np.ascontiguousarray(nv12).reshape(-1), frame_stride,
                               n_frames, width, height, pitch, uv_row_offset, k, ptr(prev),
                               ptr(rgb), ptr(hist), ptr(sad), ptr(score), ptr(last))
    if rc != 0:
        raise RuntimeError(f"oracle score_frames rc={rc}")
    return {"rgb": rgb, "hist": hist.reshape(n_frames, 256), "sad": sad, "score": score,
            "last_luma": last}


# ------------------------------------------------------------- MP4 + decode
class H264Params(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "mb_width", "mb_height", "crop_right", "crop_bottom", "log2_max_frame_num",
        "poc_type", "log2_max_poc_lsb", "delta_pic_order_always_zero",
        "bottom_field_pic_order_in_frame_present", "num_ref_idx_l0_default_active",
        "redundant_pic_cnt_present", "deblocking_filter_control_present", "pic_init_qp",
        "pps_id", "nal_length_size", "chroma_qp_index_offset")]


def _boxes(buf: bytes, start: int, end: int):
    import struct
    pos = start
    while pos + 8 <= end:
        size, typ = struct.unpack(">I4s", buf[pos:pos + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", buf[pos + 8:pos + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - pos
        if size < hdr or pos + size > end:
            raise ValueError("bad box")
        yield typ.decode("latin1"), pos + hdr, pos + size
        pos += size


def read_mp4(path) -> dict:
    """Minimal independent ISO-BMFF reader (first video track, moov only):
    sample offsets/sizes/dts, avcC parameter sets, mvhd/mdhd timing.  Files
    above 64 MiB are memory-mapped (``data`` is then a read-only mmap)."""
    import mmap
    import struct
    p = Path(path)
    if p.stat().st_size > (64 << 20):
        with open(p, "rb") as f:
            data = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    else:
        data = p.read_bytes()
    top = {t: (a, b) for t, a, b in _boxes(data, 0, len(data))}
    ma, mb = top["moov"]
    out = {"data": data}

    def child(a, b, name):
        for t, ca, cb in _boxes(data, a, b):
            if t == name:
                return ca, cb
        return None

    mv = child(ma, mb, "mvhd")
    v = data[mv[0]]
    if v == 1:
        out["movie_timescale"], out["movie_duration"] = struct.unpack(">IQ", data[mv[0] + 20:mv[0] + 32])
    else:
        out["movie_timescale"], out["movie_duration"] = struct.unpack(">II", data[mv[0] + 12:mv[0] + 20])
    for t, ta, tb in _boxes(data, ma, mb):
        if t != "trak":
            continue
        mdia = child(ta, tb, "mdia")
        hdlr = child(*mdia, "hdlr")
        if data[hdlr[0] + 8:hdlr[0] + 12] != b"vide":
            continue
        mdhd = child(*mdia, "mdhd")
        if data[mdhd[0]] == 1:
            ts, dur = struct.unpack(">IQ", data[mdhd[0] + 20:mdhd[0] + 32])
        else:
            ts, dur = struct.unpack(">II", data[mdhd[0] + 12:mdhd[0] + 20])
        stbl = child(*child(*mdia, "minf"), "stbl")
        stsd = child(*stbl, "stsd")
        ea = stsd[0] + 8
        esz = struct.unpack(">I", data[ea:ea + 4])[0]
        avcc = child(ea + 8 + 78, ea + esz, "avcC")
        a = avcc[0]
        lsize = (data[a + 4] & 3) + 1
        p = a + 5
        nsps = data[p] & 31
        p += 1
        sps = []
        for _ in range(nsps):
            n = struct.unpack(">H", data[p:p + 2])[0]
            sps.append(data[p + 2:p + 2 + n])
            p += 2 + n
        npps = data[p]
        p += 1
        pps = []
        for _ in range(npps):
            n = struct.unpack(">H", data[p:p + 2])[0]
            pps.append(data[p + 2:p + 2 + n])
            p += 2 + n
        sa, sb = child(*stbl, "stsz")
        uni, cnt = struct.unpack(">II", data[sa + 4:sa + 12])
        sizes = [uni] * cnt if uni else list(struct.unpack(f">{cnt}I", data[sa + 12:sa + 12 + 4 * cnt]))
        co = child(*stbl, "co64")
        if co:
            nc = struct.unpack(">I", data[co[0] + 4:co[0] + 8])[0]
            chunks = list(struct.unpack(f">{nc}Q", data[co[0] + 8:co[0] + 8 + 8 * nc]))
        else:
            co = child(*stbl, "stco")
            nc = struct.unpack(">I", data[co[0] + 4:co[0] + 8])[0]
            chunks = list(struct.unpack(f">{nc}I", data[co[0] + 8:co[0] + 8 + 4 * nc]))
        sc = child(*stbl, "stsc")
        ne = struct.unpack(">I", data[sc[0] + 4:sc[0] + 8])[0]
        ents = [struct.unpack(">III", data[sc[0] + 8 + 12 * i:sc[0] + 20 + 12 * i]) for i in range(ne)]
        offsets = []
        s = 0
        for i, (first, spc, _) in enumerate(ents):
            last = ents[i + 1][0] if i + 1 < ne else len(chunks) + 1
            for c in range(first, last):
                off = chunks[c - 1]
                for _ in range(spc):
                    if s >= cnt:
                        break
                    offsets.append(off)
                    off += sizes[s]
                    s += 1
        st = child(*stbl, "stts")
        ne = struct.unpack(">I", data[st[0] + 4:st[0] + 8])[0]
        dts, d = [], 0
        for i in range(ne):
            c2, delta = struct.unpack(">II", data[st[0] + 8 + 8 * i:st[0] + 16 + 8 * i])
            for _ in range(c2):
                dts.append(d)
                d += delta
        cts = [0] * cnt
        ct = child(*stbl, "ctts")
        if ct:  # composition offsets (B-frame reordering): pts = dts + offset
            ne = struct.unpack(">I", data[ct[0] + 4:ct[0] + 8])[0]
            i = 0
            for e in range(ne):
                c2, off = struct.unpack(">Ii", data[ct[0] + 8 + 8 * e:ct[0] + 16 + 8 * e])
                for _ in range(c2):
                    if i < cnt:
                        cts[i] = off
                        i += 1
        out.update(timescale=ts, duration=dur, nal_length_size=lsize, sps=sps, pps=pps,
                   offsets=offsets, sizes=sizes, dts=dts[:cnt], cts=cts,
                   pts=[a + b for a, b in zip(dts[:cnt], cts)])
        return out
    raise ValueError("no video track")


def decode_file(path):
    """Decode every frame with the scalar oracle; returns (frames uint8
    [F, H*3/2, W] display-size NV12, info dict)."""
    m = read_mp4(path)
    L = lib()
    prm = H264Params()
    sps, pps = m["sps"][0], m["pps"][0]
    rc = L.or_parse_sps_pps(sps, len(sps), pps, len(pps), m["nal_length_size"], C.byref(prm))
    if rc != 0:
        raise RuntimeError(f"oracle SPS/PPS rc={rc}")
    W = prm.mb_width * 16 - prm.crop_right
    H = prm.mb_height * 16 - prm.crop_bottom
    n = len(m["sizes"])
    out = np.zeros((n, H * 3 // 2, W), np.uint8)
    offs = np.asarray(m["offsets"], np.int64)
    sizes = np.asarray(m["sizes"], np.int64)
    bad = C.c_int64(-1)
    data = np.frombuffer(m["data"], np.uint8)
    rc = L.or_decode_samples(C.byref(prm), data.ctypes.data, offs.ctypes.data,
                             sizes.ctypes.data, n, out.ctypes.data, C.byref(bad))
    if rc != 0:
        raise RuntimeError(f"oracle decode rc={rc} at frame {bad.value}")
    info = {"width": W, "height": H, "timescale": m["timescale"], "pts": m["dts"],
            "movie_timescale": m["movie_timescale"], "movie_duration": m["movie_duration"]}
    return out, info


def recon_hash(frames: np.ndarray) -> int:
    """Hash of decoded display-size NV12 frames, same definition as
    vts_synth_info.recon_hash."""
    F = frames.shape[0]
    flat = frames.reshape(F, -1).astype(np.uint64)
    w = (np.arange(flat.shape[1], dtype=np.uint64) % np.uint64(65521)) + np.uint64(1)
    per = (flat * w).sum(axis=1, dtype=np.uint64)
    return int((per * (np.arange(F, dtype=np.uint64) + np.uint64(1))).sum(dtype=np.uint64))


def slice_commands(nal: bytes | np.ndarray, nal_abs: int, prm: "H264Params", have_ref: bool,
                   cmd_frame: np.ndarray) -> int:
    """or_slice_commands: the oracle parser's per-macroblock command words for
    one slice NAL (checker of the device parser).  Returns 0 or a negative code."""
    L = lib()
    L.or_slice_commands.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int,
                                    C.c_void_p]
    buf = np.frombuffer(bytes(nal), np.uint8)
    return L.or_slice_commands(C.byref(prm), buf.ctypes.data, len(buf), int(nal_abs),
                               1 if have_ref else 0, cmd_frame.ctypes.data)


# ------------------------------------------------------------ upload transcode

def small_width(width: int, height: int, out_height: int = 360) -> int:
    """ffmpeg scale=-2:H output width (transcode_oracle.c or_small_width)."""
    return int(lib().or_small_width(width, height, out_height))


def downscale_nv12(frame: np.ndarray, width: int, height: int, out_height: int = 360) -> np.ndarray:
    """Area downscale of one display-size NV12 frame; returns the coded NV12
    frame [ch*3/2, cw] (16-aligned, edges replicated, samples >= 1)."""
    sw = small_width(width, height, out_height)
    cw, ch = (sw + 15) & ~15, (out_height + 15) & ~15
    src = np.ascontiguousarray(frame, np.uint8).reshape(-1)
    out = np.zeros((ch * 3 // 2, cw), np.uint8)
    rc = lib().or_downscale_nv12(src.ctypes.data, width, height, out.ctypes.data, sw, out_height)
    if rc != 0:
        raise RuntimeError(f"oracle downscale rc={rc}")
    return out


def sps_pps(mbw: int, mbh: int, crop_r: int, crop_b: int, fps: float) -> tuple[bytes, bytes]:
    level = lib().or_pick_level(mbw * mbh, mbw * mbh * fps)
    sps, pps = (C.c_uint8 * 80)(), (C.c_uint8 * 80)()
    sn, pn = C.c_int64(0), C.c_int64(0)
    rc = lib().or_sps_pps(mbw, mbh, crop_r, crop_b, level, sps, C.byref(sn), pps, C.byref(pn))
    if rc != 0:
        raise RuntimeError(f"oracle sps_pps rc={rc}")
    return bytes(sps[:sn.value]), bytes(pps[:pn.value])


def transcode(frames: np.ndarray, width: int, height: int, scores: np.ndarray, *,
              threshold: float = 0.08, out_height: int = 360, search_range: int = 8,
              max_mb_sad: int = 1536, keyint: int = 250, idr_at_cuts: bool = False,
              want_recon: bool = False, qp: int = 28) -> dict:
    """The upload transcode of display-size NV12 frames [F, H*3/2, W] with
    their scene scores: output samples (bytes), per-frame sizes / sync flags,
    SPS/PPS, stats and (optionally) the encoder's reconstruction.  qp >= 1:
    P macroblocks carry a quantised residual at that QP (I_PCM only where the
    residual would cost more); qp <= 0: the round-2 encoder (no residual,
    I_PCM where the prediction misses by more than max_mb_sad)."""
    F = frames.shape[0]
    sw = small_width(width, height, out_height)
    cw, ch = (sw + 15) & ~15, (out_height + 15) & ~15
    mbw, mbh = cw // 16, ch // 16
    fr = np.ascontiguousarray(frames, np.uint8)
    sc = np.ascontiguousarray(scores, np.float32)
    cap = F * mbh * (64 + mbw * 600 + 8) + 64
    out = np.zeros(cap, np.uint8)
    off = np.zeros(F, np.int64)
    size = np.zeros(F, np.int64)
    sync = np.zeros(F, np.uint8)
    recon = np.zeros((F, ch * 3 // 2, cw), np.uint8) if want_recon else None
    stats = np.zeros(4, np.int64)
    n = C.c_int64(0)
    rc = lib().or_transcode(fr.ctypes.data, F, width, height, sc.ctypes.data, threshold,
                            int(idr_at_cuts), out_height, search_range, max_mb_sad, keyint, int(qp),
                            out.ctypes.data, cap,
                            off.ctypes.data, size.ctypes.data, sync.ctypes.data,
                            recon.ctypes.data if recon is not None else None,
                            stats.ctypes.data, C.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle transcode rc={rc}")
    samples = [bytes(out[off[i]:off[i] + size[i]]) for i in range(F)]
    return {"width": sw, "height": out_height, "coded_width": cw, "coded_height": ch,
            "samples": samples, "sync": sync.astype(bool), "recon": recon,
            "pcm_mbs": int(stats[0]), "inter_mbs": int(stats[1]), "skip_mbs": int(stats[2]),
            "n_idr": int(stats[3])}


def decode_samples(sps: bytes, pps: bytes, samples: list[bytes], nal_length_size: int = 4):
    """or_decode_samples on in-memory AVCC samples; returns display-size NV12
    frames [F, H*3/2, W]."""
    L = lib()
    prm = H264Params()
    rc = L.or_parse_sps_pps(sps, len(sps), pps, len(pps), nal_length_size, C.byref(prm))
    if rc != 0:
        raise RuntimeError(f"oracle SPS/PPS rc={rc}")
    W = prm.mb_width * 16 - prm.crop_right
    H = prm.mb_height * 16 - prm.crop_bottom
    n = len(samples)
    data = np.frombuffer(b"".join(samples) + bytes(64), np.uint8)
    sizes = np.array([len(x) for x in samples], np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    out = np.zeros((n, H * 3 // 2, W), np.uint8)
    bad = C.c_int64(-1)
    rc = L.or_decode_samples(C.byref(prm), data.ctypes.data, offs.ctypes.data, sizes.ctypes.data,
                             n, out.ctypes.data, C.byref(bad))
    if rc != 0:
        raise RuntimeError(f"oracle decode rc={rc} at frame {bad.value}")
    return out


def decode_score_gops(path, k: int, threads: int, max_frames: int | None = None,
                      decoder: str = "subset") -> dict:
    """Decode + score a whole MP4 with the scalar oracle, GOP-parallel on
    `threads` host threads (ctypes releases the GIL): every GOP (run of frames
    from an IDR access unit) is decoded by or_decode_samples and scored by
    or_score_frames on its own; the SAD / score of each GOP's first frame is
    then completed against the previous GOP's last thumbnail luma, exactly as
    or_score_frames would have over the whole sequence.  With max_frames, only
    the first GOPs covering that many frames.  decoder "full" decodes with
    the general oracle (h264_full_oracle.c fo_decode; an IDR starts every GOP,
    so GOPs are independent; with B pictures each GOP's frames are put in
    presentation order, which an IDR keeps inside the GOP).  Returns hist [F, 256] u32,
    sad [F] u64, score [F] f32, pts, timescale, the frame count and seconds."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    m = read_mp4(path)
    L = lib()
    prm = H264Params()
    sps, pps = m["sps"][0], m["pps"][0]
    nls = m["nal_length_size"]
    if decoder == "full":
        L.fo_decode.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64, C.c_int, C.c_void_p,
                                C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p,
                                C.c_void_p, C.c_char_p]
        L.fo_dims.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_void_p]
        w_, h_ = C.c_int(0), C.c_int(0)
        if L.fo_dims(sps, len(sps), C.byref(w_), C.byref(h_)):
            raise RuntimeError("oracle SPS")
        W, H = w_.value, h_.value
    else:
        if L.or_parse_sps_pps(sps, len(sps), pps, len(pps), nls, C.byref(prm)):
            raise RuntimeError("oracle SPS/PPS")
        W = prm.mb_width * 16 - prm.crop_right
        H = prm.mb_height * 16 - prm.crop_bottom
    w, h = W // k, H // k
    data = np.frombuffer(m["data"], np.uint8)
    offs = np.asarray(m["offsets"], np.int64)
    sizes = np.asarray(m["sizes"], np.int64)
    pts_all = list(m["pts"])
    idr = [i for i in range(len(offs)) if data[offs[i] + nls] & 0x1F == 5]
    if not idr or idr[0] != 0:
        raise RuntimeError("stream does not start with an IDR access unit")
    gops = list(zip(idr, idr[1:] + [len(offs)]))
    if max_frames is not None:
        keep = []
        for a, b in gops:
            if keep and keep[-1][1] >= max_frames:
                break
            keep.append((a, b))
        gops = keep
    n = gops[-1][1]
    hist = np.zeros((n, 256), np.uint32)
    sad = np.zeros(n, np.uint64)
    score = np.zeros(n, np.float32)
    first_luma: list = [None] * len(gops)
    last_luma: list = [None] * len(gops)

    def work(g):
        a, b = gops[g]
        cnt = b - a
        out = np.empty((cnt, H * 3 // 2, W), np.uint8)
        bad = C.c_int64(-1)
        if decoder == "full":
            err = C.create_string_buffer(256)
            o, z = np.ascontiguousarray(offs[a:b]), np.ascontiguousarray(sizes[a:b])
            if L.fo_decode(sps, len(sps), pps, len(pps), nls, data.ctypes.data, o.ctypes.data,
                           z.ctypes.data, cnt, 0, out.ctypes.data, C.byref(bad), err):
                raise RuntimeError(f"oracle decode_full failed in GOP at frame {a}: "
                                   f"{err.value.decode(errors='replace')}")
        elif L.or_decode_samples(C.byref(prm), data.ctypes.data, offs[a:b].ctypes.data,
                                 sizes[a:b].ctypes.data, cnt, out.ctypes.data, C.byref(bad)):
            raise RuntimeError(f"oracle decode failed in GOP at frame {a}")
        order = sorted(range(cnt), key=lambda i: pts_all[a + i])
        if order != list(range(cnt)):
            out = out[order]
        fr = out.reshape(-1)
        r = score_frames(fr, W * H * 3 // 2, cnt, W, H, W, H, k, want_rgb=False)
        hist[a:b] = r["hist"]
        sad[a:b] = r["sad"]
        score[a:b] = r["score"]
        last_luma[g] = r["last_luma"]
        first_luma[g] = score_frames(fr, W * H * 3 // 2, 1, W, H, W, H, k,
                                     want_rgb=False)["last_luma"]
        return cnt

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max(1, threads)) as ex:
        frames = sum(ex.map(work, range(len(gops))))
    for g in range(1, len(gops)):
        a = gops[g][0]
        s_ = int(np.abs(first_luma[g].astype(np.int32) - last_luma[g - 1].astype(np.int32)).sum())
        sad[a] = s_
        score[a] = np.float32(s_ / (w * h * 255.0))
    dt = time.perf_counter() - t0
    pts_sorted = sorted(pts_all[:n])
    if n < len(pts_all) and pts_sorted[-1] > min(pts_all[n:]):
        raise RuntimeError("a GOP's frames are presented after the next GOP's")
    return {"hist": hist, "sad": sad, "score": score, "frames": frames, "seconds": dt,
            "pts": [int(x) for x in pts_sorted], "timescale": int(m["timescale"]),
            "width": W, "height": H, "gops": len(gops)}


def decode_full(path, flags: int = 0, max_frames: int | None = None):
    """fo_decode (h264_full_oracle.c) over an MP4's first video track: the
    general decoder (CAVLC I/P/B, CABAC I/P; intra, residual, quarter-sample
    motion, direct and weighted prediction, deblocking).  flags bit 0 skips the
    deblocking filter.  Returns (frames uint8 [F, H*3/2, W] display-size NV12
    in presentation order, info dict)."""
    m = read_mp4(path)
    L = lib()
    L.fo_decode.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64, C.c_int, C.c_void_p,
                            C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_void_p,
                            C.c_char_p]
    L.fo_dims.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_void_p]
    sps, pps = m["sps"][0], m["pps"][0]
    w, h = C.c_int(0), C.c_int(0)
    if L.fo_dims(sps, len(sps), C.byref(w), C.byref(h)):
        raise RuntimeError("oracle SPS")
    W, H = w.value, h.value
    n = len(m["sizes"]) if max_frames is None else min(max_frames, len(m["sizes"]))
    out = np.zeros((n, H * 3 // 2, W), np.uint8)
    offs = np.asarray(m["offsets"][:n], np.int64)
    sizes = np.asarray(m["sizes"][:n], np.int64)
    data = np.frombuffer(m["data"], np.uint8)
    bad = C.c_int64(-1)
    err = C.create_string_buffer(256)
    rc = L.fo_decode(sps, len(sps), pps, len(pps), m["nal_length_size"], data.ctypes.data,
                     offs.ctypes.data, sizes.ctypes.data, n, flags, out.ctypes.data,
                     C.byref(bad), err)
    if rc != 0:
        raise RuntimeError(f"oracle decode_full rc={rc} at frame {bad.value}: "
                           f"{err.value.decode(errors='replace')}")
    # display order: frames sorted by presentation time (dts + ctts offset);
    # without B pictures this is the decoding order
    pts = m["pts"][:n]
    order = sorted(range(n), key=lambda i: pts[i])
    if order != list(range(n)):
        out = out[order]
    info = {"width": W, "height": H, "timescale": m["timescale"], "pts": [pts[i] for i in order]}
    return out, info


def table_code(table: int, a: int, b: int, c: int = 0) -> str | None:
    """The standard's VLC bit strings kept by h264_full_oracle.c: table 0
    coeff_token [column][TotalCoeff][TrailingOnes], 1 total_zeros 4x4
    [TotalCoeff-1][total_zeros], 2 total_zeros chroma DC, 3 run_before
    [min(zerosLeft,7)-1][run]."""
    L = lib()
    L.fo_table_code.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int]
    L.fo_table_code.restype = C.c_char_p
    v = L.fo_table_code(table, a, b, c)
    return None if v is None else v.decode()


def write_mp4(path, sps: bytes, pps: bytes, samples: list[bytes], dts: list[int], cts: list[int],
              timescale: int, width: int, height: int, nal_length_size: int = 4) -> None:
    """Minimal ISO-BMFF writer (one avc1 track, one chunk; ctts when any
    composition offset is non-zero; stss from the IDR samples).  TEST
    INFRASTRUCTURE for streams the oracle synthesises (cabac_convert)."""
    import struct

    def box(t, p):
        return struct.pack(">I4s", 8 + len(p), t) + p

    def full(t, v, f, p):
        return box(t, struct.pack(">I", (v << 24) | f) + p)
    n = len(samples)
    dur = (dts[-1] - dts[0] + (dts[-1] - dts[-2] if n > 1 else 1)) if n else 0
    matrix = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)
    ms = dur * 1000 // max(1, timescale)
    mvhd = full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, 1000, ms) + struct.pack(">IH", 0x10000, 0x100) +
                b"\0" * 10 + matrix + b"\0" * 24 + struct.pack(">I", 2))
    tkhd = full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, ms) + b"\0" * 8 +
                struct.pack(">HHHH", 0, 0, 0, 0) + matrix + struct.pack(">II", width << 16, height << 16))
    mdhd = full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, timescale, dur, 0x55c4, 0))
    hdlr = full(b"hdlr", 0, 0, struct.pack(">I4s", 0, b"vide") + b"\0" * 12 + b"VideoHandler\0")
    avcc = box(b"avcC", bytes([1, sps[1], sps[2], sps[3], 0xFC | (nal_length_size - 1), 0xE1]) +
               struct.pack(">H", len(sps)) + sps + bytes([1]) + struct.pack(">H", len(pps)) + pps)
    avc1 = box(b"avc1", b"\0" * 6 + struct.pack(">H", 1) + b"\0" * 16 + struct.pack(">HH", width, height) +
               struct.pack(">II", 0x480000, 0x480000) + b"\0" * 4 + struct.pack(">H", 1) + b"\0" * 32 +
               struct.pack(">Hh", 0x18, -1) + avcc)
    stsd = full(b"stsd", 0, 0, struct.pack(">I", 1) + avc1)
    deltas = [dts[i + 1] - dts[i] for i in range(n - 1)] + ([dts[-1] - dts[-2]] if n > 1 else [1])
    runs = []
    for dl in deltas:
        if runs and runs[-1][1] == dl:
            runs[-1][0] += 1
        else:
            runs.append([1, dl])
    stts = full(b"stts", 0, 0, struct.pack(">I", len(runs)) + b"".join(struct.pack(">II", c, dl) for c, dl in runs))
    extra = b""
    if any(cts):
        extra += full(b"ctts", 0, 0, struct.pack(">I", n) + b"".join(struct.pack(">Ii", 1, c) for c in cts))
    sync = []
    for i, smp in enumerate(samples):
        p = 0
        while p + nal_length_size <= len(smp):
            ln = int.from_bytes(smp[p:p + nal_length_size], "big")
            if smp[p + nal_length_size] & 31 == 5:
                sync.append(i + 1)
                break
            p += nal_length_size + ln
    extra += full(b"stss", 0, 0, struct.pack(">I", len(sync)) + b"".join(struct.pack(">I", x) for x in sync))
    stsc = full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, n, 1))
    stsz = full(b"stsz", 0, 0, struct.pack(">II", 0, n) + b"".join(struct.pack(">I", len(x)) for x in samples))
    ftyp = box(b"ftyp", b"isom" + struct.pack(">I", 512) + b"isomiso2avc1mp41")

    def build(off):
        co64 = full(b"co64", 0, 0, struct.pack(">IQ", 1, off))
        stbl = box(b"stbl", stsd + stts + extra + stsc + stsz + co64)
        dinf = box(b"dinf", full(b"dref", 0, 0, struct.pack(">I", 1) + full(b"url ", 0, 1, b"")))
        minf = box(b"minf", full(b"vmhd", 0, 1, b"\0" * 8) + dinf + stbl)
        return box(b"moov", mvhd + box(b"trak", tkhd + box(b"mdia", mdhd + hdlr + minf)))
    moov = build(0)
    payload = b"".join(samples)
    off = len(ftyp) + len(moov) + 8
    moov = build(off)
    with open(path, "wb") as f:
        f.write(ftyp + moov + struct.pack(">I4s", 8 + len(payload), b"mdat") + payload)


def cabac_convert(src, dst, seed: int = 1, t8: bool = False):
    """Re-code a CAVLC MP4 (the synthetic writer's) as CABAC with
    h264_full_oracle.c fo_cabac_convert: every slice header is kept (plus
    cabac_init_idc 0), the macroblock layer is random syntax generated by the
    oracle's own CABAC parser in synthesis mode and arithmetic-coded (9.3.4).
    Returns the frames the synthesis decoded (decode order, display size).
    TEST INFRASTRUCTURE: the resulting stream pins nothing against the
    standard beyond the parser's own restatement; it gives the device
    decoder's CABAC paths a stream with every syntax element to match."""
    m = read_mp4(src)
    L = lib()
    L.fo_cabac_convert.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64, C.c_int, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_int64, C.c_uint64, C.c_int, C.c_void_p,
                                   C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_char_p]
    L.fo_dims.argtypes = [C.c_char_p, C.c_int64, C.c_void_p, C.c_void_p]
    sps, pps = m["sps"][0], m["pps"][0]
    w, h = C.c_int(0), C.c_int(0)
    if L.fo_dims(sps, len(sps), C.byref(w), C.byref(h)):
        raise RuntimeError("oracle SPS")
    W, H = w.value, h.value
    n = len(m["sizes"])
    data = np.frombuffer(m["data"], np.uint8)
    offs = np.asarray(m["offsets"], np.int64)
    sizes = np.asarray(m["sizes"], np.int64)
    nmb = ((W + 15) // 16) * ((H + 15) // 16)
    cap = int(sizes.sum()) * 4 + n * (nmb * 512 + 4096)
    out = np.zeros(cap, np.uint8)
    osz = np.zeros(n, np.int64)
    pps_out = np.zeros(256, np.uint8)
    pps_len = C.c_int64(0)
    frames = np.zeros((n, H * 3 // 2, W), np.uint8)
    bad = C.c_int64(-1)
    err = C.create_string_buffer(256)
    rc = L.fo_cabac_convert(sps, len(sps), pps, len(pps), m["nal_length_size"], data.ctypes.data,
                            offs.ctypes.data, sizes.ctypes.data, n, seed, int(t8), out.ctypes.data, cap,
                            osz.ctypes.data, pps_out.ctypes.data, C.byref(pps_len), frames.ctypes.data,
                            C.byref(bad), err)
    if rc != 0:
        raise RuntimeError(f"fo_cabac_convert rc={rc} at frame {bad.value}: {err.value.decode(errors='replace')}")
    samples, p = [], 0
    for s in osz:
        samples.append(out[p:p + int(s)].tobytes())
        p += int(s)
    write_mp4(dst, bytes(sps), pps_out[:pps_len.value].tobytes(), samples, m["dts"], m["cts"],
              m["timescale"], W, H, m["nal_length_size"])
    return frames
