"""The device slice parser (csrc/parse_slice.h, run per slice by h264_parse on
the GPU) compiled for the host by a test-only harness, checked command word
for command word against the oracle's parser (oracle/vtseg_oracle.c
or_slice_commands) on the synthetic streams the GPU parity tests use.  Lets
parser changes be verified without a GPU; the GPU tests then check the same
code on the device (tests/test_decode_gpu.py)."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from vtseg import scene

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "video-transformer_amd" / "csrc"

SHAPES = [
    ("qvga", dict(width=320, height=240)),
    ("median", dict(width=320, height=240, slices_per_row=0, max_motion=8)),
    ("ragged", dict(width=336, height=200, slices_per_row=3, max_motion=6)),
    ("nhd", dict(width=640, height=360, slices_per_row=2, max_motion=2)),
    ("static", dict(width=96, height=64, max_motion=0)),
    ("bigpan", dict(width=320, height=240, max_motion=24)),
    ("halfpel", dict(width=320, height=240, max_motion=5, odd_motion=True)),
    ("tiny", dict(width=32, height=32, slices_per_row=0, max_motion=4)),
    ("hd720", dict(width=1280, height=720, max_motion=4)),
]

# H264DevParams int32 fields in declaration order (h264.h)
DEV_FIELDS = ["mb_width", "mb_height", "log2_max_frame_num", "poc_type", "log2_max_poc_lsb",
              "delta_pic_order_always_zero", "bottom_field_pic_order_in_frame_present",
              "num_ref_idx_l0_default_active", "redundant_pic_cnt_present",
              "deblocking_filter_control_present", "pic_init_qp", "chroma_qp_index_offset", "pps_id"]


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    out = tmp_path_factory.mktemp("ph") / "libparse_host.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", f"-I{CSRC}",
                    f"-I{ROOT / 'include'}", str(ROOT / "tests" / "native" / "parse_host.cpp"),
                    "-o", str(out)], check=True)
    lib = C.CDLL(str(out))
    lib.ph_parse_slice.restype = C.c_uint32
    lib.ph_parse_slice.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_void_p, C.c_void_p]
    return lib


def _slices(m):
    """(frame, nal_offset, nal_size) of every slice NAL in decode order."""
    data, nls = m["data"], m["nal_length_size"]
    for f, (off, size) in enumerate(zip(m["offsets"], m["sizes"])):
        p, end = off, off + size
        while p + nls <= end:
            n = int.from_bytes(data[p:p + nls], "big")
            p += nls
            if data[p] & 0x1F in (1, 5):
                yield f, p, n
            p += n


def _compare(harness, path, n_frames):
    m = oracle.read_mp4(path)
    prm = oracle.H264Params()
    sps, pps = m["sps"][0], m["pps"][0]
    assert oracle.lib().or_parse_sps_pps(sps, len(sps), pps, len(pps), m["nal_length_size"],
                                         C.byref(prm)) == 0
    nmb = prm.mb_width * prm.mb_height
    p14 = np.array([getattr(prm, f) if f else 0 for f in DEV_FIELDS], np.int32)
    es = np.zeros(len(m["data"]) + 256, np.uint8)  # device ES buffers are padded too
    es[:len(m["data"])] = np.frombuffer(m["data"], np.uint8)
    dev = np.zeros((n_frames, nmb), np.uint64)
    ref = np.zeros((n_frames, nmb), np.uint64)
    n_slices = 0
    for f, off, size in _slices(m):
        rc = oracle.slice_commands(m["data"][off:off + size], off, prm, f > 0, ref[f])
        assert rc == 0, (f, rc)
        err = harness.ph_parse_slice(es.ctypes.data, off, size, f, 0 if f > 0 else -1,
                                     p14.ctypes.data, dev.ctypes.data)
        assert err == 0, (f, off, hex(err))
        n_slices += 1
    bad = np.argwhere(dev != ref)
    assert bad.size == 0, (bad[:5].tolist(), [hex(int(dev[tuple(b)])) for b in bad[:5]],
                           [hex(int(ref[tuple(b)])) for b in bad[:5]])
    assert (dev != 0).all()
    return n_slices


@pytest.mark.parametrize("name,kw", SHAPES, ids=[s[0] for s in SHAPES])
def test_device_parser_matches_oracle(harness, tmp_path, name, kw):
    n = 24 if name == "hd720" else 40
    path = tmp_path / f"{name}.mp4"
    scene.synth_write(path, n_frames=n, cut_min_s=0.3, cut_max_s=0.8, gop_max_s=0.5, **kw)
    assert _compare(harness, path, n) > 0


def test_device_parser_rejects_bad_mb_type(harness):
    """An I slice whose macroblock type is not I_PCM is outside the subset."""
    # hand-made I slice: first_mb 0, slice_type 7, pps 0, frame_num(4 bits),
    # idr_pic_id 0, poc lsb (4 bits), dec_ref_pic_marking 00, qp delta 0,
    # deblock idc 1, then mb_type ue(0) = I_NxN, then a stop bit
    bits = "1" + "0001000" + "1" + "0000" + "1" + "0000" + "00" + "1" + "010" + "1" + "1"
    bits += "0" * (-len(bits) % 8)
    payload = int(bits, 2).to_bytes(len(bits) // 8, "big")
    nal = bytes([0x65]) + payload
    es = np.zeros(len(nal) + 256, np.uint8)
    es[:len(nal)] = np.frombuffer(nal, np.uint8)
    p14 = np.array([2, 2, 4, 0, 4, 0, 0, 1, 0, 1, 26, 0, 0], np.int32)
    cmd = np.zeros(4, np.uint64)
    err = harness.ph_parse_slice(es.ctypes.data, 0, len(nal), 0, -1, p14.ctypes.data,
                                 cmd.ctypes.data)
    assert err & (1 << 1), hex(err)  # DEC_E_MB_TYPE


class _BitWriter:
    def __init__(self):
        self.bits: list[str] = []

    def u(self, v: int, n: int):
        if n:
            self.bits.append(format(v, f"0{n}b"))

    def ue(self, v: int):
        x = v + 1
        n = x.bit_length()
        self.bits.append("0" * (n - 1) + format(x, "b"))

    def se(self, v: int):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def rbsp(self) -> bytes:
        s = "".join(self.bits) + "1"
        s += "0" * (-len(s) % 8)
        return int(s, 2).to_bytes(len(s) // 8, "big") if s else b""


def _ebsp(rbsp: bytes) -> bytes:
    """7.4.1: insert emulation_prevention_three_byte after 00 00 before 00..03."""
    out, zeros = bytearray(), 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


@pytest.mark.parametrize("seed", range(12))
def test_device_parser_matches_oracle_on_random_p_slices(harness, seed):
    """Random CAVLC P slices (skip runs, large motion-vector differences whose
    long Exp-Golomb codes make zero bytes and so emulation-prevention bytes,
    I_PCM macroblocks, slices starting mid-row) through both parsers."""
    rng = np.random.default_rng(seed)
    mbw, mbh = int(rng.integers(2, 9)), int(rng.integers(1, 6))
    nmb = mbw * mbh
    prm = oracle.H264Params()
    prm.mb_width, prm.mb_height = mbw, mbh
    prm.log2_max_frame_num, prm.poc_type = 16, 2
    prm.num_ref_idx_l0_default_active, prm.deblocking_filter_control_present = 1, 1
    prm.pic_init_qp, prm.nal_length_size = 26, 4
    p14 = np.array([getattr(prm, f) if f else 0 for f in DEV_FIELDS], np.int32)
    checked = n_epb = 0
    for trial in range(400):
        if checked >= 40 and n_epb >= 2:
            break
        first = int(rng.integers(0, nmb))
        w = _BitWriter()
        w.ue(first)
        w.ue(5)                                   # P
        w.ue(0)                                   # pps
        w.u(int(rng.integers(0, 1 << 16)) if trial % 2 else 0, 16)  # frame_num (0: zero bytes)
        w.u(0, 1)                                 # num_ref_idx_active_override
        w.u(0, 1)                                 # ref_pic_list_modification_flag_l0
        w.u(0, 1)                                 # adaptive_ref_pic_marking_mode_flag
        w.se(0)                                   # slice_qp_delta
        w.ue(1)                                   # disable_deblocking_filter_idc
        addr = first
        sign = [1, -1]
        end = int(rng.integers(first + 1, nmb + 1))
        while addr < end:
            run = int(rng.integers(0, 4)) if rng.random() < 0.6 else 0
            run = min(run, end - addr)
            w.ue(run)
            addr += run
            if addr >= end:
                break
            r = rng.random()
            if r < 0.15:
                w.ue(30)                          # I_PCM
                w.bits.append("0" * (-len("".join(w.bits)) % 8))
                for _ in range(384):
                    w.u(int(rng.integers(1, 256)), 8)
            else:
                w.ue(0)                           # P_L0_16x16
                if rng.random() < 0.4:
                    # (+m, -m) with m a power of two: the two codes meet in a
                    # run of 2k+6 zero bits, so zero bytes and emulation-
                    # prevention bytes; the sign alternates so vectors stay in range
                    sign[0] = -sign[0]
                    m = (1 << int(rng.integers(10, 12))) * 4
                    w.se(sign[0] * m)
                    w.se(-sign[0] * m)
                else:
                    w.se(int(rng.integers(-8, 9)) * 4)
                    w.se(int(rng.integers(-8, 9)) * 4)
                w.ue(0)                           # coded_block_pattern 0
            addr += 1
        rbsp = w.rbsp()
        nal = bytes([0x41]) + _ebsp(rbsp)
        ref = np.zeros(nmb, np.uint64)
        rc = oracle.slice_commands(nal, 16, prm, True, ref)
        if rc != 0:  # e.g. a motion vector beyond 16 bits: not a case to compare
            continue
        es = np.zeros(16 + len(nal) + 256, np.uint8)
        es[16:16 + len(nal)] = np.frombuffer(nal, np.uint8)
        dev = np.zeros(nmb, np.uint64)
        err = harness.ph_parse_slice(es.ctypes.data, 16, len(nal), 0, 0, p14.ctypes.data,
                                     dev.ctypes.data)
        if err == (1 << 9):  # EPB right at an I_PCM start: refused loudly by design
            continue
        assert err == 0 or err == (1 << 3), (seed, trial, hex(err))  # SUBPEL never here
        assert np.array_equal(dev, ref), (seed, trial, np.argwhere(dev != ref)[:4].tolist())
        checked += 1
        n_epb += len(nal) - 1 - len(rbsp) > 0
    assert checked >= 40
    assert n_epb >= 1  # slices with emulation-prevention bytes were compared
