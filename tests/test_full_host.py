"""The general device decoder's own code on the CPU: the host scheduler
(h264_sched.cpp: slice headers, reference lists, marking) and the exact
per-slice parser and per-macroblock reconstruction / deblocking routines the
GPU kernels run (parse_full.h, recon_full.h), driven in the kernels' order
(inter macroblocks first, then intra ones and the deblocking filter along the
x + 2y wavefront) by tests/native/full_host.cpp — must decode every stream
exactly like the independent oracle (h264_full_oracle.c), before and after
the deblocking filter.  The GPU tests then only have to show that the
kernels schedule this code faithfully."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from vtseg import scene

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "video-transformer_amd" / "csrc"


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    so = tmp_path_factory.mktemp("fh") / "libfullhost.so"
    srcs = [ROOT / "tests" / "native" / "full_host.cpp"] + [CSRC / f for f in
                                                             ("mp4.cpp", "h264.cpp", "h264_sched.cpp",
                                                              "plan.cpp")]
    subprocess.run(["g++", "-Og", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                    f"-I{CSRC}", f"-I{ROOT / 'include'}", *map(str, srcs), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    lib.fh_decode.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_char_p, C.c_int]

    def decode(path, flags=0):
        m = oracle.read_mp4(path)
        n = len(m["sizes"])
        w, h = C.c_int(0), C.c_int(0)
        cap = n * 1920 * 1088 * 3 // 2
        out = np.zeros(cap, np.uint8)
        got = C.c_int64(0)
        err = C.create_string_buffer(256)
        rc = lib.fh_decode(str(path).encode(), flags, out.ctypes.data, cap, C.byref(got),
                           C.byref(w), C.byref(h), err, 256)
        if rc:
            raise RuntimeError(err.value.decode())
        W, H = w.value, h.value
        return out[:got.value * W * H * 3 // 2].reshape(got.value, H * 3 // 2, W)
    return decode


STREAMS = [
    ("subset", dict(width=320, height=240)),
    ("subset_halfpel", dict(width=320, height=240, max_motion=5, odd_motion=True)),
    ("subset_nonref", dict(width=160, height=96, max_motion=4, gop_max_s=0.3, nonref_refresh=True)),
    ("full_tiny", dict(width=48, height=32, coding="full", max_motion=2)),
    ("full_qvga", dict(width=320, height=240, coding="full", max_motion=3)),
    ("full_ragged", dict(width=336, height=200, slices_per_row=3, max_motion=6, coding="full")),
    ("full_oneslice", dict(width=320, height=240, slices_per_row=0, max_motion=8, coding="full")),
    ("full_cip", dict(width=320, height=240, coding="full", constrained_intra=True)),
    ("full_crop", dict(width=480, height=270, slices_per_row=2, coding="full")),
]


@pytest.mark.parametrize("name,kw", STREAMS, ids=[s[0] for s in STREAMS])
def test_device_code_on_cpu_equals_oracle(tmp_path, harness, name, kw):
    kw = dict(kw)
    gop = kw.pop("gop_max_s", 0.7)
    path = tmp_path / f"{name}.mp4"
    scene.synth_write(path, n_frames=60, cut_min_s=0.5, cut_max_s=1.5, gop_max_s=gop, seed=21,
                      **kw)
    for flags in (1, 0):   # before and after the deblocking filter
        want, _ = oracle.decode_full(path, flags=flags)
        got = harness(path, flags)
        assert got.shape == want.shape
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


B_STREAMS = [
    ("spatial", {}),
    ("explicit", {"weighted": "explicit"}),
    ("implicit", {"weighted": "implicit"}),
    ("temporal", {"temporal_direct": True}),
    ("slices", {"slices_per_row": 2, "weighted": "implicit", "temporal_direct": True}),
]


@pytest.mark.parametrize("name,kw", B_STREAMS, ids=[s[0] for s in B_STREAMS])
def test_b_pictures_on_cpu_equal_oracle(tmp_path, harness, name, kw):
    """Main-profile B streams (synth_full.cpp: reordered mini-GOPs, B reference
    pictures, spatial / temporal direct, every B partition shape, explicit /
    implicit weighted prediction, P slices with explicit weights): the
    product's scheduler (POC, B list initialisation), CAVLC B parser (direct
    prediction from the colocated records) and bi-predictive reconstruction /
    B deblocking equal the oracle in presentation order."""
    path = tmp_path / f"b_{name}.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=45, coding="full", bframes=True, cut_min_s=0.5,
                      cut_max_s=1.2, gop_max_s=0.8, seed=11, chunks=1, **kw)
    for flags in (1, 0):
        want, _ = oracle.decode_full(path, flags=flags)
        got = harness(path, flags)
        assert got.shape == want.shape
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


CABAC_STREAMS = [
    ("p", {}, False),
    ("b_spatial", {"bframes": True}, False),
    ("b_spatial_t8", {"bframes": True}, True),
    ("b_explicit_t8", {"bframes": True, "weighted": "explicit"}, True),
    ("b_temporal_implicit", {"bframes": True, "temporal_direct": True, "weighted": "implicit"}, False),
    ("b_slices_t8", {"bframes": True, "slices_per_row": 2}, True),
]


@pytest.mark.parametrize("name,kw,t8", CABAC_STREAMS, ids=[s[0] for s in CABAC_STREAMS])
def test_cabac_b_streams_on_cpu_equal_oracle(tmp_path, harness, name, kw, t8):
    """CABAC P / B streams (oracle.cabac_convert: the writer's slice headers,
    CABAC macroblock layers synthesised by the oracle's parser — every B
    mb_type / sub_mb_type, both lists' ref_idx / mvd contexts, direct
    quadrants, transform_size_8x8_flag): the product's CABAC parser and
    reconstruction equal the oracle, before and after deblocking."""
    src, dst = tmp_path / "src.mp4", tmp_path / f"{name}.mp4"
    scene.synth_write(src, width=176, height=144, n_frames=30, coding="full", cut_min_s=0.5, cut_max_s=1.2,
                      gop_max_s=0.8, seed=3, chunks=1, **kw)
    oracle.cabac_convert(src, dst, seed=5, t8=t8)
    for flags in (1, 0):
        want, _ = oracle.decode_full(dst, flags=flags)
        got = harness(dst, flags)
        assert got.shape == want.shape
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


def test_real_cabac_high_profile_stream(harness):
    """A real High-profile CABAC clip (tests/golden/real/realshort.mp4:
    CABAC I/P slices, 8x8 transform, Intra 8x8) through the product's CABAC
    parser and reconstruction on the CPU equals the oracle frame for frame."""
    path = ROOT / "tests" / "golden" / "real" / "realshort.mp4"
    want, _ = oracle.decode_full(path)
    got = harness(path)
    assert got.shape == want.shape
    bad = [i for i in range(len(want)) if not np.array_equal(got[i], want[i])]
    assert bad == []


WRITER_CABAC = [
    ("ip", {}),
    ("ip_t8", {"transform_8x8": True}),
    ("ip_t8_rows", {"transform_8x8": True, "slices_per_row": 1}),
    ("ip_cip_t8", {"transform_8x8": True, "constrained_intra": True}),
    ("b", {"bframes": True}),
    ("b_t8_implicit", {"bframes": True, "transform_8x8": True, "weighted": "implicit"}),
    ("b_t8_explicit_temporal", {"bframes": True, "transform_8x8": True, "weighted": "explicit",
                                "temporal_direct": True}),
]


@pytest.mark.parametrize("name,kw", WRITER_CABAC, ids=[s[0] for s in WRITER_CABAC])
def test_writer_cabac_streams_on_cpu_equal_oracle(tmp_path, harness, name, kw):
    """The stream writer's own CABAC output (synth_full.cpp, cabac=True:
    Main / High profile, the writer's syntax decisions arithmetic-coded with
    its own binarizations and context selection; Intra_8x8 and 8x8-transform
    inter macroblocks with transform_8x8): every slice must parse to its stop
    bit in the oracle, and the product's CABAC parser and reconstruction must
    equal the oracle before and after deblocking."""
    kw = dict(kw)
    spr = kw.pop("slices_per_row", 0)
    path = tmp_path / f"wc_{name}.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=36, coding="full", cabac=True,
                      slices_per_row=spr, cut_min_s=0.4, cut_max_s=1.0, gop_max_s=0.6, seed=13,
                      chunks=1, **kw)
    for flags in (1, 0):
        want, _ = oracle.decode_full(path, flags=flags)
        got = harness(path, flags)
        assert got.shape == want.shape
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


SCALING = [
    ("cavlc_sps", {"scaling": "sps"}),
    ("cavlc_pps", {"scaling": "pps"}),
    ("cavlc_both_b", {"scaling": "both", "bframes": True}),
    ("cabac_sps_t8", {"scaling": "sps", "cabac": True, "transform_8x8": True}),
    ("cabac_pps_t8", {"scaling": "pps", "cabac": True, "transform_8x8": True}),
    ("cabac_both_t8_b", {"scaling": "both", "cabac": True, "transform_8x8": True, "bframes": True,
                         "weighted": "implicit"}),
    ("cabac_pps_no_t8", {"scaling": "pps", "cabac": True}),
]


@pytest.mark.parametrize("name,kw", SCALING, ids=[s[0] for s in SCALING])
@pytest.mark.parametrize("seed", [5, 6])
def test_scaling_matrix_streams_on_cpu_equal_oracle(tmp_path, harness, name, kw, seed):
    """Streams with scaling matrices (8.5.9; the writer's seeded lists in the
    SPS, the PPS or both: absent lists under fall-back rules A / B,
    useDefaultScalingMatrixFlag, lists that end early, full lists; 4x4 and
    8x8, intra and inter, luma and chroma, Intra16x16 and chroma DC): the
    product's LevelScale tables (h264_sched.cpp) and dequantisation must
    equal the oracle's own restatement frame for frame."""
    path = tmp_path / f"sc_{name}_{seed}.mp4"
    scene.synth_write(path, width=176, height=144, n_frames=24, coding="full", slices_per_row=0,
                      cut_min_s=0.4, cut_max_s=1.0, gop_max_s=0.6, seed=seed, **kw)
    for flags in (1, 0):
        want, _ = oracle.decode_full(path, flags=flags)
        got = harness(path, flags)
        assert got.shape == want.shape
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"
