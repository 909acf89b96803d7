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
    subprocess.run(["g++", "-Og", "-std=c++20", "-fPIC", "-shared", "-Wno-unknown-pragmas", "-pthread",
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


def _writer_list_kinds(seed: int, n: int) -> list[int]:
    """synth_full.cpp write_scaling_lists(): the kind of each list (0 absent,
    1 useDefaultScalingMatrixFlag, 2 ends early, 3 full) for one seed."""
    M = (1 << 64) - 1
    x = (seed * 0x9E3779B97F4A7C15 + 0x2545F4914F6CDD1D) & M

    def rnd(m):
        nonlocal x
        x ^= (x << 13) & M
        x ^= x >> 7
        x ^= (x << 17) & M
        return x % m
    kinds = []
    for i in range(n):
        kind = rnd(4)
        kinds.append(kind)
        if kind < 2:
            continue
        size = 16 if i < 6 else 64
        stop = 1 + rnd(size - 1) if kind == 2 else size
        for _ in range(stop):
            rnd(61)
    return kinds


def test_pps_only_scaling_falls_back_by_rule_a(tmp_path):
    """7.4.2.2 / Table 7-2: a PPS scaling matrix over an SPS without one
    (seq_scaling_matrix_present_flag 0) falls back by rule A, so absent lists
    0 (Intra Y) and 3 (Inter Y) are Default_4x4_Intra / Default_4x4_Inter
    (Table 7-3), not the SPS's Flat_16.  LevelScale4x4 = weightScale x
    normAdjust4x4 (8.5.9), checked by hand at three positions per list."""
    so = tmp_path / "libfh_scale.so"
    srcs = [ROOT / "tests" / "native" / "full_host.cpp"] + [CSRC / f for f in
                                                             ("mp4.cpp", "h264.cpp", "h264_sched.cpp",
                                                              "plan.cpp")]
    subprocess.run(["g++", "-O1", "-std=c++20", "-fPIC", "-shared", "-Wno-unknown-pragmas", "-pthread",
                    f"-I{CSRC}", f"-I{ROOT / 'include'}", *map(str, srcs), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    # the PPS's lists are seeded with seed * 2 + 2 (synth_full.cpp make_sps_pps_full)
    seed = next(s for s in range(1, 4000)
                if (lambda k: k[0] == 0 and k[3] == 0 and any(k))(_writer_list_kinds(s * 2 + 2, 6)))
    path = tmp_path / "pps_only.mp4"
    scene.synth_write(path, width=64, height=48, n_frames=4, coding="full", slices_per_row=0,
                      seed=seed, scaling="pps")
    ls4 = np.zeros((6, 6, 16), np.int32)
    ls8 = np.zeros((2, 6, 64), np.int32)
    flags = np.zeros(2, np.int32)
    err = C.create_string_buffer(256)
    assert lib.fh_scale(str(path).encode(), ls4.ctypes.data_as(C.c_void_p),
                        ls8.ctypes.data_as(C.c_void_p), flags.ctypes.data_as(C.c_void_p), err, 256) == 0, \
        err.value
    assert flags.tolist() == [0, 1]
    # raster (i, j) -> zig-zag index: (0,0) 0, (0,1) 1, (1,1) 4, (3,3) 15
    # Default_4x4_Intra[0, 1, 4, 15] = 6, 13, 20, 42; Inter = 10, 14, 20, 34
    # normAdjust4x4, qP % 6 = 0: v0 = 10 (i, j even), v1 = 16 (both odd), v2 = 13
    # qP % 6 = 5: 18, 29, 23
    assert [ls4[0, 0, 0], ls4[0, 0, 1], ls4[0, 0, 5], ls4[0, 0, 15]] == [60, 169, 320, 672]
    assert [ls4[3, 0, 0], ls4[3, 0, 1], ls4[3, 0, 5], ls4[3, 0, 15]] == [100, 182, 320, 544]
    assert [ls4[0, 5, 0], ls4[3, 5, 15]] == [6 * 18, 34 * 29]
    # rule A for the lists after an absent one: list 1 / 4 copy list 0 / 3 when absent too
    k = _writer_list_kinds(seed * 2 + 2, 6)
    for i in (1, 2, 4, 5):
        if k[i] == 0 and all(k[j] == 0 for j in range(3 * (i // 3), i)):
            assert np.array_equal(ls4[i], ls4[3 * (i // 3)])
    # and the oracle decodes the stream exactly like the product's harness
    want, _ = oracle.decode_full(path, flags=0)
    lib.fh_decode.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                              C.c_void_p, C.c_char_p, C.c_int]
    cap = 4 * 64 * 48 * 3 // 2
    out = np.zeros(cap, np.uint8)
    n, w, h = C.c_int64(0), C.c_int(0), C.c_int(0)
    assert lib.fh_decode(str(path).encode(), 0, out.ctypes.data, cap, C.byref(n), C.byref(w),
                         C.byref(h), err, 256) == 0, err.value
    assert np.array_equal(out[:want.size].reshape(want.shape), want)


LANES = [
    ("cavlc_qvga", dict(width=320, height=240, coding="full", max_motion=3)),
    ("cavlc_cip", dict(width=176, height=144, coding="full", max_motion=3, constrained_intra=True)),
    ("cabac_t8_b", dict(width=176, height=144, coding="full", cabac=True, transform_8x8=True, bframes=True,
                        weighted="implicit")),
    ("cabac_t8_scaled", dict(width=176, height=144, coding="full", cabac=True, transform_8x8=True,
                             scaling="both")),
]


@pytest.mark.parametrize("name,kw", LANES, ids=[x[0] for x in LANES])
def test_lane_parallel_intra_on_cpu_equals_oracle(tmp_path, harness, name, kw):
    """The device's lane-parallel intra reconstruction (intra_lanes.h, the
    h264_intra_v2 kernel's per-macroblock code) run with 32 host threads as
    the lanes, macroblocks in the kernel's level order with its line
    buffers: every frame equals the oracle before and after deblocking."""
    path = tmp_path / f"lanes_{name}.mp4"
    scene.synth_write(path, n_frames=16, cut_min_s=0.3, cut_max_s=0.6, gop_max_s=0.4, seed=31,
                      slices_per_row=0 if kw.get("cabac") else 1, **kw)
    for flags in (3, 2):
        want, _ = oracle.decode_full(path, flags=flags & 1)
        got = harness(path, flags)
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


TIGHT = [
    ("content_qvga", dict(width=320, height=240, n_frames=72, seed=7, content=True)),
    ("content_720p", dict(width=1280, height=720, n_frames=24, seed=3, content=True)),
    ("noise_b_t8", dict(width=320, height=240, n_frames=36, seed=9, content=False)),
]


@pytest.mark.parametrize("name,kw", TIGHT, ids=[x[0] for x in TIGHT])
def test_exact_cabac_arena_on_cpu_equals_oracle(tmp_path, harness, name, kw):
    """The CABAC arena at exactly the blocks the slices ask for (chunked
    allocation from the window's counter, h264_full.h kArenaChunk): a counting
    parse, then the decode with that capacity, a canary region after it and
    the parser's LDS poisoned (0xA5): the canaries stay (no store past the
    blocks handed out) and every frame equals the oracle before and after
    deblocking (suspect (a))."""
    kw = dict(kw)
    path = tmp_path / f"tight_{name}.mp4"
    scene.synth_write(path, fps=30, cut_min_s=0.3, cut_max_s=0.8, gop_max_s=0.5, chunks=1,
                      coding="full", slices_per_row=0, max_motion=4, bframes=True, weighted="implicit",
                      cabac=True, transform_8x8=True, **kw)
    for flags in (9, 8):
        want, _ = oracle.decode_full(path, flags=flags & 1)
        got = harness(path, flags)
        bad = np.nonzero((got != want).reshape(got.shape[0], -1).any(1))[0]
        assert bad.size == 0, f"flags {flags}: frames {bad[:8].tolist()} differ"


def test_exact_cabac_arena_real_stream(harness):
    """The same exact arena on the real High-profile CABAC clip (realshort.mp4)."""
    path = ROOT / "tests" / "golden" / "real" / "realshort.mp4"
    want, _ = oracle.decode_full(path)
    got = harness(path, 8)
    assert np.array_equal(got, want)
