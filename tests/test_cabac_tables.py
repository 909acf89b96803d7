"""The product's CABAC / 8x8-transform constants (csrc/h264_cabac_tables.h,
read by the device parser) against the oracle's own transcription
(oracle/h264_std_tables.h, typed in the standard's per-range layout, with the
8x8 zig-zag and normAdjust8x8 computed from their definitions): two
independent copies must agree entry for entry, so a transcription error in
either shows here instead of decoding identically wrong in both.

Tables 9-12..9-33 (I column and cabac_init_idc 0), 9-44 / 9-45 (rangeTabLPS,
transIdxLPS), 9-43 (frame 8x8 significant / last ctxIdxInc), 8.5.6 (8x8
zig-zag), 8.5.9 (v8x8 and its position classes).  Field-coding contexts are
outside both decoders (frame_mbs_only streams) and must be zero in the
product.  Structural checks need no transcription at all: transIdxLPS never
raises the state, rangeTabLPS falls along every row and column, and the
zig-zag is a permutation."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import pytest

import oracle

ROOT = Path(__file__).resolve().parents[1]
FIELD = set(range(277, 399)) | set(range(436, 460))


@pytest.fixture(scope="module")
def product(tmp_path_factory):
    exe = tmp_path_factory.mktemp("cabac") / "dump"
    subprocess.run(["g++", "-std=c++17", "-O0", f"-I{ROOT / 'video-transformer_amd' / 'csrc'}",
                    str(ROOT / "tests" / "native" / "cabac_tables_dump.cpp"), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    tab = {}
    for line in out.splitlines():
        name, i, j, v = line.split()
        tab[(name, int(i), int(j))] = int(v)
    return tab


def std(which: int, i: int, j: int = 0):
    L = oracle.lib()
    L.fo_std_table.restype = C.c_int
    L.fo_std_table.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    ok = C.c_int(0)
    v = L.fo_std_table(which, i, j, C.byref(ok))
    return v if ok.value else None


def test_context_init_tables_agree(product):
    defined_i = defined_p = 0
    for ctx in range(460):
        for col, name in ((0, "init_i"), (1, "init_p0")):
            for j in range(2):
                want = std(col, ctx, j)
                got = product[(name, ctx, j)]
                if ctx in FIELD or ctx == 276:
                    assert got == 0 and want is None, (name, ctx, j)
                elif want is None:
                    # P/B-only syntax in the I column: the product keeps (0, 0)
                    assert col == 0 and 11 <= ctx <= 59 and got == 0, (name, ctx, j)
                else:
                    assert got == want, (name, ctx, j, got, want)
                    defined_i += col == 0
                    defined_p += col == 1
    assert defined_i == 2 * (460 - 49 - len(FIELD) - 1)
    assert defined_p == 2 * (460 - len(FIELD) - 1)


def test_arithmetic_coder_tables_agree(product):
    for p in range(64):
        for q in range(4):
            assert product[("range_lps", p, q)] == std(2, p, q), (p, q)
        assert product[("trans_lps", p, 0)] == std(3, p), p


def test_8x8_tables_agree(product):
    for i in range(63):
        assert product[("sig8", i, 0)] == std(4, i), i
        assert product[("last8", i, 0)] == std(5, i), i
    for i in range(64):
        assert product[("zz8", i, 0)] == std(6, i), i
    for m in range(6):
        for c in range(6):
            assert product[("norm8", m, c)] == std(7, m, c), (m, c)


def test_default_scaling_lists_agree(product):
    """Tables 7-3 / 7-4 (scaling matrices, 8.5.9): both transcriptions, and
    the structure the standard gives them -- constant along each anti-diagonal
    of the scan except the 8x8 lists' third diagonal (13 11 13 / 15 13 15),
    non-decreasing from one diagonal to the next."""
    for l in range(2):
        for k in range(16):
            assert product[("default4", l, k)] == std(8, l, k), (l, k)
        for k in range(64):
            assert product[("default8", l, k)] == std(9, l, k), (l, k)
    for size, which, diag in ((16, 8, [1, 2, 3, 4, 3, 2, 1]), (64, 9, [1, 2, 3, 4, 5, 6, 7, 8, 7, 6, 5, 4, 3, 2, 1])):
        for l in range(2):
            vals = [std(which, l, k) for k in range(size)]
            runs, k = [], 0
            for n in diag:
                runs.append(vals[k:k + n])
                k += n
            for d, r in enumerate(runs):
                if size == 64 and d == 2:
                    assert r[0] == r[2] and r[1] < r[0], (l, r)
                else:
                    assert len(set(r)) == 1, (size, l, d, r)
            heads = [max(r) for r in runs]
            assert heads == sorted(heads), (size, l, heads)


def test_norm8_position_classes_follow_8_5_9(product):
    """8.5.9's six position classes, from their definition."""
    for i in range(8):
        for j in range(8):
            if i % 4 == 0 and j % 4 == 0:
                c = 0
            elif i % 2 == 1 and j % 2 == 1:
                c = 1
            elif i % 4 == 2 and j % 4 == 2:
                c = 2
            elif (i % 4 == 0 and j % 2 == 1) or (i % 2 == 1 and j % 4 == 0):
                c = 3
            elif (i % 4 == 0 and j % 4 == 2) or (i % 4 == 2 and j % 4 == 0):
                c = 4
            else:
                c = 5
            assert product[("norm8_class", i, j)] == c, (i, j)


def test_structural_properties():
    zz = [std(6, i) for i in range(64)]
    assert sorted(zz) == list(range(64))
    assert zz[:6] == [0, 1, 8, 16, 9, 2]
    for p in range(63):
        assert std(3, p) <= p                      # an LPS never raises the state
        row = [std(2, p, q) for q in range(4)]
        assert row == sorted(row)                  # wider range -> wider LPS sub-range
        assert all(std(2, p + 1, q) <= std(2, p, q) for q in range(4))
    assert std(3, 63) == 63 and [std(2, 63, q) for q in range(4)] == [2, 2, 2, 2]
    # every initialisation yields preCtxState in 1..126 for some QP (9.3.1.1)
    for ctx in range(460):
        for col in (0, 1):
            m, n = std(col, ctx, 0), std(col, ctx, 1)
            if m is None:
                continue
            assert -128 <= m <= 127 and -128 <= n <= 127
