"""Malformed inputs against the host code that reads untrusted files (VERDICT
r04 item 5): the MP4 reader, the probe, the slice-header scheduler, the
stream-copy cutter, and — through the CPU harness — the very parser,
derivation and reconstruction code the device runs.  They are built with
AddressSanitizer + UndefinedBehaviorSanitizer (tests/native/fuzz_host.cpp +
full_host.cpp) and fed truncated and bit-flipped copies of synthetic streams
(subset, CAVLC full syntax, CABAC B, video-like content) and of the real
CABAC clip, in a child process with the sanitizer runtimes preloaded; every
call must return a status (probe_duration a float, as the reference's
"never raises, returns 0.0", src/utils/video_utils.py:28-38) and no
sanitizer may report.  The product's Python probe is checked on the same
files.  The device side of the same bytes (a corrupted slice failing with
VTS_E_DECODE) is tests/test_decode_gpu.py::test_corrupted_slice_data_fails_loudly."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import fmp4
import oracle
from vtseg import scene
from vtseg.video_utils import probe_duration

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "video-transformer_amd" / "csrc"
NATIVE = ROOT / "tests" / "native"
REAL = ROOT / "tests" / "golden" / "real" / "realshort.mp4"


def _runtime(name: str) -> str | None:
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def fuzz_lib(tmp_path_factory):
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("sanitizer runtimes not installed")
    so = tmp_path_factory.mktemp("fz") / "libfz.so"
    srcs = [NATIVE / "fuzz_host.cpp", NATIVE / "full_host.cpp"] + [
        CSRC / f for f in ("mp4.cpp", "h264.cpp", "h264_sched.cpp", "plan.cpp", "probe.cpp", "remux.cpp")]
    subprocess.run(["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                    "-fno-omit-frame-pointer", "-std=c++20", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                    "-pthread", f"-I{CSRC}", f"-I{ROOT / 'include'}", *map(str, srcs), "-o", str(so)],
                   check=True)
    return so, f"{asan}:{ubsan}"


def _seeds(d: Path) -> list[Path]:
    kw = dict(width=64, height=48, n_frames=10, cut_min_s=0.1, cut_max_s=0.2, gop_max_s=0.2)
    out = []
    p = d / "subset.mp4"
    scene.synth_write(p, seed=3, **kw)
    out.append(p)
    p = d / "cavlc_b.mp4"
    scene.synth_write(p, seed=5, coding="full", bframes=True, weighted="implicit", max_motion=3, **kw)
    out.append(p)
    src, p = d / "src.mp4", d / "cabac_b.mp4"
    scene.synth_write(src, seed=7, coding="full", bframes=True, weighted="implicit", chunks=1, **kw)
    oracle.cabac_convert(src, p, seed=9, t8=True)
    out.append(p)
    p = d / "content.mp4"
    scene.synth_write(p, seed=11, coding="full", bframes=True, weighted="implicit", cabac=True,
                      transform_8x8=True, content=True, **kw)
    out.append(p)
    p = d / "fragmented.mp4"  # movie fragments (tfhd / tfdt / trun) of the CABAC B stream
    fmp4.fragment(out[2], p, per_fragment=3)
    out.append(p)
    out.append(REAL)
    return out


def _mutants(seeds: list[Path], d: Path, per_seed: int) -> list[Path]:
    """Truncations at random lengths and 1-8 flipped bits anywhere (header
    boxes, sample tables and slice data alike), seeded."""
    rng = np.random.default_rng(2024)
    out = []
    for s in seeds:
        data = np.frombuffer(s.read_bytes(), np.uint8)
        for k in range(per_seed):
            m = data.copy()
            if k % 3 == 0:
                m = m[:int(rng.integers(8, len(m)))]
            else:
                for _ in range(int(rng.integers(1, 9))):
                    i = int(rng.integers(0, len(m)))
                    m[i] ^= np.uint8(1 << int(rng.integers(0, 8)))
            p = d / f"{s.stem}_{k}.mp4"
            p.write_bytes(m.tobytes())
            out.append(p)
    return out


def test_mutated_files_never_crash_the_host_parsers(tmp_path, fuzz_lib):
    so, preload = fuzz_lib
    seeds = _seeds(tmp_path)
    files = seeds + _mutants(seeds, tmp_path, per_seed=24)
    env = dict(os.environ, LD_PRELOAD=preload,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    proc = subprocess.run([sys.executable, str(NATIVE / "fuzz_driver.py"), str(so), str(tmp_path),
                           *map(str, files)], env=env, capture_output=True, text=True, timeout=600)
    assert proc.returncode == 0, proc.stderr[-4000:]
    assert "runtime error" not in proc.stderr and "AddressSanitizer" not in proc.stderr, proc.stderr[-4000:]
    stats = json.loads(proc.stdout.strip().splitlines()[-1])
    assert stats["files"] == len(files)
    # the unmutated seeds all go through every stage
    assert stats["decode_ok"] >= len(seeds) and stats["schedule_ok"] >= len(seeds)


def test_probe_duration_returns_a_float_on_mutated_files(tmp_path):
    """The product's probe_duration (native moov rule, ffprobe fallback)
    returns a float and never raises, whatever the bytes."""
    seeds = _seeds(tmp_path)
    for p in seeds + _mutants(seeds, tmp_path, per_seed=8) + [tmp_path / "missing.mp4"]:
        d = probe_duration(str(p))
        assert isinstance(d, float) and d >= 0.0
