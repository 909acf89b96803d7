"""Guard against a gfx950 codegen hazard seen with ROCm 7.2 hipcc: pairs of
clamp(x >> 8, 0, 255) selected as v_ashr_pk_u8_i32 produced wrong bytes in the
RGB thumbnails.  The kernels must not contain that instruction."""
from __future__ import annotations

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "video-transformer_amd" / "csrc"
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.parametrize("src", ["score.hip", "decode.hip"])
def test_no_v_ashr_pk_u8_in_kernels(tmp_path, src):
    if not Path(HIPCC).exists() and shutil.which("hipcc") is None:
        pytest.skip("hipcc not available")
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT / 'include'}",
                    f"-I{CSRC}", "--cuda-device-only", "-S", "-o", str(out), str(CSRC / src)],
                   check=True, capture_output=True)
    asm = out.read_text()
    assert "s_endpgm" in asm
    assert "v_ashr_pk_u8_i32" not in asm
