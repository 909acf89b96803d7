"""The C-ABI library loads and exports every symbol include/vtseg.h declares
(no GPU needed: nothing here launches device work)."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

from vtseg import _lib

HEADER = Path(__file__).resolve().parents[1] / "include" / "vtseg.h"


def declared_functions() -> set[str]:
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return set(re.findall(r"\b(vts_[a-z0-9_]+)\s*\(", text))


def test_header_and_binding_agree():
    names = declared_functions()
    assert len(names) >= 20
    assert names == set(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    handle = C.CDLL(str(_lib.LIB_PATH))
    for name in declared_functions():
        assert hasattr(handle, name), name


def test_abi_version_and_error_string():
    lib = _lib.lib()
    assert lib.vts_abi_version() == _lib.ABI_VERSION
    n = C.c_int64()
    assert lib.vts_plan_segments(1.0, 1.0, 0.0, None, 0, None) == _lib.VTS_E_INVALID
    assert "n_out" in _lib.last_error()
    assert lib.vts_plan_segments(float("inf"), 1.0, 0.0, None, 0, C.byref(n)) == \
        _lib.VTS_E_NONTERMINATING


def test_struct_layouts_match_header(tmp_path):
    """Compile a probe against include/vtseg.h and compare sizeof/offsetof with
    the ctypes mirrors."""
    import shutil
    import subprocess
    import pytest
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"vts_segment": _lib.Segment, "vts_budget_cfg": _lib.BudgetCfg,
               "vts_plan": _lib.Plan, "vts_video_info": _lib.VideoInfo,
               "vts_score_desc": _lib.ScoreDesc, "vts_params": _lib.Params,
               "vts_synth_params": _lib.SynthParams, "vts_synth_info": _lib.SynthInfo,
               "vts_manifest_args": _lib.ManifestArgs,
               "vts_transcode_params": _lib.TranscodeParams,
               "vts_transcode_info": _lib.TranscodeInfo}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"',
             "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True,
               capture_output=True, text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)
