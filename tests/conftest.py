"""Shared test setup: import paths, the `gpu` marker, in-tree builds."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "video-transformer_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (ROOT, PKG, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built() -> None:
    lib = PKG / "vtseg" / "libvtseg.so"
    if not lib.exists():
        sys.path.insert(0, str(PKG))
        import build as _b  # video-transformer_amd/build.py
        _b.build()
    import oracle  # oracle/oracle.py
    if not oracle.LIB.exists():
        oracle.build()


_ensure_built()


def load_golden(name: str):
    return json.loads((GOLDEN / name).read_text())


def fhex(s) -> float:
    return float.fromhex(s) if isinstance(s, str) else float(s)


def same_float(a: float, b: float) -> bool:
    """Bit-exact float equality (NaN == NaN, 0.0 != -0.0)."""
    return float(a).hex() == float(b).hex()


@pytest.fixture(scope="session")
def golden():
    return load_golden
