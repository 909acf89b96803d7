"""Build libvtseg.so in-tree: host C++ with g++, device code with hipcc (gfx950).

    python video-transformer_amd/build.py [--clean] [-j N]

Objects go to video-transformer_amd/build/, the library to
video-transformer_amd/vtseg/libvtseg.so (git-ignored, travels with gpurun).
Rebuilds only sources newer than their object (headers force a full rebuild).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
OUT = PKG / "vtseg" / "libvtseg.so"
INCLUDE = ROOT / "include"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = "gfx950"

CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wextra", "-Wno-unused-parameter",
            f"-I{INCLUDE}", f"-I{CSRC}"]
HIPFLAGS = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", f"-I{INCLUDE}",
            f"-I{CSRC}", "-Wall", "-Wno-unused-parameter", "-munsafe-fp-atomics"]


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + proc.stdout + proc.stderr)
        raise SystemExit(f"build failed: {cmd[-1]}")
    if proc.stderr.strip():
        sys.stderr.write(proc.stderr)


def _newest_header() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def build(clean: bool = False, jobs: int = 8, verbose: bool = False) -> Path:
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(exist_ok=True)
    hdr = _newest_header()
    jobs_list = []
    objs = []
    for src in sorted(CSRC.glob("*.cpp")) + sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.name + ".o")
        objs.append(obj)
        if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr):
            continue
        if src.suffix == ".hip":
            cmd = [HIPCC, *HIPFLAGS, "-c", str(src), "-o", str(obj)]
        else:
            cmd = ["g++", *CXXFLAGS, "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include",
                   "-c", str(src), "-o", str(obj)]
        jobs_list.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for cmd in jobs_list:
            if verbose:
                print(" ".join(cmd))
        list(ex.map(_run, jobs_list))
    if jobs_list or not OUT.exists():
        tmp = OUT.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp),
              *map(str, objs), f"-L{ROCM}/lib", "-lamdhip64", "-Wl,-z,defs",
              "-Wl,-rpath," + str(ROCM / "lib")])
        os.replace(tmp, OUT)
    return OUT


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    print(build(a.clean, a.j, a.v))


if __name__ == "__main__":
    main()
