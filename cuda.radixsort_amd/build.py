"""Build librsort.so (HIP, gfx950) in-tree with hipcc; no torch, no JIT cache.

    python cuda.radixsort_amd/build.py            # incremental
    python cuda.radixsort_amd/build.py --force

Objects go to cuda.radixsort_amd/build/ (git-ignored); the shared library is written next to
this file as librsort.so (git-ignored, but shipped to the GPU box with the snapshot).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
LIB = PKG / "librsort.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["rsort_kernels.hip", "rsort_capi.cpp", "rsort_vendor.hip", "rsort_multi.cpp", "rsort_exchange.cpp"]
HEADERS = [CSRC / "rsort_internal.hpp", CSRC / "rsort_hooks.hpp", ROOT / "include" / "rsort.h"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fvisibility=hidden",
          f"-I{ROOT / 'include'}", f"-I{CSRC}", "-Wall"]


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _compile(src: str, force: bool) -> Path:
    s = CSRC / src
    o = BUILD / (s.stem + ".o")
    if force or _stale(o, [s, *HEADERS]):
        lang = ["-x", "hip"] if s.suffix == ".cpp" else []
        cmd = [HIPCC, *CFLAGS, *lang, "-c", str(s), "-o", str(o)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError(f"hipcc failed for {src}")
    return o


def build(force: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
               "-L/opt/rocm/lib", "-lrccl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("link of librsort.so failed")
        os.replace(tmp, LIB)
    return LIB


CLI_SRC = ROOT / "tools" / "rsort_cli.cpp"
CLI = ROOT / "tools" / "rsort_cli"


def build_cli(force: bool = False) -> Path:
    """The reference-harness CLI (tools/rsort_cli.cpp), linked against librsort.so."""
    lib = build(force)
    if force or _stale(CLI, [CLI_SRC, lib, ROOT / "include" / "radixsort.hpp"]):
        cmd = [HIPCC, "-O2", "-std=c++17", f"-I{ROOT / 'include'}", str(CLI_SRC), "-o", str(CLI),
               f"-L{PKG}", "-lrsort", "-Wl,-rpath,$ORIGIN/../cuda.radixsort_amd"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("build of tools/rsort_cli failed")
    return CLI


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
    print(build_cli())
