"""In-tree build of the native extensions (gfx950 only).

Produces, next to this file:
  * ``_C.so``  - HIP kernels (``csrc/kernels/*.hip``, ``csrc/comm/*.hip``, hipcc --offload-arch=gfx950)
                 + PyTorch bindings (``csrc/bindings/*.cpp``).
  * ``_rt.so`` - the host runtime (``csrc/runtime/*.cpp``): paged-KV block
                 manager, continuous-batching scheduler core, BPE/byte tokenizer
                 helpers. Pure C++17 + pybind11, no HIP dependency, so the CPU
                 test tier exercises it too.

Objects are cached under ``csrc/build/`` and rebuilt only when a source or a
header is newer. Kernel translation units include only HIP headers, so they
compile in seconds; only the single binding TU pulls in the torch headers.

Usage: ``python -m generativeaiexamples_amd._build [-j N] [--force] [-v]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = CSRC / "build"
ARCH = os.environ.get("GAI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _newest_header() -> float:
    hs = list((CSRC / "include").glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _includes(src: Path, seen: set | None = None) -> set:
    """Project headers a source includes, transitively (quoted includes found in csrc/include or next to it)."""
    import re

    seen = set() if seen is None else seen
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', src.read_text(errors="ignore"), re.M):
        for d in (src.parent, CSRC / "include", CSRC / "runtime"):
            h = d / name
            if h.exists() and h not in seen:
                seen.add(h)
                _includes(h, seen)
                break
    return seen


def _needs(obj: Path, src: Path, hdr_time: float) -> bool:
    """Rebuild when the object is older than its source or than any project header it includes."""
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(h.stat().st_mtime > t for h in _includes(src))


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd[:3])} ... {cmd[-1]}")
    elif verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch

    inc = ce.include_paths(device_type="cuda") if hasattr(ce, "include_paths") else []
    libdir = str(Path(torch.__file__).parent / "lib")
    return inc, libdir, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def build_rt(jobs: int = 8, force: bool = False, verbose: bool = False) -> Path:
    import pybind11

    out = PKG / "_rt.so"
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr = _newest_header()
    pyinc = sysconfig.get_paths()["include"]
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", f"-I{CSRC / 'include'}",
             f"-I{pybind11.get_include()}", f"-I{pyinc}", f"-I{CSRC / 'runtime'}", "-fvisibility=hidden"]
    objs, todo = [], []
    for s in srcs:
        o = BUILD / (s.stem + ".rt.o")
        objs.append(o)
        if force or _needs(o, s, hdr):
            todo.append([CXX, *flags, "-c", str(s), "-o", str(o)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), todo))
    if force or todo or not out.exists():
        _run([CXX, "-shared", "-o", str(out), *map(str, objs), "-lpthread"], verbose)
    return out


def build_c(jobs: int = 8, force: bool = False, verbose: bool = False) -> Path:
    out = PKG / "_C.so"
    BUILD.mkdir(parents=True, exist_ok=True)
    hdr = _newest_header()
    inc, torch_lib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    hip_flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{CSRC / 'include'}",
                 "-munsafe-fp-atomics", "-Wno-unused-result"]
    cxx_flags = ["-O2", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}", f"-I{pyinc}",
                 "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                 "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations",
                 *[f"-I{p}" for p in inc]]
    todo, objs = [], []
    for s in sorted((CSRC / "kernels").glob("*.hip")) + sorted((CSRC / "comm").glob("*.hip")):
        o = BUILD / (s.stem + ".hip.o")
        objs.append(o)
        if force or _needs(o, s, hdr):
            todo.append([HIPCC, *hip_flags, "-c", str(s), "-o", str(o)])
    for s in sorted((CSRC / "bindings").glob("*.cpp")):
        o = BUILD / (s.stem + ".bind.o")
        objs.append(o)
        if force or _needs(o, s, hdr):
            todo.append([CXX, *cxx_flags, "-c", str(s), "-o", str(o)])
    # the torch-binding TU is the slow one: start it first
    todo.sort(key=lambda c: 0 if c[0] == CXX else 1)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), todo))
    if force or todo or not out.exists():
        _run([CXX, "-shared", "-o", str(out), *map(str, objs), f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}",
              "-lamdhip64", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python"],
             verbose)
    return out


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    build_rt(jobs, force, verbose)
    build_c(jobs, force, verbose)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--only", choices=["rt", "c"], default=None)
    a = ap.parse_args()
    if a.only == "rt":
        build_rt(a.jobs or 8, a.force, a.verbose)
    elif a.only == "c":
        build_c(a.jobs or 8, a.force, a.verbose)
    else:
        build(a.jobs, a.force, a.verbose)
    print("build ok")


if __name__ == "__main__":
    main()
