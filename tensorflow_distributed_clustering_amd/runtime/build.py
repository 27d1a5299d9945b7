"""In-tree build of the native extension ``_C.so`` (HIP kernels + torch op bindings).

No hipify, no torch JIT cache: every ``csrc/*.hip`` file is compiled by ``hipcc
--offload-arch=gfx950`` into an object, ``csrc/*.cpp`` (bindings, host runtime) by the
host compiler against the torch headers, and everything is linked into
``tensorflow_distributed_clustering_amd/_C.so`` next to the package, so the built
library travels with the repository snapshot to the GPU box.

    python -m tensorflow_distributed_clustering_amd.runtime.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

PKG_DIR = Path(__file__).resolve().parent.parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "obj"
OUT = PKG_DIR / "_C.so"
ARCH = os.environ.get("TDC_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch.utils.cpp_extension as ce
    return ce.include_paths(), ce.library_paths()


def _hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return p


def _needs(obj: Path, deps: List[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: List[str], verbose: bool):
    if verbose:
        print("[tdc build]", " ".join(cmd[:3]), "...", cmd[-1], flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"compile failed: {' '.join(cmd)}")
    return r


def build(force: bool = False, verbose: bool = True, jobs: int = 0) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    cpp_srcs = sorted(CSRC.glob("*.cpp"))
    inc, libdirs = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hipcc = _hipcc()
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}"]
    tasks = []
    objs = []
    for src in hip_srcs:
        obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
        if force or _needs(obj, [src] + headers):
            tasks.append([hipcc, f"--offload-arch={ARCH}", *common, "-c", str(src), "-o", str(obj)])
    for src in cpp_srcs:
        obj = BUILD / (src.stem + ".cpp.o")
        objs.append(obj)
        if force or _needs(obj, [src] + headers):
            cxx = os.environ.get("CXX", "g++")
            tasks.append([cxx, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                          "-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_EXTENSION_NAME=_C",
                          *[f"-I{p}" for p in inc], f"-I{ROCM / 'include'}", f"-I{py_inc}",
                          "-c", str(src), "-o", str(obj)])
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(lambda c: _run(c, verbose), tasks))
    if force or tasks or not OUT.exists() or _needs(OUT, objs):
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(o) for o in objs],
                "-o", str(OUT), *[f"-L{p}" for p in libdirs],
                *[f"-Wl,-rpath,{p}" for p in libdirs],
                "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                f"-L{ROCM / 'lib'}", "-lamdhip64"]
        _run(link, verbose)
    return OUT


def _check_abi():
    import torch
    return torch._C._GLIBCXX_USE_CXX11_ABI


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-q", "--quiet", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, verbose=not a.quiet, jobs=a.jobs)
    print(out)


if __name__ == "__main__":
    main()
