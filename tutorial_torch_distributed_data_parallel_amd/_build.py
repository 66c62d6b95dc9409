"""Native build driver: compiles csrc/ for gfx950 into the in-tree extension ``_C*.so``.

No hipify, no torch.utils.cpp_extension JIT cache: device code (``*.hip``) is compiled by
``hipcc --offload-arch=gfx950``; host C++ (``*.cpp``, which includes the PyTorch and RCCL
headers) by the host compiler; everything is linked against the HIP runtime and RCCL that
PyTorch itself bundles (``torch/lib``), so the process carries exactly one HIP runtime and one
RCCL (hazard "two RCCL builds coexist").

Usage:  python -m tutorial_torch_distributed_data_parallel_amd._build [--force] [-j N]
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

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = CSRC / "build"
ARCH = os.environ.get("TDP_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_dirs():
    import torch  # noqa: F401  (import only to locate the install)

    root = Path(torch.__file__).resolve().parent
    return root / "include", root / "lib"


def so_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"_C{suffix}"


def _sources():
    return sorted(CSRC.glob("*.hip")), sorted(CSRC.glob("*.cpp"))


def _headers():
    return sorted(CSRC.glob("*.h"))


def _includes(src: Path, seen=None) -> set:
    """The in-tree headers ``src`` includes, transitively (``#include "x.h"`` lines)."""
    seen = set() if seen is None else seen
    for line in src.read_text().splitlines():
        line = line.strip()
        if line.startswith('#include "'):
            h = CSRC / line.split('"')[1]
            if h.exists() and h not in seen:
                seen.add(h)
                _includes(h, seen)
    return seen


def _needs(obj: Path, src: Path, headers) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    deps = _includes(src) & set(headers)
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hipcc = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    cxx = os.environ.get("CXX", shutil.which("g++") or "g++")
    tinc, tlib = _torch_dirs()
    py_inc = sysconfig.get_paths()["include"]
    BUILD.mkdir(parents=True, exist_ok=True)
    hip_srcs, cpp_srcs = _sources()
    headers = _headers()
    common = ["-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-I{CSRC}", f"-I{ROCM / 'include'}"]
    torch_flags = ["-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_EXTENSION_NAME=_C",
                   "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{tinc}",
                   f"-I{tinc / 'torch' / 'csrc' / 'api' / 'include'}", f"-I{py_inc}"]
    jobs_list = []
    for s in hip_srcs:
        o = BUILD / (s.stem + ".hip.o")
        if force or _needs(o, s, headers):
            # the split-bf16 GEMM keeps its f32 residual subtractions scalar: packed f32 VALU
            # (v_pk_add_f32) costs ~4x a v_sub_f32's issue slot beside MFMAs
            extra = ["-fno-slp-vectorize"] if s.name in ("gemm_f32_fast.hip", "gemm_planes.hip", "gemm_emu8.hip") else []
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", *common, "-ffp-contract=fast",
                              *extra, "-c", str(s), "-o", str(o)])
    for s in cpp_srcs:
        o = BUILD / (s.stem + ".cpp.o")
        if force or _needs(o, s, headers):
            extra = torch_flags if s.name == "bindings.cpp" else []
            jobs_list.append([cxx, *common, *extra, "-pthread", "-Wno-deprecated-declarations",
                              "-c", str(s), "-o", str(o)])
    jobs = jobs or min(len(jobs_list), max(1, min(8, os.cpu_count() or 1))) or 1
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for cmd, fut in [(c, ex.submit(_run, c)) for c in jobs_list]:
                fut.result()
                if verbose:
                    print("built", cmd[-1])
    objs = [str(BUILD / (s.stem + ".hip.o")) for s in hip_srcs] + \
           [str(BUILD / (s.stem + ".cpp.o")) for s in cpp_srcs]
    out = so_path()
    if force or jobs_list or not out.exists():
        tmp = out.with_suffix(".tmp.so")
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(tmp),
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", "-lamdhip64", "-lrccl", "-pthread", f"-Wl,-rpath,{tlib}"])
        os.replace(tmp, out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    p = build(force=a.force, jobs=a.j, verbose=True)
    print(p)


if __name__ == "__main__":
    sys.exit(main())
