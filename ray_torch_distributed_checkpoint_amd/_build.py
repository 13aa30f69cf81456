"""In-tree native build of the `_C` extension (HIP kernels for gfx950 + C++ runtime).

Drives `hipcc` directly instead of `torch.utils.cpp_extension` so no hipify pass ever touches
the sources (they are CDNA4 HIP, not CUDA): every `.hip` kernel file is compiled with
`--offload-arch=gfx950` into an object, the single torch-binding TU is compiled once, and all
are linked into `ray_torch_distributed_checkpoint_amd/_C*.so` next to this file, so the built
library travels with the repo snapshot to the GPU box.  Incremental: an object is rebuilt only
when its source or any shared header is newer.

    python -m ray_torch_distributed_checkpoint_amd._build [-v] [-j N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "build")
EXT_NAME = "_C"


def _arch() -> str:
    return os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    incs = [
        os.path.join(tdir, "include"),
        os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
        sysconfig.get_paths()["include"],
    ]
    return tdir, incs, int(torch._C._GLIBCXX_USE_CXX11_ABI)


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG_DIR, EXT_NAME + suffix)


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> str:
    os.makedirs(BUILD_DIR, exist_ok=True)
    tdir, incs, abi = _torch_paths()
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    arch = _arch()
    headers = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hdr_time = _newest(headers)

    kernel_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    binding_src = os.path.join(CSRC, "bindings.cpp")
    runtime_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))

    steps = []
    objs = []
    for src in kernel_srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_time):
            steps.append([hipcc, f"--offload-arch={arch}", "-O3", "-fPIC", "-std=c++17", "-I", CSRC,
                          "-c", src, "-o", obj])
    bobj = os.path.join(BUILD_DIR, "bindings.o")
    objs.append(bobj)
    bdeps = [binding_src] + runtime_srcs
    if force or not os.path.exists(bobj) or os.path.getmtime(bobj) < max(_newest(bdeps), hdr_time):
        cmd = [hipcc, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-DTORCH_EXTENSION_NAME={EXT_NAME}", "-DTORCH_API_INCLUDE_EXTENSION_H",
               f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", CSRC]
        for i in incs:
            cmd += ["-I", i]
        cmd += ["-c", binding_src, "-o", bobj]
        steps.append(cmd)

    if steps:
        n = jobs or int(os.environ.get("MAX_JOBS", "0") or 0) or min(16, os.cpu_count() or 4)
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            futs = [ex.submit(_run, s, verbose) for s in steps]
            for f in futs:
                f.result()

    out = ext_path()
    if force or steps or not os.path.exists(out) or os.path.getmtime(out) < _newest(objs):
        tmp = out + ".tmp"
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={arch}", *objs, "-o", tmp,
                "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                "-ltorch_hip", "-ltorch_python", "-lhsa-runtime64", "-lz", f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
        _run(link, verbose)
        os.replace(tmp, out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.verbose, a.jobs, a.force))


if __name__ == "__main__":
    sys.exit(main())
