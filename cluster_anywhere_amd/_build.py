"""In-tree native build (no setuptools, no hipify).

Two shared objects are produced next to this file:

* ``_C``      – the gfx950 HIP kernels (``csrc/kernels/*.hip``) + torch bindings,
                compiled with ``hipcc --offload-arch=gfx950`` and linked against the
                torch / HIP runtime that torch itself loads.
* ``_native`` – the C++ runtime (object store, scheduler, channels;
                ``csrc/runtime/*.cc``), compiled with g++ + pybind11. It does not
                depend on torch so CPU worker processes start without importing it.

Rebuilds are incremental on source mtime. ``python -m cluster_anywhere_amd._build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD_DIR = os.path.join(REPO, "build", "native")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("CAAMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _jobs() -> int:
    return max(1, min(int(os.environ.get("MAX_JOBS", "8")), 16))


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def kernels_path() -> str:
    return os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)


def native_path() -> str:
    return os.path.join(PKG_DIR, "_native" + EXT_SUFFIX)


# Per-source extra hipcc flags. The D = 64 attention kernels are VALU-issue-bound
# next to their MFMAs; packed f32 ops (v_pk_add/mul_f32, formed by SLP
# vectorisation of adjacent scalar adds/multiplies) cost more issue cycles there
# than the scalar pair (cdna_hip_programming.md: packed f32 VALU beside MFMAs).
PER_FILE_FLAGS = {"flash_attn_d64.hip": ["-fno-slp-vectorize"]}


def build_kernels(verbose: bool = False, force: bool = False) -> str:
    import torch
    import torch.utils.cpp_extension as ce

    src_dir = os.path.join(CSRC, "kernels")
    hip_srcs = sorted(glob.glob(os.path.join(src_dir, "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(src_dir, "*.h")))
    out = kernels_path()
    if not force and not _newer(out, hip_srcs + cpp_srcs + headers):
        return out
    os.makedirs(BUILD_DIR, exist_ok=True)
    torch_inc = ce.include_paths(device_type="cuda")
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    py_inc = sysconfig.get_paths()["include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    common = [
        "-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
    ]
    objs = []
    jobs = []
    for s in hip_srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            jobs.append([HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics",
                         *PER_FILE_FLAGS.get(os.path.basename(s), []), "-I", src_dir, "-c", s, "-o", o])
    for s in cpp_srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            inc = sum((["-I", p] for p in torch_inc + [py_inc, src_dir]), [])
            jobs.append([HIPCC, *common, "-DTORCH_EXTENSION_NAME=_C",
                         "-DTORCH_API_INCLUDE_EXTENSION_H", *inc, "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(_jobs()) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *objs, "-o", out + ".tmp",
            f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", f"-Wl,-rpath,{torch_lib}"]
    _run(link, verbose)
    os.replace(out + ".tmp", out)
    return out


def build_native(verbose: bool = False, force: bool = False) -> str:
    import pybind11

    src_dir = os.path.join(CSRC, "runtime")
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cc")))
    headers = sorted(glob.glob(os.path.join(src_dir, "*.h")))
    out = native_path()
    if not srcs:
        return ""
    if not force and not _newer(out, srcs + headers):
        return out
    os.makedirs(BUILD_DIR, exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    extra = os.environ.get("CAAMD_NATIVE_CFLAGS", "").split()
    cmd = ["g++", "-O2", "-g", "-fPIC", "-shared", "-std=c++17", "-Wall", "-Wno-unused-function",
           "-I", pybind11.get_include(), "-I", py_inc, "-I", src_dir, *extra, *srcs,
           "-o", out + ".tmp", "-lpthread", "-lrt"]
    _run(cmd, verbose)
    os.replace(out + ".tmp", out)
    return out


def build_all(verbose: bool = False, force: bool = False):
    with cf.ThreadPoolExecutor(2) as ex:
        a = ex.submit(build_native, verbose, force)
        b = ex.submit(build_kernels, verbose, force)
        return a.result(), b.result()


if __name__ == "__main__":
    v = "-v" in sys.argv
    f = "-f" in sys.argv
    print(build_all(verbose=v, force=f))
