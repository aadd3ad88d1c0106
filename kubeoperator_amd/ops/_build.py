"""In-tree build of the gfx950 HIP extension ``kubeoperator_amd/_C.so``.

No hipify step and no ``torch.utils.cpp_extension`` JIT cache: every ``csrc/*.hip`` translation unit is
compiled by ``hipcc --offload-arch=gfx950`` (they include no PyTorch headers, so each takes seconds),
``bindings.cpp`` is compiled once as host C++ against the PyTorch headers, and the objects are linked
into one shared object next to the package so it travels with the source tree (``gpurun`` snapshots it).

Incremental: an object is rebuilt only when its source or any ``csrc/*.h`` header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "_build")
SO_PATH = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("KOP_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    return root, inc, os.path.join(root, "lib"), bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc() -> str:
    for cand in (os.path.join(ROCM, "bin", "hipcc"), shutil.which("hipcc") or ""):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build kubeoperator_amd kernels)")


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _needs(obj: str, src: str, hdr_mtime: float) -> bool:
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return m < os.path.getmtime(src) or m < hdr_mtime


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError("build command failed:\n" + " ".join(cmd) + "\n" + res.stdout)


# per-file hipcc flags: the one-wave-per-SIMD dK/dV kernel keeps its builtin MFMAs in VGPR form (its dK/dV
# accumulators are AGPR inline-asm operands; hipcc's heuristic would put every MFMA in AGPR form)
FILE_FLAGS = {"flash_bwd_w1.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=true"],
              "flash_fwd4.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=true", "-fno-slp-vectorize", "-fno-honor-nans"]}


# probe builds only (tools/build_ab.py --ablations): never set for the shipped extension
EXTRA_HIPFLAGS: list[str] = []


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> str:
    """Compile every kernel for gfx950 and link ``_C.so``; returns its path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    troot, tinc, tlib, cxx11 = _torch_paths()
    hipcc = _hipcc()
    hdr = _newest_header()
    abi = f"-D_GLIBCXX_USE_CXX11_ABI={1 if cxx11 else 0}"
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _needs(obj, src, hdr):
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
                              abi, *FILE_FLAGS.get(os.path.basename(src), []), *EXTRA_HIPFLAGS, "-I", CSRC, "-c", src,
                              "-o", obj])
    bsrc = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD_DIR, "bindings.cpp.o")
    objs.append(bobj)
    if force or _needs(bobj, bsrc, hdr):
        py_inc = sysconfig.get_paths()["include"]
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", abi, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-DTORCH_EXTENSION_NAME={os.environ.get('KOP_EXT_NAME', '_C')}", "-DTORCH_API_INCLUDE_EXTENSION_H", "-w",
               "-I", CSRC, "-I", os.path.join(ROCM, "include"), "-I", py_inc]
        for i in tinc:
            cmd += ["-I", i]
        cmd += ["-c", bsrc, "-o", bobj]
        jobs_list.append(cmd)
    if jobs_list:
        n = jobs or min(len(jobs_list), int(os.environ.get("MAX_JOBS", "8")))
        with cf.ThreadPoolExecutor(max_workers=max(1, n)) as ex:
            for cmd, fut in [(c, ex.submit(_run, c)) for c in jobs_list]:
                if verbose:
                    print("[kop-build]", os.path.basename(cmd[-3] if cmd[-2] == "-o" else cmd[-1]), file=sys.stderr)
                fut.result()
    if force or jobs_list or not os.path.exists(SO_PATH) or any(os.path.getmtime(o) > os.path.getmtime(SO_PATH) for o in objs):
        tmp = SO_PATH + ".tmp"
        cmd = ["g++", "-shared", "-o", tmp, *objs, "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{tlib}"]
        _run(cmd)
        os.replace(tmp, SO_PATH)
    return SO_PATH


NATIVE_DIR = os.path.join(PKG_DIR, "native")


def build_native(force: bool = False) -> list[str]:
    """Host C++ runtime components (pybind11 modules, no GPU code): ``native/<name>.so``."""
    import pybind11

    out = []
    py_inc = sysconfig.get_paths()["include"]
    hdr = max((os.path.getmtime(h) for h in glob.glob(os.path.join(NATIVE_DIR, "*.h"))), default=0.0)
    for src in sorted(glob.glob(os.path.join(NATIVE_DIR, "*.cpp"))):
        so = os.path.splitext(src)[0] + ".so"
        out.append(so)
        if not force and os.path.exists(so) and os.path.getmtime(so) >= max(os.path.getmtime(src), hdr):
            continue
        tmp = so + ".tmp"
        _run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-fvisibility=hidden",
              "-I", pybind11.get_include(), "-I", py_inc, src, "-o", tmp])
        os.replace(tmp, so)
    return out


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
    print(build_native(force="--force" in sys.argv))
