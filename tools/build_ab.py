"""Build the gfx950 kernels of another git revision as a second extension module, ``kubeoperator_amd/_Cab.so``,
so one GPU session can A/B a kernel change against a baseline: run the probe / bench twice, once with
``KOP_EXT_MODULE=_Cab``. Usage: python tools/build_ab.py [REV]   (default HEAD: the committed kernels).

``--ablations``: build the WORKING TREE's kernels with -DKOP_ABLATIONS instead (the timing-ablation instantiations,
selected by KOP_DKDV64_DIAG / KOP_D64_DIAG, which give wrong results): a probe module only, never the shipped _C.so."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from kubeoperator_amd.ops import _build  # noqa: E402


def main():
    ablations = "--ablations" in sys.argv
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rev = args[0] if args else "HEAD"
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "csrc")
        os.makedirs(src)
        if ablations:
            import shutil

            rev = "working tree (-DKOP_ABLATIONS)"
            files = sorted(os.listdir(_build.CSRC))
            for f in files:
                shutil.copy(os.path.join(_build.CSRC, f), os.path.join(src, f))
        else:
            files = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", rev, "kubeoperator_amd/csrc/"],
                                   capture_output=True, text=True, check=True).stdout.split()
            for f in files:
                data = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{f}"], capture_output=True, check=True).stdout
                with open(os.path.join(src, os.path.basename(f)), "wb") as fh:
                    fh.write(data)
        with open(os.path.join(src, "bindings.cpp")) as fh:
            b = fh.read()
        with open(os.path.join(src, "bindings.cpp"), "w") as fh:
            fh.write(b.replace("PYBIND11_MODULE(_C, m)", "PYBIND11_MODULE(TORCH_EXTENSION_NAME, m)"))
        # reuse the build recipe with the module name, sources and output switched
        old = (_build.CSRC, _build.BUILD_DIR, _build.SO_PATH)
        _build.CSRC, _build.BUILD_DIR = src, os.path.join(d, "build")
        _build.SO_PATH = os.path.join(ROOT, "kubeoperator_amd", "_Cab.so")
        os.environ["KOP_EXT_NAME"] = "_Cab"
        if ablations:
            _build.EXTRA_HIPFLAGS[:] = ["-DKOP_ABLATIONS"]
        try:
            print(_build.build(verbose=True, force=True))
        finally:
            _build.CSRC, _build.BUILD_DIR, _build.SO_PATH = old
            _build.EXTRA_HIPFLAGS[:] = []
    print(f"built {rev} kernels as kubeoperator_amd._Cab ({len(files)} files)")


if __name__ == "__main__":
    main()
