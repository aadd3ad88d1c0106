"""Host sanitizers on the native C++ runtime: the token prefetcher core is compiled into a
standalone harness with AddressSanitizer + UBSan, and again with ThreadSanitizer, and run (CPU only)."""
import shutil
import subprocess

import pytest

from kubeoperator_amd.ops._build import NATIVE_DIR

SRC = f"{NATIVE_DIR}/prefetch_check.cc"


@pytest.mark.parametrize("flags", [["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                                   ["-fsanitize=thread"]], ids=["asan_ubsan", "tsan"])
def test_prefetcher_under_sanitizers(tmp_path, flags):
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    exe = tmp_path / "prefetch_check"
    cc = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-pthread", *flags, "-I", NATIVE_DIR, SRC, "-o", str(exe)],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    run = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=300,
                         env={"ASAN_OPTIONS": "detect_leaks=1", "TSAN_OPTIONS": "halt_on_error=1"})
    assert run.returncode == 0, run.stdout + run.stderr
    assert "prefetch_check: OK" in run.stdout
