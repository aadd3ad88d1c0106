"""Resource check of every compiled gfx950 kernel (CPU; reads the in-tree code objects): no VGPR / SGPR spills and no
scratch. A spill turns a register-resident MFMA loop into scratch traffic (5x slower, cdna_hip_programming.md
rule 20) without changing any numerics test's outcome, so it is caught here at build time -- e.g. merging the
one-wave dK/dV kernel's masked / unmasked stage loops into one loop made hipcc spill ~500 VGPRs."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "kubeoperator_amd", "_build")
LLVM = "/opt/rocm/lib/llvm/bin"


# known and accepted: (name fragment, max VGPR spills) with the reason
ALLOWED = {
    # the recompute-dQ kernel of the long-context path (dS above its 16 GiB cap): 3 VGPRs / 16 B of scratch outside
    # the key loop; that path is measured as a whole (profiles/r3_llama3_8b_32k_recompute_dkdv64_ab.jsonl)
    "fa_bwd_dq8_kernelILi128ELb1E": 4,
}


def _kernels(obj, tmp):
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(name|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|vgpr_count):\s+(\S+)",
                     line)
        if m:
            key, val = m.groups()
            if key == "name" and ("name" in cur):
                out.append(cur)
                cur = {}
            cur[key] = val if key == "name" else int(val)
    if cur:
        out.append(cur)
    return [k for k in out if "name" in k and "kop" in k["name"]]


@pytest.mark.skipif(not os.path.isdir(BUILD) or not os.path.exists(f"{LLVM}/llvm-readelf"),
                    reason="extension not built / no LLVM tools")
def test_no_kernel_spills_or_uses_scratch(tmp_path):
    objs = sorted(glob.glob(os.path.join(BUILD, "*.hip.o")))
    srcs = {os.path.basename(s) for s in glob.glob(os.path.join(ROOT, "kubeoperator_amd", "csrc", "*.hip"))}
    objs = [o for o in objs if os.path.basename(o)[:-2] in srcs]  # skip stale objects of removed sources
    assert objs
    bad, n = [], 0
    for o in objs:
        for k in _kernels(o, str(tmp_path)):
            n += 1
            allow = next((v for frag, v in ALLOWED.items() if frag in k["name"]), 0)
            if (k.get("vgpr_spill_count", 0) > allow or k.get("sgpr_spill_count", 0)
                    or (k.get("private_segment_fixed_size", 0) and not allow)):
                bad.append((os.path.basename(o), k["name"][:90], k.get("vgpr_spill_count"),
                            k.get("private_segment_fixed_size")))
    assert n > 20
    assert not bad, bad
