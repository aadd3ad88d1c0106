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
# SGPR spills go to VGPR lanes (v_writelane / v_readlane, no scratch): the hand-scheduled forward's 64-slot body keeps
# ~110 scalar values (DMA piece addresses, LDS slot bases) live and reloads 8 of them per tile
ALLOWED_SGPR = {"fa_fwd4x64_kernel": 64}


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
            allow_s = next((v for frag, v in ALLOWED_SGPR.items() if frag in k["name"]), 0)
            if (k.get("vgpr_spill_count", 0) > allow or k.get("sgpr_spill_count", 0) > allow_s
                    or (k.get("private_segment_fixed_size", 0) and not allow)):
                bad.append((os.path.basename(o), k["name"][:90], k.get("vgpr_spill_count"),
                            k.get("private_segment_fixed_size")))
    assert n > 20
    assert not bad, bad


def _compiler_agprs(asm_text, fn):
    """AGPR numbers that hipcc itself (outside inline-asm blocks) touches in function ``fn``."""
    i = asm_text.index("\n" + fn + ":")
    j = asm_text.index(".Lfunc_end", i)
    regs, inasm = set(), False
    for line in asm_text[i:j].splitlines():
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            inasm = True
        elif t.startswith(";;#ASMEND"):
            inasm = False
        elif t and not inasm and not t.startswith(";"):
            for m in re.finditer(r"\ba(\d+)\b|\ba\[(\d+):(\d+)\]", t.split(";")[0]):
                if m.group(1):
                    regs.add(int(m.group(1)))
                else:
                    regs.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return regs


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_asm_owned_agprs_stay_out_of_hipccs_hands(tmp_path):
    """flash_fwd4.hip keeps O^T / Q^T in a[64:255] by literal register names that hipcc cannot see; hipcc parks
    VGPRs in AGPRs from a0 upward under pressure. Build the file with -save-temps and require that hipcc's own AGPR
    use stays below a64, that no MFMA reads a VALU result within 2 wait states (tools/isa_mfma_hazards.py), and that
    nothing spills to scratch."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_mfma_hazards

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    src = os.path.join(ROOT, "kubeoperator_amd", "csrc", "flash_fwd4.hip")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-amdgpu-mfma-vgpr-form=true",
                    "-save-temps", "--cuda-device-only", "-c", src, "-I", os.path.dirname(src), "-o",
                    str(tmp_path / "f4.o")], check=True, cwd=tmp_path, capture_output=True)
    s_file = next(p for p in glob.glob(str(tmp_path / "*.s")) if "gfx950" in p)
    text = open(s_file).read()
    fns = re.findall(r"^(_Z\w*fa_fwd4x64\w*):", text, re.M)
    assert fns
    for fn in fns:
        regs = _compiler_agprs(text, fn)
        assert not regs or max(regs) < 64, (fn, sorted(regs)[-5:])
        body = text[text.index("\n" + fn + ":"):text.index(".Lfunc_end", text.index("\n" + fn + ":"))]
        lines = [ln.strip().split(";")[0].strip() for ln in body.splitlines()]
        lines = [ln for ln in lines if ln and not ln.startswith((".", "//")) and not ln.endswith(":")]
        assert not isa_mfma_hazards.scan(lines), fn
        assert "scratch_" not in body, fn
