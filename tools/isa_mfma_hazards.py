"""Scan a gfx950 assembly listing (hipcc --save-temps ``*.s``) for one hazard hipcc does not guard inline-asm MFMAs
against: a VALU instruction writing an MFMA's A / B source VGPRs fewer than 2 wait states before it (gfx950 requires 2;
``cdna_hip_programming.md`` §5.7 item 2). hipcc pads its own builtin MFMAs; inline-asm ones (the dK / dV kernel's AGPR
chains) carry their own ``s_nop`` -- or, where the source says the operands cannot have been just written, none, and
this scan is what checks that claim on the built code.

Usage: python tools/isa_mfma_hazards.py file.s [kernel-name-substring]   (exit status 1 if a hazard is found)
"""
from __future__ import annotations

import re
import sys

_REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")


def _regs(tok: str) -> set[tuple[str, int]]:
    out = set()
    for m in _REG.finditer(tok):
        if m.group(2) is not None:
            out.add((m.group(1), int(m.group(2))))
        else:
            out |= {(m.group(1), i) for i in range(int(m.group(3)), int(m.group(4)) + 1)}
    return out


def _ops(line: str) -> tuple[str, list[str]]:
    parts = line.split(None, 1)
    op = parts[0]
    args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
    return op, args


def scan(lines: list[str]) -> list[str]:
    """Hazards in one function body (instruction lines only)."""
    bad = []
    hist: list[tuple[int, set]] = []  # (wait states the instruction occupies, VGPRs a VALU wrote)
    for ln in lines:
        op, args = _ops(ln)
        if op.startswith("v_mfma"):
            srcs = _regs(args[1]) | _regs(args[2]) if len(args) >= 3 else set()
            ws = 0
            for n, wrote in reversed(hist):
                if ws >= 2:
                    break
                if wrote & srcs:
                    bad.append(ln)
                    break
                ws += n
        if op == "s_nop":
            hist.append((int(args[0], 0) + 1 if args else 1, set()))
        elif op.startswith("v_") and not op.startswith("v_mfma") and args:
            hist.append((1, {r for r in _regs(args[0]) if r[0] == "v"}))
        else:
            hist.append((1, set()))
        hist = hist[-8:]
    return bad


def main(path: str, name: str = "") -> int:
    text = open(path).read().split("\n")
    total = 0
    fn, body = None, []
    for raw in text + ["_end:"]:
        if re.match(r"^[_A-Za-z][\w.$]*:", raw) and not raw.startswith(".L"):
            if fn and name in fn and body:
                bad = scan(body)
                if bad:
                    print(f"{fn[:90]}: {len(bad)} MFMA(s) within 2 wait states of a VALU write of their sources")
                    for b in bad[:5]:
                        print("   ", b)
                total += len(bad)
            fn, body = raw.split(":")[0], []
            continue
        s = raw.strip()
        if s and not s.startswith((";", ".", "//")) and not s.endswith(":"):
            body.append(s.split(";")[0].strip())
    print(f"hazards: {total}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""))
