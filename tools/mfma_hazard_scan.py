"""Scan the gfx950 ISA of the K1 libraries for the inline-asm MFMA hazard.

hipcc pads the VALU-write -> MFMA-srcC hazard (and MFMA-dst -> VALU-read) only
for MFMAs it emits itself. The K1 kernels issue their MFMAs as inline asm with
AGPR accumulators, so a compiler-generated ``v_accvgpr_write`` / ``v_accvgpr_mov``
of an accumulator placed just before an asm MFMA that reads it as srcC is
unpadded, and the MFMA reads stale elements (profiles/r3_w4o/README.md: the
first overlap build parked a zero f32x4 in VGPRs and copied it into the AGPRs
2-6 instructions before each MFMA).

For every kernel with an MFMA this reports the number of
  * AGPR writes within WINDOW instructions before an MFMA that reads that AGPR
    as srcC, and
  * VALU accesses of an MFMA's destination AGPRs fewer than MFMA_TO_VALU_WS
    wait states after it (the other direction; s_nop N counts N + 1, an MFMA
    4);
and, for inline-asm MFMAs with VGPR accumulators (the fp8 persistent build,
gemm_bf16_pp6.hpp mfma_f8_vgpr; only asm ones - hipcc pads its own), the same
two counts over VGPRs: non-MFMA writes of a srcC VGPR within WINDOW
instructions before, any non-MFMA access of a dst VGPR within MFMA_TO_VALU_WS
wait states after.
Windows are counted in wait states (an s_nop N is N + 1, any other
instruction 1), so a deliberate pad in front of an asm MFMA clears it.
The scan is linear over the listing and stops at an unconditional branch
(the next block is then reached from elsewhere). Exit status 1 if a GEMM kernel (not the rate probes, whose values are unused)
has a hit.

    python tools/mfma_hazard_scan.py [--src validation/src/ntm_validation.hip ...]
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DEFAULT_SRCS = ["validation/src/ntm_validation.hip", "validation/src/ntm_experimental.hip"]
# rate / clock probes: MFMAs on don't-care values, measured for issue rate only
EXEMPT = re.compile(r"clock_probe|mfma_rate")
WINDOW = 12
# MFMA result -> VALU access of it: the 16-pass f8f6f4 MFMA's requirement
# (passes + 3), the longest of the K1 MFMAs
MFMA_TO_VALU_WS = 19

_MFMA = re.compile(r"v_mfma\S* a\[(\d+):(\d+)\], v\[\d+:\d+\], v\[\d+:\d+\], a\[(\d+):(\d+)\]")
_MFMA_V = re.compile(r"v_mfma\S* v\[(\d+):(\d+)\], v\[\d+:\d+\], v\[\d+:\d+\], v\[(\d+):(\d+)\]")
_VREF = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_AWRITE = re.compile(r"v_accvgpr_(?:write|mov)_b32 a(\d+)")
_AREAD = re.compile(r"v_accvgpr_read_b32 \S+, a(\d+)")
_NOFALL = re.compile(r"^\s*(s_branch|s_endpgm|s_setpc_b64)\b")


def _regs(lo: str, hi: str) -> set[int]:
    return set(range(int(lo), int(hi) + 1))


def _vregs(text: str) -> list[set[int]]:
    """Register sets of every VGPR operand in an instruction, in order."""
    out = []
    for m in _VREF.finditer(text):
        out.append(_regs(m.group(1), m.group(2)) if m.group(1) else {int(m.group(3))})
    return out


def _strip(lines: list[str]) -> tuple[list[str], list[bool]]:
    """Instruction lines and whether each sits between ;;#ASMSTART / ;;#ASMEND."""
    out, in_asm, inside = [], [], False
    for ln in lines:
        t = ln.strip()
        if t.startswith(";;#ASMSTART"):
            inside = True
        elif t.startswith(";;#ASMEND"):
            inside = False
        if t and not t.startswith(";"):
            out.append(ln)
            in_asm.append(inside)
    return out, in_asm


def scan_kernel_vgpr(lines: list[str]) -> tuple[int, int]:
    """The two hazard counts for inline-asm MFMAs with VGPR accumulators."""
    lines, in_asm = _strip(lines)
    before = after = 0
    for i, ln in enumerate(lines):
        m = _MFMA_V.search(ln)
        if not m or not in_asm[i]:
            continue
        dst, src = _regs(m.group(1), m.group(2)), _regs(m.group(3), m.group(4))
        ws = 0  # wait states strictly between line j and the MFMA (s_nop N = N + 1)
        for j in range(i - 1, -1, -1):
            if _NOFALL.search(lines[j]) or ws >= WINDOW:
                break
            nop = re.search(r"s_nop (\d+)", lines[j])
            if "v_mfma" not in lines[j]:
                ops = _vregs(lines[j].split(";")[0])
                op = lines[j].split()[0] if lines[j].split() else ""
                if op.startswith("v_") and ops and ops[0] & src:
                    before += 1
            ws += int(nop.group(1)) + 1 if nop else 1
        ws = 0
        for j in range(i + 1, len(lines)):
            nop = re.search(r"s_nop (\d+)", lines[j])
            ws += int(nop.group(1)) + 1 if nop else 1
            if "v_mfma" in lines[j]:
                ws += 3
                continue  # the next MFMA taking the result whole as srcC: no wait
            if ws >= MFMA_TO_VALU_WS:
                break
            if any(r & dst for r in _vregs(lines[j].split(";")[0])):
                after += 1
            if _NOFALL.search(lines[j]):
                break
    return before, after


def scan_kernel(lines: list[str]) -> tuple[int, int]:
    vb, va = scan_kernel_vgpr(lines)
    lines = [ln for ln in lines if ln.strip() and not ln.strip().startswith(";")]
    before, after = vb, va
    for i, ln in enumerate(lines):
        m = _MFMA.search(ln)
        if not m:
            continue
        dst, src = _regs(m.group(1), m.group(2)), _regs(m.group(3), m.group(4))
        ws = 0
        for j in range(i - 1, -1, -1):
            if _NOFALL.search(lines[j]) or ws >= WINDOW:
                break  # above: not this MFMA's fall-through predecessor, or far enough
            w = _AWRITE.search(lines[j])
            if w and int(w.group(1)) in src:
                before += 1
            nop = re.search(r"s_nop (\d+)", lines[j])
            ws += int(nop.group(1)) + 1 if nop else 1
        ws = 0  # wait states since the MFMA issued (s_nop N = N + 1)
        for j in range(i + 1, len(lines)):
            nop = re.search(r"s_nop (\d+)", lines[j])
            ws += int(nop.group(1)) + 1 if nop else 1
            if "v_mfma" in lines[j]:
                ws += 3  # an MFMA issue holds vector issue for >= 4 cycles
            if ws >= MFMA_TO_VALU_WS:
                break
            r = _AREAD.search(lines[j]) or _AWRITE.search(lines[j])
            if r and int(r.group(1)) in dst:
                after += 1
            if _NOFALL.search(lines[j]):
                break  # what follows is another path
    return before, after


def kernels(asm: str) -> dict[str, list[str]]:
    out: dict[str, list[str]] = {}
    name = None
    for ln in asm.split("\n"):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            name = m.group(1)
            out[name] = []
            continue
        if name is not None:
            out[name].append(ln)
            if "s_endpgm" in ln:
                name = None
    return out


def compile_asm(src: Path, tmp: Path) -> str:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{ROOT / 'validation/include'}", "--offload-device-only", "-save-temps",
                    "-c", "-x", "hip", str(src), "-o", str(tmp / (src.stem + ".o"))],
                   cwd=tmp, check=True, capture_output=True)
    return next(tmp.glob(f"{src.stem}-hip-amdgcn-amd-amdhsa-gfx950.s")).read_text()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", nargs="*", default=DEFAULT_SRCS)
    args = ap.parse_args()
    bad = 0
    with tempfile.TemporaryDirectory() as d:
        for s in args.src:
            asm = compile_asm(ROOT / s, Path(d))
            for name, body in kernels(asm).items():
                if not any("v_mfma" in ln for ln in body):
                    continue
                before, after = scan_kernel(body)
                exempt = bool(EXEMPT.search(name))
                if before or after:
                    print(f"{s} {name}: agpr-write->mfma {before}, mfma->valu {after}"
                          f"{' (exempt probe)' if exempt else ''}")
                    bad += 0 if exempt else 1
                else:
                    print(f"{s} {name}: clean")
    print("hazard scan:", "FAIL" if bad else "clean")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
