"""The inline-asm MFMA hazard scan (tools/mfma_hazard_scan.py): the detector
on hand-made listings, and the shipping library's gfx950 ISA scanned clean
(hipcc cross-compiles here; no GPU)."""
from __future__ import annotations

import importlib.util
import shutil
import tempfile
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
_spec = importlib.util.spec_from_file_location("mfma_hazard_scan", ROOT / "tools/mfma_hazard_scan.py")
scan = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(scan)

MFMA = "v_mfma_f32_16x16x32_bf16 a[196:199], v[40:43], v[8:11], a[196:199]"


def test_detects_agpr_write_right_before_asm_mfma():
    # the first overlap build: a zero f32x4 copied into the AGPRs 2-5 instructions before
    body = ["v_accvgpr_write_b32 a196, v212", "v_accvgpr_write_b32 a197, v213",
            "v_accvgpr_write_b32 a198, v214", "v_accvgpr_write_b32 a199, v215",
            "s_nop 0", MFMA]
    assert scan.scan_kernel(body) == (4, 0)


def test_detects_unpadded_read_after_mfma_and_accepts_a_drain():
    assert scan.scan_kernel([MFMA, "v_accvgpr_read_b32 v0, a196"]) == (0, 1)
    assert scan.scan_kernel([MFMA, "s_nop 15", "s_nop 15", "v_accvgpr_read_b32 v0, a196"]) == (0, 0)


def test_stops_at_an_unconditional_branch():
    body = [MFMA, "s_branch .LBB0_9", ".LBB0_8:", "v_accvgpr_write_b32 a196, 0"]
    assert scan.scan_kernel(body) == (0, 0)
    body = ["v_accvgpr_write_b32 a196, 0", "s_branch .LBB0_3", ".LBB0_2:", MFMA]
    assert scan.scan_kernel(body) == (0, 0)


def test_kernel_split():
    asm = "\n".join(["_Zfoo:", MFMA, "s_endpgm", "_Zbar:", "s_endpgm"])
    ks = scan.kernels(asm)
    assert set(ks) == {"_Zfoo", "_Zbar"} and MFMA in ks["_Zfoo"]


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
def test_shipping_library_isa_is_clean():
    with tempfile.TemporaryDirectory() as d:
        asm = scan.compile_asm(ROOT / "validation/src/ntm_validation.hip", Path(d))
    ks = {n: b for n, b in scan.kernels(asm).items() if any("v_mfma" in ln for ln in b)}
    assert len(ks) >= 10
    dirty = {n: scan.scan_kernel(b) for n, b in ks.items()
             if not scan.EXEMPT.search(n) and scan.scan_kernel(b) != (0, 0)}
    assert not dirty, dirty


VMFMA = "v_mfma_f32_16x16x128_f8f6f4 v[200:203], v[40:47], v[8:15], v[200:203]"


def test_vgpr_accumulator_asm_mfma_hazards():
    """Inline-asm MFMAs with VGPR accumulators (the fp8 persistent build): a
    VALU write of srcC right before, an unpadded VALU read of the result right
    after; only MFMAs inside ;;#ASMSTART / ;;#ASMEND count (hipcc pads its own)."""
    asm = [";;#ASMSTART", VMFMA, ";;#ASMEND"]
    assert scan.scan_kernel(["v_mov_b32_e32 v201, 0", "s_nop 0"] + asm) == (1, 0)
    assert scan.scan_kernel(asm + ["v_cvt_pk_bf16_f32 v10, v200, v201"]) == (0, 1)
    assert scan.scan_kernel(asm + ["s_nop 15", "s_nop 7", "v_cvt_pk_bf16_f32 v10, v200, v201"]) \
        == (0, 0)
    # the next MFMA accumulating into the same registers needs no padding
    assert scan.scan_kernel(asm + asm) == (0, 0)
    # a compiler-emitted (builtin) MFMA of the same form is not scanned
    assert scan.scan_kernel(["v_mov_b32_e32 v201, 0", VMFMA]) == (0, 0)


def test_windows_count_wait_states():
    """Windows are wait states, not lines: an s_nop N pad (N + 1 states) between
    a write of srcC and the asm MFMA clears it - the form the spread fp8 build
    uses after its barrier - while the same writes with only 3 instructions
    between are reported."""
    asm = [";;#ASMSTART", VMFMA, ";;#ASMEND"]
    near = ["v_mov_b32_e32 v201, v178", ".LBB0_18:", "s_barrier", "s_waitcnt lgkmcnt(0)"]
    assert scan.scan_kernel(near + asm) == (1, 0)
    padded = ["v_mov_b32_e32 v201, v178", ".LBB0_18:", "s_barrier", "s_nop 15",
              "s_waitcnt lgkmcnt(0)"]
    assert scan.scan_kernel(padded + asm) == (0, 0)
    # AGPR accumulators the same way
    assert scan.scan_kernel(["v_accvgpr_write_b32 a196, v212", "s_nop 15", MFMA]) == (0, 0)
