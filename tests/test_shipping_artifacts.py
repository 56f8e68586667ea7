"""What ships: the validation-Job binary and libntm_validation.so carry ONLY
the kernels the default K1 dispatch (and K1-fp8 / K2 / K3 / C2) can launch.
The experimental K1 builds, schedule knobs and diagnostics (r4, r4d,
pp3 knobs and stamps, the first ping-pong, fp8 knobs, MFMA probes) live in
libntm_experimental.so only (VERDICT r1 "Next round" #8). Host-only check of
the kernel symbols with nm - no GPU needed."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "validation" / "build" / "amdgpu-validate"
LIB = ROOT / "nvidia_terraform_modules_amd" / "ops" / "libntm_validation.so"
EXP = ROOT / "nvidia_terraform_modules_amd" / "ops" / "libntm_experimental.so"

# K1 kernel instantiations the default dispatch may launch: pingpong8c (LDS-staged
# epilogue when ldc % 8 == 0, register epilogue otherwise; with/without the ABFT
# row sum; F8 = 3 is K1-fp8; EPI 26 = the masked ragged-C build), pingpong8b for
# K % 128 != 0, and the 4 tile shapes
# (128x128 / 256x128 / 160x160 / 160x128 / 128x160 wave-specialised, also as K1-fp8,
# 256x160 4-wave).
ALLOWED_K1 = {
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 0, 0, 0>",
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 10, 0, 0>",
    "ntm::gemm3::gemm_bf16_pp3_kernel<true, 8, false, 0, 0, 0>",
    "ntm::gemm3::gemm_bf16_pp3_kernel<true, 8, false, 10, 0, 0>",
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 10, 0, 3>",
    "ntm::gemm3::gemm_bf16_pp3_kernel<true, 8, false, 10, 0, 3>",   # K1-fp8 + ABFT row sum
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 26, 0, 0>",  # masked edge tiles
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 26, 0, 3>",  # K1-fp8, masked
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 58, 0, 0>",  # masked + partial K
    "ntm::gemm3::gemm_bf16_pp3_kernel<false, 8, false, 58, 0, 3>",  # K1-fp8, masked + partial K
    # pingpong8o <POL, STAMP, MASK, TAIL, SPREAD, F8>: > 256 tiles of 256x256
    # (the shipping bf16 build spreads its boundary stores: SPREAD, "pingpong8od")
    "ntm::gemm6::gemm_bf16_pp6_kernel<1, 0, false, false, true, false, false>",
    "ntm::gemm6::gemm_bf16_pp6_kernel<1, 1, false, false, true, false, false>",  # clock stamps
    "ntm::gemm6::gemm_bf16_pp6_kernel<1, 0, false, false, true, true, false>",   # K1-fp8
    # stream-K over the last two rounds of 256x256 tiles (pingpong8s <TAIL, REV, STAMP>)
    "ntm::gemmsk::gemm_bf16_sk_kernel<false, false, false>",
    "ntm::gemmsk::gemm_bf16_sk_kernel<true, false, false>",
    # its split mode (at most half a round of tiles) <TAIL>
    "ntm::gemmsk::gemm_bf16_sks_kernel<false, false>",
    "ntm::gemmsk::gemm_bf16_sks_kernel<true, false>",
    # ... at S = 2: the head / tail protocol <TAIL, PAIR> (round 5)
    "ntm::gemmsk::gemm_bf16_sks_kernel<false, true>",
    "ntm::gemmsk::gemm_bf16_sks_kernel<true, true>",
    # one round of 192x256 / 256x192 ping-pong tiles <AH, BH, TAIL> (round 5)
    "ntm::gemm3h::gemm_bf16_pp3h_kernel<64, 128, false>",
    "ntm::gemm3h::gemm_bf16_pp3h_kernel<64, 128, true>",
    "ntm::gemm3h::gemm_bf16_pp3h_kernel<128, 64, false>",
    "ntm::gemm3h::gemm_bf16_pp3h_kernel<128, 64, true>",
    # ... in stream-K split mode <AH, BH, TAIL, PAIR> (round 5)
    "ntm::gemmskh::gemm_bf16_sksh_kernel<64, 128, false, false>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<64, 128, false, true>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<64, 128, true, false>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<64, 128, true, true>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<128, 64, false, false>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<128, 64, false, true>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<128, 64, true, false>",
    "ntm::gemmskh::gemm_bf16_sksh_kernel<128, 64, true, true>",
    "ntm::gemm2::gemm_bf16_pp2_kernel<false, 0>",
    "ntm::gemm2::gemm_bf16_pp2_kernel<false, 3>",
    "ntm::gemm2::gemm_bf16_pp2_kernel<true, 0>",
    "ntm::gemm2::gemm_bf16_pp2_kernel<true, 3>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 4, 0, false, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<8, 4, 0, false, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 5, 0, false, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 4, 0, false, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 5, 0, false, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 8, 0, false, false>",
    # split-K builds of the same tiles (fp32 partials; splitk_reduce_kernel sums them)
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 4, 0, true, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<8, 4, 0, true, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 5, 0, true, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 4, 0, true, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 5, 0, true, false>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 8, 0, true, false>",
    # K1-fp8 on the same tiles (fp8 consumer)
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 4, 0, false, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<8, 4, 0, false, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 5, 0, false, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 4, 0, false, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 5, 0, false, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 8, 0, false, true>",
    # ... and their split-K builds
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 4, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<8, 4, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 5, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<5, 4, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 5, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_ws_kernel<4, 8, 0, true, true>",
    "ntm::gemmt::gemm_bf16_tile_kernel<8, 5>",
}
# The 4-wave bf16 build (dma4k_d3, gemm_w4k_kernel<3, false>) ships since round 6:
# bench.select_k1 times it against the plan on each box (profiles/r6_w4kh). Its
# fp8 build (knob 12) stays experimental.
SHIPPED_4WAVE = "ntm::w4k::gemm_w4k_kernel<3, false>"
EXPERIMENTAL_ONLY = ("gemm_w4k_kernel<2, true>", "gemm_w4o_kernel", "gemm_r4k_stamp_kernel",
                     "gemm_bf16_pp3_stamp_kernel", "ntm::gemm::gemm_bf16_kernel",
                     "mfma_rate_kernel", "mfma_f8_probe_kernel", "gemm_bf16_pp3h_kernel<96")


def _kernels(path: Path) -> set:
    if not path.exists():
        pytest.skip(f"{path.name} not built (python -m nvidia_terraform_modules_amd.ops.build)")
    nm = shutil.which("nm") or "/opt/rocm/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-C", str(path)], capture_output=True, text=True, check=True).stdout
    names = set()
    for ln in out.splitlines():
        parts = ln.split(None, 2)
        if len(parts) == 3 and parts[1] in "VDTW" and "__device_stub__" not in parts[2]:
            m = re.match(r"(?:void )?(ntm::[\w:]+_kernel(?:<[^>]*>)?)\(", parts[2])
            if m:
                names.add(m.group(1))
    return names


@pytest.mark.parametrize("path", [BIN, LIB], ids=["job-binary", "libntm_validation"])
def test_shipping_artifact_has_only_default_dispatch_k1(path):
    ks = _kernels(path)
    k1 = {k for k in ks if "gemm_bf16" in k}
    assert k1 == ALLOWED_K1, (sorted(k1 - ALLOWED_K1), sorted(ALLOWED_K1 - k1))
    for bad in EXPERIMENTAL_ONLY:
        assert not [k for k in ks if bad in k], bad
    assert {k for k in ks if "gemm_w4k_kernel" in k} == {SHIPPED_4WAVE}


def test_experimental_library_holds_the_experiments():
    ks = _kernels(EXP)
    for fam in ("gemm_bf16_pp3_stamp_kernel", "gemm_bf16_sk_kernel<false, true, false>", "mfma_rate_kernel",
                "mfma_f8_probe_kernel",
                "gemm_bf16_pp6_kernel<1, 0, true, false, false, false, false>",   # pingpong8om
                "gemm_bf16_pp3h_kernel<96, 128"):                          # pp224x256
        assert any(fam in k for k in ks), fam
