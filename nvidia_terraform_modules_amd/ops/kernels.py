"""Python entry points for the gfx950 validation kernels (K1, K2, K3).

All functions launch on the current PyTorch stream and never synchronise, so
they can be captured in a ``torch.cuda.CUDAGraph`` (HIP graph on ROCm).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from ._lib import check, lib, lib_experimental, stream_handle

BM = BN = 256
BK = 64


def gemm_shape_ok(m: int, n: int, k: int) -> bool:
    """True iff the 256x256x64 MFMA kernel tiles (M, N, K) exactly."""
    return m > 0 and n > 0 and k >= 2 * BK and m % BM == 0 and n % BN == 0 and k % BK == 0


def _require(t: torch.Tensor, name: str, dtype: torch.dtype) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name} must be 2-D with unit inner stride")


GEMM_VARIANTS = {"default": 0, "pingpong8": 1, "pingpong8b": 4,
                 "pingpong8c": 5, "pingpong8cw": 10, "pingpong8cwe": 11,
                 "pingpong8cwn": 12, "pingpong8cwne": 13, "tile128": 15,
                 "tile256x128": 16, "tile160": 17, "tile256x160": 18, "tile128w4": 19,
                 "tile256x128w4": 20, "tile160w4": 21, "pingpong8cm": 22, "tile160x128": 23,
                 "tile128x160": 24, "tile128x256": 26, "pingpong8o": 25,
                 "pp8o_g128": 41, "pp8o_g128_nostore": 42, "pp8o_nostore": 43,
                 "pingpong8om": 47, "pingpong8od": 48, "pingpong8s": 49,
                 "pingpong8omd": 51, "pp192x256": 27, "pp256x192": 28,
                 "pp224x256": 29, "pp192x256s": 54, "pp256x192s": 55,
                 "dma4k_d3": 39}


# variants built only into libntm_experimental.so (tests / tools): never selected
# by the default dispatch, not present in the shipping library or Job binary
EXPERIMENTAL_VARIANTS = frozenset({"pingpong8", "pingpong8cw",
                                   "pingpong8cwe", "pingpong8cwn", "pingpong8cwne",
                                   "tile128w4", "tile256x128w4", "tile160w4",
                                   "pp8o_g128", "pp8o_g128_nostore", "pp8o_nostore",
                                   "pingpong8od", "pingpong8omd", "pingpong8om", "pp224x256"})

# (TM, TN) of the 4-wave tile kernels (gemm_bf16_t128.hpp)
TILE_SHAPES = {"tile128": (128, 128), "tile256x128": (256, 128), "tile160": (160, 160),
               "tile256x160": (256, 160), "tile128w4": (128, 128), "tile256x128w4": (256, 128),
               "tile160w4": (160, 160), "tile160x128": (160, 128), "tile128x160": (128, 160),
               "tile128x256": (128, 256)}


# wave-specialised tile kernels: any M, N % 4, K % 8 (edge tiles and the K tail masked)
MASKED_TILES = frozenset({"tile128", "tile256x128", "tile160", "tile160x128", "tile128x160",
                          "tile128x256"})


def _tile128_shape_ok(m: int, n: int, k: int, tm: int = 128, tn: int = 128,
                      masked: bool = False) -> bool:
    if masked:
        return m > 0 and n > 0 and n % 4 == 0 and k > 0 and k % 8 == 0
    return m > 0 and n > 0 and m % tm == 0 and n % tn == 0 and k >= 128 and k % 128 == 0


def k1_plan(m: int, n: int, k: int) -> tuple[int, str, str]:
    """The default dispatch's plan: (rows of C on the top kernel, top kernel,
    kernel of the remaining rows) - host-side, no GPU needed. The top kernel is
    the 256x256 one ("pingpong8c" / "pingpong8b") or a small tile; the rest is
    a small tile (ignored when the top takes every row). Raises ValueError
    when no combination of the K1 kernels tiles (M, N, K)."""
    top, tv, rest = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().ntm_k1_plan(m, n, k, ctypes.byref(top), ctypes.byref(tv), ctypes.byref(rest))
    if rc != 0:
        raise ValueError(f"shape ({m},{n},{k}) not tiled by the K1 kernels")
    names = {v: kname for kname, v in GEMM_VARIANTS.items()}
    return top.value, names[tv.value], names[rest.value]


def k1_splitk_plan(m: int, n: int, k: int) -> tuple[int, str, str, int]:
    """The default dispatch's plan with split-K allowed (what ``gemm_bf16``
    runs): ``k1_plan``'s triple plus the number of K slices (1 = unsplit; > 1 =
    all of C on the top kernel, a masked small tile, in that many K slices)."""
    top, tv, rest, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().ntm_k1_plan_splitk(m, n, k, ctypes.byref(top), ctypes.byref(tv),
                                  ctypes.byref(rest), ctypes.byref(sp))
    if rc != 0:
        raise ValueError(f"shape ({m},{n},{k}) not tiled by the K1 kernels")
    names = {v: kname for kname, v in GEMM_VARIANTS.items()}
    return top.value, names[tv.value], names[rest.value], sp.value


# (M, N, K) -> split-K workspace bytes of the default plan (0 = unsplit); a
# plan is validated once per shape
_DEFAULT_WS: dict[tuple[int, int, int], int] = {}


# (M, N, K) -> the stream-K variant of a stream-K default plan
_DEFAULT_SK: dict[tuple[int, int, int], str] = {}

# stream-K split mode on the 192-wide ping-pong tiles (gemm_bf16_skh.hpp)
SKH_VARIANTS = ("pp192x256s", "pp256x192s")
SK_VARIANTS = ("pingpong8s",) + SKH_VARIANTS


def k1_candidates(m: int, n: int, k: int, lda: int | None = None, ldb: int | None = None,
                  ldc: int | None = None) -> list[str]:
    """K1 builds worth timing on the box itself for an (m, n, k) GEMM: the default
    plan, plus the 4-wave ``dma4k_d3`` where its shape rule holds (M, N % 256,
    K % 128, K >= 256, rows 16-byte aligned, operands < 2 GiB). Under the power
    limit the two trade places box by box (profiles/r6_w4kh), so bench.py times
    both after its pre-warm and runs the faster (bench.select_k1)."""
    lda, ldb, ldc = lda or k, ldb or k, ldc or n
    ok = (m % 256 == 0 and n % 256 == 0 and k % 128 == 0 and k >= 256 and
          not (lda % 8 or ldb % 8 or ldc % 8) and m * lda * 2 < (1 << 31) and
          n * ldb * 2 < (1 << 31))
    return ["default", "dma4k_d3"] if ok else ["default"]


def set_plan_pp_tiles(on: bool = True, split: bool | None = None) -> None:
    """A/B knob for tools (tools/k1_ab.py pp-tiles): let the plan use the 192x256 /
    256x192 ping-pong tiles on all of C (``on``) and in stream-K split mode
    (``split``, default: as ``on``). The shipping plan has both. Process-wide."""
    split = on if split is None else split
    lib().ntm_set_plan_pp_tiles((1 if on else 0) | (2 if split else 0))
    _DEFAULT_WS.clear()
    _DEFAULT_SK.clear()
    _FP8_WS.clear()


def set_plan_splitk(margin: float = 0.0, long_slice_k: int = -1, fp8: bool = True) -> None:
    """A/B knob for tools (tools/k1_ab.py margin): the factor by which a split-K
    plan whose slices keep at least ``long_slice_k`` of K must beat the unsplit
    plan's predicted time (shorter slices, and any split against stream-K, keep
    1.1). margin <= 0 / long_slice_k < 0: the shipping 1.03 / 1024 (K1-fp8:
    1152 pairs of e4m3 values); margin 1.1 = round 4's plan. ``fp8`` False keeps
    K1-fp8's split-K at 1.1. Process-wide."""
    lib().ntm_set_plan_splitk(float(margin), int(long_slice_k), 1 if fp8 else 0)
    _DEFAULT_WS.clear()
    _DEFAULT_SK.clear()
    _FP8_WS.clear()


def set_plan_splitk_ragged(on: bool = True) -> None:
    """A/B knob for tools (tools/k1_ab.py margin): price long-slice split-K
    against the ragged-scaled unsplit time (the shipping plan, ``on``) or with
    round 4's rule. Process-wide; clears the per-shape plan memos here so no
    later default-dispatch call runs a stale decision."""
    lib().ntm_set_plan_splitk_ragged(1 if on else 0)
    _DEFAULT_WS.clear()
    _DEFAULT_SK.clear()
    _FP8_WS.clear()


def set_cus_override(cus: int = 0) -> None:
    """Host-only test knob: plan for ``cus`` CUs instead of the device's own (0 =
    the device's). Never set around real launches. Clears the plan memos."""
    lib().ntm_set_cus_override(int(cus))
    _DEFAULT_WS.clear()
    _DEFAULT_SK.clear()
    _FP8_WS.clear()


def skh_ws_bytes(variant: str, m: int, n: int, k: int) -> int:
    """Workspace of stream-K split mode on a 192-wide tile ("pp192x256s" /
    "pp256x192s") for (M, N, K) on this device; 0 when it does not serve it."""
    if m <= 0 or n <= 0 or k <= 0:
        return 0
    return int(lib().ntm_skh_ws_bytes(GEMM_VARIANTS[variant], m, n, k))


def _default_ws_bytes(m: int, n: int, k: int) -> int:
    """Split-K workspace bytes of the default plan; -1 when the plan is stream-K
    (its workspace is the per-stream cached one, ``_sk_workspace``)."""
    key = (m, n, k)
    wsb = _DEFAULT_WS.get(key)
    if wsb is None:
        _, top, _, sp = k1_splitk_plan(m, n, k)  # raises if no kernel serves the shape
        if top in SK_VARIANTS:
            # stream-K only where its own launch serves the shape (the plan and the
            # launch size for the same CUs; belt and braces): else the unsplit plan
            ok = (sk_ws_bytes(m, n, k) if top == "pingpong8s" else skh_ws_bytes(top, m, n, k)) > 0
            wsb = -1 if ok else 0
            if ok:
                _DEFAULT_SK[key] = top
        else:
            wsb = lib().ntm_splitk_ws_bytes(m, n, k, sp) if sp > 1 else 0
        _DEFAULT_WS[key] = wsb
    return wsb


def gemm_bf16(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
              variant: str = "default", splits: int = 1) -> torch.Tensor:
    """K1: ``out = a @ b.T`` in bf16 with fp32 accumulation on MFMA.

    a: [M, K] bf16, b: [N, K] bf16 (both K-contiguous), out: [M, N] bf16.
    ``variant``: "default" = the tile shape with the smallest predicted time
    (rounds of 256 CUs x tile area / efficiency, ``k1_plan``; split-K on a small
    tile when C cannot fill the chip and K is long, ``k1_splitk_plan``): "tile128" /
    "tile256x128" / "tile160" / "tile256x160" (128x128 / 256x128 / 160x160 /
    256x160 tiles, K % 128; the first three with 4 LDS-DMA producer + 4 MFMA
    consumer waves and masked edge tiles (any M, N % 4), 256x160 with 4 waves
    and whole tiles) for small, mid-size and ragged C,
    else "pingpong8c" when K % 128 == 0, else "pingpong8b" (8 waves, two per SIMD, staggered, balanced 8/4/8/4 LDS read
    schedule; 8c adds parity-alternating B buffers and a tail-free K loop),
    "pingpong8" (the first 12/4/8/0 schedule), "dma4k_d3" (4 waves x 128x128 per
    wave on 256x256 tiles, off the plan; bench.select_k1 times it against the plan
    on each box) - see validation/include.
    ``splits`` > 1 (masked tiles only): split-K into that many K slices, fp32
    partials in a workspace from PyTorch's allocator, then one reduction kernel.
    """
    _require(a, "a", torch.bfloat16)
    _require(b, "b", torch.bfloat16)
    m, k = a.shape
    n, kb = b.shape
    if k != kb:
        raise ValueError(f"K mismatch: a has {k}, b has {kb}")
    if variant in TILE_SHAPES:
        tm, tn = TILE_SHAPES[variant]
        if not _tile128_shape_ok(m, n, k, tm, tn, masked=variant in MASKED_TILES):
            raise ValueError(f"shape ({m},{n},{k}) not served by the {tm}x{tn} kernel "
                             "(masked tiles: N % 4, K % 8; others: whole tiles, K % 128)")
    elif variant == "default":
        _default_ws_bytes(m, n, k)  # the native plan is the one authority on what it serves
    elif variant in SKH_VARIANTS:
        if not skh_ws_bytes(variant, m, n, k):
            raise ValueError(f"shape ({m},{n},{k}) not served by {variant} (N % 8, K % 8, "
                             "K >= 128; at most half a round of its tiles, >= 2 K slices each)")
    elif variant in ("pingpong8s", "pingpong8s_rev", "pingpong8s_nopair"):  # stream-K
        if not sk_ws_bytes(m, n, k):
            raise ValueError(f"shape ({m},{n},{k}) not served by stream-K (N % 8, K % 8, K >= 128; "
                             "256x256 tiles: more than the CUs and not a multiple of them, or "
                             "few enough for >= 2 K slices per tile in one round)")
    elif variant in ("pingpong8cm", "pingpong8om", "pingpong8omd", "pp192x256", "pp256x192",
                     "pp224x256"):
        # 8-wave ping-pong tiles with masked edges (+ K tail)
        if not (m > 0 and n > 0 and n % 8 == 0 and k > 0 and k % 8 == 0):
            raise ValueError(f"shape ({m},{n},{k}) not served by {variant} (N % 8, K % 8)")
    elif not gemm_shape_ok(m, n, k):
        raise ValueError(f"shape ({m},{n},{k}) not tiled by the 256x256x64 kernel")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    _require(out, "out", torch.bfloat16)
    if tuple(out.shape) != (m, n):
        raise ValueError("out has the wrong shape")
    if variant in ("pingpong8s", "pingpong8s_rev", "pingpong8s_nopair"):
        return _gemm_bf16_sk(a, b, out, rev=variant == "pingpong8s_rev",
                             nopair=variant == "pingpong8s_nopair")
    if variant in SKH_VARIANTS:
        return _gemm_bf16_sk(a, b, out, sk_variant=variant)
    if splits > 1:
        if variant not in MASKED_TILES:
            raise ValueError(f"split-K runs on {sorted(MASKED_TILES)}, not {variant}")
        ws_bytes = lib().ntm_splitk_ws_bytes(m, n, k, splits)
        ws = torch.empty((ws_bytes + 3) // 4, dtype=torch.float32, device=a.device)
        rc = lib().ntm_gemm_bf16_splitk(
            GEMM_VARIANTS[variant], splits, a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
            a.stride(0), b.stride(0), out.stride(0), ws.data_ptr(), ws_bytes, stream_handle())
        check(rc, "ntm_gemm_bf16_splitk")
        return out
    if variant.startswith("knob"):            # experimental tuning sweep: "knob<N>"
        rc = lib_experimental().ntm_gemm_bf16_knob(
            int(variant[4:]), a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
            b.stride(0), out.stride(0), stream_handle())
        check(rc, "ntm_gemm_bf16_knob")
        return out
    if variant in EXPERIMENTAL_VARIANTS:
        rc = lib_experimental().ntm_gemm_bf16_experimental(
            GEMM_VARIANTS[variant], a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
            a.stride(0), b.stride(0), out.stride(0), stream_handle())
        check(rc, "ntm_gemm_bf16_experimental")
        return out
    if variant == "default" and _default_ws_bytes(m, n, k) < 0:
        return _gemm_bf16_sk(a, b, out, sk_variant=_DEFAULT_SK[(m, n, k)])
    if variant == "default" and _default_ws_bytes(m, n, k):
        wsb = _default_ws_bytes(m, n, k)
        ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=a.device)
        rc = lib().ntm_gemm_bf16_ex(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                                    a.stride(0), b.stride(0), out.stride(0), ws.data_ptr(), wsb,
                                    stream_handle())
        check(rc, "ntm_gemm_bf16_ex")
        return out
    rc = lib().ntm_gemm_bf16_variant(
        GEMM_VARIANTS[variant], a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
        a.stride(0), b.stride(0), out.stride(0), stream_handle())
    check(rc, "ntm_gemm_bf16")
    return out


def sk_ws_bytes(m: int, n: int, k: int) -> int:
    """Workspace of the stream-K build ("pingpong8s") for (M, N, K) on this
    device; 0 when it does not serve the shape. It serves two-round mode (more
    256x256 tiles than CUs, not a multiple of them) and split mode (each XCD's
    tiles fit its CUs at least twice: S >= 2 K slices per tile, one round)."""
    if m <= 0 or n <= 0 or k <= 0:
        return 0
    return int(lib().ntm_sk_ws_bytes(m, n, k))


# (device index, stream handle) -> the stream-K workspace of that stream: its
# counter block is zeroed once here and every completed launch leaves it zero,
# so calls on one stream reuse it with no memset dispatch
_SK_WS: dict[tuple[int, int], torch.Tensor] = {}


def _sk_workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    key = (dev.index if dev.index is not None else torch.cuda.current_device(),
           int(stream_handle() or 0))
    ws = _SK_WS.get(key)
    if ws is None or ws.numel() * 4 < nbytes:
        ws = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        _SK_WS[key] = ws
    return ws


def sk_xcc_error(device=None, clear: bool = True) -> int:
    """The XCD-placement error word of this stream's stream-K workspace
    (synchronises): 0 while every split tile's parts ran on one XCD, else the
    first violation a combiner saw (0x80000000 | mode << 28 | tile << 8 |
    combiner's XCC << 4 | other's XCC; gemm_bf16_sk.hpp). ``clear`` resets it."""
    dev = torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())
    key = (dev.index if dev.index is not None else torch.cuda.current_device(),
           int(stream_handle() or 0))
    ws = _SK_WS.get(key)
    if ws is None:
        return 0
    i = lib().ntm_sk_error_word_index()
    word = ws.view(torch.int32)[i:i + 1]
    v = int(word.item()) & 0xFFFFFFFF
    if clear and v:
        word.zero_()
    return v


class SkPlacementError(RuntimeError):
    """A stream-K launch saw parts of a split tile on different XCDs: the
    write-through / L1-only-acquire protocol's invariant broke, so C is not
    trusted (gemm_bf16_sk.hpp). Raised by the default dispatch under
    ``NTM_SK_CHECK=1`` (bench.py sets it; the validation Job checks the word
    itself)."""


def sk_check_enabled() -> bool:
    """``NTM_SK_CHECK=1``: every stream-K launch of ``gemm_bf16`` reads (and
    clears) this stream's placement error word afterwards and raises
    :class:`SkPlacementError` when it is set. Costs one host sync per stream-K
    launch, so it is opt-in; the plain 256x256 / small-tile paths are unaffected."""
    import os

    return os.environ.get("NTM_SK_CHECK", "0") not in ("", "0")


def set_sk_fault_inject(on: bool = True) -> None:
    """Fault injection for the placement check (tests): while on, the head /
    slice 0 of every split tile claims a wrong XCC, so every stream-K launch
    sets the error word. Process-wide."""
    lib().ntm_set_sk_fault_inject(1 if on else 0)


def _sk_checked(dev: torch.device, out: torch.Tensor) -> torch.Tensor:
    if sk_check_enabled():
        w = sk_xcc_error(dev, clear=True)
        if w:
            raise SkPlacementError(
                f"stream-K placement violation (error word 0x{w:08x}: tile {(w >> 8) & 0xFFFF}, "
                f"combiner XCC {(w >> 4) & 0xF}, other XCC {w & 0xF}); C is not trusted")
    return out


def _gemm_bf16_sk(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, rev: bool = False,
                  nopair: bool = False, sk_variant: str = "pingpong8s") -> torch.Tensor:
    """Stream-K (gemm_bf16_sk.hpp; sk_variant "pp192x256s" / "pp256x192s": split
    mode on the 192-wide tiles, gemm_bf16_skh.hpp): fp32 partials of the split
    tiles and one counter per split in this stream's cached workspace
    (_sk_workspace). rev / nopair: experimental builds (segments reversed; split
    mode's S-partial protocol also at S = 2)."""
    m, k = a.shape
    n = b.shape[0]
    if sk_variant in SKH_VARIANTS:
        wsb = skh_ws_bytes(sk_variant, m, n, k)
        ws = _sk_workspace(a.device, wsb)
        rc = lib().ntm_gemm_bf16_skh(GEMM_VARIANTS[sk_variant], a.data_ptr(), b.data_ptr(),
                                     out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
                                     out.stride(0), ws.data_ptr(), wsb, stream_handle())
        check(rc, "ntm_gemm_bf16_skh")
        return _sk_checked(a.device, out)
    wsb = sk_ws_bytes(m, n, k)
    ws = _sk_workspace(a.device, wsb)
    fn = (lib_experimental().ntm_gemm_bf16_sk_rev if rev else
          lib_experimental().ntm_gemm_bf16_sk_nopair if nopair else lib().ntm_gemm_bf16_sk)
    rc = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
            out.stride(0), ws.data_ptr(), wsb, stream_handle())
    check(rc, "ntm_gemm_bf16_sk")
    return _sk_checked(a.device, out)


def gemm_fp8_shape_ok(m: int, n: int, k: int) -> bool:
    return bool(lib().ntm_gemm_fp8_shape_ok(m, n, k))


# K1-fp8 variants: the 256x256 kernel and the wave-specialised tiles with the fp8 consumer
FP8_VARIANTS = ("default", "pingpong8c", "pingpong8o", "pingpong8cm", "tile128", "tile256x128",
                "tile160", "tile160x128", "tile128x160", "tile128x256")


def k1_fp8_plan(m: int, n: int, k: int) -> tuple[int, str, str]:
    """K1-fp8's default plan, as ``k1_plan`` (the same tile and row-split model
    with K counted in pairs of e4m3 values, over the tiles that have an fp8
    build). Raises ValueError for shapes the fp8 kernels do not serve."""
    top, tv, rest = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().ntm_k1_fp8_plan(m, n, k, ctypes.byref(top), ctypes.byref(tv), ctypes.byref(rest))
    if rc != 0:
        raise ValueError(f"shape ({m},{n},{k}) not served by the fp8 kernels (N % 8, K % 16)")
    names = {v: kname for kname, v in GEMM_VARIANTS.items()}
    return top.value, names[tv.value], names[rest.value]


def k1_fp8_splitk_plan(m: int, n: int, k: int) -> tuple[int, str, str, int]:
    """K1-fp8's plan with split-K allowed (what ``gemm_fp8`` runs): ``k1_fp8_plan``'s
    triple plus the number of K slices (> 1: all of C on a masked small tile)."""
    top, tv, rest, sp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().ntm_k1_fp8_plan_splitk(m, n, k, ctypes.byref(top), ctypes.byref(tv),
                                      ctypes.byref(rest), ctypes.byref(sp))
    if rc != 0:
        raise ValueError(f"shape ({m},{n},{k}) not served by the fp8 kernels (N % 8, K % 16)")
    names = {v: kname for kname, v in GEMM_VARIANTS.items()}
    return top.value, names[tv.value], names[rest.value], sp.value


_FP8_WS: dict[tuple[int, int, int], int] = {}


def _fp8_ws_bytes(m: int, n: int, k: int) -> int:
    key = (m, n, k)
    wsb = _FP8_WS.get(key)
    if wsb is None:
        sp = k1_fp8_splitk_plan(m, n, k)[3]
        wsb = lib().ntm_fp8_splitk_ws_bytes(m, n, k, sp) if sp > 1 else 0
        _FP8_WS[key] = wsb
    return wsb


def gemm_fp8(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
             knob: int = 0, variant: str = "default", splits: int = 1) -> torch.Tensor:
    """K1-fp8: ``out = a @ b.T`` with OCP e4m3 operands (``torch.float8_e4m3fn``),
    fp32 accumulation on the f8f6f4 MFMA (unit scales), bf16 output.

    a: [M, K], b: [N, K] (K-contiguous, rows 16-byte aligned), out: [M, N] bf16;
    N % 8, K % 16. ``variant``: "default" = ``k1_fp8_plan`` (256x256 tiles, or
    the wave-specialised 128x128 / 256x128 / 160x160 / 160x128 / 128x160 tiles
    and row splits where they fill the chip better); "pingpong8c" = the 256x256
    kernel (the bf16 default's schedule and LDS image, twice the MFMA rate per
    clock); "pingpong8o" = its persistent build with the C stores of one tile
    overlapping the next tile's K loop, on VGPR accumulators (whole 256x256
    tiles, K % 256, K >= 512; the plan's choice there); "tile*" = one tile shape. The default splits K over a masked small
    tile for skinny C with a long K (``k1_fp8_splitk_plan``; fp32 partials in a
    workspace from PyTorch's allocator); ``splits`` > 1 forces that on a "tile*"
    variant. ``knob`` != 0 selects an experimental schedule of the 256x256
    kernel (gemm_fp8_diag.hpp).
    """
    _require(a, "a", torch.float8_e4m3fn)
    _require(b, "b", torch.float8_e4m3fn)
    m, k = a.shape
    n, kb = b.shape
    if k != kb:
        raise ValueError(f"K mismatch: a has {k}, b has {kb}")
    if not gemm_fp8_shape_ok(m, n, k):
        raise ValueError(f"shape ({m},{n},{k}) not served by the fp8 kernel (N % 8, K % 16)")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    _require(out, "out", torch.bfloat16)
    if tuple(out.shape) != (m, n):
        raise ValueError("out has the wrong shape")
    if knob:
        rc = lib_experimental().ntm_gemm_fp8_knob(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                                     a.stride(0), b.stride(0), out.stride(0), int(knob),
                                     stream_handle())
    elif splits > 1 or (variant == "default" and _fp8_ws_bytes(m, n, k)):
        if splits > 1 and variant not in MASKED_TILES:
            raise ValueError(f"fp8 split-K runs on {sorted(MASKED_TILES)}, not {variant}")
        wsb = (lib().ntm_fp8_splitk_ws_bytes(m, n, k, splits) if splits > 1
               else _fp8_ws_bytes(m, n, k))
        ws = torch.empty((wsb + 3) // 4, dtype=torch.float32, device=a.device)
        if splits > 1:
            rc = lib().ntm_gemm_fp8_splitk(GEMM_VARIANTS[variant], splits, a.data_ptr(),
                                           b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0),
                                           b.stride(0), out.stride(0), ws.data_ptr(), wsb,
                                           stream_handle())
        else:
            rc = lib().ntm_gemm_fp8_ex(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                                       a.stride(0), b.stride(0), out.stride(0), ws.data_ptr(), wsb,
                                       stream_handle())
    else:
        if variant not in FP8_VARIANTS:
            raise ValueError(f"fp8 variant {variant!r} not in {FP8_VARIANTS}")
        rc = lib().ntm_gemm_fp8_variant(GEMM_VARIANTS[variant], a.data_ptr(), b.data_ptr(),
                                        out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
                                        out.stride(0), stream_handle())
    check(rc, "ntm_gemm_fp8")
    return out


def gemm_bf16_rowsum(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                     rowsum: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """K1 with the fused ABFT epilogue: returns ``(out, rowsum)`` where
    ``rowsum[m]`` is the fp32 sum over n of the accumulators of row m (the
    default kernel; ``rowsum`` is zeroed here, stream-ordered)."""
    _require(a, "a", torch.bfloat16)
    _require(b, "b", torch.bfloat16)
    m, k = a.shape
    n = b.shape[0]
    if b.shape[1] != k or not gemm_shape_ok(m, n, k):
        raise ValueError(f"shape ({m},{n},{k}) not tiled by the 256x256x64 kernel")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    _require(out, "out", torch.bfloat16)
    if rowsum is None:
        rowsum = torch.empty(m, dtype=torch.float32, device=a.device)
    if rowsum.dtype != torch.float32 or rowsum.numel() < m or not rowsum.is_contiguous():
        raise ValueError("rowsum must be a contiguous fp32 tensor of >= M entries")
    rowsum.zero_()
    rc = lib().ntm_gemm_bf16_rowsum(a.data_ptr(), b.data_ptr(), out.data_ptr(), rowsum.data_ptr(),
                                    m, n, k, a.stride(0), b.stride(0), out.stride(0),
                                    stream_handle())
    check(rc, "ntm_gemm_bf16_rowsum")
    return out, rowsum


def gemm_fp8_rowsum(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                    rowsum: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    """K1-fp8 with the fused ABFT epilogue (the 256x256 fp8 build, M, N, K %
    256): returns ``(out, rowsum)`` as ``gemm_bf16_rowsum`` does; check it with
    ``abft_check`` on the same e4m3 operands."""
    _require(a, "a", torch.float8_e4m3fn)
    _require(b, "b", torch.float8_e4m3fn)
    m, k = a.shape
    n = b.shape[0]
    if b.shape[1] != k or m % 256 or n % 256 or k % 256:
        raise ValueError(f"shape ({m},{n},{k}) not tiled by the 256x256 fp8 kernel (M, N, K % 256)")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    _require(out, "out", torch.bfloat16)
    if rowsum is None:
        rowsum = torch.empty(m, dtype=torch.float32, device=a.device)
    if rowsum.dtype != torch.float32 or rowsum.numel() < m or not rowsum.is_contiguous():
        raise ValueError("rowsum must be a contiguous fp32 tensor of >= M entries")
    rowsum.zero_()
    rc = lib().ntm_gemm_fp8_rowsum(a.data_ptr(), b.data_ptr(), out.data_ptr(), rowsum.data_ptr(),
                                   m, n, k, a.stride(0), b.stride(0), out.stride(0),
                                   stream_handle())
    check(rc, "ntm_gemm_fp8_rowsum")
    return out, rowsum


@dataclass
class AbftReport:
    rows: int
    bad_acc: int        # rows whose fused fp32 checksum disagrees with A . colsum(B)
    bad_store: int      # rows whose stored bf16 sum disagrees with the checksum
    max_rel_acc: float  # max |err| / ||C_m||_2
    max_rel_store: float

    @property
    def ok(self) -> bool:
        return self.bad_acc == 0 and self.bad_store == 0

    def as_dict(self) -> dict:
        return {"rows": self.rows, "bad_acc": self.bad_acc, "bad_store": self.bad_store,
                "max_rel_acc": self.max_rel_acc, "max_rel_store": self.max_rel_store,
                "ok": self.ok}


def abft_check(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor,
               rowsum: torch.Tensor) -> AbftReport:
    """K3: O(MK + NK + MN) ABFT check of ``c = a @ b.T`` against the fused
    row checksum (see aux_kernels.hpp); ``a`` / ``b`` bf16 (K1) or e4m3
    (K1-fp8). Synchronises to read the result."""
    m, k = a.shape
    n = b.shape[0]
    if c.shape != (m, n) or c.dtype != torch.bfloat16 or c.stride(1) != 1:
        raise ValueError("c must be [M, N] bf16 with unit inner stride")
    if a.dtype != b.dtype or a.dtype not in (torch.bfloat16, torch.float8_e4m3fn):
        raise ValueError("a and b must both be bf16 or both float8_e4m3fn")
    fn = lib().ntm_abft_check if a.dtype == torch.bfloat16 else lib().ntm_abft_check_fp8
    scratch = torch.empty(k, dtype=torch.float64, device=a.device)
    res = torch.empty(lib().ntm_abft_result_bytes(), dtype=torch.uint8, device=a.device)
    rc = fn(a.data_ptr(), b.data_ptr(), c.data_ptr(), rowsum.data_ptr(),
            m, n, k, a.stride(0), b.stride(0), c.stride(0),
            scratch.data_ptr(), res.data_ptr(), stream_handle())
    check(rc, "ntm_abft_check")
    raw = res.cpu().numpy().tobytes()
    return AbftReport(
        rows=m, bad_acc=int.from_bytes(raw[0:8], "little"),
        bad_store=int.from_bytes(raw[8:16], "little"),
        max_rel_acc=ctypes.c_float.from_buffer_copy(raw[16:20]).value,
        max_rel_store=ctypes.c_float.from_buffer_copy(raw[20:24]).value)


def fill_uniform_(t: torch.Tensor, seed: int, scale: float = 1.0) -> torch.Tensor:
    """K3: fill a bf16 (or OCP e4m3, ``torch.float8_e4m3fn``) tensor in place
    with ``scale * U[-1, 1)`` (hash RNG; e4m3 rounds to nearest even)."""
    if t.dtype not in (torch.bfloat16, torch.float8_e4m3fn) or not t.is_cuda or \
            not t.is_contiguous():
        raise ValueError("fill_uniform_ needs a contiguous bf16 or float8_e4m3fn GPU tensor")
    fn = lib().ntm_fill_uniform_bf16 if t.dtype == torch.bfloat16 else lib().ntm_fill_uniform_e4m3
    rc = fn(t.data_ptr(), t.numel(), seed & (2**64 - 1), float(scale), stream_handle())
    check(rc, "ntm_fill_uniform")
    return t


def ref_gemm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """K3: independent fp32-FMA reference ``a @ b.T`` (no MFMA, no hipBLASLt) for
    bf16 or OCP e4m3 operands (both of the same dtype)."""
    dt = a.dtype if a.dtype in (torch.bfloat16, torch.float8_e4m3fn) else torch.bfloat16
    _require(a, "a", dt)
    _require(b, "b", dt)
    m, k = a.shape
    n = b.shape[0]
    out = torch.empty((m, n), dtype=torch.float32, device=a.device)
    fn = lib().ntm_ref_gemm_f32 if dt == torch.bfloat16 else lib().ntm_ref_gemm_f32_e4m3
    rc = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
            out.stride(0), stream_handle())
    check(rc, "ntm_ref_gemm_f32")
    return out


@dataclass
class VerifyReport:
    n: int
    bad: int
    max_abs_err: float
    rel_rms_err: float

    @property
    def ok(self) -> bool:
        return self.bad == 0

    def as_dict(self) -> dict:
        return {"n": self.n, "bad": self.bad, "max_abs_err": self.max_abs_err,
                "rel_rms_err": self.rel_rms_err, "ok": self.ok}


def verify_bf16(c: torch.Tensor, ref: torch.Tensor, atol: float, rtol: float) -> VerifyReport:
    """K3: element-wise ``|c - ref| <= atol + rtol*|ref|`` on device (synchronises)."""
    if c.dtype != torch.bfloat16 or ref.dtype != torch.float32:
        raise ValueError("verify_bf16 expects bf16 c and fp32 ref")
    if c.shape != ref.shape or not c.is_contiguous() or not ref.is_contiguous():
        raise ValueError("c and ref must be contiguous and of equal shape")
    nbytes = lib().ntm_verify_result_bytes()
    res = torch.zeros(nbytes, dtype=torch.uint8, device=c.device)
    rc = lib().ntm_verify_bf16(c.data_ptr(), ref.data_ptr(), c.numel(), float(atol), float(rtol),
                               res.data_ptr(), stream_handle())
    check(rc, "ntm_verify_bf16")
    raw = res.cpu().numpy().tobytes()
    bad = int.from_bytes(raw[0:8], "little")
    max_err = ctypes.c_float.from_buffer_copy(raw[8:12]).value
    sse = ctypes.c_double.from_buffer_copy(raw[16:24]).value
    ssr = ctypes.c_double.from_buffer_copy(raw[24:32]).value
    rel = (sse / ssr) ** 0.5 if ssr > 0 else float("inf")
    return VerifyReport(n=c.numel(), bad=bad, max_abs_err=max_err, rel_rms_err=rel)


# (unroll, policy, grid) of the block-tiled K2 kernels; policy bit0 =
# nontemporal loads, bit1 = nontemporal stores, bit2 = software-pipelined
# copy, bit3 = chunked; grid 0 = one block per tile (no grid-stride loop);
# unroll 1 = the original grid-stride kernel. Chosen by tools/hbm_sweep.py on
# MI355X, interleaved rounds (profiles/r2_k2/): (2, 7, 0) - 2 float4 per lane,
# nontemporal load + store, one 8 KiB tile per block, so the dispatcher keeps
# every CU's wave slots full - 6.37 TB/s at 2 GiB and 6.05 at 4 GiB, against
# 5.81 / 5.41 for the earlier (8, 7, 512) grid-stride pipeline and 4.97 / 4.78
# for a plain grid-stride float4 copy on the same box. Grids <= 1024 blocks
# (at most 16 waves per CU) were all that the round-1 sweeps tried.
#   read  (8, 1, 1024) 7.08-7.13 TB/s at 1 GiB (grid-stride 6.11)
STREAM_COPY_CONFIG: tuple[int, int, int] = (2, 7, 0)
STREAM_READ_CONFIG: tuple[int, int, int] = (8, 1, 1024)


def stream_copy(src: torch.Tensor, dst: torch.Tensor,
                config: tuple[int, int, int] | None | str = "tuned") -> None:
    """K2: float4 HBM copy of ``src`` into ``dst`` (byte-identical)."""
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nbytes or nbytes % 16:
        raise ValueError("stream_copy needs 16-byte multiple sizes and a large enough dst")
    cfg = STREAM_COPY_CONFIG if config == "tuned" else (config or (1, 0, 0))
    rc = lib().ntm_stream_copy_ex(src.data_ptr(), dst.data_ptr(), nbytes, *cfg, stream_handle())
    check(rc, "ntm_stream_copy")


def stream_read(src: torch.Tensor, sink: torch.Tensor,
                config: tuple[int, int, int] | None | str = "tuned") -> None:
    """K2: read-only HBM sweep of ``src`` (``sink`` only written on NaN/inf)."""
    nbytes = src.numel() * src.element_size()
    if nbytes % 16:
        raise ValueError("stream_read needs a 16-byte multiple size")
    cfg = STREAM_READ_CONFIG if config == "tuned" else (config or (1, 0, 0))
    rc = lib().ntm_stream_read_ex(src.data_ptr(), nbytes, sink.data_ptr(), *cfg,
                                  stream_handle())
    check(rc, "ntm_stream_read")


def gemm_tolerance(k: int) -> tuple[float, float]:
    """(atol, rtol) for bf16-rounded output of an fp32-accumulated K-term dot product
    of U[-1,1) operands: bf16 output rounding (2^-8 relative) dominates; the fp32
    summation-order difference grows ~sqrt(K) * 2^-24 * |terms|."""
    atol = 1e-3 + 4.0 * (k ** 0.5) * 2.0 ** -20
    return atol, 2.0 ** -7


def clock_probe_ghz(device=None, iters: int = 20000, grid: int = 256) -> dict:
    """Shader clock this GPU holds under a dense bf16 MFMA load on random
    operands (``clock_probe_kernel``: Delta s_memtime / Delta s_memrealtime per
    wave, one 4-wave block per CU). Returns the median / min / max GHz over
    waves and the probe's wall time. Run it right after a timed loop: it reads
    the power / thermal state that loop left, which is what tells a
    power-limited GPU apart from a slow one in a multi-GPU run."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.zeros(grid * 4 * 2, dtype=torch.int64, device=dev)
    sink = torch.zeros(1, dtype=torch.float32, device=dev)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    check(lib().ntm_clock_probe(grid, iters, out.data_ptr(), sink.data_ptr(), stream_handle()),
          "ntm_clock_probe")
    t1.record()
    t1.synchronize()
    v = out.view(-1, 2).double()
    res = _ghz_summary(v[:, 0] / v[:, 1] * 0.1)
    res["probe_ms"] = round(t0.elapsed_time(t1), 3)
    res["waves"] = res.pop("n")
    return res


def _ghz_summary(ghz: torch.Tensor) -> dict:
    """median / p10 / min / max of per-wave (or per-workgroup) clocks; None
    fields when no finite sample is left (a caller in a collective must not
    raise on one rank)."""
    ghz = ghz[torch.isfinite(ghz) & (ghz > 0)]
    if ghz.numel() == 0:
        return {"median_GHz": None, "p10_GHz": None, "min_GHz": None, "max_GHz": None, "n": 0}
    q = torch.quantile(ghz, torch.tensor([0.1, 0.5], dtype=ghz.dtype, device=ghz.device))
    return {"median_GHz": round(float(q[1]), 4), "p10_GHz": round(float(q[0]), 4),
            "min_GHz": round(float(ghz.min()), 4), "max_GHz": round(float(ghz.max()), 4),
            "n": int(ghz.numel())}


def gemm_clock_ghz(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                   steps: int = 1, prequeue=None, prequeue_launches: int = 0) -> dict:
    """K1's OWN clock: ``steps`` back-to-back launches
    of the shipping pingpong8o build with a start / end s_memtime +
    s_memrealtime stamp per workgroup and the XCC_ID register of the XCD that
    ran it (gemm_bf16_pp6.hpp STAMP 1; C is the real product). Per workgroup
    and launch, clock = d(shader cycles) / d(100 MHz ticks).

    Returns median / p10 / min / max GHz over all workgroups, per-XCD medians
    keyed by the REAL XCC id, whether the dispatcher's ``blockIdx & 7`` round
    robin matched those ids, and ``bound_GHz``: per launch the slowest XCD's
    median clock (the tiles are split evenly over the XCDs, so the slowest
    one sets the launch time), median over launches. Needs whole 256x256
    tiles, K % 128, K >= 256. The MFMA-only ``clock_probe_ghz`` reads the clock
    of a different load (no LDS or HBM traffic): under shared power the two
    can differ by 15-20 %. ``prequeue`` (a launch callable) is called
    ``prequeue_launches`` times right before the stamped launches, with no host
    sync between, so they start in the steady state of a loaded GPU."""
    _require(a, "a", torch.bfloat16)
    _require(b, "b", torch.bfloat16)
    m, k = a.shape
    n = b.shape[0]
    grid = lib().ntm_gemm_bf16_clock_grid(m, n)
    if grid <= 0 or k % 128 or k < 256 or b.shape[1] != k:
        raise ValueError(f"shape ({m},{n},{k}) not served by the clock build (M, N % 256, K % 128, K >= 256)")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    _require(out, "out", torch.bfloat16)
    words = lib().ntm_gemm_bf16_clock_words()
    stamps = torch.zeros((steps, grid, words), dtype=torch.int64, device=a.device)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    for _ in range(prequeue_launches if prequeue is not None else 0):
        prequeue()
    t0.record()
    for i in range(steps):
        check(lib().ntm_gemm_bf16_clock(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                                        a.stride(0), b.stride(0), out.stride(0),
                                        stamps[i].data_ptr(), stream_handle()),
              "ntm_gemm_bf16_clock")
    t1.record()
    t1.synchronize()
    return clock_summary(stamps.cpu(), t0.elapsed_time(t1) / steps)


CLOCK_DRIFT_MAX = 0.03
CLOCK_MAX_BATCHES = 3


def gemm_clock_stable(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None,
                      steps: int = 20, prequeue=None, prequeue_launches: int = 40,
                      max_batches: int = CLOCK_MAX_BATCHES,
                      drift_max: float = CLOCK_DRIFT_MAX) -> dict:
    """``gemm_clock_ghz`` with a self-check: a batch whose
    per-launch stamp windows (``per_launch_window_us_median``) drift by more
    than ``drift_max`` (max / min - 1) caught a clock transient and is stamped
    again - each batch queued behind ``prequeue_launches`` plain launches with
    no host sync - up to ``max_batches``. Returns the first stable batch (else
    the least drifted) with ``clock_batches``, ``clock_batch_drift_pct`` (per
    batch) and ``clock_stable``."""
    best, drifts = None, []
    for _ in range(max(1, max_batches)):
        r = gemm_clock_ghz(a, b, out, steps=steps, prequeue=prequeue,
                           prequeue_launches=prequeue_launches)
        w = [x for x in r["per_launch_window_us_median"] if x > 0]
        d = (max(w) / min(w) - 1.0) if w else float("inf")
        drifts.append(round(100 * d, 2) if d != float("inf") else None)
        if best is None or d < best[0]:
            best = (d, r)
        if d <= drift_max:
            break
    r = best[1]
    r["clock_batches"] = len(drifts)
    r["clock_batch_drift_pct"] = drifts
    r["clock_stable"] = best[0] <= drift_max
    return r


def clock_summary(stamps: torch.Tensor, ms_per_launch: float) -> dict:
    """Summary of a [launches, workgroups, words] record of the clock build
    (host-side; see ``gemm_clock_ghz``)."""
    steps, grid = stamps.shape[0], stamps.shape[1]
    sv = stamps.double()
    ghz = (sv[:, :, 2] - sv[:, :, 0]) / (sv[:, :, 3] - sv[:, :, 1]) * 0.1   # [steps, grid]
    res = _ghz_summary(ghz.reshape(-1))
    res["workgroups"] = res.pop("n")
    # the XCD that really ran each workgroup (XCC_ID register) ...
    xcc = (stamps[:, :, 4] & 0xF).long()
    ids = sorted(set(xcc.reshape(-1).tolist()))
    res["xcc_ids"] = ids
    res["per_xcc_median_GHz"] = {str(x): _ghz_summary(ghz[xcc == x])["median_GHz"] for x in ids}
    # ... against the dispatcher's round robin, blockIdx & 7 (what stream-K's
    # per-XCD tile lists and its write-through / L1-only-acquire protocol assume)
    resid = torch.arange(grid) & 7
    seen = {r: sorted(set(xcc[:, resid == r].reshape(-1).tolist())) for r in range(min(8, grid))}
    one_each = all(len(v) == 1 for v in seen.values())
    res["xcc_of_blockidx_mod_8"] = {str(r): v for r, v in seen.items()}
    res["blockidx_mod_8_is_xcc"] = bool(one_each and len({v[0] for v in seen.values()}) == len(seen))
    # kept for continuity with earlier rounds' JSON: groups by b & 7
    res["per_xcd_group_median_GHz"] = [_ghz_summary(ghz[:, r::8].reshape(-1))["median_GHz"]
                                       for r in range(min(8, grid))]
    res["ms_per_launch"] = round(ms_per_launch, 4)
    res["launches"] = steps
    # per launch: medians over workgroups of the shader cycles and of the wall
    # window (us) between a workgroup's two stamps - to set against a profiler's
    # per-dispatch duration and cycle counters (tools/clock_check.py)
    cyc = (sv[:, :, 2] - sv[:, :, 0]).median(dim=1).values
    win = ((sv[:, :, 3] - sv[:, :, 1]) / 100.0).median(dim=1).values
    # the median workgroup's cycles over the median workgroup's window, median
    # over launches (2.0 / 2.7 % below GRBM_GUI_ACTIVE / 8 XCDs / duration on the
    # same dispatches, profiles/r4_clock/)
    lg = cyc / (win * 1e3)
    lg = lg[torch.isfinite(lg) & (lg > 0)]
    res["launch_GHz"] = round(float(lg.median()), 4) if lg.numel() else None
    # the launch-bounding clock: every XCD gets the same number of tiles, so the
    # slowest XCD's workgroups finish last and set the launch time
    bound, spread = [], []
    for i in range(steps):
        per = [float(ghz[i][xcc[i] == x].median()) for x in ids if bool((xcc[i] == x).any())]
        per = [v for v in per if v == v and v > 0]
        if per:
            bound.append(min(per))
            spread.append(max(per) / min(per) - 1.0)
    res["bound_GHz"] = round(sorted(bound)[len(bound) // 2], 4) if bound else None
    res["xcc_clock_spread_pct"] = round(100 * sorted(spread)[len(spread) // 2], 2) if spread else None
    # when each XCD's last workgroup ended, after the launch's first start (us,
    # median over launches): the gap between the first and the last XCD to finish
    # is how long the faster XCDs idle at the end of every launch
    rt0 = sv[:, :, 1].min(dim=1).values                      # [steps]
    fin = {x: [] for x in ids}
    for i in range(steps):
        for x in ids:
            sel = xcc[i] == x
            if bool(sel.any()):
                fin[x].append(float((sv[i, :, 3][sel].max() - rt0[i]) / 100.0))
    res["per_xcc_finish_us"] = {str(x): round(sorted(v)[len(v) // 2], 2) for x, v in fin.items() if v}
    idle = []
    for i in range(steps):
        ends = [float((sv[i, :, 3][xcc[i] == x].max() - rt0[i]) / 100.0)
                for x in ids if bool((xcc[i] == x).any())]
        if ends:
            idle.append(max(ends) - min(ends))
    res["xcc_finish_spread_us"] = round(sorted(idle)[len(idle) // 2], 2) if idle else None
    res["per_launch_cycles_median"] = [int(x) for x in cyc.tolist()]
    res["per_launch_window_us_median"] = [round(x, 2) for x in win.tolist()]
    return res
