"""Host-side K1 dispatch plan (``ntm_k1_plan``, validation/src/ntm_validation.hip):
which rows of C go on the 256x256 kernel and which small tile takes the rest.
No GPU needed - the plan is pure host code in the native library."""
import pytest

from nvidia_terraform_modules_amd.ops import kernels


@pytest.fixture(scope="module")
def k1_plan():
    from nvidia_terraform_modules_amd.ops import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("native library not built (python -m nvidia_terraform_modules_amd.ops.build)")
    from nvidia_terraform_modules_amd.ops.kernels import k1_plan as f

    return f


@pytest.mark.parametrize("m,n,k,top,top_variant,rest", [
    (1024, 1024, 1024, 1024, "tile128", None),       # < 1 round of 256x256 tiles: small tile only
    (2048, 2048, 2048, 2048, "tile128", None),
    (2560, 2560, 2560, 2560, "tile160", None),       # 256 tiles of 160x160: one full round
    (1920, 1920, 1920, 1920, "tile128", None),
    (256, 160, 128, 256, "tile128", None),           # 4 masked 128x128 tiles beat one 256x160
    (2816, 2816, 2816, 2816, "tile128x256", None),   # 242 tiles: one round (128x256 2 % above 256x128)
    (4096, 2048, 4096, 4096, "tile128x256", None),
    (4672, 1472, 6696, 4672, "tile128x256", None),   # hipBLASLt's MT128x256 there (r2_tiles)
    (3072, 3072, 3072, 3072, "pp192x256", None),     # 144 256x256 tiles -> 192 of 192x256 (+18 %)
    (3072, 3072, 512, 3072, "pingpong8c", None),     # K < 1024: the 192-wide tiles stay out
    (4096, 4096, 4096, 4096, "pingpong8c", None),
    (8192, 8192, 8192, 8192, "pingpong8o", None),    # > 256 tiles: the persistent build
    (4096, 8192, 8192, 4096, "pingpong8o", None),    # 512 tiles
    (5120, 5120, 256, 5120, "pingpong8o", None),     # 400 tiles, K = 256: the shortest tile
    (5120, 5120, 128, 5120, "pingpong8c", None),     # K = 128: below the persistent build's K
    (8192, 8192, 8128, 8192, "pingpong8cm", None),   # K % 128 != 0: partial-K build
    (6144, 6144, 6144, 5376, "pingpong8o", "tile160x128"),  # 3 rounds -> 2 + one of 160x128
    (4352, 4352, 4352, 3840, "pingpong8c", "tile128"),
    (3200, 3200, 3200, 3200, "pp192x256", None),     # one round of 192x256 tiles (+8 %)
    (3200, 3200, 616, 3200, "pingpong8cm", None),    # one round of masked 256x256 tiles
    (2080, 3844, 256, 512, "tile128", "tile160"),    # N % 8 != 0: mixed small tiles
    (4000, 4000, 4096, 4000, "pingpong8cm", None),
    (416, 1280, 128, 416, "tile128", None),          # masked edge tiles: one launch
    (1696, 2560, 2560, 1696, "tile160x128", None),   # 11 x 20 tiles: one round
    (5624, 752, 5880, 5624, "tile160x128", None),    # 216 tiles vs 180 of 160x160
    (4072, 1240, 3784, 4072, "tile128x160", None),   # 32 x 8 tiles: one full round
    (3000, 3000, 3000, 3000, "pp192x256", None),     # 16 x 12 tiles (+13 %)
    (3000, 3000, 4096, 3000, "pp192x256", None),
    (3904, 2584, 12760, 3904, "pp256x192", None),    # hipBLASLt's MT256x192 there (r5_h192)
    (5120, 5120, 256, 5120, "pingpong8o", None),     # never the rest part of a 2-launch plan
    (2400, 3200, 3200, 2400, "tile128x256", None),   # 19 x 13 tiles: one round
    (3200, 5104, 3480, 3200, "tile128x256", None),   # 2 full rounds beat 256x256 + a tile128 rest (+2.4 %)
    (8200, 8192, 8192, 8192, "pingpong8o", "tile128"),  # 8 ragged rows on masked tiles
])
def test_plan_matches_cost_model(k1_plan, m, n, k, top, top_variant, rest):
    got = k1_plan(m, n, k)
    assert got[:2] == (top, top_variant)
    if rest is not None:
        assert got[2] == rest


@pytest.mark.parametrize("m,n,k", [(256 * i, 256 * j, 512) for i in range(1, 33, 3)
                                   for j in range(1, 33, 5)])
def test_plan_is_well_formed(k1_plan, m, n, k):
    top, top_variant, rest = k1_plan(m, n, k)
    small = ("tile128", "tile256x128", "tile160", "tile256x160", "tile160x128", "tile128x160",
             "tile128x256")
    pp = ("pp192x256", "pp256x192")   # one-round, all of C only
    assert 0 < top <= m and top_variant in small + pp + ("pingpong8c", "pingpong8cm", "pingpong8o")
    if top_variant in pp:
        assert top == m and k >= 1024
    if top_variant == "pingpong8o":  # more 256x256 tiles than CUs, else pingpong8c
        assert (top // 256) * (n // 256) > 256 and k >= 256
    assert rest in small
    tm = {"tile128": 128, "tile256x128": 256, "tile160": 160, "tile256x160": 256,
          "tile160x128": 160, "tile128x160": 128, "tile128x256": 128, "pingpong8c": 256,
          "pingpong8cm": 256, "pp192x256": 192, "pp256x192": 256,
          "pingpong8o": 256}
    masked = ("tile128", "tile256x128", "tile160", "tile160x128", "tile128x160", "tile128x256",
              "pingpong8cm", "pp192x256", "pp256x192")
    assert top % tm[top_variant] == 0 or (top == m and top_variant in masked)
    if top < m:
        assert (m - top) % tm[rest] == 0 or rest in masked


@pytest.mark.parametrize("m,n,k", [(1000, 1000, 1024), (100, 4096, 4096), (8200, 8192, 8192),
                                   (3000, 5000, 2048), (1, 4, 128), (384, 256, 192),
                                   (1000, 1000, 1000), (64, 64, 8)])
def test_plan_serves_ragged_shapes(k1_plan, m, n, k):
    """Masked edge tiles and K tails: any M, N % 4 == 0 and K % 8 == 0 has a plan."""
    top, top_variant, _ = k1_plan(m, n, k)
    assert 0 < top <= m


def test_plan_rejects_bad_args(k1_plan):
    with pytest.raises(Exception):
        k1_plan(0, 256, 256)


@pytest.mark.parametrize("m,n,k", [(384, 256, 100), (100, 256, 12), (256, 256, 4),
                                   (256, 6, 128)])
def test_plan_reports_infeasible_shapes(k1_plan, m, n, k):
    """No kernel serves these (K % 8 or N % 4): the plan says so instead of
    returning a plan whose second launch would fail after the first one wrote C
    ((384,256,192) used to launch 256 rows, then fail - it is now
    served whole by the masked 128x128 tiles)."""
    with pytest.raises(ValueError):
        k1_plan(m, n, k)


@pytest.fixture(scope="module")
def splitk_plan(k1_plan):
    from nvidia_terraform_modules_amd.ops.kernels import k1_splitk_plan as f

    return f


@pytest.mark.parametrize("m,n,k,variant,splits", [
    (280, 6352, 7568, "tile160", 3),       # 80 tiles of 160x160 -> 240 in one round
    (256, 8192, 8192, "tile128", 2),       # 128 tiles -> 256
    (512, 4096, 16384, "tile256x128", 4),  # 64 tiles -> 256
    (1024, 1024, 16384, "tile128", 4),
    (128, 8192, 8192, "tile128", 4),
    (792, 3416, 6104, "tile160", 2),
])
def test_splitk_plan_for_skinny_long_k(splitk_plan, m, n, k, variant, splits):
    """C too small to fill 256 CUs with a long K: split-K on a masked small tile."""
    assert splitk_plan(m, n, k) == (m, variant, variant, splits)


@pytest.mark.parametrize("m,n,k", [(8192, 8192, 8192), (4096, 4096, 4096), (1000, 3112, 768),
                                   (3200, 3200, 3200), (6144, 6144, 6144), (2080, 3844, 256),
                                   (2048, 2048, 4096), (8008, 536, 2896)])
def test_splitk_plan_keeps_unsplit_plan(k1_plan, splitk_plan, m, n, k):
    """Chip-filling C or short K: split-K is not worth its fp32 partials, and the
    plan is exactly the unsplit one."""
    assert splitk_plan(m, n, k) == k1_plan(m, n, k) + (1,)


@pytest.mark.parametrize("m,n,k", [(5624, 752, 5880), (4672, 1472, 6696), (1456, 2696, 10744),
                                   (1872, 2224, 5208)])
def test_splitk_plan_takes_stream_k_on_ragged_one_round_c(k1_plan, splitk_plan, m, n, k):
    """One round of a small tile on ragged C runs 1.1-1.5x its modelled time;
    stream-K's split mode measured 9-39 % faster there (profiles/r4_sks/), on the
    256x256 or (round 5) the 192-wide tiles."""
    assert k1_plan(m, n, k)[1].startswith("tile")
    top, tv, rest, sp = splitk_plan(m, n, k)
    assert (top, sp) == (m, 1) and tv == rest and tv in ("pingpong8s", "pp192x256s", "pp256x192s")


@pytest.mark.parametrize("m,n,k,variant", [
    (4152, 1096, 16056, "pp256x192s"),   # 85 256x256 tiles = 22 of 32 CUs per XCD busy
    (2840, 1768, 8904, "pp192x256s"),
    (4800, 1168, 15776, "pp192x256s"),
    (3072, 2048, 6144, "pp192x256s"),    # was tile128x256: +6.7 % (profiles/r5_skh/)
    (4672, 1472, 6696, "pingpong8s"),    # 256x256 split mode stays where it is faster
])
def test_splitk_plan_split_mode_on_192_tiles(splitk_plan, m, n, k, variant):
    """Split mode on the 192-wide ping-pong tiles (gemm_bf16_skh.hpp): more CUs
    busy for 0.75 of the work each; off with the A/B knob's split bit."""
    from nvidia_terraform_modules_amd import ops

    assert splitk_plan(m, n, k) == (m, variant, variant, 1)
    try:
        ops.set_plan_pp_tiles(True, split=False)
        assert splitk_plan(m, n, k)[1] not in ("pp192x256s", "pp256x192s")
    finally:
        ops.set_plan_pp_tiles(True)


@pytest.mark.parametrize("m,n,k", [(m, n, k) for m in (64, 333, 1000, 2048)
                                   for n in (256, 1004, 4096) for k in (1024, 4104, 16384)])
def test_splitk_plan_is_well_formed(k1_plan, splitk_plan, m, n, k):
    top, tv, rest, splits = splitk_plan(m, n, k)
    assert 1 <= splits <= 16
    if tv == "pingpong8s":   # stream-K (split mode here): all of C on the 256x256 kernel
        assert top == m and rest == tv and splits == 1
    elif splits > 1:   # all of C on one masked small tile; K slices of >= 64
        assert top == m and tv == rest
        assert tv in ("tile128", "tile256x128", "tile160", "tile160x128", "tile128x160")
        assert k // splits >= 32
    else:
        assert (top, tv, rest) == k1_plan(m, n, k)


@pytest.fixture(scope="module")
def fp8_plan():
    from nvidia_terraform_modules_amd.ops import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("native library not built (python -m nvidia_terraform_modules_amd.ops.build)")
    from nvidia_terraform_modules_amd.ops.kernels import k1_fp8_plan as f

    return f


@pytest.mark.parametrize("m,n,k,plan", [
    # whole 256x256 tiles (fp8 K % 256, K >= 512) run the persistent build
    (8192, 8192, 8192, (8192, "pingpong8o", "tile128")),   # the Job's fp8 check: 256x256 only
    (4096, 4096, 4096, (4096, "pingpong8o", "tile128")),
    (6144, 6144, 6144, (5376, "pingpong8o", "tile160x128")),
    (4096, 4096, 256, (4096, "pingpong8c", "tile128")),    # K below the persistent build's 512
    (2048, 2048, 2048, (2048, "tile128", "tile128")),
    (2560, 2560, 2560, (2560, "tile160", "tile160")),
    (1000, 1000, 1008, (1000, "tile128", "tile128")),
])
def test_fp8_plan(fp8_plan, k1_plan, m, n, k, plan):
    """K1-fp8's plan is the bf16 model at K / 2 (a K-tile of 128 e4m3 values
    costs what one of 64 bf16 values does) over the tiles with an fp8 build."""
    assert fp8_plan(m, n, k) == plan


@pytest.mark.parametrize("m,n,k", [(256, 160, 256), (512, 640, 256), (5120, 5120, 8192),
                                   (8192, 5120, 8192), (1280, 2560, 1024)])
def test_fp8_plan_uses_only_fp8_builds(fp8_plan, m, n, k):
    """No 4-wave 256x160 tile (no fp8 build) and no split-K in an fp8 plan."""
    top, tv, rv = fp8_plan(m, n, k)
    assert 0 < top <= m
    assert tv in ("pingpong8c", "pingpong8o", "pingpong8cm", "tile128", "tile256x128", "tile160",
                  "tile160x128", "tile128x160")
    assert rv != "tile256x160" and tv != "tile256x160"


def test_fp8_plan_rejects_bad_shapes(fp8_plan):
    for m, n, k in [(256, 252, 256), (256, 256, 24), (0, 256, 256)]:
        with pytest.raises(ValueError):
            fp8_plan(m, n, k)


def test_fp8_entry_points_reject_bad_shapes_before_any_launch(fp8_plan):
    """The fp8 C ABI validates the shape on the host (no GPU touched): N % 8,
    K % 16, known variants only; split-K needs a masked tile and a big-enough
    workspace."""
    from nvidia_terraform_modules_amd.ops._lib import lib

    L = lib()
    for m, n, k in [(256, 252, 256), (256, 256, 24), (0, 256, 256)]:
        assert L.ntm_gemm_fp8_variant(0, None, None, None, m, n, k, k, k, n, None) != 0
        assert L.ntm_gemm_fp8(None, None, None, m, n, k, k, k, n, None) != 0
    assert L.ntm_gemm_fp8_variant(18, None, None, None, 256, 256, 256, 256, 256, 256, None) != 0
    assert L.ntm_gemm_fp8_splitk(5, 2, None, None, None, 256, 256, 256, 256, 256, 256, None, 0,
                                 None) != 0
    assert L.ntm_fp8_splitk_ws_bytes(280, 6352, 15136, 3) == 4 * 3 * 280 * 6352


def test_k1_boxes_reports_median_over_boxes(tmp_path):
    """tools/k1_boxes.py: per-box K1 / hipBLASLt ratios and their median (a +-1 %
    claim is a distribution over boxes)."""
    import json
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import k1_boxes

    logs = []
    for i, (ours, hb) in enumerate([(1600, 1620), (1650, 1630), (1640, 1640)]):
        p = tmp_path / f"box{i}.log"
        p.write_text('{"device": "x"}\n' + json.dumps(
            {"size": 8192, "pingpong8o_tflops_med": ours, "torch_tflops_med": hb}) + "\n")
        logs.append(str(p))
    r = k1_boxes.ratios(logs)
    rs = r[("8192", "pingpong8o")]
    assert len(rs) == 3 and abs(sorted(rs)[1] - 1.0) < 1e-12


@pytest.mark.parametrize("m,n,k", [(8008, 536, 2896), (4152, 1096, 16056), (1456, 2696, 10744)])
def test_plan_tie_prefers_fewer_tiles(k1_plan, m, n, k):
    """160x128 and 128x160 have the same modelled one-round cost; the one whose
    tiles span less of C won on every measured shape where the counts differ
    (profiles/r4_tiles: 8008x536x2896 34.8 vs 39.4 us)."""
    assert k1_plan(m, n, k) == (m, "tile128x160", "tile128x160")


@pytest.mark.parametrize("m,n,k,served", [
    (4472, 5688, 5832, True),    # 414 tiles: two-round mode (1.6 rounds)
    (4672, 1472, 6696, True),    # 114 tiles: split mode, 2 K slices
    (1000, 1000, 1000, True),    # 16 tiles: split mode, 8 slices of one pair
    (256, 256, 256, True),       # 1 tile: 2 slices of one pair
    (4096, 4096, 4096, False),   # 256 tiles: exactly one round, nothing to balance
    (8192, 8192, 8192, False),   # 1024 tiles: a multiple of the CUs
    (7472, 1280, 6024, False),   # 150 tiles: under 2 slices per tile fit one round
    (256, 256, 128, False),      # one K pair: cannot split
    (4096, 4100, 4096, False),   # N % 8 != 0
])
def test_stream_k_decomposition_serves(k1_plan, m, n, k, served):
    """sk_decompose (gemm_bf16_sk.hpp), seen through the host-side workspace
    query: which shapes stream-K's two-round and split modes serve."""
    from nvidia_terraform_modules_amd import ops

    assert (ops.sk_ws_bytes(m, n, k) > 0) == served


@pytest.mark.parametrize("cus", [256, 128, 80, 32])
def test_plan_and_launch_agree_on_the_cu_count(k1_plan, cus):
    """the plan's stream-K choice is made for the CU count the launch
    sizes its grid for (device_cus: 256 on MI355X in SPX mode, fewer in a DPX /
    CPX partition), so the default dispatch never picks a stream-K plan whose
    launch would refuse the shape. Forced CU counts, host only."""
    import random

    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.ops import kernels
    from nvidia_terraform_modules_amd.ops._lib import lib

    rng = random.Random(cus)
    shapes = [(4472, 5688, 5832), (4672, 1472, 6696), (1000, 1000, 1000), (8192, 8192, 8192)]
    shapes += [(rng.randrange(256, 9000), rng.randrange(32, 1200) * 8, rng.randrange(16, 1500) * 8)
               for _ in range(60)]
    kernels.set_cus_override(cus)
    kernels._DEFAULT_WS.clear()
    try:
        assert lib().ntm_plan_cus() == cus
        picked = 0
        for m, n, k in shapes:
            _, top, _, _ = ops.k1_splitk_plan(m, n, k)
            if top == "pingpong8s":
                picked += 1
                assert ops.sk_ws_bytes(m, n, k) > 0, (m, n, k)
                assert kernels._default_ws_bytes(m, n, k) == -1
        if cus % 8 == 0 and cus >= 32:
            assert picked > 0
    finally:
        kernels.set_cus_override(0)
        kernels._DEFAULT_WS.clear()
    assert lib().ntm_plan_cus() == 256      # no GPU here: the documented default



def test_pp_tiles_one_launch_and_toggle(k1_plan):
    """The 192x256 / 256x192 ping-pong tiles (gemm_bf16_pp3h.hpp) take all of C in
    one round or nothing, need N % 8 and K >= 1024, never serve fp8, and the
    tools' A/B knob turns them off and on."""
    from nvidia_terraform_modules_amd import ops

    try:
        assert k1_plan(3904, 2584, 12760)[1] == "pp256x192"
        assert k1_plan(3904, 2588, 12760)[1] != "pp256x192"      # N % 8
        ops.set_plan_pp_tiles(False)
        assert k1_plan(3904, 2584, 12760)[1] == "pingpong8cm"
        ops.set_plan_pp_tiles(True)
        assert k1_plan(3904, 2584, 12760)[1] == "pp256x192"
        for m, n, k in [(3904, 2584, 12760), (3072, 3072, 3072), (7288, 1344, 5768)]:
            assert ops.k1_fp8_plan(m, n, 2 * k)[1] not in ("pp192x256", "pp256x192")
    finally:
        ops.set_plan_pp_tiles(True)


def test_plan_cache_returns_the_search_result(k1_plan, splitk_plan):
    """Plans are memoised per host thread (a 256-slot table keyed by M, N, K, the
    CU count, split-K, fp8 and the pp-tile knob): many more shapes than slots,
    asked twice in different orders, give the same answers, and the knobs in the
    key still change the plan."""
    import random

    from nvidia_terraform_modules_amd import ops
    from nvidia_terraform_modules_amd.ops._lib import lib

    rng = random.Random(11)
    shapes = [tuple(rng.randrange(8, 8193, 8) for _ in range(3)) for _ in range(700)]
    first = [(k1_plan(*s), splitk_plan(*s)) for s in shapes]
    second = [(k1_plan(*s), splitk_plan(*s)) for s in reversed(shapes)][::-1]
    assert first == second
    assert k1_plan(3904, 2584, 12760) == (3904, "pp256x192", "pp256x192")
    try:
        kernels.set_cus_override(128)   # 231 tiles no longer fit one round
        assert k1_plan(3904, 2584, 12760) == (2816, "pingpong8cm", "tile160")
    finally:
        kernels.set_cus_override(0)
    assert k1_plan(3904, 2584, 12760) == (3904, "pp256x192", "pp256x192")
    ops.set_plan_pp_tiles(False)
    try:
        assert k1_plan(3904, 2584, 12760)[1] == "pingpong8cm"
    finally:
        ops.set_plan_pp_tiles(True)
    assert k1_plan(3904, 2584, 12760)[1] == "pp256x192"


def test_splitk_margin_by_slice_length(splitk_plan):
    """Round 5 (profiles/r5_margin): a split whose slices keep >= 1024 of K needs
    a 1.03 margin over the unsplit plan (1040x2776x5096: 160x160 / 2, 55.2 ->
    44.0 us); short slices keep 1.1 (2264x328x1392 stays unsplit: three slices
    of 464 K lost 28 %), and so does a split against stream-K (1136x2728x8072
    keeps stream-K split mode). The knob brings back round 4's rule, and it is
    part of the plan cache key."""
    from nvidia_terraform_modules_amd import ops

    assert splitk_plan(1040, 2776, 5096) == (1040, "tile160", "tile160", 2)
    assert splitk_plan(3896, 368, 2064) == (3896, "tile128", "tile128", 2)
    assert splitk_plan(2264, 328, 1392) == (2264, "tile128", "tile128", 1)
    assert splitk_plan(1136, 2728, 8072)[1] == "pingpong8s"
    from nvidia_terraform_modules_amd.ops._lib import lib

    ops.set_plan_splitk(1.1, 0)
    kernels.set_plan_splitk_ragged(False)   # round 4's rule: 1.1, no ragged pricing
    try:
        assert splitk_plan(1040, 2776, 5096) == (1040, "tile128", "tile128", 1)
        assert splitk_plan(3896, 368, 2064) == (3896, "tile128", "tile128", 1)
    finally:
        ops.set_plan_splitk()
        kernels.set_plan_splitk_ragged(True)
    assert splitk_plan(1040, 2776, 5096) == (1040, "tile160", "tile160", 2)


def test_fp8_splitk_margin_by_slice_length():
    """K1-fp8's split-K takes the long-slice margin from slices of >= 1152 pairs
    of e4m3 values (profiles/r5_margin/fp8_seed*): 496x3872x5584 splits in two
    (31.4 -> 25.4 us); 336x3856x4144 (slices of 1036 pairs, 16.2 -> 19.4 us
    when split) stays whole; fp8=False brings back round 4's fp8 plan."""
    from nvidia_terraform_modules_amd import ops

    assert ops.k1_fp8_splitk_plan(496, 3872, 5584) == (496, "tile128", "tile128", 2)
    assert ops.k1_fp8_splitk_plan(336, 3856, 4144) == (336, "tile128", "tile128", 1)
    ops.set_plan_splitk(fp8=False)
    try:
        assert ops.k1_fp8_splitk_plan(496, 3872, 5584) == (496, "tile128", "tile128", 1)
    finally:
        ops.set_plan_splitk()


def test_splitk_priced_against_ragged_unsplit_time(splitk_plan):
    """Long-slice split-K candidates are priced against the ragged-scaled
    unsplit time stream-K uses (profiles/r5_margin, fresh seed 14: 46 of 55
    changed plans faster): 3232x936x4024 splits on 160x160 (48.5 -> 40.6 us);
    with the knob off it stays on one round of 128x128 tiles."""
    from nvidia_terraform_modules_amd.ops._lib import lib

    assert splitk_plan(3232, 936, 4024) == (3232, "tile160", "tile160", 2)
    kernels.set_plan_splitk_ragged(False)
    try:
        assert splitk_plan(3232, 936, 4024) == (3232, "tile128", "tile128", 1)
    finally:
        kernels.set_plan_splitk_ragged(True)


def test_sk_check_flag_wiring(monkeypatch):
    """NTM_SK_CHECK switches the product-path check on; with it on,
    a set placement word raises SkPlacementError naming tile and XCCs, and the word is
    read with clear=True; with it off the word is not read at all."""
    calls = []

    def fake_word(device=None, clear=True):
        calls.append(clear)
        return 0x80000000 | 1 << 28 | 42 << 8 | 3 << 4 | 5

    monkeypatch.setattr(kernels, "sk_xcc_error", fake_word)
    monkeypatch.delenv("NTM_SK_CHECK", raising=False)
    assert not kernels.sk_check_enabled()
    out = object()
    assert kernels._sk_checked(None, out) is out and calls == []
    monkeypatch.setenv("NTM_SK_CHECK", "0")
    assert not kernels.sk_check_enabled()
    monkeypatch.setenv("NTM_SK_CHECK", "1")
    assert kernels.sk_check_enabled()
    with pytest.raises(kernels.SkPlacementError, match=r"tile 42, combiner XCC 3, other XCC 5"):
        kernels._sk_checked(None, out)
    assert calls == [True]
    monkeypatch.setattr(kernels, "sk_xcc_error", lambda device=None, clear=True: 0)
    assert kernels._sk_checked(None, out) is out
