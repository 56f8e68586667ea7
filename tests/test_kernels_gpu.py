"""GPU numerics for the gfx950 kernels: every HIP kernel vs a plain PyTorch
fp32 reference of the same op (run on a real MI355X via gpurun)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from nvidia_terraform_modules_amd import ops as o
    from nvidia_terraform_modules_amd.ops import _lib

    _lib.lib()  # must load the in-tree native library: no fallback
    assert _lib.LIB_PATH.exists()
    return o


def _rand(ops, shape, seed):
    t = torch.empty(shape, dtype=torch.bfloat16, device="cuda")
    return ops.fill_uniform_(t, seed)


@pytest.mark.parametrize("m,n,k", [
    (256, 256, 128), (512, 768, 320), (768, 512, 1024), (1024, 1024, 4096),
    (2048, 256, 192), (256, 2304, 256), (4096, 4096, 4096),
])
def test_gemm_vs_torch_fp32(ops, m, n, k):
    a = _rand(ops, (m, k), 11 + m)
    b = _rand(ops, (n, k), 13 + n)
    c = ops.gemm_bf16(a, b)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    rel = (err.pow(2).sum() / ref.pow(2).sum()).sqrt().item()
    assert rel < 4e-3


def test_gemm_identity_asymmetric(ops):
    # A = I with an asymmetric B catches a transposed C-write (playbook §3).
    n, k = 256, 256
    a = torch.eye(n, k, dtype=torch.bfloat16, device="cuda")
    b = (torch.arange(n * k, device="cuda", dtype=torch.float32).reshape(n, k) % 97 - 48).to(torch.bfloat16)
    c = ops.gemm_bf16(a, b)
    assert torch.equal(c, b.T.contiguous())


@pytest.mark.parametrize("k", [256, 320])        # default kernel: pingpong8c / pingpong8b
@pytest.mark.parametrize("ldc_pad", [256, 4])    # ldc % 8 == 0: widened epilogue; == 4: dwordx2
def test_gemm_strided_ld(ops, k, ldc_pad):
    m, n = 512, 512
    abig = _rand(ops, (m, k + 64), 3)
    bbig = _rand(ops, (n, k + 128), 4)
    a, b = abig[:, :k], bbig[:, :k]
    out = torch.zeros((m, n + ldc_pad), dtype=torch.bfloat16, device="cuda")
    ops.gemm_bf16(a, b, out[:, :n])
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert torch.all((out[:, :n].float() - ref).abs() <= atol + rtol * ref.abs())
    assert torch.count_nonzero(out[:, n:]) == 0  # no write past the ldc window


def test_gemm_rejects_bad_shapes(ops):
    a = torch.zeros((300, 256), dtype=torch.bfloat16, device="cuda")
    b = torch.zeros((6, 256), dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, b)                   # N % 4: no kernel stores it
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, a[:256], variant="pingpong8c")  # 256x256 kernel: M % 256
    with pytest.raises(ValueError):
        ops.gemm_bf16(b[:, :60], b[:, :60])  # K % 8


def test_fill_uniform_distribution(ops):
    t = _rand(ops, (1 << 20,), 99)
    f = t.float()
    assert f.min() >= -1.0 and f.max() <= 1.0
    assert abs(f.mean().item()) < 5e-3
    assert abs(f.var().item() - 1.0 / 3.0) < 5e-3
    t2 = _rand(ops, (1 << 20,), 99)
    assert torch.equal(t, t2)  # deterministic in (seed, index)
    t3 = _rand(ops, (1 << 20,), 100)
    assert not torch.equal(t, t3)


def test_ref_gemm_matches_torch(ops):
    a = _rand(ops, (96, 200), 5)   # odd shapes: reference kernel is general
    b = _rand(ops, (70, 200), 6)
    r = ops.ref_gemm_f32(a, b)
    t = a.float() @ b.float().T
    assert torch.allclose(r, t, atol=1e-4, rtol=1e-5)


def test_verify_detects_corruption(ops):
    a = _rand(ops, (512, 256), 1)
    b = _rand(ops, (512, 256), 2)
    c = ops.gemm_bf16(a, b)
    ref = ops.ref_gemm_f32(a, b)
    atol, rtol = ops.gemm_tolerance(256)
    assert ops.verify_bf16(c, ref, atol, rtol).ok
    c.view(-1)[777] += 2.0
    c.view(-1)[778] = float("nan")
    rep = ops.verify_bf16(c, ref, atol, rtol)
    assert rep.bad == 2 and not rep.ok


def test_stream_copy_and_read(ops):
    src = torch.randn(1 << 22, device="cuda")
    dst = torch.empty_like(src)
    ops.stream_copy(src, dst)
    sink = torch.zeros(2048, device="cuda")
    ops.stream_read(src, sink)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert torch.count_nonzero(sink) == 0
    # the default copy launches one block per 8 KiB tile: 8193 blocks + a tail here
    big = torch.randint(0, 255, ((1 << 26) + 8192 + 48,), dtype=torch.uint8, device="cuda")
    out = torch.zeros_like(big)
    ops.stream_copy(big, out)
    torch.cuda.synchronize()
    assert torch.equal(big, out)


@pytest.mark.parametrize("nbytes", [16, 4096 + 48, (1 << 20) * 3 + 16 * 7])
def test_stream_copy_all_configs_exact(ops, nbytes):
    """Every (unroll, policy) copy kernel (tiled, pipelined, chunked) is byte-exact, including sub-tile
    tails and a grid larger than the tile count."""
    src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    for cfg in [(1, 0, 0)] + [(u, p, g) for u in (2, 4, 8, 16) for p in range(12)
                              for g in (0, 7, 256)]:
        dst = torch.zeros_like(src)
        ops.stream_copy(src, dst, config=cfg)
        assert torch.equal(src, dst), cfg
    sink = torch.zeros(8192, device="cuda")
    for cfg in [(u, p, g) for u in (2, 4, 8, 16) for p in (0, 1) for g in (0, 5)]:
        ops.stream_read(src, sink, config=cfg)   # must not fault on tails
    torch.cuda.synchronize()


def test_gemm_graph_capture(ops):
    a = _rand(ops, (1024, 512), 21)
    b = _rand(ops, (1024, 512), 22)
    c = torch.empty((1024, 1024), dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.gemm_bf16(a, b, c)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ops.gemm_bf16(a, b, c)
    c.zero_()
    g.replay()
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(512)
    assert torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs())


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 1024, 320), (2048, 2048, 2048),
                                   (8192, 8192, 8192)])
def test_abft_rowsum_matches_fp64(ops, m, n, k):
    """The fused epilogue's row checksum equals the fp64 row sums of the exact
    product, and the O(n^2) checker passes a clean GEMM."""
    a = _rand(ops, (m, k), 31 + k)
    b = _rand(ops, (n, k), 37 + n)
    c, rs = ops.gemm_bf16_rowsum(a, b)
    exact = (a.double() @ b.double().sum(0)) if m * k < 2**27 else None
    if exact is not None:
        norm = (a.float() @ b.float().T).double().norm(dim=1)
        assert torch.all((rs.double() - exact).abs() <= 1e-3 + 2**-14 * norm)
    c_plain = ops.gemm_bf16(a, b)   # default variant = the one the rowsum path runs
    assert torch.equal(c, c_plain)  # the checksum epilogue does not change C
    rep = ops.abft_check(a, b, c, rs)
    assert rep.ok, rep.as_dict()
    assert rep.max_rel_acc < 2**-17


def test_abft_detects_corruption(ops):
    a = _rand(ops, (1024, 512), 41)
    b = _rand(ops, (1024, 512), 42)
    c, rs = ops.gemm_bf16_rowsum(a, b)
    assert ops.abft_check(a, b, c, rs).ok
    c2 = c.clone()
    c2[17, 300] += 64.0                       # a stored-output fault
    rep = ops.abft_check(a, b, c2, rs)
    assert rep.bad_store == 1 and rep.bad_acc == 0
    rs2 = rs.clone()
    rs2[900] += 0.5                           # an accumulator-path fault
    rep = ops.abft_check(a, b, c, rs2)
    assert rep.bad_acc == 1
    c3 = c.clone()
    c3[5, 5] = float("nan")
    assert not ops.abft_check(a, b, c3, rs).ok


@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (512, 1024, 768), (2048, 2048, 2048),
                                   (8192, 8192, 8192)])
def test_abft_fp8_rowsum_and_check(ops, m, n, k):
    """K1-fp8 with the fused row checksum: the checksum matches the fp64 row sums
    of the exact e4m3 product, C is bitwise the plain fp8 kernel's, the O(n^2)
    checker passes, and it flags a stored-output and an accumulator fault."""
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 51 + k)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 53 + n)
    c, rs = ops.gemm_fp8_rowsum(a, b)
    assert torch.equal(c, ops.gemm_fp8(a, b, variant="pingpong8c"))
    if m * k < 2**27:
        exact = a.double() @ b.double().sum(0)
        norm = (a.float() @ b.float().T).double().norm(dim=1)
        assert torch.all((rs.double() - exact).abs() <= 1e-3 + 2**-14 * norm)
    rep = ops.abft_check(a, b, c, rs)
    assert rep.ok, rep.as_dict()
    c2 = c.clone()
    c2[m // 2, n // 3] += 64.0
    rep = ops.abft_check(a, b, c2, rs)
    assert rep.bad_store == 1 and rep.bad_acc == 0
    rs2 = rs.clone()
    rs2[m - 1] += 0.5
    assert ops.abft_check(a, b, c, rs2).bad_acc == 1


def test_gemm_fp8_rowsum_rejects_ragged(ops):
    a = torch.zeros((256, 272), dtype=torch.float8_e4m3fn, device="cuda")
    with pytest.raises(ValueError):
        ops.gemm_fp8_rowsum(a, a)             # K % 256
    with pytest.raises(ValueError):
        ops.abft_check(a, a.to(torch.bfloat16), torch.zeros((256, 256), dtype=torch.bfloat16,
                                                            device="cuda"), torch.zeros(256, device="cuda"))


@pytest.mark.parametrize("variant", ["pingpong8", "pingpong8b", "pingpong8c", "pingpong8cw",
                                     "pingpong8cwe", "pingpong8cwn", "pingpong8cwne"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 256, 192), (256, 512, 256),
                                   (768, 1024, 320), (1024, 768, 2048), (2048, 2048, 4096),
                                   (512, 512, 384), (4096, 4352, 256), (8192, 8192, 512)])
def test_gemm_variants_vs_torch_fp32(ops, variant, m, n, k):
    """Every 8-wave schedule, including K-tile counts T = 2..6 that exercise
    each prologue/tail path (T = K / 64; pingpong8c and the widened *w
    epilogues need T even)."""
    if variant not in ("pingpong8", "pingpong8b") and (k // 64) % 2:
        pytest.skip(f"{variant} needs K % 128 == 0")
    a = _rand(ops, (m, k), 71 + k)
    b = _rand(ops, (n, k), 73 + n)
    c = ops.gemm_bf16(a, b, variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8"))  # same math, same order


@pytest.mark.parametrize("variant", ["tile128", "tile256x128", "tile128w4", "tile256x128w4"])
@pytest.mark.parametrize("m,n,k", [(128, 128, 128), (384, 640, 256), (1280, 896, 512),
                                   (256, 256, 1024), (2048, 2048, 2048), (3072, 1024, 384),
                                   (512, 384, 128)])
def test_gemm_tile128_vs_torch_fp32(ops, variant, m, n, k):
    """128x128 / 256x128-tile K1 (gemm_bf16_t128.hpp): N (and for tile128 M)
    multiples of 128 rather than 256, K-tile counts 2..32 (the ring's dummy
    pieces at every tail length), 1..192 workgroups; bitwise equal to the
    256x256 kernel where both apply."""
    if variant.startswith("tile256x128") and m % 256:
        pytest.skip("tile256x128 needs M % 256")
    a = _rand(ops, (m, k), 171 + k)
    b = _rand(ops, (n, k), 173 + n)
    c = ops.gemm_bf16(a, b, variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    if m % 256 == 0 and n % 256 == 0:
        assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8"))
    if variant.endswith("w4"):  # 4-wave kernel: same MFMA order as the wave-specialised one
        assert torch.equal(c, ops.gemm_bf16(a, b, variant=variant[:-2]))


@pytest.mark.parametrize("variant", ["tile160", "tile256x160", "tile160w4", "tile160x128",
                                     "tile128x160"])
@pytest.mark.parametrize("m,n,k", [(160, 160, 128), (1280, 800, 384), (2560, 2560, 2560),
                                   (1280, 160, 1024), (2560, 1600, 256), (5120, 320, 128),
                                   (640, 1280, 640)])
def test_gemm_tile160_vs_torch_fp32(ops, variant, m, n, k):
    """160-wide tiles (gemm_bf16_t128.hpp with MT or NT = 5; odd MT / NT split
    the DMA pieces across waves by global piece index): vs fp32, and bitwise
    equal to the 128-wide tile kernel where both tile the shape (same MFMA
    order)."""
    tm, tn = ops.kernels.TILE_SHAPES[variant]
    if m % tm or n % tn:
        pytest.skip(f"{variant} needs M % {tm}, N % {tn}")
    a = _rand(ops, (m, k), 371 + k)
    b = _rand(ops, (n, k), 373 + n)
    c = ops.gemm_bf16(a, b, variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    if m % 128 == 0 and n % 128 == 0:
        assert torch.equal(c, ops.gemm_bf16(a, b, variant="tile128"))


@pytest.mark.parametrize("m,n,k", [(4352, 4352, 256), (6144, 6144, 128), (4608, 4608, 128)])
def test_gemm_default_split_plan(ops, m, n, k):
    """Default dispatch that splits C by rows (k1_plan: top rows on 256x256,
    the rest on a small tile in a second launch): correct vs fp32 and
    bitwise equal to the single-kernel 256x256 result (same math, same order)."""
    top, top_variant, _ = ops.kernels.k1_plan(m, n, k)
    assert 0 < top < m and top_variant == "pingpong8c"
    a = _rand(ops, (m, k), 271 + k)
    b = _rand(ops, (n, k), 273 + n)
    c = ops.gemm_bf16(a, b)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8"))


@pytest.mark.parametrize("m,n,k,plan", [
    (2560, 2560, 512, (2560, "tile160")),               # 256 tiles of 160x160: one round
    (416, 1280, 128, (416, "tile128")),                 # masked edge tiles, one launch
    (1696, 2560, 256, (1696, "tile160x128")),           # 11 x 20 tiles: one round
    (4072, 1240, 256, (4072, "tile128x160")),           # 32 x 8 tiles: one full round
    (4608, 4608, 128, (3584, "pingpong8c", "tile160x128")),  # one-round tile as the rest
    (2080, 3844, 256, (512, "tile128", "tile160")),     # mixed small tiles, ragged N
    (2304, 3844, 256, (768, "tile128", "tile160")),
    (3200, 3200, 256, (3200, "pingpong8cm")),           # 256x256 with masked edge tiles
])
def test_gemm_default_dispatch_mixed_tiles(ops, m, n, k, plan):
    """Default dispatch without the exact 256x256 kernel: one 160x160 launch, a
    row split across two small-tile kernels (A/C row offsets top*lda /
    top*ldc, 160-row tiles after 128-row ones), or the masked 256x256 kernel:
    vs fp32 and bitwise equal to the explicit variants on the same row ranges."""
    top, top_variant, rest = ops.kernels.k1_plan(m, n, k)
    assert (top, top_variant) == plan[:2] and (top == m or rest == plan[2])
    a = _rand(ops, (m, k), 571 + k)
    b = _rand(ops, (n, k), 573 + n)
    c = ops.gemm_bf16(a, b)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c[:top], ops.gemm_bf16(a[:top], b, variant=top_variant))
    if top < m:
        assert torch.equal(c[top:], ops.gemm_bf16(a[top:].contiguous(), b, variant=rest))


def test_gemm_default_rejects_unplannable_shape_before_launch(ops):
    """an infeasible plan must fail before anything is written
    (K % 8 != 0: no kernel can load the rows in 16-byte chunks)."""
    a = _rand(ops, (384, 104), 5)[:, :100]
    b = _rand(ops, (256, 104), 6)[:, :100]
    c = torch.full((384, 256), 7.0, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, b, c)
    with pytest.raises(RuntimeError):           # the C ABI alone rejects it too
        from nvidia_terraform_modules_amd.ops._lib import check, lib, stream_handle
        check(lib().ntm_gemm_bf16_variant(0, a.data_ptr(), b.data_ptr(), c.data_ptr(), 384, 256,
                                          100, 104, 104, 256, stream_handle()), "default")
    torch.cuda.synchronize()
    assert torch.all(c == 7.0)


def test_gemm_tile128_rejects_bad_shapes(ops):
    a = torch.zeros((128, 192), dtype=torch.bfloat16, device="cuda")[:, :100]
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, a, variant="tile128")    # K % 8
    a = torch.zeros((192, 128), dtype=torch.bfloat16, device="cuda")
    b = torch.zeros((6, 128), dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, b, variant="tile128")    # N % 4 (8-byte C stores)
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, a, variant="tile256x160")  # whole tiles only (M % 256)


@pytest.mark.parametrize("variant", ["tile128", "tile256x128", "tile160", "tile160x128",
                                     "tile128x160", "tile128x256", "pingpong8cm", "pp192x256",
                                     "pp256x192", "default"])
@pytest.mark.parametrize("m,n,k", [(1000, 1000, 1024), (100, 4096, 256), (1696, 2560, 256),
                                   (2400, 3200, 128), (1, 4, 128), (333, 1004, 384),
                                   (8200, 260, 128), (4000, 4000, 512), (1000, 1000, 1000),
                                   (333, 1004, 200), (100, 512, 72), (64, 64, 8)])
def test_gemm_masked_edge_tiles(ops, variant, m, n, k):
    """Masked edge tiles on ragged C (wave-specialised tiles: any M, N % 4 and a
    zero-filled partial last K-tile for K % 8; the 256x256 kernel "pingpong8cm":
    N % 8, K % 8): vs fp32, and nothing written outside C - C is a view into
    a sentinel-filled buffer with extra rows below and extra columns to the
    right (ldc > N)."""
    if variant in ("pingpong8cm", "pp192x256", "pp256x192", "pp224x256") and n % 8:
        pytest.skip(f"{variant}: N % 8 (8-column store chunks)")
    a = _rand(ops, (m, k), 971 + m)
    b = _rand(ops, (n, k), 973 + n)
    big = torch.full((m + 37, n + 16), 3.0, dtype=torch.bfloat16, device="cuda")
    c = big[:m, :n]
    ops.gemm_bf16(a, b, c, variant=variant)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(big[m:] == 3.0) and torch.all(big[:, n:] == 3.0)
    if variant != "default" and m % 256 == 0 and n % 256 == 0:
        assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8"))
    if variant in ("pp192x256", "pp256x192", "pp224x256"):   # same MFMAs in the same K order
        assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8cm"))


@pytest.mark.parametrize("variant", ["pp192x256", "pp256x192", "pp224x256"])
@pytest.mark.parametrize("m,n,k", [(3904, 2584, 12760), (7288, 1344, 5768), (3512, 3456, 16040),
                                   (1312, 6304, 5080), (192, 192, 128), (200, 200, 136),
                                   (4032, 4032, 1024), (5000, 3000, 2000)])
def test_gemm_192_tiles(ops, variant, m, n, k):
    """192x256 / 256x192 ping-pong tiles (gemm_bf16_pp3h.hpp): the ragged one-round
    shapes hipBLASLt fills with 192-wide tiles, exact multiples of 192, more than one
    round and the partial-K build - vs fp32, bitwise equal to pingpong8cm, and
    nothing written outside C."""
    a = _rand(ops, (m, k), 17 + m)
    b = _rand(ops, (n, k), 19 + n)
    big = torch.full((m + 5, n + 8), 3.0, dtype=torch.bfloat16, device="cuda")
    c = big[:m, :n]
    ops.gemm_bf16(a, b, c, variant=variant)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(big[m:] == 3.0) and torch.all(big[:, n:] == 3.0)
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8cm"))


@pytest.mark.parametrize("variant", ["tile128", "tile256x128", "tile160", "tile160x128",
                                     "tile128x160", "tile128x256"])
@pytest.mark.parametrize("splits", [2, 3, 5, 16])
@pytest.mark.parametrize("m,n,k", [(280, 636, 7568), (100, 4096, 1000), (333, 1004, 2056),
                                   (1, 4, 1032), (256, 512, 8192), (64, 64, 136)])
def test_gemm_splitk(ops, variant, splits, m, n, k):
    """Split-K on the masked small tiles: K slices of round_up(ceil(K / S), 64)
    (the last one shorter, its partial K-tile zero-filled), fp32 partials, one
    reduction: vs fp32, within the unsplit tolerance, nothing written outside C
    (sentinel rows below and columns right of C, ldc > N)."""
    a = _rand(ops, (m, k), 1171 + m)
    b = _rand(ops, (n, k), 1173 + n)
    big = torch.full((m + 19, n + 12), 3.0, dtype=torch.bfloat16, device="cuda")
    c = big[:m, :n]
    ops.gemm_bf16(a, b, c, variant=variant, splits=splits)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(big[m:] == 3.0) and torch.all(big[:, n:] == 3.0)


@pytest.mark.parametrize("m,n,k,splits", [(280, 6352, 7568, 3), (128, 8192, 8192, 4),
                                          (333, 1004, 2056, None)])
def test_gemm_default_dispatch_splitk(ops, m, n, k, splits):
    """The default dispatch takes split-K for skinny long-K C (k1_splitk_plan),
    with a workspace from PyTorch's allocator: vs fp32, and equal to the
    explicit split of the same tile (same slices, same reduction order)."""
    top, tv, _, sp = ops.kernels.k1_splitk_plan(m, n, k)
    assert top == m and sp > 1 and (splits is None or sp == splits)
    a = _rand(ops, (m, k), 1271 + m)
    b = _rand(ops, (n, k), 1273 + n)
    c = ops.gemm_bf16(a, b)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_bf16(a, b, variant=tv, splits=sp))


def test_gemm_splitk_rejects_bad_args(ops):
    a = torch.zeros((128, 256), dtype=torch.bfloat16, device="cuda")
    with pytest.raises(ValueError):
        ops.gemm_bf16(a, a, variant="pingpong8c", splits=2)   # masked small tiles only
    from nvidia_terraform_modules_amd.ops._lib import lib
    c = torch.zeros((128, 128), dtype=torch.bfloat16, device="cuda")
    ws = torch.zeros(16, dtype=torch.float32, device="cuda")   # too small: nothing launched
    rc = lib().ntm_gemm_bf16_splitk(15, 2, a.data_ptr(), a.data_ptr(), c.data_ptr(), 128, 128, 256,
                                    256, 256, 128, ws.data_ptr(), 64, 0)
    assert rc != 0


def _rand_fp8(shape, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand(shape, generator=g, device="cuda") * 2 - 1      # uniform [-1, 1)
    return x.to(torch.float8_e4m3fn)


@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (512, 256, 768), (256, 768, 512),
                                   (1024, 1024, 2048), (2048, 4352, 1280)])
def test_gemm_fp8_vs_torch_fp32(ops, m, n, k):
    """K1-fp8 against a plain fp32 matmul of the same (dequantised) e4m3 values:
    products of e4m3 values are exact in fp32, so the only error is the
    accumulation order and the bf16 output rounding."""
    a = _rand_fp8((m, k), 11 + k)
    b = _rand_fp8((n, k), 13 + n)
    c = ops.gemm_fp8(a, b)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_fp8(a, b))    # deterministic


def test_gemm_fp8_operand_map_probe(ops):
    """The f8f6f4 MFMA sums over k, so A and B only need the SAME k order per
    lane; rows must be lane & 15. Pin both with exact small-integer data."""
    from nvidia_terraform_modules_amd.ops._lib import check, lib_experimental, stream_handle
    torch.manual_seed(0)
    a = torch.randint(-3, 4, (16, 128)).float().to(torch.float8_e4m3fn)
    b = torch.randint(-3, 4, (16, 128)).float().to(torch.float8_e4m3fn)
    ref = a.float() @ b.float().T

    def stage(mat, perm):
        u8 = mat.view(torch.uint8)
        rows = torch.arange(64) & 15
        return torch.gather(u8[rows], 1, perm[torch.arange(64) >> 4]).contiguous().cuda()

    # the kernel's map ("halves16"): lane group g holds k 16g..16g+15, 64+16g..64+16g+15
    perm = torch.stack([torch.cat([torch.arange(16 * g, 16 * g + 16),
                                   torch.arange(64 + 16 * g, 64 + 16 * g + 16)]) for g in range(4)])
    d = torch.empty((64, 4), dtype=torch.float32, device="cuda")
    sa, sb = stage(a, perm), stage(b, perm)      # keep both alive across the launch
    check(lib_experimental().ntm_mfma_f8_probe(sa.data_ptr(), sb.data_ptr(), d.data_ptr(), stream_handle()),
          "probe")
    torch.cuda.synchronize()
    got = torch.empty((16, 16))
    dc = d.cpu()
    for lane in range(64):
        for r in range(4):
            got[4 * (lane >> 4) + r, lane & 15] = dc[lane, r]
    assert torch.equal(got, ref)


@pytest.mark.parametrize("m,n,k", [(1000, 1000, 512), (300, 2056, 256), (4000, 4000, 256),
                                   (1000, 1000, 1008), (256, 256, 16), (300, 2056, 400)])
def test_gemm_fp8_masked_edge_tiles(ops, m, n, k):
    """K1-fp8 on ragged C (masked build; K % 256 != 0 adds the zero-filled
    partial last K-tile): vs fp32, nothing written outside C."""
    a = _rand_fp8((m, k), 17 + m)
    b = _rand_fp8((n, k), 19 + n)
    big = torch.full((m + 21, n + 16), 3.0, dtype=torch.bfloat16, device="cuda")
    c = big[:m, :n]
    ops.gemm_fp8(a, b, c)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(big[m:] == 3.0) and torch.all(big[:, n:] == 3.0)


@pytest.mark.parametrize("variant", ["tile128", "tile256x128", "tile160", "tile160x128",
                                     "tile128x160", "tile128x256"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (1000, 1000, 1008), (300, 2056, 400),
                                   (640, 520, 2048), (33, 8, 16)])
def test_gemm_fp8_wave_specialised_tiles(ops, variant, m, n, k):
    """K1-fp8 on the wave-specialised tiles (fp8 consumer: one f8f6f4 MFMA over
    both k-halves, fragments refilled after their last MFMA): vs fp32 on whole,
    ragged and K-tail shapes, nothing written outside C (strided C), and
    bitwise deterministic."""
    a = _rand_fp8((m, k), 23 + m + k)
    b = _rand_fp8((n, k), 29 + n)
    big = torch.full((m + 7, n + 24), 3.0, dtype=torch.bfloat16, device="cuda")
    c = big[:m, :n]
    ops.gemm_fp8(a, b, c, variant=variant)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), (variant, float(err.max()))
    assert torch.all(big[m:] == 3.0) and torch.all(big[:, n:] == 3.0)
    assert torch.equal(c, ops.gemm_fp8(a, b, variant=variant))


@pytest.mark.parametrize("m,n,k,plan", [(4352, 4352, 512, (3840, "pingpong8o", "tile128")),
                                        (4608, 4608, 256, (3584, "pingpong8c", "tile160x128")),
                                        (2816, 2816, 512, (2816, "tile128x256", "tile128x256")),
                                        (1024, 1024, 1024, (1024, "tile128", "tile128"))])
def test_gemm_fp8_default_plan(ops, m, n, k, plan):
    """K1-fp8's default dispatch runs k1_fp8_plan: row splits (256x256 rounds +
    a small-tile rest) and small tiles are bitwise equal to the explicit
    variants on their rows (same MFMA order per output), and match fp32."""
    assert ops.k1_fp8_plan(m, n, k) == plan
    a = _rand_fp8((m, k), 31 + m)
    b = _rand_fp8((n, k), 37 + n)
    c = ops.gemm_fp8(a, b)
    top, tv, rv = plan
    assert torch.equal(c[:top], ops.gemm_fp8(a[:top], b, variant=tv))
    if top < m:
        assert torch.equal(c[top:], ops.gemm_fp8(a[top:].contiguous(), b, variant=rv))
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs())


@pytest.mark.parametrize("variant,splits", [("tile128", 2), ("tile128", 5), ("tile160", 3),
                                            ("tile256x128", 4), ("tile160x128", 2),
                                            ("tile128x160", 3), ("tile128x256", 2)])
@pytest.mark.parametrize("m,n,k", [(280, 1000, 4112), (128, 256, 2048), (33, 8, 400)])
def test_gemm_fp8_splitk(ops, variant, splits, m, n, k):
    """K1-fp8 split-K (fp32 partials of the fp8 consumer, one reduction) vs fp32,
    on ragged C and partial K-tiles (K % 128 != 0)."""
    a = _rand_fp8((m, k), 41 + m)
    b = _rand_fp8((n, k), 43 + n)
    c = ops.gemm_fp8(a, b, variant=variant, splits=splits)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), (variant, splits, float(err.max()))


@pytest.mark.parametrize("m,n,k", [(280, 6352, 15136), (256, 2048, 16400), (333, 1008, 4112)])
def test_gemm_fp8_default_splitk_plan(ops, m, n, k):
    """Skinny C with a long K: the fp8 default splits K as k1_fp8_splitk_plan says,
    bitwise equal to the explicit split on that tile."""
    top, tv, _, sp = ops.k1_fp8_splitk_plan(m, n, k)
    assert sp > 1 and top == m
    a = _rand_fp8((m, k), 47 + m)
    b = _rand_fp8((n, k), 53 + n)
    c = ops.gemm_fp8(a, b)
    assert torch.equal(c, ops.gemm_fp8(a, b, variant=tv, splits=sp))
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs())


def test_gemm_fp8_rejects_bad_shapes(ops):
    a = torch.zeros((256, 136), dtype=torch.float8_e4m3fn, device="cuda")[:, :120]
    with pytest.raises(ValueError):
        ops.gemm_fp8(a, a)                       # K % 16
    with pytest.raises(ValueError):
        ops.gemm_fp8(a.to(torch.bfloat16), a.to(torch.bfloat16))


def _uniform_pm1_host(seed: int, n: int):
    """Host replica of ntm::uniform_pm1 (common.hpp): splitmix64 hash -> 24 bits."""
    import numpy as np

    def mix64(x):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))

    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        h = mix64((np.uint64(seed) * np.uint64(0x100000001B3)) ^ mix64(idx))
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return torch.from_numpy(np.float32(2.0) * u - np.float32(1.0))


def test_fill_e4m3_matches_torch_rounding(ops):
    """The device e4m3 encoder (RNE, saturating) agrees bit for bit with torch's
    float8_e4m3fn conversion of the same uniform stream, replicated on the host."""
    n = 1 << 16
    t = ops.fill_uniform_(torch.empty((n,), dtype=torch.float8_e4m3fn, device="cuda"), 77)
    want = _uniform_pm1_host(77, n).to(torch.float8_e4m3fn)
    assert torch.equal(t.cpu().view(torch.uint8), want.view(torch.uint8))
    f = t.float()
    assert f.min() >= -1.0 and f.max() <= 1.0 and abs(f.mean().item()) < 2e-2
    # the decoder, edge cases included, through the reference GEMM: A = x on the diagonal, B = I
    vals = torch.tensor([0.0, 2 ** -9, 3 * 2 ** -10, 2 ** -6, 0.9375, 1.0, 448.0, 500.0, -17.0],
                        device="cuda")
    want = vals.to(torch.float8_e4m3fn)
    a = torch.zeros((256, 256), device="cuda").to(torch.float8_e4m3fn)
    a.view(torch.uint8)[torch.arange(9), torch.arange(9)] = want.view(torch.uint8)
    eye = torch.eye(256, device="cuda").to(torch.float8_e4m3fn)
    got = ops.ref_gemm_f32(a, eye).diagonal()[:9]   # torch maps 500 to NaN (0x7f): decoded too
    assert torch.allclose(got, want.float(), rtol=0, atol=0, equal_nan=True)


def test_gemm_fp8_vs_independent_reference(ops):
    """K1-fp8 against the fp32-FMA reference kernel on device-filled e4m3."""
    m = n = k = 1024
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 5)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 6)
    ref = ops.ref_gemm_f32(a, b)
    assert torch.allclose(ref, a.float() @ b.float().T, atol=1e-4, rtol=1e-5)
    atol, rtol = ops.gemm_tolerance(k)
    assert ops.verify_bf16(ops.gemm_fp8(a, b), ref, atol, rtol).ok


def test_gemm_fp8_plain_and_scaled_mfma_forms_agree_bitwise(ops):
    """The default K1-fp8 issues v_mfma_f32_16x16x128_f8f6f4 without the scale
    prefix; knob 5 is the same schedule on the MX-scaled form with unit E8M0
    scales. Same products in the same order: the outputs must be identical."""
    m, n, k = 512, 768, 1024
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 11)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 12)
    c0 = ops.gemm_fp8(a, b)
    c5 = ops.gemm_fp8(a, b, knob=5)
    assert torch.equal(c0.view(torch.int16), c5.view(torch.int16))
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert ((c0.float() - ref).abs() <= atol + rtol * ref.abs()).all()


@pytest.mark.parametrize("variant", ["pingpong8o", "pingpong8od"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (1024, 512, 1024), (4608, 4608, 512),
                                   (8192, 8192, 256), (2304, 1792, 768)])
def test_persistent_overlap_vs_torch_fp32(ops, variant, m, n, k):
    """pingpong8o, the persistent pingpong8c whose C stores overlap the next
    tile's K loop (gemm_bf16_pp6.hpp; its shipping build spreads the boundary
    stores), and the same build through the experimental id (pingpong8od): 1 to 4
    tiles per workgroup (4608^2: 324 tiles on 256 workgroups, so both one- and
    two-tile workgroups), the shortest tile (K = 256, T = 4) included; vs fp32,
    and bitwise equal to pingpong8c (each accumulator sees the same MFMAs in
    the same K order)."""
    a = _rand(ops, (m, k), 601 + k)
    b = _rand(ops, (n, k), 603 + n)
    c = ops.gemm_bf16(a, b, variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8c"))


@pytest.mark.parametrize("m,n,k", [(256, 256, 512), (2048, 1024, 1024), (4608, 4608, 512),
                                   (8192, 8192, 2048), (8192, 8192, 512)])
def test_fp8_persistent_overlap_vs_torch_fp32(ops, m, n, k):
    """K1-fp8 on the persistent overlap kernel (fp8 knob 30: pingpong8o with
    f8f6f4 MFMAs on VGPR accumulators, round 4): 1-4 tiles per workgroup, vs
    the fp32 product of the e4m3 values, and bitwise equal to the default fp8
    build (per accumulator the same MFMAs in the same K order)."""
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 31)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 32)
    ck = ops.gemm_fp8(a, b, knob=30)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert ((ck.float() - ref).abs() <= atol + rtol * ref.abs()).all()
    assert torch.equal(ck.view(torch.int16), ops.gemm_fp8(a, b).view(torch.int16))
    # knob 31 = the spread-store build the plan ships (padded asm-MFMA srcC)
    assert torch.equal(ops.gemm_fp8(a, b, knob=31).view(torch.int16), ck.view(torch.int16))
    assert torch.equal(ops.gemm_fp8(a, b, variant="pingpong8c").view(torch.int16),
                       ck.view(torch.int16))
    if k == 512:  # 4 K-tiles of 128 e4m3 is the build's minimum: shorter K is refused
        with pytest.raises(RuntimeError):
            ops.gemm_fp8(a[:, :256], b[:, :256], knob=30)


@pytest.mark.parametrize("m,n,k", [(256, 256, 768),      # one tile, T = 6: the peeled pair is t = 2
                                   (4096, 4096, 768),    # one tile per workgroup, T = 6
                                   (8192, 4096, 768),    # 2 tiles per workgroup, T = 6
                                   (8192, 8192, 1024),   # 4 per workgroup, T = 8
                                   (4608, 4352, 4096),   # 306 tiles: 1-2 per workgroup
                                   (8192, 8192, 8192)])  # the Job's shape
def test_fp8_l2_prefetch_build_is_bitwise_equal(ops, m, n, k):
    """fp8 knob 32 (round 6): the shipping spread-store fp8 build (knob 31) with
    the next tile's K-tiles 0 / 1 touched into L2 over K-tiles T-4 / T-3 (PF).
    The touches land in a scratch slice and only change counted waits, so C is
    bitwise the default's; vs the fp32 product; K below 768 is refused."""
    a = ops.fill_uniform_(torch.empty((m, k), dtype=torch.float8_e4m3fn, device="cuda"), 41)
    b = ops.fill_uniform_(torch.empty((n, k), dtype=torch.float8_e4m3fn, device="cuda"), 42)
    c31 = ops.gemm_fp8(a, b, knob=31)
    c32 = ops.gemm_fp8(a, b, knob=32)
    assert torch.equal(c32.view(torch.int16), c31.view(torch.int16))
    for _ in range(3):
        assert torch.equal(ops.gemm_fp8(a, b, knob=32).view(torch.int16), c31.view(torch.int16))
    if m * n <= 4096 * 4096:
        ref = a.float() @ b.float().T
        atol, rtol = ops.gemm_tolerance(k)
        assert ((c32.float() - ref).abs() <= atol + rtol * ref.abs()).all()
    with pytest.raises(RuntimeError):
        ops.gemm_fp8(a[:, :512], b[:, :512], knob=32)


@pytest.mark.parametrize("m,n,k", [(1000, 1000, 256), (4472, 5688, 640), (4608, 4360, 512),
                                   (8192, 8192, 256), (333, 1000, 384), (5000, 4104, 768),
                                   # partial K (K % 128 != 0): 4, 6, 8 K-tiles, the last
                                   # pair partial or all past K
                                   (4472, 5688, 200), (1000, 4104, 328), (4608, 4360, 456),
                                   (2056, 3000, 1000), (4472, 5688, 5832)])
@pytest.mark.parametrize("variant", ["pingpong8om", "pingpong8omd"])
def test_persistent_masked_vs_torch_fp32(ops, m, n, k, variant):
    """pingpong8om (round 4): the persistent overlap kernel on ragged C - edge
    tiles with clamped sources and masked stores, 1-2 tiles per workgroup
    (4472x5688: 414 tiles on 256 workgroups), K % 128 != 0 on the partial-K
    build (chunks past K load zeros), rows / columns past C never written
    (the guard columns of a wider out stay untouched), and bitwise equal to
    pingpong8cm (same MFMAs in the same K order). pingpong8omd spreads the
    boundary stores; both issue every masked store (buffer range check), so
    the counted vmcnt waits stay exact at ragged edges."""
    a = _rand(ops, (m, k), 641 + k)
    b = _rand(ops, (n, k), 643 + n)
    out = torch.full((m, n + 8), 7.0, dtype=torch.bfloat16, device="cuda")
    c = ops.gemm_bf16(a, b, out[:, :n], variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8cm"))
    assert torch.all(out[:, n:] == 7.0)


@pytest.mark.parametrize("m,n,k", [(8192, 8192, 1024), (2048, 2048, 256)])
def test_gemm_clock_build(ops, m, n, k):
    """The GEMM's own clock: the shipping pingpong8o with a
    start / end clock stamp per workgroup writes the same C as the default
    build, and every workgroup reports a plausible shader clock."""
    a = _rand(ops, (m, k), 631)
    b = _rand(ops, (n, k), 633)
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    r = ops.gemm_clock_ghz(a, b, c, steps=3)
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8o"))
    assert r["launches"] == 3 and r["workgroups"] == 3 * min(256, (m // 256) * (n // 256))
    assert 0.5 < r["p10_GHz"] <= r["median_GHz"] <= r["max_GHz"] < 3.0, r
    assert r["min_GHz"] <= r["launch_GHz"] <= r["max_GHz"], r
    assert len(r["per_launch_cycles_median"]) == 3 and len(r["per_launch_window_us_median"]) == 3
    xg = r["per_xcd_group_median_GHz"]
    assert len(xg) == 8 and all(r["min_GHz"] <= x <= r["max_GHz"] for x in xg)
    # the groups are labelled by the XCC_ID register, and on
    # MI355X (SPX) the dispatcher's blockIdx & 7 round robin IS the XCD - the
    # placement stream-K's fix-up protocol relies on
    assert r["xcc_ids"] == list(range(8)), r["xcc_of_blockidx_mod_8"]
    assert r["blockidx_mod_8_is_xcc"] is True, r["xcc_of_blockidx_mod_8"]
    assert set(r["per_xcc_median_GHz"]) == {str(x) for x in range(8)}
    assert r["min_GHz"] <= r["bound_GHz"] <= r["median_GHz"] and r["xcc_clock_spread_pct"] >= 0
    with pytest.raises(ValueError):
        ops.gemm_clock_ghz(a[:, :200], b[:, :200])


def test_default_runs_persistent_build_past_one_round(ops):
    """The default plan puts a multi-round 256x256 part on pingpong8o: same
    bytes as pingpong8c; strided ldc (% 8 != 0) falls back to pingpong8c."""
    m, n, k = 5120, 5120, 256
    a = _rand(ops, (m, k), 621)
    b = _rand(ops, (n, k), 623)
    assert ops.k1_plan(m, n, k) == (m, "pingpong8o", "tile128")
    ref = ops.gemm_bf16(a, b, variant="pingpong8c")
    assert torch.equal(ops.gemm_bf16(a, b), ref)
    out = torch.zeros((m, n + 4), dtype=torch.bfloat16, device="cuda")
    ops.gemm_bf16(a, b, out[:, :n], variant="pingpong8o")
    assert torch.equal(out[:, :n], ref)


SK_SHAPES = [(4472, 5688, 5832),   # 414 tiles: stream-K over all of them, K % 128 = 72
             (4608, 4608, 1024),   # 324 whole tiles
             (6144, 6144, 2048),   # 576 tiles: 256 whole, then stream-K over 320
             (4472, 5688, 200),    # two K-tile pairs per tile, the second partial
             (8192, 2304, 128),    # one pair per tile: nothing to split, balanced tiles only
             (5000, 4104, 4096),
             (1000, 17000, 384)]


@pytest.mark.parametrize("m,n,k", SK_SHAPES)
def test_stream_k_vs_torch_fp32(ops, m, n, k):
    """pingpong8s (round 4, gemm_bf16_sk.hpp): the last two rounds of 256x256
    tiles dealt out as K-tile pairs per XCD, split tiles fixed up through fp32
    partials and a counter. vs the fp32 product; rows / columns past C never
    written; a second launch gives the same bytes (counters were left at 0);
    the REV build (segments last-first: heads usually reach the fix-up first,
    the protocol's other branches) is bitwise equal."""
    a = _rand(ops, (m, k), 651 + k)
    b = _rand(ops, (n, k), 653 + n)
    out = torch.full((m, n + 8), 7.0, dtype=torch.bfloat16, device="cuda")
    c = ops.gemm_bf16(a, b, out[:, :n], variant="pingpong8s")
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(out[:, n:] == 7.0)
    first = c.clone()
    assert torch.equal(ops.gemm_bf16(a, b, variant="pingpong8s"), first)
    assert ops.sk_xcc_error() == 0   # every split tile's parts ran on one XCD
    assert torch.equal(ops.gemm_bf16(a, b, variant="pingpong8s_rev"), first)


def test_stream_k_counters_left_zero_and_refusals(ops):
    """The fix-up counters are zero after a launch (the combiner resets them), so
    a workspace zeroed once serves every later launch on its stream; partial
    slots may hold anything. Shapes stream-K does not serve are refused before
    anything launches."""
    from nvidia_terraform_modules_amd.ops._lib import lib, stream_handle

    m, n, k = 4472, 5688, 5832
    a = _rand(ops, (m, k), 661)
    b = _rand(ops, (n, k), 663)
    c = torch.empty((m, n), dtype=torch.bfloat16, device="cuda")
    wsb = ops.sk_ws_bytes(m, n, k)
    ws = torch.full(((wsb + 3) // 4,), -1.0, dtype=torch.float32, device="cuda")
    ws[:1024].zero_()  # the counter block: zero on entry (the caller's contract)
    assert lib().ntm_gemm_bf16_sk(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, k, k, n,
                                  ws.data_ptr(), wsb, stream_handle()) == 0
    torch.cuda.synchronize()
    assert torch.all(ws[:1024].view(torch.int32) == 0)
    assert torch.equal(c, ops.gemm_bf16(a, b, variant="pingpong8s"))
    c2 = torch.empty_like(c)  # the same workspace again, no re-zeroing
    assert lib().ntm_gemm_bf16_sk(a.data_ptr(), b.data_ptr(), c2.data_ptr(), m, n, k, k, k, n,
                                  ws.data_ptr(), wsb, stream_handle()) == 0
    assert torch.equal(c2, c)
    # too small a workspace, and shapes without a partial second round
    assert lib().ntm_gemm_bf16_sk(a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, k, k, n,
                                  ws.data_ptr(), wsb - 4, stream_handle()) != 0
    assert ops.sk_ws_bytes(8192, 8192, 8192) == 0     # 1024 tiles: whole rounds
    assert ops.sk_ws_bytes(4096, 4096, 4096) == 0     # 256 tiles: one round
    with pytest.raises(ValueError):  # exactly one round of 256x256 tiles: neither mode
        ops.gemm_bf16(a[:4096, :4096], b[:4096, :4096], variant="pingpong8s")


@pytest.mark.parametrize("m,n,k", [(4864, 3608, 5696), (6496, 2752, 5416),
                                   (4672, 1472, 6696), (976, 5712, 9680)])
def test_default_plan_runs_stream_k(ops, m, n, k):
    """Where the split-K plan prices stream-K below the unsplit plan (a small
    partial second round at long K; split mode on ragged one-round C, the last
    two shapes - on the 256x256 or, since round 5, the 192-wide tiles), the
    default dispatch runs it: the same bytes as that variant, within tolerance
    of the fp32 product."""
    top = ops.k1_splitk_plan(m, n, k)[1]
    assert top in ops.kernels.SK_VARIANTS
    a = _rand(ops, (m, k), 671)
    b = _rand(ops, (n, k), 673)
    c = ops.gemm_bf16(a, b)
    assert torch.equal(c, ops.gemm_bf16(a, b, variant=top))
    assert ops.sk_xcc_error() == 0
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    assert torch.all((c.float() - ref).abs() <= atol + rtol * ref.abs())


SKS_SHAPES = [(4672, 1472, 6696),   # 114 tiles: 2 K slices each (head / tail protocol)
              (4096, 2048, 8192),   # 128 tiles, whole K pairs: 2 slices
              (2048, 2048, 4096),   # 64 tiles: 4 slices
              (280, 6352, 7568),    # 50 tiles: 4 slices, K % 128 != 0
              (1000, 1000, 1000),   # 16 tiles: 8 slices of one pair, partial K
              (256, 256, 256)]      # 1 tile: 2 slices of one pair


@pytest.mark.parametrize("m,n,k", SKS_SHAPES)
def test_stream_k_split_mode_vs_torch_fp32(ops, m, n, k):
    """pingpong8s on at most half a round of 256x256 tiles (round 4, split
    mode): every tile in S K slices at once, the slice that completes the
    counter sums all S partials in slice order. vs the fp32 product; no row /
    column past C written; a second launch gives the same bytes (counters left
    at 0, combiner-independent sum)."""
    assert ops.sk_ws_bytes(m, n, k) > 0
    a = _rand(ops, (m, k), 681 + k)
    b = _rand(ops, (n, k), 683 + n)
    out = torch.full((m, n + 8), 7.0, dtype=torch.bfloat16, device="cuda")
    c = ops.gemm_bf16(a, b, out[:, :n], variant="pingpong8s")
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(out[:, n:] == 7.0)
    first = c.clone()
    for _ in range(3):
        assert torch.equal(ops.gemm_bf16(a, b, variant="pingpong8s"), first)
    assert ops.sk_xcc_error() == 0   # every slice of a tile ran on the combiner's XCD
    # the round-4 S-partial protocol: at S = 2 the head / tail protocol's own + other
    # is the same fp32 sum as partial0 + partial1 (commutative), so bitwise equal
    assert torch.equal(ops.gemm_bf16(a, b, variant="pingpong8s_nopair"), first)


SKH_SHAPES = [(4152, 1096, 16056),  # 110 192x256 / 102 256x192 tiles: 2 slices, K % 16 == 8
              (2840, 1768, 8904),   # the shapes the plan sends there
              (5976, 888, 8720),
              (1000, 1000, 4096),   # 24 / 20 tiles: 8 slices
              (1000, 1000, 1000),   # partial K, one pair per slice
              (192, 256, 256),      # one tile, 2 slices of one pair
              (2048, 1536, 6144)]   # exact tiles


@pytest.mark.parametrize("variant", ["pp192x256s", "pp256x192s"])
@pytest.mark.parametrize("m,n,k", SKH_SHAPES)
def test_stream_k_split_mode_192_tiles_vs_torch_fp32(ops, variant, m, n, k):
    """Split mode on the 192-wide ping-pong tiles (gemm_bf16_skh.hpp, round 5):
    vs the fp32 product, no column past C written, repeat launches give the same
    bytes, every slice ran on the combiner's XCD."""
    if not ops.kernels.skh_ws_bytes(variant, m, n, k):
        pytest.skip(f"{variant}: more than half a round of its tiles")
    a = _rand(ops, (m, k), 681 + k)
    b = _rand(ops, (n, k), 683 + n)
    out = torch.full((m, n + 8), 7.0, dtype=torch.bfloat16, device="cuda")
    c = ops.gemm_bf16(a, b, out[:, :n], variant=variant)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    err = (c.float() - ref).abs()
    assert torch.all(err <= atol + rtol * ref.abs()), float(err.max())
    assert torch.all(out[:, n:] == 7.0)
    first = c.clone()
    for _ in range(3):
        assert torch.equal(ops.gemm_bf16(a, b, variant=variant), first)
    assert ops.sk_xcc_error() == 0


@pytest.mark.parametrize("m,n,k", [(4152, 1096, 16056), (2840, 1768, 8904)])
def test_default_runs_split_mode_on_192_tiles(ops, m, n, k):
    """The default plan picks split mode on a 192-wide tile for these shapes, and
    the default dispatch gives that variant's bytes."""
    top = ops.k1_splitk_plan(m, n, k)[1]
    assert top in ("pp192x256s", "pp256x192s")
    a = _rand(ops, (m, k), 5)
    b = _rand(ops, (n, k), 6)
    assert torch.equal(ops.gemm_bf16(a, b), ops.gemm_bf16(a, b, variant=top))
    assert ops.sk_xcc_error() == 0



@pytest.mark.parametrize("variant,m,n,k", [("default", 4152, 1096, 16056),   # skh, head/tail
                                           ("pp192x256s", 1000, 1000, 4096),  # skh, 8 slices
                                           ("pingpong8s", 4672, 1472, 6696),  # sks, head/tail
                                           ("pingpong8s", 2048, 2048, 4096),   # sks, 4 slices
                                           ("pingpong8s", 4608, 4352, 2048)])  # two-round mode
def test_sk_placement_fault_raises_on_the_product_path(ops, monkeypatch, variant, m, n, k):
    """with NTM_SK_CHECK=1 the dispatch reads and clears the
    placement word after every stream-K launch; the injected wrong-XCC tag
    (set_sk_fault_inject) makes it raise SkPlacementError, naming the tile. Off
    again, the same call passes and the word is clear."""
    if variant == "pingpong8s":
        assert ops.sk_ws_bytes(m, n, k) > 0
    a = _rand(ops, (m, k), 11)
    b = _rand(ops, (n, k), 12)
    monkeypatch.setenv("NTM_SK_CHECK", "1")
    good = ops.gemm_bf16(a, b, variant=variant)          # no fault: no raise
    ops.set_sk_fault_inject(True)
    try:
        with pytest.raises(ops.SkPlacementError, match="not trusted"):
            ops.gemm_bf16(a, b, variant=variant)
    finally:
        ops.set_sk_fault_inject(False)
    assert ops.sk_xcc_error() == 0                       # read and cleared by the raise
    assert torch.equal(ops.gemm_bf16(a, b, variant=variant), good)
    monkeypatch.setenv("NTM_SK_CHECK", "0")               # off: the word stays sticky, no raise
    ops.set_sk_fault_inject(True)
    try:
        ops.gemm_bf16(a, b, variant=variant)
    finally:
        ops.set_sk_fault_inject(False)
    assert ops.sk_xcc_error() != 0 and ops.sk_xcc_error() == 0


@pytest.mark.parametrize("m,n,k", [(256, 256, 512), (2048, 1024, 1024), (4608, 4352, 2048)])
def test_dma4k_energy_study_builds_match_the_default(ops, m, n, k):
    """The 4-wave 128x128-per-wave builds restored for the energy study
    (profiles/r6_fp8, tools/experiments/energy_ab.py): bf16 variant dma4k_d3 and
    fp8 knob 12 agree with the default within tolerance (different MFMA order)."""
    a = _rand(ops, (m, k), 51)
    b = _rand(ops, (n, k), 52)
    ref = a.float() @ b.float().T
    atol, rtol = ops.gemm_tolerance(k)
    c = ops.gemm_bf16(a, b, variant="dma4k_d3")
    assert ((c.float() - ref).abs() <= atol + rtol * ref.abs()).all()
    a8 = ops.fill_uniform_(torch.empty((m, 2 * k), dtype=torch.float8_e4m3fn, device="cuda"), 53)
    b8 = ops.fill_uniform_(torch.empty((n, 2 * k), dtype=torch.float8_e4m3fn, device="cuda"), 54)
    ref8 = a8.float() @ b8.float().T
    atol8, rtol8 = ops.gemm_tolerance(2 * k)
    c8 = ops.gemm_fp8(a8, b8, knob=12)
    assert ((c8.float() - ref8).abs() <= atol8 + rtol8 * ref8.abs()).all()
