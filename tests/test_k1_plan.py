"""Host-side K1 dispatch plan (``ntm_k1_plan``, validation/src/ntm_validation.hip):
which rows of C go on the 256x256 kernel and which small tile takes the rest.
No GPU needed - the plan is pure host code in the native library."""
import pytest


@pytest.fixture(scope="module")
def k1_plan():
    from nvidia_terraform_modules_amd.ops import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("native library not built (python -m nvidia_terraform_modules_amd.ops.build)")
    from nvidia_terraform_modules_amd.ops.kernels import k1_plan as f

    return f


@pytest.mark.parametrize("m,n,k,top,rest", [
    (1024, 1024, 1024, 0, "tile128"),          # < 1 round of 256x256 tiles: small tile only
    (2048, 2048, 2048, 0, "tile128"),
    (2560, 2560, 2560, 0, "tile160"),         # 256 tiles of 160x160: one full round
    (1920, 1920, 1920, 0, "tile128"),
    (256, 160, 128, 0, "tile256x160"),
    (4096, 2048, 4096, 0, "tile256x128"),
    (3072, 3072, 3072, 3072, "tile128"),       # whole rounds: 256x256 only
    (4096, 4096, 4096, 4096, "tile128"),
    (8192, 8192, 8192, 8192, "tile128"),
    (6144, 6144, 6144, 5376, "tile256x128"),   # 3 rounds -> 2 + one of 256x128
    (4352, 4352, 4352, 3840, "tile128"),
    (416, 1280, 128, 256, "tile160"),          # split with a 160-row remainder
    (1696, 2560, 256, 1536, "tile160"),
])
def test_plan_matches_cost_model(k1_plan, m, n, k, top, rest):
    assert k1_plan(m, n, k) == (top, rest)


@pytest.mark.parametrize("m,n,k", [(256 * i, 256 * j, 512) for i in range(1, 33, 3)
                                   for j in range(1, 33, 5)])
def test_plan_is_well_formed(k1_plan, m, n, k):
    top, rest = k1_plan(m, n, k)
    assert 0 <= top <= m and top % 256 == 0
    assert rest in ("tile128", "tile256x128", "tile160", "tile256x160")
    if top < m and rest == "tile256x128":
        assert (m - top) % 256 == 0


def test_plan_rejects_bad_args(k1_plan):
    with pytest.raises(Exception):
        k1_plan(0, 256, 256)


@pytest.mark.parametrize("m,n,k", [(384, 256, 192), (100, 256, 256), (256, 256, 64)])
def test_plan_reports_infeasible_shapes(k1_plan, m, n, k):
    """No kernel combination tiles these: the plan says so instead of returning
    a plan whose second launch would fail after the first one wrote C (ADVICE r1:
    (384,256,192) used to launch 256 rows, then fail)."""
    with pytest.raises(ValueError):
        k1_plan(m, n, k)
