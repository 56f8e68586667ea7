"""CPU model of the LDS-DMA schedule of the 8-wave ping-pong K1 kernels
(gemm_bf16_pp3.hpp "pingpong8c", and gemm_bf16_pp3h.hpp's 192x256 / 256x192 /
224x256 builds whose 64-row halves take one DMA piece per lane instead of two).

One wave's program is replayed exactly as the kernel issues it: the 7-issue
prologue, then per phase P of K-tile t the fragment reads, the issue of one
half (P0 A-hi(t+1), P1 B-lo(t+2), P2 A-lo(t+2), P3 B-hi(t+2); K-tiles >= T are
dummy pieces into the scratch region) and the counted ``s_waitcnt vmcnt`` that
the native library reports for that build (``ntm_pp3h_vmcnt``, the kernel's own
``Geo::vmc``). Loads retire in issue order, so after ``vmcnt(N)`` every piece but
the newest N has landed. Checked for every build and K-tile count:

* RAW: every half a phase reads was retired by the wait of an earlier phase
  (that wait precedes the barrier the partner wave group also passes);
* no drain: each wait leaves exactly the pieces of the 5 newest issues in
  flight, the deepest wait the RAW rule allows;
* WAR: a slot is re-staged at least 2 phases after its last fragment read
  (1.5 for the prologue's read of B-lo(0));
* every dummy piece targets the scratch region, and the K loop ends with
  vmcnt(0) before the epilogue reuses the LDS.
"""
import pytest

ALO, AHI, BLO, BHI = "A-lo", "A-hi", "B-lo", "B-hi"


@pytest.fixture(scope="module")
def vmcnt():
    from nvidia_terraform_modules_amd.ops import _lib

    if not _lib.LIB_PATH.exists():
        pytest.skip("native library not built (python -m nvidia_terraform_modules_amd.ops.build)")
    return lambda ah, bh, p: _lib.lib().ntm_pp3h_vmcnt(ah, bh, p)


def _pieces(ah, bh):
    # a 64-row half is one 16-B piece per lane; 96 and 128 rows are two
    return {ALO: 2, BLO: 2, AHI: 1 if ah == 64 else 2, BHI: 1 if bh == 64 else 2}


def replay(ah, bh, T, vm):
    """Events of one wave: returns (issues, waits, reads) where issues are
    (phase, half, ktile, first_piece, n_pieces, dummy), waits (phase,
    issued_pieces_so_far, N) and reads (phase, half, ktile)."""
    n = _pieces(ah, bh)
    issues, waits, reads = [], [], []
    count = 0

    def issue(ph, h, kt):
        nonlocal count
        issues.append((ph, h, kt, count, n[h], kt >= T))
        count += n[h]

    # prologue: virtual phases -7..-1, then the wait of phase -1 (a B-hi issue: P3)
    for i, (h, kt) in enumerate([(BLO, 0), (ALO, 0), (BHI, 0), (AHI, 0), (BLO, 1), (ALO, 1),
                                 (BHI, 1)]):
        issue(-7 + i, h, kt)
    waits.append((-1, count, vm(ah, bh, 3)))
    reads.append((-0.5, BLO, 0))   # after the prologue wait and barrier
    for t in range(T):
        for p in range(4):
            ph = 4 * t + p
            if p == 0:
                reads.append((ph, ALO, t))
                issue(ph, AHI, t + 1)
            elif p == 1:
                reads.append((ph, BHI, t))
                issue(ph, BLO, t + 2)
            elif p == 2:
                reads.append((ph, AHI, t))
                issue(ph, ALO, t + 2)
            else:
                if t + 1 < T:
                    reads.append((ph, BLO, t + 1))
                issue(ph, BHI, t + 2)
            waits.append((ph, count, vm(ah, bh, p)))
    waits.append((4 * T, count, 0))   # wait_vmcnt<0> before the epilogue
    return issues, waits, reads


BUILDS = [(128, 128), (64, 128), (128, 64), (96, 128)]


@pytest.mark.parametrize("ah,bh", BUILDS)
@pytest.mark.parametrize("T", [2, 4, 6, 10, 36])
def test_raw_every_read_was_retired(vmcnt, ah, bh, T):
    issues, waits, reads = replay(ah, bh, T, vmcnt)
    last_piece = {(h, kt): first + np - 1 for _, h, kt, first, np, dummy in issues if not dummy}
    for ph, h, kt in reads:
        # the newest wait before this read's phase (the kernel reads first, then waits)
        w = [x for x in waits if x[0] < ph]
        assert w, (ph, h, kt)
        _, issued, nleft = w[-1]
        retired = issued - nleft
        assert last_piece[(h, kt)] < retired, (ah, bh, T, ph, h, kt)


@pytest.mark.parametrize("ah,bh", BUILDS)
def test_waits_keep_the_5_newest_issues_in_flight(vmcnt, ah, bh):
    issues, waits, _ = replay(ah, bh, 12, vmcnt)
    for ph, issued, nleft in waits[:-1]:
        newest = [x for x in issues if x[0] <= ph][-5:]
        assert nleft == sum(x[4] for x in newest), (ah, bh, ph)
    if (ah, bh) == (128, 128):
        assert {vmcnt(ah, bh, p) for p in range(4)} == {10}   # pingpong8c's vmcnt(10)


@pytest.mark.parametrize("ah,bh", BUILDS)
@pytest.mark.parametrize("T", [2, 4, 10])
def test_war_and_dummy_pieces(vmcnt, ah, bh, T):
    issues, waits, reads = replay(ah, bh, T, vmcnt)
    last_read = {}
    for ph, h, kt in reads:
        last_read[(h, kt)] = max(ph, last_read.get((h, kt), ph))
    for ph, h, kt, _, _, dummy in issues:
        if dummy:
            assert kt >= T
            continue
        prev = (h, kt - 2)             # the occupant of the same buffer slot (kt & 1)
        if prev in last_read:
            # 2 phases (4 barriers) in the loop; the prologue's B-lo(0) fragment read,
            # made after the prologue barrier, sits 1.5 phases (3 barriers) before
            # B-lo(2)'s issue - still behind a full phase of MFMAs, while the DMA's
            # own L2 round trip is longer than an LDS read
            need = 1.5 if last_read[prev] < 0 else 2
            assert ph >= last_read[prev] + need, (ah, bh, T, h, kt, ph, last_read[prev])
    # every real K-tile's four halves are read, and nothing is issued for them twice
    real = [(h, kt) for _, h, kt, _, _, dummy in issues if not dummy]
    assert len(real) == len(set(real)) == 4 * T
    assert waits[-1][2] == 0


def test_unsupported_builds_are_refused(vmcnt):
    assert vmcnt(32, 128, 0) == -1 and vmcnt(64, 96, 0) == -1 and vmcnt(64, 128, 4) == -1
