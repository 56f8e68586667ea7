"""Exhaustive interleaving model of stream-K's wait-free fix-up protocols
(validation/include/ntm/gemm_bf16_sk.hpp), on the CPU.

Each part of a split tile is a small program of atomic steps on the tile's
counter word (fetch-add returning the old value) and on its partial slot; the
model runs EVERY interleaving of the parts' steps and checks what the kernels
rely on:

* exactly one part combines, and it adds the other parts' partials only after
  they were written (the release is the writer's drain + counter add);
* the combiner leaves the counter at 0 (the next launch reuses the workspace
  without a memset);
* the XCC tags decoded from the counter equal the parts' XCDs, so a part placed
  on another XCD is always reported, and never a false alarm.

Protocols: the head / tail pair (two-round mode, and split mode at S = 2 since
round 5) and the S-slice protocol (split mode, S >= 3).
"""
import itertools
import random

import pytest

HEAD_TAG_SHIFT, TAIL_TAG_SHIFT = 8, 16


def _pair_programs(writer_is_head: bool, xcc_head: int, xcc_tail: int):
    """Steps of the head / tail protocol; each step is a generator stage that
    reads / updates the shared state dict and yields between atomics."""

    def part(tail: bool):
        def run(st):
            xc = xcc_tail if tail else xcc_head
            arrive = 4 if tail else 1
            written = arrive << 1
            other_written = 2 if tail else 8
            tag = (xc + 1) << (TAIL_TAG_SHIFT if tail else HEAD_TAG_SHIFT)
            writer = (not tail) if writer_is_head else tail
            if writer:
                o = 0
            else:
                o = st["cnt"]
                st["cnt"] += arrive + tag          # atomic fetch-add
                yield
            if not (o & other_written):
                st["partial"][tail] = True         # write-through partial (drained)
                yield
                o = st["cnt"]
                st["cnt"] += written + (tag if writer else 0)
                yield
            if o & other_written:
                other_xcc = ((o >> (HEAD_TAG_SHIFT if tail else TAIL_TAG_SHIFT)) & 0xFF) - 1
                st["combines"].append(("tail" if tail else "head", other_xcc, xc))
                assert st["partial"][not tail], "combined before the other partial was written"
                st["cnt"] = 0                      # reset
                yield
        return run

    return [part(False), part(True)]


def _slice_programs(S: int, xccs):
    def part(q):
        def run(st):
            xc = xccs[q]
            tag = 1 + (xc << 8) + ((xc * xc) << 16)
            st["partial"][q] = True
            yield
            o = st["cnt"]
            st["cnt"] += tag
            yield
            if (o & 0xFF) == S - 1:
                total = o + tag
                ok = ((total >> 8) & 0xFF) == S * xc and (total >> 16) == S * xc * xc
                st["combines"].append((q, ok))
                assert all(st["partial"]), "combined before every partial was written"
                st["cnt"] = 0
                yield
        return run

    return [part(q) for q in range(S)]


def _run(programs, state_factory, chooser):
    st = state_factory()
    gens = [p(st) for p in programs]
    alive = list(range(len(programs)))
    while alive:
        i = chooser(alive)
        if i is None:
            return None, list(alive)               # an unexplored decision point
        try:
            next(gens[i])
        except StopIteration:
            alive.remove(i)
    return st, None


def _interleavings(programs, state_factory, limit=None, rng=None):
    """Final states of EVERY interleaving of the programs' atomic steps (or of
    `limit` random ones)."""
    if limit is not None:
        return [_run(programs, state_factory, lambda alive: rng.choice(alive))[0]
                for _ in range(limit)]
    done = []

    def explore(prefix):
        it = iter(prefix)

        def chooser(alive):
            if len(alive) == 1:
                return alive[0]
            return next(it, None)

        st, branch = _run(programs, state_factory, chooser)
        if st is not None:
            done.append(st)
            return
        for c in branch:
            explore(prefix + [c])

    explore([])
    return done


@pytest.mark.parametrize("writer_is_head", [True, False])
@pytest.mark.parametrize("xcc_head,xcc_tail", [(3, 3), (0, 0), (7, 7), (2, 5), (0, 1)])
def test_pair_protocol_every_interleaving(writer_is_head, xcc_head, xcc_tail):
    progs = _pair_programs(writer_is_head, xcc_head, xcc_tail)
    runs = _interleavings(progs, lambda: {"cnt": 0, "partial": {False: False, True: False},
                                          "combines": []})
    assert len(runs) >= 3
    for st in runs:
        assert len(st["combines"]) == 1, st          # exactly one combiner
        assert st["cnt"] == 0                         # workspace reusable
        who, other_xcc, mine = st["combines"][0]
        assert other_xcc == (xcc_tail if who == "head" else xcc_head)
        assert (other_xcc != mine) == (xcc_head != xcc_tail)   # mismatch <=> reported


@pytest.mark.parametrize("S", [3, 4, 8])
@pytest.mark.parametrize("placement", ["same", "one_off"])
def test_slice_protocol_random_interleavings(S, placement):
    rng = random.Random(S * 31 + len(placement))
    for xc in (0, 5, 15):
        xccs = [xc] * S
        if placement == "one_off":
            xccs[rng.randrange(S)] = (xc + 1) % 16
        progs = _slice_programs(S, xccs)
        runs = _interleavings(progs, lambda: {"cnt": 0, "partial": [False] * S, "combines": []},
                              limit=300, rng=rng)
        for st in runs:
            assert len(st["combines"]) == 1 and st["cnt"] == 0
            _, ok = st["combines"][0]
            assert ok == (placement == "same")   # whichever part combines


def test_slice_tags_detect_every_single_misplacement():
    """Sum and sum of squares agree with S * x and S * x^2 only when every part
    ran on x: checked for every S <= 8, every combiner XCC and every single
    other part's XCC (the arithmetic, without interleavings)."""
    for S in range(3, 9):
        for x in range(16):
            for y in range(16):
                xccs = [x] * (S - 1) + [y]
                total = sum(1 + (c << 8) + ((c * c) << 16) for c in xccs)
                ok = ((total >> 8) & 0xFF) == S * x and (total >> 16) == S * x * x
                assert ok == (x == y), (S, x, y)
                assert (total & 0xFF) == S


def test_pair_tags_fit_their_fields():
    for a, b in itertools.product(range(16), repeat=2):
        cnt = 1 + 2 + 4 + 8 + ((a + 1) << HEAD_TAG_SHIFT) + ((b + 1) << TAIL_TAG_SHIFT)
        assert ((cnt >> HEAD_TAG_SHIFT) & 0xFF) - 1 == a
        assert ((cnt >> TAIL_TAG_SHIFT) & 0xFF) - 1 == b
        assert cnt & 0xF == 0xF
