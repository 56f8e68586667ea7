"""XgmiAllReduce set-up on the host: the export retry of parallel/xgmi.py's
_alloc_exported, against a fake native library (no GPU)."""
import ctypes

import pytest

from nvidia_terraform_modules_amd.parallel.xgmi import _alloc_exported


class _FakeLib:
    """ntm_malloc hands out increasing addresses; ntm_ipc_handle refuses the
    addresses in ``refuse`` with hipErrorInvalidValue (1)."""

    def __init__(self, refuse):
        self.refuse, self.next = set(refuse), 0x1000

    def ntm_malloc(self, pp, nbytes, uncached):
        ctypes.cast(pp, ctypes.POINTER(ctypes.c_void_p))[0] = self.next
        self.next += 0x1000
        return 0

    def ntm_ipc_handle(self, p, out):
        if p in self.refuse:
            return 1
        out.raw = p.to_bytes(8, "little") + bytes(56)
        return 0


def test_export_first_try():
    own = []
    p, h = _alloc_exported(_FakeLib(()), 64, 0, own)
    assert own == [p] and h[:8] == p.to_bytes(8, "little")


def test_refused_export_keeps_the_range_and_retries_once():
    own = []
    p, h = _alloc_exported(_FakeLib({0x1000}), 64, 0, own)
    assert own == [0x1000, 0x2000] and p == 0x2000     # the refused range stays owned


def test_two_refusals_in_a_row_still_export():
    """Seen at world 8 at the end of round 5: two fresh ranges refused in a row."""
    own = []
    p, h = _alloc_exported(_FakeLib({0x1000, 0x2000}), 64, 0, own)
    assert own == [0x1000, 0x2000, 0x3000] and p == 0x3000


def test_last_refusal_raises_and_everything_stays_owned():
    from nvidia_terraform_modules_amd.parallel.xgmi import EXPORT_ATTEMPTS

    own = []
    refused = {0x1000 * (i + 1) for i in range(EXPORT_ATTEMPTS)}
    with pytest.raises(RuntimeError, match="ntm_ipc_handle failed with hipError 1"):
        _alloc_exported(_FakeLib(refused), 64, 0, own)
    assert sorted(own) == sorted(refused)              # close() frees them all
