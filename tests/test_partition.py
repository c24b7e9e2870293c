"""bench.py's CU reservation for rank 0's fusion stream (host logic, no GPU): mask bit i is CU
i // 8 of XCD i % 8, and a mask that leaves an XCD without CUs is not applied by the runtime, so
the reservation must give every XCD the same number of CUs (test_gpu_kernels.py checks the
placement on the hardware)."""
from collections import Counter

import pytest

from boxfusion_amd import _lib


@pytest.mark.parametrize("reserve,expect", [(32, 32), (20, 24), (8, 8), (1, 8), (64, 64)])
def test_fusion_cus_cover_every_xcd_equally(reserve, expect):
    det, fus = _lib.partition_cus(reserve, n_cu=256)
    assert len(fus) == expect and len(det) == 256 - expect
    assert sorted(det + fus) == list(range(256))
    per_xcd = Counter(c % _lib.XCDS for c in fus)
    assert set(per_xcd) == set(range(_lib.XCDS)) and len(set(per_xcd.values())) == 1
    per_xcd_det = Counter(c % _lib.XCDS for c in det)
    assert len(set(per_xcd_det.values())) == 1


def test_reservation_must_leave_detect_cus():
    with pytest.raises(_lib.HipError):
        _lib.partition_cus(256, n_cu=256)
