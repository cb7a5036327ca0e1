"""GPU: the box bandwidth probes bench.py reports next to every roofline
(crdt_bw_probe).  Not a merge: checked for plausible rates and, for the copy,
that the bytes really moved."""

import pytest

import crdtgpu
from crdtgpu import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need a HIP device"
    return t


def test_probes_rates_and_copy(torch):
    eng = crdtgpu.Engine(0)
    try:
        n = 1 << 30
        a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda:0")
        b = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
        r = eng.bw_probe(abi.CRDT_PROBE_READ, a, b, n, 5)
        w = eng.bw_probe(abi.CRDT_PROBE_WRITE, None, b, n, 5)
        c = eng.bw_probe(abi.CRDT_PROBE_COPY, a, b, n, 5)
        for g in (r, w, c):
            assert 500.0 < g < 12000.0, (r, w, c)  # HBM3E: well under the 8 TB/s spec + cache effects
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        mhz = eng.clock_probe()
        assert 500.0 < mhz < 3000.0, mhz  # MI355X: up to 2400 MHz
        with pytest.raises(crdtgpu.CrdtError):
            eng.bw_probe(7, a, b, n, 1)
        with pytest.raises(crdtgpu.CrdtError):
            eng.bw_probe(abi.CRDT_PROBE_COPY, a, b, 8, 1)
    finally:
        eng.close()
