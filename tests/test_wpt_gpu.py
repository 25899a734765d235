"""WaveletPacketTransform on the MI355X vs the oracle (WaveletPacketTransform.java:60-191).
Integer/ordering work plus the same per-packet arithmetic as the FWT: bit-exact in STRICT."""
import numpy as np
import pytest

import oracle as orc
from _util import bits_equal
from jwave import WaveletPacketTransform
from jwave.transforms import wavelets as W
from test_fwt_gpu import CREATE2ARR, wavelet

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wname", CREATE2ARR + ["Haar1Orthogonal", "Legendre1", "Legendre3"])
def test_wpt_bit_exact_all_wavelets(wname):
    wv = wavelet(wname)
    t = WaveletPacketTransform(wv)
    for n, levels in [(2, [1]), (8, [0, 1, 3]), (64, [2, 6]), (1024, [10, 4]), (4096, [12])]:
        x = orc.fill_uniform(n, 5 + n)
        for lvl in levels:
            y = t.forward(x, lvl)
            ref = orc.wpt_forward(x, lvl, wv)
            assert bits_equal(y, ref), (n, lvl)
            assert bits_equal(t.reverse(ref, lvl), orc.wpt_reverse(ref, lvl, wv)), (n, lvl)


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies8", "Symlet8", "Haar1Orthogonal"])
def test_wpt_long_and_generic(wname, knobs):
    # n > 4096 runs the per-level global kernels; JW_FWT_GENERIC forces them for n <= 4096 too
    wv = wavelet(wname)
    t = WaveletPacketTransform(wv)
    for n, lvl in [(16384, 14), (16384, 5), (2048, 11)]:
        x = orc.fill_uniform(n, 9 + n)
        ref = orc.wpt_forward(x, lvl, wv)
        rref = orc.wpt_reverse(ref, lvl, wv)
        assert bits_equal(t.forward(x, lvl), ref)
        assert bits_equal(t.reverse(ref, lvl), rref)
        knobs.setenv("JW_FWT_GENERIC", "1")
        assert bits_equal(t.forward(x, lvl), ref)
        assert bits_equal(t.reverse(ref, lvl), rref)
        knobs.delenv("JW_FWT_GENERIC")


def test_wpt_batch_device_and_2d(device):
    import torch
    wv = W.Daubechies4()
    t = WaveletPacketTransform(wv)
    xs = np.stack([orc.fill_uniform(512, 20 + b) for b in range(5)])
    got = t.forwardBatch(torch.from_numpy(xs).to(device), 9)
    torch.cuda.synchronize()
    for b in range(5):
        assert bits_equal(got[b].cpu().numpy(), orc.wpt_forward(xs[b], 9, wv))
    m = orc.fill_uniform(64 * 32, 4).reshape(64, 32)
    y = t.forward(m, 6, 5)
    rows = np.stack([orc.wpt_forward(r, 5, wv) for r in m])
    ref = np.stack([orc.wpt_forward(c, 6, wv) for c in rows.T]).T
    assert bits_equal(y, ref)
    assert np.max(np.abs(t.reverse(y, 6, 5) - m)) < 1e-10  # db4 taps: ~1e-11 in 2-D
