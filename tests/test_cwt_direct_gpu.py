"""Direct CWT on the GPU (jw_cwt_direct) against the oracle's restatement of
ContinuousWaveletTransform.transform (ContinuousWaveletTransform.java:153-172,
computeCoefficient :240-260).  The wavelet tables are evaluated on the host with the
reference's operation order and the kernel adds the terms in the reference's order, so STRICT
is bit-identical to the oracle (same libm on both sides); FMA is held to the north_star's
1e-10 relative.  The reference's own CWT tests only check the direct path qualitatively (FFT vs
direct mean |d| < 0.1, ContinuousWaveletTransformTest.java:170-208), restated below."""
import math

import numpy as np
import pytest

import oracle as orc
from _util import bits_equal
from jwave import ContinuousWaveletTransform as CWT
from jwave.transforms.wavelets.continuous import (DOGWavelet, MeyerWavelet, MexicanHatWavelet,
                                                   MorletWavelet, PaulWavelet)

pytestmark = pytest.mark.gpu

WAVELETS = [
    (MorletWavelet(1.0, 6.0 / (2 * math.pi)), "morlet"),
    (MorletWavelet(2.0, 0.5), "morlet"),
    (MexicanHatWavelet(1.0), "mexhat"),
    (MexicanHatWavelet(0.6), "mexhat"),
    (PaulWavelet(4), "paul"),
    (PaulWavelet(1), "paul"),
    (DOGWavelet(2, 1.0), "dog"),
    (DOGWavelet(5, 0.8), "dog"),
    (MeyerWavelet(), "meyer"),
]


@pytest.mark.parametrize("wv,kind", WAVELETS, ids=lambda v: str(v)[-12:])
@pytest.mark.parametrize("n,fs", [(1, 1.0), (7, 1.0), (300, 1.0), (1000, 2.5)])
def test_direct_bit_exact(wv, kind, n, fs):
    x = orc.fill_uniform(n, 13 + n)
    scales = [0.5, 1.0, 2.0, 3.7, 16.0, 64.0]
    got = CWT(wv).transform(x, scales, fs).getCoefficients()
    ref = orc.cwt_direct(x, kind, wv.params(), scales, fs)
    assert got.shape == (len(scales), n)
    assert bits_equal(got.real, ref.real) and bits_equal(got.imag, ref.imag)
    fm = CWT(wv).transform(x, scales, fs, arith="fma").getCoefficients()
    assert np.max(np.abs(fm - ref)) <= 1e-10 * max(np.max(np.abs(ref)), 1e-300)


def test_direct_negative_scale_gives_zeros_and_batch():
    wv = MorletWavelet(1.0, 1.0)
    xs = np.stack([orc.fill_uniform(257, 5 + b) for b in range(3)])
    scales = [-3.0, 2.0, 40.0]
    got = CWT(wv).transformBatch(xs, scales)
    assert np.all(got[:, 0] == 0)
    for b in range(3):
        ref = orc.cwt_direct(xs[b], "morlet", wv.params(), scales)
        assert bits_equal(got[b].real, ref.real) and bits_equal(got[b].imag, ref.imag)


def test_direct_device_tensors(device):
    import torch
    wv = MexicanHatWavelet(1.0)
    xs = np.stack([orc.fill_uniform(2048, 9 + b) for b in range(2)])
    scales = CWT.generateLogScales(1.0, 100.0, 8)
    host = CWT(wv).transformBatch(xs, scales)
    dev = CWT(wv).transformBatch(torch.from_numpy(xs).to(device), scales)
    torch.cuda.synchronize()
    assert dev.is_cuda and np.array_equal(host, dev.cpu().numpy())


def test_cwt_fft_vs_direct_reference_case():
    # ContinuousWaveletTransformTest.testCWTFFT (:170-208): fs = 100, 64 samples of
    # sin(2 pi 5 t) + 0.5 sin(2 pi 15 t), Morlet(1, 1), 20 log scales 0.5..5: the mean
    # |magnitude difference| of direct and FFT over all coefficients is < 0.1
    fs, n = 100.0, 64
    x = np.array([math.sin(2.0 * math.pi * 5.0 * (i / fs)) + 0.5 * math.sin(2.0 * math.pi * 15.0 * (i / fs))
                  for i in range(n)])
    cwt = CWT(MorletWavelet(1.0, 1.0))
    scales = CWT.generateLogScales(0.5, 5.0, 20)
    d = cwt.transform(x, scales, fs)
    f = cwt.transformFFT(x, scales, fs)
    assert np.mean(np.abs(d.getMagnitude() - f.getMagnitude())) < 0.1
    ref = orc.cwt_direct(x, "morlet", (1.0, 1.0), scales, fs)
    assert bits_equal(d.getCoefficients().real, ref.real)
    assert bits_equal(d.getCoefficients().imag, ref.imag)
