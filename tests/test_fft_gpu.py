"""FastFourierTransform.forward/reverse (FastFourierTransform.java:112-164) on the MI355X vs
the oracle's restatement (recurrence twiddles, Bluestein for other lengths) and the
reference's own fixtures (testdata/fft_dc_*, fft_impulse_*; CrossValidationTest.java:120-153).

Bar: under JW_ARITH_FMA the engine uses correctly rounded twiddles, the reference a recurrence
(:188-201); both are compared with an exact DFT (numpy, 1e-12 relative) and with each other at
the tolerance the reference's own FFT tests use (FastFourierTransformTest.java:39-75: 1e-10).
The default JW_ARITH_STRICT transform is bit-exact with the reference for power-of-two lengths
(tests/test_modwt_strict_gpu.py) and is held here to the reference's tolerances.
"""
import numpy as np
import pytest

import oracle as orc
from _util import load_vector
from jwave import FastFourierTransform

pytestmark = pytest.mark.gpu


def rel(a, b):
    return np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300)


@pytest.mark.parametrize("n", [2, 4, 8, 64, 256, 1024, 4096, 8192, 1 << 16, 1 << 18, 1 << 20,
                               3, 5, 6, 7, 12, 100, 1000, 4097, 70001])
def test_forward_reverse_vs_oracle_and_dft(n):
    rng = np.random.default_rng(n)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    f = FastFourierTransform(arith="fma")
    X = f.forwardComplex(z)
    assert rel(X, np.fft.fft(z)) < 1e-12
    assert rel(X, orc.fft(z)) < 1e-10
    zr = f.reverseComplex(X)
    assert rel(zr, np.fft.ifft(X)) < 1e-12  # includes the 1/n
    assert rel(zr, orc.fft(X, inverse=True)) < 1e-10
    assert np.max(np.abs(zr - z)) < 1e-12
    s = FastFourierTransform()  # strict: the reference's arithmetic
    Xs = s.forwardComplex(z)
    assert rel(Xs, orc.fft(z)) < 1e-10 and rel(Xs, np.fft.fft(z)) < 1e-9
    assert np.max(np.abs(s.reverseComplex(Xs) - z)) < 1e-10


def test_edge_lengths():
    f = FastFourierTransform()
    assert f.forwardComplex(np.zeros(0, dtype=complex)).shape == (0,)
    one = np.array([3.0 - 2.0j])
    assert np.array_equal(f.forwardComplex(one), one) and np.array_equal(f.reverseComplex(one), one)


def test_reference_fixtures():
    # CrossValidationTest.java:120-153: DC and impulse, real input through forward(double[])
    f = FastFourierTransform()
    for stem in ("fft_dc", "fft_impulse"):
        x = load_vector(stem + "_input.txt")
        y = f.forward(x)
        assert np.max(np.abs(y[0::2] - load_vector(stem + "_output_real.txt"))) < 1e-10
        assert np.max(np.abs(y[1::2] - load_vector(stem + "_output_imag.txt"))) < 1e-10
        assert np.max(np.abs(f.reverse(y) - x)) < 1e-12


def test_batch_and_device(device):
    import torch
    B, n = 7, 3000
    rng = np.random.default_rng(1)
    z = rng.uniform(-1, 1, (B, n)) + 1j * rng.uniform(-1, 1, (B, n))
    f = FastFourierTransform(arith="fma")
    host = f.forwardComplex(z)
    dev = f.forwardComplex(torch.from_numpy(z).to(device))
    torch.cuda.synchronize()
    for b in range(B):
        assert rel(host[b], np.fft.fft(z[b])) < 1e-12
    assert np.array_equal(dev.cpu().numpy(), host)
    back = f.reverseComplex(dev)
    torch.cuda.synchronize()
    assert np.max(np.abs(back.cpu().numpy() - z)) < 1e-12
