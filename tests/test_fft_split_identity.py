"""The last-stage identity the long STRICT FFT tests lean on, pinned on the oracle (CPU only).

fftCooleyTukey (FastFourierTransform.java:172-212) bit-reverses, then runs the stages of size
2, 4, .., n; every block of a stage uses the twiddles wn_k of that size (:188-201: angle
2 pi / size, the recurrence wn = wn.mul(w) from (1, 0)), whatever n.  After the stages up to
n / 2 the first half of the array therefore holds the n/2-point transform of the even samples
and the second half that of the odd ones, and the last stage makes
    X[k] = E[k] + t,  X[k + n/2] = E[k] - t,  t = wn_k.mul(O[k])  (Complex.mul :286-288)
bit for bit.  reverse() scales by 1.0 / n at the end (:207-211), a power of two: exact.
tests/test_jfft_limits_gpu.py checks the engine's 2^28 .. 2^30 transforms this way, where the
oracle itself would take minutes; here the identity is checked against the oracle's own
transforms.
"""
import numpy as np
import pytest

import oracle as orc


def last_stage(E, O, w):
    """Java's last butterfly stage in its operation order (numpy: every op rounded on its own)."""
    tr = w.real * O.real - w.imag * O.imag
    ti = w.real * O.imag + w.imag * O.real
    X = np.empty(2 * E.shape[0], dtype=np.complex128)
    h = E.shape[0]
    X.real[:h], X.imag[:h] = E.real + tr, E.imag + ti
    X.real[h:], X.imag[h:] = E.real - tr, E.imag - ti
    return X


@pytest.mark.parametrize("n", [2, 4, 64, 1024, 1 << 16])
@pytest.mark.parametrize("inverse", [False, True])
def test_last_stage_identity(n, inverse):
    rng = np.random.default_rng(n + inverse)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    X = orc.fft(z, inverse=inverse)
    E, O = orc.fft(z[0::2], inverse=inverse), orc.fft(z[1::2], inverse=inverse)
    w = orc.fft_stage_twiddles(n, inverse)
    assert w.shape == (n // 2,) and w[0] == 1
    if inverse:  # undo the halves' 1 / (n/2), redo the whole one's 1 / n: powers of two
        ref = last_stage(E * (n // 2), O * (n // 2), w) * (1.0 / n)
    else:
        ref = last_stage(E, O, w)
    assert np.array_equal(X.view(np.uint64), ref.view(np.uint64))


def test_stage_twiddles_independent_of_n():
    # the size-1024 stage's twiddles are the same in a 1024- and a 4096-point transform: the
    # impulse at index 1 of a 1024-point transform returns them (E = 0, O = 1 exactly)
    w = orc.fft_stage_twiddles(1024)
    d = np.zeros(1024, dtype=np.complex128)
    d[1] = 1.0
    X = orc.fft(d)
    assert np.array_equal(X[:512].view(np.uint64), w.view(np.uint64))
