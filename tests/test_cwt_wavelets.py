"""Paul / DOG / Meyer continuous wavelets: host API and the oracle's Fourier transforms.

Restates the reference's own unit tests (src/test/java/jwave/transforms/wavelets/continuous/
{Paul,DOG,Meyer}WaveletTest.java) on the host mirror, and pins the oracle's psi_hat
(jwo_cwt_wavelet_ft_c, which the GPU parity tests check against) to the host closed forms.
"""
import math

import numpy as np
import pytest

import oracle as orc
from jwave.exceptions import IllegalArgumentException
from jwave.transforms.wavelets.continuous import (DOGWavelet, MeyerWavelet, MexicanHatWavelet,
                                                   MorletWavelet, PaulWavelet)

DELTA = 1e-10


# ---------------------------------------------------------------- Paul (PaulWaveletTest.java)
def test_paul_construction_and_messages():
    assert PaulWavelet().getOrder() == 4 and PaulWavelet(6).getOrder() == 6
    assert PaulWavelet().getName() == "Paul"
    with pytest.raises(IllegalArgumentException, match="positive integer"):
        PaulWavelet(0)
    with pytest.raises(IllegalArgumentException, match="numerical issues"):
        PaulWavelet(21)
    assert PaulWavelet(4).getCenterFrequency() == pytest.approx(4.5 / (2 * math.pi))


def test_paul_time_domain():
    p = PaulWavelet(4)
    v0 = complex(p.wavelet(0.0))
    assert abs(v0.imag) < DELTA and v0.real > 0           # :79-80
    assert abs(complex(p.wavelet(1.0)).imag) > DELTA      # complex-valued
    assert abs(complex(p.wavelet(20.0))) < 0.01           # decays
    for m in range(1, 9):                                 # i^m carried through
        assert abs(complex(PaulWavelet(m).wavelet(0.5))) > 0


def test_paul_fourier_transform():
    p = PaulWavelet(4)
    assert abs(complex(p.fourierTransform(-1.0))) < DELTA  # analytic: no negative frequencies
    pos = complex(p.fourierTransform(2.0))
    assert abs(pos) > 0 and abs(pos.imag) < DELTA
    om = np.linspace(0.01, 20, 4000)
    assert abs(om[np.argmax(np.abs(p.fourierTransform(om)))] - 4.0) < 0.5  # peak near m


def test_paul_aux():
    assert PaulWavelet(2).getAdmissibilityConstant() == pytest.approx(2 * math.pi / 5)
    assert PaulWavelet(4).getAdmissibilityConstant() == pytest.approx(2 * math.pi / 9)
    assert PaulWavelet(4).getEffectiveSupport() == [-1.0, 10.0]
    bw = PaulWavelet(4).getBandwidth()
    assert bw[0] == 0.0 and bw[1] == pytest.approx(10 / (2 * math.pi))
    assert PaulWavelet.fromResolutionBalance(1).getOrder() == 2
    assert PaulWavelet.fromResolutionBalance(10).getOrder() == 20
    assert 10 <= PaulWavelet.fromResolutionBalance(5.5).getOrder() <= 12
    with pytest.raises(IllegalArgumentException, match="between 1 and 10"):
        PaulWavelet.fromResolutionBalance(0.5)


# ---------------------------------------------------------------- DOG (DOGWaveletTest.java)
def test_dog_construction_and_messages():
    d = DOGWavelet()
    assert d.getDerivativeOrder() == 2 and d.getSigma() == 1.0 and d.isMexicanHat()
    assert DOGWavelet(3).getSigma() == 1.0 and DOGWavelet(4, 2.0).getSigma() == 2.0
    assert DOGWavelet(3).getName() == "DOG (n=3)"
    with pytest.raises(IllegalArgumentException, match="positive integer"):
        DOGWavelet(0)
    with pytest.raises(IllegalArgumentException, match="numerical issues"):
        DOGWavelet(11)
    with pytest.raises(IllegalArgumentException, match="positive"):
        DOGWavelet(2, -1.0)
    T = DOGWavelet.WaveletType
    assert [DOGWavelet.createStandard(t, 1.0).getDerivativeOrder()
            for t in (T.EDGE, T.MEXICAN_HAT, T.RICKER, T.ZERO_CROSSING, T.RIDGE)] == [1, 2, 2, 3, 4]
    with pytest.raises(IllegalArgumentException, match="cannot be null"):
        DOGWavelet.createStandard(None, 1.0)
    assert DOGWavelet(1).getCenterFrequency() == pytest.approx(1 / (2 * math.pi))
    assert DOGWavelet(4, 2.0).getCenterFrequency() == pytest.approx(2 / (4 * math.pi))


def test_dog_symmetries():
    t = np.array([0.5, 1.0, 1.7])
    for n in (1, 2, 3, 4):
        d = DOGWavelet(n)
        a, b = d.wavelet(t).real, d.wavelet(-t).real
        assert np.allclose(a, b if n % 2 == 0 else -b, atol=1e-12)
        if n % 2:
            assert abs(complex(d.wavelet(0.0))) < 1e-12
        else:
            assert abs(complex(d.wavelet(0.0))) > DELTA
    assert complex(DOGWavelet(1).wavelet(1.0)).real > 0
    assert complex(DOGWavelet(2).wavelet(0.0)).real > 0
    # Hermite recurrence: H_3 = 8x^3 - 12x, sign (-1)^(n+1) = +1
    assert DOGWavelet(3)._hermiteCoeffs == [0.0, -12.0, 0.0, 8.0]


def test_dog_fourier_transform():
    for n in (1, 2, 3, 4):
        d = DOGWavelet(n)
        assert abs(complex(d.fourierTransform(0.0))) < DELTA
        assert abs(complex(d.fourierTransform(1.5))) > 0
        p, m = complex(d.fourierTransform(1.5)), complex(d.fourierTransform(-1.5))
        if n % 2 == 0:
            assert p == pytest.approx(m) and p.imag == 0
        else:
            assert p.real == 0 and p.imag == pytest.approx(-m.imag)
    # DOG(2) and the Mexican hat share the sign pattern at the reference's points (:222-233)
    t = np.array([0.0, 0.5, 1.0, 1.5, 2.0])
    a, b = DOGWavelet(2).wavelet(t).real, MexicanHatWavelet().wavelet(t).real
    both = (np.abs(a) > DELTA) & (np.abs(b) > DELTA)
    assert np.all(np.sign(a[both]) == np.sign(b[both]))


def test_dog_aux():
    assert DOGWavelet(2).getEffectiveSupport() == [-4.0, 4.0]
    assert DOGWavelet(4, 2.0).getEffectiveSupport() == [-10.0, 10.0]
    assert DOGWavelet(4).getBandwidth()[1] > DOGWavelet(1).getBandwidth()[1]
    x = np.linspace(-20, 20, 40001)
    norm = math.sqrt(np.sum(np.abs(DOGWavelet(2).wavelet(x)) ** 2) * (x[1] - x[0]))
    assert 0.1 < norm < 10.0


# ---------------------------------------------------------------- Meyer (MeyerWaveletTest.java)
def test_meyer_basics():
    m = MeyerWavelet()
    assert m.getName() == "Meyer" and m.getCenterFrequency() == pytest.approx(0.7 / (2 * math.pi))
    t = np.array([-3.0, -1.0, 0.0, 0.5, 2.0])
    assert np.all(m.wavelet(t).imag == 0)
    assert np.allclose(m.wavelet(t).real, m.wavelet(-t).real)
    assert abs(complex(m.wavelet(0.0))) > abs(complex(m.wavelet(5.0))) > abs(complex(m.wavelet(14.0)))
    assert complex(m.wavelet(20.0)) == 0 and complex(m.wavelet(15.0 + 1e-9)) == 0
    assert abs(complex(m.wavelet(15.0))) > 0
    assert m.getEffectiveSupport() == [-15.0, 15.0]
    bw = m.getBandwidth()
    assert bw[0] == pytest.approx(2 / 3 / (2 * math.pi)) and bw[1] == pytest.approx(8 / 3 / (2 * math.pi))
    assert m.getAdmissibilityConstant() == pytest.approx(2 * math.pi)


def test_meyer_fourier_transform():
    m = MeyerWavelet()
    lo, mid, hi = 2 * math.pi / 3, 4 * math.pi / 3, 8 * math.pi / 3
    assert complex(m.fourierTransform(lo * 0.99)) == 0 and complex(m.fourierTransform(hi * 1.01)) == 0
    assert abs(complex(m.fourierTransform(lo * 1.2))) > 0 and abs(complex(m.fourierTransform(mid * 1.2))) > 0
    # the two branches meet continuously at 4 pi / 3
    a, b = abs(complex(m.fourierTransform(mid - 1e-9))), abs(complex(m.fourierTransform(mid + 1e-9)))
    assert abs(a - b) < 1e-6
    om = np.linspace(0.1, 10, 999)
    f, g = m.fourierTransform(om), m.fourierTransform(-om)
    assert np.allclose(f.real, g.real) and np.allclose(f.imag, -g.imag)
    assert 0 < np.max(np.abs(f)) < 10


# ---------------------------------------------------------------- oracle psi_hat == host
WAVELETS = [
    (MorletWavelet(1.0, 6 / (2 * math.pi)), "morlet", (1.0, 6 / (2 * math.pi))),
    (MexicanHatWavelet(1.5), "mexhat", (1.5,)),
    (PaulWavelet(1), "paul", (1.0,)), (PaulWavelet(4), "paul", (4.0,)),
    (PaulWavelet(20), "paul", (20.0,)),
    (DOGWavelet(1, 2.0), "dog", (1.0, 2.0)), (DOGWavelet(2), "dog", (2.0, 1.0)),
    (DOGWavelet(3, 0.5), "dog", (3.0, 0.5)), (DOGWavelet(4), "dog", (4.0, 1.0)),
    (DOGWavelet(10), "dog", (10.0, 1.0)),
    (MeyerWavelet(), "meyer", ()),
]


@pytest.mark.parametrize("wv,kind,params", WAVELETS, ids=lambda v: str(v)[:12])
def test_oracle_psi_hat_matches_host(wv, kind, params):
    om = np.concatenate([np.linspace(-7, 7, 57), [0.0, 2 * math.pi / 3, 4 * math.pi / 3]])
    for a in (0.3, 1.0, 2.5, 17.0):
        host = wv.fourierTransform(om, a)
        orac = np.array([orc.cwt_wavelet_ft(kind, params, o, a) for o in om])
        scale = max(np.max(np.abs(host)), 1e-300)
        assert np.max(np.abs(host - orac)) / scale < 1e-14, (kind, a)
