"""Non-finite data through the other transforms: the engine against the oracle, STRICT.

JWave multiplies every filter tap in Wavelet.forward / reverse (Wavelet.java:236-303; the
oracle's cascades are pinned to a literal restatement of those loops on non-finite data in
tests/test_oracle_nonfinite.py), every butterfly in FastFourierTransform (:172-212, Bluestein
:259-324), and every in-range term of the direct CWT (ContinuousWaveletTransform.java:240-260).
So +-Inf / NaN samples must come out where, and as, the reference has them: equal NaN-ness and
equal bits everywhere else -- through the LDS cascades, the per-level global kernels, the 2-D
row / column kernels at the cfg4 size, the packet transform, JWave's FFT and the direct CWT.
"""
import math

import numpy as np
import pytest

import oracle as orc
from jwave import ContinuousWaveletTransform as CWT
from jwave import FastFourierTransform, FastWaveletTransform, WaveletPacketTransform
from jwave.transforms import wavelets as W
from jwave.transforms.wavelets.continuous import MexicanHatWavelet, MorletWavelet

pytestmark = pytest.mark.gpu


def same(got, ref):
    got, ref = np.asarray(got).ravel(), np.asarray(ref).ravel()
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), (
        f"NaN-ness differs at {np.argwhere(gn != rn)[:8].ravel().tolist()} "
        f"({int(np.sum(gn != rn))} positions)")
    assert np.array_equal(got[~gn].view(np.uint64), ref[~rn].view(np.uint64))


def poison(x, spots):
    y = np.array(x, dtype=np.float64, copy=True)
    for idx, v in spots:
        y[idx] = v
    return y


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "Haar1Orthogonal"])
@pytest.mark.parametrize("n", [64, 4096, 16384])
def test_fwt_1d_nonfinite(wname, n):
    wv = W.Haar1Orthogonal() if wname == "Haar1Orthogonal" else W.by_name(wname)
    f = FastWaveletTransform(wv)
    x = poison(orc.fill_uniform(n, 21), [(0, math.inf), (n // 3, math.nan), (n - 1, -math.inf)])
    lvl = n.bit_length() - 1
    for level in (2, lvl):
        same(f.forward(x, level), orc.fwt_forward(x, level, wv))
        same(f.reverse(x, level), orc.fwt_reverse(x, level, wv))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies8"])
@pytest.mark.parametrize("n", [256, 4096, 16384])
def test_wpt_nonfinite(wname, n):
    wv = W.by_name(wname)
    t = WaveletPacketTransform(wv)
    x = poison(orc.fill_uniform(n, 22), [(5, math.inf), (n // 2 + 3, -math.inf), (n - 2, math.nan)])
    lvl = n.bit_length() - 1
    for level in (3, lvl):
        same(t.forward(x, level), orc.wpt_forward(x, level, wv))
        same(t.reverse(x, level), orc.wpt_reverse(x, level, wv))


@pytest.mark.parametrize("shape", [(64, 64), (256, 512), (4096, 4096)])
def test_fwt_2d_nonfinite(shape):
    # 4096 x 4096 is cfg4's geometry: the 4096-sample row kernels and the column stream / tail
    wv = W.Daubechies8()
    f = FastWaveletTransform(wv)
    R, C = shape
    x = orc.fill_uniform(R * C, 23).reshape(R, C)
    x = poison(x, [((0, 0), math.inf), ((R // 2, C - 1), math.nan), ((R - 1, C // 3), -math.inf)])
    lM, lN = R.bit_length() - 1, C.bit_length() - 1
    same(f.forward(x, lM, lN), orc.fwt2d_forward(x, lM, lN, wv))
    same(f.reverse(x, lM, lN), orc.fwt2d_reverse(x, lM, lN, wv))


@pytest.mark.parametrize("n", [8, 1024, 1 << 16, 1 << 20, 1000, 4097])
def test_jwave_fft_nonfinite(n):
    z = orc.fill_uniform(n, 24) + 1j * orc.fill_uniform(n, 25)
    z[n // 2] = complex(math.inf, 0.0)
    z[1] = complex(0.0, math.nan)
    s = FastFourierTransform()  # STRICT: the reference's own FFT
    with np.errstate(invalid="ignore", over="ignore"):
        X = s.forwardComplex(z)
        ref = orc.fft(z)
        same(X.real, ref.real)
        same(X.imag, ref.imag)
        Xr = s.reverseComplex(ref)
        rr = orc.fft(ref, inverse=True)
    same(Xr.real, rr.real)
    same(Xr.imag, rr.imag)


@pytest.mark.parametrize("wv,kind", [(MorletWavelet(1.0, 6.0 / (2 * math.pi)), "morlet"),
                                     (MexicanHatWavelet(1.0), "mexhat")])
def test_cwt_direct_nonfinite(wv, kind):
    n = 600
    x = poison(orc.fill_uniform(n, 26), [(10, math.inf), (300, math.nan)])
    scales = [0.5, 2.0, 16.0, 64.0]
    got = CWT(wv).transform(x, scales, 1.0).getCoefficients()
    ref = orc.cwt_direct(x, kind, wv.params(), scales, 1.0)
    same(got.real, ref.real)
    same(got.imag, ref.imag)
