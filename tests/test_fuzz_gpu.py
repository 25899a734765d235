"""Seeded random sweep over the engine's parameter space, each case against the oracle.

The other GPU tests pin chosen shapes; this one draws (wavelet, length, levels, batch,
convolution method, arithmetic contract, 2-D / 3-D geometry) at random from fixed seeds, so
combinations nobody picked by hand get checked too.  Case k draws from default_rng(7000 + k):
a failure names its case and reproduces alone.  Bars as everywhere else: STRICT bit for bit
(MODWT DIRECT / FFT / AUTO against the oracle's faithful restatements of MODWTTransform.java
:256-375,640-837; FWT / WPT / 2-D / 3-D against Wavelet.java:236-303 and the transform
cascades; JWave's FFT against FastFourierTransform.java:112-324); FMA within 1e-10 normwise
of the oracle's DIRECT path.  Sizes keep each oracle call well under a second.
"""
import numpy as np
import pytest

import oracle as orc
from _util import bits_equal
from jwave import FastFourierTransform, FastWaveletTransform, MODWTTransform, WaveletPacketTransform
from jwave.transforms import wavelets as W
from jwave.transforms.modwt import ConvolutionMethod

pytestmark = pytest.mark.gpu

FMA_TOL = 1e-10


def normwise(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def draw_modwt(rng):
    while True:
        wname = str(rng.choice(W.ALL))
        L = len(W.by_name(wname).getScalingDeComposition())
        n = int(rng.choice([rng.integers(2, 64), rng.integers(64, 5000), rng.integers(5000, 40000),
                            1 << int(rng.integers(1, 16))]))
        jmax = min(n.bit_length() - 1, 13)
        if jmax < 1:
            continue
        J = int(rng.integers(1, jmax + 1))
        method = str(rng.choice(["direct", "fft", "auto"]))
        arith = str(rng.choice(["strict", "fma"]))
        batch = int(rng.integers(1, 4))
        # the oracle's DIRECT cost (STRICT AUTO levels may be DIRECT; FMA checks against it)
        cost = batch * n * sum((L - 1) * (1 << (j - 1)) + 1 for j in range(1, J + 1))
        if (method != "fft" or arith == "fma") and cost > 2e8:
            continue
        threshold = int(rng.choice([4096, 4096, -1, n * 20, 2**31 - 1]))
        return wname, n, J, method, arith, batch, threshold


@pytest.mark.parametrize("case", range(256))
def test_modwt_random(case):
    rng = np.random.default_rng(7000 + case)
    wname, n, J, method, arith, batch, threshold = draw_modwt(rng)
    wv = W.by_name(wname)
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    m = MODWTTransform(wv, fftThreshold=threshold, arith=arith)
    m.setConvolutionMethod({"direct": ConvolutionMethod.DIRECT, "fft": ConvolutionMethod.FFT,
                            "auto": ConvolutionMethod.AUTO}[method])
    xs = np.stack([orc.fill_uniform(n, 100 * case + b) for b in range(batch)])
    c = m.forwardMODWT(xs, J)
    xr = m.inverseMODWT(c)
    what = (wname, n, J, method, arith, batch, threshold)
    for b in range(batch):
        if arith == "strict":
            ref = orc.modwt_forward(xs[b], J, g, h, method, threshold)
            assert bits_equal(c[b], ref), what
            assert bits_equal(xr[b], orc.modwt_inverse(c[b], g, h, method, threshold)), what
        else:  # the fast contract: within 1e-10 of the reference's DIRECT path, row by row
            ref = orc.modwt_forward(xs[b], J, g, h, "direct")
            for j in range(J + 1):
                assert normwise(c[b][j], ref[j]) <= FMA_TOL, (what, j)
            assert normwise(xr[b], orc.modwt_inverse(c[b], g, h, "direct")) <= FMA_TOL, what


@pytest.mark.parametrize("case", range(96))
def test_fwt_wpt_random(case):
    rng = np.random.default_rng(8000 + case)
    wv = W.Haar1Orthogonal() if rng.random() < 0.05 else W.by_name(str(rng.choice(W.ALL[2:] + ["Haar1"])))
    n = 1 << int(rng.integers(1, 15))
    level = int(rng.integers(0, n.bit_length()))
    batch = int(rng.integers(1, 4))
    xs = np.stack([orc.fill_uniform(n, 300 + 10 * case + b) for b in range(batch)])
    what = (wv.getName(), n, level, batch)
    for T, fwd, rev in ((FastWaveletTransform, orc.fwt_forward, orc.fwt_reverse),
                        (WaveletPacketTransform, orc.wpt_forward, orc.wpt_reverse)):
        t = T(wv)
        y = t.forwardBatch(xs, level)
        z = t.reverseBatch(xs, level)
        for b in range(batch):
            assert bits_equal(y[b], fwd(xs[b], level, wv)), (T.__name__, what)
            assert bits_equal(z[b], rev(xs[b], level, wv)), (T.__name__, what)


@pytest.mark.parametrize("case", range(48))
def test_fwt_2d_3d_random(case):
    rng = np.random.default_rng(9000 + case)
    wv = W.by_name(str(rng.choice(W.ALL[2:] + ["Haar1"])))
    f = FastWaveletTransform(wv)
    if case % 2 == 0:
        R, C = (1 << int(rng.integers(1, 10)) for _ in range(2))
        lM, lN = int(rng.integers(0, R.bit_length())), int(rng.integers(0, C.bit_length()))
        x = orc.fill_uniform(R * C, 500 + case).reshape(R, C)
        assert bits_equal(f.forward(x, lM, lN), orc.fwt2d_forward(x, lM, lN, wv)), (wv.getName(), R, C, lM, lN)
        assert bits_equal(f.reverse(x, lM, lN), orc.fwt2d_reverse(x, lM, lN, wv)), (wv.getName(), R, C, lM, lN)
    else:
        d = [1 << int(rng.integers(1, 6)) for _ in range(3)]
        # lvlP runs along the second dimension, lvlQ the third, lvlR the first
        # (BasicTransform.java:510-560: 2-D forward(spc[i], lvlP, lvlQ), then the first axis)
        lv = [int(rng.integers(0, d[k].bit_length())) for k in (1, 2, 0)]
        x = orc.fill_uniform(d[0] * d[1] * d[2], 600 + case).reshape(d)
        assert bits_equal(f.forward(x, *lv), orc.fwt3d_forward(x, *lv, wv)), (wv.getName(), d, lv)
        assert bits_equal(f.reverse(x, *lv), orc.fwt3d_reverse(x, *lv, wv)), (wv.getName(), d, lv)


@pytest.mark.parametrize("case", range(64))
def test_jwave_fft_random(case):
    rng = np.random.default_rng(9500 + case)
    n = int(rng.choice([rng.integers(1, 300), rng.integers(300, 20000), 1 << int(rng.integers(0, 17))]))
    batch = int(rng.integers(1, 4))
    z = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    f = FastFourierTransform()  # STRICT: the reference's own FFT
    X = f.forwardComplex(z)
    Y = f.reverseComplex(z)
    for b in range(batch):
        assert bits_equal(X[b].view(np.float64), orc.fft(z[b]).view(np.float64)), (n, batch)
        assert bits_equal(Y[b].view(np.float64), orc.fft(z[b], inverse=True).view(np.float64)), (n, batch)


# CWT transformFFT: engine against the oracle with correctly rounded twiddles (1e-12, engine
# error) and the faithful recurrence one (1e-10, JWave's own output), normwise over the
# scalogram, as tests/test_cwt_gpu.py; random wavelet, parameters, padding, length, scales
def draw_cwt(rng):
    from jwave.transforms.wavelets.continuous import (DOGWavelet, MeyerWavelet, MexicanHatWavelet,
                                                       MorletWavelet, PaulWavelet)
    k = int(rng.integers(0, 5))
    if k == 0:
        fb, fc = float(rng.uniform(0.5, 2.0)), float(rng.uniform(0.5, 1.5))
        return MorletWavelet(fb, fc), "morlet", (fb, fc)
    if k == 1:
        s = float(rng.uniform(0.5, 3.0))
        return MexicanHatWavelet(s), "mexhat", (s, 0.0)
    if k == 2:
        m = int(rng.integers(1, 12))
        return PaulWavelet(m), "paul", (float(m),)
    if k == 3:
        m, s = int(rng.integers(1, 8)), float(rng.uniform(0.5, 2.0))
        return DOGWavelet(m, s), "dog", (float(m), s)
    return MeyerWavelet(), "meyer", ()


@pytest.mark.parametrize("case", range(64))
def test_cwt_fft_random(case):
    from jwave import ContinuousWaveletTransform as CWT
    from jwave.transforms.cwt import PaddingType
    rng = np.random.default_rng(9800 + case)
    wv, kind, params = draw_cwt(rng)
    n = int(rng.choice([rng.integers(1, 200), rng.integers(200, 20000), 1 << int(rng.integers(8, 17))]))
    padding = list(PaddingType)[int(rng.integers(0, len(PaddingType)))]
    ns = int(rng.integers(2, 24))  # generateLogScales needs two (ContinuousWaveletTransform.java:362)
    lo = float(rng.uniform(0.3, 4.0))
    hi = lo * float(rng.uniform(1.5, 400.0))
    scales = CWT.generateLogScales(lo, hi, ns) if rng.random() < 0.7 else CWT.generateLinearScales(lo, hi, ns)
    fs = float(rng.choice([1.0, 1.0, 2.5, 0.25]))
    x = orc.fill_uniform(n, 900 + case)
    got = CWT(wv, padding).transformFFT(x, scales, fs).getCoefficients()
    ex = orc.cwt_fft(x, scales, fs, kind, params, int(padding), exact=True)
    jw = orc.cwt_fft(x, scales, fs, kind, params, int(padding), exact=False)
    what = (kind, params, n, padding, ns, lo, hi, fs)
    assert got.shape == (len(scales), n), what
    assert normwise(got, ex) < 1e-12, (what, normwise(got, ex))
    assert normwise(got, jw) < 1e-10, (what, normwise(got, jw))


@pytest.mark.parametrize("case", range(32))
def test_cwt_direct_random(case):
    from jwave import ContinuousWaveletTransform as CWT
    rng = np.random.default_rng(9900 + case)
    wv, kind, params = draw_cwt(rng)
    n = int(rng.integers(1, 3000))
    scales = CWT.generateLogScales(float(rng.uniform(0.3, 2.0)), float(rng.uniform(3.0, 200.0)),
                                   int(rng.integers(2, 10)))
    fs = float(rng.choice([1.0, 2.0, 0.5]))
    x = orc.fill_uniform(n, 950 + case)
    got = CWT(wv).transform(x, scales, fs).getCoefficients()
    ref = orc.cwt_direct(x, kind, wv.params(), scales, fs)
    assert bits_equal(got.real, ref.real) and bits_equal(got.imag, ref.imag), (kind, n, fs)
