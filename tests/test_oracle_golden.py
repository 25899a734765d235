"""Pin the oracle (oracle/jwave_oracle.c) to every known answer and fixture the reference's own
test suite holds for the hot path.  CPU only.

Each test names the reference test it restates (paths under src/test/java/jwave/).
"""
import math

import numpy as np
import pytest

import oracle as orc
from _util import bits_equal, clean_signal, load_vector, mse
from jwave.transforms import wavelets as W

ORTHO = W.ORTHONORMAL
# WaveletBuilder.create2arr (transforms/wavelets/WaveletBuilder.java:427-502), orthonormal part
CREATE2ARR = (["Haar1"] + [f"Daubechies{k}" for k in range(2, 21)]
              + [f"Coiflet{k}" for k in range(1, 6)] + [f"Symlet{k}" for k in range(2, 21)])


def filters(wv):
    return orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())


# ---------------------------------------------------------------- java.util.Random
def test_java_random_known_values():
    # JDK java.util.Random: new Random(42).nextDouble() and new Random(0).nextDouble()
    assert orc.java_random_doubles(42, 2) == [0.7275636800328681, 0.6832234717598454]
    assert orc.java_random_doubles(0, 1)[0] == 0.730967787376657


def test_uniform_jump_ahead_matches_stream():
    full = orc.fill_uniform(5000, 77)
    assert bits_equal(orc.fill_uniform(1234, 77, start=3000), full[3000:4234])
    assert np.all(full >= -1.0) and np.all(full < 1.0)


# ---------------------------------------------------------------- MODWT known answers
def test_modwt_haar_filters_are_exact_halves():
    # MODWTTransformTest.testKnownValuesWithHaar comment: filters {0.5,-0.5}, {0.5,0.5}
    g, h = filters(W.Haar1())
    assert list(g) == [0.5, 0.5] and list(h) == [0.5, -0.5]


def test_modwt_haar_known_values():
    # transforms/MODWTTransformTest.java:38-71 (exact in any order: taps are +-0.5)
    g, h = filters(W.Haar1())
    c = orc.modwt_forward(np.arange(1.0, 9.0), 1, g, h)
    assert list(c[0]) == [-3.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5]
    assert list(c[1]) == [4.5, 1.5, 2.5, 3.5, 4.5, 5.5, 6.5, 7.5]


def test_modwt_haar_energy_conservation():
    # transforms/MODWTTransformTest.java:73-89: variance of x == sum of coefficient variances
    g, h = filters(W.Haar1())
    x = np.arange(1.0, 9.0)
    c = orc.modwt_forward(x, 3, g, h)
    assert abs(np.var(x) - sum(np.var(r) for r in c)) < 1e-9


@pytest.mark.parametrize("wname,n,J", [("Haar1", 256, 4), ("Daubechies4", 128, 3),
                                       ("Haar1", 64, 3), ("Daubechies4", 128, 4),
                                       ("Daubechies6", 256, 5), ("Symlet8", 512, 6)])
def test_modwt_reconstruction(wname, n, J):
    # transforms/MODWTInverseTest.java:17-70
    g, h = filters(W.by_name(wname))
    x = clean_signal(n)
    xr = orc.modwt_inverse(orc.modwt_forward(x, J, g, h), g, h)
    assert mse(x, xr) < 1e-10


@pytest.mark.parametrize("n", [100, 288, 500, 1000])
def test_modwt_non_power_of_two(n):
    # transforms/MODWTInverseTest.java:75-91
    g, h = filters(W.Daubechies6())
    x = clean_signal(n)
    xr = orc.modwt_inverse(orc.modwt_forward(x, 3, g, h), g, h)
    assert xr.shape == (n,) and mse(x, xr) < 1e-10


def test_modwt_constant_and_linear():
    # transforms/MODWTInverseTest.java:175-205
    g, h = filters(W.Daubechies4())
    x = np.full(100, 5.0)
    assert np.max(np.abs(orc.modwt_inverse(orc.modwt_forward(x, 3, g, h), g, h) - x)) < 1e-10
    g, h = filters(W.Symlet8())
    x = 0.5 * np.arange(200.0)
    assert mse(orc.modwt_inverse(orc.modwt_forward(x, 4, g, h), g, h), x) < 1e-10


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8"])
@pytest.mark.parametrize("n,J", [(256, 3), (8, 2), (64, 4), (100, 3)])
def test_modwt_direct_vs_fft(wname, n, J):
    # transforms/MODWTFFTConvolutionTest.java:41-71,155-180,206-232 (1e-8 coeffs, 1e-10 recon)
    g, h = filters(W.by_name(wname))
    x = clean_signal(n)
    cd = orc.modwt_forward(x, J, g, h, "direct")
    cf = orc.modwt_forward(x, J, g, h, "fft")
    assert np.max(np.abs(cd - cf)) < 1e-8
    assert np.max(np.abs(orc.modwt_inverse(cf, g, h, "fft") - x)) < 1e-10
    assert np.max(np.abs(orc.modwt_inverse(cd, g, h, "direct") - x)) < 1e-10


def test_modwt_shift_invariance():
    # PropertyBasedTest.java:315-352: MODWT is circularly shift-equivariant (exactly)
    g, h = filters(W.Daubechies4())
    x = orc.fill_uniform(128, 5)
    c = orc.modwt_forward(x, 3, g, h)
    cs = orc.modwt_forward(np.roll(x, 5), 3, g, h)
    assert bits_equal(np.roll(c, 5, axis=1), cs)


def test_modwt_auto_rule_int32_wrap():
    # MODWTTransform.java:653 -- int multiply; db4 level 10 at N=2^20 wraps negative -> DIRECT
    assert orc.auto_uses_fft(1 << 20, 7 * 128 + 1)
    assert not orc.auto_uses_fft(1 << 20, 7 * 512 + 1)
    assert not orc.auto_uses_fft(8, 2)


# ---------------------------------------------------------------- FFT
def test_fft_reference_fixtures():
    # transforms/CrossValidationTest.java:120-153 with testdata/fft_*.txt
    for stem in ("fft_dc", "fft_impulse"):
        x = load_vector(stem + "_input.txt")
        y = orc.fft(x)
        assert np.max(np.abs(y.real - load_vector(stem + "_output_real.txt"))) < 1e-10
        assert np.max(np.abs(y.imag - load_vector(stem + "_output_imag.txt"))) < 1e-10


@pytest.mark.parametrize("n", [2, 4, 8, 16, 64, 256, 100, 12])
def test_fft_vs_dft(n):
    # transforms/FastFourierTransformTest.java:44-75 (power of 2) + Bluestein lengths
    x = orc.fill_uniform(2 * n, 3)
    z = x[:n] + 1j * x[n:]
    k = np.arange(n)
    dft = np.exp(-2j * np.pi * np.outer(k, k) / n) @ z
    assert np.max(np.abs(orc.fft(z) - dft)) < 1e-10
    assert np.max(np.abs(orc.fft(orc.fft(z), inverse=True) - z)) < 1e-10


# ---------------------------------------------------------------- FWT
def test_haar_filters_vs_fixtures():
    # transforms/CrossValidationTest.java:158-180 with testdata/filter_haar_*.txt
    hw = W.Haar1()
    assert np.max(np.abs(np.array(hw.getScalingDeComposition()) - load_vector("filter_haar_dec_lo.txt"))) < 1e-10
    assert np.max(np.abs(np.array(hw.getWaveletDeComposition()) - load_vector("filter_haar_dec_hi.txt"))) < 1e-10


def test_haar_reconstruction_filters_vs_fixtures():
    # testdata/filter_haar_rec_{lo,hi}.txt against Haar1.getScalingReConstruction /
    # getWaveletReConstruction (Haar1.java:44-70 copies the decomposition filters into the
    # reconstruction ones), at the reference's 1e-10 (CrossValidationTest.java:158-180).  The
    # fixture generator writes the high-pass in the time-reversed (pywt) convention,
    # [-1/sqrt2, 1/sqrt2] (scripts/generate_basic_reference.py:91-92), where JWave keeps
    # _waveletReCon = _waveletDeCom = [1/sqrt2, -1/sqrt2]: the fixture pins JWave's taps reversed.
    # No reference test reads these two files; the low-pass is symmetric either way.
    hw = W.Haar1()
    lo, hi = load_vector("filter_haar_rec_lo.txt"), load_vector("filter_haar_rec_hi.txt")
    assert np.max(np.abs(np.array(hw.getScalingReConstruction()) - lo)) < 1e-10
    assert np.max(np.abs(np.array(hw.getWaveletReConstruction())[::-1] - hi)) < 1e-10
    assert np.max(np.abs(np.array(hw.getWaveletReConstruction()) - hi)) > 1.0  # not the same order
    # the reconstruction pair is the decomposition pair (orthonormal), exactly
    assert np.array_equal(hw.getScalingReConstruction(), hw.getScalingDeComposition())
    assert np.array_equal(hw.getWaveletReConstruction(), hw.getWaveletDeComposition())


def test_daubechies_filters_vs_fixtures():
    # testdata/filter_db2_dec_lo.txt ("Daubechies 2 = Haar", 2 taps) and filter_db4_dec_{lo,hi}.txt
    # (4 taps) use the tap-count naming; JWave names by vanishing moments (DaubechiesK = 2K
    # taps, Daubechies4.java:50-60), so they pin Haar1 and Daubechies2.  The high-pass fixture
    # checks _buildOrthonormalSpace's alternating flip (Wavelet.java:104-122).  JWave's own
    # decimal literals sit 3.4e-13 from the fixture's 17-digit values, inside the 1e-10 the
    # reference's fixture tests use (CrossValidationTest.java:158-180).
    assert np.array_equal(np.array(W.Haar1().getScalingDeComposition()),
                          load_vector("filter_db2_dec_lo.txt"))
    d2 = W.Daubechies2()
    lo, hi = load_vector("filter_db4_dec_lo.txt"), load_vector("filter_db4_dec_hi.txt")
    assert np.max(np.abs(np.array(d2.getScalingDeComposition()) - lo)) < 1e-12
    assert np.max(np.abs(np.array(d2.getWaveletDeComposition()) - hi)) < 1e-12
    # the flip itself is exact: wD[i] = (-1)^i sD[M-1-i]
    sd = np.array(d2.getScalingDeComposition())
    assert np.array_equal(np.array(d2.getWaveletDeComposition()), sd[::-1] * np.array([1, -1, 1, -1]))
    # and the MODWT plan normalises these taps exactly as the oracle (MODWTTransform.java:599-606)
    g, h = orc.modwt_filters(lo, hi)
    assert abs(np.sum(g * g) - 0.5) < 1e-15 and abs(np.sum(h * h) - 0.5) < 1e-15


def test_haar_level1_vs_fixtures():
    # transforms/CrossValidationTest.java:183-208 (fixtures are (a+-b)/sqrt2, 1 ulp off JWave)
    x = load_vector("haar_simple_input.txt")
    y = orc.fwt_forward(x, 1, W.Haar1())
    assert np.max(np.abs(y[:4] - load_vector("haar_level1_approx_manual.txt"))) < 1e-10
    assert np.max(np.abs(y[4:] - load_vector("haar_level1_detail_manual.txt"))) < 1e-10


@pytest.mark.parametrize("wname", CREATE2ARR)
def test_fwt_decompose_constant(wname):
    # DecomposeTest.java:40-120 (every wavelet of WaveletBuilder.create2arr, delta 1e-8)
    wv = W.by_name(wname)
    s2 = math.sqrt(2.)
    x = np.ones(4)
    assert np.max(np.abs(orc.fwt_forward(x, 1, wv) - [s2, s2, 0, 0])) < 1e-8
    assert np.max(np.abs(orc.fwt_forward(x, 2, wv) - [2, 0, 0, 0])) < 1e-8
    x64 = np.ones(64)
    for lvl, (val, cnt) in enumerate([(1, 64), (s2, 32), (2, 16), (2 * s2, 8), (4, 4),
                                      (4 * s2, 2), (8, 1)]):
        exp = np.zeros(64)
        exp[:cnt] = val
        assert np.max(np.abs(orc.fwt_forward(x64, lvl, wv) - exp)) < 1e-8
        assert np.max(np.abs(orc.fwt_reverse(orc.fwt_forward(x64, lvl, wv), lvl, wv) - x64)) < 1e-8


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "Coiflet5",
                                   "Haar1Orthogonal", "Legendre2"])
def test_fwt_rounding(wname):
    # RoundingTest.java:40-120: 1000 forward+reverse of ones(1024) stay within 1e-8
    wv = W.by_name(wname) if wname != "Haar1Orthogonal" else W.Haar1Orthogonal()
    x = np.ones(1024)
    y = x.copy()
    for _ in range(1000):
        y = orc.fwt_reverse(orc.fwt_forward(y, 10, wv), 10, wv)
    assert np.max(np.abs(y - x)) < 1e-8


def test_haar_orthogonal_round_trip_exact_on_integers():
    # Haar1Orthogonal: integer taps, reverse x0.5 -> exact on small integers
    wv = W.Haar1Orthogonal()
    x = np.arange(-16.0, 16.0)
    y = orc.fwt_forward(x, 5, wv)
    assert np.all(y == np.round(y))
    assert bits_equal(orc.fwt_reverse(y, 5, wv), x)


def test_fwt3d_is_slab_2d_then_dimension_1():
    # BasicTransform.java:509-565 / :602-659 restated as compositions of the 2-D and 1-D
    # oracles (slab transforms, then the lines along dimension 1), and the round trip
    wv = W.Daubechies4()
    x = orc.fill_uniform(8 * 16 * 32, 5).reshape(8, 16, 32)
    y = orc.fwt3d_forward(x, 4, 5, 3, wv)
    ref = np.stack([orc.fwt2d_forward(x[i], 4, 5, wv) for i in range(8)])
    for j in range(16):
        for k in range(32):
            ref[:, j, k] = orc.fwt_forward(ref[:, j, k].copy(), 3, wv)
    assert bits_equal(y, ref)
    xr = np.stack([orc.fwt2d_reverse(y[i], 4, 5, wv) for i in range(8)])
    for j in range(16):
        for k in range(32):
            xr[:, j, k] = orc.fwt_reverse(xr[:, j, k].copy(), 3, wv)
    assert bits_equal(orc.fwt3d_reverse(y, 4, 5, 3, wv), xr)
    assert np.max(np.abs(xr - x)) < 1e-10


def test_fwt2d_round_trip():
    wv = W.Daubechies8()
    x = orc.fill_uniform(64 * 32, 11).reshape(64, 32)
    y = orc.fwt2d_forward(x, 6, 5, wv)
    assert np.max(np.abs(orc.fwt2d_reverse(y, 6, 5, wv) - x)) < 1e-10


def test_get_exponent_powers_of_two():
    # MathToolKit.getExponent (int)(log f / log 2) must be exact for every int power of 2
    for k in range(31):
        assert int(math.log(float(1 << k)) / math.log(2.)) == k


# ---------------------------------------------------------------- CWT
def test_cwt_fft_matches_closed_form():
    # ContinuousWaveletTransform.transformFFT (:183-229): an independent numpy evaluation of
    # X * conj(psi_hat) -> IFFT agrees within 1e-12 (FFT twiddles differ: recurrence vs exact)
    n = 256
    x = orc.fill_uniform(n, 7)
    scales = np.exp(np.log(2.0) + np.arange(8) * (np.log(64.0) - np.log(2.0)) / 7)
    fb, fc = 1.0, 6.0 / (2 * math.pi)
    got = orc.cwt_fft(x, scales, 1.0, "morlet", (fb, fc))
    omega = 2.0 * np.pi * np.arange(n) * 1.0 / n
    omega[np.arange(n) > n // 2] -= 2.0 * np.pi
    X = np.fft.fft(x)
    for s, a in enumerate(scales):
        f = a * omega / (2 * np.pi)
        psi = np.sqrt(2 * np.pi * fb) * np.exp(-2 * np.pi ** 2 * fb * (f - fc) ** 2) * np.sqrt(a)
        ref = np.fft.ifft(X * psi)
        assert np.max(np.abs(got[s] - ref)) < 1e-12 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("wname,n,J", [("Haar1", 64, 6), ("Daubechies4", 100, 6),
                                       ("Symlet8", 8, 3), ("Daubechies8", 512, 5),
                                       ("Daubechies20", 300, 4)])
def test_modwt_nonzero_tap_variant_is_bit_identical(wname, n, J):
    # skipping the up-sampled zeros of MODWTTransform.upsample (:618-630) changes no bit
    g, h = filters(W.by_name(wname))
    x = orc.fill_uniform(n, 9) * 1e3
    c = orc.modwt_forward(x, J, g, h, "direct")
    assert bits_equal(c, orc.modwt_forward(x, J, g, h, "direct_nz"))
    assert bits_equal(orc.modwt_inverse(c, g, h, "direct"), orc.modwt_inverse(c, g, h, "direct_nz"))


# ---------------------------------------------------------------- WPT
@pytest.mark.parametrize("wname", CREATE2ARR)
def test_wpt_stepping_constant(wname):
    # SteppingTest.java:180-215: WPT of {1,1,1,1} at levels 0..2, delta 1e-8, and reverse
    wv = W.by_name(wname)
    s2 = math.sqrt(2.)
    x = np.ones(4)
    for lvl, exp in enumerate([[1, 1, 1, 1], [s2, s2, 0, 0], [2, 0, 0, 0]]):
        y = orc.wpt_forward(x, lvl, wv)
        assert np.max(np.abs(y - exp)) < 1e-8
        assert np.max(np.abs(orc.wpt_reverse(y, lvl, wv) - x)) < 1e-8


def test_wpt_transforms_every_packet():
    # WaveletPacketTransform.java:86-108: at level 2 both halves of level 1 are transformed --
    # the second half of the packet transform is the FWT of the level-1 detail half
    wv = W.Daubechies4()
    x = orc.fill_uniform(64, 3)
    l1 = orc.fwt_forward(x, 1, wv)
    l2 = orc.wpt_forward(x, 2, wv)
    assert bits_equal(l2[:32], orc.fwt_forward(l1[:32], 1, wv))
    assert bits_equal(l2[32:], orc.fwt_forward(l1[32:], 1, wv))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8", "Haar1Orthogonal",
                                   "Legendre2"])
def test_wpt_rounding(wname):
    # RoundingTest.java:160-204: 256 forward+reverse WPT of ones(1024) within 1e-8
    wv = W.by_name(wname) if wname != "Haar1Orthogonal" else W.Haar1Orthogonal()
    x = np.ones(1024)
    y = x.copy()
    for _ in range(256):
        y = orc.wpt_reverse(orc.wpt_forward(y, 10, wv), 10, wv)
    assert np.max(np.abs(y - x)) < 1e-8
