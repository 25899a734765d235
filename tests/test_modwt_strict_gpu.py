"""JWave's default MODWT path on the MI355X: ConvolutionMethod.AUTO (and FFT) under
JW_ARITH_STRICT run the reference's own FFT convolution level by level
(MODWTTransform.java:640-664, :752-837; FastFourierTransform.java:172-212), so the engine's
values are the JVM's bit for bit -- checked against the oracle's restatement of the same path
(oracle "auto" / "fft": recurrence twiddles, per-call filter FFT, per-level AUTO rule with the
int32 product).  Also the JW_ARITH_STRICT FFT entry points (jw_fft_forward_ex / _reverse_ex).

Bar: bit-exact (np.array_equal of the IEEE bits) for every case, including lengths where the
rule mixes DIRECT and FFT levels and N = 2^20 (cfg2 / cfg5 geometry).
"""
import ctypes

import numpy as np
import pytest

import oracle as orc
from _util import bits_equal, clean_signal, mse
from jwave import FastFourierTransform, MODWTTransform
from jwave.transforms import wavelets as W
from jwave.transforms.modwt import ConvolutionMethod

pytestmark = pytest.mark.gpu


def ofilters(wv):
    return orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())


def levels_fft(n, L, J, threshold=4096):
    return [orc.auto_uses_fft(n, (L - 1) * (1 << (j - 1)) + 1, threshold) for j in range(1, J + 1)]


# (wavelet, n, J, threshold): one-column lengths (n <= 4096), the two-pass column path
# (n >= 8192), mixed DIRECT/FFT levels, multi-wrap filters (sym8 on n = 8), all-DIRECT and
# all-FFT thresholds
AUTO_CASES = [
    ("Haar1", 8, 3, 4096), ("Haar1", 4096, 12, 4096), ("Daubechies4", 64, 6, 4096),
    ("Daubechies4", 512, 4, 4096), ("Daubechies4", 512, 1, 4096), ("Symlet8", 8, 3, 4096),
    ("Symlet8", 512, 6, 4096), ("Daubechies4", 4096, 8, 4096), ("Daubechies4", 8192, 8, 4096),
    ("Daubechies8", 1 << 15, 7, 4096), ("Coiflet5", 2048, 5, 4096), ("Daubechies2", 16, 4, 4096),
    ("Daubechies4", 1 << 14, 6, (1 << 14) * 30), ("Daubechies4", 256, 3, -1),
    ("Daubechies4", 4096, 5, 2**31 - 1), ("Symlet8", 1 << 13, 6, 4096),
    ("Daubechies20", 1024, 6, 4096), ("Haar1", 2, 1, -1), ("Daubechies4", 4, 2, -1),
]


@pytest.mark.parametrize("wname,n,J,threshold", AUTO_CASES)
def test_auto_bit_exact_vs_reference_path(wname, n, J, threshold):
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    xs = np.stack([orc.fill_uniform(n, 11 + n + b) for b in range(3)])
    m = MODWTTransform(wv, fftThreshold=threshold)  # AUTO, JW_ARITH_STRICT: the defaults
    c = m.forwardMODWT(xs, J)
    for b in range(3):
        assert bits_equal(c[b], orc.modwt_forward(xs[b], J, g, h, "auto", threshold)), b
    xr = m.inverseMODWT(c)
    for b in range(3):
        assert bits_equal(xr[b], orc.modwt_inverse(c[b], g, h, "auto", threshold)), b
    # the reference's own reconstruction bar (MODWTInverseTest.java:17-232, MSE < 1e-10)
    assert mse(xr, xs) < 1e-10


@pytest.mark.parametrize("wname,n,J", [("Daubechies4", 128, 3), ("Symlet8", 8, 3),
                                       ("Haar1", 256, 4), ("Daubechies6", 1 << 13, 5),
                                       ("Symlet8", 1 << 16, 6)])
def test_fft_method_bit_exact(wname, n, J):
    # setConvolutionMethod(FFT): every level through circularConvolveFFT (:752-837)
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    x = clean_signal(n) + orc.fill_uniform(n, n)
    m = MODWTTransform(wv)
    m.setConvolutionMethod(ConvolutionMethod.FFT)
    c = m.forwardMODWT(x, J)
    assert bits_equal(c, orc.modwt_forward(x, J, g, h, "fft"))
    assert bits_equal(m.inverseMODWT(c), orc.modwt_inverse(c, g, h, "fft"))


def test_mixed_levels_keep_direct_levels_exact():
    # db4, n = 512: level 1 has N*M = 512*8 = 4096, not > 4096 -> DIRECT in the reference; the
    # other levels take the FFT path.  Level 1's row is the DIRECT value, bit for bit.
    wv = W.Daubechies4()
    g, h = ofilters(wv)
    x = orc.fill_uniform(512, 9)
    assert levels_fft(512, 8, 4) == [False, True, True, True]
    c = MODWTTransform(wv).forwardMODWT(x, 4)
    assert bits_equal(c[0], orc.modwt_forward(x, 1, g, h, "direct_nz")[0])
    assert not bits_equal(c[1], orc.modwt_forward(x, 4, g, h, "direct_nz")[1])


@pytest.mark.parametrize("wname,J", [("Daubechies4", 8), ("Symlet8", 6), ("Daubechies4", 10)])
def test_auto_full_size(wname, J, device):
    # cfg2 / cfg5 geometry through JWave's default path.  db4 J=10: level 10's N*M product
    # wraps negative in int32 (:653), so the reference -- and the engine -- run it DIRECT
    # between FFT levels.
    import torch
    from jwave import _native
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    B, n = 2, 1 << 20
    if J == 10:
        assert levels_fft(n, wv.getMotherWavelength(), J)[-1] is False
    x = torch.empty((B, n), dtype=torch.float64, device=device)
    _native.check(_native.lib().jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 42, None))
    m = MODWTTransform(wv)
    c = m.forwardMODWT(x, J)
    xr = m.inverseMODWT(c)
    torch.cuda.synchronize()
    x1 = orc.fill_uniform(n, 43)
    got = c[1].cpu().numpy()
    ref = orc.modwt_forward(x1, J, g, h, "auto")
    assert bits_equal(got, ref)
    assert bits_equal(xr[1].cpu().numpy(), orc.modwt_inverse(ref, g, h, "auto"))
    # JWave's FFT path reconstructs to ~4e-10 here: the engine's is the same
    assert (xr - x).abs().max().item() < 1e-8


# (2^21, 2^22: two passes over 2048-point columns, 4 per workgroup; 2^23: three passes, the
# plain-transform split)
POW2 = [2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 1 << 14, 1 << 15, 1 << 16,
        1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 23]


@pytest.mark.parametrize("n", POW2)
def test_fft_strict_bit_exact(n):
    rng = np.random.default_rng(n)
    B = 3 if n <= (1 << 18) else 1
    z = rng.uniform(-1, 1, (B, n)) + 1j * rng.uniform(-1, 1, (B, n))
    f = FastFourierTransform()  # arith="strict" is the default
    X = f.forwardComplex(z)
    for b in range(B):
        assert bits_equal(X[b].view(np.float64), orc.fft(z[b]).view(np.float64))
    zr = f.reverseComplex(X)
    for b in range(B):
        assert bits_equal(zr[b].view(np.float64), orc.fft(X[b], inverse=True).view(np.float64))


def test_fft_strict_in_place_and_device(device):
    import torch
    from jwave import _native
    n, B = 1 << 14, 4
    rng = np.random.default_rng(5)
    z = rng.uniform(-1, 1, (B, n)) + 1j * rng.uniform(-1, 1, (B, n))
    t = torch.from_numpy(z).to(device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    _native.check(_native.lib().jw_fft_forward_ex(ctypes.c_void_p(t.data_ptr()),
                                                  ctypes.c_void_p(t.data_ptr()), n, B,
                                                  _native.JW_ARITH_STRICT, _native.JW_DEVICE,
                                                  stream))
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    for b in range(B):
        assert bits_equal(got[b].view(np.float64), orc.fft(z[b]).view(np.float64))


def test_fft_strict_largest_column():
    # the 4096-point column kernels: pass 1 of 2^24 (three passes for plain transforms from 2^23,
    # jw_jfft_host.hpp plain_three_pass_min) and the two-pass chirp-z convolution of n = 2^23 - 1
    # (m = 2^24 = 4096 x 4096: kp1 / kp2p / kp2s on 4096-point columns, 2 per workgroup)
    n = 1 << 24
    rng = np.random.default_rng(24)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    X = FastFourierTransform().forwardComplex(z)
    assert bits_equal(X.view(np.float64), orc.fft(z).view(np.float64))
    n = (1 << 23) - 1
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    X = FastFourierTransform().forwardComplex(z)
    assert bits_equal(X.view(np.float64), orc.fft(z).view(np.float64))


# ---- lengths that are not powers of two: the reference's Bluestein transform (:259-324) ----
BLUESTEIN = [3, 5, 6, 7, 12, 100, 1000, 2049, 4097, 70001, 1000003]


@pytest.mark.parametrize("n", BLUESTEIN)
def test_fft_strict_bluestein_bit_exact(n):
    rng = np.random.default_rng(n)
    B = 2
    z = rng.uniform(-1, 1, (B, n)) + 1j * rng.uniform(-1, 1, (B, n))
    f = FastFourierTransform()
    X = f.forwardComplex(z)
    for b in range(B):
        assert bits_equal(X[b].view(np.float64), orc.fft(z[b]).view(np.float64)), b
    zr = f.reverseComplex(X)
    for b in range(B):
        assert bits_equal(zr[b].view(np.float64), orc.fft(X[b], inverse=True).view(np.float64)), b


@pytest.mark.parametrize("wname,n,J", [("Daubechies6", 100, 3), ("Daubechies6", 288, 3),
                                       ("Daubechies6", 500, 3), ("Daubechies6", 1000, 3),
                                       ("Haar1", 3, 1), ("Symlet8", 12, 2), ("Daubechies4", 5, 2),
                                       ("Daubechies4", 4097, 8), ("Daubechies6", 70001, 3),
                                       ("Symlet8", 3000, 5)])
def test_auto_bluestein_lengths_bit_exact(wname, n, J):
    # MODWTInverseTest.java:75-91 lengths and wrap-heavy short ones, JWave's default AUTO: DIRECT
    # levels where N*M_j <= 4096, the reference's Bluestein FFT convolution elsewhere
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    xs = np.stack([clean_signal(n) + orc.fill_uniform(n, n + b) for b in range(3)])
    m = MODWTTransform(wv)
    c = m.forwardMODWT(xs, J)
    for b in range(3):
        assert bits_equal(c[b], orc.modwt_forward(xs[b], J, g, h, "auto")), b
    xr = m.inverseMODWT(c)
    for b in range(3):
        assert bits_equal(xr[b], orc.modwt_inverse(c[b], g, h, "auto")), b
    assert mse(xr, xs) < 1e-10


@pytest.mark.parametrize("wname,n,J", [("Daubechies4", 100, 3), ("Symlet8", 7, 2),
                                       ("Daubechies6", 5000, 4)])
def test_fft_method_bluestein_bit_exact(wname, n, J):
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    x = orc.fill_uniform(n, 3 * n)
    m = MODWTTransform(wv)
    m.setConvolutionMethod(ConvolutionMethod.FFT)
    c = m.forwardMODWT(x, J)
    assert bits_equal(c, orc.modwt_forward(x, J, g, h, "fft"))
    assert bits_equal(m.inverseMODWT(c), orc.modwt_inverse(c, g, h, "fft"))


# ---- three column passes (powers of two past 2^24, up to 2^28) ----
# JW_JFFT_3PASS_MIN lowers the length where the three-pass transform (jw_jfft_host.hpp
# fft_rows3) and the unfused long-line MODWT (jw_jfft.hip modwt_strict_long) take over, so they
# are checked against the oracle at lengths it finishes in seconds; one real 2^25 transform too.
@pytest.mark.parametrize("n", [1 << 18, 1 << 19, 1 << 20, 1 << 22])
def test_fft_strict_three_pass_bit_exact(n, knobs):
    knobs.setenv("JW_JFFT_3PASS_MIN", str(1 << 18))
    rng = np.random.default_rng(n + 3)
    B = 2 if n <= (1 << 20) else 1
    z = rng.uniform(-1, 1, (B, n)) + 1j * rng.uniform(-1, 1, (B, n))
    f = FastFourierTransform()
    X = f.forwardComplex(z)
    for b in range(B):
        assert bits_equal(X[b].view(np.float64), orc.fft(z[b]).view(np.float64)), b
    zr = f.reverseComplex(X)
    for b in range(B):
        assert bits_equal(zr[b].view(np.float64), orc.fft(X[b], inverse=True).view(np.float64)), b


# (wavelet, n, J, threshold, method): all-FFT, mixed DIRECT/FFT levels (a threshold that keeps
# the short filters DIRECT), the int32 wrap (db4 level 12 at 2^18: N M_12 >= 2^31 -> DIRECT)
LONG_CASES = [("Daubechies4", 1 << 18, 4, 4096, "auto"), ("Symlet8", 1 << 19, 3, 4096, "fft"),
              ("Daubechies4", 1 << 18, 7, (1 << 18) * 100, "auto"),
              ("Daubechies4", 1 << 18, 12, 4096, "auto"), ("Haar1", 1 << 20, 2, 4096, "auto")]


@pytest.mark.parametrize("wname,n,J,threshold,method", LONG_CASES)
def test_modwt_long_lines_bit_exact(wname, n, J, threshold, method, knobs):
    knobs.setenv("JW_JFFT_3PASS_MIN", str(1 << 18))
    wv = W.by_name(wname)
    g, h = ofilters(wv)
    xs = np.stack([orc.fill_uniform(n, 5 + b) for b in range(2)])
    m = MODWTTransform(wv, fftThreshold=threshold)
    if method == "fft":
        m.setConvolutionMethod(ConvolutionMethod.FFT)
    c = m.forwardMODWT(xs, J)
    xr = m.inverseMODWT(c)
    for b in range(2):
        ref = orc.modwt_forward(xs[b], J, g, h, method, threshold)
        assert bits_equal(c[b], ref), b
        assert bits_equal(xr[b], orc.modwt_inverse(ref, g, h, method, threshold)), b


def test_long_lines_workspace_bounded(knobs, device):
    # modwt_strict_long handed its own allocator to every transform, so the
    # three-pass workspaces piled up over batch x levels x transforms (db4 J=8, 8 signals at
    # 2^18: 8 x 56 transforms x 4 MB = 1.8 GB).  Each transform's workspace is now scoped to it:
    # the device memory a batch-8 call reserves stays bounded by a few line-sized buffers.
    import ctypes
    import torch
    from jwave import _native
    knobs.setenv("JW_JFFT_3PASS_MIN", str(1 << 18))
    n, J, B = 1 << 18, 8, 8
    wv = W.Daubechies4()
    x = torch.empty((B, n), dtype=torch.float64, device=device)
    _native.check(_native.lib().jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 3, None))
    c = torch.empty((B, J + 1, n), dtype=torch.float64, device=device)
    xr = torch.empty_like(x)
    m = MODWTTransform(wv)  # AUTO STRICT: every level through the long-line path at 2^18
    plan = m.initializeFilterCache()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run(b):
        _native.check(_native.lib().jw_modwt_forward(plan, P(x), P(c), n, J, b, _native.JW_CONV_AUTO,
                                                     _native.JW_DEVICE, None))
        _native.check(_native.lib().jw_modwt_inverse(plan, P(c), P(xr), n, J, b, _native.JW_CONV_AUTO,
                                                     _native.JW_DEVICE, None))
        torch.cuda.synchronize()

    run(1)  # tables (twiddles, filter spectra) and one signal's workspaces
    free0 = torch.cuda.mem_get_info(device)[0]
    run(B)
    grew = free0 - torch.cuda.mem_get_info(device)[0]
    assert grew < (256 << 20), f"batch {B} reserved {grew / 2**20:.0f} MiB more than batch 1"
    g, h = ofilters(wv)
    ref = orc.modwt_forward(orc.fill_uniform(n, 3 + B - 1), J, g, h, "auto")
    assert bits_equal(c[B - 1].cpu().numpy(), ref)
    assert bits_equal(xr[B - 1].cpu().numpy(), orc.modwt_inverse(ref, g, h, "auto"))


@pytest.mark.parametrize("lg", [25, 26, 27])
def test_fft_strict_three_pass_default_geometry(lg):
    # past the two-pass split, with the default geometry (jw_jfft_host.hpp split3: 2^12 x 2^6 x
    # 2^(lg - 18)); the oracle takes ~6 / 13 / 28 s for these on one core
    n = 1 << lg
    rng = np.random.default_rng(lg)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    X = FastFourierTransform().forwardComplex(z)
    assert bits_equal(X.view(np.float64), orc.fft(z).view(np.float64))


def test_auto_2_23_fused_columns_bit_exact():
    # JWave's default path at 2^23: the fused two-pass levels on 2048 x 4096 columns (kp2p / kp2r
    # on 4096-point columns, 2 per workgroup) and filter spectra through the plain three-pass
    # transform (jw_jfft_host.hpp plain_three_pass_min), forward and inverse
    n = 1 << 23
    wv = W.Daubechies4()
    g, h = ofilters(wv)
    x = orc.fill_uniform(n, 23)
    m = MODWTTransform(wv)
    c = m.forwardMODWT(x[None, :], 1)
    ref = orc.modwt_forward(x, 1, g, h, "auto")
    assert bits_equal(c[0], ref)
    assert bits_equal(m.inverseMODWT(c)[0], orc.modwt_inverse(ref, g, h, "auto"))


def test_auto_2_25_forward_bit_exact():
    # JWave's default path at a length past the two-pass FFT: db4 level 1 through the
    # unfused long-line MODWT (jw_jfft.hip modwt_strict_long) on three-pass transforms
    n = 1 << 25
    wv = W.Daubechies4()
    g, h = ofilters(wv)
    x = orc.fill_uniform(n, 25)
    c = MODWTTransform(wv).forwardMODWT(x[None, :], 1)
    assert bits_equal(c[0], orc.modwt_forward(x, 1, g, h, "auto"))


@pytest.mark.parametrize("n", [70001, 200001])
def test_bluestein_three_pass_bit_exact(n, knobs):
    # Bluestein's m-point convolution on three-pass transforms (jw_jfft_bs.hip bs_conv3): the
    # path of non-power-of-two lengths past 2^23 (m > 2^24), at lengths the oracle runs quickly
    knobs.setenv("JW_JFFT_3PASS_MIN", str(1 << 18))
    rng = np.random.default_rng(n)
    z = rng.uniform(-1, 1, (2, n)) + 1j * rng.uniform(-1, 1, (2, n))
    f = FastFourierTransform()
    X = f.forwardComplex(z)
    for b in range(2):
        assert bits_equal(X[b].view(np.float64), orc.fft(z[b]).view(np.float64)), b
    zr = f.reverseComplex(X)
    for b in range(2):
        assert bits_equal(zr[b].view(np.float64), orc.fft(X[b], inverse=True).view(np.float64)), b
    wv = W.Daubechies4()
    g, h = ofilters(wv)
    xs = np.stack([orc.fill_uniform(n, 9 + b) for b in range(2)])
    m = MODWTTransform(wv)  # AUTO
    c = m.forwardMODWT(xs, 3)
    xr = m.inverseMODWT(c)
    for b in range(2):
        ref = orc.modwt_forward(xs[b], 3, g, h, "auto")
        assert bits_equal(c[b], ref), b
        assert bits_equal(xr[b], orc.modwt_inverse(ref, g, h, "auto")), b


def test_bluestein_three_pass_1024_columns_bit_exact(knobs):
    # bs_conv3 with m = 2^22 under the lowered switch: split3 gives 1024-point first-pass columns,
    # run with the plain transforms' geometry (16 points per thread, jw_jfft.hpp kPlainEPT)
    knobs.setenv("JW_JFFT_3PASS_MIN", str(1 << 18))
    n = (1 << 20) + 3
    rng = np.random.default_rng(n)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    f = FastFourierTransform()
    X = f.forwardComplex(z)
    assert bits_equal(X.view(np.float64), orc.fft(z).view(np.float64))
    assert bits_equal(f.reverseComplex(X).view(np.float64), orc.fft(X, inverse=True).view(np.float64))


@pytest.mark.parametrize("n,J", [(1 << 20, 2), (1 << 19, 3)])
def test_wave_column_kp2p_bit_exact(n, J, knobs):
    # JW_AUTO_WCOL=1 (A/B setting, measured slower, profiles/r06/ab/auto_wcol): the 1024-point
    # kp2p columns through kp2p_w (8 columns per workgroup, points in registers, re/im LDS
    # exchanges) -- the same butterflies and twiddles, so the same bits as the reference path
    knobs.setenv("JW_AUTO_WCOL", "1")
    wv = W.Daubechies4()
    g, h = ofilters(wv)
    xs = np.stack([orc.fill_uniform(n, 5 + b) for b in range(2)])
    m = MODWTTransform(wv)
    c = m.forwardMODWT(xs, J)
    xr = m.inverseMODWT(c)
    for b in range(2):
        assert bits_equal(c[b], orc.modwt_forward(xs[b], J, g, h, "auto")), b
        assert bits_equal(xr[b], orc.modwt_inverse(c[b], g, h, "auto")), b
