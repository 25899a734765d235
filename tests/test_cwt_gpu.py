"""CWT (ContinuousWaveletTransform.transformFFT) on the MI355X vs the oracle.

Bar (north_star): within 1e-10 relative for Morlet.  The engine's FFT uses correctly rounded
twiddles; the reference's uses a recurrence (FastFourierTransform.java:188-201).  Each case is
checked against the oracle with exact twiddles (engine error, expected ~1e-14) and against the
faithful recurrence-twiddle oracle (the JWave output, <= 1e-10), normwise:
max|a - b| / max|b| over the whole scalogram.
"""
import math

import numpy as np
import pytest

import oracle as orc
from jwave import ContinuousWaveletTransform as CWT
from jwave.transforms.cwt import PaddingType
from jwave.transforms.wavelets.continuous import (DOGWavelet, MeyerWavelet, MexicanHatWavelet,
                                                   MorletWavelet, PaulWavelet)

pytestmark = pytest.mark.gpu

TOL_JWAVE = 1e-10   # north_star: Morlet within 1e-10 relative of JWave's CPU path
TOL_EXACT = 1e-12   # vs the same algorithm with correctly rounded twiddles


def nw(a, b):
    return np.max(np.abs(a - b)) / np.max(np.abs(b))


def check(wv, kind, params, n, scales, padding, seed=7, fs=1.0):
    x = orc.fill_uniform(n, seed)
    got = CWT(wv, padding).transformFFT(x, scales, fs).getCoefficients()
    ex = orc.cwt_fft(x, scales, fs, kind, params, int(padding), exact=True)
    jw = orc.cwt_fft(x, scales, fs, kind, params, int(padding), exact=False)
    assert got.shape == (len(scales), n)
    assert nw(got, ex) < TOL_EXACT, nw(got, ex)
    assert nw(got, jw) < TOL_JWAVE, nw(got, jw)


MORLET6 = (1.0, 6.0 / (2 * math.pi))  # cfg3 "omega0 = 6": MorletWavelet(1, 6/(2 pi))


@pytest.mark.parametrize("n", [1, 2, 5, 100, 512, 1000, 4096])
@pytest.mark.parametrize("padding", list(PaddingType))
def test_small_lengths_all_paddings(n, padding):
    scales = CWT.generateLogScales(1.0, 64.0, 5)
    check(MorletWavelet(*MORLET6), "morlet", MORLET6, n, scales, padding)


@pytest.mark.parametrize("n", [300, 4096, 10000])
def test_mexican_hat(n):
    scales = CWT.generateLinearScales(0.5, 40.0, 6)
    check(MexicanHatWavelet(1.5), "mexhat", (1.5, 0.0), n, scales, PaddingType.SYMMETRIC)


OTHERS = [(PaulWavelet(1), "paul", (1.0,)), (PaulWavelet(4), "paul", (4.0,)),
          (PaulWavelet(20), "paul", (20.0,)),
          (DOGWavelet(1, 2.0), "dog", (1.0, 2.0)), (DOGWavelet(2), "dog", (2.0, 1.0)),
          (DOGWavelet(3, 0.5), "dog", (3.0, 0.5)), (DOGWavelet(4), "dog", (4.0, 1.0)),
          (DOGWavelet(7, 1.3), "dog", (7.0, 1.3)), (MeyerWavelet(), "meyer", ())]


@pytest.mark.parametrize("wv,kind,params", OTHERS, ids=lambda v: str(v)[:14])
@pytest.mark.parametrize("n", [300, 4096, 1 << 17])
def test_paul_dog_meyer(wv, kind, params, n):
    # psi_hat real (Paul, even-n DOG) or complex (odd-n DOG, Meyer): X * conj(psi_hat)
    scales = CWT.generateLogScales(0.5, 200.0, 5)
    check(wv, kind, params, n, scales, PaddingType.PERIODIC, fs=1.7)


def test_paul_negative_scale_not_rejected():
    # PaulWavelet's fourierTransform(omega, scale, b) override has no scale check: the
    # reference returns NaN columns (sqrt of a negative scale) rather than throwing
    x = orc.fill_uniform(64, 3)
    c = CWT(PaulWavelet(4)).transformFFT(x, np.array([-1.0, 2.0]), 1.0).getCoefficients()
    assert np.all(np.isnan(c[0])) and np.all(np.isfinite(c[1]))


@pytest.mark.parametrize("n", [1 << 13, 1 << 17, 1 << 18, 300001])
def test_four_step_lengths(n):
    # 2^13 = 128 x 64 (generic passes), 2^17 = 512 x 256, 2^18 = 512 x 512 (both passes on
    # the wavefront engine: the cfg3 geometry), 300001 -> 2^19 = 1024 x 512 with padding
    scales = CWT.generateLogScales(2.0, 1024.0, 3)
    check(MorletWavelet(*MORLET6), "morlet", MORLET6, n, scales, PaddingType.SYMMETRIC, fs=2.5)


def np_cwt_morlet(x, scales, fs, params):
    """transformFFT for Morlet with zero padding, restated on numpy's FFT (correctly rounded
    twiddles, error ~1e-16 log N): omega and psi_hat as the oracle's jwo_cwt_fft /
    jwo_cwt_wavelet_ft_c (ContinuousWaveletTransform.java, MorletWavelet.java:117-125)."""
    n = x.shape[0]
    N = 1 << max(0, (n - 1).bit_length())
    X = np.fft.fft(np.concatenate([x, np.zeros(N - n)]))
    om = 2.0 * math.pi * np.arange(N) * fs / N
    om[N // 2 + 1:] -= 2.0 * math.pi * fs
    fb, fc = params
    out = np.empty((len(scales), n), complex)
    for i, a in enumerate(scales):
        f = a * om / (2.0 * math.pi)
        psi = math.sqrt(2.0 * math.pi * fb) * np.exp(-2.0 * math.pi ** 2 * fb * (f - fc) ** 2)
        out[i] = np.fft.ifft(X * (psi * math.sqrt(a)))[:n]
    return out


@pytest.mark.parametrize("n", [(1 << 24) + 5, (1 << 25) + 1])
def test_lengths_past_2_24(n):
    # nextPowerOfTwo(n) = 2^25, 2^26 (JWave pads with no cap): 8192-point lines through the
    # generic passes in 128 KB of LDS; scale 2 runs two-pass, 900 on a coarse grid.  Checked
    # per scale against the numpy restatement, which at 2^25 is itself checked against the
    # oracle with exact twiddles (~50 s of CPU; at 2^26 the oracle would take ~2 minutes).
    scales = np.array([2.0, 900.0])
    x = orc.fill_uniform(n, 7)
    got = CWT(MorletWavelet(*MORLET6), PaddingType.ZERO).transformFFT(x, scales, 1.0).getCoefficients()
    ref = np_cwt_morlet(x, scales, 1.0, MORLET6)
    for i in range(len(scales)):
        assert nw(got[i], ref[i]) < TOL_EXACT, (i, nw(got[i], ref[i]))
    if n < (1 << 25):
        ex = orc.cwt_fft(x, scales, 1.0, "morlet", MORLET6, 0, exact=True)
        assert nw(ref, ex) < TOL_EXACT
        assert nw(got, ex) < TOL_EXACT


@pytest.mark.parametrize("n,scales", [((1 << 26) + 1, (2.0, 900.0)), ((1 << 27) + 3, (900.0,))])
def test_lengths_past_2_26_three_passes(n, scales):
    # nextPowerOfTwo(n) = 2^27, 2^28 (ContinuousWaveletTransform.java:188-189, MathUtils.java:46-49:
    # no cap in the reference): 8192-point columns, then the 16384 / 32768-point rows as two-pass
    # FFTs of their own (three passes through two workspaces), every scale two-pass.  Per scale
    # against the numpy restatement (correctly rounded FFT), at the same bar as 2^25 / 2^26.
    scales = np.array(scales)
    x = orc.fill_uniform(n, 9)
    got = CWT(MorletWavelet(*MORLET6), PaddingType.ZERO).transformFFT(x, scales, 1.0).getCoefficients()
    ref = np_cwt_morlet(x, scales, 1.0, MORLET6)
    for i in range(len(scales)):
        assert nw(got[i], ref[i]) < TOL_EXACT, (i, nw(got[i], ref[i]))


def test_length_past_2_28_refused():
    with pytest.raises(NotImplementedError, match="2\\^28"):
        CWT(MorletWavelet(*MORLET6)).transformFFT(np.zeros((1 << 28) + 1), np.array([4.0]), 1.0)


def test_batch_and_device_tensors(device):
    import torch
    n, B = 1 << 18, 3
    scales = CWT.generateLogScales(2.0, 1024.0, 4)
    xs = np.stack([orc.fill_uniform(n, 7 + b) for b in range(B)])
    t = CWT(MorletWavelet(*MORLET6))
    host = t.transformFFTBatch(xs, scales)
    dev = t.transformFFTBatch(torch.from_numpy(xs).to(device), scales)
    torch.cuda.synchronize()
    assert dev.is_cuda and dev.shape == (B, 4, n)
    assert np.array_equal(host, dev.cpu().numpy())
    for b in range(B):
        ex = orc.cwt_fft(xs[b], scales, 1.0, "morlet", MORLET6, 1, exact=True)
        assert nw(host[b], ex) < TOL_EXACT


@pytest.mark.parametrize("kind", ["morlet", "mexhat", "dog"])
def test_pipelined_groups_bit_identical(kind, knobs):
    # N = 2^18 runs the (signal, scale) inverse FFTs in groups, pass 2 of one group beside
    # pass 1 of the next; an 8 MiB workspace makes groups of 2 pairs (7 groups, last one
    # short).  The pipelined and sequential schedules do the same arithmetic: equal bits.
    n, B = 1 << 18, 2
    scales = CWT.generateLogScales(2.0, 1024.0, 7)
    xs = np.stack([orc.fill_uniform(n, 21 + b) for b in range(B)])
    wv, params = {"morlet": (MorletWavelet(*MORLET6), MORLET6),
                  "mexhat": (MexicanHatWavelet(1.5), (1.5, 0.0)),
                  "dog": (DOGWavelet(3, 0.5), (3.0, 0.5))}[kind]
    knobs.setenv("JW_CWT_GROUP_MB", "8")
    knobs.setenv("JW_CWT_PIPE", "1")
    piped = CWT(wv).transformFFTBatch(xs, scales)
    knobs.setenv("JW_CWT_PIPE", "0")
    seq = CWT(wv).transformFFTBatch(xs, scales)
    assert np.array_equal(piped, seq)
    for b in range(B):
        ex = orc.cwt_fft(xs[b], scales, 1.0, kind, params, 1, exact=True)
        assert nw(piped[b], ex) < TOL_EXACT


def test_sinusoid_peaks_at_matching_scale():
    # Morlet with fc = 6/(2 pi): scale a resonates with frequency fc / a (scaleToFrequency)
    n, fs = 1 << 14, 1.0
    t = np.arange(n)
    f0 = 0.05
    x = np.cos(2 * np.pi * f0 * t)
    scales = CWT.generateLogScales(2.0, 256.0, 64)
    r = CWT(MorletWavelet(*MORLET6)).transformFFT(x, scales, fs)
    best = scales[int(np.argmax(r.getScalogram()))]
    assert abs(MORLET6[1] / best - f0) / f0 < 0.08


@pytest.mark.parametrize("kind", ["morlet", "mexhat"])
@pytest.mark.parametrize("n", [1 << 13, 1 << 16, 1 << 18, 300001])
def test_band_scales_one_pass(kind, n, knobs):
    # Scales whose psi_hat band spans few 512-bin blocks run the one-pass band kernel
    # (cwt_band512); JW_CWT_BAND=0 sends every scale through the two-pass FFT.  The band drops
    # only bins below e^-60 of psi_hat's peak, so both agree far inside the oracle tolerance.
    scales = CWT.generateLogScales(2.0, 1024.0, 12)
    wv, params = {"morlet": (MorletWavelet(*MORLET6), MORLET6),
                  "mexhat": (MexicanHatWavelet(1.5), (1.5, 0.0))}[kind]
    x = orc.fill_uniform(n, 5)
    knobs.setenv("JW_CWT_INTERP", "0")  # no coarse grids: the band kernel itself
    knobs.setenv("JW_CWT_BAND", "1000")
    band = CWT(wv).transformFFT(x, scales, 1.0).getCoefficients()
    knobs.setenv("JW_CWT_BAND", "0")
    two = CWT(wv).transformFFT(x, scales, 1.0).getCoefficients()
    assert nw(band, two) < 1e-13, nw(band, two)
    ex = orc.cwt_fft(x, scales, 1.0, kind, params, 1, exact=True)
    assert nw(band, ex) < TOL_EXACT
    for i in range(len(scales)):  # per scale, against that scale's own magnitude
        assert nw(band[i], ex[i]) < 1e-11, (i, nw(band[i], ex[i]))


@pytest.mark.parametrize("kind", ["morlet", "mexhat"])
@pytest.mark.parametrize("n", [1 << 14, 1 << 16, 1 << 18, 300001, 1 << 20])
@pytest.mark.parametrize("pmin", ["4", "2"])
def test_coarse_grid_scales(kind, n, pmin, knobs):
    # Band scales whose band fits a grid of M = N / P points (P >= JW_CWT_INTERP) run as an
    # M-point inverse DFT (the band kernel on the coarse grid, the band divided by the
    # Kaiser-Bessel kernel's transform) and a 19-tap interpolation to the N-point coefficients.
    # Against the same scales through the two-pass FFT (JW_CWT_INTERP=0, JW_CWT_BAND=0): the
    # interpolation error is ~1e-14 of each scale's peak (W = 18, oversampling 1.25); against the
    # oracle per scale as the other paths.  pmin = 2 also runs the P = 2 grids.
    scales = CWT.generateLogScales(2.0, 1024.0, 14)
    wv, params = {"morlet": (MorletWavelet(*MORLET6), MORLET6),
                  "mexhat": (MexicanHatWavelet(1.5), (1.5, 0.0))}[kind]
    x = orc.fill_uniform(n, 11)
    knobs.setenv("JW_CWT_INTERP", pmin)
    got = CWT(wv).transformFFT(x, scales, 1.0).getCoefficients()
    knobs.setenv("JW_CWT_INTERP", "0")
    knobs.setenv("JW_CWT_BAND", "0")
    two = CWT(wv).transformFFT(x, scales, 1.0).getCoefficients()
    for i in range(len(scales)):
        assert nw(got[i], two[i]) < 1e-12, (i, nw(got[i], two[i]))
    if n <= (1 << 18):
        ex = orc.cwt_fft(x, scales, 1.0, kind, params, 1, exact=True)
        assert nw(got, ex) < TOL_EXACT
        for i in range(len(scales)):
            assert nw(got[i], ex[i]) < 1e-11, (i, nw(got[i], ex[i]))


def test_coarse_grid_workspace_chunks(knobs):
    # The coarse rows of a group go through a ~128 MB workspace a few signals at a time: at
    # N = 2^18 the P = 4 grids (65536 points) hold 17 signals of 7 scales, so 20 signals take
    # two chunks.  Same values as the two-pass FFT per scale, and the same bits whether the
    # signals come in one call or one at a time (the chunking changes no operation).
    import torch
    n = 1 << 18
    scales = np.array([17.7, 19.5, 21.5, 23.8, 26.3, 29.0, 32.0])
    xs = np.stack([orc.fill_uniform(n, 60 + b) for b in range(20)])
    t = CWT(MorletWavelet(*MORLET6))
    got = t.transformFFTBatch(torch.from_numpy(xs).cuda(), scales, 1.0).cpu().numpy()
    one = t.transformFFT(xs[19], scales, 1.0).getCoefficients()
    assert np.array_equal(got[19], one)
    knobs.setenv("JW_CWT_INTERP", "0")
    knobs.setenv("JW_CWT_BAND", "0")
    for b in (0, 16, 19):
        two = t.transformFFT(xs[b], scales, 1.0).getCoefficients()
        for i in range(len(scales)):
            assert nw(got[b, i], two[i]) < 1e-12, (b, i, nw(got[b, i], two[i]))


@pytest.mark.parametrize("kind", ["morlet", "mexhat"])
def test_band_and_pass1_variants_bit_identical(kind, knobs):
    # The band kernel's schedules (JW_CWT_BAND_V: load prefetch, one or eight row groups per
    # workgroup at 6 or 4 waves per SIMD) and the two-pass first pass with the X read issued
    # before or after psi_hat's exp (JW_CWT_EARLY) do the same operations: equal bits, at the
    # cfg3 length with both one-pass and two-pass scales.
    n = 1 << 18
    scales = CWT.generateLogScales(2.0, 1024.0, 10)
    wv = {"morlet": MorletWavelet(*MORLET6), "mexhat": MexicanHatWavelet(1.5)}[kind]
    x = orc.fill_uniform(n, 9)
    ref = None
    for v, e in [("3", "1"), ("0", "0"), ("2", "1"), ("1", "0")]:
        knobs.setenv("JW_CWT_BAND_V", v)
        knobs.setenv("JW_CWT_EARLY", e)
        got = CWT(wv).transformFFT(x, scales, 1.0).getCoefficients()
        if ref is None:
            ref = got
        else:
            assert np.array_equal(got, ref), (v, e)


def test_result_accessors_on_device(device):
    # CWTResult.getMagnitude / getPhase / getScalogram (CWTResult.java:94-126, :272-287) on
    # device coefficients (jw_cwt_magnitude / _phase / _scalogram): no host copy of the
    # scalogram's input.  Magnitude bit-identical to Complex.getMag's sqrt(re^2 + im^2).
    import torch
    from jwave.transforms import cwt
    n, B = 1 << 14, 2
    scales = CWT.generateLogScales(2.0, 256.0, 9)
    xs = np.stack([orc.fill_uniform(n, 31 + b) for b in range(B)])
    t = CWT(MorletWavelet(*MORLET6))
    dev = t.transformFFTBatch(torch.from_numpy(xs).to(device), scales)
    host = dev.cpu().numpy()
    r = t.resultOf(dev[1], scales)
    hr = t.resultOf(host[1], scales)
    mag = r.getMagnitude()
    assert mag.is_cuda and mag.shape == (9, n)
    assert np.array_equal(mag.cpu().numpy(), hr.getMagnitude())
    assert np.max(np.abs(r.getPhase().cpu().numpy() - hr.getPhase())) < 1e-13
    sg = r.getScalogram().cpu().numpy()
    assert np.max(np.abs(sg - hr.getScalogram()) / hr.getScalogram()) < 1e-13
    sgb = cwt.scalogram(dev).cpu().numpy()  # B x ns in one launch
    assert sgb.shape == (B, 9) and np.allclose(sgb[1], sg, rtol=1e-15, atol=0)
    hm = cwt.magnitude(host)  # JW_HOST staging path
    assert np.array_equal(hm, np.sqrt(host.real * host.real + host.imag * host.imag))
    # quadrant edge cases of Complex.getPhi
    c = np.array([1 + 1j, -1 + 0j, 0j, -2 - 2j, 1 - 1j, -0.0 + 3j, 0.0 - 3j])
    ph = cwt.phase(torch.from_numpy(c).to(device)).cpu().numpy()
    ref = CWTResult_host_phase(c)
    assert np.max(np.abs(ph - ref)) < 1e-15


def CWTResult_host_phase(c):
    from jwave.transforms import CWTResult
    return CWTResult(c.reshape(1, -1), [1.0], np.arange(c.size), 1.0, "x").getPhase()[0]


def test_fft_scalogram_fused(device):
    # jw_cwt_fft_scalogram: transformFFT(...).getScalogram() with the coefficients kept in HBM
    import torch
    n, B = 5000, 3
    scales = CWT.generateLogScales(1.0, 300.0, 11)
    xs = np.stack([orc.fill_uniform(n, 41 + b) for b in range(B)])
    t = CWT(MorletWavelet(*MORLET6))
    e = t.transformFFTScalogram(xs, scales)
    assert e.shape == (B, 11)
    for b in range(B):
        ref = t.transformFFT(xs[b], scales).getScalogram()
        assert np.max(np.abs(e[b] - ref) / ref) < 1e-13
    e1 = t.transformFFTScalogram(xs[1], scales)
    assert np.array_equal(e1, e[1])
    ed = t.transformFFTScalogram(torch.from_numpy(xs).to(device), scales)
    assert ed.is_cuda and np.array_equal(ed.cpu().numpy(), e)
    assert np.array_equal(t.transformFFTScalogram(np.zeros((2, 0)), scales), np.zeros((2, 11)))


def test_concurrent_host_threads_with_side_streams(knobs):
    # Host arrays (JW_HOST) from four threads at once: each thread stages on its own streams
    # and runs its band and coarse-grid scales on its own side stream (forked from and joined
    # into its staging stream; JW_CWT_OVERLAP=1 forces the side stream, which by default only
    # band-kernel scales take).  Every thread's result equals the same call made alone, bit for
    # bit, and with the side stream off (JW_CWT_OVERLAP=0: the same kernels on one stream).
    import threading
    knobs.setenv("JW_CWT_OVERLAP", "1")
    n = 1 << 16
    scales = CWT.generateLogScales(2.0, 1024.0, 16)
    xs = [orc.fill_uniform(n, 100 + i) for i in range(4)]
    alone = [CWT(MorletWavelet(*MORLET6)).transformFFT(x, scales, 1.0).getCoefficients()
             for x in xs]
    got = [None] * 4
    errs = []

    def work(i):
        try:
            for _ in range(3):
                got[i] = CWT(MorletWavelet(*MORLET6)).transformFFT(xs[i], scales, 1.0).getCoefficients()
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for i in range(4):
        assert np.array_equal(got[i], alone[i]), i
    knobs.setenv("JW_CWT_OVERLAP", "0")
    one = CWT(MorletWavelet(*MORLET6)).transformFFT(xs[0], scales, 1.0).getCoefficients()
    assert np.array_equal(one, alone[0])


def test_cfg3_full_scale_set():
    # BASELINE configs[2] as the bench runs it (64 log scales 2..1024, fs = 1, N = 2^18,
    # Morlet omega0 = 6), batch 2 through transformFFTBatch (the bench's device path), every
    # (signal, scale) against the oracle at both bars: normwise over the whole scalogram, and
    # per scale against that scale's own magnitude
    n = 1 << 18
    scales = CWT.generateLogScales(2.0, 1024.0, 64)
    xs = np.stack([orc.fill_uniform(n, 7 + b) for b in range(2)])
    import torch
    got = CWT(MorletWavelet(*MORLET6)).transformFFTBatch(torch.from_numpy(xs).cuda(), scales, 1.0)
    got = got.cpu().numpy()
    assert got.shape == (2, 64, n)
    for b in range(2):
        ex = orc.cwt_fft(xs[b], scales, 1.0, "morlet", MORLET6, 1, exact=True)
        jw = orc.cwt_fft(xs[b], scales, 1.0, "morlet", MORLET6, 1, exact=False)
        assert nw(got[b], ex) < TOL_EXACT, nw(got[b], ex)
        assert nw(got[b], jw) < TOL_JWAVE, nw(got[b], jw)
        for i in range(64):
            assert nw(got[b, i], ex[i]) < 1e-11, (b, i, nw(got[b, i], ex[i]))


def test_error_after_side_stream_launches_joins(knobs):
    # an error return after some coarse-grid groups have launched on the side stream
    # must still join them before the call's buffers are freed.  JW_TEST_CWT_FAIL_GROUP=1 fails
    # at the second group (groups 0 launched); the call raises, then the same call without the
    # injection equals the one made before it, bit for bit, with the side stream forced on.
    from jwave.exceptions import JWaveFailure
    knobs.setenv("JW_CWT_OVERLAP", "1")
    n = 1 << 16
    scales = CWT.generateLogScales(2.0, 1024.0, 24)
    x = orc.fill_uniform(n, 31)
    t = CWT(MorletWavelet(*MORLET6))
    before = t.transformFFT(x, scales, 1.0).getCoefficients()
    knobs.setenv("JW_TEST_CWT_FAIL_GROUP", "1")
    for _ in range(3):
        with pytest.raises(JWaveFailure, match="injected failure"):
            t.transformFFT(x, scales, 1.0)
    knobs.delenv("JW_TEST_CWT_FAIL_GROUP")
    import torch
    torch.cuda.synchronize()
    assert np.array_equal(t.transformFFT(x, scales, 1.0).getCoefficients(), before)


def test_split_coarse_path_bit_identical(knobs):
    # JW_CWT_SPLIT=1 (A/B setting): every coarse-grid band kernel first, on the side stream beside
    # the two-pass chain, into one workspace per group; the interpolations after the chain.  Same
    # kernels on the same inputs: the same bits as the default order.
    import torch
    n = 1 << 18
    scales = CWT.generateLogScales(2.0, 1024.0, 20)
    xs = np.stack([orc.fill_uniform(n, 80 + b) for b in range(3)])
    t = CWT(MorletWavelet(*MORLET6))
    base = t.transformFFTBatch(torch.from_numpy(xs).cuda(), scales, 1.0).cpu().numpy()
    knobs.setenv("JW_CWT_SPLIT", "1")
    got = t.transformFFTBatch(torch.from_numpy(xs).cuda(), scales, 1.0).cpu().numpy()
    assert np.array_equal(got, base)


def test_reference_cwt_test_params_fixture():
    # the reference's own CWT test parameters (scripts/generate_basic_reference.py:120-130 ->
    # testdata/cwt_test_params.txt: fs = 1000, 256 samples, 20 scales 1 .. 50), run through both
    # CWT paths on its clean test signal: transformFFT against the oracle (exact twiddles 1e-12,
    # JWave's recurrence 1e-10, normwise), the direct transform bit for bit, for the wavelets
    # ContinuousWaveletTransformTest.java uses (Morlet(1, 1) :48, MexicanHat(1) :72, Paul(4) :281,
    # Meyer :301), linear and log scales
    import os
    from _util import GOLDEN, clean_signal
    p = {}
    with open(os.path.join(GOLDEN, "reference_testdata", "cwt_test_params.txt")) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                k, v = line.split("=")
                p[k] = float(v)
    fs, n, ns = p["sampling_rate"], int(p["signal_length"]), int(p["num_scales"])
    x = clean_signal(n)
    for scales in (CWT.generateLinearScales(p["scale_min"], p["scale_max"], ns),
                   CWT.generateLogScales(p["scale_min"], p["scale_max"], ns)):
        for wv, kind, params in ((MorletWavelet(1.0, 1.0), "morlet", (1.0, 1.0)),
                                 (MexicanHatWavelet(1.0), "mexhat", (1.0, 0.0)),
                                 (PaulWavelet(4), "paul", (4.0,)), (MeyerWavelet(), "meyer", ())):
            got = CWT(wv).transformFFT(x, scales, fs).getCoefficients()
            ex = orc.cwt_fft(x, scales, fs, kind, params, int(PaddingType.SYMMETRIC), exact=True)
            jw = orc.cwt_fft(x, scales, fs, kind, params, int(PaddingType.SYMMETRIC), exact=False)
            assert got.shape == (ns, n)
            if np.max(np.abs(ex)) == 0:  # Meyer at fs = 1000: its band misses every bin, all zeros
                assert np.max(np.abs(jw)) == 0 and not np.any(got), kind
            else:
                assert nw(got, ex) < TOL_EXACT and nw(got, jw) < TOL_JWAVE, (kind, nw(got, ex), nw(got, jw))
            d = CWT(wv).transform(x, scales, fs).getCoefficients()
            ref = orc.cwt_direct(x, kind, wv.params(), scales, fs)
            assert np.array_equal(d.real.view(np.uint64), ref.real.view(np.uint64))
            assert np.array_equal(d.imag.view(np.uint64), ref.imag.view(np.uint64))
