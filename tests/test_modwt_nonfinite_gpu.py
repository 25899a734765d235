"""MODWT DIRECT on non-finite data: the engine against the FAITHFUL oracle (every up-sampled tap).

JWave's circularConvolve / circularConvolveAdjoint (MODWTTransform.java:677-716) multiply every
tap of the up-sampled filter (upsample, :618-630), zeros included, and 0 * +-Inf = 0 * NaN = NaN.
So from level 2 on, one +-Inf or NaN sample turns every output whose window holds it on a zero
tap into NaN.  The engine's kernels skip the zero taps; a signal whose final row comes out
non-finite is re-run by the zero-tap pass (jw_modwt.hip).  These tests compare with the oracle's
"direct" method (the literal Java loop), never "direct_nz":
  * STRICT: equal NaN-ness, and equal bits everywhere else (+-Inf included);
  * FMA: equal NaN-ness and equal +-Inf positions, finite values within the FMA bar.
Every kernel family is driven: the fast streaming kernels (N >= 512 even), the generic
streaming kernels (odd N, or JW_MODWT_KERNEL=generic), the per-level kernels (H > 4096), each
inverse kernel (JW_INV_KERNEL = wave2 / wave / wg), and AUTO's DIRECT levels.
"""
import numpy as np
import pytest

import oracle as orc
from jwave import MODWTTransform
from jwave.transforms import wavelets as W

pytestmark = pytest.mark.gpu

INF, NINF, NAN = np.inf, -np.inf, np.nan
FMA_TOL = 1e-10


def filters(wv):
    return orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())


def engine(wv, arith="strict", method="DIRECT", threshold=4096):
    m = MODWTTransform(wv, fftThreshold=threshold, arith=arith)
    m.setConvolutionMethod(getattr(MODWTTransform.ConvolutionMethod, method))
    return m


def check(got, ref, arith="strict"):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), (
        f"NaN-ness differs at {np.argwhere(gn != rn)[:8].tolist()} "
        f"({int(np.sum(gn != rn))} positions; engine NaN {int(gn.sum())}, reference {int(rn.sum())})")
    g, r = got[~gn], ref[~rn]
    if arith == "strict":
        assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), \
            f"finite/Inf values differ, max {np.max(np.abs(g - r))}"
    else:
        gi, ri = np.isinf(g), np.isinf(r)
        assert np.array_equal(gi, ri) and np.array_equal(g[gi], r[ri])
        scale = max(np.max(np.abs(r[~ri])), 1e-300) if np.any(~ri) else 1.0
        assert np.max(np.abs(g[~gi] - r[~ri]), initial=0.0) <= FMA_TOL * scale


def poison(x, spots):
    y = np.array(x, dtype=np.float64, copy=True)
    for p, v in spots:
        y[..., p] = v
    return y


SPOTS = {
    "interior_inf": lambda n: [(n // 3, INF)],
    "interior_nan": lambda n: [(n // 2 + 1, NAN)],
    "first": lambda n: [(0, NINF)],
    "last": lambda n: [(n - 1, INF)],
    "several": lambda n: [(1, INF), (n // 4, NINF), (n // 2, NAN), (n - 2, INF)],
    "inf_pair": lambda n: [(n // 5, INF), (n // 5 + 1, NINF)],
}

FWD_CASES = [
    # (wavelet, n, J): fast kernels (even n >= 512), generic (odd n, small n), per-level (H > 4096)
    ("Haar1", 1024, 6), ("Daubechies4", 4096, 8), ("Symlet8", 2048, 6), ("Daubechies4", 600, 4),
    ("Haar1", 777, 8), ("Daubechies4", 5001, 8), ("Symlet8", 999, 5), ("Daubechies4", 40, 5),
    ("Haar1", 8, 3), ("Daubechies4", 13, 3),
    ("Daubechies4", 4096, 10), ("Haar1", 8192, 13), ("Symlet8", 1500, 9),
]


@pytest.mark.parametrize("arith", ["strict", "fma"])
@pytest.mark.parametrize("spot", sorted(SPOTS))
@pytest.mark.parametrize("wname,n,J", FWD_CASES)
def test_forward_nonfinite(wname, n, J, spot, arith):
    wv = W.by_name(wname)
    g, h = filters(wv)
    x = poison(orc.fill_uniform(n, 7 + n), SPOTS[spot](n))
    ref = orc.modwt_forward(x, J, g, h, "direct")
    check(engine(wv, arith).forwardMODWT(x, J), ref, arith)


def _coeffs_with(c, spots):
    c = np.array(c, copy=True)
    for r, p, v in spots:
        c[r, p] = v
    return c


@pytest.mark.parametrize("inv_kernel", [None, "wave2", "wave", "wg"])
@pytest.mark.parametrize("arith", ["strict", "fma"])
@pytest.mark.parametrize("wname,n,J", [("Haar1", 1024, 6), ("Daubechies4", 4096, 8),
                                       ("Symlet8", 2048, 6), ("Daubechies4", 5001, 8),
                                       ("Haar1", 777, 8), ("Daubechies4", 4096, 10),
                                       ("Symlet8", 1500, 9), ("Daubechies4", 40, 5)])
def test_inverse_nonfinite(wname, n, J, arith, inv_kernel, knobs):
    if inv_kernel:
        knobs.setenv("JW_INV_KERNEL", inv_kernel)
    wv = W.by_name(wname)
    g, h = filters(wv)
    c0 = orc.modwt_forward(orc.fill_uniform(n, 3 + n), J, g, h, "direct")
    m = engine(wv, arith)
    for spots in ([(J, n // 3, INF)],                      # V_J
                  [(J - 1, 0, NAN)],                       # W_J at index 0
                  [(1, n - 1, NINF)],                      # W_2 at the wrap
                  [(0, n // 2, INF)],                      # W_1 (no zero taps at level 1)
                  [(J, 5 % n, INF), (J // 2, n // 2, NINF), (0, n - 1, NAN)]):
        c = _coeffs_with(c0, spots)
        check(m.inverseMODWT(c), orc.modwt_inverse(c, g, h, "direct"), arith)


@pytest.mark.parametrize("wname,n,J", [("Daubechies4", 4096, 8), ("Daubechies4", 5001, 8),
                                       ("Symlet8", 1500, 9)])
def test_generic_kernels_nonfinite(wname, n, J, knobs):
    knobs.setenv("JW_MODWT_KERNEL", "generic")
    wv = W.by_name(wname)
    g, h = filters(wv)
    x = poison(orc.fill_uniform(n, 11), SPOTS["several"](n))
    ref = orc.modwt_forward(x, J, g, h, "direct")
    m = engine(wv)
    check(m.forwardMODWT(x, J), ref)
    c = _coeffs_with(orc.modwt_forward(orc.fill_uniform(n, 12), J, g, h, "direct"),
                     [(J, 3, INF), (J - 2, n // 2, NAN)])
    check(m.inverseMODWT(c), orc.modwt_inverse(c, g, h, "direct"))


def test_batch_only_flagged_signals_change():
    # one poisoned signal among clean ones: the clean rows stay bit-exact with the finite path
    wv = W.Daubechies4()
    g, h = filters(wv)
    n, J, B = 4096, 8, 6
    xs = np.stack([orc.fill_uniform(n, 100 + b) for b in range(B)])
    xs[2, 17] = INF
    xs[4, n - 1] = NAN
    m = engine(wv)
    got = m.forwardMODWT(xs, J)
    for b in range(B):
        check(got[b], orc.modwt_forward(xs[b], J, g, h, "direct"))
    cs = np.stack([orc.modwt_forward(orc.fill_uniform(n, 200 + b), J, g, h, "direct")
                   for b in range(B)])
    cs[1, J, 9] = NINF
    cs[5, 3, 0] = INF
    xr = m.inverseMODWT(cs)
    for b in range(B):
        check(xr[b], orc.modwt_inverse(cs[b], g, h, "direct"))


def test_overflow_from_finite_input():
    # finite samples near DBL_MAX overflow to +-Inf inside the cascade; the zero taps of the
    # next level then turn that into NaN in JWave
    wv = W.Daubechies4()
    g, h = filters(wv)
    n, J = 2048, 6
    x = orc.fill_uniform(n, 5)
    x[100:104] = 1.7e308
    ref = orc.modwt_forward(x, J, g, h, "direct")
    assert np.isnan(ref).any()
    check(engine(wv).forwardMODWT(x, J), ref)


@pytest.mark.parametrize("threshold", [1 << 30, 20000])
def test_auto_direct_levels_nonfinite(threshold):
    # AUTO with a threshold that sends the low levels (or all) DIRECT, STRICT arithmetic
    wv = W.Daubechies4()
    g, h = filters(wv)
    n, J = 1024, 6
    x = poison(orc.fill_uniform(n, 9), [(n // 3, INF)])
    m = engine(wv, method="AUTO", threshold=threshold)
    ref = orc.modwt_forward(x, J, g, h, "auto", threshold)
    check(m.forwardMODWT(x, J), ref)
    c = _coeffs_with(orc.modwt_forward(orc.fill_uniform(n, 19), J, g, h, "direct"),
                     [(J, 10, INF), (2, n // 2, NAN)])
    check(m.inverseMODWT(c), orc.modwt_inverse(c, g, h, "auto", threshold))


def test_headline_shape_one_poisoned_signal():
    # cfg2 geometry (db4, J = 8, N = 2^20), two signals, one with a +Inf: the zero-tap pass at
    # full length against the faithful oracle; the clean signal bit-exact as before
    wv = W.Daubechies4()
    g, h = filters(wv)
    n, J = 1 << 20, 8
    xs = np.stack([orc.fill_uniform(n, 42), orc.fill_uniform(n, 43)])
    xs[1, 123457] = INF
    m = engine(wv)
    got = m.forwardMODWT(xs, J)
    check(got[0], orc.modwt_forward(xs[0], J, g, h, "direct_nz"))
    ref1 = orc.modwt_forward(xs[1], J, g, h, "direct")
    check(got[1], ref1)
    xr = m.inverseMODWT(got)
    check(xr[1], orc.modwt_inverse(ref1, g, h, "direct"))
