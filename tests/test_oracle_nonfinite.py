"""The oracle's faithful DIRECT MODWT on non-finite data, pinned to a literal Python loop.

MODWTTransform.circularConvolve / circularConvolveAdjoint (MODWTTransform.java:677-716) walk
every tap of the up-sampled filter (upsample, :618-630), zeros included, so 0 * +-Inf and
0 * NaN make NaN.  The oracle's "direct" method (and AUTO's DIRECT levels) must do the same:
the GPU non-finite tests (test_modwt_nonfinite_gpu.py) use it as the reference.  The loop below
is the Java text restated in pure Python (sizes kept tiny).  CPU only.
"""
import math

import numpy as np
import pytest

import oracle as orc
from jwave.transforms import wavelets as W


def upsample(f, level):  # :618-630
    if level <= 1:
        return list(f)
    gap = (1 << (level - 1)) - 1
    out = [0.0] * (len(f) + (len(f) - 1) * gap)
    for i, c in enumerate(f):
        out[i * (gap + 1)] = c
    return out


def conv(sig, filt, adjoint):  # :677-716
    N, M = len(sig), len(filt)
    out = []
    for n in range(N):
        s = 0.0
        for m in range(M):
            idx = (n + m) % N if adjoint else (n - m) % N
            s += sig[idx] * filt[m]
        out.append(s)
    return out


def java_forward(x, J, g, h):  # forwardMODWT :256-306
    v, rows = list(x), []
    for j in range(1, J + 1):
        rows.append(conv(v, upsample(h, j), False))
        v = conv(v, upsample(g, j), False)
    return np.array(rows + [v])


def java_inverse(c, g, h):  # inverseMODWT :337-375
    J = len(c) - 1
    v = list(c[J])
    for j in range(J, 0, -1):
        a = conv(v, upsample(g, j), True)
        d = conv(list(c[j - 1]), upsample(h, j), True)
        v = [p + q for p, q in zip(a, d)]
    return np.array(v)


def same(a, b):
    a, b = np.asarray(a, dtype=float).ravel(), np.asarray(b, dtype=float).ravel()
    an, bn = np.isnan(a), np.isnan(b)
    return np.array_equal(an, bn) and np.array_equal(a[~an].view(np.uint64), b[~bn].view(np.uint64))


CASES = [("Haar1", 16, 4), ("Daubechies4", 24, 3), ("Symlet8", 40, 3), ("Daubechies4", 7, 2),
         ("Daubechies2", 33, 4)]


@pytest.mark.parametrize("wname,n,J", CASES)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_direct_matches_java_loop_nonfinite(wname, n, J, seed):
    rng = np.random.default_rng(seed)
    wv = W.by_name(wname)
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    x = orc.fill_uniform(n, seed)
    for p in rng.integers(0, n, 2):
        x[p] = rng.choice([math.inf, -math.inf, math.nan])
    with np.errstate(invalid="ignore", over="ignore"):
        ref = java_forward(list(x), J, list(g), list(h))
    assert np.isnan(ref).any()
    assert same(orc.modwt_forward(x, J, g, h, "direct"), ref)
    assert same(orc.modwt_forward(x, J, g, h, "auto", 1 << 30), ref)  # every level DIRECT
    c = orc.modwt_forward(orc.fill_uniform(n, seed + 9), J, g, h, "direct")
    c[J, rng.integers(0, n)] = math.inf
    c[int(rng.integers(1, J)), rng.integers(0, n)] = -math.inf
    with np.errstate(invalid="ignore", over="ignore"):
        refi = java_inverse([list(r) for r in c], list(g), list(h))
    assert same(orc.modwt_inverse(c, g, h, "direct"), refi)
    assert same(orc.modwt_inverse(c, g, h, "auto", 1 << 30), refi)


def test_zero_skipping_variant_differs_on_nonfinite():
    # why the GPU non-finite tests never compare with "direct_nz": it equals JWave only on
    # finite data (test_oracle_golden.py pins that), and here it does not
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    x = orc.fill_uniform(32, 5)
    x[10] = math.inf
    assert not same(orc.modwt_forward(x, 4, g, h, "direct_nz"), orc.modwt_forward(x, 4, g, h, "direct"))


# ---- FWT / WPT: Wavelet.forward / reverse (Wavelet.java:236-303) multiply every tap too ----
def w_forward(a, h2, sD, wD):  # Wavelet.forward(arrTime, arrTimeLength) :236-262
    out = [0.0] * h2
    h = h2 >> 1
    for i in range(h):
        out[i] = out[i + h] = 0.0
        for j in range(len(sD)):
            k = (i << 1) + j
            while k >= h2:
                k -= h2
            out[i] += a[k] * sD[j]
            out[i + h] += a[k] * wD[j]
    return out


def w_reverse(a, h2, sR, wR):  # Wavelet.reverse(arrHilb, arrHilbLength) :277-303
    out = [0.0] * h2
    h = h2 >> 1
    for i in range(h):
        for j in range(len(sR)):
            k = (i << 1) + j
            while k >= h2:
                k -= h2
            out[k] += (a[i] * sR[j]) + (a[i + h] * wR[j])
    return out


def java_fwt(x, level, wv, rev):  # FastWaveletTransform.forward / reverse :71-153
    arr, n, tw = list(x), len(x), wv.getTransformWavelength()
    if not rev:
        f = (wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        h, l = n, 0
        while h >= tw and l < level:
            arr[:h] = w_forward(arr, h, *f)
            h, l = h >> 1, l + 1
        return np.array(arr)
    f = (wv.getScalingReConstruction(), wv.getWaveletReConstruction())
    h = tw
    for _ in range(level, n.bit_length() - 1):
        h <<= 1
    while tw <= h <= n:
        arr[:h] = w_reverse(arr, h, *f)
        h <<= 1
    return np.array(arr)


def java_wpt(x, level, wv, rev):  # WaveletPacketTransform.forward / reverse :60-191
    arr, n, tw = list(x), len(x), wv.getTransformWavelength()
    if not rev:
        f = (wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        h, l = n, 0
        while h >= tw and l < level:
            for p in range(n // h):
                arr[p * h:(p + 1) * h] = w_forward(arr[p * h:(p + 1) * h], h, *f)
            h, l = h >> 1, l + 1
        return np.array(arr)
    f = (wv.getScalingReConstruction(), wv.getWaveletReConstruction())
    h = tw
    for _ in range(level, n.bit_length() - 1):
        h <<= 1
    while tw <= h <= n:
        for p in range(n // h):
            arr[p * h:(p + 1) * h] = w_reverse(arr[p * h:(p + 1) * h], h, *f)
        h <<= 1
    return np.array(arr)


@pytest.mark.parametrize("wname,n", [("Haar1", 16), ("Daubechies4", 32), ("Symlet8", 16),
                                     ("Daubechies8", 64)])
def test_fwt_wpt_match_java_loops_nonfinite(wname, n):
    rng = np.random.default_rng(n)
    wv = W.by_name(wname)
    lvl = n.bit_length() - 1
    x = orc.fill_uniform(n, 4)
    for p in rng.integers(0, n, 2):
        x[p] = rng.choice([math.inf, -math.inf, math.nan])
    with np.errstate(invalid="ignore", over="ignore"):
        for level in (1, lvl):
            assert same(orc.fwt_forward(x, level, wv), java_fwt(x, level, wv, False))
            assert same(orc.fwt_reverse(x, level, wv), java_fwt(x, level, wv, True))
            assert same(orc.wpt_forward(x, level, wv), java_wpt(x, level, wv, False))
            assert same(orc.wpt_reverse(x, level, wv), java_wpt(x, level, wv, True))
