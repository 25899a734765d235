"""FWT parity on the MI355X: the HIP cascade (through the C-ABI) vs the oracle.

JW_ARITH_STRICT must be bit-identical to the JVM sequence of Wavelet.forward / the
Wavelet.reverse scatter (src/main/java/jwave/transforms/wavelets/Wavelet.java:236-303) for
every wavelet, length and level; 2-D follows BasicTransform.java:361-474.
"""
import math

import numpy as np
import pytest

import oracle as orc
from _util import bits_equal, load_vector
from jwave import FastWaveletTransform, Transform
from jwave.transforms import wavelets as W

pytestmark = pytest.mark.gpu

CREATE2ARR = (["Haar1"] + [f"Daubechies{k}" for k in range(2, 21)]
              + [f"Coiflet{k}" for k in range(1, 6)] + [f"Symlet{k}" for k in range(2, 21)])


def wavelet(name):
    return W.Haar1Orthogonal() if name == "Haar1Orthogonal" else W.by_name(name)


@pytest.mark.parametrize("wname", CREATE2ARR + ["Haar1Orthogonal", "Legendre1", "Legendre3"])
def test_fwt_bit_exact_all_wavelets(wname):
    wv = wavelet(wname)
    f = FastWaveletTransform(wv)
    fm = FastWaveletTransform(wv, arith="fma")
    for n, levels in [(2, [1]), (8, [0, 1, 3]), (64, [2, 6]), (1024, [10, 4])]:
        x = orc.fill_uniform(n, 3 + n)
        for lvl in levels:
            y = f.forward(x, lvl)
            ref = orc.fwt_forward(x, lvl, wv)
            assert bits_equal(y, ref), (n, lvl)
            rref = orc.fwt_reverse(ref, lvl, wv)
            assert bits_equal(f.reverse(ref, lvl), rref), (n, lvl)
            # FMA contract: fused products, tap order free; north_star tolerance 1e-10
            assert np.max(np.abs(fm.forward(x, lvl) - ref)) <= 1e-10 * np.max(np.abs(ref)), (n, lvl)
            assert np.max(np.abs(fm.reverse(ref, lvl) - rref)) <= 1e-10 * np.max(np.abs(rref)), (n, lvl)


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies8", "Symlet8", "Haar1Orthogonal"])
@pytest.mark.parametrize("n", [4096, 16384])
def test_fwt_long_signals(wname, n):
    # n = 4096 runs one workgroup per signal in LDS, 16384 the per-level global path
    wv = wavelet(wname)
    f = FastWaveletTransform(wv)
    x = orc.fill_uniform(n, 17)
    lvl = int(math.log2(n))
    ref = orc.fwt_forward(x, lvl, wv)
    assert bits_equal(f.forward(x, lvl), ref)
    assert bits_equal(f.reverse(ref, lvl), orc.fwt_reverse(ref, lvl, wv))
    assert bits_equal(f.forward(x, 3), orc.fwt_forward(x, 3, wv))


def test_fwt_batch():
    wv = W.Daubechies4()
    f = FastWaveletTransform(wv)
    xs = np.stack([orc.fill_uniform(1024, b) for b in range(7)])
    ys = f.forwardBatch(xs, 10)
    for b in range(7):
        assert bits_equal(ys[b], orc.fwt_forward(xs[b], 10, wv))
    xr = f.reverseBatch(ys, 10)
    for b in range(7):
        assert bits_equal(xr[b], orc.fwt_reverse(ys[b], 10, wv))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies8"])
@pytest.mark.parametrize("rows,cols,lvlM,lvlN", [(64, 32, 6, 5), (256, 256, 8, 8), (128, 512, 3, 9)])
def test_fwt2d_bit_exact(wname, rows, cols, lvlM, lvlN):
    wv = W.by_name(wname)
    f = FastWaveletTransform(wv)
    x = orc.fill_uniform(rows * cols, 11).reshape(rows, cols)
    ref = orc.fwt2d_forward(x, lvlM, lvlN, wv)
    assert bits_equal(f.forward(x, lvlM, lvlN), ref)
    assert bits_equal(f.reverse(ref, lvlM, lvlN), orc.fwt2d_reverse(ref, lvlM, lvlN, wv))


@pytest.mark.parametrize("wname", ["Haar1", "Haar1Orthogonal", "Daubechies8", "Symlet8",
                                   "Daubechies2", "Coiflet5"])
@pytest.mark.parametrize("rows,cols,lvlM,lvlN,tail", [
    (256, 128, 8, 7, "64"),     # two strip levels, tail of 64 rows x 6 levels
    (512, 64, 2, 6, "64"),      # every column level a strip: no tail
    (128, 64, 7, 6, "64"),      # one strip level
    (256, 64, 5, 6, "64"),      # tail with fewer levels than its length allows
    (4096, 128, 12, 7, None),   # the cfg4 column geometry: levels 1-4 streamed + 256-row tail
    (4096, 64, 4, 3, None),     # exactly the streamed levels: the level-4 approximations final
])
def test_fwt2d_strip_columns_bit_exact(wname, rows, cols, lvlM, lvlN, tail, knobs):
    # tall matrices run the first column levels as row-strip kernels (4096 rows and filters of
    # up to 16 taps: the one-pass streaming kernel) and the rest in an LDS tail (JW_FWT_TAIL
    # shrinks the tail so small matrices take that path too)
    if tail:
        knobs.setenv("JW_FWT_TAIL", tail)
    wv = W.by_name(wname)
    f = FastWaveletTransform(wv)
    x = orc.fill_uniform(rows * cols, 17).reshape(rows, cols)
    ref = orc.fwt2d_forward(x, lvlM, lvlN, wv)
    assert bits_equal(f.forward(x, lvlM, lvlN), ref)
    assert bits_equal(f.reverse(ref, lvlM, lvlN), orc.fwt2d_reverse(ref, lvlM, lvlN, wv))
    fm = FastWaveletTransform(wv, arith="fma")
    assert np.max(np.abs(fm.forward(x, lvlM, lvlN) - ref)) <= 1e-10 * np.max(np.abs(ref))
    # FMA reverse (fused tap pairs): within the north_star's 1e-10 of the reference order
    rref = orc.fwt2d_reverse(ref, lvlM, lvlN, wv)
    assert np.max(np.abs(fm.reverse(ref, lvlM, lvlN) - rref)) <= 1e-10 * np.max(np.abs(rref))


@pytest.mark.parametrize("wname,shape,lv", [
    ("Haar1", (8, 16, 32), (4, 5, 3)),
    ("Daubechies8", (16, 32, 64), (5, 6, 4)),
    ("Daubechies4", (4, 64, 8), (6, 3, 2)),   # non-cubic, fused column path along dim 1
    ("Symlet8", (32, 8, 4), (3, 2, 5)),
    ("Coiflet1", (8, 8, 8), (2, 1, 3)),        # 6 taps, cubic
    ("Haar1Orthogonal", (16, 16, 16), (4, 4, 4)),
    ("Daubechies8", (2, 4, 8), (0, 2, 1)),
])
def test_fwt3d_bit_exact(wname, shape, lv):
    # BasicTransform.forward/reverse(double[][][], lvlP, lvlQ, lvlR) (:509-659)
    wv = W.by_name(wname)
    f = FastWaveletTransform(wv)
    x = orc.fill_uniform(int(np.prod(shape)), 23).reshape(shape)
    ref = orc.fwt3d_forward(x, *lv, wv)
    assert bits_equal(f.forward(x, *lv), ref)
    rref = orc.fwt3d_reverse(ref, *lv, wv)
    assert bits_equal(f.reverse(ref, *lv), rref)
    fm = FastWaveletTransform(wv, arith="fma")
    assert np.max(np.abs(fm.forward(x, *lv) - ref)) <= 1e-10 * np.max(np.abs(ref))
    assert np.max(np.abs(fm.reverse(ref, *lv) - rref)) <= 1e-10 * np.max(np.abs(rref))


def test_fwt3d_default_levels_and_batch():
    wv = W.Daubechies8()
    f = FastWaveletTransform(wv)
    xs = np.stack([orc.fill_uniform(16 ** 3, 31 + b).reshape(16, 16, 16) for b in range(3)])
    # forward(double[][][]) uses log2 of each dimension (:487-495)
    assert bits_equal(f.forward(xs[0]), orc.fwt3d_forward(xs[0], 4, 4, 4, wv))
    ys = f.forward3DBatch(xs, 3, 4, 2)
    for b in range(3):
        assert bits_equal(ys[b], orc.fwt3d_forward(xs[b], 3, 4, 2, wv))
    xr = f.reverse3DBatch(ys, 3, 4, 2)
    for b in range(3):
        assert bits_equal(xr[b], orc.fwt3d_reverse(ys[b], 3, 4, 2, wv))


def test_wpt3d_matches_composition():
    from jwave.transforms.fwt import WaveletPacketTransform
    wv = W.Daubechies4()
    w = WaveletPacketTransform(wv)
    x = orc.fill_uniform(8 * 16 * 32, 41).reshape(8, 16, 32)
    y = w.forward(x, 3, 4, 2)
    ref = np.stack([w.forward(x[i], 3, 4) for i in range(8)])
    for j in range(16):
        for k in range(32):
            ref[:, j, k] = orc.wpt_forward(ref[:, j, k].copy(), 2, wv)
    assert bits_equal(y, ref)
    assert np.max(np.abs(w.reverse(y, 3, 4, 2) - x)) < 1e-10


def test_fwt2d_batch():
    wv = W.Daubechies8()
    f = FastWaveletTransform(wv)
    xs = np.stack([orc.fill_uniform(64 * 64, 11 + b).reshape(64, 64) for b in range(3)])
    ys = f.forward2DBatch(xs, 6, 6)
    for b in range(3):
        assert bits_equal(ys[b], orc.fwt2d_forward(xs[b], 6, 6, wv))
    xr = f.reverse2DBatch(ys, 6, 6)
    for b in range(3):
        assert np.max(np.abs(xr[b] - xs[b])) < 1e-10


@pytest.mark.parametrize("wname", CREATE2ARR)
def test_decompose_constant(wname):
    # DecomposeTest.java:40-120 through the facade
    t = Transform(FastWaveletTransform(W.by_name(wname)))
    s2 = math.sqrt(2.)
    m = t.decompose(np.ones(4))
    assert np.max(np.abs(m - np.array([[1, 1, 1, 1], [s2, s2, 0, 0], [2, 0, 0, 0]]))) < 1e-8
    assert np.max(np.abs(t.recompose(m, 0) - 1.0)) < 1e-8


def test_haar_fixtures_through_gpu():
    # transforms/CrossValidationTest.java:183-208
    x = load_vector("haar_simple_input.txt")
    y = Transform(FastWaveletTransform(W.Haar1())).forward(x, 1)
    assert np.max(np.abs(y[:4] - load_vector("haar_level1_approx_manual.txt"))) < 1e-10
    assert np.max(np.abs(y[4:] - load_vector("haar_level1_detail_manual.txt"))) < 1e-10


def test_haar_orthogonal_integer_exact():
    wv = W.Haar1Orthogonal()
    f = FastWaveletTransform(wv)
    x = np.arange(-512.0, 512.0)
    y = f.forward(x, 10)
    assert np.all(y == np.round(y)) and bits_equal(f.reverse(y, 10), x)


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies2", "Daubechies8", "Symlet20", "Coiflet5",
                                   "Haar1Orthogonal"])
def test_fast_and_generic_lds_kernels_agree(wname, knobs):
    # JW_FWT_GENERIC forces the original LDS kernels; both are bit-identical to the oracle
    wv = wavelet(wname)
    f = FastWaveletTransform(wv)
    for n, lvl in [(4, 2), (32, 5), (4096, 12), (4096, 3)]:
        x = orc.fill_uniform(n, 17 + n)
        ref = orc.fwt_forward(x, lvl, wv)
        y_fast = f.forward(x, lvl)
        r_fast = f.reverse(ref, lvl)
        knobs.setenv("JW_FWT_GENERIC", "1")
        y_gen = f.forward(x, lvl)
        r_gen = f.reverse(ref, lvl)
        knobs.delenv("JW_FWT_GENERIC")
        rref = orc.fwt_reverse(ref, lvl, wv)
        assert bits_equal(y_fast, ref) and bits_equal(y_gen, ref), (n, lvl)
        assert bits_equal(r_fast, rref) and bits_equal(r_gen, rref), (n, lvl)


@pytest.mark.parametrize("wname", CREATE2ARR + ["Haar1Orthogonal", "Legendre1", "Legendre3"])
def test_row4096_kernels_bit_exact(wname, knobs):
    # n = 4096 rows run fwt_fwd_row / fwt_rev_row (compile-time level sizes, wrap copy, details
    # straight to HBM) for filters of up to 20 taps; JW_FWT_ROW=0 runs the runtime-level
    # cascades (which longer filters always use).  STRICT: both bit-identical
    # to the oracle at every level count; FMA: the two kernels add the same fused products in
    # the same order, so they agree bit for bit too.
    wv = wavelet(wname)
    f = FastWaveletTransform(wv)
    fm = FastWaveletTransform(wv, arith="fma")
    n = 4096
    x = orc.fill_uniform(n, 29)
    for lvl in [0, 1, 2, 5, 11, 12]:
        ref = orc.fwt_forward(x, lvl, wv)
        rref = orc.fwt_reverse(ref, lvl, wv)
        assert bits_equal(f.forward(x, lvl), ref), lvl
        assert bits_equal(f.reverse(ref, lvl), rref), lvl
        yf, rf = fm.forward(x, lvl), fm.reverse(ref, lvl)
        knobs.setenv("JW_FWT_ROW", "0")
        assert bits_equal(fm.forward(x, lvl), yf), lvl
        assert bits_equal(fm.reverse(ref, lvl), rf), lvl
        knobs.delenv("JW_FWT_ROW")


@pytest.mark.parametrize("arith", ["strict", "fma"])
def test_cfg4_full_images(arith, device):
    # BASELINE configs[3] at its own size: FastWaveletTransform(Daubechies8) 2-D forward and
    # reverse of 4096 x 4096 images, 12 x 12 levels (BasicTransform.java:361-474), two images
    # of the batched call on HBM (the bench's synthetic inputs, seeds 11 and 12).  STRICT is
    # bit-exact with the oracle's rows-then-columns restatement; FMA within 1e-10 normwise.
    import ctypes

    import torch
    from jwave import _native
    wv = W.Daubechies8()
    R, lvl, B = 4096, 12, 2
    x = torch.empty((B, R, R), dtype=torch.float64, device=device)
    _native.check(_native.lib().jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), R * R, B, 11, None))
    f = FastWaveletTransform(wv, arith=arith)
    y = f.forward2DBatch(x, lvl, lvl)
    torch.cuda.synchronize()
    refs = []
    for b in range(B):
        xb = orc.fill_uniform(R * R, 11 + b).reshape(R, R)
        assert bits_equal(x[b].cpu().numpy(), xb)
        ref = orc.fwt2d_forward(xb, lvl, lvl, wv)
        got = y[b].cpu().numpy()
        if arith == "strict":
            assert bits_equal(got, ref), b
        else:
            assert np.max(np.abs(got - ref)) <= 1e-10 * np.max(np.abs(ref)), b
        refs.append(ref)
    yr = torch.from_numpy(np.stack(refs)).to(device)
    xr = f.reverse2DBatch(yr, lvl, lvl)
    torch.cuda.synchronize()
    for b in range(B):
        rref = orc.fwt2d_reverse(refs[b], lvl, lvl, wv)
        got = xr[b].cpu().numpy()
        if arith == "strict":
            assert bits_equal(got, rref), b
        else:
            assert np.max(np.abs(got - rref)) <= 1e-10 * np.max(np.abs(rref)), b
