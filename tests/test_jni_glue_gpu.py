"""Every compute entry of the shipped JNI glue (jni/jwave_hip_jni.c, compiled against the
test-only mock JNIEnv into tests/c/libjni_harness.so) on the GPU, exactly as a JVM calls it:
Java arrays in, Java arrays out, JW_HOST staging inside.  MODWT, FWT, WPT, 2-D / 3-D FWT, the
direct CWT and JWave's FFT are bit-exact against the oracle (JW_ARITH_STRICT); the CWT FFT path
within 1e-12 of the exact-twiddle restatement.  Reference seams: MODWTTransform.java:256,337;
FastWaveletTransform.java:71,119; BasicTransform.java:361,436,509,602;
WaveletPacketTransform.java:73,141; ContinuousWaveletTransform.java:153,183;
FastFourierTransform.java:112-164."""
import numpy as np
import pytest

import oracle as orc
from _jni import Harness, JavaException
from _util import bits_equal
from jwave.transforms import wavelets as W

pytestmark = pytest.mark.gpu


@pytest.fixture()
def jni():
    h = Harness()
    yield h
    assert h.violations() == 0, "the glue broke a JNI rule"
    h.reset()


def _modwt_plan(jni, wv, arith=0):
    return jni.call("HipMODWTTransform_nPlanCreate", jni.darray(wv.getScalingDeComposition()),
                    jni.darray(wv.getWaveletDeComposition()), 4096, arith)


@pytest.mark.parametrize("wname,n,J", [("Daubechies4", 4096, 8), ("Symlet8", 1000, 6),
                                       ("Haar1", 17, 4), ("Daubechies4", 1 << 16, 10)])
@pytest.mark.parametrize("method", [1, 0], ids=["direct", "auto"])
def test_modwt_forward_inverse_bit_exact(jni, wname, n, J, method):
    wv = W.by_name(wname)
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    x = orc.fill_uniform(n, 42 + n)
    p = _modwt_plan(jni, wv)
    c = jni.read(jni.call("HipMODWTTransform_nForward", p, jni.darray(x), J, method))
    om = "direct_nz" if method == 1 else "auto"
    ref = orc.modwt_forward(x, J, g, h, om)
    assert c.shape == (J + 1, n) and bits_equal(c, ref)
    xr = jni.read(jni.call("HipMODWTTransform_nInverse", p, jni.matrix(c), method))
    assert bits_equal(xr, orc.modwt_inverse(ref, g, h, om))
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def test_modwt_direct_buffers_batch_bit_exact(jni):
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    n, J, B = 8192, 7, 3
    x = np.stack([orc.fill_uniform(n, 7 + b) for b in range(B)])
    c = np.empty((B, J + 1, n))
    xr = np.empty((B, n))
    p = _modwt_plan(jni, wv)
    jni.call("HipMODWTTransform_nForwardDirect", p, jni.direct(x), jni.direct(c), n, J, B, 1)
    jni.call("HipMODWTTransform_nInverseDirect", p, jni.direct(c), jni.direct(xr), n, J, B, 1)
    for b in range(B):
        ref = orc.modwt_forward(x[b], J, g, h, "direct_nz")
        assert bits_equal(c[b], ref)
        assert bits_equal(xr[b], orc.modwt_inverse(ref, g, h, "direct_nz"))
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def _fwt_plan(jni, wv, arith=0):
    kind = getattr(wv, "kind", 0)  # JW_WAVELET_HAAR_ORTH for Haar1Orthogonal
    return jni.call("HipFastWaveletTransform_nPlanCreate", jni.darray(wv.getScalingDeComposition()),
                    jni.darray(wv.getWaveletDeComposition()),
                    jni.darray(wv.getScalingReConstruction()),
                    jni.darray(wv.getWaveletReConstruction()), wv.getMotherWavelength(),
                    wv.getTransformWavelength(), kind, arith)


@pytest.mark.parametrize("wname", ["Haar1", "Haar1Orthogonal", "Daubechies4", "Daubechies8",
                                   "Symlet8", "Coiflet3"])
def test_fwt_and_wpt_lines_bit_exact(jni, wname):
    wv = W.by_name(wname)
    p = _fwt_plan(jni, wv)
    for n, level in ((1024, 10), (4096, 12), (256, 3), (1 << 15, 15)):
        x = orc.fill_uniform(n, 3 + n)
        y = jni.read(jni.call("HipFastWaveletTransform_nLine", p, 0, jni.darray(x), level))
        assert bits_equal(y, orc.fwt_forward(x, level, wv)), (n, level)
        z = jni.read(jni.call("HipFastWaveletTransform_nLine", p, 1, jni.darray(y), level))
        assert bits_equal(z, orc.fwt_reverse(y, level, wv)), (n, level)
        yw = jni.read(jni.call("HipFastWaveletTransform_nLine", p, 2, jni.darray(x), level))
        assert bits_equal(yw, orc.wpt_forward(x, level, wv)), (n, level)
        zw = jni.read(jni.call("HipFastWaveletTransform_nLine", p, 3, jni.darray(yw), level))
        assert bits_equal(zw, orc.wpt_reverse(yw, level, wv)), (n, level)
    jni.call("HipFastWaveletTransform_nPlanDestroy", p)


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies8"])
def test_fwt_matrix_and_space_bit_exact(jni, wname):
    wv = W.by_name(wname)
    p = _fwt_plan(jni, wv)
    rng = np.random.default_rng(5)
    m = rng.uniform(-1, 1, (128, 256))
    y = jni.read(jni.call("HipFastWaveletTransform_nMatrix", p, 0, jni.matrix(m), 7, 8))
    assert bits_equal(y, orc.fwt2d_forward(m, 7, 8, wv))
    z = jni.read(jni.call("HipFastWaveletTransform_nMatrix", p, 1, jni.matrix(y), 7, 8))
    assert bits_equal(z, orc.fwt2d_reverse(y, 7, 8, wv))
    s = rng.uniform(-1, 1, (8, 16, 32))
    ys = jni.read(jni.call("HipFastWaveletTransform_nSpace", p, 0, jni.space(s), 4, 5, 3))
    assert ys.shape == s.shape and bits_equal(ys, orc.fwt3d_forward(s, 4, 5, 3, wv))
    zs = jni.read(jni.call("HipFastWaveletTransform_nSpace", p, 1, jni.space(ys), 4, 5, 3))
    assert bits_equal(zs, orc.fwt3d_reverse(ys, 4, 5, 3, wv))
    # slabs past the first may be larger: the reference copies slab 0's box of each and ignores
    # the rest (BasicTransform.java:518-528)
    o = jni.L.mock_oarray(s.shape[0], b"[[D")
    for i in range(s.shape[0]):
        big = rng.uniform(-1, 1, (16 + i % 3, 32 + 2 * (i % 2))) if i else s[0]
        if i:
            big[:16, :32] = s[i]
        jni.L.mock_oset(o, i, jni.matrix(big))
    yb = jni.read(jni.call("HipFastWaveletTransform_nSpace", p, 0, o, 4, 5, 3))
    assert yb.shape == s.shape and bits_equal(yb, ys)
    jni.call("HipFastWaveletTransform_nPlanDestroy", p)


def test_cwt_fft_scalogram_and_direct(jni):
    fb, fc = 1.0, 6.0 / (2 * np.pi)
    x = orc.fill_uniform(3000, 11)  # padded to 4096 (SYMMETRIC, the reference's default)
    scales = np.exp(np.log(2.0) + np.arange(12) * (np.log(512.0) - np.log(2.0)) / 11)
    prm = jni.darray(np.array([fb, fc]))
    rows = jni.read(jni.call("HipContinuousWaveletTransform_nTransformFFT", 0, prm, jni.darray(x),
                             jni.darray(scales), 1.0, 1))
    got = rows[:, 0::2] + 1j * rows[:, 1::2]
    ref = orc.cwt_fft(x, scales, 1.0, "morlet", (fb, fc), 1, exact=True)
    assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-12
    e = jni.read(jni.call("HipContinuousWaveletTransform_nScalogramFFT", 0, prm, jni.darray(x),
                          jni.darray(scales), 1.0, 1))
    eref = np.sum(np.abs(ref) ** 2, axis=1)
    assert np.max(np.abs(e - eref) / eref) < 1e-11
    xs = orc.fill_uniform(256, 12)
    sd = np.array([1.0, 2.5, 8.0])
    rows = jni.read(jni.call("HipContinuousWaveletTransform_nTransformDirect", 1,
                             jni.darray(np.array([1.0])), jni.darray(xs), jni.darray(sd), 1.0, 0))
    refd = orc.cwt_direct(xs, "mexhat", (1.0,), sd)
    assert bits_equal(rows[:, 0::2], refd.real) and bits_equal(rows[:, 1::2], refd.imag)


@pytest.mark.parametrize("padding", [0, 1, 2, 3], ids=["zero", "symmetric", "periodic", "constant"])
@pytest.mark.parametrize("n", [3000, 70001])
def test_cwt_fft_every_padding_non_power_of_two(jni, n, padding):
    # ContinuousWaveletTransform.java:183-229 with each PaddingType (the ordinal the Java
    # drop-in passes, :29-44; SYMMETRIC = 1 is the one-argument constructor's default, :91-93):
    # n = 3000 pads to 4096, n = 70001 to 131072, so the extension is most of the line
    fb, fc = 1.0, 6.0 / (2 * np.pi)
    x = orc.fill_uniform(n, 100 + n + padding)
    scales = np.exp(np.log(2.0) + np.arange(10) * (np.log(1024.0) - np.log(2.0)) / 9)
    prm = jni.darray(np.array([fb, fc]))
    rows = jni.read(jni.call("HipContinuousWaveletTransform_nTransformFFT", 0, prm, jni.darray(x),
                             jni.darray(scales), 1.0, padding))
    assert rows.shape == (len(scales), 2 * n)
    got = rows[:, 0::2] + 1j * rows[:, 1::2]
    ref = orc.cwt_fft(x, scales, 1.0, "morlet", (fb, fc), padding, exact=True)
    assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-12
    # and against JWave's own recurrence-twiddle FFT path, north_star's 1e-10 relative
    jref = orc.cwt_fft(x, scales, 1.0, "morlet", (fb, fc), padding, exact=False)
    assert np.max(np.abs(got - jref)) / np.max(np.abs(jref)) < 1e-10


@pytest.mark.parametrize("n", [1024, 1 << 14, 1000])
def test_fft_strict_matches_reference_fft(jni, n):
    rng = np.random.default_rng(n)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    reim = np.empty(2 * n)
    reim[0::2], reim[1::2] = z.real, z.imag
    out = jni.read(jni.call("HipFastFourierTransform_nFFT", jni.darray(reim), 0, 0))
    ref = orc.fft(z)
    assert bits_equal(out[0::2], ref.real) and bits_equal(out[1::2], ref.imag)
    back = jni.read(jni.call("HipFastFourierTransform_nFFT", jni.darray(out), 1, 0))
    refb = orc.fft(ref, inverse=True)
    assert bits_equal(back[0::2], refb.real) and bits_equal(back[1::2], refb.imag)


def test_engine_device_entries(jni):
    assert jni.call("HipEngine_nDeviceCount") >= 1
    jni.call("HipEngine_nSetDevice", 0)
    with pytest.raises(JavaException) as e:
        jni.call("HipEngine_nSetDevice", 4096)
    assert e.value.cls == "java/lang/IllegalArgumentException" and "out of range" in e.value.msg
    assert jni.call("HipEngine_nReleaseCaches") >= 0


def test_glue_from_threads_on_one_plan(jni):
    # MODWTThreadSafetyTest.java:23-104 through the glue: one shared plan, four threads, each with
    # its own JNIEnv (as a JVM gives them), forward + inverse of its own signals, every result
    # bit-exact against the oracle
    import threading
    wv = W.Daubechies4()
    g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    p = _modwt_plan(jni, wv)
    errors = []
    inputs = {t: orc.fill_uniform(8192 + 512 * t, 100 + t) for t in range(4)}
    refs = {t: orc.modwt_forward(inputs[t], 6, g, h, "direct_nz") for t in range(4)}

    def worker(t):
        env = jni.new_env()
        try:
            for it in range(3):
                method = 0 if it == 2 else 1  # AUTO on the last pass (JWave's FFT path)
                c, exc = jni.call_env(env, "HipMODWTTransform_nForward", p, jni.darray(inputs[t]), 6,
                                      method)
                if exc:
                    errors.append((t, exc))
                    return
                got = jni.read(c)
                ref = refs[t] if method == 1 else orc.modwt_forward(inputs[t], 6, g, h, "auto")
                if not bits_equal(got, ref):
                    errors.append((t, it, "forward differs"))
                xr, exc = jni.call_env(env, "HipMODWTTransform_nInverse", p, jni.matrix(got), method)
                if exc or not bits_equal(jni.read(xr),
                                         orc.modwt_inverse(ref, g, h, "direct_nz" if method == 1
                                                           else "auto")):
                    errors.append((t, it, "inverse differs", exc))
        finally:
            jni.L.mock_env_free(env)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths)
    assert not errors, errors
    jni.call("HipMODWTTransform_nPlanDestroy", p)
