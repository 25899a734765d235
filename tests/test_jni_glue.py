"""The shipped JNI glue (jni/jwave_hip_jni.c), compiled against a mock JNIEnv
(tests/c/jni_mock/, no JDK in this image) into tests/c/libjni_harness.so, on the paths that end
before any device work: argument checks, buffer capacity checks, empty inputs and the mapping
of every C-ABI status to the exception class the reference throws.  CPU only;
tests/test_jni_glue_gpu.py runs the compute entries against the oracle."""
import numpy as np
import pytest

from _jni import Harness, JavaException
from jwave.transforms import wavelets as W

IAE = "java/lang/IllegalArgumentException"
FAILURE = "jwave/exceptions/JWaveFailure"


@pytest.fixture()
def jni():
    h = Harness()
    yield h
    assert h.violations() == 0, "the glue broke a JNI rule (call with an exception pending / null array)"
    h.reset()


def _modwt_plan(jni, wavelet=None):
    wv = wavelet or W.Daubechies4()
    p = jni.call("HipMODWTTransform_nPlanCreate", jni.darray(wv.getScalingDeComposition()),
                 jni.darray(wv.getWaveletDeComposition()), 4096, 0)
    assert p != 0
    return p


def test_plan_create_mismatched_filters_is_iae(jni):
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nPlanCreate", jni.darray(np.ones(8)), jni.darray(np.ones(6)),
                 4096, 0)
    assert e.value.cls == IAE


def test_forward_level_checks_map_to_iae(jni):
    # MODWTTransform.java:257-282: < 1, > 13, > floor(log2 N), checked in that order
    p = _modwt_plan(jni)
    x = jni.darray(np.ones(8))
    for J, text in ((0, "at least 1"), (14, "maximum supported decomposition level is 13"),
                    (4, "exceeds theoretical limit 3 for signal length 8")):
        with pytest.raises(JavaException) as e:
            jni.call("HipMODWTTransform_nForward", p, x, J, 1)
        assert e.value.cls == IAE and text in e.value.msg, e.value
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def test_forward_of_empty_data_gives_empty_rows(jni):
    # MODWTTransform.java:266-273: null / empty data -> maxLevel + 1 empty rows
    p = _modwt_plan(jni)
    for x in (jni.darray(np.zeros(0)), None):
        rows = jni.read_rows(jni.call("HipMODWTTransform_nForward", p, x, 3, 1))
        assert len(rows) == 4 and all(r is not None and r.size == 0 for r in rows)
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def test_inverse_of_empty_or_single_row_is_empty(jni):
    # MODWTTransform.java:338-346: null, no rows, or one row -> new double[0]
    p = _modwt_plan(jni)
    for c in (None, jni.rows([]), jni.rows([np.ones(8)])):
        out = jni.call("HipMODWTTransform_nInverse", p, c, 1)
        got = jni.read(out)
        assert got is not None and got.size == 0
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def test_inverse_ragged_rows_is_iae(jni):
    p = _modwt_plan(jni)
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nInverse", p, jni.rows([np.ones(8), np.ones(7)]), 1)
    assert e.value.cls == IAE and "same length" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nInverse", p, jni.rows([np.ones(8), None]), 1)
    assert e.value.cls == IAE
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def test_direct_buffers_checked_before_the_engine(jni):
    p = _modwt_plan(jni)
    n, J, B = 64, 3, 2
    x = np.zeros(B * n)
    c = np.zeros(B * (J + 1) * n)
    # a coefficient buffer one double short
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nForwardDirect", p, jni.direct(x), jni.direct(c, c.nbytes - 8),
                 n, J, B, 1)
    assert e.value.cls == IAE and "coefficient buffer holds" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nInverseDirect", p, jni.direct(c), jni.direct(x, 8 * n), n, J,
                 B, 1)
    assert e.value.cls == IAE and "signal buffer holds" in e.value.msg
    # a heap (non-direct) buffer: GetDirectBufferAddress gives NULL
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nForwardDirect", p, jni.darray(x), jni.direct(c), n, J, B, 1)
    assert e.value.cls == IAE and "direct ByteBuffers required" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipMODWTTransform_nForwardDirect", p, jni.direct(x), jni.direct(c), -1, J, B, 1)
    assert e.value.cls == IAE
    jni.call("HipMODWTTransform_nPlanDestroy", p)


def _fwt_plan(jni, wv):
    return jni.call("HipFastWaveletTransform_nPlanCreate", jni.darray(wv.getScalingDeComposition()),
                    jni.darray(wv.getWaveletDeComposition()),
                    jni.darray(wv.getScalingReConstruction()),
                    jni.darray(wv.getWaveletReConstruction()), wv.getMotherWavelength(),
                    wv.getTransformWavelength(), 0, 0)


def test_fwt_failures_map_to_jwavefailure(jni):
    # JW_ERR_FAILURE -> the checked jwave.exceptions.JWaveFailure with the reference's text
    # (FastWaveletTransform.java:74-83)
    p = _fwt_plan(jni, W.Daubechies4())
    with pytest.raises(JavaException) as e:
        jni.call("HipFastWaveletTransform_nLine", p, 0, jni.darray(np.ones(12)), 1)
    assert e.value.cls == FAILURE and "given array length is not 2^p" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipFastWaveletTransform_nLine", p, 1, jni.darray(np.ones(8)), 4)
    assert e.value.cls == FAILURE and "given level is out of range" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipFastWaveletTransform_nLine", p, 2, jni.darray(np.ones(8)), 4)
    assert e.value.cls == FAILURE
    with pytest.raises(JavaException) as e:  # 2-D: rows with lvlN first
        jni.call("HipFastWaveletTransform_nMatrix", p, 0, jni.matrix(np.ones((8, 16))), 3, 5)
    assert e.value.cls == FAILURE and "out of range" in e.value.msg
    with pytest.raises(JavaException) as e:  # 3-D: BasicTransform.java:509-565 check order
        jni.call("HipFastWaveletTransform_nSpace", p, 0, jni.space(np.ones((4, 8, 16))), 3, 4, 3)
    assert e.value.cls == FAILURE and "out of range" in e.value.msg
    jni.call("HipFastWaveletTransform_nPlanDestroy", p)


NPE = "java/lang/NullPointerException"
AIOOBE = "java/lang/ArrayIndexOutOfBoundsException"


def test_fwt_space_malformed_throws_what_the_reference_throws(jni):
    # BasicTransform.forward/reverse(double[][][], ...) (:509-528, :602-621) take the shape from
    # spc.length, spc[0].length, spc[0][0].length and copy spc[i][j][k] over that box: a null
    # array or slab throws NullPointerException, an empty one or a slab shorter than slab 0
    # ArrayIndexOutOfBoundsException (the glue threw IllegalArgumentException, or
    # went on with zero dimensions)
    import ctypes
    p = _fwt_plan(jni, W.Haar1())
    for op in (0, 1):
        with pytest.raises(JavaException) as e:
            jni.call("HipFastWaveletTransform_nSpace", p, op, ctypes.c_void_p(None), 1, 1, 1)
        assert e.value.cls == NPE
        with pytest.raises(JavaException) as e:
            jni.call("HipFastWaveletTransform_nSpace", p, op, jni.L.mock_oarray(0, b"[[D"), 1, 1, 1)
        assert e.value.cls == AIOOBE and "Index 0 out of bounds for length 0" in e.value.msg
        with pytest.raises(JavaException) as e:  # spc[0] == null
            jni.call("HipFastWaveletTransform_nSpace", p, op, jni.L.mock_oarray(2, b"[[D"), 1, 1, 1)
        assert e.value.cls == NPE
        with pytest.raises(JavaException) as e:  # spc[0].length == 0: spc[0][0]
            o = jni.L.mock_oarray(2, b"[[D")
            jni.L.mock_oset(o, 0, jni.L.mock_oarray(0, b"[D"))
            jni.call("HipFastWaveletTransform_nSpace", p, op, o, 1, 1, 1)
        assert e.value.cls == AIOOBE
        with pytest.raises(JavaException) as e:  # slab 1 narrower than slab 0
            o = jni.L.mock_oarray(2, b"[[D")
            jni.L.mock_oset(o, 0, jni.matrix(np.ones((4, 8))))
            jni.L.mock_oset(o, 1, jni.matrix(np.ones((4, 4))))
            jni.call("HipFastWaveletTransform_nSpace", p, op, o, 1, 1, 1)
        assert e.value.cls == AIOOBE and "Index 4 out of bounds for length 4" in e.value.msg
        with pytest.raises(JavaException) as e:  # slab 1 with fewer rows
            o = jni.L.mock_oarray(2, b"[[D")
            jni.L.mock_oset(o, 0, jni.matrix(np.ones((4, 8))))
            jni.L.mock_oset(o, 1, jni.matrix(np.ones((2, 8))))
            jni.call("HipFastWaveletTransform_nSpace", p, op, o, 1, 1, 1)
        assert e.value.cls == AIOOBE and "Index 2 out of bounds for length 2" in e.value.msg
        with pytest.raises(JavaException) as e:  # a null slab past the first
            o = jni.L.mock_oarray(2, b"[[D")
            jni.L.mock_oset(o, 0, jni.matrix(np.ones((4, 8))))
            jni.call("HipFastWaveletTransform_nSpace", p, op, o, 1, 1, 1)
        assert e.value.cls == NPE
        # invalid lvlP / lvlQ with a null (or short) later slab: the reference's slab-0 2-D
        # transform throws first (BasicTransform.java:530 / :623), before slab 1 is read
        for bad in (None, np.ones((4, 4))):
            with pytest.raises(JavaException) as e:
                o = jni.L.mock_oarray(2, b"[[D")
                jni.L.mock_oset(o, 0, jni.matrix(np.ones((4, 8))))
                if bad is not None:
                    jni.L.mock_oset(o, 1, jni.matrix(bad))
                jni.call("HipFastWaveletTransform_nSpace", p, op, o, 3, 1, 1)
            assert e.value.cls == FAILURE and "out of range" in e.value.msg
        # invalid lvlR only: reported after every slab was read (the 1-D pass comes last), so
        # the malformed slab's exception wins
        with pytest.raises(JavaException) as e:
            o = jni.L.mock_oarray(2, b"[[D")
            jni.L.mock_oset(o, 0, jni.matrix(np.ones((4, 8))))
            jni.call("HipFastWaveletTransform_nSpace", p, op, o, 1, 1, 5)
        assert e.value.cls == NPE
    jni.call("HipFastWaveletTransform_nPlanDestroy", p)


def test_cwt_parameter_errors_map_to_iae(jni):
    x, sc = jni.darray(np.ones(64)), jni.darray(np.array([1.0, 2.0]))
    with pytest.raises(JavaException) as e:
        jni.call("HipContinuousWaveletTransform_nTransformFFT", 0, jni.darray(np.array([0.0, 1.0])),
                 x, sc, 1.0, 1)
    assert e.value.cls == IAE and "Bandwidth parameter must be positive" in e.value.msg
    with pytest.raises(JavaException) as e:
        jni.call("HipContinuousWaveletTransform_nTransformFFT", 0, jni.darray(np.array([1.0, 1.0])),
                 x, jni.darray(np.array([1.0, -2.0])), 1.0, 1)
    assert e.value.cls == IAE and "Scale must be positive" in e.value.msg


def test_engine_entries_without_a_device(jni):
    v = jni.call("HipEngine_nVersion")
    assert "gfx950" in jni.text(v)
    assert jni.call("HipEngine_nDeviceCount") >= 0
    with pytest.raises(JavaException) as e:
        jni.call("HipEngine_nSetDevice", -1)
    assert e.value.cls == IAE and "must be >= 0" in e.value.msg


def test_unsupported_maps_to_unsupported_operation(jni):
    # JW_ERR_UNSUPPORTED (an FFT level past the engine's FFT range) ->
    # java.lang.UnsupportedOperationException carrying the limit
    wv = W.Daubechies4()
    p = jni.call("HipMODWTTransform_nPlanCreate", jni.darray(wv.getScalingDeComposition()),
                 jni.darray(wv.getWaveletDeComposition()), 4096, 1)  # ARITH_FMA
    n = (1 << 23) + 2
    with pytest.raises(JavaException) as e:  # ConvolutionMethod.FFT past the pyramid's 2^23
        jni.call("HipMODWTTransform_nForward", p, jni.darray(np.zeros(n)), 2, 2)
    assert e.value.cls == "java/lang/UnsupportedOperationException" and "2^23" in e.value.msg
    jni.call("HipMODWTTransform_nPlanDestroy", p)
