"""The C-ABI boundary without a GPU: the library loads, exports every symbol the header
declares, builds plans bit-identical to the oracle's filter cache, and reproduces the
reference's validation order, exception classes and messages (all raised before any
device work).  CPU only.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as orc
from _util import bits_equal
from conftest import ROOT
from jwave import MODWTTransform, FastWaveletTransform, Transform, _native
from jwave.exceptions import IllegalArgumentException, JWaveFailure
from jwave.transforms import wavelets as W

HEADER = os.path.join(ROOT, "include", "jwave_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(jw_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _native.lib()
    declared = header_functions()
    assert declared, "no declarations parsed"
    assert sorted(_native.EXPORTS) == declared
    for name in declared:
        assert hasattr(lib, name), name
    assert b"gfx950" in lib.jw_version()


def test_knobs_read_once_and_overridable(knobs):
    # engine settings: the environment's value, read on first use and not again (a setenv after
    # that changes nothing); jw_set_knob replaces it, None unsets; names outside JW_* refused
    os.environ["JW_TEST_KNOB_A"] = "7"
    assert _native.get_knob("JW_TEST_KNOB_A") == "7"
    os.environ["JW_TEST_KNOB_A"] = "8"
    assert _native.get_knob("JW_TEST_KNOB_A") == "7"
    del os.environ["JW_TEST_KNOB_A"]
    knobs.setenv("JW_TEST_KNOB_A", "9")
    assert _native.get_knob("JW_TEST_KNOB_A") == "9"
    knobs.delenv("JW_TEST_KNOB_A")
    assert _native.get_knob("JW_TEST_KNOB_A") is None
    assert _native.get_knob("JW_TEST_KNOB_NEVER_SET") is None
    with pytest.raises(IllegalArgumentException, match="JW_"):
        _native.set_knob("OMP_NUM_THREADS", "1")
    # host-staging sizes are fixed at first use: refused, never silently ignored
    for fixed in ("JW_PIN_MB", "JW_PIN_RING", "JW_COPY_THREADS"):
        with pytest.raises(IllegalArgumentException, match="fixed at first use"):
            _native.set_knob(fixed, "4")


def test_jni_glue_binds_only_exported_symbols():
    # jni/jwave_hip_jni.c (no JDK here to compile it): every engine call it makes is a declared,
    # exported C-ABI symbol, and every native method of java/jwave/hip/ has its JNI function
    src = open(os.path.join(ROOT, "jni", "jwave_hip_jni.c")).read()
    src_nc = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    called = set(re.findall(r"\b(jw_[a-z0-9_]+)\s*\(", src_nc)) - {"jw_throw"}
    assert called and called <= set(header_functions()), called - set(header_functions())
    lib = _native.lib()
    for name in called:
        assert hasattr(lib, name), name
    jdir = os.path.join(ROOT, "java", "jwave", "hip")
    for f in sorted(os.listdir(jdir)):
        cls = f[:-len(".java")]
        for m in re.findall(r"\bnative\s+[\w\[\]]+\s+(n\w+)\s*\(", open(os.path.join(jdir, f)).read()):
            assert f"Java_jwave_hip_{cls}_{m}(" in src, f"{cls}.{m} has no JNI function"


@pytest.mark.parametrize("wname", W.ORTHONORMAL)
def test_plan_filters_bit_identical_to_oracle(wname):
    # MODWTTransform.initializeFilterCache (:452-484) in the C-ABI plan vs the oracle
    wv = W.by_name(wname)
    g, h = MODWTTransform(wv).getModwtFilters()
    og, oh = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
    assert bits_equal(g, og) and bits_equal(h, oh)


# ---- MODWTTheoreticalLimitTest.java:129-162, MODWTLevelLimitTest.java ----
def test_forward_level_below_one():
    m = MODWTTransform(W.Daubechies4())
    with pytest.raises(IllegalArgumentException, match="at least 1"):
        m.forwardMODWT(np.ones(8), 0)


def test_forward_level_above_13_checked_before_theoretical_limit():
    m = MODWTTransform(W.Daubechies4())
    with pytest.raises(IllegalArgumentException) as e:
        m.forwardMODWT(np.ones(8), 14)
    assert "maximum supported decomposition level is 13" in str(e.value)
    assert "theoretical limit" not in str(e.value)


@pytest.mark.parametrize("n,limit", [(8, 3), (100, 6), (1023, 9), (1024, 10), (1025, 10)])
def test_forward_theoretical_limit(n, limit):
    m = MODWTTransform(W.Haar1())
    with pytest.raises(IllegalArgumentException) as e:
        m.forwardMODWT(np.ones(n), limit + 1)
    msg = str(e.value)
    assert "exceeds theoretical limit" in msg and str(limit) in msg and str(n) in msg


def test_forward_empty_input():
    # MODWTTransformTest.testEmptyInput: J+1 empty rows
    c = MODWTTransform(W.Haar1()).forwardMODWT(np.zeros(0), 3)
    assert len(c) == 4 and all(len(r) == 0 for r in c)


def test_inverse_empty_and_single_row():
    m = MODWTTransform(W.Haar1())
    assert len(m.inverseMODWT(None)) == 0
    assert len(m.inverseMODWT([])) == 0
    assert len(m.inverseMODWT(np.ones((1, 8)))) == 0


def test_inverse_level_above_13():
    m = MODWTTransform(W.Haar1())
    with pytest.raises(IllegalArgumentException, match="maximum supported decomposition level is 13"):
        m.inverseMODWT(np.zeros((15, 16)))


# ---- MODWT1DInterfaceTest.java:107-136 ----
def test_flat_interface_errors():
    m = MODWTTransform(W.Haar1())
    with pytest.raises(JWaveFailure, match=r"2\^p"):
        m.forward(np.ones(7), 1)
    with pytest.raises(JWaveFailure, match="out of range"):
        m.forward(np.ones(8), 4)
    with pytest.raises(JWaveFailure, match="does not match|Invalid coefficient array"):
        m.reverse(np.ones(10), 1)


def test_facade_swallows_checked_exceptions(capsys):
    # Transform.java:81-90: JWaveException -> printed, null returned
    t = Transform(FastWaveletTransform(W.Haar1()))
    assert t.forward(np.ones(6)) is None
    assert "2^p" in capsys.readouterr().out


def test_fwt_validation():
    f = FastWaveletTransform(W.Daubechies4())
    with pytest.raises(JWaveFailure, match="FastWaveletTransform#forward - given array length is not 2"):
        f.forward(np.ones(12), 1)
    with pytest.raises(JWaveFailure, match="given level is out of range"):
        f.forward(np.ones(8), 4)
    with pytest.raises(JWaveFailure, match="FastWaveletTransform#reverse - given level is out of range"):
        f.reverse(np.ones(8), -1)
    with pytest.raises(JWaveFailure, match="WaveletTransform#forward - given array length"):
        f.forward(np.ones(6))


def test_fwt3d_validation_order():
    # BasicTransform.forward(double[][][], lvlP, lvlQ, lvlR) (:509-565) fails at its first
    # 1-D call: slab 0's rows (d3, lvlQ), then its columns (d2, lvlP), then dimension 1
    # (d1, lvlR); the reverse (:602-659) checks slab 0's columns first.
    f = FastWaveletTransform(W.Haar1())
    x = np.zeros((4, 8, 16))
    with pytest.raises(JWaveFailure, match="forward - given level is out of range"):
        f.forward(x, 3, 5, 2)  # lvlQ = 5 > log2 16
    with pytest.raises(JWaveFailure, match="forward - given level is out of range"):
        f.forward(x, 4, 4, 2)  # lvlP = 4 > log2 8
    with pytest.raises(JWaveFailure, match="forward - given level is out of range"):
        f.forward(x, 3, 4, 3)  # lvlR = 3 > log2 4
    with pytest.raises(JWaveFailure, match="given array length is not 2"):
        f.forward(np.zeros((4, 8, 12)), 1, 1, 1)
    with pytest.raises(JWaveFailure, match="reverse - given level is out of range"):
        f.reverse(x, 4, 4, 2)
    # the no-level overload passes log2 of dimensions 1, 2, 3 as (lvlP, lvlQ, lvlR)
    # (:487-495): lvlQ = log2 8 = 3 for the 16-sample rows is fine, lvlP = log2 4 = 2 for
    # the 8-sample columns too, but lvlR = log2 16 = 4 > log2 4 for dimension 1
    with pytest.raises(JWaveFailure, match="forward - given level is out of range"):
        f.forward(x)
    t = Transform(f)
    assert t.forward(x, 4, 4, 2) is None  # facade prints and returns null


def test_precompute_filters_limits():
    m = MODWTTransform(W.Daubechies4())
    with pytest.raises(IllegalArgumentException, match="precomputeFilters - decomposition level must be at least 1"):
        m.precomputeFilters(0)
    with pytest.raises(IllegalArgumentException, match="maximum supported decomposition level is 13"):
        m.precomputeFilters(14)
    assert MODWTTransform.getMaxDecompositionLevel() == 13


def test_raw_capi_rejects_bad_arguments():
    lib = _native.lib()
    plan = ctypes.c_void_p()
    g = np.ones(8)
    assert lib.jw_modwt_plan_create(ctypes.byref(plan), ctypes.c_void_p(g.ctypes.data),
                                    ctypes.c_void_p(g.ctypes.data), 0, 4096, 0) == _native.JW_ERR_ILLEGAL_ARGUMENT
    assert lib.jw_modwt_plan_create(ctypes.byref(plan), ctypes.c_void_p(g.ctypes.data),
                                    ctypes.c_void_p(g.ctypes.data), 8, 4096, 0) == _native.JW_OK
    x = np.ones(16)
    c = np.empty(16 * 3)
    st = lib.jw_modwt_forward(plan, ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(c.ctypes.data),
                              16, 2, 1, 1, 7, None)
    assert st == _native.JW_ERR_ILLEGAL_ARGUMENT and "where" in _native.last_error()
    lib.jw_modwt_plan_destroy(plan)


# ---------------------------------------------------------------- CWT (validation only)
def test_cwt_wavelet_constructor_messages():
    from jwave.transforms.wavelets.continuous import MexicanHatWavelet, MorletWavelet
    with pytest.raises(IllegalArgumentException, match="Bandwidth parameter must be positive"):
        MorletWavelet(0.0, 1.0)
    with pytest.raises(IllegalArgumentException, match="Center frequency must be positive"):
        MorletWavelet(1.0, -1.0)
    with pytest.raises(IllegalArgumentException, match="Width parameter sigma must be positive"):
        MexicanHatWavelet(0.0)
    with pytest.raises(IllegalArgumentException, match="Scale must be positive"):
        MorletWavelet().fourierTransform([1.0], 0.0)


def test_cwt_scale_generators():
    # ContinuousWaveletTransform.generateLogScales / generateLinearScales (:355-405)
    from jwave import ContinuousWaveletTransform as C
    s = C.generateLogScales(2.0, 1024.0, 64)
    assert s[0] == 2.0 and abs(s[-1] - 1024.0) < 1e-9 and len(s) == 64
    assert np.all(np.diff(np.log(s)) > 0)
    assert list(C.generateLinearScales(1.0, 4.0, 4)) == [1.0, 2.0, 3.0, 4.0]
    for args, msg in [((0.0, 1.0, 4), "Scales must be positive"),
                      ((2.0, 1.0, 4), "minScale must be less than maxScale"),
                      ((1.0, 2.0, 1), "Need at least 2 scales")]:
        with pytest.raises(IllegalArgumentException, match=msg):
            C.generateLogScales(*args)


def test_cwt_capi_rejects_bad_arguments():
    L = _native.lib()
    x = np.zeros(8)
    sc = np.array([1.0, -2.0])
    out = np.zeros(2 * 8 * 2)
    p = (ctypes.c_double * 2)(1.0, 1.0)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert L.jw_cwt_fft(0, p, ptr(x), 8, ptr(sc), 2, 1.0, 1, ptr(out), 1, 0, None) == -1
    assert "Scale must be positive" in _native.last_error()
    bad = (ctypes.c_double * 2)(0.0, 1.0)
    assert L.jw_cwt_fft(0, bad, ptr(x), 8, ptr(sc[:1]), 1, 1.0, 1, ptr(out), 1, 0, None) == -1
    assert "Bandwidth parameter must be positive" in _native.last_error()
    assert L.jw_cwt_fft(7, p, ptr(x), 8, ptr(sc[:1]), 1, 1.0, 1, ptr(out), 1, 0, None) == -1
    assert L.jw_cwt_fft(0, p, ptr(x), 8, ptr(sc[:1]), 1, 1.0, 9, ptr(out), 1, 0, None) == -1
    assert "padding" in _native.last_error()
    # empty input is a no-op (no device work)
    assert L.jw_cwt_fft(0, p, ptr(x), 0, ptr(sc[:1]), 1, 1.0, 1, ptr(out), 1, 0, None) == 0


def test_cwt_capi_paul_dog_meyer_validation():
    L = _native.lib()
    x, sc, out = np.zeros(8), np.array([1.0]), np.zeros(2 * 8)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    cases = [(_native.JW_CWT_PAUL, (0.0, 0.0), "Order parameter m must be a positive integer"),
             (_native.JW_CWT_PAUL, (2.5, 0.0), "Order parameter m must be a positive integer"),
             (_native.JW_CWT_PAUL, (21.0, 0.0), "Order parameter m > 20 may cause numerical issues"),
             (_native.JW_CWT_DOG, (0.0, 1.0), "Derivative order n must be a positive integer"),
             (_native.JW_CWT_DOG, (11.0, 1.0), "Derivative order n > 10 may cause numerical issues"),
             (_native.JW_CWT_DOG, (2.0, 0.0), "Width parameter sigma must be positive")]
    for kind, prm, msg in cases:
        p = (ctypes.c_double * 2)(*prm)
        assert L.jw_cwt_fft(kind, p, ptr(x), 8, ptr(sc), 1, 1.0, 1, ptr(out), 1, 0, None) == -1
        assert msg in _native.last_error(), (kind, prm)
    neg = np.array([-1.0])
    p = (ctypes.c_double * 2)(2.0, 1.0)
    for kind in (_native.JW_CWT_DOG, _native.JW_CWT_MEYER):
        assert L.jw_cwt_fft(kind, p, ptr(x), 8, ptr(neg), 1, 1.0, 1, ptr(out), 1, 0, None) == -1
        assert "Scale must be positive" in _native.last_error()
    # Meyer takes no parameters; empty input is a no-op for every kind
    assert L.jw_cwt_fft(_native.JW_CWT_MEYER, None, ptr(x), 0, ptr(sc), 1, 1.0, 1, ptr(out), 1,
                        0, None) == 0
    assert L.jw_cwt_fft(_native.JW_CWT_MEYER + 1, p, ptr(x), 8, ptr(sc), 1, 1.0, 1, ptr(out), 1,
                        0, None) == -1


def test_cwt_direct_scale_validation():
    # computeCoefficient (:240-260) calls wavelet(t, scale, 0) only inside a non-empty window:
    # scale 0 -> "Scale must be positive" (ContinuousWavelet.java:91-93); a negative scale
    # turns the window around and gives zeros without an exception (checked on the GPU)
    from jwave.transforms.cwt import ContinuousWaveletTransform as CWT
    from jwave.transforms.wavelets.continuous import MorletWavelet, PaulWavelet
    for wv in (MorletWavelet(1.0, 1.0), PaulWavelet(4)):
        with pytest.raises(IllegalArgumentException, match="Scale must be positive"):
            CWT(wv).transform(np.ones(16), [2.0, 0.0])
    with pytest.raises(ValueError, match="Scale must be positive"):
        orc.cwt_direct(np.ones(16), "morlet", (1.0, 1.0), [2.0, 0.0])
    assert np.all(orc.cwt_direct(np.ones(16), "morlet", (1.0, 1.0), [-2.0]) == 0)


def test_cwt_direct_oracle_matches_host_closed_forms():
    # the oracle's time-domain psi against the host mirror's closed forms (same formulas)
    import ctypes
    from jwave.transforms.wavelets.continuous import (MorletWavelet, MexicanHatWavelet,
                                                      DOGWavelet)
    for kind, wv in (("morlet", MorletWavelet(1.5, 0.8)), ("mexhat", MexicanHatWavelet(0.7)),
                     ("dog", DOGWavelet(3, 1.2))):
        prm = (ctypes.c_double * 2)(*wv.params())
        for t in (-3.1, -0.4, 0.0, 0.25, 2.9):
            re, im, sup = ctypes.c_double(), ctypes.c_double(), (ctypes.c_double * 2)()
            orc.lib().jwo_cwt_wavelet_t(orc.CWT_KINDS[kind], prm, ctypes.c_double(t),
                                        ctypes.byref(re), ctypes.byref(im), sup)
            ref = complex(wv.wavelet(t))
            assert abs(complex(re.value, im.value) - ref) <= 1e-14 * max(1.0, abs(ref))
            assert list(sup) == list(wv.getEffectiveSupport())


def test_cwt_result_accessors():
    from jwave.transforms import CWTResult
    c = np.array([[1 + 1j, -1 + 0j, 0j, -2 - 2j], [3 - 4j, 0 + 2j, -1 + 1e-300j, 1 - 1j]])
    r = CWTResult(c, [1.0, 2.0], np.arange(4.0), 2.0, "Morlet")
    assert np.allclose(r.getMagnitude()[1, 0], 5.0)
    ph = r.getPhase()  # Complex.getPhi quadrant rules, radians in [0, 2 pi)
    assert np.isclose(ph[0, 0], np.pi / 4) and np.isclose(ph[0, 1], np.pi)
    assert ph[0, 2] == 0.0 and np.isclose(ph[0, 3], 5 * np.pi / 4)
    assert np.isclose(ph[1, 3], 7 * np.pi / 4)
    assert list(r.scaleToFrequency(1.0)) == [2.0, 1.0]
    assert np.allclose(r.getScalogram(), (np.abs(c) ** 2).sum(axis=1))
    assert r.getNumberOfScales() == 2 and r.getNumberOfTimePoints() == 4
    with pytest.raises(IndexError):
        r.getCoefficientsAtScale(2)


def test_wpt_validation_messages():
    # WaveletPacketTransform.java:63-72 / :122-131 (checked JWaveFailure, exact text)
    from jwave import WaveletPacketTransform
    t = WaveletPacketTransform(W.Daubechies4())
    with pytest.raises(JWaveFailure, match="given array length is not 2"):
        t.forward(np.ones(6), 1)
    with pytest.raises(JWaveFailure, match="WaveletPacketTransform#forward - given level is out"):
        t.forward(np.ones(8), 4)
    with pytest.raises(JWaveFailure, match="WaveletPacketTransform#reverse - given level is out"):
        t.reverse(np.ones(8), -1)


def test_cwt_result_abi_validation():
    # jw_cwt_magnitude / jw_cwt_phase / jw_cwt_scalogram: argument checks before any HIP call
    L = _native.lib()
    x = np.zeros(8)
    out = np.zeros(4)
    p = x.ctypes.data_as(ctypes.c_void_p)
    o = out.ctypes.data_as(ctypes.c_void_p)
    assert L.jw_cwt_magnitude(p, -1, o, 0, None) == -1
    assert L.jw_cwt_phase(p, 4, o, 5, None) == -1
    assert L.jw_cwt_scalogram(p, -1, 4, o, 0, None) == -1
    assert L.jw_cwt_scalogram(p, 1, -4, o, 0, None) == -1
    assert L.jw_cwt_magnitude(p, 0, o, 0, None) == 0
    assert L.jw_cwt_scalogram(p, 0, 4, o, 1, None) == 0
    assert L.jw_cwt_magnitude(None, 4, o, 0, None) == -1


def test_device_ordinal_errors():
    # jw_set_device: the C-ABI's device choice for JVM callers that fan out over GPUs
    # (ParallelTransform.java:83-86 style); invalid ordinals are IllegalArgumentException
    lib = _native.lib()
    n = _native.device_count()
    assert n >= 0
    assert lib.jw_set_device(-1) == _native.JW_ERR_ILLEGAL_ARGUMENT
    assert "must be >= 0" in _native.last_error()
    assert lib.jw_set_device(n) == _native.JW_ERR_ILLEGAL_ARGUMENT
    assert f"out of range: {n} HIP device(s) visible" in _native.last_error()
    with pytest.raises(IllegalArgumentException):
        _native.set_device(1 << 20)


def test_release_caches_without_calls():
    # nothing cached yet in this process (no GPU here): frees nothing, never fails
    assert _native.release_caches() >= 0


# ---- no silent method switch past the FFT range (verdict r03: jw_capi.cpp modwt_path) ----
def test_fft_levels_past_2_23_are_unsupported_not_direct():
    # JWave runs these levels through its FFT convolution (MODWTTransform.java:640-664,
    # FastFourierTransform.java:112-164); the engine's FFT paths stop at 2^23, so the call must
    # fail with the limit named instead of returning DIRECT values (~1e-10 away).
    # STRICT (JWave's FFT): powers of two to 2^30, Bluestein to 2^29 (the reference's own int
    # limits); FMA's pyramid: 2^23
    lib = _native.lib()
    J = 2
    vp = ctypes.c_void_p
    for arith, method, n, lim, where in (
            # (2^29 + 1000) * 8 wraps to 8000 > 4096 in the int32 rule: level 1 is FFT
            (_native.JW_ARITH_STRICT, _native.JW_CONV_AUTO, (1 << 29) + 1000, "2^29", _native.JW_DEVICE),
            (_native.JW_ARITH_STRICT, _native.JW_CONV_FFT, (1 << 29) + 1000, "2^29", _native.JW_DEVICE),
            (_native.JW_ARITH_FMA, _native.JW_CONV_FFT, (1 << 23) + 2, "2^23", _native.JW_HOST)):
        # JW_HOST: calloc'd, untouched pages; JW_DEVICE: the range check precedes every access
        x = np.zeros(n if where == _native.JW_HOST else 1)
        c = np.zeros((J + 1) * n if where == _native.JW_HOST else 1)
        wv = W.Daubechies4()
        sd, wd = np.asarray(wv.getScalingDeComposition()), np.asarray(wv.getWaveletDeComposition())
        plan = vp()
        assert lib.jw_modwt_plan_create(ctypes.byref(plan), vp(sd.ctypes.data), vp(wd.ctypes.data),
                                        8, 4096, arith) == _native.JW_OK
        for fn, a, b in ((lib.jw_modwt_forward, x, c), (lib.jw_modwt_inverse, c, x)):
            st = fn(plan, vp(a.ctypes.data), vp(b.ctypes.data), n, J, 1, method, where, None)
            assert st == _native.JW_ERR_UNSUPPORTED, (arith, method, st)
            msg = _native.last_error()
            assert lim in msg and str(n) in msg and "level 1" in msg, msg
        lib.jw_modwt_plan_destroy(plan)
        del x, c
    # the Python mirror raises it (NotImplementedError), never a DIRECT result
    m = MODWTTransform(W.Daubechies4(), arith="fma")
    m.setConvolutionMethod(MODWTTransform.ConvolutionMethod.FFT)
    with pytest.raises(NotImplementedError, match="2\\^23"):
        m.forwardMODWT(np.zeros((1 << 23) + 2), J)


def test_strict_fft_past_its_range_is_unsupported():
    # STRICT runs the reference's FFT for powers of two up to 2^30 (three column passes past
    # 2^24) and Bluestein up to 2^29 (m <= 2^30) -- the reference's own domain: a Java array
    # holds at most 2^30 as a power of two, and its Bluestein `int m` doubling overflows past
    # n = 2^29 (FastFourierTransform.java:261-265); past those, an error naming the limits
    lib = _native.lib()
    vp = ctypes.c_void_p
    z = np.zeros(2)  # JW_DEVICE: the range check precedes every access
    for n in ((1 << 29) + 1, (1 << 30) - 1, 1 << 31):
        st = lib.jw_fft_forward_ex(vp(z.ctypes.data), vp(z.ctypes.data), n, 1,
                                   _native.JW_ARITH_STRICT, _native.JW_DEVICE, None)
        msg = _native.last_error()
        assert st == _native.JW_ERR_UNSUPPORTED and "2^30" in msg and "2^29" in msg, msg
        assert "(1073741824)" in msg and "(536870912)" in msg, msg


def test_strict_range_contains_the_pyramid_range():
    # verdict r04 item 6: a STRICT level outside JWave's FFT range is JW_ERR_UNSUPPORTED, never
    # the FMA pyramid; that is sound only while the STRICT range contains the pyramid's
    # (static_assert in jw_internal.hpp).  Read both limits back from the C-ABI's own messages.
    lib = _native.lib()
    vp = ctypes.c_void_p
    wv = W.Daubechies4()
    sd, wd = np.asarray(wv.getScalingDeComposition()), np.asarray(wv.getWaveletDeComposition())
    n = (1 << 30) + 2
    x = np.zeros(1)
    msgs = {}
    for arith in (_native.JW_ARITH_STRICT, _native.JW_ARITH_FMA):
        plan = vp()
        assert lib.jw_modwt_plan_create(ctypes.byref(plan), vp(sd.ctypes.data), vp(wd.ctypes.data),
                                        8, 4096, arith) == _native.JW_OK
        # the range check precedes every read of the buffers (JW_DEVICE: nothing is staged)
        st = lib.jw_modwt_forward(plan, vp(x.ctypes.data), vp(x.ctypes.data), n, 1, 1,
                                  _native.JW_CONV_FFT, _native.JW_DEVICE, None)
        assert st == _native.JW_ERR_UNSUPPORTED
        msgs[arith] = _native.last_error()
        lib.jw_modwt_plan_destroy(plan)
    lim = {a: [int(v) for v in re.findall(r"\((\d+)\)", m)] for a, m in msgs.items()}
    pow2_max, other_max = lim[_native.JW_ARITH_STRICT]
    (pyr_max,) = lim[_native.JW_ARITH_FMA]
    assert (pow2_max, other_max, pyr_max) == (1 << 30, 1 << 29, 1 << 23)
    assert pyr_max <= other_max <= pow2_max


def test_cwt_fft_paths_reports_the_split(knobs):
    # jw_cwt_fft_paths: the scale split jw_cwt_fft takes (host rule, no device work).  cfg3
    # (Morlet omega0 = 6, 64 log scales 2..1024, N = 2^18): 22 two-pass scales and 42 on coarse
    # grids; without coarse grids the band scales go to the band kernel
    import ctypes
    import math
    from jwave import ContinuousWaveletTransform as CWT
    lib = _native.lib()
    scales = np.ascontiguousarray(CWT.generateLogScales(2.0, 1024.0, 64), dtype=np.float64)
    params = (ctypes.c_double * 2)(1.0, 6.0 / (2 * math.pi))
    out = [ctypes.c_int(-1) for _ in range(3)]

    def split(n):
        _native.check(lib.jw_cwt_fft_paths(_native.JW_CWT_MORLET, params, n,
                                           scales.ctypes.data_as(ctypes.c_void_p), 64, 1.0,
                                           *[ctypes.byref(o) for o in out]))
        return tuple(o.value for o in out)

    assert split(1 << 18) == (22, 0, 42)
    knobs.setenv("JW_CWT_INTERP", "0")
    t, b, c = split(1 << 18)
    assert c == 0 and t + b == 64 and b > 0
    knobs.setenv("JW_CWT_BAND", "0")
    assert split(1 << 18) == (64, 0, 0)
    assert split(1000) == (64, 0, 0)  # N = 1024 < 8192: no band paths at all
    with pytest.raises(IllegalArgumentException):
        _native.check(lib.jw_cwt_fft_paths(_native.JW_CWT_MORLET, params, -1, None, 64, 1.0,
                                           *[ctypes.byref(o) for o in out]))
