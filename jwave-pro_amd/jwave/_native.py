"""ctypes binding of libjwave_hip.so (the C-ABI in include/jwave_hip.h).

The HIP engine is the only compute path: if the shared library is missing or cannot be
loaded, every transform raises instead of falling back to anything on the CPU.
"""
import ctypes
import os

from .exceptions import IllegalArgumentException, JWaveError, JWaveFailure

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JWAVE_HIP_LIB", os.path.join(os.path.dirname(_HERE), "libjwave_hip.so"))

JW_OK = 0
JW_ERR_ILLEGAL_ARGUMENT = -1
JW_ERR_FAILURE = -2
JW_ERR_DEVICE = -3
JW_ERR_NO_MEMORY = -4
JW_ERR_UNSUPPORTED = -5

JW_HOST = 0
JW_DEVICE = 1

JW_CWT_MORLET = 0
JW_CWT_MEXHAT = 1
JW_CWT_PAUL = 2
JW_CWT_DOG = 3
JW_CWT_MEYER = 4
JW_PAD_ZERO = 0
JW_PAD_SYMMETRIC = 1
JW_PAD_PERIODIC = 2
JW_PAD_CONSTANT = 3

JW_CONV_AUTO = 0
JW_CONV_DIRECT = 1
JW_CONV_FFT = 2

JW_ARITH_STRICT = 0
JW_ARITH_FMA = 1

JW_WAVELET_GENERIC = 0
JW_WAVELET_HAAR_ORTH = 1

# Every symbol include/jwave_hip.h declares (checked by
# tests/test_capi.py::test_library_exports_every_header_symbol).
EXPORTS = (
    "jw_last_error", "jw_version", "jw_device_count", "jw_set_device", "jw_get_device",
    "jw_release_caches", "jw_set_knob", "jw_get_knob",
    "jw_modwt_plan_create", "jw_modwt_plan_destroy", "jw_modwt_plan_filters",
    "jw_modwt_forward", "jw_modwt_inverse",
    "jw_fwt_plan_create", "jw_fwt_plan_destroy", "jw_fwt_forward", "jw_fwt_reverse",
    "jw_fwt2d_forward", "jw_fwt2d_reverse", "jw_fwt3d_forward", "jw_fwt3d_reverse",
    "jw_synth_uniform", "jw_cwt_fft", "jw_cwt_direct", "jw_wpt_forward", "jw_wpt_reverse",
    "jw_fft_forward", "jw_fft_reverse", "jw_fft_forward_ex", "jw_fft_reverse_ex", "jw_cwt_magnitude", "jw_cwt_phase", "jw_cwt_scalogram",
    "jw_cwt_fft_scalogram", "jw_cwt_fft_paths",
)

_lib = None


def _prepare_runtime():
    # torch bundles its own libamdhip64.so.7; importing torch first makes our library bind to
    # the already-loaded runtime (same SONAME), so device pointers are shared between them.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is optional for host-only use
        pass


def lib():
    """Load (once) and return the ctypes handle; raises if the HIP engine is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise JWaveError(f"HIP engine not built: {LIB_PATH} is missing (run __graft_entry__.build())")
    _prepare_runtime()
    L = ctypes.CDLL(LIB_PATH)
    c_dp = ctypes.c_void_p
    i, l = ctypes.c_int, ctypes.c_long
    L.jw_last_error.restype = ctypes.c_char_p
    L.jw_last_error.argtypes = []
    L.jw_version.restype = ctypes.c_char_p
    L.jw_version.argtypes = []
    L.jw_device_count.argtypes = [ctypes.POINTER(i)]
    L.jw_set_device.argtypes = [i]
    L.jw_get_device.argtypes = [ctypes.POINTER(i)]
    L.jw_release_caches.argtypes = []
    L.jw_release_caches.restype = l
    L.jw_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.jw_get_knob.argtypes = [ctypes.c_char_p]
    L.jw_get_knob.restype = ctypes.c_char_p
    L.jw_modwt_plan_create.argtypes = [ctypes.POINTER(c_dp), c_dp, c_dp, i, i, i]
    L.jw_modwt_plan_destroy.argtypes = [c_dp]
    L.jw_modwt_plan_destroy.restype = None
    L.jw_modwt_plan_filters.argtypes = [c_dp, c_dp, c_dp]
    L.jw_modwt_forward.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, i, c_dp]
    L.jw_modwt_inverse.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, i, c_dp]
    L.jw_fwt_plan_create.argtypes = [ctypes.POINTER(c_dp), c_dp, c_dp, c_dp, c_dp, i, i, i, i]
    L.jw_fwt_plan_destroy.argtypes = [c_dp]
    L.jw_fwt_plan_destroy.restype = None
    L.jw_fwt_forward.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_fwt_reverse.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_wpt_forward.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_wpt_reverse.argtypes = [c_dp, c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_fwt2d_forward.argtypes = [c_dp, c_dp, c_dp, i, i, i, i, i, i, c_dp]
    L.jw_fwt2d_reverse.argtypes = [c_dp, c_dp, c_dp, i, i, i, i, i, i, c_dp]
    L.jw_fwt3d_forward.argtypes = [c_dp, c_dp, c_dp, i, i, i, i, i, i, i, i, c_dp]
    L.jw_fwt3d_reverse.argtypes = [c_dp, c_dp, c_dp, i, i, i, i, i, i, i, i, c_dp]
    L.jw_synth_uniform.argtypes = [c_dp, l, i, l, c_dp]
    L.jw_fft_forward.argtypes = [c_dp, c_dp, l, i, i, c_dp]
    L.jw_fft_reverse.argtypes = [c_dp, c_dp, l, i, i, c_dp]
    L.jw_fft_forward_ex.argtypes = [c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_fft_reverse_ex.argtypes = [c_dp, c_dp, l, i, i, i, c_dp]
    L.jw_cwt_fft.argtypes = [i, c_dp, c_dp, l, c_dp, i, ctypes.c_double, i, c_dp, i, i, c_dp]
    L.jw_cwt_direct.argtypes = [i, c_dp, c_dp, l, c_dp, i, ctypes.c_double, i, c_dp, i, i, c_dp]
    L.jw_cwt_magnitude.argtypes = [c_dp, l, c_dp, i, c_dp]
    L.jw_cwt_phase.argtypes = [c_dp, l, c_dp, i, c_dp]
    L.jw_cwt_scalogram.argtypes = [c_dp, l, l, c_dp, i, c_dp]
    L.jw_cwt_fft_scalogram.argtypes = [i, c_dp, c_dp, l, c_dp, i, ctypes.c_double, i, c_dp, i, i,
                                       c_dp]
    c_ip = ctypes.POINTER(ctypes.c_int)
    L.jw_cwt_fft_paths.argtypes = [i, c_dp, l, c_dp, i, ctypes.c_double, c_ip, c_ip, c_ip]
    non_int = ("jw_last_error", "jw_version", "jw_modwt_plan_destroy", "jw_fwt_plan_destroy",
               "jw_release_caches", "jw_get_knob")
    for name in EXPORTS:
        if name not in non_int:
            getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def set_knob(name, value):
    """jw_set_knob: an engine setting (JW_*, A/B runs and tests) for later calls; None = unset."""
    check(lib().jw_set_knob(name.encode(), None if value is None else str(value).encode()))


def get_knob(name):
    v = lib().jw_get_knob(name.encode())
    return None if v is None else v.decode()


def last_error():
    return lib().jw_last_error().decode()


def check(status):
    """Map a C-ABI status to the reference's exception classes."""
    if status == JW_OK:
        return
    msg = last_error()
    if status == JW_ERR_ILLEGAL_ARGUMENT:
        raise IllegalArgumentException(msg)
    if status == JW_ERR_FAILURE:
        raise JWaveFailure(msg)
    if status == JW_ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise JWaveError(f"HIP engine error {status}: {msg}")


def set_device(ordinal):
    """jw_set_device: the calling thread's device for every later call."""
    check(lib().jw_set_device(int(ordinal)))


def device_count():
    n = ctypes.c_int(0)
    check(lib().jw_device_count(ctypes.byref(n)))
    return n.value


def release_caches():
    """jw_release_caches: free every cached device table (MODWTTransform.clearFilterCache's
    device-side counterpart); returns the bytes freed."""
    return int(lib().jw_release_caches())
