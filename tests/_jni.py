"""ctypes driver for tests/c/libjni_harness.so: the shipped JNI glue (jni/jwave_hip_jni.c)
linked with a mock JNIEnv (tests/c/jni_mock/).  Builds Java arrays / direct buffers in C
memory, calls the glue's Java_jwave_hip_* functions as a JVM would, and reads results and
pending exceptions back.  Test infrastructure only."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "c", "libjni_harness.so")

vp, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double

# the native methods of java/jwave/hip/*.java: name -> (restype, argtypes after env, class)
_SIGS = {
    "HipEngine_nVersion": (vp, []),
    "HipEngine_nSetDevice": (None, [i32]),
    "HipEngine_nDeviceCount": (i32, []),
    "HipEngine_nReleaseCaches": (i64, []),
    "HipMODWTTransform_nPlanCreate": (i64, [vp, vp, i32, i32]),
    "HipMODWTTransform_nPlanDestroy": (None, [i64]),
    "HipMODWTTransform_nForward": (vp, [i64, vp, i32, i32]),
    "HipMODWTTransform_nInverse": (vp, [i64, vp, i32]),
    "HipMODWTTransform_nForwardDirect": (None, [i64, vp, vp, i64, i32, i32, i32]),
    "HipMODWTTransform_nInverseDirect": (None, [i64, vp, vp, i64, i32, i32, i32]),
    "HipFastWaveletTransform_nPlanCreate": (i64, [vp, vp, vp, vp, i32, i32, i32, i32]),
    "HipFastWaveletTransform_nPlanDestroy": (None, [i64]),
    "HipFastWaveletTransform_nLine": (vp, [i64, i32, vp, i32]),
    "HipFastWaveletTransform_nMatrix": (vp, [i64, i32, vp, i32, i32]),
    "HipFastWaveletTransform_nSpace": (vp, [i64, i32, vp, i32, i32, i32]),
    "HipContinuousWaveletTransform_nTransformFFT": (vp, [i32, vp, vp, vp, f64, i32]),
    "HipContinuousWaveletTransform_nScalogramFFT": (vp, [i32, vp, vp, vp, f64, i32]),
    "HipContinuousWaveletTransform_nTransformDirect": (vp, [i32, vp, vp, vp, f64, i32]),
    "HipFastFourierTransform_nFFT": (vp, [vp, i32, i32]),
}


class JavaException(Exception):
    def __init__(self, cls, msg):
        super().__init__(f"{cls}: {msg}")
        self.cls, self.msg = cls, msg


class Harness:
    def __init__(self):
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} is built by __graft_entry__.build()")
        from jwave import _native
        _native.lib()  # libjwave_hip.so bound to torch's HIP runtime first
        L = ctypes.CDLL(LIB_PATH)
        self.L = L
        L.mock_env_new.restype = vp
        L.mock_darray.restype = vp
        L.mock_darray.argtypes = [vp, i32]
        L.mock_oarray.restype = vp
        L.mock_oarray.argtypes = [i32, ctypes.c_char_p]
        L.mock_oset.argtypes = [vp, i32, vp]
        L.mock_oget.restype = vp
        L.mock_oget.argtypes = [vp, i32]
        L.mock_direct.restype = vp
        L.mock_direct.argtypes = [vp, i64]
        L.mock_length.restype = i32
        L.mock_length.argtypes = [vp]
        L.mock_kind.argtypes = [vp]
        L.mock_text.restype = ctypes.c_char_p
        L.mock_text.argtypes = [vp]
        L.mock_darray_read.argtypes = [vp, vp]
        L.mock_exception.argtypes = [vp, ctypes.c_char_p, i32, ctypes.c_char_p, i32]
        L.mock_env_free.argtypes = [vp]
        self.env = vp(L.mock_env_new())
        self.fns = {}
        for name, (res, args) in _SIGS.items():
            f = getattr(L, "Java_jwave_hip_" + name)
            f.restype = res
            f.argtypes = [vp, vp] + args
            self.fns[name] = f

    # ---- Java objects
    def darray(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64).ravel()
        return vp(self.L.mock_darray(a.ctypes.data if a.size else None, a.size))

    def matrix(self, m):
        m = np.asarray(m, dtype=np.float64)
        o = vp(self.L.mock_oarray(m.shape[0], b"[D"))
        for r in range(m.shape[0]):
            self.L.mock_oset(o, r, self.darray(m[r]))
        return o

    def rows(self, rows):
        """double[][] from a list of 1-D arrays (ragged allowed), None entries = null rows."""
        o = vp(self.L.mock_oarray(len(rows), b"[D"))
        for r, row in enumerate(rows):
            self.L.mock_oset(o, r, None if row is None else self.darray(row))
        return o

    def space(self, s):
        s = np.asarray(s, dtype=np.float64)
        o = vp(self.L.mock_oarray(s.shape[0], b"[[D"))
        for i in range(s.shape[0]):
            self.L.mock_oset(o, i, self.matrix(s[i]))
        return o

    def direct(self, arr, capacity_bytes=None):
        cap = arr.nbytes if capacity_bytes is None else capacity_bytes
        return vp(self.L.mock_direct(arr.ctypes.data, cap))

    def read(self, obj):
        """double[] / double[][] / double[][][] -> ndarray (None for a null reference)."""
        if not obj:
            return None
        n = self.L.mock_length(obj)
        if self.L.mock_kind(obj) == 1:  # double[]
            out = np.empty(n)
            self.L.mock_darray_read(obj, out.ctypes.data if n else None)
            return out
        return np.array([self.read(vp(self.L.mock_oget(obj, i))) for i in range(n)])

    def read_rows(self, obj):
        n = self.L.mock_length(obj)
        return [self.read(vp(self.L.mock_oget(obj, i))) for i in range(n)]

    def text(self, obj):
        return self.L.mock_text(obj).decode()

    # ---- calls
    def exception(self):
        cls, msg = ctypes.create_string_buffer(128), ctypes.create_string_buffer(512)
        if self.L.mock_exception(self.env, cls, 128, msg, 512):
            return cls.value.decode(), msg.value.decode()
        return None

    def new_env(self):
        """A separate JNIEnv (a JVM gives every thread its own)."""
        return vp(self.L.mock_env_new())

    def call_env(self, env, name, *args):
        """call() on a given environment (per-thread use); returns (result, exception or None)."""
        r = self.fns[name](env, None, *args)
        cls, msg = ctypes.create_string_buffer(128), ctypes.create_string_buffer(512)
        if self.L.mock_exception(env, cls, 128, msg, 512):
            return r, (cls.value.decode(), msg.value.decode())
        return r, None

    def call(self, name, *args):
        """Calls Java_jwave_hip_<name>(env, class, *args); raises JavaException when the glue
        left one pending (and asserts it returned nothing then)."""
        r = self.fns[name](self.env, None, *args)
        exc = self.exception()
        if exc:
            assert not r, f"{name} returned a value with an exception pending"
            raise JavaException(*exc)
        return r

    def violations(self):
        return self.L.mock_violations()

    def reset(self):
        self.L.mock_reset()
