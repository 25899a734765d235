"""MODWT host mirror: jwave.transforms.MODWTTransform on the MI355X.

Same names, argument meaning and error behaviour as the reference
(src/main/java/jwave/transforms/MODWTTransform.java).  The filter cache
(initializeFilterCache :452-484) lives in the immutable C-ABI plan; the pyramid and its
adjoint run in the HIP engine (jw_modwt_forward / jw_modwt_inverse).  Extension beyond
the Java API: ``forwardMODWT`` / ``inverseMODWT`` also accept a batch (B x N) /
(B x (J+1) x N), and HIP-device torch tensors (computed in place on HBM, no copies).
"""
import ctypes
import enum
import threading

import numpy as np

from .. import _native
from .._arrays import as_input
from ..exceptions import IllegalArgumentException, JWaveFailure
from .fwt import WaveletTransform, _is_binary

MAX_DECOMPOSITION_LEVEL = 13  # MODWTTransform.java:111


class ConvolutionMethod(enum.IntEnum):  # MODWTTransform.java:149-153
    AUTO = _native.JW_CONV_AUTO
    DIRECT = _native.JW_CONV_DIRECT
    FFT = _native.JW_CONV_FFT


class MODWTTransform(WaveletTransform):
    """jwave.transforms.MODWTTransform"""

    ConvolutionMethod = ConvolutionMethod

    def __init__(self, wavelet, fftThreshold=4096, arith="strict"):
        super().__init__(wavelet)
        self._name = "MODWT"
        self.fftConvolutionThreshold = int(fftThreshold)
        self._convolutionMethod = ConvolutionMethod.AUTO
        self._arith = _native.JW_ARITH_FMA if arith == "fma" else _native.JW_ARITH_STRICT
        self._lock = threading.Lock()
        self._plan = None
        self._retired = []  # plans dropped by clearFilterCache; other threads may still use them

    def __del__(self):
        if _native._lib is None:
            return
        for plan in [getattr(self, "_plan", None)] + getattr(self, "_retired", []):
            if plan:
                _native._lib.jw_modwt_plan_destroy(plan)

    # ---- configuration ----
    def setConvolutionMethod(self, method):
        self._convolutionMethod = ConvolutionMethod(method)

    def getConvolutionMethod(self):
        return self._convolutionMethod

    @staticmethod
    def getMaxDecompositionLevel():
        return MAX_DECOMPOSITION_LEVEL

    # ---- filter cache (:452-630) ----
    def initializeFilterCache(self):
        with self._lock:
            if self._plan is None:
                L = _native.lib()
                g = np.ascontiguousarray(self._wavelet.getScalingDeComposition(), dtype=np.float64)
                h = np.ascontiguousarray(self._wavelet.getWaveletDeComposition(), dtype=np.float64)
                plan = ctypes.c_void_p()
                _native.check(L.jw_modwt_plan_create(ctypes.byref(plan),
                                                     ctypes.c_void_p(g.ctypes.data),
                                                     ctypes.c_void_p(h.ctypes.data), len(g),
                                                     self.fftConvolutionThreshold, self._arith))
                self._plan = plan
            return self._plan

    def clearFilterCache(self):
        # Plans are immutable and may be in use by another thread (MODWTThreadSafetyTest), so
        # clearing retires ours until this object dies; a new one is built lazily.
        with self._lock:
            if self._plan is not None:
                self._retired.append(self._plan)
            self._plan = None

    def precomputeFilters(self, maxLevel):
        if maxLevel < 1:
            raise IllegalArgumentException(
                "MODWTTransform#precomputeFilters - decomposition level must be at least 1, "
                f"requested: {maxLevel}")
        if maxLevel > MAX_DECOMPOSITION_LEVEL:
            raise IllegalArgumentException(
                "MODWTTransform#precomputeFilters - maximum supported decomposition level is "
                f"{MAX_DECOMPOSITION_LEVEL}, requested: {maxLevel}")
        self.initializeFilterCache()

    def getModwtFilters(self):
        """The cached base filters (g_modwt_base, h_modwt_base)."""
        plan = self.initializeFilterCache()
        L = self._wavelet.getMotherWavelength()
        g = np.empty(L)
        h = np.empty(L)
        _native.check(_native.lib().jw_modwt_plan_filters(plan, ctypes.c_void_p(g.ctypes.data),
                                                          ctypes.c_void_p(h.ctypes.data)))
        return g, h

    # ---- forwardMODWT / inverseMODWT (:256-375) ----
    def forwardMODWT(self, data, maxLevel):
        maxLevel = int(maxLevel)
        if maxLevel < 1:
            raise IllegalArgumentException(
                "MODWTTransform#forwardMODWT - decomposition level must be at least 1, "
                f"requested: {maxLevel}")
        if maxLevel > MAX_DECOMPOSITION_LEVEL:
            raise IllegalArgumentException(
                "MODWTTransform#forwardMODWT - maximum supported decomposition level is "
                f"{MAX_DECOMPOSITION_LEVEL}, requested: {maxLevel}")
        if data is None or len(data) == 0:
            return np.zeros((maxLevel + 1, 0))
        a = as_input(data)
        batch = len(a.shape) == 2
        B, N = (a.shape[0], a.shape[1]) if batch else (1, a.shape[0])
        plan = self.initializeFilterCache()
        out = a.empty((B, maxLevel + 1, N) if batch else (maxLevel + 1, N))
        _native.check(_native.lib().jw_modwt_forward(plan, a.ptr, out.ptr, N, maxLevel, B,
                                                     int(self._convolutionMethod), a.where,
                                                     a.stream))
        return out.result()

    def inverseMODWT(self, coefficients):
        if coefficients is None or len(coefficients) == 0:
            return np.zeros(0)
        if isinstance(coefficients, (list, tuple)):
            coefficients = np.asarray([np.asarray(r, dtype=np.float64) for r in coefficients])
        a = as_input(coefficients)
        batch = len(a.shape) == 3
        if batch:
            B, rows, N = a.shape
        else:
            B, (rows, N) = 1, a.shape
        maxLevel = rows - 1
        if maxLevel <= 0:
            return np.zeros(0)
        plan = self.initializeFilterCache()
        out = a.empty((B, N) if batch else (N,))
        _native.check(_native.lib().jw_modwt_inverse(plan, a.ptr, out.ptr, N, maxLevel, B,
                                                     int(self._convolutionMethod), a.where,
                                                     a.stream))
        return out.result()

    # ---- flattened 1-D interface (:388-443, :853-912) ----
    def forward(self, arrTime, level=None):
        if arrTime is None or len(arrTime) == 0:
            return np.zeros(0)
        n = len(arrTime)
        if level is None:  # forward(double[]) :853-874 -- full depth, no 2^p check first
            maxLevel = self.calcExponent(n)
            return np.asarray(self.forwardMODWT(arrTime, maxLevel)).reshape(-1)
        if not _is_binary(n):
            raise JWaveFailure("MODWTTransform#forward - given array length is not 2^p | p E N "
                               "... = 1, 2, 4, 8, 16, 32, .. ")
        maxLevel = self.calcExponent(n)
        if level < 0 or level > maxLevel:
            raise JWaveFailure("MODWTTransform#forward - given level is out of range for given "
                               "array")
        if level > MAX_DECOMPOSITION_LEVEL:
            raise JWaveFailure("MODWTTransform#forward - maximum supported decomposition level "
                               f"is {MAX_DECOMPOSITION_LEVEL}, requested: {level}")
        return np.asarray(self.forwardMODWT(arrTime, level)).reshape(-1)

    def reverse(self, arrHilb, level=None):
        if arrHilb is None or len(arrHilb) == 0:
            return np.zeros(0)
        arr = np.asarray(arrHilb, dtype=np.float64)
        total = arr.shape[0]
        if level is None:  # reverse(double[]) :876-912 -- smallest-N inference
            N = 0
            levels = 0
            for testN in range(1, total + 1):
                if total % testN == 0:
                    testLevels = total // testN - 1
                    if testLevels >= 0 and _is_binary(testN) and testLevels <= self.calcExponent(testN):
                        N, levels = testN, testLevels
                        break
            if N == 0:
                raise JWaveFailure("MODWTTransform#reverse - Invalid flattened coefficient array "
                                   "length. Cannot determine original signal dimensions.")
            return self.inverseMODWT(arr.reshape(levels + 1, N))
        N = total // (level + 1)
        if not _is_binary(N):
            raise JWaveFailure("MODWTTransform#reverse - Invalid coefficient array for given level")
        if total != N * (level + 1):
            raise JWaveFailure("MODWTTransform#reverse - Coefficient array length does not match "
                               "expected size for given level")
        return self.inverseMODWT(arr.reshape(level + 1, N))
