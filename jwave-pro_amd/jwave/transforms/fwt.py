"""FWT host mirror: BasicTransform / WaveletTransform / FastWaveletTransform.

Same names, argument meaning and error behaviour as the reference
(src/main/java/jwave/transforms/BasicTransform.java, WaveletTransform.java:77-182,
FastWaveletTransform.java:71-153); the cascade itself runs in the HIP engine
(jw_fwt_* in include/jwave_hip.h).  Extensions beyond the Java API are the batched
``forwardBatch`` / ``reverseBatch`` / ``forward2DBatch`` / ``reverse2DBatch``.
"""
import ctypes
import math

import numpy as np

from .. import _native
from .._arrays import as_input
from ..exceptions import JWaveFailure


def _is_binary(n):  # MathToolKit.isBinary :185-188
    return n > 0 and (n & (n - 1)) == 0


def _get_exponent(f):  # MathToolKit.getExponent :202-206: (int)(log f / log 2)
    return int(math.log(f) / math.log(2.))


class BasicTransform:
    """jwave.transforms.BasicTransform (abstract)."""

    _name = None

    def getName(self):
        return self._name

    def isBinary(self, number):
        return _is_binary(number)

    def calcExponent(self, number):  # BasicTransform.java:688-697
        if not _is_binary(number):
            raise JWaveFailure("BasicTransform#calcExponent - given number is not binary: "
                               "2^p | pEN .. = 1, 2, 4, 8, 16, 32, .. ")
        return _get_exponent(number)


class WaveletTransform(BasicTransform):
    """jwave.transforms.WaveletTransform (abstract, holds the wavelet)."""

    def __init__(self, wavelet):
        self._wavelet = wavelet

    def getWavelet(self):
        return self._wavelet


class FastWaveletTransform(WaveletTransform):
    """jwave.transforms.FastWaveletTransform -- the FWT cascade on the MI355X."""

    def __init__(self, wavelet, arith="strict"):
        super().__init__(wavelet)
        self._name = "Fast Wavelet Transform"
        self._arith = _native.JW_ARITH_FMA if arith == "fma" else _native.JW_ARITH_STRICT
        L = _native.lib()
        M = wavelet.getMotherWavelength()
        arrs = [np.ascontiguousarray(f, dtype=np.float64)
                for f in (wavelet.getScalingDeComposition(), wavelet.getWaveletDeComposition(),
                          wavelet.getScalingReConstruction(), wavelet.getWaveletReConstruction())]
        self._plan = ctypes.c_void_p()
        _native.check(L.jw_fwt_plan_create(ctypes.byref(self._plan),
                                           *[ctypes.c_void_p(a.ctypes.data) for a in arrs], M,
                                           wavelet.getTransformWavelength(),
                                           getattr(wavelet, "kind", 0), self._arith))

    def __del__(self):
        plan = getattr(self, "_plan", None)
        if plan and _native._lib is not None:
            _native._lib.jw_fwt_plan_destroy(plan)

    # ---- 1-D (WaveletTransform.forward/reverse(double[]) :77-112, FWT :71-153) ----
    def forward(self, arr, level=None, lvlN=None, lvlR=None):
        if lvlR is not None:  # forward(double[][][], lvlP, lvlQ, lvlR)
            return self._forward3d(arr, level, lvlN, lvlR)
        if lvlN is not None:  # forward(double[][], lvlM, lvlN)
            return self._forward2d(arr, level, lvlN)
        a = as_input(arr)
        if len(a.shape) == 3:  # forward(double[][][]) (BasicTransform.java:487-495)
            return self._forward3d(arr, *(_get_exponent(d) for d in a.shape))
        if len(a.shape) == 2:  # forward(double[][]) (BasicTransform.java:336-342)
            return self._forward2d(arr, _get_exponent(a.shape[0]), _get_exponent(a.shape[1]))
        if level is None:
            n = a.shape[0]
            if not _is_binary(n):
                raise JWaveFailure(
                    "WaveletTransform#forward - given array length is not 2^p | p E N ... = 1, 2, "
                    "4, 8, 16, 32, .. please use the Ancient Egyptian Decomposition for any other "
                    "array length!")
            level = self.calcExponent(n)
        return self._run1d(a, level, batch=False, reverse=False)

    def reverse(self, arr, level=None, lvlN=None, lvlR=None):
        if lvlR is not None:
            return self._reverse3d(arr, level, lvlN, lvlR)
        if lvlN is not None:
            return self._reverse2d(arr, level, lvlN)
        a = as_input(arr)
        if len(a.shape) == 3:  # reverse(double[][][]) (BasicTransform.java:579-585)
            return self._reverse3d(arr, *(_get_exponent(d) for d in a.shape))
        if len(a.shape) == 2:
            return self._reverse2d(arr, _get_exponent(a.shape[0]), _get_exponent(a.shape[1]))
        if level is None:
            n = a.shape[0]
            if not _is_binary(n):
                raise JWaveFailure(
                    "WaveletTransform#reverse - given array length is not 2^p | p E N ... = 1, 2, "
                    "4, 8, 16, 32, .. please use the Ancient Egyptian Decomposition for any other "
                    "array length!")
            level = self.calcExponent(n)
        return self._run1d(a, level, batch=False, reverse=True)

    def forwardBatch(self, signals, level):
        """Batched extension: every row of ``signals`` (B x n) with ``level``."""
        return self._run1d(as_input(signals), level, batch=True, reverse=False)

    def reverseBatch(self, coeffs, level):
        return self._run1d(as_input(coeffs), level, batch=True, reverse=True)

    def _run1d(self, a, level, batch, reverse):
        L = _native.lib()
        n = a.shape[-1]
        B = a.shape[0] if batch else 1
        out = a.empty(a.shape)
        fn = L.jw_fwt_reverse if reverse else L.jw_fwt_forward
        _native.check(fn(self._plan, a.ptr, out.ptr, n, int(level), B, a.where, a.stream))
        return out.result()

    # ---- 2-D (BasicTransform.forward/reverse(double[][], lvlM, lvlN) :361-474) ----
    def _forward2d(self, mat, lvlM, lvlN, batch=False):
        a = as_input(mat)
        L = _native.lib()
        rows, cols = a.shape[-2], a.shape[-1]
        B = a.shape[0] if batch else 1
        out = a.empty(a.shape)
        _native.check(L.jw_fwt2d_forward(self._plan, a.ptr, out.ptr, rows, cols, int(lvlM),
                                         int(lvlN), B, a.where, a.stream))
        return out.result()

    def _reverse2d(self, mat, lvlM, lvlN, batch=False):
        a = as_input(mat)
        L = _native.lib()
        rows, cols = a.shape[-2], a.shape[-1]
        B = a.shape[0] if batch else 1
        out = a.empty(a.shape)
        _native.check(L.jw_fwt2d_reverse(self._plan, a.ptr, out.ptr, rows, cols, int(lvlM),
                                         int(lvlN), B, a.where, a.stream))
        return out.result()

    def forward2DBatch(self, images, lvlM, lvlN):
        return self._forward2d(images, lvlM, lvlN, batch=True)

    def reverse2DBatch(self, images, lvlM, lvlN):
        return self._reverse2d(images, lvlM, lvlN, batch=True)

    # ---- 3-D (BasicTransform.forward/reverse(double[][][], lvlP, lvlQ, lvlR) :509-659) ----
    # Java applies lvlP to dimension 2, lvlQ to dimension 3 (the slab's 2-D transform) and
    # lvlR to dimension 1; the no-level overloads pass the exponents of dimensions 1, 2, 3.
    def _run3d(self, spc, lvlP, lvlQ, lvlR, batch, reverse):
        a = as_input(spc)
        L = _native.lib()
        d1, d2, d3 = a.shape[-3], a.shape[-2], a.shape[-1]
        B = a.shape[0] if batch else 1
        out = a.empty(a.shape)
        fn = L.jw_fwt3d_reverse if reverse else L.jw_fwt3d_forward
        _native.check(fn(self._plan, a.ptr, out.ptr, d1, d2, d3, int(lvlP), int(lvlQ), int(lvlR),
                         B, a.where, a.stream))
        return out.result()

    def _forward3d(self, spc, lvlP, lvlQ, lvlR, batch=False):
        return self._run3d(spc, lvlP, lvlQ, lvlR, batch, False)

    def _reverse3d(self, spc, lvlP, lvlQ, lvlR, batch=False):
        return self._run3d(spc, lvlP, lvlQ, lvlR, batch, True)

    def forward3DBatch(self, spaces, lvlP, lvlQ, lvlR):
        """Batched extension: every space of ``spaces`` (B x d1 x d2 x d3)."""
        return self._forward3d(spaces, lvlP, lvlQ, lvlR, batch=True)

    def reverse3DBatch(self, spaces, lvlP, lvlQ, lvlR):
        return self._reverse3d(spaces, lvlP, lvlQ, lvlR, batch=True)

    # ---- decompose / recompose (WaveletTransform.java:136-182) ----
    def decompose(self, arrTime):
        a = np.asarray(arrTime, dtype=np.float64)
        levels = self.calcExponent(a.shape[0])
        return np.stack([np.asarray(self.forward(a, p)) for p in range(levels + 1)])

    def recompose(self, matDeComp, level=None):
        if level is None:
            level = 0
        if level < 0 or level >= len(matDeComp):
            raise JWaveFailure("WaveletTransform#recompose - given level is out of range")
        return self.reverse(np.asarray(matDeComp[level], dtype=np.float64), level)


class WaveletPacketTransform(FastWaveletTransform):
    """jwave.transforms.WaveletPacketTransform (WaveletPacketTransform.java:60-191): every level
    transforms all packets.  1-D through jw_wpt_forward / jw_wpt_reverse; the 2-D methods
    (BasicTransform.java:361-474) run the 1-D packet transform over rows, then columns."""

    def __init__(self, wavelet, arith="strict"):
        super().__init__(wavelet, arith)
        self._name = "Wavelet Packet Transform"

    def _run1d(self, a, level, batch, reverse):
        L = _native.lib()
        n = a.shape[-1]
        B = a.shape[0] if batch else 1
        out = a.empty(a.shape)
        fn = L.jw_wpt_reverse if reverse else L.jw_wpt_forward
        _native.check(fn(self._plan, a.ptr, out.ptr, n, int(level), B, a.where, a.stream))
        return out.result()

    def _rows(self, m, level, reverse):
        return self._run1d(as_input(m), level, batch=True, reverse=reverse)

    @staticmethod
    def _t(m):
        return m.t().contiguous() if hasattr(m, "is_cuda") else np.ascontiguousarray(m.T)

    def _forward2d(self, mat, lvlM, lvlN, batch=False):
        if batch:
            return [self._forward2d(m, lvlM, lvlN) for m in mat]
        y = self._rows(mat, lvlN, False)
        return self._t(self._rows(self._t(y), lvlM, False))

    def _reverse2d(self, mat, lvlM, lvlN, batch=False):
        if batch:
            return [self._reverse2d(m, lvlM, lvlN) for m in mat]
        x = self._t(self._rows(self._t(mat), lvlM, True))
        return self._rows(x, lvlN, True)

    # 3-D (BasicTransform.java:509-659) over the packet transform: the 2-D packet transform of
    # every slab, then the 1-D packet transform along dimension 1.
    @staticmethod
    def _stack(ms):
        return __import__("torch").stack(ms) if hasattr(ms[0], "is_cuda") else np.stack(ms)

    def _forward3d(self, spc, lvlP, lvlQ, lvlR, batch=False):
        if batch:
            return self._stack([self._forward3d(m, lvlP, lvlQ, lvlR) for m in spc])
        y = self._stack([self._forward2d(m, lvlP, lvlQ) for m in spc])
        d1 = y.shape[0]
        lines = self._rows(self._t(y.reshape(d1, -1)), lvlR, False)
        return self._t(lines).reshape(y.shape)

    def _reverse3d(self, spc, lvlP, lvlQ, lvlR, batch=False):
        if batch:
            return self._stack([self._reverse3d(m, lvlP, lvlQ, lvlR) for m in spc])
        x = self._stack([self._reverse2d(m, lvlP, lvlQ) for m in spc])
        d1 = x.shape[0]
        lines = self._rows(self._t(x.reshape(d1, -1)), lvlR, True)
        return self._t(lines).reshape(x.shape)
