"""CWT host mirror: jwave.transforms.ContinuousWaveletTransform on the MI355X.

transformFFT / transformFFTParallel (src/main/java/jwave/transforms/
ContinuousWaveletTransform.java:183-229, :511-565) run in the HIP engine (jw_cwt_fft): one
FFT per signal, one pointwise product and IFFT per scale.  Extension beyond the Java API:
``transformFFTBatch`` takes B x n signals (numpy, or HIP-device torch tensors computed in
place) and returns B x ns x n complex coefficients.
"""
import ctypes
import enum
import math

import numpy as np

from .. import _native
from .._arrays import as_input
from ..exceptions import IllegalArgumentException


class PaddingType(enum.IntEnum):  # ContinuousWaveletTransform.java:74-79
    ZERO = _native.JW_PAD_ZERO
    SYMMETRIC = _native.JW_PAD_SYMMETRIC
    PERIODIC = _native.JW_PAD_PERIODIC
    CONSTANT = _native.JW_PAD_CONSTANT


def _reim(c):
    """(Arr over the interleaved (re, im) doubles of complex coefficients, leading shape)."""
    from .._arrays import Arr, _is_torch
    if _is_torch(c):
        import torch
        if c.device.type == "cuda":
            return Arr(torch.view_as_real(c.detach().to(torch.complex128).contiguous()), True), \
                tuple(c.shape)
        c = c.detach().cpu().numpy()
    a = np.ascontiguousarray(np.asarray(c, dtype=np.complex128))
    return Arr(a.view(np.float64), False), a.shape


def magnitude(coefficients):
    """CWTResult.getMagnitude on the engine (jw_cwt_magnitude): |c| for any shape of complex
    coefficients -- a HIP-device torch tensor stays on the device (JW_DEVICE)."""
    x, shape = _reim(coefficients)
    out = x.empty(shape)
    _native.check(_native.lib().jw_cwt_magnitude(x.ptr, int(np.prod(shape)), out.ptr, x.where,
                                                 x.stream))
    return out.obj


def phase(coefficients):
    """CWTResult.getPhase on the engine (jw_cwt_phase): Complex.getPhi in radians."""
    x, shape = _reim(coefficients)
    out = x.empty(shape)
    _native.check(_native.lib().jw_cwt_phase(x.ptr, int(np.prod(shape)), out.ptr, x.where,
                                             x.stream))
    return out.obj


def scalogram(coefficients):
    """CWTResult.getScalogram on the engine (jw_cwt_scalogram): sum over the last axis of |c|^2
    (ns x n -> ns; B x ns x n -> B x ns)."""
    x, shape = _reim(coefficients)
    n = shape[-1] if shape else 1
    rows = int(np.prod(shape[:-1])) if len(shape) > 1 else 1
    out = x.empty(shape[:-1] if len(shape) > 1 else (1,))
    _native.check(_native.lib().jw_cwt_scalogram(x.ptr, rows, n, out.ptr, x.where, x.stream))
    return out.obj


class CWTResult:
    """jwave.transforms.CWTResult (CWTResult.java:33-287); coefficients as complex128.

    Coefficients held as a HIP-device torch tensor (``ContinuousWaveletTransform.resultOf``)
    keep getMagnitude / getPhase / getScalogram on the device (magnitude, phase, scalogram)."""

    def __init__(self, coefficients, scales, timeAxis, samplingRate, waveletName):
        self._c = coefficients
        self._scales = np.asarray(scales, dtype=np.float64)
        self._time = timeAxis
        self._fs = samplingRate
        self._name = waveletName

    def getCoefficients(self):
        return self._c

    def _on_device(self):
        return type(self._c).__module__.startswith("torch")

    def getMagnitude(self):  # Complex.getMag :202-204
        if self._on_device():
            return magnitude(self._c)
        return np.sqrt(self._c.real * self._c.real + self._c.imag * self._c.imag)

    def getPhase(self):  # Complex.getPhi :213-226 (degrees, quadrant rules) -> radians
        if self._on_device():
            return phase(self._c)
        r, j = self._c.real, self._c.imag
        with np.errstate(divide="ignore", invalid="ignore"):
            phi = np.degrees(np.arctan(np.abs(j / r)))
        out = np.where(r >= 0, np.where(j >= 0, phi, 360.0 - phi),
                       np.where(j >= 0, 180.0 - phi, phi + 180.0))
        out = np.where((r == 0) & (j == 0), 0.0, out)
        return out * math.pi / 180.0

    def getReal(self):
        r = self._c.real
        return r.clone() if self._on_device() else r.copy()

    def getImaginary(self):
        r = self._c.imag
        return r.clone() if self._on_device() else r.copy()

    def getScales(self):
        return self._scales

    def getTimeAxis(self):
        return self._time

    def scaleToFrequency(self, centerFreq):
        return centerFreq * self._fs / self._scales

    def getCoefficientsAtScale(self, scaleIndex):
        if scaleIndex < 0 or scaleIndex >= self._c.shape[0]:
            raise IndexError("Scale index out of bounds")
        return self._c[scaleIndex]

    def getCoefficientsAtTime(self, timeIndex):
        if timeIndex < 0 or timeIndex >= self._c.shape[1]:
            raise IndexError("Time index out of bounds")
        r = self._c[:, timeIndex]
        return r.clone() if self._on_device() else r.copy()

    def getSamplingRate(self):
        return self._fs

    def getWaveletName(self):
        return self._name

    def getNumberOfScales(self):
        return len(self._scales)

    def getNumberOfTimePoints(self):
        return len(self._time)

    def getScalogram(self):  # sum_t |c|^2 per scale (CWTResult.java:272-287)
        if self._on_device():
            return scalogram(self._c)
        m = self.getMagnitude()
        return np.array([float(np.sum(row * row)) for row in m])


class ContinuousWaveletTransform:
    """jwave.transforms.ContinuousWaveletTransform (FFT path on the GPU)."""

    PaddingType = PaddingType

    def __init__(self, wavelet, paddingType=PaddingType.SYMMETRIC):
        self._wavelet = wavelet
        self._paddingType = PaddingType(paddingType)
        self._name = "Continuous Wavelet Transform"

    def getContinuousWavelet(self):
        return self._wavelet

    def getName(self):
        return self._name

    # ---- scale generators (ContinuousWaveletTransform.java:355-405) ----
    @staticmethod
    def generateLogScales(minScale, maxScale, numScales):
        if minScale <= 0 or maxScale <= 0:
            raise IllegalArgumentException("Scales must be positive")
        if minScale >= maxScale:
            raise IllegalArgumentException("minScale must be less than maxScale")
        if numScales < 2:
            raise IllegalArgumentException("Need at least 2 scales")
        lo, hi = math.log(minScale), math.log(maxScale)
        step = (hi - lo) / (numScales - 1)
        return np.array([math.exp(lo + i * step) for i in range(numScales)])

    @staticmethod
    def generateLinearScales(minScale, maxScale, numScales):
        if minScale <= 0 or maxScale <= 0:
            raise IllegalArgumentException("Scales must be positive")
        if minScale >= maxScale:
            raise IllegalArgumentException("minScale must be less than maxScale")
        if numScales < 2:
            raise IllegalArgumentException("Need at least 2 scales")
        step = (maxScale - minScale) / (numScales - 1)
        return np.array([minScale + i * step for i in range(numScales)])

    # ---- transforms ----
    def _run(self, x, scales, samplingRate):
        sc = np.ascontiguousarray(np.asarray(scales, dtype=np.float64).ravel())
        B, n = x.shape
        ns = sc.shape[0]
        out = x.empty((B, ns, n, 2))
        params = (ctypes.c_double * 2)(*self._wavelet.params())
        _native.check(_native.lib().jw_cwt_fft(
            self._wavelet._kind, params, x.ptr, n, sc.ctypes.data_as(ctypes.c_void_p), ns,
            float(samplingRate), int(self._paddingType), out.ptr, B, x.where, x.stream))
        return out

    def transformFFT(self, signal, scales, samplingRate=1.0):
        x = as_input(np.asarray(signal, dtype=np.float64).reshape(1, -1))
        out = self._run(x, scales, samplingRate).obj
        coeffs = out[0, ..., 0] + 1j * out[0, ..., 1]
        n = coeffs.shape[1]
        dt = 1.0 / samplingRate
        time_axis = np.array([i * dt for i in range(n)])  # createTimeAxis
        return CWTResult(coeffs, scales, time_axis, samplingRate, self._wavelet.getName())

    transformFFTParallel = transformFFT  # same values (ContinuousWaveletTransform.java:511-565)

    def transformFFTScalogram(self, signals, scales, samplingRate=1.0):
        """transformFFT(x, scales, fs).getScalogram() for one signal (-> ns) or B x n signals
        (-> B x ns), numpy or HIP-device torch; the coefficients never leave the GPU
        (jw_cwt_fft_scalogram)."""
        x = as_input(signals)
        one = len(x.shape) == 1
        if one:
            x = as_input(x.obj.reshape(1, -1))
        sc = np.ascontiguousarray(np.asarray(scales, dtype=np.float64).ravel())
        B, n = x.shape
        out = x.empty((B, sc.shape[0]))
        params = (ctypes.c_double * 2)(*self._wavelet.params())
        _native.check(_native.lib().jw_cwt_fft_scalogram(
            self._wavelet._kind, params, x.ptr, n, sc.ctypes.data_as(ctypes.c_void_p), sc.shape[0],
            float(samplingRate), int(self._paddingType), out.ptr, B, x.where, x.stream))
        return out.obj[0] if one else out.obj

    def resultOf(self, coefficients, scales, samplingRate=1.0):
        """A CWTResult over ns x n coefficients as they are (e.g. one signal of a device-resident
        transformFFTBatch): its accessors then run on the engine without a host copy."""
        n = coefficients.shape[-1]
        dt = 1.0 / samplingRate
        time_axis = np.array([i * dt for i in range(n)])  # createTimeAxis
        return CWTResult(coefficients, scales, time_axis, samplingRate, self._wavelet.getName())

    # ---- direct (time-domain) path: transform :141-172, computeCoefficient :240-260 ----
    def _run_direct(self, x, scales, samplingRate, arith):
        sc = np.ascontiguousarray(np.asarray(scales, dtype=np.float64).ravel())
        B, n = x.shape
        ns = sc.shape[0]
        out = x.empty((B, ns, n, 2))
        params = (ctypes.c_double * 2)(*self._wavelet.params())
        _native.check(_native.lib().jw_cwt_direct(
            self._wavelet._kind, params, x.ptr, n, sc.ctypes.data_as(ctypes.c_void_p), ns,
            float(samplingRate), arith, out.ptr, B, x.where, x.stream))
        return out

    def transform(self, signal, scales, samplingRate=1.0, arith="strict"):
        """Direct CWT on the GPU; arith "strict" is the reference's exact sum order."""
        a = _native.JW_ARITH_FMA if arith == "fma" else _native.JW_ARITH_STRICT
        x = as_input(np.asarray(signal, dtype=np.float64).reshape(1, -1))
        out = self._run_direct(x, scales, samplingRate, a).obj
        coeffs = out[0, ..., 0] + 1j * out[0, ..., 1]
        n = coeffs.shape[1]
        dt = 1.0 / samplingRate
        time_axis = np.array([i * dt for i in range(n)])  # createTimeAxis :423-430
        return CWTResult(coeffs, scales, time_axis, samplingRate, self._wavelet.getName())

    def transformParallel(self, signal, scales, samplingRate=1.0):  # :470-500, same values
        return self.transform(signal, scales, samplingRate)

    def transformParallelCustom(self, signal, scales, samplingRate, parallelism):  # :577-680
        return self.transform(signal, scales, samplingRate)

    def transformBatch(self, signals, scales, samplingRate=1.0, arith="strict"):
        """Direct CWT of B x n signals -> B x ns x n complex (numpy or device torch)."""
        a = _native.JW_ARITH_FMA if arith == "fma" else _native.JW_ARITH_STRICT
        x = as_input(signals)
        if len(x.shape) == 1:
            x = as_input(x.obj.reshape(1, -1))
        out = self._run_direct(x, scales, samplingRate, a)
        if out.device:
            import torch
            return torch.view_as_complex(out.obj)
        o = out.obj
        return o[..., 0] + 1j * o[..., 1]

    def transformFFTBatch(self, signals, scales, samplingRate=1.0):
        """B x n signals -> B x ns x n complex coefficients (numpy or device torch)."""
        x = as_input(signals)
        if len(x.shape) == 1:
            x = as_input(x.obj.reshape(1, -1))
        out = self._run(x, scales, samplingRate)
        if out.device:
            import torch
            return torch.view_as_complex(out.obj)
        o = out.obj
        return o[..., 0] + 1j * o[..., 1]
