"""Continuous wavelets of the CWT hot path (jwave.transforms.wavelets.continuous).

MorletWavelet (src/main/java/jwave/transforms/wavelets/continuous/MorletWavelet.java:56-124)
and MexicanHatWavelet (MexicanHatWavelet.java:56-119) with the reference's constructors,
validation messages and closed forms.  The GPU engine evaluates fourierTransform per frequency
bin itself (jw_cwt_fft); the host methods here are the reference's public API for callers.
"""
import math

import numpy as np

from ...exceptions import IllegalArgumentException
from ... import _native


class ContinuousWavelet:
    """jwave.transforms.wavelets.continuous.ContinuousWavelet"""

    _kind = None

    def __init__(self):
        self._name = None
        self._centerFrequency = 0.0

    def getName(self):
        return self._name

    def getCenterFrequency(self):
        return self._centerFrequency

    def params(self):  # the C-ABI parameter block
        raise NotImplementedError

    def wavelet(self, t, scale=None, translation=0.0):
        """psi(t), or psi_{a,b}(t) = psi((t-b)/a)/sqrt(a) (ContinuousWavelet.java:90-102)."""
        if scale is None:
            return self._psi(np.asarray(t, dtype=np.float64))
        if scale <= 0:
            raise IllegalArgumentException("Scale must be positive")
        return self._psi((np.asarray(t, dtype=np.float64) - translation) / scale) * (
            1.0 / math.sqrt(scale))

    def fourierTransform(self, omega, scale=None, translation=0.0):
        """F(omega), or sqrt(a) exp(-i omega b) F(a omega) (ContinuousWavelet.java:122-141)."""
        omega = np.asarray(omega, dtype=np.float64)
        if scale is None:
            return self._ft(omega).astype(np.complex128)
        if scale <= 0:
            raise IllegalArgumentException("Scale must be positive")
        ft = self._ft(scale * omega) * math.sqrt(scale)
        ft = ft.astype(np.complex128)
        if translation != 0:
            ft = ft * np.exp(-1j * omega * translation)
        return ft


class MorletWavelet(ContinuousWavelet):
    """MorletWavelet(fb, fc): psi(t) = exp(-t^2/(2 fb)) exp(2 pi i fc t) / sqrt(2 pi fb)."""

    _kind = _native.JW_CWT_MORLET

    def __init__(self, fb=1.0, fc=1.0):
        super().__init__()
        if fb <= 0:
            raise IllegalArgumentException("Bandwidth parameter must be positive")
        if fc <= 0:
            raise IllegalArgumentException("Center frequency must be positive")
        self._name = "Morlet"
        self._fb = float(fb)
        self._fc = float(fc)
        self._centerFrequency = float(fc)

    def getBandwidth(self):
        return self._fb

    def params(self):
        return (self._fb, self._fc)

    def _psi(self, t):  # MorletWavelet.java:85-100
        norm = 1.0 / math.sqrt(2.0 * math.pi * self._fb)
        env = np.exp(-t * t / (2.0 * self._fb))
        ph = 2.0 * math.pi * self._fc * t
        return norm * env * np.cos(ph) + 1j * (norm * env * np.sin(ph))

    def _ft(self, omega):  # MorletWavelet.java:112-124
        f = omega / (2.0 * math.pi)
        norm = math.sqrt(2.0 * math.pi * self._fb)
        return norm * np.exp(-2.0 * math.pi * math.pi * self._fb * (f - self._fc) * (f - self._fc))


class MexicanHatWavelet(ContinuousWavelet):
    """MexicanHatWavelet(sigma): the Ricker wavelet (real)."""

    _kind = _native.JW_CWT_MEXHAT

    def __init__(self, sigma=1.0):
        super().__init__()
        if sigma <= 0:
            raise IllegalArgumentException("Width parameter sigma must be positive")
        self._name = "Mexican Hat (Ricker)"
        self._sigma = float(sigma)
        self._normConstant = 2.0 / (math.sqrt(3.0 * sigma) * math.pow(math.pi, 0.25))
        self._centerFrequency = 1.0 / (2.0 * math.pi * sigma)

    def params(self):
        return (self._sigma, 0.0)

    def _psi(self, t):  # MexicanHatWavelet.java:85-95
        tn2 = (t / self._sigma) ** 2
        return (self._normConstant * (1.0 - tn2) * np.exp(-0.5 * tn2)).astype(np.complex128)

    def _ft(self, omega):  # MexicanHatWavelet.java:107-119
        ft_norm = self._normConstant * self._sigma * math.sqrt(2.0 * math.pi)
        om2 = omega * omega
        return ft_norm * om2 * np.exp(-0.5 * self._sigma * self._sigma * om2)
