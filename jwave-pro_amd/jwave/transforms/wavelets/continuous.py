"""Continuous wavelets of the CWT hot path (jwave.transforms.wavelets.continuous).

MorletWavelet (src/main/java/jwave/transforms/wavelets/continuous/MorletWavelet.java:56-124),
MexicanHatWavelet (MexicanHatWavelet.java:56-119), PaulWavelet (PaulWavelet.java:67-290),
DOGWavelet (DOGWavelet.java:40-405) and MeyerWavelet (MeyerWavelet.java:56-335) with the
reference's constructors, validation messages and closed forms.  The GPU engine evaluates
fourierTransform per frequency bin itself (jw_cwt_fft); the host methods here are the
reference's public API for callers.
"""
import enum
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
            return np.asarray(self._ft(omega)).astype(np.complex128)
        if scale <= 0:
            raise IllegalArgumentException("Scale must be positive")
        ft = np.asarray(self._ft(scale * omega)).astype(np.complex128) * math.sqrt(scale)
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

    def getBandwidthParameter(self):
        return self._fb

    def getCenterFrequencyParameter(self):
        return self._fc

    def getAdmissibilityConstant(self):  # MorletWavelet.java getAdmissibilityConstant
        return 2.0 * math.pi * 1.1 if self._fc < 0.8 else 2.0 * math.pi

    def getEffectiveSupport(self):
        r = 4.0 * math.sqrt(self._fb)
        return [-r, r]

    def getBandwidth(self):
        hw = 2.0 / math.sqrt(2.0 * math.pi * self._fb)
        return [self._fc - hw, self._fc + hw]

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

    def getSigma(self):
        return self._sigma

    def getAdmissibilityConstant(self):
        return math.pi

    def getEffectiveSupport(self):
        return [-5.0 * self._sigma, 5.0 * self._sigma]

    def getBandwidth(self):
        return [0.0, 3.0 / (2.0 * math.pi * self._sigma)]

    def params(self):
        return (self._sigma, 0.0)

    def _psi(self, t):  # MexicanHatWavelet.java:85-95
        tn2 = (t / self._sigma) ** 2
        return (self._normConstant * (1.0 - tn2) * np.exp(-0.5 * tn2)).astype(np.complex128)

    def _ft(self, omega):  # MexicanHatWavelet.java:107-119
        ft_norm = self._normConstant * self._sigma * math.sqrt(2.0 * math.pi)
        om2 = omega * omega
        return ft_norm * om2 * np.exp(-0.5 * self._sigma * self._sigma * om2)


def _factorial(n):
    r = 1.0
    for i in range(2, n + 1):
        r *= i
    return r


class PaulWavelet(ContinuousWavelet):
    """PaulWavelet(m): psi(t) = norm i^m (1 - it)^-(m+1), analytic (PaulWavelet.java:76-164)."""

    _kind = _native.JW_CWT_PAUL

    def __init__(self, m=4):
        super().__init__()
        if m < 1:
            raise IllegalArgumentException("Order parameter m must be a positive integer")
        if m > 20:
            raise IllegalArgumentException("Order parameter m > 20 may cause numerical issues")
        self._name = "Paul"
        self._m = int(m)
        self._normConstant = math.pow(2, m) * _factorial(m) / math.sqrt(
            math.pi * _factorial(2 * m))
        self._iPowerM = (1, 1j, -1, -1j)[m % 4]
        self._centerFrequency = (m + 0.5) / (2.0 * math.pi)

    def getOrder(self):
        return self._m

    def getAdmissibilityConstant(self):
        return 2.0 * math.pi / (2 * self._m + 1)

    def getEffectiveSupport(self):
        return [-1.0, 2.0 * (self._m + 1)]

    def getBandwidth(self):
        return [0.0, (2 * self._m + 2) / (2.0 * math.pi)]

    @staticmethod
    def fromResolutionBalance(frequencyResolution):  # PaulWavelet.java:278-290
        if frequencyResolution < 1 or frequencyResolution > 10:
            raise IllegalArgumentException("Resolution balance must be between 1 and 10")
        # Math.round: floor(x + 0.5)
        return PaulWavelet(int(math.floor(2 + (frequencyResolution - 1) * 2 + 0.5)))

    def params(self):
        return (float(self._m), 0.0)

    def _psi(self, t):  # (1 - it)^-(m+1) by magnitude and argument (complexPower :262-271)
        p = -(self._m + 1)
        mag = np.hypot(1.0, t)
        arg = np.arctan2(-t, 1.0)
        pw = np.power(mag, p) * np.cos(p * arg) + 1j * (np.power(mag, p) * np.sin(p * arg))
        return self._iPowerM * self._normConstant * pw

    def _ft(self, omega):  # :128-140
        omega = np.asarray(omega, dtype=np.float64)
        pos = omega > 0
        w = np.where(pos, omega, 0.0)
        return np.where(pos, math.sqrt(2.0 * math.pi) * np.power(w, self._m) * np.exp(-w), 0.0)

    def fourierTransform(self, omega, scale=None, translation=0.0):
        """The (omega, scale, b) override :152-164: sqrt(a) sqrt(2 pi) (a w)^m e^{-a w} for
        w > 0, no scale check and no translation phase."""
        if scale is None:
            return super().fourierTransform(omega)
        omega = np.asarray(omega, dtype=np.float64)
        pos = omega > 0
        so = scale * np.where(pos, omega, 0.0)
        v = math.sqrt(scale) * math.sqrt(2.0 * math.pi) * np.power(so, self._m) * np.exp(-so)
        return np.where(pos, v, 0.0).astype(np.complex128)


class DOGWavelet(ContinuousWavelet):
    """DOGWavelet(n, sigma): n-th derivative of a Gaussian (DOGWavelet.java:40-405)."""

    _kind = _native.JW_CWT_DOG

    class WaveletType(enum.Enum):  # DOGWavelet.WaveletType :46-80
        EDGE = (1, "Edge detection")
        MEXICAN_HAT = (2, "Mexican Hat / Ricker wavelet")
        RICKER = (2, "Ricker wavelet (alias for Mexican Hat)")
        ZERO_CROSSING = (3, "Zero-crossing detection")
        RIDGE = (4, "Ridge detection")

        def getOrder(self):
            return self.value[0]

        def getDescription(self):
            return self.value[1]

    def __init__(self, n=2, sigma=1.0):
        super().__init__()
        if n < 1:
            raise IllegalArgumentException("Derivative order n must be a positive integer")
        if n > 10:
            raise IllegalArgumentException("Derivative order n > 10 may cause numerical issues")
        if sigma <= 0:
            raise IllegalArgumentException("Width parameter sigma must be positive")
        self._name = "DOG (n=%d)" % n
        self._n = int(n)
        self._sigma = float(sigma)
        self._hermiteCoeffs = self._hermite(self._n)
        df = 1.0
        for i in range(2 * n - 1, 0, -2):  # doubleFactorial :376-382
            df *= i
        self._normConstant = math.sqrt(df / (math.pow(2, n) * math.sqrt(math.pi) *
                                             math.pow(sigma, 2 * n + 1)))
        self._centerFrequency = math.sqrt(n) / (2.0 * math.pi * sigma)

    @staticmethod
    def _hermite(n):  # computeHermiteCoefficients :289-335, sign (-1)^(n+1)
        c = [[1.0], [0.0, 2.0]]
        for k in range(2, n + 1):
            h = [0.0] * (k + 1)
            for i in range(1, k + 1):
                if i - 1 < len(c[k - 1]):
                    h[i] += 2.0 * c[k - 1][i - 1]
            for i in range(k - 1):
                h[i] -= 2.0 * (k - 1) * c[k - 2][i]
            c.append(h)
        sign = 1.0 if (n + 1) % 2 == 0 else -1.0
        return [sign * v for v in c[n]]

    def getDerivativeOrder(self):
        return self._n

    def getSigma(self):
        return self._sigma

    def isMexicanHat(self):
        return self._n == 2

    @staticmethod
    def createStandard(type_, sigma=1.0):
        if type_ is None:
            raise IllegalArgumentException("DOG wavelet type cannot be null")
        return DOGWavelet(type_.getOrder(), sigma)

    def getAdmissibilityConstant(self):
        return 2.0 * math.pi

    def getEffectiveSupport(self):
        r = (3.0 + self._n / 2.0) * self._sigma
        return [-r, r]

    def getBandwidth(self):
        return [0.0, (1.0 + self._n / 2.0) / (2.0 * math.pi * self._sigma)]

    def params(self):
        return (float(self._n), self._sigma)

    def _psi(self, t):  # :166-180, Horner over the Hermite coefficients
        x = t / self._sigma
        h = np.zeros_like(x)
        for c in reversed(self._hermiteCoeffs):
            h = h * x + c
        return (self._normConstant * h * np.exp(-0.5 * x * x)).astype(np.complex128)

    def _ft(self, omega):  # :187-220, phase i^n
        mag = (math.sqrt(2.0 * math.pi) * math.pow(self._sigma, self._n + 1) *
               np.power(np.abs(omega), self._n) *
               np.exp(-0.5 * self._sigma * self._sigma * omega * omega)) * self._normConstant
        r = self._n % 4
        if r == 0:
            return mag + 0j
        if r == 1:
            return 1j * (mag * np.sign(omega))
        if r == 2:
            return -mag + 0j
        return 1j * (-mag * np.sign(omega))


class MeyerWavelet(ContinuousWavelet):
    """MeyerWavelet(): compact frequency support [2 pi/3, 8 pi/3] (MeyerWavelet.java:56-335)."""

    _kind = _native.JW_CWT_MEYER
    _LO, _MID, _HI = 2.0 * math.pi / 3.0, 4.0 * math.pi / 3.0, 8.0 * math.pi / 3.0

    def __init__(self):
        super().__init__()
        self._name = "Meyer"
        self._centerFrequency = 0.7 / (2.0 * math.pi)

    def getAdmissibilityConstant(self):
        return 2.0 * math.pi

    def getEffectiveSupport(self):
        return [-15.0, 15.0]

    def getBandwidth(self):
        return [2.0 / 3.0 / (2.0 * math.pi), 8.0 / 3.0 / (2.0 * math.pi)]

    def params(self):
        return (0.0, 0.0)

    @staticmethod
    def _nu(x):  # transitionFunction :279-295
        x = np.asarray(x, dtype=np.float64)
        x2 = x * x
        x3 = x2 * x
        x4 = x3 * x
        p = x4 * (35.0 + -84.0 * x + 70.0 * x2 + -20.0 * x3)
        return np.where(x <= 0, 0.0, np.where(x >= 1, 1.0, p))

    @staticmethod
    def _sinc(x):  # :262-270
        x = np.asarray(x, dtype=np.float64)
        x2 = x * x
        with np.errstate(invalid="ignore", divide="ignore"):
            s = np.sin(x) / x
        return np.where(np.abs(x) < 1e-10, 1.0 - x2 / 6.0 + x2 * x2 / 120.0, s)

    def _psi(self, t):  # :180-214, modulated-sinc approximation
        t = np.asarray(t, dtype=np.float64)
        env = np.exp(-0.5 * t * t / 25.0)
        w0 = 0.7
        v = w0 * self._sinc(w0 * t) * env
        w1 = 1.4 * w0
        v = v + 0.2 * w1 * self._sinc(w1 * t) * env
        w2 = 0.5 * w0
        v = v + -0.1 * w2 * self._sinc(w2 * t) * env
        v = v * math.sqrt(2.0 / math.pi)
        return np.where(np.abs(t) > 15.0, 0.0, v).astype(np.complex128)

    def _ft(self, omega):  # :223-253
        omega = np.asarray(omega, dtype=np.float64)
        a = np.abs(omega)
        lo = np.sin(math.pi / 2.0 * self._nu(3.0 * a / (2.0 * math.pi) - 1.0))
        hi = np.cos(math.pi / 2.0 * self._nu(3.0 * a / (4.0 * math.pi) - 1.0))
        v = np.where(a <= self._MID, lo, hi) * math.sqrt(2.0 * math.pi)
        v = np.where((a < self._LO) | (a > self._HI), 0.0, v)
        return v * np.cos(omega / 2.0) + 1j * (v * np.sin(omega / 2.0))
