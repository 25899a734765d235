"""Discrete wavelets: the filter banks the hot path consumes.

Mirrors ``jwave.transforms.wavelets.Wavelet`` (Wavelet.java:44-303) and its orthonormal
subclasses.  The per-class scaling-decomposition taps are data generated from the
reference into ``_tables.py``; the other three filters are derived exactly as
``_buildOrthonormalSpace`` does (Wavelet.java:104-122).  The filter-bank kernels
(``forward``/``reverse``) run on the GPU through the FWT plan, never here.
"""
from ._tables import TABLES


class Wavelet:
    """jwave.transforms.wavelets.Wavelet -- filters + names (no CPU compute path)."""

    kind = 0  # JW_WAVELET_GENERIC

    def __init__(self):
        self._name = None
        self._motherWavelength = 0
        self._transformWavelength = 0
        self._scalingDeCom = None
        self._waveletDeCom = None
        self._scalingReCon = None
        self._waveletReCon = None

    def _buildOrthonormalSpace(self):  # Wavelet.java:104-122
        m = self._motherWavelength
        s = self._scalingDeCom
        self._waveletDeCom = [s[(m - 1) - i] if i % 2 == 0 else -s[(m - 1) - i] for i in range(m)]
        self._scalingReCon = list(s)
        self._waveletReCon = list(self._waveletDeCom)

    def getName(self):
        return self._name

    def __str__(self):
        return self.getName()

    def getMotherWavelength(self):
        return self._motherWavelength

    def getTransformWavelength(self):
        return self._transformWavelength

    def getScalingDeComposition(self):
        return list(self._scalingDeCom)

    def getWaveletDeComposition(self):
        return list(self._waveletDeCom)

    def getScalingReConstruction(self):
        return list(self._scalingReCon)

    def getWaveletReConstruction(self):
        return list(self._waveletReCon)


class Haar1(Wavelet):
    """haar/Haar1.java:44-70 -- orthonormal Haar, taps 1/sqrt(2)."""

    def __init__(self):
        super().__init__()
        import math
        self._name = "Haar"
        self._transformWavelength = 2
        self._motherWavelength = 2
        sqrt2 = math.sqrt(2.)
        self._scalingDeCom = [1. / sqrt2, 1. / sqrt2]
        self._waveletDeCom = [self._scalingDeCom[1], -self._scalingDeCom[0]]
        self._scalingReCon = list(self._scalingDeCom)
        self._waveletReCon = list(self._waveletDeCom)


class Haar1Orthogonal(Wavelet):
    """haar/Haar1Orthogonal.java:39-207 -- integer taps {1,1}/{1,-1}; reverse scales by .5."""

    kind = 1  # JW_WAVELET_HAAR_ORTH

    def __init__(self):
        super().__init__()
        self._name = "Haar orthogonal"
        self._transformWavelength = 2
        self._motherWavelength = 2
        self._scalingDeCom = [1., 1.]
        self._waveletDeCom = [self._scalingDeCom[1], -self._scalingDeCom[0]]
        self._scalingReCon = list(self._scalingDeCom)
        self._waveletReCon = list(self._waveletDeCom)


def _make_class(cls_name, display, tw, mw, taps, src):
    def __init__(self):
        Wavelet.__init__(self)
        self._name = display
        self._transformWavelength = tw
        self._motherWavelength = mw
        self._scalingDeCom = list(taps)
        self._buildOrthonormalSpace()

    return type(cls_name, (Wavelet,), {"__init__": __init__,
                                       "__doc__": f"{src} (taps from _tables.py)"})


for _cls, (_disp, _tw, _mw, _taps, _src) in TABLES.items():
    globals()[_cls] = _make_class(_cls, _disp, _tw, _mw, _taps, _src)

ORTHONORMAL = ["Haar1"] + list(TABLES.keys())
ALL = ["Haar1", "Haar1Orthogonal"] + list(TABLES.keys())


def by_name(cls_name):
    """Instantiate a wavelet by its Java class name (e.g. ``"Daubechies4"``)."""
    return globals()[cls_name]()


__all__ = ["Wavelet", "Haar1", "Haar1Orthogonal", "by_name", "ALL", "ORTHONORMAL"] + list(TABLES)
