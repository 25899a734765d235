"""jwave -- MI355X-native engine for JWave-Pro's hot path, behind the reference's own API.

Module layout mirrors the reference's Java packages (jwave.transforms.MODWTTransform,
jwave.transforms.FastWaveletTransform, jwave.transforms.wavelets.*, jwave.exceptions).
All compute goes through libjwave_hip.so (include/jwave_hip.h); there is no CPU path.
"""
from . import exceptions, transforms
from .Transform import Transform
from .transforms import (ContinuousWaveletTransform, FastFourierTransform, FastWaveletTransform,
                         MODWTTransform, WaveletPacketTransform)
from .transforms import wavelets

__version__ = "0.1.0"
__all__ = ["Transform", "FastWaveletTransform", "MODWTTransform", "ContinuousWaveletTransform",
           "WaveletPacketTransform", "FastFourierTransform",
           "wavelets", "exceptions", "transforms"]
