"""jwave.transforms -- host mirror of the reference's transform classes (hot path only)."""
from .fwt import BasicTransform, FastWaveletTransform, WaveletPacketTransform, WaveletTransform
from .modwt import ConvolutionMethod, MODWTTransform
from .cwt import CWTResult, ContinuousWaveletTransform, PaddingType
from .fft import FastFourierTransform

__all__ = ["BasicTransform", "WaveletTransform", "FastWaveletTransform", "WaveletPacketTransform",
           "MODWTTransform",
           "ConvolutionMethod", "ContinuousWaveletTransform", "CWTResult", "PaddingType",
           "FastFourierTransform"]
