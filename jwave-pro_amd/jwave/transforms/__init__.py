"""jwave.transforms -- host mirror of the reference's transform classes (hot path only)."""
from .fwt import BasicTransform, FastWaveletTransform, WaveletTransform
from .modwt import ConvolutionMethod, MODWTTransform
from .cwt import CWTResult, ContinuousWaveletTransform, PaddingType

__all__ = ["BasicTransform", "WaveletTransform", "FastWaveletTransform", "MODWTTransform",
           "ConvolutionMethod", "ContinuousWaveletTransform", "CWTResult", "PaddingType"]
