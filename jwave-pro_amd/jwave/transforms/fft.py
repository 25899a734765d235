"""FastFourierTransform host mirror (src/main/java/jwave/transforms/FastFourierTransform.java).

Same names and semantics as the reference, computed by the HIP engine (jw_fft_forward_ex /
jw_fft_reverse_ex).  The default arithmetic is "strict": power-of-two lengths run the
reference's own radix-2 algorithm with its recurrence twiddles (:172-212), bit for bit;
"fma" selects the correctly rounded twiddle tables:
* ``forward(double[])``: real input -> interleaved (re, im) spectrum of length 2n (:48-75);
* ``reverse(double[])``: interleaved spectrum -> real part of the inverse (:83-103);
* ``forward(Complex[])`` / ``reverse(Complex[])`` on complex arrays (:112-164), the reverse
  scaled by 1/n (:207-211); length 0 gives an empty result, length 1 a copy, powers of two
  the four-step engine and other lengths a chirp-z (Bluestein, :259-324) transform.
Extensions beyond the Java API: a batch (B x n) of lines, and HIP-device torch tensors
(complex128, or float64 with a trailing (re, im) axis) computed in place on HBM.
"""
import ctypes

import numpy as np

from .. import _native
from .._arrays import _is_torch


def _run(fn, z, arith):
    """z: complex ndarray / tensor of shape (n,) or (B, n) -> same type and shape."""
    if _is_torch(z) and z.device.type == "cuda":
        import torch
        t = z if z.dtype == torch.complex128 else z.to(torch.complex128)
        t = t.contiguous()
        out = torch.empty_like(t)
        n = t.shape[-1]
        batch = 1 if t.dim() == 1 else int(np.prod(t.shape[:-1]))
        stream = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
        _native.check(fn(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), n, batch,
                         arith, _native.JW_DEVICE, stream))
        return out
    a = np.ascontiguousarray(np.asarray(z, dtype=np.complex128))
    out = np.empty_like(a)
    n = a.shape[-1] if a.ndim else 0
    if a.size == 0:
        return out
    batch = 1 if a.ndim == 1 else int(np.prod(a.shape[:-1]))
    _native.check(fn(ctypes.c_void_p(a.ctypes.data), ctypes.c_void_p(out.ctypes.data), n, batch,
                     arith, _native.JW_HOST, None))
    return out


class FastFourierTransform:
    """jwave.transforms.FastFourierTransform"""

    def __init__(self, arith="strict"):
        self._name = "Fast Fourier Transform"
        self._arith = _native.JW_ARITH_FMA if arith == "fma" else _native.JW_ARITH_STRICT

    def getName(self):
        return self._name

    # ---- Complex[] API (:112-164) ----
    def forwardComplex(self, x):
        return _run(_native.lib().jw_fft_forward_ex, x, self._arith)

    def reverseComplex(self, x):
        return _run(_native.lib().jw_fft_reverse_ex, x, self._arith)

    # ---- double[] API (:48-103) ----
    def forward(self, arr):
        """Real samples -> interleaved spectrum; complex input -> complex spectrum."""
        a = np.asarray(arr) if not _is_torch(arr) else arr
        if np.iscomplexobj(a) if not _is_torch(a) else a.is_complex():
            return self.forwardComplex(a)
        z = self.forwardComplex(np.asarray(a, dtype=np.float64).astype(np.complex128))
        out = np.empty(2 * z.shape[-1])
        out[0::2], out[1::2] = z.real, z.imag
        return out

    def reverse(self, arr):
        """Interleaved spectrum -> real part of the inverse; complex input -> complex result."""
        a = np.asarray(arr) if not _is_torch(arr) else arr
        if np.iscomplexobj(a) if not _is_torch(a) else a.is_complex():
            return self.reverseComplex(a)
        a = np.asarray(a, dtype=np.float64)
        n = a.shape[0] // 2
        z = a[0:2 * n:2] + 1j * a[1:2 * n:2]
        return np.ascontiguousarray(self.reverseComplex(z).real)
