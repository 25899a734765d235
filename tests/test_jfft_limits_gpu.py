"""JWave's own FFT (JW_ARITH_STRICT) at the reference's longest lengths: powers of two to 2^30
and Bluestein to 2^29 (m = 2^30) -- FastFourierTransform.java:112-324 has no other limit than
its int arithmetic (jw_internal.hpp kStrictFft*).

The oracle needs minutes per transform here, so the powers of two are checked through the
last-stage identity pinned on the oracle in tests/test_fft_split_identity.py: the engine's
n-point transform must equal, bit for bit, Java's last butterfly stage (twiddles from the
oracle's recurrence) applied to the engine's own n/2-point transforms of the even and odd
samples.  2^27 is bit-exact against the oracle itself (test_modwt_strict_gpu.py), so the chain
2^27 -> 2^28 -> 2^29 -> 2^30 carries bit-exactness to every three-pass geometry (pass 3 of
2^10, 2^11, 2^12 points).  The arithmetic below runs as separate torch ops on the device: each
op is rounded on its own, as in Java.  Bluestein past 2^27 and MODWT at 2^29 are checked
against exact-twiddle references within a norm-wise 1e-6 (the reference's recurrence
drift there is ~1e-8; an indexing fault is O(1)) -- torch.fft and the DIRECT kernels; a one-off bit-exact oracle run is in
profiles/r06/fft_limits/.
"""
import ctypes

import numpy as np
import pytest

import oracle as orc
from jwave import _native

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def fft(t, n, batch, inverse, arith=_native.JW_ARITH_STRICT):
    import torch
    out = torch.empty_like(t)
    fn = _native.lib().jw_fft_reverse_ex if inverse else _native.lib().jw_fft_forward_ex
    stream = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
    _native.check(fn(_p(t), _p(out), n, batch, arith, _native.JW_DEVICE, stream))
    torch.cuda.synchronize()
    return out


def bits(t):
    import torch
    return t.contiguous().view(torch.int64)


@pytest.mark.parametrize("lg,inverse", [(28, False), (29, False), (29, True), (30, False)])
def test_long_pow2_bit_exact_by_last_stage(lg, inverse, device):
    import torch
    n, h = 1 << lg, 1 << (lg - 1)
    gen = torch.Generator(device=device).manual_seed(lg)
    z = torch.rand((n, 2), dtype=torch.float64, device=device, generator=gen) * 2 - 1
    X = fft(z, n, 1, inverse)
    halves = torch.stack([z[0::2], z[1::2]])  # (2, n/2, 2): even, odd samples
    del z
    EO = fft(halves, h, 2, inverse)
    del halves
    if inverse:  # the halves' 1 / (n/2) undone, exactly (a power of two)
        EO.mul_(float(h))
    E, O = EO[0], EO[1]
    w = torch.from_numpy(orc.fft_stage_twiddles(n, inverse).view(np.float64).reshape(h, 2)).to(device)
    tr = w[:, 0] * O[:, 0] - w[:, 1] * O[:, 1]  # t = wn.mul(x[k + half]) (Complex.mul :286-288)
    ti = w[:, 0] * O[:, 1] + w[:, 1] * O[:, 0]
    del w
    for part, sign in ((X[:h], 1.0), (X[h:], -1.0)):
        ref = torch.stack([E[:, 0] + tr, E[:, 1] + ti], 1) if sign > 0 else \
            torch.stack([E[:, 0] - tr, E[:, 1] - ti], 1)
        if inverse:
            ref.mul_(1.0 / n)  # x[i].mul(1.0 / n) (:207-211): exact
        assert torch.equal(bits(part), bits(ref)), f"2^{lg} {'reverse' if inverse else 'forward'}"
        del ref


@pytest.mark.timeout(300)  # host chirp tables of up to 4e8 correctly rounded sin/cos per direction
@pytest.mark.parametrize("n", [3 << 25, 3 << 26, 3 << 27])
def test_long_bluestein_near_exact(n, device):
    # m = 2^28, 2^29, 2^30: the three-pass m-point convolution (jw_jfft_bs.hip bs_conv3; 2^28
    # puts its last pass on 1024-point columns), up to its longest,
    # against torch.fft (exact-twiddle mixed radix on these 3 x 2^k lengths)
    import torch
    gen = torch.Generator(device=device).manual_seed(n)
    z = torch.rand((n, 2), dtype=torch.float64, device=device, generator=gen) * 2 - 1
    X = fft(z, n, 1, False)
    R = torch.view_as_real(torch.fft.fft(torch.view_as_complex(z)))
    err = (torch.linalg.vector_norm(X - R) / torch.linalg.vector_norm(R)).item()
    assert err < 1e-6, err
    if n < (3 << 27):  # reverse(forward(z)) = z to the same tolerance (the longest: forward only)
        Xr = fft(X, n, 1, True)
        assert (torch.linalg.vector_norm(Xr - z) / torch.linalg.vector_norm(z)).item() < 1e-6


def test_modwt_fft_method_at_2_29(device):
    # ConvolutionMethod.FFT under STRICT at a length past the old 2^28 range: one level of
    # circularConvolveFFT (MODWTTransform.java:752-786) on 2^29-point transforms, against the
    # DIRECT kernels (the same convolution, exact up to the FFT's rounding)
    import torch
    from jwave import MODWTTransform
    from jwave.transforms import wavelets as W
    n, J = 1 << 29, 1
    x = torch.empty(n, dtype=torch.float64, device=device)
    _native.check(_native.lib().jw_synth_uniform(_p(x), n, 1, 7, None))
    c = torch.empty((J + 1, n), dtype=torch.float64, device=device)
    d = torch.empty_like(c)
    m = MODWTTransform(W.Daubechies4())  # owns the plan: kept alive for the calls below
    plan = m.initializeFilterCache()
    for out, method in ((c, _native.JW_CONV_FFT), (d, _native.JW_CONV_DIRECT)):
        _native.check(_native.lib().jw_modwt_forward(plan, _p(x), _p(out), n, J, 1, method,
                                                     _native.JW_DEVICE, None))
    torch.cuda.synchronize()
    err = (torch.linalg.vector_norm(c - d) / torch.linalg.vector_norm(d)).item()
    assert err < 1e-6, err


def test_host_allocation_failure_is_a_status(knobs, device):
    # a C++ exception inside the engine (here std::bad_alloc from a twiddle-table build, injected
    # by JW_TEST_THROW_BADALLOC) comes back as JW_ERR_NO_MEMORY with a message -- never an unwind
    # into the caller -- and the table is not kept: the same call succeeds afterwards, bit-exact
    import torch
    n = 3 << 11  # not a power of two: Bluestein over m = 8192 (a table no other test builds first)
    z = torch.rand((n, 2), dtype=torch.float64, device=device)
    out = torch.empty_like(z)
    knobs.setenv("JW_TEST_THROW_BADALLOC", "1")
    st = _native.lib().jw_fft_forward_ex(_p(z), _p(out), n, 1, _native.JW_ARITH_STRICT,
                                         _native.JW_DEVICE, None)
    assert st == _native.JW_ERR_NO_MEMORY and "bad_alloc" in _native.last_error()
    knobs.delenv("JW_TEST_THROW_BADALLOC")
    X = fft(z, n, 1, False)
    ref = orc.fft(torch.view_as_complex(z).cpu().numpy())
    assert torch.equal(bits(X.cpu()), bits(torch.view_as_real(torch.from_numpy(ref))))
