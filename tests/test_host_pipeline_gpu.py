"""The multi-sub-batch JW_HOST pipeline (jw_capi.cpp run_items: three streams, double-buffered
HBM workspaces, loaded/done/drained events) against the JW_DEVICE path, bit for bit.

Every call here has batch x (in + out) well above the 128 MiB sub-batch, so each runs >= 3
sub-batches; four host threads run them at once on one shared plan (the
MODWTThreadSafetyTest.java:23-104 pattern), with JW_DEVICE work queued on the default stream in
between, so workspaces freed by one call are handed to another thread's H2D stream.  The
reference is the same plan through JW_DEVICE, called alone (itself bit-exact against the oracle
in test_modwt_gpu.py / test_modwt_strict_gpu.py / test_cwt_gpu.py)."""
import ctypes
import threading

import numpy as np
import pytest

import oracle as orc
from jwave import _native
from jwave.transforms import wavelets as W

pytestmark = pytest.mark.gpu

N = 1 << 20
J = 8
B = 4  # 4 x (1 + 9) x 8 MiB per call: 4 sub-batches of one signal


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def plan():
    wv = W.Daubechies4()
    sd = np.ascontiguousarray(wv.getScalingDeComposition(), dtype=np.float64)
    wd = np.ascontiguousarray(wv.getWaveletDeComposition(), dtype=np.float64)
    p = ctypes.c_void_p()
    L = _native.lib()
    _native.check(L.jw_modwt_plan_create(ctypes.byref(p), _vp(sd), _vp(wd), len(sd), 4096,
                                         _native.JW_ARITH_STRICT))
    yield p
    L.jw_modwt_plan_destroy(p)


def _device_ref(plan, xs, method):
    import torch
    L = _native.lib()
    x = torch.from_numpy(xs).cuda()
    c = torch.empty((xs.shape[0], J + 1, N), dtype=torch.float64, device="cuda")
    r = torch.empty_like(x)
    _native.check(L.jw_modwt_forward(plan, ctypes.c_void_p(x.data_ptr()),
                                     ctypes.c_void_p(c.data_ptr()), N, J, xs.shape[0], method,
                                     _native.JW_DEVICE, None))
    _native.check(L.jw_modwt_inverse(plan, ctypes.c_void_p(c.data_ptr()),
                                     ctypes.c_void_p(r.data_ptr()), N, J, xs.shape[0], method,
                                     _native.JW_DEVICE, None))
    torch.cuda.synchronize()
    return c.cpu().numpy(), r.cpu().numpy()


@pytest.mark.parametrize("method", [_native.JW_CONV_DIRECT, _native.JW_CONV_AUTO],
                         ids=["direct", "auto_strict"])
def test_modwt_host_pipeline_threads_bit_exact(plan, method):
    import torch
    L = _native.lib()
    T = 4
    inputs = [np.stack([orc.fill_uniform(N, 1000 + 10 * t + b) for b in range(B)]) for t in range(T)]
    refs = [_device_ref(plan, xs, method) for xs in inputs]
    outs = [None] * T
    errors = []
    noise = torch.empty((64, N), dtype=torch.float64, device="cuda")  # JW_DEVICE work in between

    def worker(t):
        try:
            for it in range(2):
                xs = inputs[t]
                c = np.empty((B, J + 1, N))
                xr = np.empty((B, N))
                _native.check(L.jw_modwt_forward(plan, _vp(xs), _vp(c), N, J, B, method,
                                                 _native.JW_HOST, None))
                _native.check(L.jw_modwt_inverse(plan, _vp(c), _vp(xr), N, J, B, method,
                                                 _native.JW_HOST, None))
                outs[t] = (c, xr)
                if not (np.array_equal(c.view(np.uint64), refs[t][0].view(np.uint64))
                        and np.array_equal(xr.view(np.uint64), refs[t][1].view(np.uint64))):
                    errors.append(f"thread {t} iteration {it}: JW_HOST differs from JW_DEVICE")
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {t}: {e!r}")

    def device_noise():
        try:
            coeffs = torch.empty((64, J + 1, N), dtype=torch.float64, device="cuda")
            for _ in range(3):
                _native.check(L.jw_modwt_forward(plan, ctypes.c_void_p(noise.data_ptr()),
                                                 ctypes.c_void_p(coeffs.data_ptr()), N, J, 64,
                                                 _native.JW_CONV_DIRECT, _native.JW_DEVICE, None))
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(f"device thread: {e!r}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    ths.append(threading.Thread(target=device_noise))
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "a JW_HOST thread did not finish"
    assert not errors, errors
    # the device reference itself is the oracle's (DIRECT, bit for bit)
    if method == _native.JW_CONV_DIRECT:
        wv = W.Daubechies4()
        g, h = orc.modwt_filters(wv.getScalingDeComposition(), wv.getWaveletDeComposition())
        ref0 = orc.modwt_forward(inputs[0][0], J, g, h, "direct_nz")
        assert np.array_equal(outs[0][0][0].view(np.uint64), ref0.view(np.uint64))


def test_cwt_host_pipeline_threads_bit_exact():
    import torch
    L = _native.lib()
    n, ns, Bc, T = 1 << 16, 64, 3, 3  # 3 x (1 + 128) x 0.5 MiB per call: 3 sub-batches
    scales = np.exp(np.log(2.0) + np.arange(ns) * (np.log(1024.0) - np.log(2.0)) / (ns - 1))
    params = np.array([1.0, 6.0 / (2 * np.pi)])
    inputs = [np.stack([orc.fill_uniform(n, 7 + 10 * t + b) for b in range(Bc)]) for t in range(T)]

    def call(xs, out, where, stream_ptrs):
        xp, op = stream_ptrs
        _native.check(L.jw_cwt_fft(_native.JW_CWT_MORLET, _vp(params), xp, n, _vp(scales), ns,
                                   1.0, _native.JW_PAD_SYMMETRIC, op, xs.shape[0], where, None))

    refs = []
    for xs in inputs:
        x = torch.from_numpy(xs).cuda()
        o = torch.empty((Bc, ns, n, 2), dtype=torch.float64, device="cuda")
        call(xs, o, _native.JW_DEVICE, (ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(o.data_ptr())))
        torch.cuda.synchronize()
        refs.append(o.cpu().numpy())
    errors = []

    def worker(t):
        try:
            for it in range(2):
                o = np.empty((Bc, ns, n, 2))
                call(inputs[t], o, _native.JW_HOST, (_vp(inputs[t]), _vp(o)))
                if not np.array_equal(o.view(np.uint64), refs[t].view(np.uint64)):
                    errors.append(f"thread {t} iteration {it}: JW_HOST CWT differs from JW_DEVICE")
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {t}: {e!r}")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths)
    assert not errors, errors
