"""Time the MODWT FFT path (forward + inverse, db4 J=8, 32 signals) at a power-of-two length
and at nearby non-power-of-two (chirp-z) lengths, next to the DIRECT path.  Measurement only."""
import ctypes, sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jwave-pro_amd"))
import torch
from jwave import MODWTTransform, _native
from jwave.transforms import wavelets as W

dev = torch.device("cuda", 0)
lib = _native.lib()
s = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
m = MODWTTransform(W.by_name("Daubechies4"))
plan = m.initializeFilterCache()
J, B = 8, 32
LENGTHS = [int(a) for a in sys.argv[1:]] or [1 << 20, 1000000, 1048577, 1 << 22, 4000000]
for n in LENGTHS:
    x = torch.empty((B, n), dtype=torch.float64, device=dev)
    _native.check(lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 42, sp))
    c = torch.empty((B, J + 1, n), dtype=torch.float64, device=dev)
    xr = torch.empty_like(x)
    for meth, name in ((_native.JW_CONV_FFT, "fft"), (_native.JW_CONV_DIRECT, "direct")):
        def step():
            _native.check(lib.jw_modwt_forward(plan, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(c.data_ptr()), n, J, B, meth, _native.JW_DEVICE, sp))
            _native.check(lib.jw_modwt_inverse(plan, ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(xr.data_ptr()), n, J, B, meth, _native.JW_DEVICE, sp))
        step(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / 3
        err = (xr - x).abs().amax().item()
        print(f"n={n} {name}: {ms:.2f} ms/step  {B*n/ms/1e3:.0f} Msamples/s  max recon err {err:.2e}", flush=True)
    del x, c, xr
