#!/usr/bin/env python3
"""Time one MODWT configuration (forward + inverse, inputs in HBM) -- a microbenchmark for the
non-headline paths (AUTO / FFT, either arithmetic), also run under rocprofv3 for kernel stats.
Prints one JSON line per configuration."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd")]

import torch  # noqa: E402

from jwave import MODWTTransform, _native  # noqa: E402
from jwave.transforms import wavelets as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--wavelet", default="Daubechies4")
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--levels", type=int, default=8)
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--method", choices=["auto", "direct", "fft"], default="auto")
ap.add_argument("--arith", choices=["strict", "fma"], default="strict")
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _native.lib()
n, J, B = a.n, a.levels, a.batch
x = torch.empty((B, n), dtype=torch.float64, device=dev)
c = torch.empty((B, J + 1, n), dtype=torch.float64, device=dev)
xr = torch.empty_like(x)
s = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)
_native.check(lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 42, sp))
xform = MODWTTransform(W.by_name(a.wavelet), arith=a.arith)  # owns the plan: keep it alive
plan = xform.initializeFilterCache()
method = {"auto": _native.JW_CONV_AUTO, "direct": _native.JW_CONV_DIRECT, "fft": _native.JW_CONV_FFT}[a.method]
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731


def step():
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(s)
    _native.check(lib.jw_modwt_forward(plan, P(x), P(c), n, J, B, method, _native.JW_DEVICE, sp))
    ev[1].record(s)
    _native.check(lib.jw_modwt_inverse(plan, P(c), P(xr), n, J, B, method, _native.JW_DEVICE, sp))
    ev[2].record(s)
    return ev


step()
torch.cuda.synchronize()
evs = [step() for _ in range(a.reps)]
torch.cuda.synchronize()
f = sum(e[0].elapsed_time(e[1]) for e in evs) / a.reps
i = sum(e[1].elapsed_time(e[2]) for e in evs) / a.reps
print(json.dumps({"wavelet": a.wavelet, "n": n, "J": J, "batch": B, "method": a.method,
                  "arith": a.arith, "fwd_ms": round(f, 3), "inv_ms": round(i, 3),
                  "msamples_s": round(B * n / ((f + i) * 1e-3) / 1e6, 1),
                  "recon_max_abs": (xr - x).abs().max().item()}), flush=True)
