#!/usr/bin/env python3
"""Time JWave's own FFT (jw_fft_forward_ex, JW_ARITH_STRICT) on a batch of lines in HBM -- the
per-pass rate question behind the AUTO path's geometry (two column passes of 64-byte pieces vs
three of >= 512-byte pieces).  Run it under rocprofv3 --kernel-trace --stats for per-kernel
times, with JW_JFFT_3PASS_MIN=<n> in the environment to force the three-pass split.
Prints one JSON line: ms per transform batch and the bytes a pass moves."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd")]

import torch  # noqa: E402

from jwave import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--batch", type=int, default=128)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _native.lib()
x = torch.rand((a.batch, a.n, 2), dtype=torch.float64, device=dev)
y = torch.empty_like(x)
s = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(s.cuda_stream)


def one():
    _native.check(lib.jw_fft_forward_ex(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                        a.n, a.batch, _native.JW_ARITH_STRICT, _native.JW_DEVICE, sp))


one()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(a.reps):
    one()
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
# plain transforms: three passes from min(JW_JFFT_3PASS_MIN or 2^25, 2^23) (jw_jfft_host.hpp
# plain_three_pass_min); Bluestein lengths report their m-point convolution's two passes
pow2 = a.n & (a.n - 1) == 0
passes = 3 if pow2 and a.n >= min(int(os.environ.get("JW_JFFT_3PASS_MIN", 1 << 25)), 1 << 23) else 2
pass_bytes = 32 * a.n * a.batch  # one pass reads and writes every complex point once
print(json.dumps({"n": a.n, "batch": a.batch, "passes": passes, "ms": round(ms, 3),
                  "pass_bytes": pass_bytes,
                  "tb_s_per_pass": round(passes * pass_bytes / (ms * 1e-3) / 1e12, 3)}), flush=True)
