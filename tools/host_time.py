#!/usr/bin/env python3
"""JW_HOST throughput: jw_modwt_forward + jw_modwt_inverse on host (numpy) arrays, PCIe staging
included (what a JNI caller passing Java arrays gets), checked bit for bit against the same
calls on HBM-resident data.  One JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from jwave import MODWTTransform, _native  # noqa: E402
from jwave.transforms import wavelets as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--levels", type=int, default=8)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
lib = _native.lib()
n, J, B = a.n, a.levels, a.batch
xf = MODWTTransform(W.Daubechies4(), arith="fma")
plan = xf.initializeFilterCache()
xd = torch.empty((B, n), dtype=torch.float64, device="cuda:0")
_native.check(lib.jw_synth_uniform(ctypes.c_void_p(xd.data_ptr()), n, B, 42, None))
xh = np.ascontiguousarray(xd.cpu().numpy())
ch = np.empty((B, J + 1, n))
xrh = np.empty((B, n))
P = lambda arr: ctypes.c_void_p(arr.ctypes.data)  # noqa: E731


def step():
    _native.check(lib.jw_modwt_forward(plan, P(xh), P(ch), n, J, B, _native.JW_CONV_DIRECT,
                                       _native.JW_HOST, None))
    _native.check(lib.jw_modwt_inverse(plan, P(ch), P(xrh), n, J, B, _native.JW_CONV_DIRECT,
                                       _native.JW_HOST, None))


step()
t0 = time.perf_counter()
for _ in range(a.reps):
    step()
th = (time.perf_counter() - t0) / a.reps
cd = torch.empty((B, J + 1, n), dtype=torch.float64, device="cuda:0")
xrd = torch.empty_like(xd)
_native.check(lib.jw_modwt_forward(plan, ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(cd.data_ptr()),
                                   n, J, B, _native.JW_CONV_DIRECT, _native.JW_DEVICE, None))
_native.check(lib.jw_modwt_inverse(plan, ctypes.c_void_p(cd.data_ptr()), ctypes.c_void_p(xrd.data_ptr()),
                                   n, J, B, _native.JW_CONV_DIRECT, _native.JW_DEVICE, None))
torch.cuda.synchronize()
same = bool(np.array_equal(cd.cpu().numpy(), ch) and np.array_equal(xrd.cpu().numpy(), xrh))
gb = (B * n * 8 * (1 + (J + 1)) * 2) / 1e9
print(json.dumps({"signals": B, "n": n, "J": J, "ms_per_fwd_inv": round(th * 1e3, 2),
                  "msamples_s": round(B * n / th / 1e6, 1), "pcie_gb_per_pair": round(gb, 3),
                  "effective_gb_s": round(gb / th, 1), "bit_identical_to_device_path": same,
                  "copy_threads": os.environ.get("JW_COPY_THREADS", "auto"),
                  "pin_mb": os.environ.get("JW_PIN_MB", "32"),
                  "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}), flush=True)
