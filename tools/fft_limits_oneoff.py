#!/usr/bin/env python3
"""One-off evidence: JWave's own FFT (jw_fft_forward_ex, JW_ARITH_STRICT) past the round-5
limits, bit-exact against the oracle itself (FastFourierTransform.java:112-324 restated in
oracle/jwave_oracle.c) -- a power of two (2^29: pass 3 of 2048 points) and a Bluestein length
(2^27 + 3: m = 2^29).  The oracle takes minutes here, too long for the GPU suite (which checks
2^28 .. 2^30 through the last-stage identity, tests/test_jfft_limits_gpu.py): the two oracle
runs go on threads of their own (ctypes drops the GIL) and the main thread prints a heartbeat.
Prints one JSON line per case."""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from jwave import _native  # noqa: E402

CASES = [int(a, 0) for a in sys.argv[1:]] or [1 << 29, (1 << 27) + 3]
dev = torch.device("cuda:0")
lib = _native.lib()
inputs, got, ref, secs = {}, {}, {}, {}


def engine(n):
    rng = np.random.default_rng(n)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    t = torch.from_numpy(z.view(np.float64)).to(dev)
    o = torch.empty_like(t)
    t0 = time.time()
    _native.check(lib.jw_fft_forward_ex(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(o.data_ptr()),
                                        n, 1, _native.JW_ARITH_STRICT, _native.JW_DEVICE, None))
    torch.cuda.synchronize()
    secs[("engine", n)] = time.time() - t0
    inputs[n], got[n] = z, o.cpu().numpy()


def oracle(n):
    t0 = time.time()
    ref[n] = orc.fft(inputs[n]).view(np.float64)
    secs[("oracle", n)] = time.time() - t0


for n in CASES:
    engine(n)
    print(f"engine n={n}: {secs[('engine', n)]:.1f} s (tables included)", flush=True)
torch.cuda.empty_cache()
threads = [threading.Thread(target=oracle, args=(n,)) for n in CASES]
for th in threads:
    th.start()
t0 = time.time()
while any(th.is_alive() for th in threads):
    time.sleep(20)
    print(f"oracle running {time.time() - t0:.0f} s", flush=True)
for n in CASES:
    g, r = got[n], ref[n]
    same = bool(np.array_equal(g.view(np.uint64), r.view(np.uint64)))
    print(json.dumps({"n": n, "kind": "pow2" if n & (n - 1) == 0 else "bluestein",
                      "bit_exact_vs_oracle": same, "differing_doubles": int(np.sum(g != r)),
                      "engine_s": round(secs[("engine", n)], 2),
                      "oracle_s": round(secs[("oracle", n)], 1)}), flush=True)
