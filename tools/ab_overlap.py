"""A/B: does running the headline's forward and inverse kernels side by side (sub-batches on two
streams: inverse of chunk k beside the forward of chunk k + 1) move more bytes per second than
running them one after the other?  Each kernel alone sits at ~5.5 TB/s, the ceiling of its own
1 -> 9 / 9 -> 1 row shape (profiles/r04/rowshape_a.log), below a plain copy's ~6.3 TB/s.
db4 J=8, N=2^20, 1024 signals, DIRECT, FMA; every schedule computes the same outputs (checked).
Usage: python3 tools/ab_overlap.py [reps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jwave-pro_amd")]
import torch  # noqa: E402
from jwave import _native  # noqa: E402
from jwave.transforms import wavelets as W  # noqa: E402
from jwave.transforms.modwt import MODWTTransform  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    n, J, B = 1 << 20, 8, 1024
    lib = _native.lib()
    x = torch.empty((B, n), dtype=torch.float64, device=dev)
    c = torch.empty((B, J + 1, n), dtype=torch.float64, device=dev)
    xr = torch.empty((B, n), dtype=torch.float64, device=dev)
    s0 = torch.cuda.current_stream(dev)
    lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, B, 42, ctypes.c_void_p(s0.cuda_stream))
    m = MODWTTransform(W.Daubechies4(), arith="fma")
    m.setConvolutionMethod(MODWTTransform.ConvolutionMethod.DIRECT)
    plan = m.initializeFilterCache()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def fwd(lo, cnt, s):
        _native.check(lib.jw_modwt_forward(plan, ctypes.c_void_p(x[lo].data_ptr()),
                                           ctypes.c_void_p(c[lo].data_ptr()), n, J, cnt,
                                           _native.JW_CONV_DIRECT, _native.JW_DEVICE,
                                           ctypes.c_void_p(s.cuda_stream)))

    def inv(lo, cnt, s):
        _native.check(lib.jw_modwt_inverse(plan, ctypes.c_void_p(c[lo].data_ptr()),
                                           ctypes.c_void_p(xr[lo].data_ptr()), n, J, cnt,
                                           _native.JW_CONV_DIRECT, _native.JW_DEVICE,
                                           ctypes.c_void_p(s.cuda_stream)))

    def serial():
        fwd(0, B, sa)
        inv(0, B, sa)

    def overlapped(k):
        ch = B // k
        sb.wait_stream(sa)
        for q in range(k):
            fwd(q * ch, ch, sa)
            e = torch.cuda.Event()
            e.record(sa)
            sb.wait_event(e)
            inv(q * ch, ch, sb)
        sa.wait_stream(sb)

    def timeit(fn, name):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        print(f"{name:28s} {t * 1e3:8.2f} ms  {B * n / t / 1e6:9.1f} Msamples/s  "
              f"(all {', '.join(f'{v * 1e3:.2f}' for v in ts)})", flush=True)
        return xr.clone() if name == "serial" else None

    ref = timeit(serial, "serial")
    for k in (2, 4, 8, 16):
        timeit(lambda: overlapped(k), f"overlapped k={k}")
        assert torch.equal(xr, ref), f"k={k}: outputs differ"
    timeit(serial, "serial")


if __name__ == "__main__":
    main()
