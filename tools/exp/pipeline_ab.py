"""A/B: sequential fwd+inv of 1024 db4 J=8 N=2^20 signals vs. sub-batch pipelining on two
streams (inverse of part q beside forward of part q+1).  Experiment only."""
import ctypes, sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "jwave-pro_amd"))
import torch
from jwave import MODWTTransform, _native
from jwave.transforms import wavelets as W

n, J, Bl = 1 << 20, 8, 1024
dev = torch.device("cuda", 0)
lib = _native.lib()
x = torch.empty((Bl, n), dtype=torch.float64, device=dev)
xr = torch.empty_like(x)
s0 = torch.cuda.current_stream(dev)
_native.check(lib.jw_synth_uniform(ctypes.c_void_p(x.data_ptr()), n, Bl, 42, ctypes.c_void_p(s0.cuda_stream)))
m = MODWTTransform(W.by_name("Daubechies4"))
m.setConvolutionMethod(MODWTTransform.ConvolutionMethod.DIRECT)
plan = m.initializeFilterCache()

def run(parts, reps=5):
    B = Bl // parts
    cs = [torch.empty((B, J + 1, n), dtype=torch.float64, device=dev) for _ in range(min(parts, 2))]
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    def one():
        evs = []
        for q in range(parts):
            c = cs[q % len(cs)]
            if q >= 2:
                sa.wait_event(evs_inv[q - 2])
            _native.check(lib.jw_modwt_forward(plan, ctypes.c_void_p(x[q * B].data_ptr()), ctypes.c_void_p(c.data_ptr()), n, J, B,
                                               _native.JW_CONV_DIRECT, _native.JW_DEVICE, ctypes.c_void_p(sa.cuda_stream)))
            e = torch.cuda.Event(); e.record(sa); sb.wait_event(e)
            _native.check(lib.jw_modwt_inverse(plan, ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(xr[q * B].data_ptr()), n, J, B,
                                               _native.JW_CONV_DIRECT, _native.JW_DEVICE, ctypes.c_void_p(sb.cuda_stream)))
            ei = torch.cuda.Event(); ei.record(sb); evs_inv.append(ei)
    for _ in range(2):
        evs_inv = []; one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        evs_inv = []; one()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    err = (xr - x).abs().amax().item()
    print(f"parts={parts} ms/step={ms:.2f} Msamples/s={Bl*n/ms/1e3:.0f} maxerr={err:.2e}", flush=True)

for p in (1, 2, 4, 8, 16):
    run(p)
